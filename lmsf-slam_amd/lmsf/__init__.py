"""lmsf -- MI355X-native LOAM edge/surface registration hot path of LMSF-Slam.

The compute path is liblmsf_hip.so (hand-written HIP for gfx950) behind the C ABI of
include/lmsf/lmsf.h; this package is the Python host mirror of the reference's plugin surface
(RegistrationBase / PointCloudProcessBase) plus the synthetic workload generator.
"""
from . import _lib  # noqa: F401
from ._lib import Context, LmsfError  # noqa: F401
from .registration import (CeresEdgeSurfFeatureRegistrationHIP, EdgeSurfFeatureRegistrationHIP,  # noqa: F401
                           LOAMFeatureProcessorHIP, make_registration)

__all__ = ["Context", "LmsfError", "CeresEdgeSurfFeatureRegistrationHIP", "EdgeSurfFeatureRegistrationHIP",
           "LOAMFeatureProcessorHIP", "make_registration"]
