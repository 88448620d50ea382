"""Host-side mirror of the reference's plugin interfaces for the LOAM hot path, backed by the HIP
library (liblmsf_hip.so).  Names, argument meaning and state behaviour follow the reference so
that a caller (or a test) reads like the reference's own code:

* RegistrationBase<P> (REG/registration_base.hpp:25-34):
    SetInputSource((name, cloud)), SetInputTarget({name: cloud}), Solve(T)
  implemented by CeresEdgeSurfFeatureRegistrationHIP (REG/ceres_edgeSurfFeatureRegistration.hpp)
  and EdgeSurfFeatureRegistrationHIP (GN, REG/edgeSurfFeatureRegistration.hpp);
* PointCloudProcessBase<In, Out>::Process(LidarData, CloudContainer)
  (INC/Algorithm/PointClouds/processing/process_base.hpp:26-39)
  implemented by LOAMFeatureProcessorHIP (FX/LOAMFeatureProcessor_base.hpp);
* PointCloudCommonProcess<P> (INC/Algorithm/PointClouds/processing/common_processing.hpp:39-122)
  implemented by PointCloudCommonProcessHIP (removeNaN? -> VoxelGrid -> DistanceFilter);
* the factory selection strings (INC/factory/System/ML_SystemFactory.hpp:141-198):
  "feature_based_hip" (LOAM processor + CeresEdgeSurfFeatureRegistration("loam_edge", "loam_surf")) and
  "sparse_point_plane_icp_hip" (PointCloudCommonProcess("filtered") + CeresEdgeSurfFeatureRegistration("",
  "filtered")), each with a LidarTrackerLocalMap sliding window (ScanMapSystem).

Clouds are (N, 4) float32 arrays of x, y, z, intensity (PointXYZI payload).  Poses are either
(q, t) 7-vectors (qx qy qz qw tx ty tz) or 4x4 isometries; Solve accepts and returns the same
kind it was given, converting with Eigen's quaternion <-> matrix algorithms.
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib

EDGE_NAME, SURF_NAME = "loam_edge", "loam_surf"


# ----------------------------------------------------------------------------- pose conversions
def quat_to_matrix(q):
    """Eigen QuaternionBase::toRotationMatrix (no normalisation, like the reference)."""
    x, y, z, w = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]])


def matrix_to_quat(m):
    """Eigen quaternionbase_assign_impl<Matrix3> (Shepperd's method) -> (x, y, z, w)."""
    t = m[0, 0] + m[1, 1] + m[2, 2]
    q = np.zeros(4)
    if t > 0:
        t = math.sqrt(t + 1.0)
        q[3] = 0.5 * t
        t = 0.5 / t
        q[0] = (m[2, 1] - m[1, 2]) * t
        q[1] = (m[0, 2] - m[2, 0]) * t
        q[2] = (m[1, 0] - m[0, 1]) * t
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = math.sqrt(m[i, i] - m[j, j] - m[k, k] + 1.0)
        q[i] = 0.5 * t
        t = 0.5 / t
        q[3] = (m[k, j] - m[j, k]) * t
        q[j] = (m[j, i] + m[i, j]) * t
        q[k] = (m[k, i] + m[i, k]) * t
    return q


def to_pose7(T):
    T = np.asarray(T, dtype=np.float64)
    if T.shape == (7,):
        return T.copy()
    if T.shape == (4, 4):
        return np.concatenate([matrix_to_quat(T[:3, :3]), T[:3, 3]])
    raise ValueError("pose must be a 7-vector (qx qy qz qw tx ty tz) or a 4x4 isometry")


def to_matrix(x):
    T = np.eye(4)
    T[:3, :3] = quat_to_matrix(x[:4])
    T[:3, 3] = x[4:]
    return T


# ----------------------------------------------------------------------------- registration
class _RegistrationHIP:
    solver = _lib.SOLVER_CERES_LM

    def __init__(self, edge_name=EDGE_NAME, surf_name=SURF_NAME, device=0, max_features=1 << 17,
                 schedule=_lib.SCHEDULE_REFERENCE_DECAY, max_iterations=10):
        self.edge_name, self.surf_name = edge_name, surf_name
        self.ctx = _lib.Context(device=device, solver=self.solver, schedule=schedule,
                                max_iterations=max_iterations, max_features=max_features,
                                max_scan_points=max_features)
        self.last_stats = None

    def SetInputSource(self, source_input):
        """(name, cloud): the local feature map of that name (ceres_...:56-71)."""
        name, cloud = source_input
        if cloud is None or len(cloud) == 0:
            return                                     # ceres_...:60
        if name == self.edge_name:
            self.ctx.set_map(_lib.EDGE, cloud)
        elif name == self.surf_name:
            self.ctx.set_map(_lib.SURF, cloud)

    def SetInputTarget(self, target_input):
        """{name: cloud}: current scan features; missing names keep the previous cloud (:73-84)."""
        if self.edge_name in target_input:
            self.ctx.set_scan(_lib.EDGE, target_input[self.edge_name])
        if self.surf_name in target_input:
            self.ctx.set_scan(_lib.SURF, target_input[self.surf_name])

    def SetMaxIteration(self, n):
        self.ctx.set_max_iterations(n)

    def Solve(self, T):
        """Predicted pose in, refined pose out (same representation as given)."""
        x, st = self.ctx.solve(to_pose7(T))
        self.last_stats = st
        T = np.asarray(T)
        if T.shape == (4, 4):
            out = to_matrix(x)
            if T.flags.writeable and T.dtype == np.float64:
                T[...] = out
            return out
        if T.shape == (7,) and T.flags.writeable and T.dtype == np.float64:
            T[...] = x
        return x

    def Trace(self):
        return self.ctx.trace()


class CeresEdgeSurfFeatureRegistrationHIP(_RegistrationHIP):
    """CeresEdgeSurfFeatureRegistration (REG/ceres_edgeSurfFeatureRegistration.hpp:26-245) on gfx950."""
    solver = _lib.SOLVER_CERES_LM


class EdgeSurfFeatureRegistrationHIP(_RegistrationHIP):
    """EdgeSurfFeatureRegistration, GN mode (REG/edgeSurfFeatureRegistration.hpp:27-352) on gfx950."""
    solver = _lib.SOLVER_GN


# ----------------------------------------------------------------------------- feature processor
class LOAMFeatureProcessorHIP:
    """LOAMFeatureProcessorBase(N_SCANS, min_distance, max_distance, edge_thresh,
    surf_voxel_grid_size, RemovalBadPoints) (FX/LOAMFeatureProcessor_base.hpp:36-50).
    The voxel filters are constructed but never applied by the reference (FX:48-49); the
    parameter is accepted for signature parity and ignored."""

    def __init__(self, N_SCANS, min_distance=0.0, max_distance=9999.0, edge_thresh=1.0,
                 surf_voxel_grid_size=0.1, RemovalBadPoints=True, device=0, max_scan_points=1 << 17,
                 beam_lo_deg=0.0, beam_spacing_deg=0.0):
        self.ctx = _lib.Context(device=device, n_scans=N_SCANS, min_distance=min_distance,
                                max_distance=max_distance, edge_threshold=edge_thresh,
                                remove_bad_points=int(bool(RemovalBadPoints)), max_scan_points=max_scan_points,
                                max_features=max_scan_points, beam_lo_deg=beam_lo_deg,
                                beam_spacing_deg=beam_spacing_deg)

    def Process(self, data_in, data_out=None):
        """LidarData (or an (N, 4) cloud) -> CloudContainer {"loam_edge", "loam_surf"} (FX:59-126)."""
        cloud = getattr(data_in, "point_cloud", data_in)
        self.ctx.extract(cloud)
        edge, _ = self.ctx.copy_features(_lib.EDGE)
        surf, _ = self.ctx.copy_features(_lib.SURF)
        out = {EDGE_NAME: edge, SURF_NAME: surf}
        if data_out is not None:
            data_out.update(out)
        return out


FILTERED_NAME = "filtered"


class PointCloudCommonProcessHIP:
    """PointCloudCommonProcess<P>(output_name, removal_nan=false) (common_processing.hpp:39-122): the
    "sparse_point_plane_icp" preprocessor.  SetVoxelGrid / SetDistanceFilter as the factory calls them
    (ML_SystemFactory.hpp:158-171); Process runs lmsf_common_process on the device."""

    def __init__(self, output_name=FILTERED_NAME, removal_nan=False, device=0, max_points=1 << 17, ctx=None):
        self.output_name = output_name
        self.ctx = ctx or _lib.Context(device=device, max_scan_points=max_points, max_features=max_points)
        self.params = dict(removal_nan=int(bool(removal_nan)), voxel_leaf=0.0, distance_near=0.0, distance_far=0.0)

    def SetVoxelGrid(self, name, cell_size):
        if name != "VoxelGrid":       # ApproximateVoxelGrid (voxel_grid.hpp) is not on the MI355X path
            raise ValueError(f"downsample filter {name!r} is not provided (VoxelGrid only)")
        self.params["voxel_leaf"] = float(cell_size)

    def SetDistanceFilter(self, distance_near_thresh, distance_far_thresh):
        self.params["distance_near"] = float(distance_near_thresh)
        self.params["distance_far"] = float(distance_far_thresh)

    def run(self, cloud):
        """Filter on the device; the result stays there as the context's current surf target."""
        return self.ctx.common_process(cloud, **self.params)

    def Process(self, data_in, data_out=None):
        """LidarData (or an (N, 4) cloud) -> CloudContainer {output_name: filtered cloud} (:87-112)."""
        self.run(getattr(data_in, "point_cloud", data_in))
        out = {self.output_name: self.ctx.copy_features(_lib.SURF)[0]}
        if data_out is not None:
            data_out.update(out)
        return out


def make_registration(method: str, **kw):
    """tracker.scan_map.registration_method (ML_SystemFactory.hpp:82-83, 141-198)."""
    if method == "feature_based_hip":
        return CeresEdgeSurfFeatureRegistrationHIP("loam_edge", "loam_surf", **kw)
    if method == "feature_based_hip_gn":
        return EdgeSurfFeatureRegistrationHIP("loam_edge", "loam_surf", **kw)
    if method == "sparse_point_plane_icp_hip":
        return CeresEdgeSurfFeatureRegistrationHIP("", FILTERED_NAME, **kw)
    raise ValueError(f"registration method {method!r} is not provided by the MI355X path "
                     "(scope: the Ceres edge/surf registration; see DESIGN.md)")


# point_plane_icp_test.yaml:16-24, 36-37 (the only shipped config reaching this registration)
SPARSE_ICP_DEFAULTS = dict(voxel_size=0.5, distance_min=2.0, distance_max=100.0, window=10)


class ScanMapSystem:
    """One LiDAR's scan-to-map tracking as MultiLidarSystem builds it from
    tracker.scan_map.registration_method (ML_SystemFactory.hpp:141-198): processor -> LidarTrackerLocalMap
    (sliding window) -> CeresEdgeSurfFeatureRegistration, all on one device context, the processed
    clouds staying in HBM between the processor and the tracker.

      "feature_based_hip":          LOAMFeatureProcessorBase(16, 2, 80); window on {loam_edge, loam_surf}
                                    (the build's sliding_Localmap, VoxelGrid 0.2 / 0.4 m)
      "sparse_point_plane_icp_hip": PointCloudCommonProcess("filtered") = VoxelGrid(voxel_size) ->
                                    DistanceFilter(distance_min, distance_max); registration ("", "filtered");
                                    window on {filtered} of `window` keyframes, downsampled with the same
                                    voxel_size (build-defined)
    process(scan, timestamp) -> (pose 4x4 in the tracker frame, update type)."""

    def __init__(self, method, ctx=None, device=0, max_points=1 << 17, **cfg):
        self.method = method
        self.ctx = ctx or _lib.Context(device=device, max_scan_points=max_points, max_features=max_points)
        if method == "feature_based_hip":
            self.processor = None
            self.tracker = _lib.Tracker(self.ctx, window_frames=cfg.get("window", 10))
        elif method == "sparse_point_plane_icp_hip":
            c = dict(SPARSE_ICP_DEFAULTS, **cfg)
            self.processor = PointCloudCommonProcessHIP(FILTERED_NAME, ctx=self.ctx)
            self.processor.SetVoxelGrid("VoxelGrid", c["voxel_size"])
            self.processor.SetDistanceFilter(c["distance_min"], c["distance_max"])
            self.tracker = _lib.Tracker(self.ctx, window_frames=c["window"], leaf_edge=0.0, leaf_surf=c["voxel_size"])
        else:
            raise ValueError(f"scan-map method {method!r} is not provided by the MI355X path")
        self.last = None

    def process(self, scan, timestamp, deltaT=None):
        if self.processor is None:
            self.ctx.extract(scan)
        else:
            self.processor.run(scan)
        _, r = self.tracker.solve_extracted(timestamp, deltaT)
        self.last = r
        return self.tracker.pose(), r.update_type

    def close(self):
        self.tracker.close()
