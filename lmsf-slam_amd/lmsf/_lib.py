"""ctypes binding of liblmsf_hip.so (the C ABI declared in include/lmsf/lmsf.h).

The HIP library is the product path: there is no CPU fallback.  Importing this module on a
machine without the built library raises immediately; calling into it without a GPU returns
LMSF_ERR_HIP, which is raised as LmsfError.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # lmsf-slam_amd/
LIB_PATH = os.environ.get("LMSF_LIB") or os.path.join(PKG_ROOT, "liblmsf_hip.so")   # LMSF_LIB: A/B builds
HEADER_PATH = os.path.join(os.path.dirname(PKG_ROOT), "include", "lmsf", "lmsf.h")

OK, ERR_ARG, ERR_HIP, ERR_NO_MAP, ERR_CAPACITY, ERR_STATE = 0, -1, -2, -3, -4, -5
EDGE, SURF = 1, 2
UPDATE_NONE, UPDATE_MOTION, UPDATE_TIME = 0, 1, 2
SOLVER_CERES_LM, SOLVER_GN = 0, 1
SCHEDULE_REFERENCE_DECAY, SCHEDULE_FIXED = 0, 1
(OPT_QUERY_MEMO, OPT_MEMO_REFIT, OPT_MEMO_EXACT, OPT_MEMO_ORDER, OPT_MEMO_BOUND, OPT_GRAPH, OPT_MEMO_SKIP1, OPT_LM_LOOP,
 OPT_LOOP_FAULT_TEST, OPT_GROWTH_TEST, OPT_FAULT_INJECT) = range(11)
TERM_NAMES = {0: "max_iterations", 1: "function_tol", 2: "parameter_tol", 3: "gradient_tol",
              4: "no_residuals", 5: "gn_converged", 6: "gn_too_few"}

RECORD_DTYPE = np.dtype([("p", np.float32, 3), ("kind", np.int32), ("v0", np.float64, 3), ("v1", np.float64, 3)])


class Config(C.Structure):
    _fields_ = [("device", C.c_int32), ("solver", C.c_int32), ("schedule", C.c_int32),
                ("max_iterations", C.c_int32), ("max_batch", C.c_int32), ("max_scan_points", C.c_int32),
                ("max_features", C.c_int32), ("n_scans", C.c_int32), ("min_distance", C.c_float),
                ("max_distance", C.c_float), ("edge_threshold", C.c_float), ("remove_bad_points", C.c_int32),
                ("beam_lo_deg", C.c_double), ("beam_spacing_deg", C.c_double), ("libm_float", C.c_int32)]


class SolveStats(C.Structure):
    _fields_ = [("outer_iterations", C.c_int32), ("edge_matches", C.c_int32), ("surf_matches", C.c_int32),
                ("inner_iterations", C.c_int32), ("evaluations", C.c_int32), ("termination", C.c_int32),
                ("initial_cost", C.c_double), ("final_cost", C.c_double)]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class FeatureCounts(C.Structure):
    _fields_ = [("n_edge", C.c_int64), ("n_surf", C.c_int64)]


class KernelStats(C.Structure):
    _fields_ = [("launches", C.c_int64), ("total_ms", C.c_double), ("queries", C.c_int64), ("n27_sum", C.c_int64),
                ("fused_launches", C.c_int64), ("reused_queries", C.c_int64),
                ("refit_queries", C.c_int64), ("loop_recoveries", C.c_int64),
                ("buffer_growths", C.c_int64), ("split_searches", C.c_int64),
                ("lookahead_solves", C.c_int64)]


class ExtractParams(C.Structure):
    _fields_ = [("n_scans", C.c_int32), ("min_distance", C.c_float), ("max_distance", C.c_float),
                ("edge_threshold", C.c_float), ("remove_bad_points", C.c_int32), ("beam_lo_deg", C.c_double),
                ("beam_spacing_deg", C.c_double), ("libm_float", C.c_int32)]


class CommonParams(C.Structure):
    _fields_ = [("removal_nan", C.c_int32), ("voxel_leaf", C.c_float), ("distance_near", C.c_float),
                ("distance_far", C.c_float)]


class TrackerConfig(C.Structure):
    _fields_ = [("window_frames", C.c_int32), ("threshold_trans", C.c_double), ("threshold_rot", C.c_double),
                ("time_interval", C.c_double), ("manual_map_update", C.c_int32), ("leaf_edge", C.c_double),
                ("leaf_surf", C.c_double), ("keyframe_lookahead", C.c_int32)]


class IngestParams(C.Structure):
    _fields_ = [("point_step", C.c_uint32), ("offset_x", C.c_int32), ("offset_y", C.c_int32),
                ("offset_z", C.c_int32), ("offset_intensity", C.c_int32), ("is_bigendian", C.c_int32),
                ("scan_period", C.c_float), ("distance_near", C.c_float), ("distance_far", C.c_float)]


class TrackerResult(C.Structure):
    _fields_ = [("initialized", C.c_int32), ("update_type", C.c_int32), ("local_map_edge", C.c_int64),
                ("local_map_surf", C.c_int64), ("solve", SolveStats)]


class LmsfError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"lmsf error {code}: {msg}")
        self.code = code


# every entry point of include/lmsf/lmsf.h: name -> (restype, argtypes)
_P = C.c_void_p
_SIGS = {
    "lmsf_config_init": (C.c_int32, [C.POINTER(Config)]),
    "lmsf_ctx_create": (C.c_int32, [C.POINTER(Config), C.POINTER(_P)]),
    "lmsf_ctx_destroy": (None, [_P]),
    "lmsf_last_error": (C.c_char_p, [_P]),
    "lmsf_set_map": (C.c_int32, [_P, C.c_int32, _P, C.c_size_t]),
    "lmsf_set_scan": (C.c_int32, [_P, C.c_int32, _P, C.c_size_t]),
    "lmsf_set_max_iterations": (C.c_int32, [_P, C.c_int32]),
    "lmsf_set_schedule": (C.c_int32, [_P, C.c_int32]),
    "lmsf_set_extract_params": (C.c_int32, [_P, C.POINTER(ExtractParams)]),
    "lmsf_solve": (C.c_int32, [_P, _P, C.POINTER(SolveStats)]),
    "lmsf_solve_trace": (C.c_int32, [_P, _P, C.c_int32, C.POINTER(C.c_int32)]),
    "lmsf_extract_features": (C.c_int32, [_P, _P, C.c_size_t, C.POINTER(FeatureCounts)]),
    "lmsf_prefetch_features": (C.c_int32, [_P, _P, C.c_size_t]),
    "lmsf_common_params_init": (C.c_int32, [C.POINTER(CommonParams)]),
    "lmsf_common_process": (C.c_int32, [_P, _P, C.c_size_t, C.POINTER(CommonParams), C.POINTER(FeatureCounts)]),
    "lmsf_copy_features": (C.c_int32, [_P, C.c_int32, _P, _P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "lmsf_batch_load_scans": (C.c_int32, [_P, _P, _P, C.c_int32]),
    "lmsf_batch_load_scans_async": (C.c_int32, [_P, _P, _P, C.c_int32]),
    "lmsf_batch_run": (C.c_int32, [_P, C.c_int32, _P, _P]),
    "lmsf_batch_launch": (C.c_int32, [_P, C.c_int32, _P]),
    "lmsf_batch_wait": (C.c_int32, [_P, C.c_int32, _P, _P]),
    "lmsf_batch_trace": (C.c_int32, [_P, C.c_int32, _P, C.c_int32, C.POINTER(C.c_int32)]),
    "lmsf_batch_copy_features": (C.c_int32, [_P, C.c_int32, C.c_int32, _P, _P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "lmsf_set_option": (C.c_int32, [_P, C.c_int32, C.c_int32]),
    "lmsf_batch_capture": (C.c_int32, [_P, _P, C.c_int32]),
    "lmsf_batch_records": (C.c_int32, [_P, C.c_int32, C.c_int32, _P, _P, C.c_size_t, _P, C.POINTER(C.c_size_t)]),
    "lmsf_match": (C.c_int32, [_P, _P, _P, _P, C.c_size_t]),
    "lmsf_eval": (C.c_int32, [_P, _P, _P]),
    "lmsf_eigen_selfadjoint": (C.c_int32, [_P, C.c_int32, _P, C.c_size_t, _P, _P, _P]),
    "lmsf_kernel_stats_get": (C.c_int32, [_P, C.POINTER(KernelStats)]),
    "lmsf_kernel_stats_reset": (C.c_int32, [_P, C.c_int32]),
    "lmsf_version": (C.c_char_p, []),
    "lmsf_tracker_config_init": (C.c_int32, [C.POINTER(TrackerConfig)]),
    "lmsf_tracker_create": (C.c_int32, [_P, C.POINTER(TrackerConfig), C.POINTER(_P)]),
    "lmsf_tracker_destroy": (None, [_P]),
    "lmsf_tracker_solve": (C.c_int32, [_P, _P, C.c_size_t, _P, C.c_size_t, C.c_double, _P, C.POINTER(TrackerResult)]),
    "lmsf_tracker_register": (C.c_int32, [_P, _P, C.c_size_t, _P, C.c_size_t, _P, C.POINTER(SolveStats)]),
    "lmsf_tracker_pose": (C.c_int32, [_P, _P]),
    "lmsf_tracker_local_map": (C.c_int32, [_P, C.c_int32, _P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "lmsf_tracker_solve_extracted": (C.c_int32, [_P, C.c_double, _P, C.POINTER(TrackerResult)]),
    "lmsf_tracker_register_extracted": (C.c_int32, [_P, _P, C.POINTER(SolveStats)]),
    "lmsf_tracker_set_initial_pose": (C.c_int32, [_P, _P]),
    "lmsf_tracker_set_prior_map": (C.c_int32, [_P, C.c_int32, _P, C.c_size_t]),
    "lmsf_tracker_add_keyframe": (C.c_int32, [_P, _P, C.c_size_t, _P, C.c_size_t, _P]),
    "lmsf_tracker_add_keyframe_extracted": (C.c_int32, [_P, _P]),
    "lmsf_tracker_commit_map": (C.c_int32, [_P]),
    "lmsf_voxel_filter": (C.c_int32, [_P, _P, C.c_size_t, C.c_float, _P, C.c_size_t, C.POINTER(C.c_size_t)]),
    "lmsf_ingest_params_init": (C.c_int32, [C.POINTER(IngestParams)]),
    "lmsf_ingest_pointcloud2": (C.c_int32, [_P, _P, C.c_size_t, C.POINTER(IngestParams), _P, C.c_size_t,
                                            C.POINTER(C.c_size_t)]),
    "lmsf_extract_pointcloud2": (C.c_int32, [_P, _P, C.c_size_t, C.POINTER(IngestParams),
                                             C.POINTER(FeatureCounts)]),
    "lmsf_align_set_target": (C.c_int32, [_P, _P, C.c_size_t]),
    "lmsf_align_score": (C.c_int32, [_P, _P, C.c_size_t, _P, C.c_double, C.c_double, C.POINTER(C.c_double),
                                     C.POINTER(C.c_double)]),
    "lmsf_handeye_create": (C.c_int32, [C.POINTER(_P)]),
    "lmsf_handeye_destroy": (None, [_P]),
    "lmsf_handeye_add_pose": (C.c_int32, [_P, _P, _P, C.POINTER(C.c_int32)]),
    "lmsf_handeye_calib_rotation": (C.c_int32, [_P, C.POINTER(C.c_int32), _P]),
    "lmsf_handeye_calib_translation": (C.c_int32, [_P, C.POINTER(C.c_int32)]),
    "lmsf_handeye_result": (C.c_int32, [_P, _P, C.POINTER(C.c_int32)]),
    "lmsf_handeye_pair_count": (C.c_int32, [_P, C.POINTER(C.c_int32)]),
}

_lib = None


def _share_torch_hip_runtime():
    """PyTorch-ROCm bundles its own libamdhip64 / libhsa-runtime64 (SONAME libamdhip64.so.7, as
    /opt/rocm's).  glibc reuses an already-loaded library by SONAME, but torch asks for
    "libamdhip64.so", which does not match /opt/rocm's copy: loading liblmsf first would put two HIP
    runtimes in the process (torch then fails to initialise, and device pointers cannot be passed
    between torch/RCCL buffers and the library).  Loading torch first gives one runtime."""
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def load():
    """Load liblmsf_hip.so (raises if it has not been built: there is no fallback path)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: build it with `make -C lmsf-slam_amd` "
                              "(__graft_entry__.build()); the HIP path has no CPU fallback")
        _share_torch_hip_runtime()
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def default_config(**kw) -> Config:
    cfg = Config()
    load().lmsf_config_init(C.byref(cfg))
    for k, v in kw.items():
        setattr(cfg, k, v)
    return cfg


def _f4(a):
    a = np.ascontiguousarray(a, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] != 4:
        raise ValueError("points must be (N, 4) float32 x y z intensity")
    return a


class Context:
    """One lmsf_ctx: a registration object + feature processor bound to one device stream."""

    def __init__(self, **cfg):
        self.cfg = default_config(**cfg)
        h = C.c_void_p()
        rc = load().lmsf_ctx_create(C.byref(self.cfg), C.byref(h))
        if rc != OK:
            raise LmsfError(rc, "lmsf_ctx_create failed (no HIP device or bad config)")
        self.h = h

    def _check(self, rc):
        if rc != OK:
            raise LmsfError(rc, load().lmsf_last_error(self.h).decode(errors="replace"))
        return rc

    def close(self):
        if getattr(self, "h", None):
            load().lmsf_ctx_destroy(self.h)
            self.h = None

    __del__ = close

    # ---- reference surface
    def set_map(self, kind, pts):
        p, n, keep = _buf(pts)
        self._check(load().lmsf_set_map(self.h, kind, p, n))

    def set_scan(self, kind, pts):
        p = _f4(pts) if len(pts) else np.zeros((0, 4), np.float32)
        self._check(load().lmsf_set_scan(self.h, kind, p.ctypes.data, p.shape[0]))

    def set_max_iterations(self, n):
        self._check(load().lmsf_set_max_iterations(self.h, int(n)))

    def set_schedule(self, schedule):
        self._check(load().lmsf_set_schedule(self.h, int(schedule)))

    def set_extract_params(self, **kw):
        """LOAMFeatureProcessorBase(N_SCANS, min, max, edge_thresh, RemovalBadPoints) + beam model;
        unspecified fields keep the context's current values."""
        c = self.cfg
        p = ExtractParams(c.n_scans, c.min_distance, c.max_distance, c.edge_threshold, c.remove_bad_points,
                          c.beam_lo_deg, c.beam_spacing_deg, c.libm_float)
        for k, v in kw.items():
            setattr(p, k, v)
        self._check(load().lmsf_set_extract_params(self.h, C.byref(p)))
        for f, _ in ExtractParams._fields_:
            setattr(self.cfg, f, getattr(p, f))

    def solve(self, pose):
        x = np.ascontiguousarray(pose, dtype=np.float64).copy()
        st = SolveStats()
        self._check(load().lmsf_solve(self.h, x.ctypes.data, C.byref(st)))
        return x, st

    def trace(self, cap=32):
        out = np.zeros((cap, 7), np.float64)
        n = C.c_int32()
        self._check(load().lmsf_solve_trace(self.h, out.ctypes.data, cap, C.byref(n)))
        return out[:min(n.value, cap)].copy()

    def extract(self, pts):
        p, n, keep = _buf(pts)
        fc = FeatureCounts()
        self._check(load().lmsf_extract_features(self.h, p, n, C.byref(fc)))
        self._prefetched = None
        return fc.n_edge, fc.n_surf

    def prefetch(self, pts):
        """lmsf_prefetch_features: extract the next scan beside the current work; the next extract(pts) of
        the same buffer adopts it (the buffer is kept alive until then)."""
        p, n, keep = _buf(pts)
        self._check(load().lmsf_prefetch_features(self.h, p, n))
        self._prefetched = keep

    @staticmethod
    def common_params(**kw):
        p = CommonParams()
        load().lmsf_common_params_init(C.byref(p))
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    def common_process(self, pts, **kw):
        """lmsf_common_process (PointCloudCommonProcess "filtered": NaN removal?, VoxelGrid, distance
        filter); the result is the current surf target.  Returns its point count."""
        prm = self.common_params(**kw)
        p, n, keep = _buf(pts)
        fc = FeatureCounts()
        self._check(load().lmsf_common_process(self.h, p, n, C.byref(prm), C.byref(fc)))
        return fc.n_surf

    def copy_features(self, kind, slot=None):
        n = C.c_size_t()
        cap = int(self.cfg.max_scan_points) if slot is not None else max(int(self.cfg.max_features),
                                                                          int(self.cfg.max_scan_points))
        out = np.zeros((cap, 4), np.float32)
        src = np.zeros(cap, np.int32)
        if slot is None:
            self._check(load().lmsf_copy_features(self.h, kind, out.ctypes.data, src.ctypes.data, cap, C.byref(n)))
        else:
            self._check(load().lmsf_batch_copy_features(self.h, slot, kind, out.ctypes.data, src.ctypes.data, cap,
                                                         C.byref(n)))
        return out[:n.value].copy(), src[:n.value].copy()

    def copy_features_into(self, kind, out):
        """Copy the extracted features of one kind into a preallocated (cap, 4) float32 torch tensor
        (device memory: a device-to-device copy); returns the feature count."""
        n = C.c_size_t()
        self._check(load().lmsf_copy_features(self.h, kind, out.data_ptr(), None, int(out.shape[0]), C.byref(n)))
        return n.value

    def voxel_filter(self, pts, leaf):
        """lmsf_voxel_filter (pcl::VoxelGrid centroids) of an (n, 4) cloud; returns a numpy array."""
        p, n, keep = _buf(pts)
        out = np.zeros((max(n, 1), 4), np.float32)
        m = C.c_size_t()
        self._check(load().lmsf_voxel_filter(self.h, p, n, float(leaf), out.ctypes.data, out.shape[0], C.byref(m)))
        return out[:m.value].copy()

    @staticmethod
    def ingest_params(**kw):
        p = IngestParams()
        load().lmsf_ingest_params_init(C.byref(p))
        for k, v in kw.items():
            setattr(p, k, v)
        return p

    def _msg(self, data):
        if hasattr(data, "data_ptr"):
            return data.data_ptr(), data
        d = np.ascontiguousarray(data, dtype=np.uint8)
        return d.ctypes.data, d

    def ingest_pointcloud2(self, data, n_points, **kw):
        """PointCloud2 bytes (numpy uint8 or a device tensor) -> (n, 4) xyzi after removeNaN, rotary
        relative time and the optional distance filter."""
        p = self.ingest_params(**kw)
        ptr, keep = self._msg(data)
        out = np.zeros((max(n_points, 1), 4), np.float32)
        m = C.c_size_t()
        self._check(load().lmsf_ingest_pointcloud2(self.h, ptr, n_points, C.byref(p), out.ctypes.data, out.shape[0],
                                                   C.byref(m)))
        return out[:m.value].copy()

    def extract_pointcloud2(self, data, n_points, **kw):
        p = self.ingest_params(**kw)
        ptr, keep = self._msg(data)
        fc = FeatureCounts()
        self._check(load().lmsf_extract_pointcloud2(self.h, ptr, n_points, C.byref(p), C.byref(fc)))
        return fc.n_edge, fc.n_surf

    def align_set_target(self, pts):
        """PointCloudAlignmentEvaluate::SetTargetPoints."""
        p, n, keep = _buf(pts)
        self._check(load().lmsf_align_set_target(self.h, p, n))

    def align_score(self, pts, relpose, inlier_thresh, inlier_ratio_thresh):
        """PointCloudAlignmentEvaluate::AlignmentScore -> (score, overlap_ratio)."""
        p, n, keep = _buf(pts)
        T = np.ascontiguousarray(relpose, dtype=np.float32)
        sc, ov = C.c_double(), C.c_double()
        self._check(load().lmsf_align_score(self.h, p, n, T.ctypes.data, float(inlier_thresh),
                                            float(inlier_ratio_thresh), C.byref(sc), C.byref(ov)))
        return sc.value, ov.value

    # ---- batch path
    def load_scans(self, scans):
        counts = np.array([len(s) for s in scans], np.int64)
        cat = np.ascontiguousarray(np.concatenate([_f4(s) for s in scans], 0)) if counts.sum() else np.zeros((0, 4), np.float32)
        self._check(load().lmsf_batch_load_scans(self.h, cat.ctypes.data, counts.ctypes.data, len(scans)))

    def load_scans_async(self, buf, counts):
        """lmsf_batch_load_scans_async: buf is a contiguous (sum(counts), 4) float32 torch tensor
        (pinned host memory for an asynchronous copy) holding the next launch's scans back to back.
        The buffer and counts are kept alive here until the following batch_wait."""
        counts = np.ascontiguousarray(counts, dtype=np.int64)
        p, n, keep = _buf(buf)
        if n != int(counts.sum()):
            raise ValueError("buffer rows != sum(counts)")
        self._check(load().lmsf_batch_load_scans_async(self.h, p, counts.ctypes.data, len(counts)))
        self._uploads = (getattr(self, "_uploads", ()) + ((keep, counts),))[-2:]   # this one and the one in flight

    def batch_run(self, poses):
        x = np.ascontiguousarray(poses, dtype=np.float64).copy()
        n = x.shape[0]
        st = (SolveStats * n)()
        self._check(load().lmsf_batch_run(self.h, n, x.ctypes.data, C.cast(st, C.c_void_p)))
        return x, list(st)

    def batch_launch(self, poses):
        x = np.ascontiguousarray(poses, dtype=np.float64)
        self._check(load().lmsf_batch_launch(self.h, x.shape[0], x.ctypes.data))

    def batch_wait(self, n):
        x = np.zeros((n, 7), np.float64)
        st = (SolveStats * n)()
        self._check(load().lmsf_batch_wait(self.h, n, x.ctypes.data, C.cast(st, C.c_void_p)))
        return x, list(st)

    def batch_trace(self, slot, cap=32):
        """Per-outer-iteration poses of one slot of the last batch_wait / batch_run."""
        out = np.zeros((cap, 7), np.float64)
        n = C.c_int32()
        self._check(load().lmsf_batch_trace(self.h, int(slot), out.ctypes.data, cap, C.byref(n)))
        return out[:min(n.value, cap)].copy()

    def set_option(self, option, value):
        """lmsf_set_option (OPT_* switches, 0 | 1; OPT_FAULT_INJECT also 2)."""
        self._check(load().lmsf_set_option(self.h, int(option), int(value)))

    # ---- diagnostics
    def batch_capture(self, slots):
        """Capture the records / neighbour indices of these batch slots after every outer iteration of
        the following launches ([] stops it)."""
        s = np.ascontiguousarray(slots, dtype=np.int32)
        self._check(load().lmsf_batch_capture(self.h, s.ctypes.data if len(s) else None, len(s)))

    def batch_records(self, slot, it):
        """(records, nn (n, 5), pose) of a captured slot at outer iteration `it` of the last launch."""
        n = C.c_size_t()
        self._check(load().lmsf_batch_records(self.h, int(slot), int(it), None, None, 0, None, C.byref(n)))
        rec = np.zeros(n.value, RECORD_DTYPE)
        nn = np.zeros((n.value, 5), np.int32)
        pose = np.zeros(7, np.float64)
        self._check(load().lmsf_batch_records(self.h, int(slot), int(it), rec.ctypes.data, nn.ctypes.data, n.value,
                                              pose.ctypes.data, C.byref(n)))
        return rec, nn, pose

    def match(self, pose, n_queries):
        rec = np.zeros(n_queries, RECORD_DTYPE)
        nn = np.zeros((n_queries, 5), np.int32)
        x = np.ascontiguousarray(pose, dtype=np.float64)
        self._check(load().lmsf_match(self.h, x.ctypes.data, rec.ctypes.data, nn.ctypes.data, n_queries))
        return rec, nn

    def eval(self, pose):
        out = np.zeros(29, np.float64)
        x = np.ascontiguousarray(pose, dtype=np.float64)
        self._check(load().lmsf_eval(self.h, x.ctypes.data, out.ctypes.data))
        return out

    def eigen_selfadjoint(self, a):
        """The device's restated SelfAdjointEigenSolver on a stack of 3x3 (Matrix3d path) or 6x6 (MatrixXd
        path) symmetric matrices -> (eigenvalues ascending, eigenvectors in columns, info)."""
        a = np.ascontiguousarray(a, dtype=np.float64)
        n, dim = a.shape[0], a.shape[1]
        d = np.zeros((n, dim))
        v = np.zeros((n, dim, dim))
        info = np.zeros(n, np.int32)
        self._check(load().lmsf_eigen_selfadjoint(self.h, dim, a.ctypes.data, n, d.ctypes.data, v.ctypes.data,
                                                  info.ctypes.data))
        return d, v, info

    def kernel_stats_reset(self, timing=True, n27=False):
        """timing: HIP-event time, launches and queries of the neighbour search; n27: the n27
        accounting (extra loads inside the launch -- use it on untimed launches)."""
        self._check(load().lmsf_kernel_stats_reset(self.h, (1 if timing else 0) | (2 if n27 else 0)))

    def kernel_stats(self):
        ks = KernelStats()
        self._check(load().lmsf_kernel_stats_get(self.h, C.byref(ks)))
        return ks


def _pts(a):
    return _f4(a) if len(a) else np.zeros((0, 4), np.float32)


def _buf(a):
    """(pointer, rows, keep-alive) of an (n, 4) float32 xyzi array: numpy (host) or a torch tensor
    (host or device memory; the C ABI copies with hipMemcpyDefault)."""
    if hasattr(a, "data_ptr"):
        if a.dtype != __import__("torch").float32 or a.dim() != 2 or a.shape[1] != 4 or not a.is_contiguous():
            raise ValueError("expected a contiguous (n, 4) float32 tensor")
        return (a.data_ptr() if a.shape[0] else None), int(a.shape[0]), a
    p = _pts(a)
    return p.ctypes.data, p.shape[0], p


class Tracker:
    """lmsf_tracker: LidarTrackerLocalMap over a Context (poses are 4x4 row-major matrices)."""

    def __init__(self, ctx: Context, window_frames=10, threshold_trans=0.3, threshold_rot=0.1, time_interval=10.0,
                 manual_map_update=False, leaf_edge=0.2, leaf_surf=0.4, keyframe_lookahead=True):
        cfg = TrackerConfig()
        load().lmsf_tracker_config_init(C.byref(cfg))
        cfg.window_frames, cfg.threshold_trans = window_frames, threshold_trans
        cfg.threshold_rot, cfg.time_interval = threshold_rot, time_interval
        cfg.manual_map_update = int(bool(manual_map_update))
        cfg.leaf_edge, cfg.leaf_surf = leaf_edge, leaf_surf
        cfg.keyframe_lookahead = int(bool(keyframe_lookahead))
        self.ctx = ctx
        h = C.c_void_p()
        ctx._check(load().lmsf_tracker_create(ctx.h, C.byref(cfg), C.byref(h)))
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            load().lmsf_tracker_destroy(self.h)
            self.h = None

    __del__ = close

    def solve(self, edge, surf, timestamp, deltaT=None):
        e, s = _pts(edge), _pts(surf)
        d = np.ascontiguousarray(np.eye(4) if deltaT is None else deltaT, dtype=np.float64).copy()
        r = TrackerResult()
        self.ctx._check(load().lmsf_tracker_solve(self.h, e.ctypes.data, e.shape[0], s.ctypes.data, s.shape[0],
                                                  float(timestamp), d.ctypes.data, C.byref(r)))
        return d, r

    def register(self, edge, surf, pose):
        e, s = _pts(edge), _pts(surf)
        T = np.ascontiguousarray(pose, dtype=np.float64).copy()
        st = SolveStats()
        self.ctx._check(load().lmsf_tracker_register(self.h, e.ctypes.data, e.shape[0], s.ctypes.data, s.shape[0],
                                                     T.ctypes.data, C.byref(st)))
        return T, st

    def pose(self):
        T = np.zeros((4, 4))
        self.ctx._check(load().lmsf_tracker_pose(self.h, T.ctypes.data))
        return T

    def local_map(self, kind):
        n = C.c_size_t()
        self.ctx._check(load().lmsf_tracker_local_map(self.h, kind, None, 0, C.byref(n)))
        out = np.zeros((n.value, 4), np.float32)
        self.ctx._check(load().lmsf_tracker_local_map(self.h, kind, out.ctypes.data, n.value, C.byref(n)))
        return out

    # ---- multi-stream extensions
    def solve_extracted(self, timestamp, deltaT=None):
        d = np.ascontiguousarray(np.eye(4) if deltaT is None else deltaT, dtype=np.float64).copy()
        r = TrackerResult()
        self.ctx._check(load().lmsf_tracker_solve_extracted(self.h, float(timestamp), d.ctypes.data, C.byref(r)))
        return d, r

    def register_extracted(self, pose):
        T = np.ascontiguousarray(pose, dtype=np.float64).copy()
        st = SolveStats()
        self.ctx._check(load().lmsf_tracker_register_extracted(self.h, T.ctypes.data, C.byref(st)))
        return T, st

    def set_initial_pose(self, T):
        T = np.ascontiguousarray(T, dtype=np.float64)
        self.ctx._check(load().lmsf_tracker_set_initial_pose(self.h, T.ctypes.data))

    def set_prior_map(self, kind, pts):
        p, n, keep = _buf(pts)
        self.ctx._check(load().lmsf_tracker_set_prior_map(self.h, kind, p, n))

    def add_keyframe(self, edge, surf, pose):
        pe, ne, ke = _buf(edge)
        ps, ns, ks = _buf(surf)
        T = np.ascontiguousarray(pose, dtype=np.float64)
        self.ctx._check(load().lmsf_tracker_add_keyframe(self.h, pe, ne, ps, ns, T.ctypes.data))

    def add_keyframe_extracted(self, pose):
        """The context's extracted features (lmsf_extract_features) as a keyframe at pose (4x4)."""
        T = np.ascontiguousarray(pose, dtype=np.float64)
        self.ctx._check(load().lmsf_tracker_add_keyframe_extracted(self.h, T.ctypes.data))

    def commit_map(self):
        self.ctx._check(load().lmsf_tracker_commit_map(self.h))


def header_symbols(path=HEADER_PATH):
    """Function names declared in include/lmsf/lmsf.h (for the ABI export test)."""
    import re
    text = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:lmsf_status|void|const char\*)\s+(lmsf_\w+)\s*\(", text, re.M)))


class HandEye:
    """lmsf_handeye: HandEyeCalibrationBase (host arithmetic; usable without a GPU)."""

    def __init__(self):
        h = C.c_void_p()
        rc = load().lmsf_handeye_create(C.byref(h))
        if rc != OK:
            raise LmsfError(rc, "lmsf_handeye_create failed")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            load().lmsf_handeye_destroy(self.h)
            self.h = None

    __del__ = close

    @staticmethod
    def _rc(rc):
        if rc != OK:
            raise LmsfError(rc, "lmsf_handeye call failed")

    def add_pose(self, primary, sub):
        a = np.ascontiguousarray(primary, dtype=np.float64)
        b = np.ascontiguousarray(sub, dtype=np.float64)
        ok = C.c_int32()
        self._rc(load().lmsf_handeye_add_pose(self.h, a.ctypes.data, b.ctypes.data, C.byref(ok)))
        return bool(ok.value)

    def calib_rotation(self):
        ok = C.c_int32()
        sv = np.zeros(4)
        self._rc(load().lmsf_handeye_calib_rotation(self.h, C.byref(ok), sv.ctypes.data))
        return bool(ok.value), sv

    def calib_translation(self):
        ok = C.c_int32()
        self._rc(load().lmsf_handeye_calib_translation(self.h, C.byref(ok)))
        return bool(ok.value)

    def result(self):
        T = np.zeros((4, 4))
        ok = C.c_int32()
        self._rc(load().lmsf_handeye_result(self.h, T.ctypes.data, C.byref(ok)))
        return T if ok.value else None

    def pair_count(self):
        n = C.c_int32()
        self._rc(load().lmsf_handeye_pair_count(self.h, C.byref(n)))
        return n.value
