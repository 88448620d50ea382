"""TEST INFRASTRUCTURE ONLY -- ctypes wrapper of the CPU restatement (liblmsf_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
Parity status vs the real reference: unpinned (see oracle/lmsf_oracle.h).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liblmsf_oracle.so")

KIND_EDGE, KIND_SURF = 1, 2
SOLVER_CERES_LM, SOLVER_GN = 0, 1

RECORD_DTYPE = np.dtype([("p", np.float32, 3), ("kind", np.int32), ("v0", np.float64, 3), ("v1", np.float64, 3)])
assert RECORD_DTYPE.itemsize == 64


class ExtractParams(C.Structure):
    _fields_ = [("n_scans", C.c_int32), ("min_distance", C.c_float), ("max_distance", C.c_float),
                ("edge_threshold", C.c_float), ("remove_bad_points", C.c_int32),
                ("beam_lo_deg", C.c_double), ("beam_spacing_deg", C.c_double), ("libm_float", C.c_int32)]


class SolveStats(C.Structure):
    _fields_ = [("outer_iterations", C.c_int32), ("edge_matches", C.c_int32), ("surf_matches", C.c_int32),
                ("inner_iterations", C.c_int32), ("evaluations", C.c_int32), ("termination", C.c_int32),
                ("initial_cost", C.c_double), ("final_cost", C.c_double)]


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        P = C.c_void_p
        fp = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")
        dp = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
        ip = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
        L.lmsfo_extract.argtypes = [C.POINTER(ExtractParams), fp, C.c_int64, fp, ip, C.POINTER(C.c_int64),
                                    fp, ip, C.POINTER(C.c_int64), C.c_int64]
        L.lmsfo_map_build.restype = P
        L.lmsfo_map_build.argtypes = [fp, C.c_int64]
        L.lmsfo_map_free.argtypes = [P]
        L.lmsfo_map_knn.argtypes = [P, fp, C.c_int64, C.c_int, ip, fp]
        L.lmsfo_brute_knn.argtypes = [fp, C.c_int64, fp, C.c_int64, C.c_int, ip, fp]
        L.lmsfo_reg_create.restype = P
        L.lmsfo_reg_create.argtypes = [C.c_int]
        L.lmsfo_reg_free.argtypes = [P]
        L.lmsfo_reg_set_map.argtypes = [P, C.c_int, fp, C.c_int64]
        L.lmsfo_reg_set_scan.argtypes = [P, C.c_int, fp, C.c_int64]
        L.lmsfo_reg_set_max_iterations.argtypes = [P, C.c_int]
        L.lmsfo_reg_set_fixed_schedule.argtypes = [P, C.c_int]
        L.lmsfo_reg_solve.argtypes = [P, dp, C.c_void_p, C.c_int, C.POINTER(SolveStats)]
        L.lmsfo_reg_match.argtypes = [P, dp, C.c_void_p, C.c_void_p]
        L.lmsfo_reg_num_queries.restype = C.c_int64
        L.lmsfo_reg_num_queries.argtypes = [P]
        L.lmsfo_eval.argtypes = [C.c_void_p, C.c_int64, dp, dp]
        L.lmsfo_pose_plus.argtypes = [dp, dp, dp]
        L.lmsfo_set_num_threads.argtypes = [C.c_int]
        L.lmsfo_voxel_filter.restype = C.c_int64
        L.lmsfo_ingest.restype = C.c_int64
        L.lmsfo_ingest.argtypes = [C.c_void_p, C.c_int64, C.c_uint32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                   C.c_float, C.c_float, C.c_float, fp]
        L.lmsfo_voxel_filter.argtypes = [fp, C.c_int64, C.c_float, fp]
        L.lmsfo_saes3.argtypes = [dp, dp, dp]
        L.lmsfo_saesx.argtypes = [C.c_int, dp, dp, dp]
        _lib = L
    return _lib


def voxel_filter(points, leaf):
    """pcl::VoxelGrid restatement (oracle/voxel.cpp)."""
    p = _f32(points)
    out = np.zeros((max(len(p), 1), 4), np.float32)
    m = lib().lmsfo_voxel_filter(p, len(p), float(leaf), out)
    return out[:m].copy()


def common_process(points, removal_nan=False, voxel_leaf=0.5, distance_near=2.0, distance_far=100.0):
    """PointCloudCommonProcess("filtered")::Process (INC/Algorithm/PointClouds/processing/
    common_processing.hpp:87-112): removeNaN (optional) -> VoxelGrid (voxel.cpp) -> DistanceFilter
    (distance_filter.hpp:24-43: float |p| promoted to double, near < d < far; both 0: pass-through)."""
    p = _f32(points)
    if removal_nan:
        p = p[np.isfinite(p[:, :3]).all(1)]
    if voxel_leaf > 0 and len(p):
        p = voxel_filter(p, voxel_leaf)
    if not (distance_near == 0 and distance_far == 0) and len(p):
        x, y, z = p[:, 0], p[:, 1], p[:, 2]
        d = np.sqrt(x * x + y * y + z * z).astype(np.float64)       # float32 arithmetic, as getVector3fMap().norm()
        p = p[(d > float(np.float32(distance_near))) & (d < float(np.float32(distance_far)))]
    return np.ascontiguousarray(p)


def ingest(data: np.ndarray, n: int, point_step=32, offsets=(0, 4, 8, 16), scan_period=0.1, distance_near=0.0,
           distance_far=0.0):
    """PointCloud2 bytes -> xyzi rows (oracle/ingest.cpp)."""
    buf = np.ascontiguousarray(data, dtype=np.uint8)
    out = np.zeros((max(n, 1), 4), np.float32)
    m = lib().lmsfo_ingest(buf.ctypes.data, n, point_step, *offsets, scan_period, distance_near, distance_far, out)
    return out[:m].copy()


def set_threads(n: int):
    lib().lmsfo_set_num_threads(int(n))


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def extract(points, n_scans=16, min_distance=2.0, max_distance=80.0, edge_threshold=1.0,
            remove_bad_points=True, beam_lo_deg=0.0, beam_spacing_deg=0.0, libm_float=False):
    """LOAMFeatureProcessorBase::Process -> (edge xyzi, surf xyzi, edge src idx, surf src idx)."""
    pts = _f32(points)
    n = pts.shape[0]
    prm = ExtractParams(n_scans, min_distance, max_distance, edge_threshold, int(remove_bad_points),
                        beam_lo_deg, beam_spacing_deg, int(libm_float))
    cap = max(n, 1)
    e = np.empty((cap, 4), np.float32)
    s = np.empty((cap, 4), np.float32)
    ei = np.empty(cap, np.int32)
    si = np.empty(cap, np.int32)
    ne, ns = C.c_int64(), C.c_int64()
    rc = lib().lmsfo_extract(C.byref(prm), pts, n, e, ei, C.byref(ne), s, si, C.byref(ns), cap)
    if rc != 0:
        raise RuntimeError(f"lmsfo_extract failed: {rc}")
    return e[:ne.value].copy(), s[:ns.value].copy(), ei[:ne.value].copy(), si[:ns.value].copy()


class KdMap:
    def __init__(self, points):
        self.pts = _f32(points)
        self.h = lib().lmsfo_map_build(self.pts, self.pts.shape[0])

    def knn(self, q, k=5):
        q4 = np.zeros((len(q), 4), np.float32)
        q4[:, :3] = np.asarray(q, np.float32)[:, :3]
        idx = np.empty((len(q), k), np.int32)
        d2 = np.empty((len(q), k), np.float32)
        lib().lmsfo_map_knn(self.h, q4, len(q), k, idx, d2)
        return idx, d2

    def __del__(self):
        if getattr(self, "h", None):
            lib().lmsfo_map_free(self.h)
            self.h = None


def brute_knn(map_pts, q, k=5):
    m = _f32(map_pts)
    q4 = np.zeros((len(q), 4), np.float32)
    q4[:, :3] = np.asarray(q, np.float32)[:, :3]
    idx = np.empty((len(q), k), np.int32)
    d2 = np.empty((len(q), k), np.float32)
    lib().lmsfo_brute_knn(m, m.shape[0], q4, len(q), k, idx, d2)
    return idx, d2


class Registration:
    """CeresEdgeSurfFeatureRegistration / EdgeSurfFeatureRegistration(GN) restated on the CPU."""

    def __init__(self, solver=SOLVER_CERES_LM):
        self.h = lib().lmsfo_reg_create(solver)
        self._keep = []

    def set_map(self, kind, pts):
        p = _f32(pts)
        lib().lmsfo_reg_set_map(self.h, kind, p, p.shape[0])

    def set_scan(self, kind, pts):
        p = _f32(pts)
        lib().lmsfo_reg_set_scan(self.h, kind, p, p.shape[0])

    def set_max_iterations(self, n):
        lib().lmsfo_reg_set_max_iterations(self.h, n)

    def set_fixed_schedule(self, fixed=True):
        lib().lmsfo_reg_set_fixed_schedule(self.h, int(fixed))

    def solve(self, pose, trace_cap=16):
        x = np.ascontiguousarray(pose, dtype=np.float64).copy()
        tr = np.zeros((trace_cap, 7), np.float64)
        st = SolveStats()
        lib().lmsfo_reg_solve(self.h, x, tr.ctypes.data, trace_cap, C.byref(st))
        return x, tr[:st.outer_iterations].copy(), st

    def match(self, pose):
        n = lib().lmsfo_reg_num_queries(self.h)
        rec = np.zeros(n, RECORD_DTYPE)
        nn = np.zeros((n, 5), np.int32)
        x = np.ascontiguousarray(pose, dtype=np.float64)
        lib().lmsfo_reg_match(self.h, x, rec.ctypes.data, nn.ctypes.data)
        return rec, nn

    def __del__(self):
        if getattr(self, "h", None):
            lib().lmsfo_reg_free(self.h)
            self.h = None


def eval_records(rec, pose):
    out = np.zeros(29, np.float64)
    r = np.ascontiguousarray(rec)
    lib().lmsfo_eval(r.ctypes.data, len(r), np.ascontiguousarray(pose, np.float64), out)
    return out


def saes(a, fixed3=None):
    """Eigen 3.3 SelfAdjointEigenSolver restated (saes.cpp) -> (eigenvalues ascending, eigenvectors in
    columns, info).  fixed3 (default: n == 3) selects the Matrix3d path, else the MatrixXd path."""
    a = np.ascontiguousarray(a, np.float64)
    n = a.shape[0]
    d = np.zeros(n)
    v = np.zeros((n, n))
    if fixed3 is None:
        fixed3 = n == 3
    if fixed3:
        info = lib().lmsfo_saes3(a.reshape(-1), d, v.reshape(-1))
    else:
        info = lib().lmsfo_saesx(n, a.reshape(-1), d, v.reshape(-1))
    return d, v, info


def pose_plus(x, delta):
    out = np.zeros(7)
    lib().lmsfo_pose_plus(np.ascontiguousarray(x, np.float64), np.ascontiguousarray(delta, np.float64), out)
    return out
