"""TEST INFRASTRUCTURE ONLY -- CPU restatement of LidarTrackerLocalMap (tracking mode).

Follows INC/LidarTracker/LidarTrackerLocalMap.hpp:107-262 (INC = src/MultiSensorFusionEstimator3D/
include) on top of the oracle registration (oracle.Registration, which keeps the reference's
per-object optimization_count_ decay across Solve calls).  The local map class is absent from the
reference snapshot; this restates the build-defined "sliding_Localmap" (DESIGN.md): a window of the
last W = 10 keyframes per feature kind (the LOAM MultiLidar config's sliding_window.size),
concatenated oldest -> newest and VoxelGrid-downsampled (0.2 m edge / 0.4 m surf), every keyframe
appended.
Parity vs the reference: unpinned (see lmsf_oracle.h).
"""
from __future__ import annotations

import math
from collections import deque

import numpy as np

import oracle as O


def iso_mul(A, B):
    C = np.eye(4)
    C[:3, :3] = A[:3, :3] @ B[:3, :3]
    C[:3, 3] = A[:3, :3] @ B[:3, 3] + A[:3, 3]
    return C


def iso_inv(A):
    B = np.eye(4)
    B[:3, :3] = A[:3, :3].T
    B[:3, 3] = -B[:3, :3] @ A[:3, 3]
    return B


def quat_from_R(m):
    """Eigen quaternion-from-matrix (x, y, z, w)."""
    q = np.zeros(4)
    tr = m[0, 0] + m[1, 1] + m[2, 2]
    if tr > 0:
        t = math.sqrt(tr + 1.0)
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


def R_from_quat(q):
    x, y, z, w = q
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]])


def transform_cloud(pts, T):
    """pcl::transformPointCloud(cloud, out, Matrix4d): float((m0 x + m1 y) + m2 z + m3) in double."""
    x, y, z = (pts[:, k].astype(np.float64) for k in range(3))
    out = pts.copy()
    for r in range(3):
        out[:, r] = (T[r, 0] * x + T[r, 1] * y + T[r, 2] * z + T[r, 3]).astype(np.float32)
    return out


class Tracker:
    """Extensions mirrored from include/lmsf/lmsf.h (multi-stream configurations, not reference
    surface): `origin` (lmsf_tracker_set_initial_pose), `prior` maps in front of the window
    (lmsf_tracker_set_prior_map), manual keyframe mode (add_keyframe + commit)."""

    def __init__(self, window_frames=10, threshold_trans=0.3, threshold_rot=0.1, time_interval=10.0, solver=0,
                 manual_map_update=False, leaf_edge=0.2, leaf_surf=0.4):
        self.reg = O.Registration(solver)
        self.W = window_frames
        self.th_t, self.th_r, self.dt_kf = threshold_trans, threshold_rot, time_interval
        self.manual = manual_map_update
        self.init = False
        self.origin = np.eye(4)
        self.curr = self.prev = self.motion = self.last_kf = np.eye(4)
        self.last_kf_time = 0.0
        self.win = {1: deque(), 2: deque()}
        self.prior = {1: None, 2: None}
        self.dirty = {1: False, 2: False}
        self.leaf = {1: leaf_edge, 2: leaf_surf}

    def local_map(self, kind):
        """[prior | VoxelGrid(window keyframes, oldest -> newest)] (the build's sliding_Localmap)."""
        parts = [self.prior[kind]] if self.prior[kind] is not None else []
        if self.win[kind]:
            w = np.concatenate(list(self.win[kind]), 0)
            parts.append(O.voxel_filter(w, self.leaf[kind]) if self.leaf[kind] > 0 else w)
        return np.concatenate(parts, 0) if parts else np.zeros((0, 4), np.float32)

    def set_prior_map(self, kind, pts):
        self.prior[kind] = np.asarray(pts, np.float32) if len(pts) else None
        self.dirty[kind] = True
        self.commit()

    def _push(self, kind, f, T):
        if len(f) == 0:
            return
        w = self.win[kind]
        if len(w) == self.W:
            w.popleft()
        w.append(transform_cloud(f, T))
        self.dirty[kind] = True

    def commit(self):
        for kind in (1, 2):
            if self.dirty[kind]:
                m = self.local_map(kind)
                if len(m):
                    self.reg.set_map(kind, m)
                self.dirty[kind] = False

    def add_keyframe(self, edge, surf, T):
        self._push(1, edge, T)
        self._push(2, surf, T)

    def _update_local_map(self, feats, T):
        self.add_keyframe(feats[1], feats[2], T)
        self.commit()

    def _register(self, feats, T):
        self.reg.set_scan(1, feats[1])
        self.reg.set_scan(2, feats[2])
        x0 = np.concatenate([quat_from_R(T[:3, :3]), T[:3, 3]])
        x, _, st = self.reg.solve(x0)
        out = np.eye(4)
        out[:3, :3] = R_from_quat(x[:4])
        out[:3, 3] = x[4:]
        return out, st

    def solve(self, edge, surf, timestamp, deltaT=None):
        feats = {1: edge, 2: surf}
        deltaT = np.eye(4) if deltaT is None else np.asarray(deltaT, dtype=np.float64)
        if not self.init:
            self.curr = self.prev = self.last_kf = self.origin.copy()
            self.motion = np.eye(4)
            if not self.manual:
                self._update_local_map(feats, self.origin)
            self.last_kf_time = timestamp
            self.init = True
            return deltaT, 1, None
        if np.array_equal(deltaT, np.eye(4)):
            self.curr = iso_mul(self.prev, self.motion)
        else:
            self.curr = iso_mul(self.prev, deltaT)
        self.curr, st = self._register(feats, self.curr)
        self.motion = iso_mul(iso_inv(self.prev), self.curr)
        self.prev = self.curr
        typ = 0
        if timestamp - self.last_kf_time > self.dt_kf:
            typ = 2
        else:
            d = iso_mul(iso_inv(self.last_kf), self.curr)
            q = quat_from_R(d[:3, :3])
            q = q / np.linalg.norm(q)
            if np.linalg.norm(d[:3, 3]) > self.th_t or math.acos(q[3]) * 2 > self.th_r:
                typ = 1
        if typ:
            self.last_kf = self.curr
            self.last_kf_time = timestamp
            if not self.manual:
                self._update_local_map(feats, self.curr)
        return self.motion.copy(), typ, st
