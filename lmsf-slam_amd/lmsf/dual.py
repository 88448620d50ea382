"""Dual-LiDAR front end (configuration C3): MultiLidarSystem::process for NUM_OF_LIDAR = 2
(INC/System/ML_System.hpp:232-323, INC = src/MultiSensorFusionEstimator3D/include) on the HIP path.

* phase 0 (EXTRINSIC_CALIB_STATUS_ == 0, :243-281): each LiDAR runs its own tracker; the two
  inter-frame motions feed the hand-eye initialisation (lmsf_handeye); once rotation and
  translation are calibrated the system moves to phase 1;
* phase 1 (:284-322): only the primary LiDAR is tracked; the sub LiDAR's features are registered
  against the primary tracker's local map from primary * extrinsic (RegistrationLocalMap, :304-305)
  and the extrinsic becomes primary^-1 * sub (:306).

Both scans are extracted on the device; in phase 1 the sub scan is extracted on the primary
tracker's context after the primary Solve, so its features never leave HBM.  The reference then
falls through to a second Solve of tracker 0 on the already moved-from feature container
(:331-334); that defect is not reproduced.  Poses are 4x4 row-major matrices.
"""
from __future__ import annotations

import numpy as np

from . import _lib


def iso_mul(A, B):
    """Eigen Isometry3d product: linear * linear, linear * t + t."""
    C = np.eye(4)
    C[:3, :3] = A[:3, :3] @ B[:3, :3]
    C[:3, 3] = A[:3, :3] @ B[:3, 3] + A[:3, 3]
    return C


def iso_inv(A):
    B = np.eye(4)
    B[:3, :3] = A[:3, :3].T
    B[:3, 3] = -B[:3, :3] @ A[:3, 3]
    return B


class DualLidarSystem:
    def __init__(self, ctx_primary: _lib.Context, ctx_sub: _lib.Context | None = None, extrinsic=None,
                 **tracker_kw):
        self.ctx = [ctx_primary, ctx_sub]
        # the trackers' keyframe appends (updateLocalMap, LidarTrackerLocalMap.hpp:205-232) are made explicitly
        # after each Solve (_track): the same keyframe at the same pose, but the window rebuild is then enqueued
        # by the tracker's commit worker and completes beside the next extraction on the context
        tracker_kw = dict(tracker_kw, manual_map_update=True)
        self.trackers = [_lib.Tracker(ctx_primary, **tracker_kw)]
        if extrinsic is None:
            if ctx_sub is None:
                raise ValueError("extrinsic initialisation (phase 0) needs a context for the sub LiDAR")
            self.trackers.append(_lib.Tracker(ctx_sub, **tracker_kw))
            self.handeye = _lib.HandEye()
            self.status = 0
            self.extrinsic = np.eye(4)
        else:
            self.handeye = None
            self.status = 1
            self.extrinsic = np.asarray(extrinsic, dtype=np.float64).copy()
        self.pose = [np.eye(4), np.eye(4)]       # pose_lidar_cur_
        self.last = {}

    def _track(self, i, scan, timestamp, prefetch=None):
        """LidarTrackerLocalMap::Solve of LiDAR i on its device-extracted features, keyframe included; the
        scan its context extracts next (prefetch) is extracted beside the Solve."""
        self.ctx[i].extract(scan)
        if prefetch is not None:
            self.ctx[i].prefetch(prefetch)
        d, r = self.trackers[i].solve_extracted(timestamp)
        if r.update_type:
            self.trackers[i].add_keyframe_extracted(self.trackers[i].pose())
            self.trackers[i].commit_map()
        return d, r

    def process(self, scan_primary, scan_sub, timestamp, next_frame=None):
        """One synchronized frame; returns (primary pose, sub pose) in the tracker's local frame.  next_frame
        (the next (primary, sub) scans, optional): their extraction starts beside this frame's registrations,
        as the reference's preprocess thread runs ahead of its estimate thread (the results do not change)."""
        nxt = next_frame if next_frame is not None else (None, None)
        if self.status == 0:
            deltas = []
            for i, scan in enumerate((scan_primary, scan_sub)):
                d, r = self._track(i, scan, timestamp, prefetch=nxt[i])
                self.pose[i] = iso_mul(self.pose[i], d)
                deltas.append(d)
            if self.handeye.add_pose(deltas[0], deltas[1]):              # :268-281
                ok_r, sv = self.handeye.calib_rotation()
                self.last["rot_cov"] = sv
                if ok_r and self.handeye.calib_translation():
                    self.extrinsic = self.handeye.result()
                    self.status = 1
            return self.pose[0], self.pose[1]
        t0 = self.trackers[0]
        d, r = self._track(0, scan_primary, timestamp, prefetch=scan_sub)  # :296-297
        primary = t0.pose()                                               # :299
        sub0 = iso_mul(primary, self.extrinsic)                                   # :301
        self.pose[0] = iso_mul(self.pose[0], d)                                   # :302
        self.ctx[0].extract(scan_sub)
        if nxt[0] is not None:
            self.ctx[0].prefetch(nxt[0])
        sub, st = t0.register_extracted(sub0)                             # :304-305
        self.extrinsic = iso_mul(iso_inv(primary), sub)                     # :306
        self.pose[1] = iso_mul(self.pose[0], self.extrinsic)                      # :307
        self.last = {"primary_update": r.update_type, "refine": st}
        return primary, sub

    def close(self):
        for t in self.trackers:
            t.close()
        if self.handeye is not None:
            self.handeye.close()
