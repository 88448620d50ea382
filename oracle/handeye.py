"""TEST INFRASTRUCTURE ONLY -- CPU restatement of Algorithm::HandEyeCalibrationBase.

Follows INC/Algorithm/calibration/handeye_calibration_base.hpp (INC = src/MultiSensorFusionEstimator3D/
include): AddPose :71-106, CalibExRotation :113-148 (SVD of the stacked 4N x 4 matrix of
Math::QuanternionLeftProductMatrix(q_p) - QuanternionRightProductMatrix(q_s), INC/Math.hpp:79-95),
calibExTranslationNonPlanar :160-184, checkScrewMotion :207-242, Slam3D::Pose products
(INC/Common/pose.hpp:59-98).  Uses numpy's LAPACK SVD on the full stacked matrices (the reference
uses Eigen::JacobiSVD), so it is independent of the library's normal-matrix formulation.
Parity vs Eigen: unpinned.
"""
from __future__ import annotations

import heapq
import math

import numpy as np


def q_from_R(m):
    """Eigen Quaterniond(Matrix3d) -> (x, y, z, w)."""
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


def qmul(a, b):
    ax, ay, az, aw = a
    bx, by, bz, bw = b
    return np.array([aw * bx + ax * bw + ay * bz - az * by, aw * by + ay * bw + az * bx - ax * bz,
                     aw * bz + az * bw + ax * by - ay * bx, aw * bw - ax * bx - ay * by - az * bz])


def R_of(q):
    x, y, z, w = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


class Pose:
    def __init__(self, q=(0, 0, 0, 1), t=(0, 0, 0)):
        q = np.asarray(q, dtype=np.float64)
        self.q = q / np.linalg.norm(q)
        self.t = np.asarray(t, dtype=np.float64)

    @staticmethod
    def from_matrix(T):
        return Pose(q_from_R(T[:3, :3]), T[:3, 3])

    def __mul__(self, o):
        return Pose(qmul(self.q, o.q), R_of(self.q) @ o.t + self.t)

    def angle_axis(self):
        x, y, z, w = self.q
        n = math.sqrt(x * x + y * y + z * z)
        if n == 0:
            return 0.0, np.array([1.0, 0.0, 0.0])
        ang = 2 * math.atan2(n, abs(w))
        if w < 0:
            n = -n
        return ang, np.array([x, y, z]) / n


def L_mat(q):
    x, y, z, w = q
    return np.array([[w, -x, -y, -z], [x, w, -z, y], [y, z, w, -x], [z, -y, x, w]])


def R_mat(q):
    x, y, z, w = q
    return np.array([[w, -x, -y, -z], [x, w, z, -y], [y, -z, w, x], [z, y, -x, w]])


class HandEye:
    N_POSE = 300
    EPS_R, EPS_T, ROT_COV_THRE = 0.05, 0.1, 0.25

    def __init__(self):
        self.heap = []          # (-w, seq, idx): top = largest w
        self.seq = 0
        self.fresh = []
        self.storage = []
        self.Q = np.zeros((self.N_POSE * 4, 4))
        self.acc_p, self.acc_s = Pose(), Pose()
        self.ext_q, self.ext_t, self.done = np.array([0, 0, 0, 1.0]), np.zeros(3), False

    def _check(self, p, s):
        ap, xp = p.angle_axis()
        as_, xs = s.angle_axis()
        if abs(ap - as_) > self.EPS_R or abs(p.t @ xp - s.t @ xs) > self.EPS_T:
            self.acc_p, self.acc_s = Pose(), Pose()
            return False
        self.acc_p = self.acc_p * p
        self.acc_s = self.acc_s * s
        return self.acc_p.angle_axis()[0] > 0 or self.acc_s.angle_axis()[0] > 0

    def add_pose(self, Tp, Ts):
        if not self._check(Pose.from_matrix(Tp), Pose.from_matrix(Ts)):
            return False
        pr = (self.acc_p, self.acc_s)
        if len(self.storage) < self.N_POSE:
            idx = len(self.storage)
            self.storage.append(pr)
        else:
            idx = heapq.heappop(self.heap)[2]
            self.storage[idx] = pr
        self.fresh.append((idx, pr))
        heapq.heappush(self.heap, (-pr[0].q[3], self.seq, idx))
        self.seq += 1
        self.acc_p, self.acc_s = Pose(), Pose()
        return len(self.storage) >= 3

    def calib_rotation(self):
        for idx, (p, s) in self.fresh:
            self.Q[4 * idx:4 * idx + 4] = L_mat(p.q) - R_mat(s.q)
        self.fresh = []
        _, sv, Vt = np.linalg.svd(self.Q, full_matrices=False)
        x = Vt[3].copy()                     # [w, x, y, z]
        if x[0] < 0:
            x = -x
        if sv[2] > self.ROT_COV_THRE:
            q = np.array([x[1], x[2], x[3], x[0]])
            self.ext_q = q / np.linalg.norm(q)
            return True, sv
        return False, sv

    def calib_translation(self):
        A = np.zeros((3 * len(self.storage), 3))
        b = np.zeros(3 * len(self.storage))
        Rx = R_of(self.ext_q)
        for i, (p, s) in enumerate(self.storage):
            A[3 * i:3 * i + 3] = R_of(p.q) - np.eye(3)
            b[3 * i:3 * i + 3] = Rx @ s.t - p.t
        self.ext_t = np.linalg.lstsq(A, b, rcond=None)[0]
        self.done = True
        return True

    def result(self):
        if not self.done:
            return None
        T = np.eye(4)
        T[:3, :3] = R_of(self.ext_q)
        T[:3, 3] = self.ext_t
        return T
