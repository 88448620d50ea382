"""TEST INFRASTRUCTURE ONLY -- CPU restatement of Slam3D::PointCloudAlignmentEvaluate::AlignmentScore
(REG/alignEvaluate.hpp:55-87, REG = src/MultiSensorFusionEstimator3D/include/Algorithm/PointClouds/
registration): pcl::transformPointCloud with an Eigen::Matrix4f (float arithmetic, m0 x + m1 y +
m2 z + m3 left to right), exact 1-NN on the oracle kd-tree (float L2), inliers nn_d2 <= thresh
(float promoted to double), sequential double sum.  Parity vs PCL/FLANN: unpinned.
"""
from __future__ import annotations

import sys

import numpy as np

import oracle as O


def transform_f32(pts, T):
    T = np.asarray(T, dtype=np.float32)
    x, y, z = (np.asarray(pts[:, k], dtype=np.float32) for k in range(3))
    out = np.array(pts, dtype=np.float32, copy=True)
    for r in range(3):
        out[:, r] = T[r, 0] * x + T[r, 1] * y + T[r, 2] * z + T[r, 3]
    return out


def alignment_score(target, cloud, relpose, inlier_thresh, inlier_ratio_thresh, tree=None):
    if len(cloud) == 0:                                   # :61
        return sys.float_info.max, 0.0
    tree = tree or O.KdMap(target)
    q = transform_f32(cloud, relpose)
    _, d2 = tree.knn(q, 1)
    fitness, nr = 0.0, 0
    for v in d2[:, 0]:                                     # :69-79
        if float(v) <= inlier_thresh:
            fitness += float(v)
            nr += 1
    overlap = nr / len(q)                                  # :81
    if overlap > inlier_ratio_thresh:                      # :83-86
        return fitness / nr, overlap
    return sys.float_info.max, overlap
