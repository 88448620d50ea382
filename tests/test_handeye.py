"""Dual-LiDAR extrinsic initialisation (C3, phase 0): lmsf_handeye (host code in liblmsf_hip.so,
no GPU needed) against oracle/handeye.py and against the known extrinsic.

The motions are synthetic screw motions A_i of the primary LiDAR and B_i = X^-1 A_i X of the sub
LiDAR for the reference's PS-Calib extrinsic X (config/MultiLidar_system/
loam_feature_multi_lidar_system.yaml:73-74), with rotations about varied axes (a car's planar yaw
alone leaves the rotation unobservable, the reference's rot_cov threshold then refuses)."""
import numpy as np
import pytest


def _T(q, t):
    from lmsf import synth
    T = np.eye(4)
    T[:3, :3] = synth.quat_to_mat(q)
    T[:3, 3] = t
    return T


def _motions(n, seed, planar=False, noise=0.0):
    from lmsf import synth
    rng = np.random.default_rng(seed)
    X = _T(*np.split(synth.unit_extrinsic(synth.DUAL_EXTRINSIC), [4]))
    Xi = np.linalg.inv(X)
    out = []
    for _ in range(n):
        axis = np.array([0.0, 0.0, 1.0]) if planar else rng.normal(size=3)
        axis /= np.linalg.norm(axis)
        A = _T(synth.axis_angle_quat(axis * rng.uniform(0.05, 0.4)), rng.normal(0, 0.5, 3))
        B = Xi @ A @ X
        if noise:
            B = B @ _T(synth.axis_angle_quat(rng.normal(0, noise, 3)), rng.normal(0, noise, 3))
        out.append((A, B))
    return X, out


@pytest.fixture(scope="module")
def lib():
    from lmsf import _lib
    _lib.load()
    return _lib


def _run(lib, motions):
    import handeye as OH
    h, o = lib.HandEye(), OH.HandEye()
    log = []
    for A, B in motions:
        ok_h, ok_o = h.add_pose(A, B), o.add_pose(A, B)
        assert ok_h == ok_o
        if ok_h:
            rh, svh = h.calib_rotation()
            ro, svo = o.calib_rotation()
            # sqrt(eig(Q^T Q)) resolves a ~0 singular value only to sqrt(eps)*|Q| ~ 1e-8
            np.testing.assert_allclose(svh, svo, rtol=1e-9, atol=1e-7)
            assert rh == ro
            if rh:
                assert h.calib_translation() and o.calib_translation()
                log.append((h.result(), o.result()))
    return h, o, log


def test_handeye_recovers_extrinsic(lib):
    X, motions = _motions(12, 5)
    h, o, log = _run(lib, motions)
    assert log, "rotation never observable"
    Th, To = log[-1]
    np.testing.assert_allclose(Th, To, atol=1e-9)
    np.testing.assert_allclose(Th, X, atol=1e-9)
    assert h.pair_count() == 12


def test_handeye_noisy_and_screw_rejection(lib):
    X, motions = _motions(30, 7, noise=2e-3)
    # a pair violating the screw-motion invariants (different rotation angles) is refused
    A, B = motions[3]
    bad = B.copy()
    bad[:3, :3] = B[:3, :3] @ _T(np.array([0, 0, np.sin(0.05), np.cos(0.05)]), np.zeros(3))[:3, :3]
    motions.insert(4, (A, bad))
    h, o, log = _run(lib, motions)
    Th, To = log[-1]
    np.testing.assert_allclose(Th, To, atol=1e-7)
    assert np.linalg.norm(Th[:3, 3] - X[:3, 3]) < 0.05
    assert h.pair_count() == 30


def test_handeye_planar_motion_is_refused(lib):
    """Yaw-only motion: 2nd-smallest singular value stays below 0.25 (rotation unobservable)."""
    X, motions = _motions(20, 9, planar=True)
    h, o, log = _run(lib, motions)
    assert not log
    assert h.result() is None
