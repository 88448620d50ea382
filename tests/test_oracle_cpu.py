"""CPU checks of the oracle (the parity checker) against independent implementations.

The reference has no runnable tests or golden vectors for this path, so
the CPU restatement is pinned here by: scipy cKDTree (exact k-NN), numpy eigh (PCA line; plus an independent transcription of Eigen's SelfAdjointEigenSolver),
numpy lstsq (plane fit), finite differences (Jacobians / gradient), closed-form SE(3) algebra
(Plus), the reference's own commented-out known-answer test re-created on synthetic clouds
(feature_registration_test.cpp:73-112: yaw 5 deg, t = (0.9, 0.4, 0.5)), and the committed
golden fixtures under tests/golden/.
"""
import math
import os

import numpy as np
import pytest

from conftest import pose_err, saes_cases

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def tiny():
    """C1-shaped scans (1800 columns) against a 100k-point map of a 40 m region: fast on one thread."""
    from lmsf import synth
    return synth.make_workload("C1", n_scans=2, map_points=100_000, n_cols=1800, road_length=20.0, radius=40.0)


def test_kdtree_exact_vs_brute_and_scipy(oracle_mod):
    from scipy.spatial import cKDTree
    rng = np.random.default_rng(5)
    pts = np.zeros((20000, 4), np.float32)
    pts[:, :3] = rng.uniform(-20, 20, (20000, 3)).astype(np.float32)
    pts[10000:10100, :3] = pts[:100, :3]              # exact duplicates -> distance ties
    pts[:, :3] = np.round(pts[:, :3] * 4) / 4         # lattice values -> many equal distances
    q = np.zeros((3000, 4), np.float32)
    q[:, :3] = rng.uniform(-20, 20, (3000, 3)).astype(np.float32)
    q[:500, :3] = pts[rng.integers(0, 20000, 500), :3]
    m = oracle_mod.KdMap(pts)
    i1, d1 = m.knn(q, 5)
    i2, d2 = oracle_mod.brute_knn(pts, q, 5)
    np.testing.assert_array_equal(i1, i2)
    np.testing.assert_array_equal(d1, d2)
    # scipy: same distance multiset (float64 distances; ties may be ordered differently)
    dd, _ = cKDTree(pts[:, :3].astype(np.float64)).query(q[:, :3].astype(np.float64), k=5)
    np.testing.assert_allclose(np.sqrt(d1.astype(np.float64)), dd, rtol=1e-5, atol=1e-5)
    # ties are broken by ascending index
    tie = d1[:, 1:] == d1[:, :-1]
    assert tie.any() and (i1[:, 1:][tie] > i1[:, :-1][tie]).all()


def _registration(oracle_mod, wl, scan_idx, solver=0):
    e, s, _, _ = oracle_mod.extract(wl.scans[scan_idx])
    reg = oracle_mod.Registration(solver)
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    return reg, e, s


def test_edge_line_fit_vs_numpy(oracle_mod, tiny):
    from lmsf import synth
    reg, e, s = _registration(oracle_mod, tiny, 0)
    rec, nn = reg.match(tiny.guess[0])
    idx = np.nonzero(rec["kind"] == 1)[0]
    assert len(idx) > 10
    for i in idx[:200]:
        P = tiny.edge_map[nn[i], :3].astype(np.float64)
        c = P.mean(0)
        w, V = np.linalg.eigh((P - c).T @ (P - c))
        u = V[:, 2]
        a, b = rec["v0"][i], rec["v1"][i]
        np.testing.assert_allclose((a + b) / 2, c, atol=1e-9)
        d = (a - b) / 0.2
        assert abs(abs(d @ u) - 1.0) < 1e-9                      # same principal direction (sign free)
        assert w[2] > 3 * w[1]                                    # linearity test passed (EdgeFeatureMatch.hpp:68)


# ---------------------------------------------------------------- Eigen SelfAdjointEigenSolver
# A second, independent transcription of Eigen 3.3's published algorithm (pure Python floats: IEEE double,
# no FMA) -- the C restatement (oracle/saes.cpp) must agree with it bit for bit, which pins the rotation
# signs, the deflation test and the sort, i.e. the eigenvector sign convention the reference's edge fit
# inherits (a = c + 0.1 u, b = c - 0.1 u: EdgeFeatureMatch.hpp:65-73).
_DBL_MIN = 2.2250738585072014e-308
_EPS = 2.220446049250313e-16


def _py_givens(p, q):
    if q == 0.0:
        return (-1.0 if p < 0.0 else 1.0), 0.0
    if p == 0.0:
        return 0.0, (1.0 if q < 0.0 else -1.0)
    if abs(p) > abs(q):
        t = q / p
        u = math.sqrt(1.0 + t * t)
        u = -u if p < 0.0 else u
        c = 1.0 / u
        return c, -t * c
    t = p / q
    u = math.sqrt(1.0 + t * t)
    u = -u if q < 0.0 else u
    s = -1.0 / u
    return -t * s, s


def _py_saes3(A):
    m = [[float(A[r][c]) if c <= r else 0.0 for c in range(3)] for r in range(3)]
    scale = 0.0
    for c in range(3):                      # column-major walk; max is order-free
        for r in range(3):
            scale = max(scale, abs(m[r][c]))
    if scale == 0.0:
        scale = 1.0
    for r in range(3):
        for c in range(r + 1):
            m[r][c] = m[r][c] / scale
    diag = [m[0][0], 0.0, 0.0]
    v1 = m[2][0] * m[2][0]
    if v1 <= _DBL_MIN:
        diag[1], diag[2] = m[1][1], m[2][2]
        sub = [m[1][0], m[2][1]]
        Q = [[1.0, 0.0, 0.0], [0.0, 1.0, 0.0], [0.0, 0.0, 1.0]]
    else:
        beta = math.sqrt(m[1][0] * m[1][0] + v1)
        ib = 1.0 / beta
        m01, m02 = m[1][0] * ib, m[2][0] * ib
        q = 2.0 * m01 * m[2][1] + m02 * (m[2][2] - m[1][1])
        diag[1] = m[1][1] + m02 * q
        diag[2] = m[2][2] - m02 * q
        sub = [beta, m[2][1] - m01 * q]
        Q = [[1.0, 0.0, 0.0], [0.0, m01, m02], [0.0, m02, -m01]]
    n, end, start, it = 3, 2, 0, 0
    while end > 0:
        for i in range(start, end):
            if abs(sub[i]) <= (abs(diag[i]) + abs(diag[i + 1])) * (2 * _EPS) or abs(sub[i]) <= _DBL_MIN:
                sub[i] = 0.0
        while end > 0 and sub[end - 1] == 0.0:
            end -= 1
        if end <= 0:
            break
        it += 1
        if it > 30 * n:
            break
        start = end - 1
        while start > 0 and sub[start - 1] != 0.0:
            start -= 1
        td = (diag[end - 1] - diag[end]) * 0.5
        e = sub[end - 1]
        mu = diag[end]
        if td == 0.0:
            mu -= abs(e)
        else:
            ax, ay = abs(td), abs(e)
            p, qp = (ax, ay / ax) if ax > ay else (ay, ax / ay)
            h = 0.0 if p == 0.0 else p * math.sqrt(1.0 + qp * qp)
            mu -= (e / (td + (1.0 if td > 0 else -1.0))) * (e / h) if e * e == 0.0 else e * e / (td + (h if td > 0 else -h))
        x, z = diag[start] - mu, sub[start]
        for k in range(start, end):
            c, s = _py_givens(x, z)
            sdk = s * diag[k] + c * sub[k]
            dkp1 = s * sub[k] + c * diag[k + 1]
            diag[k] = c * (c * diag[k] - s * sub[k]) - s * (c * sub[k] - s * diag[k + 1])
            diag[k + 1] = s * sdk + c * dkp1
            sub[k] = c * sdk - s * dkp1
            if k > start:
                sub[k - 1] = c * sub[k - 1] - s * z
            x = sub[k]
            if k < end - 1:
                z = -s * sub[k + 1]
                sub[k + 1] = c * sub[k + 1]
            for r in range(3):
                a_, b_ = Q[r][k], Q[r][k + 1]
                Q[r][k], Q[r][k + 1] = c * a_ - s * b_, s * a_ + c * b_
    if it <= 30 * n:
        for i in range(n - 1):
            k = min(range(n - i), key=lambda j: (diag[i + j], j))
            if k > 0:
                diag[i], diag[i + k] = diag[i + k], diag[i]
                for r in range(3):
                    Q[r][i], Q[r][i + k] = Q[r][i + k], Q[r][i]
    return np.array([d * scale for d in diag]), np.array(Q)


def test_saes3_matches_independent_transcription(oracle_mod):
    for A in saes_cases():
        d, V, info = oracle_mod.saes(A)
        assert info == 0
        pd, pV = _py_saes3(A)
        assert d.tobytes() == pd.tobytes() and V.tobytes() == pV.tobytes(), A


def test_saes_vs_numpy_eigh_up_to_sign(oracle_mod):
    rng = np.random.default_rng(3)
    cases = [(A, True) for A in saes_cases()[:2000]]
    for _ in range(500):                    # the GN path: 6x6 J^T J, dynamic size
        J = rng.normal(size=(40, 6)) * rng.uniform(0.01, 10, 6)
        cases.append((J.T @ J, False))
    for _ in range(200):                    # the dynamic path on 3x3 too
        P = rng.normal(size=(5, 3))
        cases.append(((P - P.mean(0)).T @ (P - P.mean(0)), False))
    for A, fixed in cases:
        d, V, info = oracle_mod.saes(A, fixed3=fixed)
        assert info == 0
        w, W = np.linalg.eigh(A)
        sc = max(abs(w).max(), 1e-300)
        np.testing.assert_allclose(d, w, rtol=0, atol=1e-13 * sc)
        assert np.all(np.diff(d) >= 0)                                   # ascending (Eigen's sort)
        np.testing.assert_allclose(V.T @ V, np.eye(len(d)), atol=1e-13)
        np.testing.assert_allclose(A @ V, V * d, atol=1e-13 * sc)
        gap = np.diff(w)
        for i in range(len(d)):              # well-separated eigenvalues: same vector up to sign
            g = min(gap[i - 1] if i > 0 else np.inf, gap[i] if i < len(gap) else np.inf)
            if g > 1e-6 * sc:
                assert abs(abs(V[:, i] @ W[:, i]) - 1.0) < 1e-8


def test_saes_sign_convention(oracle_mod):
    """What the published algorithm implies for the signs: an already-diagonal matrix keeps +unit
    eigenvectors (only column swaps by the sort); a tridiagonal 3x3 starts from Q = I; otherwise Q
    starts from the Householder [1 0 0; 0 m01 m02; 0 m02 -m01], so column 0 of the tridiagonal basis
    stays e0 -- and the QR rotations fix the rest, pinned by the transcription test above."""
    d, V, _ = oracle_mod.saes(np.diag([3.0, 1.0, 2.0]))
    assert list(d) == [1.0, 2.0, 3.0]
    assert V.tolist() == [[0.0, 0.0, 1.0], [1.0, 0.0, 0.0], [0.0, 1.0, 0.0]]
    d, V, _ = oracle_mod.saes(np.diag([5.0, -1.0, 7.0, 2.0, 0.5, 3.0]), fixed3=False)
    assert list(d) == [-1.0, 0.5, 2.0, 3.0, 5.0, 7.0]
    assert sorted(V.reshape(-1).tolist()) == [0.0] * 30 + [1.0] * 6
    # a 2x2-block rotation: [[2, 1], [1, 2]] (+ an isolated 5): Eigen's QR step gives the eigenvectors
    # (1, -1)/sqrt2 for 1 and (1, 1)/sqrt2 for 3 with these signs
    d, V, _ = oracle_mod.saes(np.array([[2.0, 1.0, 0.0], [1.0, 2.0, 0.0], [0.0, 0.0, 5.0]]))
    pd, pV = _py_saes3([[2.0, 1.0, 0.0], [1.0, 2.0, 0.0], [0.0, 0.0, 5.0]])
    assert V.tobytes() == pV.tobytes()
    np.testing.assert_allclose(d, [1.0, 3.0, 5.0], atol=1e-15)
    r = math.sqrt(0.5)
    np.testing.assert_allclose(np.abs(V), [[r, r, 0], [r, r, 0], [0, 0, 1]], atol=1e-15)


def test_edge_records_carry_saes3_direction(oracle_mod, tiny):
    """The oracle's edge records are a = 0.1 u + c, b = -0.1 u + c with u = column 2 of the restated
    SelfAdjointEigenSolver<Matrix3d> of the 5-point covariance, bit for bit (EdgeFeatureMatch.hpp:44-73)."""
    reg, e, s = _registration(oracle_mod, tiny, 0)
    rec, nn = reg.match(tiny.guess[0])
    idx = np.nonzero(rec["kind"] == 1)[0]
    assert len(idx) > 10
    for i in idx[:300]:
        P = [[float(v) for v in tiny.edge_map[j, :3]] for j in nn[i]]
        c = [0.0, 0.0, 0.0]
        for p in P:
            c = [c[k] + p[k] for k in range(3)]
        c = [v / 5.0 for v in c]
        cov = [[0.0] * 3 for _ in range(3)]
        for p in P:
            ev = [p[k] - c[k] for k in range(3)]
            for r in range(3):
                for q in range(3):
                    cov[r][q] = cov[r][q] + ev[r] * ev[q]
        d, V = _py_saes3(cov)
        assert d[2] > 3 * d[1]
        a = [0.1 * V[k][2] + c[k] for k in range(3)]
        b = [-0.1 * V[k][2] + c[k] for k in range(3)]
        assert np.array(a).tobytes() == rec["v0"][i].tobytes() and np.array(b).tobytes() == rec["v1"][i].tobytes()


def test_surf_plane_fit_vs_lstsq(oracle_mod, tiny):
    from lmsf import synth
    reg, e, s = _registration(oracle_mod, tiny, 1)
    rec, nn = reg.match(tiny.guess[1])
    ne = len(e)
    idx = ne + np.nonzero(rec["kind"][ne:] == 2)[0]
    assert len(idx) > 1000
    for i in idx[:500]:
        A = tiny.surf_map[nn[i], :3].astype(np.float64)
        x, *_ = np.linalg.lstsq(A, -np.ones(5), rcond=None)
        D = 1.0 / np.linalg.norm(x)
        n = x / np.linalg.norm(x)
        got_n, got_D = rec["v0"][i], rec["v1"][i][0]
        if got_n @ n < 0:
            n, D = -n, -D
        np.testing.assert_allclose(got_n, n, atol=1e-7)
        assert abs(got_D - D) < 1e-6 * max(1.0, abs(D))
        assert np.all(np.abs(A @ got_n + got_D) <= 0.2)          # plane validity (surfFeatureMatch.hpp:57-65)


def _rotvec_to_mat(w):
    th = np.linalg.norm(w)
    if th < 1e-15:
        return np.eye(3)
    k = w / th
    K = np.array([[0, -k[2], k[1]], [k[2], 0, -k[0]], [-k[1], k[0], 0]])
    return np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K


def test_pose_plus_closed_form(oracle_mod):
    from lmsf import synth
    rng = np.random.default_rng(1)
    for _ in range(50):
        x = np.concatenate([synth.axis_angle_quat(rng.normal(0, 1, 3)), rng.normal(0, 10, 3)])
        d = np.concatenate([rng.normal(0, 0.3, 3), rng.normal(0, 1, 3)])
        out = oracle_mod.pose_plus(x, d)
        w, u = d[:3], d[3:]
        Rd = _rotvec_to_mat(w)
        th = np.linalg.norm(w)
        K = np.array([[0, -w[2], w[1]], [w[2], 0, -w[0]], [-w[1], w[0], 0]])
        J = np.eye(3) + (1 - math.cos(th)) / th ** 2 * K + (th - math.sin(th)) / th ** 3 * K @ K
        np.testing.assert_allclose(synth.quat_to_mat(out[:4]), Rd @ synth.quat_to_mat(x[:4]), atol=1e-12)
        np.testing.assert_allclose(out[4:], Rd @ x[4:] + J @ u, atol=1e-10)
    # small-angle branch (theta < 1e-10): Taylor factor, J = dq.matrix()
    out = oracle_mod.pose_plus(np.array([0, 0, 0, 1.0, 1, 2, 3]), np.array([1e-12, 0, 0, 0.5, 0, 0]))
    np.testing.assert_allclose(out[4:], [1.5, 2 - 3e-12, 3 + 2e-12], atol=1e-14)


def test_gradient_and_hessian_vs_finite_differences(oracle_mod, tiny):
    reg, e, s = _registration(oracle_mod, tiny, 0)
    x0 = tiny.guess[0]
    rec, _ = reg.match(x0)
    rec = rec[rec["kind"] > 0]
    P = oracle_mod.eval_records(rec, x0)
    g = P[22:28]
    h = 1e-7
    num = np.zeros(6)
    for k in range(6):
        dp, dm = np.zeros(6), np.zeros(6)
        dp[k], dm[k] = h, -h
        cp = oracle_mod.eval_records(rec, oracle_mod.pose_plus(x0, dp))[0]
        cm = oracle_mod.eval_records(rec, oracle_mod.pose_plus(x0, dm))[0]
        num[k] = (cp - cm) / (2 * h)
    np.testing.assert_allclose(g, num, rtol=2e-4, atol=1e-6 * np.abs(g).max())
    assert P[28] == len(rec)
    H = np.zeros((6, 6))
    k = 1
    for i in range(6):
        for j in range(i, 6):
            H[i, j] = H[j, i] = P[k]
            k += 1
    assert np.all(np.linalg.eigvalsh(H) > 0)                      # Gauss-Newton Hessian is SPD


def test_extraction_invariants(oracle_mod, tiny):
    scan = tiny.scans[0]
    e, s, ei, si = oracle_mod.extract(scan)
    assert len(e) > 0 and len(s) > 0.8 * len(scan)
    assert len(set(ei.tolist()) | set(si.tolist())) == len(ei) + len(si)   # each point at most once
    np.testing.assert_array_equal(e, scan[ei])
    np.testing.assert_array_equal(s, scan[si])
    # deterministic
    e2, s2, ei2, si2 = oracle_mod.extract(scan)
    np.testing.assert_array_equal(ei, ei2)
    np.testing.assert_array_equal(si, si2)
    # at most 20 edges per sector: 16 rings x 6 sectors
    assert len(e) <= 16 * 6 * 20
    # range gate 2 <= sqrt(x^2 + y^2) <= 80 (float expression as in splitScan)
    d = np.sqrt((scan[:, 0] * scan[:, 0] + scan[:, 1] * scan[:, 1]).astype(np.float64))
    used = np.concatenate([ei, si])
    assert np.all((d[used] >= 2.0) & (d[used] <= 80.0))
    # no bad-point removal and threshold 0.1 -> more edges
    e3, *_ = oracle_mod.extract(scan, remove_bad_points=False, edge_threshold=0.1)
    assert len(e3) >= len(e)
    # empty / tiny inputs
    e4, s4, _, _ = oracle_mod.extract(np.zeros((0, 4), np.float32))
    assert len(e4) == len(s4) == 0
    e5, s5, _, _ = oracle_mod.extract(scan[:50])
    assert len(e5) == 0 and len(s5) == 0


@pytest.mark.parametrize("solver", [0, 1])
def test_known_answer_transform(oracle_mod, tiny, solver):
    """feature_registration_test.cpp:73-112 re-created: target = source transformed by yaw 5 deg,
    t = (0.9, 0.4, 0.5); solving from identity recovers the inverse transform."""
    from lmsf import synth
    c = tiny.truth[0][4:]
    near = lambda m: m[np.linalg.norm(m[:, :3] - c, axis=1) < 30.0]
    edge_src, surf_src = near(tiny.edge_map), near(tiny.surf_map)
    T = np.concatenate([synth.quat_from_rpy(0, 0, math.radians(5)), [0.9, 0.4, 0.5]])
    reg = oracle_mod.Registration(solver)
    reg.set_map(1, edge_src)
    reg.set_map(2, surf_src)
    rng = np.random.default_rng(3)
    reg.set_scan(1, synth.transform_points(T, edge_src[rng.permutation(len(edge_src))[:2000]]))
    reg.set_scan(2, synth.transform_points(T, surf_src[rng.permutation(len(surf_src))[:20000]]))
    reg.set_fixed_schedule(True)
    # GN rotates by |dtheta|/2 per step (AngleAxis(norm/2, ...), edgeSurfFeatureRegistration.hpp:317),
    # so it needs more iterations and its convergence gate (:326) stops ~3e-3 rad short
    reg.set_max_iterations(10 if solver == 0 else 30)
    x, tr, st = reg.solve(np.array([0, 0, 0, 1.0, 0, 0, 0]), trace_cap=32)
    R = synth.quat_to_mat(T[:4])
    inv = np.concatenate([synth.quat_from_rpy(0, 0, -math.radians(5)), -R.T @ T[4:]])
    dt, dr = pose_err(x, inv)
    if solver == 0:
        assert dt < 2e-3 and dr < 2e-4, (dt, dr, st.termination)
    else:
        assert st.termination == 5 and dt < 5e-3 and dr < 5e-3, (dt, dr, st.termination)


def test_registration_converges_and_schedule(oracle_mod, tiny):
    reg, e, s = _registration(oracle_mod, tiny, 0)
    x, tr, st = reg.solve(tiny.guess[0])       # reference decay: 10 -> 9 outer iterations
    assert st.outer_iterations == 9 and len(tr) == 9
    dt, dr = pose_err(x, tiny.truth[0])
    assert dt < 0.05 and dr < 0.01
    x2, tr2, st2 = reg.solve(tiny.guess[0])
    assert st2.outer_iterations == 8
    reg.set_max_iterations(2)
    assert reg.solve(tiny.guess[0])[2].outer_iterations == 2    # no decrement at 2


def test_oracle_tracker_follows_trajectory(oracle_mod, sequence_workload):
    """LidarTrackerLocalMap restated: first scan seeds the map, constant-velocity prediction,
    keyframe gate (0.3 m / 0.1 rad / 10 s), sliding-window local map."""
    import tracker as OT
    from conftest import mat_err, relative_truth
    wl = sequence_workload
    rel = relative_truth(wl.truth)
    tr = OT.Tracker(window_frames=3)
    kinds = []
    for i, scan in enumerate(wl.scans):
        e, s, _, _ = oracle_mod.extract(scan, n_scans=wl.n_scans)
        d, typ, st = tr.solve(e, s, wl.dt * i)
        kinds.append(typ)
        dt, dr = mat_err(tr.curr, rel[i])
        assert dt < 0.05 and dr < 0.01, (i, dt, dr)
    # 0.25 m per scan: every other scan crosses the 0.3 m keyframe gate
    assert kinds[0] == 1 and 0 in kinds[1:] and 1 in kinds[1:]
    assert len(tr.win[2]) == 3                                      # window capped
    assert np.allclose(d, tr.motion) and np.array_equal(tr.prev, tr.curr)


def test_golden_fixtures_reproduced(oracle_mod):
    """Fixtures generated by tests/golden/make_golden.py (oracle outputs + numpy cross-checks)."""
    path = os.path.join(GOLDEN, "c1_small.npz")
    assert os.path.exists(path), "run tests/golden/make_golden.py"
    g = np.load(path)
    e, s, ei, si = oracle_mod.extract(g["scan"])
    np.testing.assert_array_equal(ei, g["edge_src"])
    np.testing.assert_array_equal(si, g["surf_src"])
    reg = oracle_mod.Registration()
    reg.set_map(1, g["edge_map"])
    reg.set_map(2, g["surf_map"])
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    rec, nn = reg.match(g["guess"])
    np.testing.assert_array_equal(nn, g["nn"])
    np.testing.assert_array_equal(rec["kind"], g["kind"])
    np.testing.assert_array_equal(rec["v0"], g["v0"])
    np.testing.assert_array_equal(rec["v1"], g["v1"])
    reg.set_fixed_schedule(True)
    reg.set_max_iterations(5)
    x, tr, st = reg.solve(g["guess"])
    np.testing.assert_allclose(tr, g["trace"], rtol=0, atol=1e-12)
    # independent numpy pins stored in the fixture
    np.testing.assert_allclose(g["np_edge_dir_dot"], 1.0, atol=1e-9)
    np.testing.assert_allclose(g["np_plane_err"], 0.0, atol=1e-7)


def _numpy_voxel(p, leaf):
    """Independent numpy restatement of pcl::VoxelGrid (float voxel coords, z-major index order)."""
    inv = np.float32(1.0) / np.float32(leaf)
    c = np.floor(p[:, :3].astype(np.float32) * inv).astype(np.int64)
    c -= c.min(0)
    d = c.max(0) + 1
    key = c[:, 0] + c[:, 1] * d[0] + c[:, 2] * d[0] * d[1]
    order = np.lexsort((np.arange(len(p)), key))
    ks = key[order]
    starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
    out = []
    for a, b in zip(starts, np.r_[starts[1:], len(p)]):
        s = np.zeros(4)
        for i in order[a:b]:
            s += p[i].astype(np.float64)      # sequential double sums, input order inside a voxel
        out.append((s / (b - a)).astype(np.float32))
    return np.array(out, np.float32).reshape(-1, 4)


def test_oracle_voxel_filter(oracle_mod):
    rng = np.random.default_rng(4)
    p = np.concatenate([rng.uniform(-20, 20, (3000, 3)), rng.random((3000, 1))], 1).astype(np.float32)
    p[:500, :3] = np.round(p[:500, :3] * 2.5) / 2.5          # points exactly on voxel boundaries
    for leaf in (0.2, 0.4, 1.0, 3.0):
        got = oracle_mod.voxel_filter(p, leaf)
        assert got.tobytes() == _numpy_voxel(p, leaf).tobytes()
    assert len(oracle_mod.voxel_filter(p[:0], 0.4)) == 0
    assert oracle_mod.voxel_filter(p[:1], 0.4).tobytes() == p[:1].tobytes()
    # PCL refuses when the voxel index would overflow int32: input returned unchanged
    far = np.array([[0, 0, 0, 0], [1e4, 1e4, 1e4, 1]], np.float32)
    assert oracle_mod.voxel_filter(far, 0.01).tobytes() == far.tobytes()


def test_oracle_alignment_score_vs_scipy(oracle_mod, tiny):
    """AlignmentScore restatement (oracle/align.py) vs scipy cKDTree 1-NN on the same float inputs."""
    import sys
    from scipy.spatial import cKDTree
    import align as OA
    from conftest import pose_matrix
    wl = tiny
    e, s, _, _ = oracle_mod.extract(wl.scans[0])
    T = pose_matrix(wl.truth[0]).astype(np.float32)
    for thresh, ratio in ((0.1, 0.6), (1.0, 0.6), (0.1, 0.0)):
        score, overlap = OA.alignment_score(wl.surf_map, s, T, thresh, ratio)
        q = OA.transform_f32(s, T)
        d, _ = cKDTree(wl.surf_map[:, :3].astype(np.float64)).query(q[:, :3].astype(np.float64), k=1)
        inl = d * d <= thresh
        assert abs(overlap - inl.mean()) < 2e-3                     # float vs double distances at the edge
        if overlap > ratio:
            assert abs(score - (d[inl] ** 2).mean()) < 1e-4 * max(1.0, score)
        else:
            assert score == sys.float_info.max
    assert OA.alignment_score(wl.surf_map, s[:0], T, 0.1, 0.6) == (sys.float_info.max, 0.0)


def _python_rotary(pts, period=0.1):
    """Independent line-by-line restatement of RotaryLidarPreProcess::Process
    (RotaryLidar_preprocessing.hpp:31-91) with float32 variables and double M_PI expressions."""
    f32 = np.float32

    def neg_atan2(y, x):
        return f32(-math.atan2(float(y), float(x)))

    start = neg_atan2(pts[0, 1], pts[0, 0])
    end = f32(float(neg_atan2(pts[-1, 1], pts[-1, 0])) + 2 * math.pi)
    if float(f32(end - start)) > 3 * math.pi:
        end = f32(float(end) - 2 * math.pi)
    elif float(f32(end - start)) < math.pi:
        end = f32(float(end) + 2 * math.pi)
    half = False
    out = np.empty(len(pts), np.float32)
    for i in range(len(pts)):
        ori = neg_atan2(pts[i, 1], pts[i, 0])
        if not half:
            if float(ori) < float(start) - math.pi / 2:
                ori = f32(float(ori) + 2 * math.pi)
            elif float(ori) > float(start) + math.pi * 3 / 2:
                ori = f32(float(ori) - 2 * math.pi)
            if float(f32(ori - start)) > math.pi:
                half = True
        else:
            ori = f32(float(ori) + 2 * math.pi)
            if float(ori) < float(end) - math.pi * 3 / 2:
                ori = f32(float(ori) + 2 * math.pi)
            elif float(ori) > float(end) + math.pi / 2:
                ori = f32(float(ori) - 2 * math.pi)
        out[i] = f32(f32(f32(ori - start) / f32(end - start)) * f32(period))
    return out


def test_oracle_ingest_pointcloud2(oracle_mod, tiny):
    """PointCloud2 decode + removeNaN + rotary relative time + distance filter (oracle/ingest.cpp)
    vs numpy and a line-by-line Python restatement of RotaryLidar_preprocessing.hpp."""
    from lmsf import synth
    org = synth.make_scan(tiny.scene, tiny.truth[0], 11, n_cols=900, organized=True, clockwise=True)
    valid = np.isfinite(org[:, :3]).all(1)
    assert (~valid).any() and valid.sum() > 0.8 * len(org)
    msg = synth.to_pointcloud2(org)
    got = oracle_mod.ingest(msg, len(org), scan_period=0.0)                    # decode + removeNaN only
    assert got.tobytes() == org[valid].tobytes()
    rot = oracle_mod.ingest(msg, len(org))
    np.testing.assert_array_equal(rot[:, :3], org[valid, :3])
    assert rot[:, 3].tobytes() == _python_rotary(org[valid]).tobytes()
    assert rot[0, 3] == 0.0 and 0.099 < rot[:, 3].max() <= 0.1001            # one revolution = one period
    near, far = 5.0, 40.0
    dist = oracle_mod.ingest(msg, len(org), scan_period=0.0, distance_near=near, distance_far=far)
    v = org[valid]
    d = np.sqrt((v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1] + v[:, 2] * v[:, 2]).astype(np.float32)).astype(np.float64)
    assert dist.tobytes() == v[(d > near) & (d < far)].tobytes()
    assert len(oracle_mod.ingest(msg[:0], 0)) == 0


def test_oracle_libm_overload_choice(oracle_mod):
    """libm_float selects which overloads the reference's unqualified sqrt / atan2 on float arguments bind
    to (FX:223-224, :247-252, :300-301; lmsf_config::libm_float).  A point with x*x + y*y = 6400 + 2^-11 in
    float: sqrt in double is 80.000003 > max_distance 80 (rejected, GCC 5 / kinetic), sqrtf rounds to
    80.0f (kept, GCC >= 6 with <math.h>) -- the two toolchains extract different features."""
    from conftest import libm_probe_scan
    scan = libm_probe_scan()
    x, y = np.float32(80.0), np.float32(0.0221)
    s = np.float32(x * x) + np.float32(y * y)
    assert s == np.float32(6400.0 + 2.0 ** -11)
    assert np.sqrt(np.float64(s)) > 80.0 and np.sqrt(s) == np.float32(80.0)
    e0, s0, ei0, si0 = oracle_mod.extract(scan)
    e1, s1, ei1, si1 = oracle_mod.extract(scan, libm_float=True)
    assert 900 not in set(ei0) | set(si0)                    # double sqrt: out of range
    assert 900 in set(ei1) | set(si1)                        # float sqrt: kept, becomes a feature
