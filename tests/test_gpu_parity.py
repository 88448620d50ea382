"""GPU parity: liblmsf_hip.so (through its C ABI) against the CPU restatement in oracle/.

Bars (DESIGN.md "Parity"):
* feature extraction and correspondence search are index work -> bit-exact (same points, same
  order, same neighbour indices, same line/plane doubles);
* the 29-double normal-equation packet differs only by summation order -> rel 1e-9;
* poses per outer iteration <= 1e-4 m / 1e-4 rad (north_star tolerance).
"""

import numpy as np
import pytest

from conftest import assert_captured_records, mat_err, pose_err, saes_cases

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4


@pytest.fixture(scope="module")
def lib():
    from lmsf import _lib
    _lib.load()
    return _lib


def _ctx(lib, **kw):
    cfg = dict(max_batch=4, max_scan_points=70000, max_features=70000)
    cfg.update(kw)
    return lib.Context(**cfg)


def _features(oracle_mod, scan):
    e, s, ei, si = oracle_mod.extract(scan)
    return e, s


def test_extract_bitexact(lib, oracle_mod, small_workload):
    ctx = _ctx(lib)
    for scan in small_workload.scans:
        e, s, ei, si = oracle_mod.extract(scan)
        ne, ns = ctx.extract(scan)
        assert (ne, ns) == (len(e), len(s))
        ge, gei = ctx.copy_features(lib.EDGE)
        gs, gsi = ctx.copy_features(lib.SURF)
        np.testing.assert_array_equal(gei, ei)
        np.testing.assert_array_equal(gsi, si)
        assert ge.tobytes() == e.tobytes()
        assert gs.tobytes() == s.tobytes()


def test_eigen_selfadjoint_device_bitexact(lib, oracle_mod):
    """The kernels' SelfAdjointEigenSolver restatement (devmath.h saes3 / saesx<6>) against the oracle's
    (saes.cpp), bit for bit: eigenvalues, eigenvectors (signs included) and the convergence flag."""
    ctx = _ctx(lib, max_batch=1)
    A3 = np.array(saes_cases())
    d, v, info = ctx.eigen_selfadjoint(A3)
    for i, A in enumerate(A3):
        od, ov, oi = oracle_mod.saes(A)
        assert info[i] == oi and d[i].tobytes() == od.tobytes() and v[i].tobytes() == ov.tobytes(), A
    rng = np.random.default_rng(7)
    A6 = []
    for _ in range(2000):
        J = rng.normal(size=(30, 6)) * rng.uniform(0.01, 10, 6)
        A6.append(J.T @ J)
    A6 += [np.diag([5.0, -1.0, 7.0, 2.0, 0.5, 3.0]), np.zeros((6, 6)), np.ones((6, 6))]
    A6 = np.array(A6)
    d, v, info = ctx.eigen_selfadjoint(A6)
    for i, A in enumerate(A6):
        od, ov, oi = oracle_mod.saes(A, fixed3=False)
        assert info[i] == oi and d[i].tobytes() == od.tobytes() and v[i].tobytes() == ov.tobytes(), A


def test_prefetch_features_bitexact(lib, oracle_mod, small_workload):
    """lmsf_prefetch_features: the next scan extracted beside a solve and adopted by the extract call of the
    same buffer gives the oracle's features and source indices; a prefetch of another buffer is discarded
    and the extract of the buffer asked for is exact; a solve between prefetch and adoption is unchanged."""
    import torch
    wl = small_workload
    scans = [torch.from_numpy(sc).to("cuda:0") for sc in wl.scans]
    ref = _ctx(lib, max_batch=1)
    ref.set_map(lib.EDGE, wl.edge_map)
    ref.set_map(lib.SURF, wl.surf_map)
    ctx = _ctx(lib, max_batch=1)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.extract(scans[0])
    for i in range(1, len(scans)):
        ctx.prefetch(scans[i])
        ref.extract(scans[i - 1])
        assert ctx.solve(wl.guess[i - 1])[0].tobytes() == ref.solve(wl.guess[i - 1])[0].tobytes()   # beside it
        ne, ns = ctx.extract(scans[i])                                                   # adopted
        e, s, ei, si = oracle_mod.extract(wl.scans[i])
        assert (ne, ns) == (len(e), len(s))
        ge, gei = ctx.copy_features(lib.EDGE)
        gs, gsi = ctx.copy_features(lib.SURF)
        np.testing.assert_array_equal(gei, ei)
        np.testing.assert_array_equal(gsi, si)
        assert ge.tobytes() == e.tobytes() and gs.tobytes() == s.tobytes()
    # an adopted extraction did not load raw slot 0: a batch launch is refused, not run on a stale scan
    # (ADVICE r03); a plain extraction loads it again
    with pytest.raises(lib.LmsfError) as ei:
        ctx.batch_run(np.stack([wl.guess[0]]))
    assert ei.value.code == lib.ERR_STATE
    ctx.prefetch(scans[0])                      # not adopted: another buffer is extracted
    other = scans[1].clone()
    ctx.extract(other)
    e, s, _, _ = oracle_mod.extract(wl.scans[1])
    assert ctx.copy_features(lib.EDGE)[0].tobytes() == e.tobytes()
    assert ctx.copy_features(lib.SURF)[0].tobytes() == s.tobytes()
    _, st = ctx.batch_run(np.stack([wl.guess[1]]))   # a plain extraction loaded slot 0
    assert st[0].surf_matches > 0
    # destroyed right after a prefetch: the worker and the prefetch stream are drained before any buffer is
    # freed; the device stays usable
    for _ in range(3):
        tmp = _ctx(lib, max_batch=1)
        tmp.set_map(lib.EDGE, wl.edge_map)
        tmp.set_map(lib.SURF, wl.surf_map)
        tmp.extract(scans[0])
        tmp.prefetch(scans[1])
        tmp.close()
    ne, ns = ctx.extract(scans[2])
    e, s, _, _ = oracle_mod.extract(wl.scans[2])
    assert (ne, ns) == (len(e), len(s))


@pytest.mark.parametrize("n_scans,cols,kw", [
    (32, 2048, {}),
    (64, 1024, {}),
    (128, 512, dict(beam_lo_deg=-25.0, beam_spacing_deg=40.0 / 127)),
    (16, 1800, dict(remove_bad_points=0)),
    (16, 1800, dict(edge_threshold=0.1, min_distance=1.0, max_distance=50.0)),
    (16, 4096, dict(libm_float=1)),
    (64, 1024, dict(libm_float=1)),
])
def test_extract_variants_bitexact(lib, oracle_mod, small_workload, n_scans, cols, kw):
    from lmsf import synth
    if n_scans == 32:
        elev = np.linspace(-30.67, 10.67, 32)
    elif n_scans == 64:
        elev = np.concatenate([np.linspace(2.0, -8.33, 32), np.linspace(-8.83, -24.33, 32)])
    elif n_scans == 128:
        elev = np.linspace(-25.0, 15.0, 128)
    else:
        elev = synth.VLP16_FIRING_DEG
    scan = synth.make_scan(small_workload.scene, small_workload.truth[0], 77, n_cols=cols, elev_deg=elev)
    okw = dict(n_scans=n_scans)
    okw.update(kw)
    e, s, ei, si = oracle_mod.extract(scan, **okw)
    ctx = _ctx(lib, n_scans=n_scans, **kw)
    ctx.extract(scan)
    ge, gei = ctx.copy_features(lib.EDGE)
    gs, gsi = ctx.copy_features(lib.SURF)
    np.testing.assert_array_equal(gei, ei)
    np.testing.assert_array_equal(gsi, si)
    assert ge.tobytes() == e.tobytes() and gs.tobytes() == s.tobytes()


@pytest.mark.parametrize("libm_float", [0, 1])
def test_extract_libm_overload_bitexact(lib, oracle_mod, libm_float):
    """The device takes the reference's sqrt / atan2 overload decision exactly as the oracle does on a
    point that the two choices keep / reject (conftest.libm_probe_scan)."""
    from conftest import libm_probe_scan
    scan = libm_probe_scan()
    e, s, ei, si = oracle_mod.extract(scan, libm_float=bool(libm_float))
    assert (900 in set(ei) | set(si)) == bool(libm_float)
    ctx = _ctx(lib, libm_float=libm_float)
    ctx.extract(scan)
    ge, gei = ctx.copy_features(lib.EDGE)
    gs, gsi = ctx.copy_features(lib.SURF)
    np.testing.assert_array_equal(gei, ei)
    np.testing.assert_array_equal(gsi, si)
    assert ge.tobytes() == e.tobytes() and gs.tobytes() == s.tobytes()


def test_runtime_extract_params_and_schedule(lib, oracle_mod, small_workload):
    """lmsf_set_extract_params / lmsf_set_schedule change a live context (SURVEY 8(b) surface)."""
    from lmsf import synth
    ctx = _ctx(lib)
    scan = synth.make_scan(small_workload.scene, small_workload.truth[0], 91, n_cols=1024, elev_deg=synth.HDL64_DEG)
    ctx.set_extract_params(n_scans=64, edge_threshold=0.5)
    ctx.extract(scan)
    e, s, _, _ = oracle_mod.extract(scan, n_scans=64, edge_threshold=0.5)
    ge, _ = ctx.copy_features(lib.EDGE)
    gs, _ = ctx.copy_features(lib.SURF)
    assert ge.tobytes() == e.tobytes() and gs.tobytes() == s.tobytes()
    with pytest.raises(lib.LmsfError):
        ctx.set_extract_params(n_scans=0)
    wl = small_workload
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.set_max_iterations(3)
    ctx.set_schedule(lib.SCHEDULE_FIXED)
    _, st = ctx.solve(wl.guess[0])
    assert st.outer_iterations == 3
    ctx.set_schedule(lib.SCHEDULE_REFERENCE_DECAY)
    _, st = ctx.solve(wl.guess[0])
    assert st.outer_iterations == 2


@pytest.mark.parametrize("extracted", [False, True])
def test_match_bitexact(lib, oracle_mod, small_workload, extracted):
    """8-lane teams (single-scan launch); queries in slot order (host features) or in ring order
    (device extraction)."""
    wl = small_workload
    e, s = _features(oracle_mod, wl.scans[0])
    ctx = _ctx(lib)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    if extracted:
        assert ctx.extract(wl.scans[0]) == (len(e), len(s))
    else:
        ctx.set_scan(lib.EDGE, e)
        ctx.set_scan(lib.SURF, s)
    reg = oracle_mod.Registration()
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    for pose in (wl.guess[0], wl.truth[0]):
        orec, onn = reg.match(pose)
        grec, gnn = ctx.match(pose, len(e) + len(s))
        # the oracle reports the unbounded 5-NN (nearestKSearch); the device reports the ranks
        # with d^2 < 1 and -1 beyond: every reported rank must equal the oracle's
        found = gnn >= 0
        np.testing.assert_array_equal(gnn[found], onn[found])
        assert (found[:, 1:] <= found[:, :-1]).all()      # found ranks form a prefix
        np.testing.assert_array_equal(grec["kind"], orec["kind"])
        assert grec.tobytes() == orec.tobytes()
        assert (orec["kind"] > 0).sum() > 0.5 * len(orec)


def _slice_density(m):
    """Points per occupied 0.25 m x 1 m x 1 m slice (the statistic lmsf_set_map uses to choose the
    pruned one-lane walk: >= 8)."""
    p = m[:, :3].astype(np.float32)
    c = np.stack([np.floor(p[:, 0] * 4), np.floor(p[:, 1]), np.floor(p[:, 2])], 1).astype(np.int64)
    return len(p) / len(np.unique(c, axis=0))


@pytest.fixture(scope="module")
def dense_workload():
    """C2 scans against a 1M-point map over a 30 m radius: ~25 points per occupied slice, the
    density regime of C5's 10M-point map (pruned search)."""
    from lmsf import synth
    return synth.make_workload("C2", n_scans=1, map_points=1_000_000, radius=30.0, road_length=20.0)


@pytest.mark.parametrize("extracted", [False, True])
@pytest.mark.parametrize("dense", [False, True])
def test_match_bitexact_one_lane(lib, oracle_mod, small_workload, dense_workload, dense, extracted):
    """The one-lane-per-query search (query slots >= 2^20): plain walk on the sparse map, pruned
    two-pass walk on the dense one, queries in slot order (host features) or in ring order
    (features extracted on the device); neighbour sets and records byte-identical to the oracle."""
    wl = dense_workload if dense else small_workload
    assert (_slice_density(wl.surf_map) >= 8) == dense
    e, s = _features(oracle_mod, wl.scans[0])
    ctx = _ctx(lib, max_batch=1, max_features=1 << 20)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    if extracted:
        assert ctx.extract(wl.scans[0]) == (len(e), len(s))
    else:
        ctx.set_scan(lib.EDGE, e)
        ctx.set_scan(lib.SURF, s)
    reg = oracle_mod.Registration()
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    for pose in (wl.guess[0], wl.truth[0]):
        orec, onn = reg.match(pose)
        grec, gnn = ctx.match(pose, len(e) + len(s))
        found = gnn >= 0
        np.testing.assert_array_equal(gnn[found], onn[found])
        assert (found[:, 1:] <= found[:, :-1]).all()
        assert grec.tobytes() == orec.tobytes()
        assert (orec["kind"] > 0).sum() > 0.2 * len(orec)


def test_eval_packet(lib, oracle_mod, small_workload):
    wl = small_workload
    e, s = _features(oracle_mod, wl.scans[1])
    ctx = _ctx(lib)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.set_scan(lib.EDGE, e)
    ctx.set_scan(lib.SURF, s)
    rec, _ = ctx.match(wl.guess[1], len(e) + len(s))
    for pose in (wl.guess[1], wl.truth[1]):
        g = ctx.eval(pose)
        o = oracle_mod.eval_records(rec, pose)
        np.testing.assert_allclose(g, o, rtol=1e-9, atol=1e-9)


def _solve_both(lib, oracle_mod, wl, i, solver, fixed, iters, n_solves=1):
    e, s = _features(oracle_mod, wl.scans[i])
    ctx = _ctx(lib, solver=solver, schedule=1 if fixed else 0, max_iterations=iters)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.set_scan(lib.EDGE, e)
    ctx.set_scan(lib.SURF, s)
    reg = oracle_mod.Registration(solver)
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    reg.set_fixed_schedule(fixed)
    reg.set_max_iterations(iters)
    out = []
    for _ in range(n_solves):
        gx, gst = ctx.solve(wl.guess[i])
        gtr = ctx.trace()
        ox, otr, ost = reg.solve(wl.guess[i])
        out.append((gx, gst, gtr, ox, ost, otr))
    return out


@pytest.mark.parametrize("i", [0, 1, 2])
def test_solve_trace_parity_lm(lib, oracle_mod, small_workload, i):
    for gx, gst, gtr, ox, ost, otr in _solve_both(lib, oracle_mod, small_workload, i, 0, True, 5):
        assert gtr.shape == otr.shape == (5, 7)
        for a, b in zip(gtr, otr):
            dt, dr = pose_err(a, b)
            assert dt <= POSE_TOL and dr <= POSE_TOL, (dt, dr)
        assert (gst.edge_matches, gst.surf_matches) == (ost.edge_matches, ost.surf_matches)
        assert gst.termination == ost.termination
        # registration actually recovers the ground truth
        dt, dr = pose_err(gx, small_workload.truth[i])
        assert dt < 0.05 and dr < 0.01


def test_solve_reference_decay_schedule(lib, oracle_mod, small_workload):
    res = _solve_both(lib, oracle_mod, small_workload, 0, 0, False, 10, n_solves=3)
    for k, (gx, gst, gtr, ox, ost, otr) in enumerate(res):
        assert gst.outer_iterations == ost.outer_iterations == 9 - k    # 10 -> 9, 8, 7
        dt, dr = pose_err(gx, ox)
        assert dt <= POSE_TOL and dr <= POSE_TOL


def test_solve_trace_parity_gn(lib, oracle_mod, small_workload):
    for gx, gst, gtr, ox, ost, otr in _solve_both(lib, oracle_mod, small_workload, 1, 1, True, 10):
        assert len(gtr) == len(otr)
        for a, b in zip(gtr, otr):
            dt, dr = pose_err(a, b)
            assert dt <= POSE_TOL and dr <= POSE_TOL, (dt, dr)


def test_batch_run_matches_oracle(lib, oracle_mod, small_workload):
    """Batch path with 16 slots: 16 x 70k query slots >= 2^20 selects the one-lane-per-query knn
    team (the single-scan tests above run the 8-lane team)."""
    wl = small_workload
    ctx = _ctx(lib, schedule=1, max_iterations=5, max_batch=16)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    n = len(wl.scans)
    ctx.load_scans([wl.scans[i % n] for i in range(16)])
    ctx.kernel_stats_reset(timing=True)
    poses, stats = ctx.batch_run(np.stack([wl.guess[i % n] for i in range(16)]))
    ks = ctx.kernel_stats()
    assert ks.launches == 5 and ks.fused_launches == 5               # the fused search + fit path ran
    assert ks.reused_queries > 0.1 * ks.queries                      # ... and the query memo fired
    assert ks.refit_queries > 0                                      # ... and refitted reordered sets
    # outer iterations > 0 reuse the 5-NN set and fit of queries that moved less than half their
    # neighbour-distance gap, and refit (without a walk) those whose set only changed order: same
    # records, packets summed in another grouping (the searching lanes are packed), so the poses
    # agree with re-searching every query (and with searching the reordered ones) to rounding
    for opt in (lib.OPT_QUERY_MEMO, lib.OPT_MEMO_REFIT, lib.OPT_MEMO_EXACT, lib.OPT_MEMO_ORDER, lib.OPT_MEMO_BOUND,
                lib.OPT_MEMO_SKIP1):
        ctx.set_option(opt, 0)
        try:
            poses0, _ = ctx.batch_run(np.stack([wl.guess[i % n] for i in range(16)]))
        finally:
            ctx.set_option(opt, 1)
        assert np.abs(poses0 - poses).max() <= 1e-12, opt
    # byte-level: every outer iteration's records of two slots (memo reuses, refits and bounded searches
    # included) equal the oracle's fresh match at the pose the GPU matched at
    ctx.batch_capture([1, 4])
    ctx.kernel_stats_reset(timing=True)
    posesc, _ = ctx.batch_run(np.stack([wl.guess[i % n] for i in range(16)]))
    ksc = ctx.kernel_stats()
    assert ksc.reused_queries > 0 and np.array_equal(posesc, poses)   # capture changes nothing
    for slot in (1, 4):
        e, s = _features(oracle_mod, wl.scans[slot % n])
        reg = oracle_mod.Registration()
        reg.set_map(1, wl.edge_map)
        reg.set_map(2, wl.surf_map)
        reg.set_scan(1, e)
        reg.set_scan(2, s)
        assert_captured_records(ctx, reg, slot, 5)
    ctx.batch_capture([])
    np.testing.assert_array_equal(poses[n:2 * n], poses[:n])          # same scan + guess -> same pose
    for i in range(len(wl.scans)):
        e, s = _features(oracle_mod, wl.scans[i])
        ge, _ = ctx.copy_features(lib.EDGE, slot=i)
        gs, _ = ctx.copy_features(lib.SURF, slot=i)
        assert ge.tobytes() == e.tobytes() and gs.tobytes() == s.tobytes()
        reg = oracle_mod.Registration()
        reg.set_map(1, wl.edge_map)
        reg.set_map(2, wl.surf_map)
        reg.set_scan(1, e)
        reg.set_scan(2, s)
        reg.set_fixed_schedule(True)
        reg.set_max_iterations(5)
        ox, _, _ = reg.solve(wl.guess[i])
        dt, dr = pose_err(poses[i], ox)
        assert dt <= POSE_TOL and dr <= POSE_TOL
        assert stats[i].outer_iterations == 5


def test_batch_capacity_flag_is_per_batch(lib, small_workload):
    """A batch whose scan overflows the extraction kernel's ring capacity fails with ERR_CAPACITY; the
    next valid batch on the same context succeeds (the flag is cleared per launch)."""
    wl = small_workload
    ctx = _ctx(lib, schedule=1, max_iterations=2, max_batch=2)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    az = np.linspace(0, 2 * np.pi, 10000, endpoint=False)        # 10,000 points in ring 0 (> 8,192)
    r = 10.0
    bad = np.stack([r * np.cos(az), r * np.sin(az), np.full_like(az, -r * np.tan(np.radians(15.0))),
                    np.zeros_like(az)], 1).astype(np.float32)
    ctx.load_scans([bad, wl.scans[0]])
    with pytest.raises(lib.LmsfError) as ei:
        ctx.batch_run(np.stack([wl.guess[0], wl.guess[0]]))
    assert ei.value.code == lib.ERR_CAPACITY
    ctx.load_scans([wl.scans[0], wl.scans[1]])
    poses, st = ctx.batch_run(np.stack([wl.guess[0], wl.guess[1]]))
    assert st[0].outer_iterations == 2 and st[0].surf_matches > 0


def test_batch_streamed_upload(lib, small_workload):
    """lmsf_batch_load_scans_async: the next batch's scans upload (pinned host memory, copy stream)
    while the current batch registers; results equal the synchronous loads, batch by batch."""
    import torch
    wl = small_workload
    A = [wl.scans[i] for i in (0, 1, 2, 0)]
    B = [wl.scans[i] for i in (2, 1, 0, 1)]
    gA = np.stack([wl.guess[i] for i in (0, 1, 2, 0)])
    gB = np.stack([wl.guess[i] for i in (2, 1, 0, 1)])

    def mk():
        c = _ctx(lib, schedule=1, max_iterations=3, max_batch=4)
        c.set_map(lib.EDGE, wl.edge_map)
        c.set_map(lib.SURF, wl.surf_map)
        return c

    ref = mk()
    ref.load_scans(A)
    pA, _ = ref.batch_run(gA)
    ref.load_scans(B)
    pB, _ = ref.batch_run(gB)

    def pinned(scans):
        return torch.from_numpy(np.concatenate(scans, 0)).pin_memory(), np.array([len(x) for x in scans])

    ctx = mk()
    ctx.load_scans_async(*pinned(A))
    ctx.batch_launch(gA)
    ctx.load_scans_async(*pinned(B))          # overlaps batch A's registration
    qA, _ = ctx.batch_wait(4)
    ctx.batch_launch(gB)
    qB, _ = ctx.batch_wait(4)
    np.testing.assert_array_equal(qA, pA)
    np.testing.assert_array_equal(qB, pB)
    for i in range(4):                         # per-slot outer-iteration trace of the last batch
        tr = ctx.batch_trace(i)
        assert tr.shape == (3, 7) and np.array_equal(tr[-1], qB[i])


def test_batch_memo_dense(lib, oracle_mod, dense_workload):
    """Dense maps (the C5 density regime) take the query memo since r05 (VERDICT r04 #3b): outer iteration 1 keeps
    6 exact keys and leaves the anchors, iterations >= 2 run the memo pass and search only its misses on the
    first-pass grid.  The memo served queries; memo on and off give the same poses bit for bit; the records after
    every outer iteration -- reused, refitted and re-searched alike -- are byte-identical to the oracle's fresh match
    at the same pose; the poses match the oracle."""
    wl = dense_workload
    ctx = _ctx(lib, schedule=1, max_iterations=5, max_batch=16)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.load_scans([wl.scans[0]] * 16)
    rng = np.random.default_rng(5)
    from lmsf import synth
    guesses = np.stack([synth.perturb(wl.truth[0], rng) for _ in range(16)])
    ctx.kernel_stats_reset(timing=True)
    poses, _ = ctx.batch_run(guesses)
    ks = ctx.kernel_stats()
    assert ks.fused_launches == 5 and ks.reused_queries + ks.refit_queries > 0.2 * ks.queries
    ctx.set_option(lib.OPT_QUERY_MEMO, 0)
    try:
        poses0, _ = ctx.batch_run(guesses)
    finally:
        ctx.set_option(lib.OPT_QUERY_MEMO, 1)
    assert np.array_equal(poses0, poses)
    e, s = _features(oracle_mod, wl.scans[0])
    reg = oracle_mod.Registration()
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    reg.set_fixed_schedule(True)
    reg.set_max_iterations(5)
    ctx.batch_capture([3])
    posesc, _ = ctx.batch_run(guesses)
    assert np.array_equal(posesc, poses)
    assert_captured_records(ctx, reg, 3, 5)
    ox, _, _ = reg.solve(guesses[3])
    dt, dr = pose_err(poses[3], ox)
    assert dt <= POSE_TOL and dr <= POSE_TOL


def test_batch_dense_wide_extent(lib, dense_workload):
    """a dense map whose first-pass grid would exceed the cell limit.  Two far points stretch the
    surf map to 4,000 x 100 x 100 m: its 1 m grid has 1.6e8 cells (4 x-slices per metre), the 0.5 m first-pass grid
    would need 1.3e9 > 2^30 -- it is refused (recorded against the map build, not retried per launch) and the first
    pass runs on the 1 m grid.  Both launches on the wide map equal the compact map's poses bit for bit (the far
    points are never within 1 m of a query: the same neighbour sets and records)."""
    wl = dense_workload
    ctx = _ctx(lib, schedule=1, max_iterations=5, max_batch=16)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.load_scans([wl.scans[0]] * 16)
    rng = np.random.default_rng(9)
    from lmsf import synth
    guesses = np.stack([synth.perturb(wl.truth[0], rng) for _ in range(16)])
    ref, _ = ctx.batch_run(guesses)
    far = np.array([[2000.0, 50.0, 50.0, 0.0], [-2000.0, -50.0, -50.0, 0.0]], np.float32)
    ctx.set_map(lib.SURF, np.concatenate([wl.surf_map, far]))
    wide, _ = ctx.batch_run(guesses)
    wide2, _ = ctx.batch_run(guesses)
    assert np.array_equal(wide, ref) and np.array_equal(wide2, ref)


def test_edge_cases(lib, oracle_mod, small_workload):
    wl = small_workload
    ctx = _ctx(lib)
    # no map -> LMSF_ERR_NO_MAP, pose untouched
    with pytest.raises(lib.LmsfError) as ei:
        ctx.solve(wl.guess[0])
    assert ei.value.code == lib.ERR_NO_MAP
    # tiny map (< 5 points): every kNN fails -> no residuals, pose unchanged
    ctx.set_map(lib.SURF, wl.surf_map[:4])
    e, s = _features(oracle_mod, wl.scans[0])
    ctx.set_scan(lib.SURF, s)
    x, st = ctx.solve(wl.guess[0])
    np.testing.assert_array_equal(x, wl.guess[0])
    assert st.termination == 4 and st.surf_matches == 0
    # empty scan
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.set_scan(lib.SURF, np.zeros((0, 4), np.float32))
    x, st = ctx.solve(wl.guess[0])
    np.testing.assert_array_equal(x, wl.guess[0])
    # empty map upload keeps the previous map (ceres_...:60)
    ctx.set_map(lib.SURF, np.zeros((0, 4), np.float32))
    ctx.set_scan(lib.SURF, s)
    x, st = ctx.solve(wl.guess[0])
    assert st.surf_matches > 0
    # capacity
    with pytest.raises(lib.LmsfError) as ei:
        ctx.extract(np.zeros((80000, 4), np.float32))
    assert ei.value.code == lib.ERR_CAPACITY
    # extraction of a scan with fewer than 20 points per ring -> no features
    ne, ns = ctx.extract(wl.scans[0][:100])
    assert ne == 0 and ns == 0


@pytest.mark.parametrize("fused", [False, True])
def test_n27_accounting(lib, oracle_mod, small_workload, fused):
    """The per-launch candidate count equals the map points in the 3x3x3 cells around each query;
    8-lane knn_kernel (host features) or the fused one-lane search + fit (extracted features,
    >= 2^20 query slots)."""
    from lmsf import synth
    wl = small_workload
    e, s = _features(oracle_mod, wl.scans[2])
    ctx = _ctx(lib, max_batch=1, max_features=1 << 20) if fused else _ctx(lib)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    if fused:
        assert ctx.extract(wl.scans[2]) == (len(e), len(s))
    else:
        ctx.set_scan(lib.EDGE, e)
        ctx.set_scan(lib.SURF, s)
    ctx.kernel_stats_reset(timing=True)   # timed launches carry no n27 accounting
    ctx.match(wl.guess[2], len(e) + len(s))
    ks = ctx.kernel_stats()
    assert ks.queries == len(e) + len(s) and ks.n27_sum == 0
    ctx.kernel_stats_reset(timing=False, n27=True)
    ctx.match(wl.guess[2], len(e) + len(s))
    ks = ctx.kernel_stats()
    assert ks.queries == len(e) + len(s)
    expect = 0
    for pts, m in ((e, wl.edge_map), (s, wl.surf_map)):
        w = synth.transform_points(wl.guess[2], pts)[:, :3]
        cells = np.floor(m[:, :3]).astype(np.int64)
        lo = cells.min(0)
        key = lambda c: ((c[:, 2] - lo[2]) * 100000 + (c[:, 1] - lo[1])) * 100000 + (c[:, 0] - lo[0])
        ks_sorted = np.sort(key(cells))
        qc = np.floor(w).astype(np.int64)
        for dz in (-1, 0, 1):
            for dy in (-1, 0, 1):
                for dx in (-1, 0, 1):
                    k = key(qc + np.array([dx, dy, dz]))
                    expect += int((np.searchsorted(ks_sorted, k, "right") - np.searchsorted(ks_sorted, k, "left")).sum())
    assert abs(ks.n27_sum - expect) <= 1e-4 * expect


def test_cpp_facade(lib, oracle_mod, small_workload, tmp_path):
    """A C++ program written against RegistrationBase / PointCloudProcessBase (include/lmsf/lmsf.hpp)
    reproduces the oracle: default factory settings, reference decay schedule (10 -> 9 iterations)."""
    import subprocess
    from test_abi import build_facade_example
    wl = small_workload
    exe = build_facade_example(tmp_path)
    paths = []
    for name, arr in (("scan", wl.scans[0]), ("edge", wl.edge_map), ("surf", wl.surf_map)):
        p = tmp_path / f"{name}.bin"
        np.ascontiguousarray(arr, np.float32).tofile(p)
        paths.append(str(p))
    g = wl.guess[0]
    out = subprocess.run([exe, *paths, *[repr(float(v)) for v in g], "10"], capture_output=True, text=True,
                         timeout=300)
    assert out.returncode == 0, out.stderr
    f = out.stdout.split()
    ne, ns, x, outer = int(f[0]), int(f[1]), np.array([float(v) for v in f[2:9]]), int(f[9])
    e, s = _features(oracle_mod, wl.scans[0])
    assert (ne, ns) == (len(e), len(s)) and outer == 9
    reg = oracle_mod.Registration()
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    ox, _, _ = reg.solve(g)
    dt, dr = pose_err(x, ox)
    assert dt <= POSE_TOL and dr <= POSE_TOL


def test_tracker_sequence_parity(lib, oracle_mod, sequence_workload):
    """lmsf_tracker (device-resident sliding-window local map) vs oracle/tracker.py on a 10-scan
    64-beam sequence: same update decisions and map sizes, poses <= 1e-4, tracking within 5 cm."""
    import tracker as OT
    from conftest import mat_err, relative_truth
    wl = sequence_workload
    rel = relative_truth(wl.truth)
    ctx = _ctx(lib, n_scans=wl.n_scans)
    gt = lib.Tracker(ctx, window_frames=3)
    ot = OT.Tracker(window_frames=3)
    types = []
    for i, scan in enumerate(wl.scans):
        e, s, _, _ = oracle_mod.extract(scan, n_scans=wl.n_scans)
        ctx.extract(scan)
        ge, _ = ctx.copy_features(lib.EDGE)
        gs, _ = ctx.copy_features(lib.SURF)
        assert ge.tobytes() == e.tobytes() and gs.tobytes() == s.tobytes()
        gd, r = gt.solve(ge, gs, wl.dt * i)
        od, otyp, _ = ot.solve(e, s, wl.dt * i)
        assert r.update_type == otyp, i
        assert bool(r.initialized) == (i == 0)
        assert (r.local_map_edge, r.local_map_surf) == (len(ot.local_map(1)), len(ot.local_map(2)))
        dt, dr = mat_err(gt.pose(), ot.curr)
        assert dt <= POSE_TOL and dr <= POSE_TOL, (i, dt, dr)
        np.testing.assert_allclose(gd, od, atol=POSE_TOL)
        dt, dr = mat_err(gt.pose(), rel[i])
        assert dt < 0.05 and dr < 0.01, (i, dt, dr)
        types.append(otyp)
    assert 0 in types[1:] and 1 in types[1:]
    for kind in (lib.EDGE, lib.SURF):
        np.testing.assert_allclose(gt.local_map(kind), ot.local_map(kind), atol=1e-4)
    # refine (dual-LiDAR / external prediction path): register against the current local map
    T0 = rel[-1].copy()
    T0[:3, 3] += (0.05, -0.03, 0.02)
    e, s, _, _ = oracle_mod.extract(wl.scans[-1], n_scans=wl.n_scans)
    GT, st = gt.register(e, s, T0)
    OTp, _ = ot._register({1: e, 2: s}, T0)
    dt, dr = mat_err(GT, OTp)
    assert dt <= POSE_TOL and dr <= POSE_TOL and st.outer_iterations > 0
    gt.close()


def test_tracker_time_gate_and_capacity(lib, oracle_mod, sequence_workload):
    """TIME keyframes after time_interval; window eviction keeps only the newest W frames;
    a keyframe larger than the slot capacity is an error, not a truncation."""
    wl = sequence_workload
    ctx = _ctx(lib, n_scans=wl.n_scans)
    gt = lib.Tracker(ctx, window_frames=2, threshold_trans=1e9, threshold_rot=1e9, time_interval=0.15,
                     leaf_edge=0.0, leaf_surf=0.0)    # raw window: sizes add up
    kf_sizes = []
    types = []
    for i, scan in enumerate(wl.scans[:5]):
        e, s, _, _ = oracle_mod.extract(scan, n_scans=wl.n_scans)
        _, r = gt.solve(e, s, 0.1 * i)
        types.append(r.update_type)
        if r.update_type != lib.UPDATE_NONE:
            kf_sizes.append(len(s))
        assert r.local_map_surf == sum(kf_sizes[-2:])
    assert types == [lib.UPDATE_MOTION, lib.UPDATE_NONE, lib.UPDATE_TIME, lib.UPDATE_NONE, lib.UPDATE_TIME]
    gt.close()
    small = _ctx(lib, n_scans=wl.n_scans, max_features=1000, max_scan_points=1000)   # capacity = max of both
    t2 = lib.Tracker(small, window_frames=2)
    e, s, _, _ = oracle_mod.extract(wl.scans[0], n_scans=wl.n_scans)
    assert len(s) > 1000
    with pytest.raises(lib.LmsfError):
        t2.solve(e[:500], s, 0.0)
    t2.close()


def test_voxel_filter_bitexact(lib, oracle_mod, small_workload):
    """lmsf_voxel_filter (radix-sorted voxel keys + ordered double centroids) == oracle/voxel.cpp."""
    import torch
    ctx = _ctx(lib)
    e, s, _, _ = oracle_mod.extract(small_workload.scans[0])
    for pts in (s, e, small_workload.surf_map[:200_000]):
        for leaf in (0.1, 0.4, 1.0):
            want = oracle_mod.voxel_filter(pts, leaf)
            assert ctx.voxel_filter(pts, leaf).tobytes() == want.tobytes()
    got = ctx.voxel_filter(torch.from_numpy(s).to("cuda:0"), 0.4)            # device input
    assert got.tobytes() == oracle_mod.voxel_filter(s, 0.4).tobytes()
    far = np.array([[0, 0, 0, 0], [1e4, 1e4, 1e4, 1]], np.float32)
    assert ctx.voxel_filter(far, 0.01).tobytes() == far.tobytes()


def test_voxel_filter_small_bitexact(lib, oracle_mod, small_workload):
    """Window-sized clouds (a C4 edge window is ~4.5k points) == oracle/voxel.cpp: random subsets from 1 to
    9000 points, long voxels of duplicated points and the int32 key-overflow case (input returned)."""
    ctx = _ctx(lib)
    _, s, _, _ = oracle_mod.extract(small_workload.scans[0])
    rng = np.random.default_rng(5)
    for n in (1, 2, 63, 100, 1000, 4550, 8191, 8192, 8193, 9000):
        pts = s[rng.permutation(len(s))[:n]] if n <= len(s) else s
        for leaf in (0.2, 0.4, 2.0):
            assert ctx.voxel_filter(pts, leaf).tobytes() == oracle_mod.voxel_filter(pts, leaf).tobytes(), (n, leaf)
    dup = np.repeat(s[:50], 40, axis=0)                      # 40 copies of each point: long voxels
    assert ctx.voxel_filter(dup, 0.4).tobytes() == oracle_mod.voxel_filter(dup, 0.4).tobytes()
    far = np.concatenate([s[:500], np.array([[1e5, -1e5, 1e5, 2]], np.float32)])   # key range overflows
    assert ctx.voxel_filter(far, 0.001).tobytes() == oracle_mod.voxel_filter(far, 0.001).tobytes()


def test_ingest_pointcloud2_parity(lib, oracle_mod, small_workload):
    """lmsf_ingest_pointcloud2 / lmsf_extract_pointcloud2 vs oracle/ingest.cpp: decode + removeNaN
    and the distance filter bit-exact; rotary relative time (double atan2 rounded to float on both
    sides) within 1e-6 s; the extracted features equal the oracle's extraction of the oracle's
    ingest (points and order)."""
    import torch
    from lmsf import synth
    wl = small_workload
    ctx = _ctx(lib)
    for seed in (21, 22):
        org = synth.make_scan(wl.scene, wl.truth[0], seed, n_cols=4096, organized=True, clockwise=True)
        msg = synth.to_pointcloud2(org)
        for kw in (dict(scan_period=0.0), dict(), dict(scan_period=0.0, distance_near=3.0, distance_far=50.0),
                   dict(distance_near=3.0, distance_far=50.0)):
            g = ctx.ingest_pointcloud2(msg, len(org), **kw)
            o = oracle_mod.ingest(msg, len(org), **kw)
            assert g.shape == o.shape
            assert g[:, :3].tobytes() == o[:, :3].tobytes()
            assert np.abs(g[:, 3] - o[:, 3]).max() <= 1e-6
        g = ctx.ingest_pointcloud2(torch.from_numpy(msg).to("cuda:0"), len(org))        # device message
        assert g[:, :3].tobytes() == oracle_mod.ingest(msg, len(org))[:, :3].tobytes()
        ne, ns = ctx.extract_pointcloud2(msg, len(org))
        e, s, _, _ = oracle_mod.extract(oracle_mod.ingest(msg, len(org)))
        ge, _ = ctx.copy_features(lib.EDGE)
        gs, _ = ctx.copy_features(lib.SURF)
        assert (ne, ns) == (len(e), len(s))
        assert ge[:, :3].tobytes() == e[:, :3].tobytes() and gs[:, :3].tobytes() == s[:, :3].tobytes()


def test_alignment_score_parity(lib, oracle_mod, small_workload):
    """lmsf_align_score vs oracle/align.py (AlignmentScore, REG/alignEvaluate.hpp:55-87): inlier
    count exact, mean inlier d2 rel 1e-12 (reduction order), thresholds of the reference's callers
    (0.1, 1.0) plus 4.0 (two-cell search radius)."""
    import sys
    import torch
    import align as OA
    from conftest import pose_matrix
    wl = small_workload
    ctx = _ctx(lib)
    ctx.align_set_target(wl.surf_map)
    tree = oracle_mod.KdMap(wl.surf_map)
    e, s, _, _ = oracle_mod.extract(wl.scans[1])
    for pose in (wl.truth[1], wl.guess[1]):
        T = pose_matrix(pose).astype(np.float32)
        for thresh, ratio in ((0.1, 0.6), (1.0, 0.6), (4.0, 0.5), (0.1, 0.99)):
            gs, go = ctx.align_score(s, T, thresh, ratio)
            os_, oo = OA.alignment_score(wl.surf_map, s, T, thresh, ratio, tree=tree)
            assert go == oo
            if os_ == sys.float_info.max:
                assert gs == os_
            else:
                assert abs(gs - os_) <= 1e-12 * os_
    # the true pose overlaps better and scores lower than the perturbed guess (device input)
    st, ot_ = ctx.align_score(torch.from_numpy(s).to("cuda:0"), pose_matrix(wl.truth[1]), 1.0, 0.3)
    sg, og = ctx.align_score(s, pose_matrix(wl.guess[1]), 1.0, 0.3)
    assert ot_ > og and st < sg
    assert ctx.align_score(s[:0], np.eye(4), 0.1, 0.6) == (sys.float_info.max, 0.0)


def test_tracker_shared_map_streams(lib, oracle_mod, sequence_workload):
    """C4 flow on one GPU: two streams (scans 0-4 and 5-9) with a shared world-frame prior map,
    initial poses in that frame, keyframes exchanged in stream order and committed once per step
    (device-tensor keyframe buffers), against two oracle trackers doing the same."""
    import torch
    import tracker as OT
    from conftest import mat_err, pose_matrix
    wl = sequence_workload
    streams = [list(range(0, 5)), list(range(5, 10))]
    ctxs = [_ctx(lib, n_scans=wl.n_scans) for _ in streams]
    gts = [lib.Tracker(c, window_frames=4, manual_map_update=True) for c in ctxs]
    ots = [OT.Tracker(window_frames=4, manual_map_update=True) for _ in streams]
    dev = torch.device("cuda", 0)
    for s, idx in enumerate(streams):
        T0 = pose_matrix(wl.truth[idx[0]])
        gts[s].set_initial_pose(T0)
        ots[s].origin = T0.copy()
        gts[s].set_prior_map(lib.EDGE, torch.from_numpy(wl.edge_map).to(dev))
        gts[s].set_prior_map(lib.SURF, wl.surf_map)
        ots[s].set_prior_map(1, wl.edge_map)
        ots[s].set_prior_map(2, wl.surf_map)
    buf = {k: torch.zeros((70000, 4), dtype=torch.float32, device=dev) for k in (lib.EDGE, lib.SURF)}
    nq = {}
    for step in range(5):
        kfs_g, kfs_o = [], []
        for s, idx in enumerate(streams):
            scan = wl.scans[idx[step]]
            e, su, _, _ = oracle_mod.extract(scan, n_scans=wl.n_scans)
            ctxs[s].extract(torch.from_numpy(scan).to(dev))
            _, r = gts[s].solve_extracted(wl.dt * step)
            _, otyp, _ = ots[s].solve(e, su, wl.dt * step)
            assert r.update_type == otyp
            nq[s] = len(e) + len(su)
            dt, dr = mat_err(gts[s].pose(), ots[s].curr)
            assert dt <= POSE_TOL and dr <= POSE_TOL, (step, s, dt, dr)
            dt, dr = mat_err(gts[s].pose(), pose_matrix(wl.truth[idx[step]]))
            assert dt < 0.05 and dr < 0.01, (step, s, dt, dr)
            if otyp:
                ne = ctxs[s].copy_features_into(lib.EDGE, buf[lib.EDGE])
                ns = ctxs[s].copy_features_into(lib.SURF, buf[lib.SURF])
                assert (ne, ns) == (len(e), len(su))
                kfs_g.append((s, buf[lib.EDGE][:ne].clone(), buf[lib.SURF][:ns].clone(), gts[s].pose()))
                kfs_o.append((e, su, ots[s].curr.copy()))
        for g, o in zip(kfs_g, kfs_o):              # every stream appends every keyframe, same order
            for s in range(len(streams)):
                if g[0] == s:                       # its own: from the context's extracted features
                    gts[s].add_keyframe_extracted(g[3])
                else:                               # the other stream's: device tensors (in place)
                    gts[s].add_keyframe(*g[1:])
                ots[s].add_keyframe(*o)
        for s in range(len(streams)):
            gts[s].commit_map()                     # returns with the rebuild enqueued (deferred finish)
            ots[s].commit()
            if s == 0 and kfs_g:                    # a context-level map consumer completes it first
                rec_a, nn_a = ctxs[0].match(wl.truth[streams[0][step]], nq[0])
                gts[0].local_map(lib.EDGE)
                rec_b, nn_b = ctxs[0].match(wl.truth[streams[0][step]], nq[0])
                same = rec_a.tobytes() == rec_b.tobytes() and bool((nn_a == nn_b).all())   # no byte-string diff
                assert same, "a match right after commit_map differs from one after the completed commit"
            assert len(gts[s].local_map(lib.SURF)) == len(ots[s].local_map(2))
    # replica 0 added stream 0's keyframes from its context and stream 1's from tensors, replica 1 the reverse
    np.testing.assert_allclose(gts[0].local_map(lib.SURF), gts[1].local_map(lib.SURF), atol=0)
    np.testing.assert_allclose(gts[0].local_map(lib.EDGE), gts[1].local_map(lib.EDGE), atol=0)
    np.testing.assert_allclose(gts[0].local_map(lib.EDGE), ots[0].local_map(1), atol=1e-4)
    for t in gts:
        t.close()


def test_deferred_commit_settles(lib, oracle_mod, sequence_workload):
    """A keyframe commit left pending by lmsf_tracker_commit_map completes (a) before lmsf_solve's map check on
    a context whose only map is that first commit, and (b) when the tracker is destroyed, so the context keeps
    searching a consistent window grid.  Both equal the explicitly completed commit."""
    from conftest import pose_matrix
    wl = sequence_workload
    scan = wl.scans[1]
    e, su, _, _ = oracle_mod.extract(wl.scans[0], n_scans=wl.n_scans)
    T0 = pose_matrix(wl.truth[0])
    guess = wl.truth[1]

    def setup(finish):
        ctx = _ctx(lib, n_scans=wl.n_scans)
        t = lib.Tracker(ctx, window_frames=3, manual_map_update=True)
        t.add_keyframe(e, su, T0)
        t.commit_map()                                   # deferred finish
        if finish:
            t.local_map(lib.SURF)                        # any tracker call completes it
        return ctx, t

    ref_ctx, ref_t = setup(True)
    ref_ctx.extract(scan)
    ref_pose, _ = ref_ctx.solve(guess)
    ctx, t = setup(False)
    ctx.extract(scan)
    pose, _ = ctx.solve(guess)                           # (a): no LMSF_ERR_NO_MAP
    assert np.array_equal(pose, ref_pose)
    ctx2, t2 = setup(False)
    t2.close()                                           # (b): completes the pending rebuild first
    nq = sum(ctx2.extract(scan))
    rec_a, nn_a = ctx2.match(guess, nq)
    ref_ctx.extract(scan)
    rec_b, nn_b = ref_ctx.match(guess, nq)
    assert rec_a.tobytes() == rec_b.tobytes() and np.array_equal(nn_a, nn_b)
    assert (rec_a["kind"] > 0).sum() > 0.2 * nq
    for x in (ref_t, t):
        x.close()


@pytest.mark.parametrize("workers", [True, False], ids=["commit_workers", "inline_commit"])
def test_tracker_growth_on_commit_streams(lib, oracle_mod, sequence_workload, workers):
    """a tracker whose window buffers -- the voxel filter's workspace and look-back words, the window
    grid's points, cells and scan look-back words -- are regrown at nearly every keyframe commit
    (LMSF_OPT_GROWTH_TEST: exact growth, 2^10 first cells) on the commit streams (workers: manual keyframes +
    lmsf_tracker_commit_map, the rebuild enqueued by the two worker threads on the aux streams and finished beside
    the next extraction; inline: the automatic updateLocalMap) equals the oracle tracker: same update decisions,
    poses <= 1e-4 at every scan, same windows.  The growths happened (buffer_growths), and no device look-back
    fault was flagged (a set fault word fails the next Solve)."""
    import tracker as OT
    from conftest import mat_err
    wl = sequence_workload
    ctx = _ctx(lib, n_scans=wl.n_scans)
    ctx.set_option(lib.OPT_GROWTH_TEST, 1)
    gt = lib.Tracker(ctx, window_frames=4, manual_map_update=workers)
    ot = OT.Tracker(window_frames=4, manual_map_update=workers)
    g0 = ctx.kernel_stats().buffer_growths
    keyframes = 0
    for i, scan in enumerate(wl.scans):
        e, s, _, _ = oracle_mod.extract(scan, n_scans=wl.n_scans)
        ctx.extract(scan)                        # a deferred commit completes beside this extraction
        _, r = gt.solve_extracted(wl.dt * i)
        _, otyp, _ = ot.solve(e, s, wl.dt * i)
        assert r.update_type == otyp, i
        dt, dr = mat_err(gt.pose(), ot.curr)
        assert dt <= POSE_TOL and dr <= POSE_TOL, (i, dt, dr)
        if otyp:
            keyframes += 1
            if workers:
                gt.add_keyframe_extracted(gt.pose())
                ot.add_keyframe(e, s, ot.curr.copy())
                gt.commit_map()
                ot.commit()
    assert keyframes >= 5
    for kind in (lib.EDGE, lib.SURF):
        np.testing.assert_allclose(gt.local_map(kind), ot.local_map(kind), atol=1e-4)
    growths = ctx.kernel_stats().buffer_growths - g0
    assert growths >= 6, growths
    gt.close()


@pytest.mark.parametrize("inject", [1, 2], ids=["stale_prefix", "foreign_epoch"])
def test_lookback_fault_flagged(lib, oracle_mod, sequence_workload, inject):
    """The device look-back checks (radix.h) catch what r04's null-stream memset race produced, injected into the
    window voxel filter's first radix pass (LMSF_OPT_FAULT_INJECT): a stale prefix that puts a tile's scatter outside
    the pairs (1) and a look-back word of another allocation (2).  Nothing is written or read outside the buffers,
    the next Solve fails with LMSF_ERR_HIP "device look-back fault", the fault word is cleared by that report, a
    retried Solve with no re-commit finds the windows rebuilt from the keyframe slots (the faulted filter
    had left its window empty) and tracks as a tracker that never faulted, and so does the next commit (look-back words
    re-zeroed)."""
    from conftest import pose_matrix
    wl = sequence_workload
    e, s, _, _ = oracle_mod.extract(wl.scans[0], n_scans=wl.n_scans)
    T0 = pose_matrix(wl.truth[0])
    guess = wl.truth[1]

    def tracker(ctx):
        t = lib.Tracker(ctx, window_frames=4, manual_map_update=True)
        for _ in range(2):                        # >= 2 radix tiles of 8192 pairs in the surf window
            t.add_keyframe(e, s, T0)
        return t

    assert 2 * len(s) > 8192
    ref_ctx = _ctx(lib, n_scans=wl.n_scans)
    ref_t = tracker(ref_ctx)
    ref_t.add_keyframe(e, s, T0)
    ref_t.commit_map()
    ref_ctx.extract(wl.scans[1])
    ref_pose, _ = ref_ctx.solve(guess)

    ref2_ctx = _ctx(lib, n_scans=wl.n_scans)      # the faulted commit's window (2 keyframes), never faulted
    ref2_t = tracker(ref2_ctx)
    ref2_t.commit_map()
    ref2_ctx.extract(wl.scans[1])
    ref2_pose, _ = ref2_ctx.solve(guess)

    ctx = _ctx(lib, n_scans=wl.n_scans)
    t = tracker(ctx)
    ctx.set_option(lib.OPT_FAULT_INJECT, inject)
    t.commit_map()
    ctx.extract(wl.scans[1])                      # completes the faulted commit
    ctx.set_option(lib.OPT_FAULT_INJECT, 0)
    with pytest.raises(lib.LmsfError, match="device look-back fault") as ei:
        ctx.solve(guess)
    assert ei.value.code == lib.ERR_HIP
    pose2, _ = ctx.solve(guess)                   # retried without a commit: the windows were rebuilt
    assert np.array_equal(pose2, ref2_pose)
    t.add_keyframe(e, s, T0)                      # window = 3 copies, as the reference tracker's
    t.commit_map()
    ctx.extract(wl.scans[1])
    pose, _ = ctx.solve(guess)
    assert np.array_equal(pose, ref_pose)
    for x in (t, ref_t, ref2_t):
        x.close()


def test_context_created_beside_running_batch(lib, small_workload):
    """a context is zeroed on its own stream at creation (no hipDeviceSynchronize), so creating one
    while another context's batch runs neither waits for that batch nor disturbs it: the batch's poses equal a
    batch run alone bit for bit, the new context registers, and (when the batch is long enough to tell) its creation
    returned well before the batch finished."""
    import time
    wl = small_workload
    n, B = len(wl.scans), 256
    ctx = _ctx(lib, schedule=1, max_iterations=5, max_batch=B)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.load_scans([wl.scans[i % n] for i in range(B)])
    guesses = np.stack([wl.guess[i % n] for i in range(B)])
    ref, _ = ctx.batch_run(guesses)
    t0 = time.perf_counter()
    ctx.batch_run(guesses)
    dur = time.perf_counter() - t0
    t0 = time.perf_counter()
    _ctx(lib, max_batch=1).close()
    idle = time.perf_counter() - t0
    ctx.batch_launch(guesses)
    t0 = time.perf_counter()
    other = _ctx(lib, max_batch=1)
    busy = time.perf_counter() - t0
    poses, _ = ctx.batch_wait(B)
    assert np.array_equal(poses, ref)
    other.set_map(lib.EDGE, wl.edge_map)
    other.set_map(lib.SURF, wl.surf_map)
    other.extract(wl.scans[0])
    other.set_schedule(lib.SCHEDULE_FIXED)
    other.set_max_iterations(5)
    x, st = other.solve(wl.guess[0])
    dt, dr = pose_err(x, ref[0])              # the 8-lane single-scan path: same registration, other sum order
    assert st.surf_matches > 0 and dt <= POSE_TOL and dr <= POSE_TOL
    if dur > 4 * idle:
        assert busy < idle + 0.5 * dur, (busy, idle, dur)


def test_lm_loop_fault_recovery(lib, oracle_mod, small_workload):
    """A single-scan Solve whose one-launch LM loop gives up its bounded waits (forced: LMSF_OPT_LOOP_FAULT_TEST)
    is re-run on the 9-launch form in the same call: it returns a pose, no error, bit-identical to a Solve on
    the 9-launch form and within rounding of the unfaulted loop (their packet sums differ only in order),
    and later Solves on the loop run clean (the arrival counters were reset).  VERDICT r03 #6, ADVICE r03."""
    wl = small_workload
    ctx = _ctx(lib, max_batch=1, schedule=1, max_iterations=3)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    ctx.extract(wl.scans[0])
    ctx.kernel_stats_reset()
    x_loop, st_loop = ctx.solve(wl.guess[0])
    assert ctx.kernel_stats().loop_recoveries == 0
    ctx.set_option(lib.OPT_LM_LOOP, 0)
    x_multi, _ = ctx.solve(wl.guess[0])
    ctx.set_option(lib.OPT_LM_LOOP, 1)
    ctx.set_option(lib.OPT_LOOP_FAULT_TEST, 1)
    x_rec, st_rec = ctx.solve(wl.guess[0])
    assert ctx.kernel_stats().loop_recoveries >= 1
    assert x_rec.tobytes() == x_multi.tobytes()
    dt, dr = pose_err(x_rec, x_loop)
    assert dt < 1e-9 and dr < 1e-9
    assert st_rec.outer_iterations == st_loop.outer_iterations
    ctx.set_option(lib.OPT_LOOP_FAULT_TEST, 0)
    ctx.kernel_stats_reset()
    for _ in range(2):
        x2, _ = ctx.solve(wl.guess[0])
        assert x2.tobytes() == x_loop.tobytes()
    assert ctx.kernel_stats().loop_recoveries == 0


def test_batch_launch_after_single_load_refused(lib, small_workload):
    """lmsf_extract_features loads one scan into slot 0: a following launch of more slots (whose streamed or
    loaded scans it replaced) fails with LMSF_ERR_STATE instead of extracting stale offsets."""
    import torch
    wl = small_workload
    ctx = _ctx(lib, schedule=1, max_iterations=2, max_batch=2)
    ctx.set_map(lib.EDGE, wl.edge_map)
    ctx.set_map(lib.SURF, wl.surf_map)
    buf = torch.from_numpy(np.concatenate([wl.scans[0], wl.scans[1]], 0)).pin_memory()
    ctx.load_scans_async(buf, np.array([len(wl.scans[0]), len(wl.scans[1])]))
    ctx.extract(wl.scans[2])
    with pytest.raises(lib.LmsfError) as ei:
        ctx.batch_launch(np.stack([wl.guess[0], wl.guess[1]]))
    assert ei.value.code == lib.ERR_STATE
    poses, st = ctx.batch_run(np.stack([wl.guess[2]]))  # one slot: the extracted scan
    assert st[0].surf_matches > 0


@pytest.mark.parametrize("cols", [1800, 4096])
def test_dual_lidar_refine_parity(lib, oracle_mod, cols):
    """C3 phase 1 (ML_System.hpp:284-322): primary tracker Solve, sub-LiDAR features extracted on
    the same context and registered against the primary local map from primary * extrinsic,
    extrinsic = primary^-1 * sub -- against the oracle tracker doing the same.  4096 columns is the
    C3 configuration (2 x ~63k points per frame)."""
    import tracker as OT
    from conftest import mat_err, pose_matrix, relative_truth
    from lmsf import dual, synth
    ds = synth.make_dual_sequence(6, n_cols=cols, step=0.5)
    X = pose_matrix(ds.extrinsic)
    X0 = X @ pose_matrix(np.concatenate([synth.axis_angle_quat(np.radians([0.5, -0.5, 0.5])), [0.03, -0.02, 0.02]]))
    rel = relative_truth(ds.truth)
    sysg = dual.DualLidarSystem(_ctx(lib), extrinsic=X0)
    ot = OT.Tracker()
    ext = X0.copy()
    for i in range(len(ds.truth)):                   # the next frame's extractions run ahead (prefetch)
        nxt = (ds.primary[i + 1], ds.sub[i + 1]) if i + 1 < len(ds.truth) else None
        prim_g, sub_g = sysg.process(ds.primary[i], ds.sub[i], 0.1 * i, next_frame=nxt)
        ep, sp, _, _ = oracle_mod.extract(ds.primary[i])
        es, ss, _, _ = oracle_mod.extract(ds.sub[i])
        _, typ, _ = ot.solve(ep, sp, 0.1 * i)
        prim_o = ot.curr.copy()
        sub_o, _ = ot._register({1: es, 2: ss}, dual.iso_mul(prim_o, ext))
        ext = dual.iso_mul(dual.iso_inv(prim_o), sub_o)
        assert sysg.last["primary_update"] == typ
        for a, b in ((prim_g, prim_o), (sub_g, sub_o), (sysg.extrinsic, ext)):
            dt, dr = mat_err(a, b)
            assert dt <= POSE_TOL and dr <= POSE_TOL, (i, dt, dr)
        dt, dr = mat_err(prim_g, rel[i])
        assert dt < 0.05 and dr < 0.01
    dt, dr = mat_err(sysg.extrinsic, X)
    assert dt < 0.03 and dr < 0.005                   # refined from 6 cm / 0.9 deg
    sysg.close()


def test_reference_interface(lib, oracle_mod, small_workload):
    """The Python mirror of RegistrationBase / PointCloudProcessBase drives the same library."""
    from lmsf import registration as R
    wl = small_workload
    proc = R.LOAMFeatureProcessorHIP(16, 2, 80, max_scan_points=70000)
    feats = proc.Process(wl.scans[0])
    e, s = _features(oracle_mod, wl.scans[0])
    assert feats["loam_edge"].tobytes() == e.tobytes()
    reg = R.make_registration("feature_based_hip", max_features=70000)
    reg.SetInputSource(("loam_edge", wl.edge_map))
    reg.SetInputSource(("loam_surf", wl.surf_map))
    reg.SetInputTarget(feats)
    T = R.to_matrix(wl.guess[0])
    out = reg.Solve(T)
    dt, dr = pose_err(R.to_pose7(out), wl.truth[0])
    assert dt < 0.05 and dr < 0.01
    assert reg.last_stats.outer_iterations == 9


def test_common_process_parity(lib, oracle_mod, small_workload):
    """lmsf_common_process (PointCloudCommonProcess "filtered": removeNaN? -> VoxelGrid -> DistanceFilter)
    == oracle.common_process, points and order, for the shipped parameters and variants."""
    from lmsf import synth
    wl = small_workload
    ctx = _ctx(lib)
    org = synth.make_scan(wl.scene, wl.truth[0], 31, n_cols=4096, organized=True)      # NaN rows kept
    for scan, kw in ((wl.scans[0], {}), (wl.scans[1], dict(voxel_leaf=0.2, distance_near=5.0, distance_far=40.0)),
                     (wl.scans[2], dict(voxel_leaf=0.0)), (wl.scans[0], dict(distance_near=0.0, distance_far=0.0)),
                     (org, dict(removal_nan=1))):
        n = ctx.common_process(scan, **kw)
        want = oracle_mod.common_process(scan, **{k: bool(v) if k == "removal_nan" else v for k, v in kw.items()})
        got, _ = ctx.copy_features(lib.SURF)
        assert n == len(want) and got.tobytes() == want.tobytes(), kw
        assert ctx.copy_features(lib.EDGE)[0].shape[0] == 0


def test_sparse_point_plane_icp_tracking(lib, oracle_mod, sequence_workload):
    """"sparse_point_plane_icp_hip" (ML_SystemFactory.hpp:141-178, point_plane_icp_test.yaml:16-24, 36-37):
    VoxelGrid 0.5 m -> distance 2..100 m -> CeresEdgeSurfFeatureRegistration("", "filtered") against a
    10-keyframe sliding window on {filtered}, 10 scans, against the oracle tracker doing the same."""
    import tracker as OT
    from conftest import relative_truth
    from lmsf import registration as R
    wl = sequence_workload
    rel = relative_truth(wl.truth)
    system = R.ScanMapSystem("sparse_point_plane_icp_hip", ctx=_ctx(lib))
    ot = OT.Tracker(window_frames=10, leaf_edge=0.0, leaf_surf=0.5)
    empty = np.zeros((0, 4), np.float32)
    types = []
    for i, scan in enumerate(wl.scans):
        f = oracle_mod.common_process(scan, voxel_leaf=0.5, distance_near=2.0, distance_far=100.0)
        pose, typ = system.process(scan, wl.dt * i)
        got, _ = system.ctx.copy_features(lib.SURF)
        assert got.tobytes() == f.tobytes()
        _, otyp, _ = ot.solve(empty, f, wl.dt * i)
        assert typ == otyp, i
        assert system.last.local_map_surf == len(ot.local_map(2)) and system.last.local_map_edge == 0
        dt, dr = mat_err(pose, ot.curr)
        assert dt <= POSE_TOL and dr <= POSE_TOL, (i, dt, dr)
        dt, dr = mat_err(pose, rel[i])
        assert dt < 0.1 and dr < 0.02, (i, dt, dr)
        types.append(typ)
    assert 1 in types[1:]
    system.close()
    with pytest.raises(ValueError):
        R.PointCloudCommonProcessHIP().SetVoxelGrid("ApproximateVoxelGrid", 0.5)
    reg = R.make_registration("sparse_point_plane_icp_hip", max_features=70000)
    assert (reg.edge_name, reg.surf_name) == ("", "filtered")


def test_dist_example(lib, oracle_mod, small_workload, tmp_path):
    """The C multi-GPU plumbing (liblmsf_dist.so over RCCL) driven by a C program, one rank: map broadcast
    into device memory, extraction + registration from it, pose all-gather, keyframe exchange, max --
    the pose equals the oracle's, the gathered pose and keyframe buffer equal the rank's own."""
    import subprocess
    from test_abi import build_dist_example
    wl = small_workload
    exe = build_dist_example(tmp_path)
    paths = []
    for name, arr in (("scan", wl.scans[0]), ("edge", wl.edge_map), ("surf", wl.surf_map)):
        p = tmp_path / f"{name}.bin"
        np.ascontiguousarray(arr, np.float32).tofile(p)
        paths.append(str(p))
    g = wl.guess[0]
    out = subprocess.run([exe, "1", "0", str(tmp_path / "group.id"), *paths, *[repr(float(v)) for v in g], "5"],
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    f = out.stdout.strip().splitlines()[-1].split()     # RCCL may print its banner first
    x = np.array([float(v) for v in f[2:9]])
    assert f[9] == "1" and f[10] == "1" and float(f[11]) == 1.5
    e, s = _features(oracle_mod, wl.scans[0])
    assert (int(f[0]), int(f[1])) == (len(e), len(s))
    reg = oracle_mod.Registration()
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    reg.set_fixed_schedule(True)
    reg.set_max_iterations(5)
    ox, _, _ = reg.solve(g)
    dt, dr = pose_err(x, ox)
    assert dt <= POSE_TOL and dr <= POSE_TOL


def test_tracker_keyframe_lookahead_exact(lib, oracle_mod, sequence_workload):
    """The keyframe lookahead (lmsf_tracker_config.keyframe_lookahead: the window rebuild with the scan's features at
    the Solve's device-resident result, posted while the Solve runs; used while the tracker is alone on its device,
    with the flag-ordered fork / join) changes nothing: a manual-mode tracker on an extracted sequence, lookahead on and
    off, gives bit-identical poses, decisions, map sizes and final local maps -- while the caller adopts it (its own
    keyframe at lmsf_tracker_pose), skips a keyframe the gate asked for, appends host features instead, or appends at a
    different pose (each of the last three undoes it), where the prediction and the gate disagree (window of 3,
    mixed decisions), and where the Solve is recovered (LMSF_OPT_LOOP_FAULT_TEST: the lookahead is undone and the
    window rebuilt before the re-run)."""
    wl = sequence_workload

    def run(look):
        import gc
        gc.collect()   # earlier tests' unreferenced trackers gone: the lookahead needs its tracker alone on the device
        ctx = _ctx(lib, n_scans=wl.n_scans, max_batch=1)
        tr = lib.Tracker(ctx, window_frames=3, manual_map_update=True, keyframe_lookahead=look)
        ctx.kernel_stats_reset(timing=False)
        steps, faulted_look = [], []
        for i, scan in enumerate(wl.scans):
            ctx.extract(scan)
            ctx.set_option(lib.OPT_LOOP_FAULT_TEST, 1 if i in (2, 6) else 0)   # recovered Solves (undo first)
            l0 = ctx.kernel_stats().lookahead_solves
            _, r = tr.solve_extracted(wl.dt * i)
            if i in (2, 6):
                faulted_look.append(ctx.kernel_stats().lookahead_solves > l0)
            P = tr.pose()
            if r.update_type:
                if i == 3:
                    pass                                          # the gate's keyframe skipped by the caller
                elif i == 5:
                    ge, _ = ctx.copy_features(lib.EDGE)
                    gs, _ = ctx.copy_features(lib.SURF)
                    tr.add_keyframe(ge, gs, P)                    # the same frame, as host data
                    tr.commit_map()
                elif i == 7:
                    Q = P.copy()
                    Q[0, 3] += 0.01
                    tr.add_keyframe_extracted(Q)                  # another pose
                    tr.commit_map()
                else:
                    tr.add_keyframe_extracted(P)
                    tr.commit_map()
            steps.append((P, r.update_type, r.local_map_edge, r.local_map_surf))
        maps = [tr.local_map(k) for k in (lib.EDGE, lib.SURF)]
        ks = ctx.kernel_stats()
        tr.close()
        return steps, maps, ks.lookahead_solves, ks.loop_recoveries, faulted_look

    a, ma, la, ra, fa = run(True)
    b, mb, lb, rb, _ = run(False)
    assert la >= 3 and lb == 0, (la, lb)
    assert ra == rb == 2 and any(fa), (ra, rb, fa)      # a recovered Solve with its lookahead posted
    for i, ((Pa, ta, ea, sa), (Pb, tb, eb, sb)) in enumerate(zip(a, b)):
        assert np.array_equal(Pa, Pb), (i, Pa - Pb)
        assert (ta, ea, sa) == (tb, eb, sb), i
    assert 0 in [s[1] for s in a[1:]] and 1 in [s[1] for s in a[1:]]
    for x, y in zip(ma, mb):
        assert x.tobytes() == y.tobytes()
