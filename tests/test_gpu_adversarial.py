"""GPU parity on SURVEY §7's hard parts: the adversarial fixture (tests/golden/adversarial.npz,
tests/adversarial_fixture.py) merged into the synthetic background, run through every search path --

* `knn8`:  the single-scan 8-lane `knn_kernel<8>` with the slot memo + `fit_eval` + the LM loop (3 x 70k slots),
* `fused`: the batch path's fused `match_fit_kernel` with the query memo (`match_memo_kernel`, listed searches),
* `dense`: the same on a dense background (the C5 regime): first-pass grid `dense_pass1` / `dense_pass2` /
           `dense_fit2`, the dense memo from outer iteration 3 and its listed passes --

over 5 outer iterations (`lmsf_batch_capture`): the records (kRecNone unmatched markers included; NaN fields
compared by NaN-ness, adversarial_fixture.canon) and the 5-NN indices after every outer iteration equal the
oracle's fresh match at the pose the GPU matched at, the per-iteration poses equal the oracle's, and the slot
whose record is a degenerate NaN fit keeps its guess like the oracle.  REG/FeatureMatch/EdgeFeatureMatch.hpp:38-84,
surfFeatureMatch.hpp:37-85, ceres_factor/edge_factor.hpp:41-57, ceres_edgeSurfFeatureRegistration.hpp:105-125."""
import numpy as np
import pytest

import adversarial_fixture as af
from conftest import pose_err

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-4


@pytest.fixture(scope="module")
def lib():
    from lmsf import _lib
    _lib.load()
    return _lib


@pytest.fixture(scope="module")
def adv(oracle_mod, small_workload):
    from lmsf import synth
    fx = af.load()
    wl = small_workload
    scan = wl.scans[0]
    assert af.scan_sha(scan) == str(fx["scan_sha"]), "synthetic scan 0 changed: regenerate the fixture"
    e, s, _, _ = oracle_mod.extract(scan)
    sets, ts = af.sets_from_fixture(fx, e, s)
    planted, first = af.planted_maps(sets)
    truth = wl.truth[0]
    sparse = {k: af.combined_map(planted, af.to_lidar(bg, truth), sets, k) for k, bg in ((1, wl.edge_map), (2, wl.surf_map))}
    dw = synth.make_workload("C2", n_scans=1, map_points=1_000_000, radius=30.0, road_length=20.0)
    assert np.array_equal(dw.truth[0], truth)
    dense = {k: af.combined_map(planted, af.to_lidar(bg, truth), sets, k) for k, bg in ((1, dw.edge_map), (2, dw.surf_map))}
    guesses = np.stack([af.pose(t) for t in ts])
    return dict(fx=fx, scan=scan, e=e, s=s, sets=sets, maps={"sparse": sparse, "dense": dense}, guesses=guesses)


def _slice_density(m):
    p = m[:, :3].astype(np.float32)
    c = np.stack([np.floor(p[:, 0] * 4), np.floor(p[:, 1]), np.floor(p[:, 2])], 1).astype(np.int64)
    return len(p) / len(np.unique(c, axis=0))


def _oracle(oracle_mod, maps, e, s):
    reg = oracle_mod.Registration()
    reg.set_map(1, maps[1])
    reg.set_map(2, maps[2])
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    reg.set_fixed_schedule(True)
    reg.set_max_iterations(5)
    return reg


def _same_records(grec, gnn, orec, onn, what):
    assert len(grec) == len(orec), what
    found = gnn >= 0
    assert np.array_equal(gnn[found], onn[found]), (what, int((gnn[found] != onn[found]).sum()))
    assert found[orec["kind"] > 0].all(), what                 # a record needs its 5 found within 1 m
    a, b = af.canon(grec), af.canon(orec)
    if a.tobytes() != b.tobytes():
        diff = np.nonzero((a.view(np.uint8).reshape(len(a), -1) != b.view(np.uint8).reshape(len(b), -1)).any(1))[0]
        raise AssertionError(f"{what}: {len(diff)} records differ, first {diff[:5]}: gpu {grec[diff[:2]]} "
                             f"oracle {orec[diff[:2]]}")


def _planted_rows(adv, slot):
    """(record row, fixture row) of every planted query of `slot` (records: edges first, slot order)."""
    ne = len(adv["e"])
    return [((st[2] if st[1] == 1 else ne + st[2]), k) for k, st in enumerate(adv["sets"]) if st[0] == slot]


PATHS = {"knn8": ("sparse", 70000), "fused": ("sparse", 1 << 19), "dense": ("dense", 1 << 19)}


@pytest.mark.parametrize("path", list(PATHS))
def test_adversarial_batch_parity(lib, oracle_mod, adv, path):
    which, F = PATHS[path]
    maps = adv["maps"][which]
    assert (_slice_density(maps[2]) >= 8) == (which == "dense")
    e, s, g = adv["e"], adv["s"], adv["guesses"]
    ctx = lib.Context(max_batch=3, max_scan_points=70000, max_features=F, schedule=1, max_iterations=5)
    ctx.set_map(lib.EDGE, maps[1])
    ctx.set_map(lib.SURF, maps[2])
    ctx.load_scans([adv["scan"]] * 3)
    ctx.batch_capture([0, 1, 2])
    ctx.kernel_stats_reset(timing=True)
    poses, stats = ctx.batch_run(g)
    ks = ctx.kernel_stats()
    assert ks.fused_launches == (0 if path == "knn8" else 5), path
    assert ks.reused_queries > 0                                 # the memo served queries beside the corner cases
    reg = _oracle(oracle_mod, maps, e, s)
    fx = adv["fx"]
    for slot in range(3):
        for it in range(5):
            grec, gnn, gpose = ctx.batch_records(slot, it)
            orec, onn = reg.match(gpose)
            _same_records(grec, gnn, orec, onn, f"{path} slot {slot} outer iteration {it}")
            if it == 0:   # the planted queries at the guess: the committed oracle vectors (planted points alone)
                assert np.array_equal(gpose, g[slot])
                for row, k in _planted_rows(adv, slot):
                    assert af.canon(grec[row:row + 1]).tobytes() == af.canon(fx["rec"][k:k + 1]).tobytes(), \
                        (path, str(fx["label"][k]))
                    f = gnn[row] >= 0
                    assert np.array_equal(gnn[row][f], fx["nn"][k][f]), (path, str(fx["label"][k]))
        ox, otr, ost = reg.solve(g[slot])
        gtr = ctx.batch_trace(slot)
        assert gtr.shape == otr.shape == (5, 7), (path, slot)
        for a, b in zip(gtr, otr):
            dt, dr = pose_err(a, b)
            assert dt <= POSE_TOL and dr <= POSE_TOL, (path, slot, dt, dr)
        assert (stats[slot].edge_matches, stats[slot].surf_matches) == (ost.edge_matches, ost.surf_matches)
    # the degenerate NaN record (slot 2) stops the LM at its guess, as in the oracle
    assert np.array_equal(poses[2], g[2]) and all(np.array_equal(t, g[2]) for t in ctx.batch_trace(2))
    if path != "knn8":    # memo on / off: the same poses bit for bit
        ctx.batch_capture([])
        ctx.set_option(lib.OPT_QUERY_MEMO, 0)
        try:
            poses0, _ = ctx.batch_run(g)
        finally:
            ctx.set_option(lib.OPT_QUERY_MEMO, 1)
        assert np.array_equal(poses0, poses), path


@pytest.mark.parametrize("path", list(PATHS))
def test_adversarial_single_match(lib, oracle_mod, adv, path):
    """lmsf_match (SetInputSource + one Match at a pose) on the device-extracted scan at each slot's guess:
    8-lane teams (70k slots) or the one-lane search + fit (2^19 slots; the pruned walk on the dense map)."""
    which, F = PATHS[path]
    maps = adv["maps"][which]
    ctx = lib.Context(max_batch=1, max_scan_points=70000, max_features=F)
    ctx.set_map(lib.EDGE, maps[1])
    ctx.set_map(lib.SURF, maps[2])
    assert ctx.extract(adv["scan"]) == (len(adv["e"]), len(adv["s"]))
    reg = _oracle(oracle_mod, maps, adv["e"], adv["s"])
    for slot in range(3):
        g = adv["guesses"][slot]
        grec, gnn = ctx.match(g, len(adv["e"]) + len(adv["s"]))
        orec, onn = reg.match(g)
        _same_records(grec, gnn, orec, onn, f"{path} match slot {slot}")


def _same_traces(gtr, otr, what):
    """Per-outer-iteration poses: equal NaN pattern (a NaN record poisons Gauss-Newton's normal equations on both
    sides), else within POSE_TOL."""
    assert gtr.shape == otr.shape, (what, gtr.shape, otr.shape)
    for a, b in zip(gtr, otr):
        assert np.array_equal(np.isnan(a), np.isnan(b)), (what, a, b)
        if not np.isnan(a).any():
            dt, dr = pose_err(a, b)
            assert dt <= POSE_TOL and dr <= POSE_TOL, (what, dt, dr)


def test_adversarial_gauss_newton(lib, oracle_mod, adv):
    """The GN variant (REG/edgeSurfFeatureRegistration.hpp:218-330: JᵀJ by colPivHouseholderQr, the degeneracy
    projection from SelfAdjointEigenSolver<MatrixXd> at iteration 0, its convergence test) on the adversarial scene,
    every slot to convergence: the records after every outer iteration equal the oracle's at the GPU's pose, and the
    per-iteration poses (NaN pattern included: the origin slot's NaN record) equal the oracle GN's."""
    maps = adv["maps"]["sparse"]
    e, s, g = adv["e"], adv["s"], adv["guesses"]
    ctx = lib.Context(max_batch=3, max_scan_points=70000, max_features=70000, solver=lib.SOLVER_GN, schedule=1,
                      max_iterations=5)
    ctx.set_map(lib.EDGE, maps[1])
    ctx.set_map(lib.SURF, maps[2])
    ctx.load_scans([adv["scan"]] * 3)
    ctx.batch_capture([0, 1, 2])
    poses, stats = ctx.batch_run(g)
    reg = oracle_mod.Registration(oracle_mod.SOLVER_GN)
    reg.set_map(1, maps[1])
    reg.set_map(2, maps[2])
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    reg.set_fixed_schedule(True)
    reg.set_max_iterations(5)
    for slot in range(3):
        gtr = ctx.batch_trace(slot)
        for it in range(len(gtr)):
            grec, gnn, gpose = ctx.batch_records(slot, it)
            if np.isnan(gpose).any():
                break
            orec, onn = reg.match(gpose)
            _same_records(grec, gnn, orec, onn, f"GN slot {slot} outer iteration {it}")
        ox, otr, ost = reg.solve(g[slot])
        _same_traces(gtr, otr, f"GN slot {slot}")
        assert stats[slot].termination == ost.termination, (slot, stats[slot].termination, ost.termination)


def test_tracker_split_search_ties(lib, oracle_mod, adv):
    """A tracker Solve whose outer iteration 0 runs split (ctx_presearch: the prior grids' walk enqueued beside the
    keyframe window rebuild, then the window pass seeded with its keys; knn_kernel SPLIT 1 / 2) on the adversarial
    scene as the prior map and a keyframe of exact copies of every planted point as the window (identity pose, no
    voxel filter): every planted candidate ties across the two grids at equal d^2, so each query's kept keys interleave
    prior and window points and only the index order (prior first) decides them.  The records and 5-NN indices after
    every outer iteration equal the oracle's fresh match over [prior | window] at the GPU's pose, and the poses follow
    the oracle's registration (LidarTrackerLocalMap.hpp:125-133 / ceres_edgeSurfFeatureRegistration.hpp:100-125)."""
    maps = adv["maps"]["sparse"]
    planted, _ = af.planted_maps(adv["sets"])
    g = adv["guesses"][0]
    T0 = np.eye(4)
    T0[:3, 3] = g[4:]
    ctx = lib.Context(max_batch=1, max_scan_points=70000, max_features=70000)
    tr = lib.Tracker(ctx, manual_map_update=True, leaf_edge=0.0, leaf_surf=0.0)
    tr.set_initial_pose(T0)
    tr.set_prior_map(lib.EDGE, maps[1])
    tr.set_prior_map(lib.SURF, maps[2])
    ctx.extract(adv["scan"])
    _, r0 = tr.solve_extracted(0.0)
    assert r0.initialized
    tr.add_keyframe(planted[1], planted[2], np.eye(4))
    tr.commit_map()
    ctx.batch_capture([0])
    ctx.kernel_stats_reset()
    ctx.extract(adv["scan"])       # settles the commit: the prior pass at the prediction T0 goes first
    _, r = tr.solve_extracted(0.1)
    assert ctx.kernel_stats().split_searches == 1
    assert (r.local_map_edge, r.local_map_surf) == (len(maps[1]) + len(planted[1]), len(maps[2]) + len(planted[2]))
    reg = oracle_mod.Registration()
    for k in (1, 2):
        reg.set_map(k, np.concatenate([maps[k], planted[k]], 0))
    reg.set_scan(1, adv["e"])
    reg.set_scan(2, adv["s"])
    ox, otr, ost = reg.solve(g)
    n = r.solve.outer_iterations
    assert n == len(otr), (n, otr.shape)
    window_nn = 0
    for it in range(min(n, 10)):
        grec, gnn, gpose = ctx.batch_records(0, it)
        if it == 0:
            assert np.array_equal(gpose, g)
        else:
            dt, dr = pose_err(gpose, otr[it - 1])
            assert dt <= POSE_TOL and dr <= POSE_TOL, (it, dt, dr)
        orec, onn = reg.match(gpose)
        _same_records(grec, gnn, orec, onn, f"split tracker outer iteration {it}")
        ne = len(adv["e"])
        window_nn += int((gnn[:ne] >= len(maps[1])).sum() + (gnn[ne:] >= len(maps[2])).sum())
    assert window_nn > 0                                        # window points won places in the kept sets
