"""The adversarial fixture (tests/golden/adversarial.npz, SURVEY §7's hard parts) on the CPU: the planted
geometry regenerates bit for bit, every designed property holds by independent arithmetic (numpy float
d^2, a brute-force (d^2, index) sort), and the oracle's records / 5-NN equal the committed ones.
REG/FeatureMatch/EdgeFeatureMatch.hpp:38-84, surfFeatureMatch.hpp:37-85, ceres_factor/edge_factor.hpp:41-57."""
import numpy as np
import pytest

import adversarial_fixture as af

F32 = np.float32


@pytest.fixture(scope="module")
def adv(oracle_mod):
    from lmsf import synth
    fx = af.load()
    wl = synth.make_workload("C2", n_scans=3, map_points=1000)
    assert af.scan_sha(wl.scans[0]) == str(fx["scan_sha"]), "synthetic scan 0 changed: regenerate the fixture"
    e, s, _, _ = oracle_mod.extract(wl.scans[0])
    sets, ts = af.sets_from_fixture(fx, e, s)
    return fx, sets, ts, e, s


def test_planted_geometry_regenerates(adv):
    fx, sets, ts, e, s = adv
    maps, first = af.planted_maps(sets)
    assert maps[1].tobytes() == fx["edge_map"].tobytes() and maps[2].tobytes() == fx["surf_map"].tobytes()
    np.testing.assert_array_equal(first, fx["first"])
    np.testing.assert_array_equal(np.stack([st[4] for st in sets]), fx["W"])
    for slot, kind, i, label, W, pts, exp in sets:
        q = (e if kind == 1 else s)[i]
        if slot == 0:    # the LM's double point is the float W (pointAssociateToMap under the identity)
            assert np.array_equal(W.astype(np.float64), np.asarray(q[:3], np.float64) + ts[0]), label
    Wc = [st[4] for st in sets if st[3] == "edge_corner_on_line"][0]
    assert float(Wc[0]) * 4 == np.floor(float(Wc[0]) * 4) and float(Wc[1]) == np.floor(Wc[1]) and \
        float(Wc[2]) == np.floor(Wc[2])                       # x on a slice boundary, y / z on cell boundaries


def _brute_5nn(mp, W):
    d = af.d2f(W, mp[:, :3])
    order = np.lexsort((np.arange(len(mp)), d))              # ascending d^2, ties by map index
    return order[:5], d[order[:5]]


def test_designed_properties(adv):
    fx, sets, ts, e, s = adv
    maps, first = af.planted_maps(sets)
    for k, (slot, kind, i, label, W, pts, exp) in enumerate(sets):
        nn, d = _brute_5nn(maps[kind], W)
        f = first[k]
        if label.endswith("gate_eq") or label.endswith("gate_round"):
            assert d[4] == F32(1.0), label
        if label.endswith("gate_below"):
            assert d[4] == np.nextafter(F32(1.0), F32(0)), label
        if label == "surf_gate_round":
            assert af.d2f(W, pts[4]) == F32(1.0) and pts[4][1] != W[1]   # off-axis: 1.0f by rounding
        if label == "surf_ulp56":      # 5th / 6th tied by rounding (index order), 7th one ulp above
            assert d[4] == F32(0.25) and af.d2f(W, pts[5]) == F32(0.25) and \
                af.d2f(W, pts[6]) == np.nextafter(F32(0.25), F32(1)) and nn[4] == f + 4
            assert not np.array_equal(pts[4], pts[5])
        if label == "edge_ulp56":
            assert d[4] == F32(0.25) and nn[4] == f + 5 and af.d2f(W, pts[4]) == np.nextafter(F32(0.25), F32(1))
        if label.endswith("dup56"):    # an exact duplicate pair at ranks 5 / 6
            j = 4 if label.startswith("surf") else 4
            assert np.array_equal(pts[j], pts[j + 1]) and nn[4] == f + j, label
        if label.endswith("equi567"):  # three distinct points at one float d^2
            dd = af.d2f(W, pts[4:7])
            assert dd[0] == dd[1] == dd[2] and len({p.tobytes() for p in pts[4:7]}) == 3 and nn[4] == f + 4, label
        if label.endswith("coincident5") or label == "surf_origin_nan":
            assert all(np.array_equal(p, pts[0]) for p in pts), label
        if exp in ("match", "online", "nan"):
            assert d[4] < F32(1.0), label


def test_oracle_pinned_on_fixture(adv, oracle_mod):
    """The oracle's records and 5-NN of the planted queries (planted points alone) equal the committed
    fixture; the 5-NN equal the brute-force sort; kinds follow the design (unmatched at the gate and for
    a zero edge covariance, a matched NaN surf record at the origin, |nu| = 0 on the fitted line)."""
    fx, sets, ts, e, s = adv
    maps, first = af.planted_maps(sets)
    import sys
    sys.path.insert(0, af.HERE + "/golden")
    from make_adversarial import oracle_planted
    recs, nns = oracle_planted(sets, maps, ts, e, s)
    np.testing.assert_array_equal(nns, fx["nn"])
    assert af.canon(recs).tobytes() == af.canon(fx["rec"]).tobytes()
    for k, (slot, kind, i, label, W, pts, exp) in enumerate(sets):
        nn, _ = _brute_5nn(maps[kind], W)
        np.testing.assert_array_equal(nns[k], nn, err_msg=label)
        r = recs[k]
        vals = np.concatenate([r["v0"], r["v1"]])
        if exp == "none":
            assert r["kind"] == 0, label
        elif exp in ("match", "online"):
            assert r["kind"] == kind and np.isfinite(vals).all(), label
        elif exp == "nan":
            assert r["kind"] == kind and np.isnan(vals).any(), label
        if exp == "online":            # residual 0 and the zero Jacobian at the guess (edge_factor.hpp:57)
            pk = oracle_mod.eval_records(recs[k:k + 1], af.pose(ts[slot]))
            assert pk[0] == 0.0 and not pk[1:28].any() and pk[28] == 1.0, label


def test_origin_nan_record_stalls_lm(adv, oracle_mod):
    """A matched record of NaN (5 map points at the origin: the QR solution is non-finite) makes the first
    evaluation's cost NaN: the LM stops with the pose unchanged at every outer iteration (Ceres: the
    initial evaluation fails, x untouched)."""
    fx, sets, ts, e, s = adv
    maps, _ = af.planted_maps(sets)
    st = [st for st in sets if st[3] == "surf_origin_nan"][0]
    reg = oracle_mod.Registration()
    reg.set_map(2, maps[2])
    reg.set_scan(2, s[st[2]:st[2] + 1])
    reg.set_fixed_schedule(True)
    reg.set_max_iterations(5)
    g = af.pose(ts[2])
    x, tr, ost = reg.solve(g)
    assert np.array_equal(x, g) and ost.outer_iterations == 5 and ost.surf_matches == 1
    assert all(np.array_equal(t, g) for t in tr)
