"""Adversarial registration fixture: SURVEY.md §7's "hard parts" planted around chosen scan features
(VERDICT r05 #1).  Test infrastructure only (imported by tests/ and tests/golden/make_adversarial.py).

The scene is the C2-shaped synthetic scan of `conftest.small_workload` (scan 0) in its own LiDAR frame
(truth = identity), registered from guesses with the identity rotation, so a feature q matches at the
world point W = float(q + t) (pointAssociateToMap, REG/ceres_edgeSurfFeatureRegistration.hpp:235-244:
double transform, stored as float) -- exactly computable here.  Around chosen features the background
map is cleared (CLEAR m) and hand-built neighbourhoods are planted at float-exact positions:

* exact duplicate map points at ranks 5 / 6, three distinct points at one float d^2 (ranks 5-7), a 5th /
  6th pair one ulp apart and a 5th / 7th pair tied by rounding (EdgeFeatureMatch.hpp:38 /
  surfFeatureMatch.hpp:37 nearestKSearch(5): FLANN leaves equal distances unordered; the canonical
  order is ascending map index);
* the `sqd[4] < 1.0` gate (EdgeFeatureMatch.hpp:40, surfFeatureMatch.hpp:42) with the 5th neighbour at
  float d^2 == 1.0f (on the axis, and reached by rounding from an off-axis point) and one ulp below;
* degenerate fits: 5 coincident points (zero edge covariance, EdgeFeatureMatch.hpp:63; rank-1 plane
  system, surfFeatureMatch.hpp:52-54), collinear points (rank-2 QR), two clusters, fewer than 5 points
  within 1 m, and 5 points at the world origin, whose column-pivoting QR solution is non-finite: a
  matched surf record of NaN / inf (D = 1 / |n|, surfFeatureMatch.hpp:54) that stalls Ceres' LM;
* an edge query exactly on its fitted line (|nu| = 0, ceres_factor/edge_factor.hpp:57);
* a query on a cell corner (x on a 0.25 m slice boundary, y / z on 1 m cell boundaries) with neighbours
  on the boundary planes and points exactly 1 m across them.

Slot 0 (guess t0, a multiple of 2^-10: every chosen W equals q + t0 exactly in double, so the LM's
double-precision point is the float W) holds most cases; slot 1 aligns one edge query to a cell corner;
slot 2 translates a surf feature next to the origin structure.
"""
from __future__ import annotations

import hashlib
import os

import numpy as np

F32 = np.float32
HERE = os.path.dirname(os.path.abspath(__file__))
FIXTURE = os.path.join(HERE, "golden", "adversarial.npz")
SEP = 6.0          # chosen queries' world points at least this far apart (and from the origin)
CLEAR = 2.5        # background map points removed within this radius of every planted query / the origin
T0 = np.array([41.0, -31.0, 20.0]) / 1024.0     # slot 0 translation (2^-10 grid)
ORIGIN_W = np.array([0.125, -0.25, 0.1875])     # slot 2: where the origin case's query lands
NEAR4 = np.array([[0.125, 0.0625, 0.0], [-0.1875, 0.109375, 0.015625],
                  [0.21875, -0.125, -0.0078125], [-0.09375, -0.25, 0.0117188]])


def pose(t):
    return np.array([0.0, 0.0, 0.0, 1.0, t[0], t[1], t[2]])


def d2f(W, M):
    """float d^2 as FLANN L2_Simple and the kernels compute it: ((dx*dx + dy*dy) + dz*dz) in float32."""
    d = np.asarray(W, F32) - np.asarray(M, F32)
    sq = d * d
    return (sq[..., 0] + sq[..., 1]) + sq[..., 2]


def world(q, t):
    """float(q + t): pointAssociateToMap under the identity rotation (exact)."""
    return (np.asarray(q[:3], np.float64) + t).astype(F32)


def to_lidar(points, truth):
    """World map rows into the LiDAR frame of `truth` (float64 math, float32 out)."""
    from lmsf import synth
    R = synth.quat_to_mat(truth[:4])
    out = points.copy()
    out[:, :3] = ((points[:, :3].astype(np.float64) - np.asarray(truth[4:])) @ R).astype(F32)
    return out


def scan_sha(scan):
    return hashlib.sha256(np.ascontiguousarray(scan, F32).tobytes()).hexdigest()


def find_point(W, target, axis, sign, adj, need_adj=False, K=64, J=1 << 14):
    """A float32 point M with d2f(W, M) == target exactly: M[axis] near W[axis] + sign sqrt(target)
    (+- K ulps), M[adj] = W[adj] + j ulps (0 <= j < J; j > 0 when need_adj), the third coordinate W's."""
    W = np.asarray(W, F32)
    target = F32(target)
    r = float(np.sqrt(np.float64(target)))
    base = F32(np.float64(W[axis]) + sign * r)
    ua = np.spacing(np.abs(base)) if base != 0 else np.spacing(F32(1e-30))
    ca = (np.float64(base) + np.arange(-K, K + 1) * np.float64(ua)).astype(F32)
    ub = np.spacing(np.abs(W[adj])) if W[adj] != 0 else np.spacing(F32(1e-6))
    cb = (np.float64(W[adj]) + np.arange(0, J) * np.float64(ub)).astype(F32)
    M = np.empty((ca.size, cb.size, 3), F32)
    M[...] = W
    M[:, :, axis] = ca[:, None]
    M[:, :, adj] = cb[None, :]
    ok = d2f(W, M) == target
    if need_adj:
        ok[:, 0] = False
    ii, jj = np.nonzero(ok)
    if ii.size == 0:
        raise RuntimeError(f"no float point at d2 {target!r} around {W}")
    k = np.lexsort((np.abs(ii - K), jj))[0]
    return M[ii[k], jj[k]].copy()


def near_points(W, offsets):
    return [(np.asarray(W, np.float64) + o).astype(F32) for o in offsets]


# ----------------------------------------------------------------------------------------------- cases
def surf_cases(W):
    """label -> (planted points in index order, expectation) for a surf query at W (slot 0)."""
    near = near_points(W, NEAR4)
    c = {}
    dup = (np.asarray(W, np.float64) + [0.375, 0.375, 0.0]).astype(F32)
    c["surf_dup56"] = lambda: (near + [dup, dup.copy(), *near_points(W, [[0.5, -0.4375, 0.0]])], "match")
    def equi():
        e1 = find_point(W, d2f(W, (np.asarray(W, np.float64) + [0.5, 0.3, 0.0]).astype(F32)), 0, +1, 1)
        D = d2f(W, e1)
        return near + [find_point(W, D, 1, -1, 0), find_point(W, D, 0, -1, 1), e1], "match"   # lowest index wins

    def ulp56():
        p5 = find_point(W, F32(0.25), 0, +1, 1)
        p6 = find_point(W, np.nextafter(F32(0.25), F32(1)), 0, +1, 1, need_adj=True)
        p7 = find_point(W, F32(0.25), 1, +1, 0, need_adj=True)      # equal float d^2, other coordinates
        return near + [p7, p5, p6], "match"
    c["surf_equi567"] = equi
    c["surf_ulp56"] = ulp56
    c["surf_gate_eq"] = lambda: (near + [find_point(W, F32(1.0), 0, +1, 1),
                                 *near_points(W, [[0.0, 1.25, 0.0]])], "none")
    c["surf_gate_round"] = lambda: (near + [find_point(W, F32(1.0), 0, -1, 1, need_adj=True)], "none")
    c["surf_gate_below"] = lambda: (near + [find_point(W, np.nextafter(F32(1.0), F32(0)), 0, +1, 1, need_adj=True),
                                    find_point(W, F32(1.0), 0, -1, 1)], "match")
    c["surf_collinear_axis"] = lambda: (near_points(W, [[a, 0.25, 0.125] for a in (-0.296875, -0.09375, 0.046875,
                                                                           0.203125, 0.34375)]), "any")
    c["surf_collinear_diag"] = lambda: (near_points(W, [[0.0625 + k * 0.09375, -0.125 + k * 0.0625, k * 0.03125]
                                                for k in (-3, -1, 0, 2, 4)]), "any")
    co = (np.asarray(W, np.float64) + [0.1875, 0.125, 0.0625]).astype(F32)
    c["surf_coincident5"] = lambda: ([co.copy() for _ in range(5)], "any")
    co7 = (np.asarray(W, np.float64) + [-0.1875, 0.125, -0.0625]).astype(F32)
    c["surf_coincident7"] = lambda: ([co7.copy() for _ in range(7)], "any")
    a = (np.asarray(W, np.float64) + [0.25, 0.0, 0.0]).astype(F32)
    b = (np.asarray(W, np.float64) + [-0.125, 0.3125, 0.0]).astype(F32)
    c["surf_two_clusters"] = lambda: ([a, a.copy(), a.copy(), b, b.copy()], "any")
    c["surf_few4"] = lambda: (near + near_points(W, [[1.3125, 0.0, 0.0], [0.0, -1.375, 0.0]]), "none")
    c["surf_plane_fail"] = lambda: (near_points(W, [[0.5, 0.0, 0.0], [-0.5, 0.0, 0.0], [0.0, 0.0, 0.75],
                                            [0.0, 0.0, -0.75], [0.0, 0.625, 0.0]]), "any")
    c["surf_q_on_point"] = lambda: ([np.asarray(W, F32).copy()] + near, "match")
    # neighbours on the cell / slice boundary planes nearest W (x: 0.25 m slices, y / z: 1 m cells)
    Wd = np.asarray(W, np.float64)
    bx, by, bz = np.round(Wd[0] * 4) / 4, np.round(Wd[1]), np.round(Wd[2])
    pts = [np.array([bx, Wd[1] + 0.0625, Wd[2]]), np.array([Wd[0] + 0.125, by, Wd[2]]),
           np.array([Wd[0], Wd[1] - 0.125, bz]), np.array([bx, by, Wd[2] + 0.0625]),
           np.array([bx, Wd[1] - 0.1875, bz])]
    c["surf_boundary_pts"] = lambda: ([p.astype(F32) for p in pts], "any")
    return c


def edge_cases(W):
    near_line = near_points(W, [[0.125, 0.0, 0.0078125], [-0.1875, 0.0, -0.0078125],
                                [0.25, 0.0078125, 0.0], [-0.3125, -0.0078125, 0.0]])
    c = {}
    co = (np.asarray(W, np.float64) + [0.125, 0.1875, 0.0625]).astype(F32)
    c["edge_coincident5"] = lambda: ([co.copy() for _ in range(5)], "none")   # zero covariance: no line
    c["edge_on_line"] = lambda: (near_points(W, [[a, 0.0, 0.0] for a in (-0.375, -0.1875, 0.0625, 0.25, 0.4375)]), "online")
    dup = (np.asarray(W, np.float64) + [0.4375, 0.0, 0.0]).astype(F32)
    c["edge_dup56"] = lambda: (near_line + [dup, dup.copy()], "match")
    def equi():
        e1 = find_point(W, d2f(W, (np.asarray(W, np.float64) + [0.5, 0.05, 0.0]).astype(F32)), 0, +1, 1)
        D = d2f(W, e1)
        return near_line + [find_point(W, D, 0, -1, 1), find_point(W, D, 0, +1, 2, need_adj=True), e1], "match"
    c["edge_equi567"] = equi
    c["edge_gate_eq"] = lambda: (near_line + [find_point(W, F32(1.0), 0, +1, 1)], "none")
    c["edge_gate_below"] = lambda: (near_line + [find_point(W, np.nextafter(F32(1.0), F32(0)), 0, -1, 1, need_adj=True)],
                            "match")
    c["edge_ulp56"] = lambda: (near_line + [find_point(W, np.nextafter(F32(0.25), F32(1)), 0, -1, 1, need_adj=True),
                                            find_point(W, F32(0.25), 0, +1, 1)], "match")
    a = (np.asarray(W, np.float64) + [0.25, 0.125, 0.0]).astype(F32)
    b = (np.asarray(W, np.float64) + [-0.25, -0.125, 0.0]).astype(F32)
    c["edge_two_points"] = lambda: ([a, a.copy(), a.copy(), b, b.copy()], "match")
    c["edge_planar"] = lambda: (near_points(W, [[0.25, 0.0, 0.0], [-0.25, 0.0, 0.0], [0.0, 0.25, 0.0], [0.0, -0.25, 0.0],
                                        [0.1875, 0.1875, 0.0]]), "none")
    c["edge_collinear_diag"] = lambda: (near_points(W, [[k * 0.09375, k * 0.0625, -k * 0.03125] for k in (-4, -2, 1, 3, 5)]),
                                "match")
    return c


def boundary_edge_case(T):
    """Slot 1: an edge query exactly on a cell corner T, its line along the slice boundaries through T
    and points exactly 1 m across the cell faces."""
    on = [(np.asarray(T, np.float64) + [a, 0.0, 0.0]).astype(F32) for a in (-0.75, -0.25, 0.25, 0.5, 0.875)]
    across = [(np.asarray(T, np.float64) + o).astype(F32) for o in ([0, 1, 0], [0, -1, 0], [0, 0, 1], [0, 0, -1])]
    return {"edge_corner_on_line": lambda: (on + across, "online")}


def origin_case():
    return {"surf_origin_nan": lambda: ([np.zeros(3, F32) for _ in range(5)], "nan")}


# ----------------------------------------------------------------------------------------------- build
def choose(scan, e, s):
    """Deterministic choice of the planted queries: [(slot, kind, feature index, label, W, points, expect)]
    and the three guesses."""
    rng = np.random.default_rng(20261018)
    taken = []

    def far(Wp):
        return np.linalg.norm(Wp) >= SEP and all(np.linalg.norm(Wp - w) >= SEP for w in taken)

    def pick(feats, exact_t=None):
        for i in rng.permutation(len(feats)):
            q = feats[i]
            if not 4.0 <= np.linalg.norm(q[:3]) <= 40.0:
                continue
            if exact_t is not None:
                Wq = world(q, exact_t)
                if not np.array_equal(Wq.astype(np.float64), np.asarray(q[:3], np.float64) + exact_t):
                    continue     # the LM's double point would not be the float W
            else:
                Wq = np.asarray(q[:3], np.float64)
            if far(Wq):
                taken.append(np.asarray(Wq, np.float64))
                return int(i)
        raise RuntimeError("no feature left for a planted case")

    out = []
    W0 = {}
    for label in surf_cases(np.zeros(3, F32) + F32(10.0)):
        i = pick(s, T0)
        W0[label] = world(s[i], T0)
        out.append((0, 2, i, label))
    for label in edge_cases(np.zeros(3, F32) + F32(10.0)):
        i = pick(e, T0)
        W0[label] = world(e[i], T0)
        out.append((0, 1, i, label))
    # slot 1: the edge feature nearest a cell corner (0.25 m slices in x, 1 m cells in y / z)
    used_e = {o[2] for o in out if o[1] == 1}
    best, bi = None, -1
    for i, q in enumerate(e):
        if i in used_e or not 4.0 <= np.linalg.norm(q[:3]) <= 40.0:
            continue
        T = np.array([np.round(q[0] * 4) / 4, np.round(q[1]), np.round(q[2])])
        if not far(T):
            continue
        dev = np.abs(T - q[:3]).max()
        if best is None or dev < best:
            best, bi = dev, i
    q = e[bi]
    Tc = np.array([np.round(q[0] * 4) / 4, np.round(q[1]), np.round(q[2])])
    t1 = Tc - np.asarray(q[:3], np.float64)
    assert np.array_equal(world(q, t1).astype(np.float64), Tc)
    taken.append(Tc)
    out.append((1, 1, bi, "edge_corner_on_line"))
    # slot 2: a surf feature translated next to the origin structure
    used_s = {o[2] for o in out if o[1] == 2}
    for i in rng.permutation(len(s)):
        if i not in used_s and 3.0 <= np.linalg.norm(s[i][:3]) <= 8.0:
            io = int(i)
            break
    t2 = ORIGIN_W - np.asarray(s[io][:3], np.float64)
    assert np.array_equal(world(s[io], t2).astype(np.float64), ORIGIN_W)
    out.append((2, 2, io, "surf_origin_nan"))
    return out, [T0, t1, t2]


def planted_sets(scan, e, s, chosen=None, ts=None):
    """[(slot, kind, feature index, label, W, points (n, 3) float32, expect)] for the chosen queries."""
    if chosen is None:
        chosen, ts = choose(scan, e, s)
    sets = []
    for slot, kind, i, label in chosen:
        q = (e if kind == 1 else s)[i]
        W = world(q, ts[slot])
        if label == "edge_corner_on_line":
            pts, exp = boundary_edge_case(W)[label]()
        elif label == "surf_origin_nan":
            pts, exp = origin_case()[label]()
        elif kind == 2:
            pts, exp = surf_cases(W)[label]()
        else:
            pts, exp = edge_cases(W)[label]()
        sets.append((slot, kind, i, label, W, np.stack(pts).astype(F32), exp))
    return sets, ts


def planted_maps(sets):
    """Planted edge / surf map rows (intensity 0) in case order, and each case's first map index."""
    out = {1: [], 2: []}
    first = []
    for slot, kind, i, label, W, pts, exp in sets:
        first.append(sum(len(p) for p in out[kind]))
        out[kind].append(pts)
    maps = {}
    for k in (1, 2):
        p = np.concatenate(out[k], 0) if out[k] else np.zeros((0, 3), F32)
        m = np.zeros((len(p), 4), F32)
        m[:, :3] = p
        maps[k] = m
    return maps, np.array(first)


def combined_map(planted, background, sets, kind):
    """Planted points first (their indices fixed), then the background with every point within CLEAR of a
    planted query or of the origin removed."""
    centres = [np.asarray(W, np.float64) for slot, k, i, label, W, pts, exp in sets] + [np.zeros(3)]
    bg = background
    keep = np.ones(len(bg), bool)
    p = bg[:, :3].astype(np.float64)
    for c in centres:
        keep &= ((p - c) ** 2).sum(1) > CLEAR * CLEAR
    return np.ascontiguousarray(np.concatenate([planted[kind], bg[keep]], 0))


def load():
    z = np.load(FIXTURE, allow_pickle=False)
    return {k: z[k] for k in z.files}


def sets_from_fixture(fx, e, s):
    chosen = [(int(a), int(b), int(c), str(d)) for a, b, c, d in zip(fx["slot"], fx["kind"], fx["feat"], fx["label"])]
    ts = [fx["t"][k] for k in range(3)]
    return planted_sets(None, e, s, chosen, ts)


def canon(rec):
    """Records with every NaN in v0 / v1 replaced by one bit pattern: the sign and payload of a NaN an
    operation produces are hardware-defined (x86's default NaN is negative, gfx950's positive), so a
    degenerate fit compares by NaN-ness there and bit for bit everywhere else."""
    r = rec.copy()
    for f in ("v0", "v1"):
        v = r[f]
        v[np.isnan(v)] = np.float64("nan")
        r[f] = v
    return r
