"""Query-memo outcome model (CPU only, oracle kd-tree + oracle Ceres-LM trace on one scan): per outer iteration
>= 2, how many queries the memo pass reuses (consecutive-gap test or re-keyed set in the same order), refits (same
set, new order) or sends to the bounded search -- and how many of those searches return the stored 5 in the stored
order (their fit would reproduce the stored record).  python tools/memo_model.py [C2|C5]
C5 (dense 10M-point map, VERDICT r04 #3b) also reports what a bounded re-key of the misses would read: the
candidates inside radius s5 + d (the stored 5th distance plus the query's displacement) against those inside pass
1's first-pass ball (sqrt(lim1), lim1 = 1 / rho from the map density, api.cpp knn_first_radius2)."""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "lmsf-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from lmsf import synth  # noqa: E402
import oracle  # noqa: E402

CFG = sys.argv[1] if len(sys.argv) > 1 else "C2"
wl = synth.make_workload(CFG, n_scans=1)
e, s, _, _ = oracle.extract(np.asarray(wl.scans[0]), **synth.CONFIGS[CFG].get("extract", {}))
reg = oracle.Registration()
reg.set_map(0, wl.edge_map) if False else None
EDGE, SURF = 1, 2
reg.set_map(EDGE, wl.edge_map)
reg.set_map(SURF, wl.surf_map)
reg.set_scan(EDGE, e)
reg.set_scan(SURF, s)
reg.set_fixed_schedule(True)
reg.set_max_iterations(5)
x, tr, st = reg.solve(wl.guess[0])
poses = [np.asarray(wl.guess[0])] + [tr[i] for i in range(len(tr) - 1)]
kd = oracle.KdMap(np.asarray(wl.surf_map))
# pass 1's first-pass radius^2 on this map: 1 / rho, rho = points per occupied 1/4 m x-slice of the 1 m grid
_c = np.floor(np.asarray(wl.surf_map)[:, :3] * np.array([4.0, 1.0, 1.0])).astype(np.int64)
_occ = len(np.unique(_c, axis=0))
LIM1 = min(1.0, max(0.01, _occ / len(_c))) if len(_c) / _occ >= 8 else 1.0
if CFG == "C5":
    from scipy.spatial import cKDTree
    CK = cKDTree(np.asarray(wl.surf_map)[:, :3].astype(np.float64))
print(f"{CFG}: {len(_c)} surf map points, {len(s)} surf queries, first-pass radius^2 {LIM1:.4f}")
S = np.asarray(s)[:, :3].astype(np.float64)


def associate(p, pose):
    return synth.transform_points(pose, p).astype(np.float32)


def knn6(w):
    idx, d2 = kd.knn(w, 6)
    return idx, d2.astype(np.float64)


state = None
for it, pose in enumerate(poses):
    w = associate(S, pose)
    idx, d2 = knn6(w)
    s_all = np.sqrt(np.minimum(d2, 1.0))
    if it < 2:
        state = dict(w0=w.astype(np.float64), nbr=idx[:, :5].copy(), s6=s_all[:, 5], gap=s_all[:, 5] - s_all[:, 4],
                     gord=np.minimum(np.min(np.diff(s_all[:, :5], axis=1), axis=1), s_all[:, 5] - s_all[:, 4]))
        print(f"iteration {it}: full search")
        continue
    dd = np.linalg.norm(w.astype(np.float64) - state["w0"], axis=1)
    same_gap = 2 * dd + 1e-5 < state["gord"]
    # re-key the stored 5 at w (float d2 as the kernel computes it)
    P = np.asarray(wl.surf_map)[:, :3].astype(np.float32)
    nb = state["nbr"]
    dv = (w[:, None, :] - P[nb]).astype(np.float32)
    rk = (dv[..., 0] * dv[..., 0] + dv[..., 1] * dv[..., 1] + dv[..., 2] * dv[..., 2]).astype(np.float32)
    order = np.lexsort((nb, rk), axis=1) if False else np.array([np.lexsort((nb[i], rk[i])) for i in range(len(nb))])
    k4 = np.sqrt(rk[np.arange(len(nb)), order[:, 4]].astype(np.float64))
    inside = k4 + dd + 1e-5 < state["s6"]
    in_order = (order == np.arange(5)).all(axis=1)
    reuse = same_gap | (inside & in_order)
    refit = ~same_gap & inside & ~in_order
    search = ~reuse & ~refit
    unchanged = search & (idx[:, :5] == nb).all(axis=1)
    n = len(w)
    print(f"iteration {it}: reuse {reuse.mean():.3f} (gap test {same_gap.mean():.3f}), refit {refit.mean():.3f}, "
          f"search {search.mean():.3f}, of which same 5 in the stored order {unchanged.sum() / max(search.sum(), 1):.3f}")
    if CFG == "C5":   # dense map: candidates a bounded re-key of the misses would read vs pass 1's ball
        s5 = np.sqrt(rk[np.arange(len(nb)), order[:, 4]].astype(np.float64))
        r_memo = np.minimum(s5 + dd + 1e-5, 1.0)
        sub = np.flatnonzero(search)[:4000]
        c_memo = CK.query_ball_point(w[sub].astype(np.float64), r_memo[sub], return_length=True)
        c_ball = CK.query_ball_point(w[sub].astype(np.float64), np.full(len(sub), np.sqrt(LIM1)), return_length=True)
        print(f"  misses ({search.mean():.3f} of the queries): mean candidates within s5 + d {c_memo.mean():.1f} "
              f"vs pass 1's first-pass ball {c_ball.mean():.1f} (sample of {len(sub)}); every query's memo test "
              f"re-keys 5 stored points")
    # the kernel's state updates: refits reorder the stored set (anchor kept), searches re-anchor
    state["nbr"][refit] = nb[refit][np.arange(refit.sum())[:, None], order[refit]]
    state["gord"][refit] = -1.0
    for key, val in (("w0", w.astype(np.float64)), ("s6", s_all[:, 5]), ("gap", s_all[:, 5] - s_all[:, 4])):
        state[key][search] = val[search]
    state["nbr"][search] = idx[search, :5]
    state["gord"][search] = np.minimum(np.min(np.diff(s_all[search, :5], axis=1), axis=1), s_all[search, 5] - s_all[search, 4])

# Full searches: how many queries' ordered 5-NN equal those of the previous outer iteration's match (a full search
# whose fit could be skipped when the record is kept by position)
prev = None
for it, pose in enumerate(poses[:5]):
    w = associate(S, pose)
    idx, d2 = knn6(w)
    ok = d2[:, 4] < 1.0
    if prev is not None:
        same = (idx[:, :5] == prev).all(axis=1) & ok
        print(f"iteration {it}: ordered 5-NN unchanged from iteration {it - 1}: {same.mean():.3f} (matched {ok.mean():.3f})")
    prev = idx[:, :5]
