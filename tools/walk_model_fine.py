"""C2 walk on a finer y-z grid (CPU model): candidates and rows entered per query when the map's y-z cells are
1/sy m (sy = 1: the kernel's 1 m grid, 3 x 3 rows; sy = 2: 0.5 m, 5 x 5 rows), rows nearest first, a row skipped
when its yz-gap bound exceeds the current 6th key, x-windows trimmed to the 1 m radius (trim=0) or to the current
6th key (trim=1).  python tools/walk_model_fine.py"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "lmsf-slam_amd"))
from lmsf import synth  # noqa: E402

wl = synth.make_workload("C2", n_scans=1)
M = np.asarray(wl.surf_map)[:, :3].astype(np.float32)
scan = np.asarray(wl.scans[0])[:, :3]
Q = synth.transform_points(wl.truth[0], scan).astype(np.float32)
Q = Q[np.random.default_rng(0).choice(len(Q), 3000, replace=False)]


def model(sy, sx, trim):
    R = sy   # rings holding the 1 m radius
    ox = int(np.floor(M[:, 0] * sx).min()); oy = int(np.floor(M[:, 1] * sy).min()); oz = int(np.floor(M[:, 2] * sy).min())
    cx = np.floor(M[:, 0] * sx).astype(int) - ox; cy = np.floor(M[:, 1] * sy).astype(int) - oy
    cz = np.floor(M[:, 2] * sy).astype(int) - oz
    nx, ny, nz = cx.max() + 1, cy.max() + 1, cz.max() + 1
    lin = (cz * ny + cy) * nx + cx
    order = np.argsort(lin, kind="stable"); P = M[order]; L = lin[order]
    off = np.searchsorted(L, np.arange(nx * ny * nz + 1))
    h = 1.0 / sy
    ring = sorted([(dy, dz) for dy in range(-R, R + 1) for dz in range(-R, R + 1)], key=lambda t: (max(abs(t[0]), abs(t[1])), abs(t[0]) + abs(t[1])))
    cands, rows_in = [], []
    for w in Q:
        fx = np.floor(w[0]); fy = np.floor(w[1] * sy); fz = np.floor(w[2] * sy)
        cxs = int(fx * sx) - ox
        xa, xb = max(cxs - sx, 0), min(cxs + 2 * sx - 1, nx - 1)
        keys = []; d6 = 1.0; cand = 0; nrow = 0
        rr = []
        for dy, dz in ring:
            ylo, zlo = (fy + dy) * h, (fz + dz) * h
            gy = max(0., ylo - w[1], w[1] - (ylo + h)); gz = max(0., zlo - w[2], w[2] - (zlo + h))
            rr.append((gy * gy + gz * gz, dy, dz))
        for lb, dy, dz in rr:
            if lb > d6: continue
            ccy, ccz = int(fy) - oy + dy, int(fz) - oz + dz
            if not (0 <= ccy < ny and 0 <= ccz < nz): continue
            lim = min(1.0, d6) * (1 + 1e-5) if trim else 1.0 + 1e-5
            rem = lim - lb
            if rem < 0: continue
            rad = np.sqrt(rem)
            sa = max(xa, int(np.floor((w[0] - rad) * sx)) - ox); sb = min(xb, int(np.floor((w[0] + rad) * sx)) - ox)
            nrow += 1
            if sa > sb: continue
            base = (ccz * ny + ccy) * nx
            a, b = off[base + sa], off[base + sb + 1]
            cand += b - a
            if b > a:
                d = ((P[a:b] - w) ** 2).sum(1)
                keys = sorted(list(keys) + list(d[d < 1 + 1e-5]))[:6]
                if len(keys) == 6: d6 = keys[5]
        cands.append(cand); rows_in.append(nrow)
    return np.mean(cands), np.mean(rows_in)


for sy, sx in ((1, 4), (2, 4), (2, 8), (4, 8)):
    for trim in (0, 1):
        c, r = model(sy, sx, trim)
        print(f"sy={sy} sx={sx} trim={trim}: candidates {c:.1f}, rows entered {r:.1f}")
