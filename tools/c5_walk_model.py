"""C5 pruned-walk work model (CPU only): per-query candidate counts of match_fit_kernel<PRUNE>'s two-pass walk
on the 10M-point map, and what they imply for a 64-lane wave -- the divergence VERDICT r03 named (lane utilisation
0.525).  Prints, over contiguous waves of the search order (edges then surfs, emission order):
  lane-loop utilisation of the per-row loops (sum over rows of mean(len) / sum over rows of max(len)),
  of a flattened walk (mean(total) / max(total)), and after sorting each 256-query block by a work estimate.
python tools/c5_walk_model.py [n_waves]"""
import os
import sys

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "lmsf-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from lmsf import synth  # noqa: E402
import oracle  # noqa: E402

RU = 4
N_WAVES = int(sys.argv[1]) if len(sys.argv) > 1 else 24


class Grid:
    def __init__(self, M):
        M = M[:, :3].astype(np.float32)
        n = len(M)
        cx = np.floor(M[:, 0]).astype(np.int64)
        # slices per metre: as k_map.hip (sx from density; 4 for these maps)
        self.sx = 4
        sx = self.sx
        self.ox = int(np.floor(M[:, 0] * sx).min())
        self.oy, self.oz = int(np.floor(M[:, 1]).min()), int(np.floor(M[:, 2]).min())
        cxs = np.floor(M[:, 0] * sx).astype(np.int64) - self.ox
        cy = np.floor(M[:, 1]).astype(np.int64) - self.oy
        cz = np.floor(M[:, 2]).astype(np.int64) - self.oz
        self.nx, self.ny, self.nz = int(cxs.max()) + 1, int(cy.max()) + 1, int(cz.max()) + 1
        lin = (cz * self.ny + cy) * self.nx + cxs
        order = np.argsort(lin, kind="stable")
        self.P = M[order]
        L = lin[order]
        self.off = np.searchsorted(L, np.arange(self.nx * self.ny * self.nz + 1))
        occ = len(np.unique(L))
        rho = n / occ
        self.lim1 = 1.0 if rho < 8 else min(1.0, max(0.01, 1.0 / rho))
        del cx


def walk(g, w):
    """(pass-1 row lengths, pass-2 row lengths) of the pruned walk (k_match.hip knn_walk PRUNE, NK = 5)."""
    fx, fy, fz = np.floor(w)
    near = [4, 1, 3, 5, 7, 0, 2, 6, 8]
    geo = []
    for rr in near:
        dyo, dzo = rr % 3 - 1, rr // 3 - 1
        cxs = int(np.floor(fx * g.sx)) - g.ox
        cy, cz = int(fy) - g.oy + dyo, int(fz) - g.oz + dzo
        xa, xb = max(cxs - g.sx, 0), min(cxs + 2 * g.sx - 1, g.nx - 1)
        if not (0 <= cy < g.ny and 0 <= cz < g.nz) or xa > xb:
            geo.append(None)
            continue
        ylo, zlo = fy + dyo, fz + dzo
        gy = max(0., ylo - w[1], w[1] - (ylo + 1))
        gz = max(0., zlo - w[2], w[2] - (zlo + 1))
        geo.append(((cz * g.ny + cy) * g.nx, xa, xb, gy * gy + gz * gz))

    def window(lim, lb, xa, xb):
        rem = lim - lb
        if rem < 0:
            return 1, 0
        r = np.sqrt(rem)
        return max(xa, int(np.floor((w[0] - r) * g.sx)) - g.ox), min(xb, int(np.floor((w[0] + r) * g.sx)) - g.ox)

    keys = []
    d4 = 1.0

    def scan(a, b):
        nonlocal keys, d4
        if b > a:
            d = ((g.P[a:b] - w) ** 2).sum(1)
            keys = sorted(keys + list(d[d < 1.0]))[:5]
            if len(keys) == 5:
                d4 = keys[4]
        return b - a

    lim1 = g.lim1 * (1 + 1e-5)
    p1, p2, scanned = [], [], set()
    for i, r in enumerate(geo):
        if r is None:
            p1.append(0)
            continue
        base, xa, xb, lb = r
        if lb > d4 or lb > lim1:
            p1.append(0)
            continue
        sa, sb = window(lim1, lb, xa, xb)
        scanned.add(i)
        p1.append(scan(g.off[base + sa], g.off[base + sb + 1]) if sa <= sb else 0)
    for i, r in enumerate(geo):
        if r is None or r[3] > d4:
            p2.append(0)
            continue
        base, xa, xb, lb = r
        sa, sb = window(d4 * (1 + 1e-5), lb, xa, xb)
        ta, tb = window(lim1, lb, xa, xb) if i in scanned else (1, 0)
        n = 0
        if ta > tb:
            if sa <= sb:
                n += scan(g.off[base + sa], g.off[base + sb + 1])
        else:
            l1, r0 = min(sb, ta - 1), max(sa, tb + 1)
            if sa <= l1:
                n += scan(g.off[base + sa], g.off[base + l1 + 1])
            if r0 <= sb:
                n += scan(g.off[base + r0], g.off[base + sb + 1])
        p2.append(n)
    return p1, p2


def steps(n):
    return n // RU + n % RU   # RU-wide steps + one-at-a-time tail (the kernel's loop shape)


def main():
    wl = synth.make_workload("C5", n_scans=1)
    c = synth.CONFIGS["C5"]
    e, s, _, _ = oracle.extract(wl.scans[0], **c["extract"])
    ge, gs = Grid(np.asarray(wl.edge_map)), Grid(np.asarray(wl.surf_map))
    print(f"edge map {len(wl.edge_map)} lim1 {ge.lim1:.4f}; surf map {len(wl.surf_map)} lim1 {gs.lim1:.4f}; "
          f"queries {len(e)} edge + {len(s)} surf")
    Q = np.concatenate([e, s])
    Qw = synth.transform_points(wl.guess[0], Q)[:, :3]
    rng = np.random.default_rng(1)
    starts = np.sort(rng.choice((len(Q) - 64) // 64, N_WAVES, replace=False)) * 64
    util_rows, util_pass, util_flat, tot, p2frac, insph = [], [], [], [], [], []
    for st in starts:
        rows1, rows2, totals = [], [], []
        for q in range(st, st + 64):
            g = ge if q < len(e) else gs
            p1, p2 = walk(g, Qw[q])
            rows1.append(p1)
            rows2.append(p2)
            totals.append(sum(p1) + sum(p2))
            d = ((g.P - Qw[q]) ** 2).sum(1) if q % 16 == 0 else None
            if d is not None:
                d5 = np.sort(d)[4]
                insph.append((int((d < g.lim1).sum()), int((d <= d5).sum()), sum(p1) + sum(p2)))
        R = np.concatenate([np.array(rows1), np.array(rows2)], 1)
        S = np.vectorize(steps)(R)
        util_rows.append(S.mean(0).sum() / max(S.max(0).sum(), 1))
        C = np.vectorize(lambda n: -(-n // RU))(R)   # masked RU steps per row
        s1, s2 = C[:, :9].sum(1), C[:, 9:].sum(1)
        util_pass.append((s1.mean() + s2.mean()) / max(s1.max() + s2.max(), 1))
        F = C.sum(1)
        util_flat.append(F.mean() / max(F.max(), 1))
        p2frac.append((np.array(rows2).sum(1) > 0).mean())
        tot.append(np.array(totals))
    tot = np.concatenate(tot)
    print(f"candidates per query: mean {tot.mean():.1f} median {np.median(tot):.0f} p90 {np.percentile(tot, 90):.0f} "
          f"max {tot.max()}; queries with a pass-2 scan {np.mean(p2frac):.3f}")
    ins = np.array(insph)
    print(f"map points inside the pass-1 sphere: mean {ins[:, 0].mean():.1f}; scanned {ins[:, 2].mean():.1f}")
    print(f"lane-loop utilisation, per-row loops (the kernel): {np.mean(util_rows):.3f}")
    print(f"lane-loop utilisation, flattened per pass:        {np.mean(util_pass):.3f}")
    print(f"lane-loop utilisation, flattened walk:           {np.mean(util_flat):.3f}")
    srt = np.sort(tot.reshape(-1, 64), axis=1)
    print(f"flattened walk, wave-sorted by work (bound):     {np.mean(srt.mean(1) / np.maximum(srt.max(1), 1)):.3f}")


if __name__ == "__main__":
    main()


def fine_model(h=0.25, sxf=8, n_waves=16, lim_scale=1.0):
    """Candidates of a first pass on a fine grid (yz cells of h m, x slices of 1/sxf m; 3 x 3 rows, x-window of
    radius sqrt(lim1 - lb)), the queries it resolves (5th key <= lim1), and its flattened lane-loop utilisation."""
    wl = synth.make_workload("C5", n_scans=1)
    c = synth.CONFIGS["C5"]
    e, s, _, _ = oracle.extract(wl.scans[0], **c["extract"])
    out = []
    for M, Q in ((np.asarray(wl.surf_map), s),):
        M = M[:, :3].astype(np.float32)
        g = Grid(M)
        lim1 = g.lim1 * lim_scale
        ox = int(np.floor(M[:, 0] * sxf).min())
        oy, oz = int(np.floor(M[:, 1] / h).min()), int(np.floor(M[:, 2] / h).min())
        cxs = np.floor(M[:, 0] * sxf).astype(np.int64) - ox
        cy = np.floor(M[:, 1] / h).astype(np.int64) - oy
        cz = np.floor(M[:, 2] / h).astype(np.int64) - oz
        nx, ny, nz = int(cxs.max()) + 1, int(cy.max()) + 1, int(cz.max()) + 1
        print(f"fine grid {nx} x {ny} x {nz} = {nx * ny * nz / 1e6:.0f}M cells")
        lin = (cz * ny + cy) * nx + cxs
        order = np.argsort(lin, kind="stable")
        P = M[order]
        L = lin[order]
        Qw = synth.transform_points(wl.guess[0], Q)[:, :3]
        rng = np.random.default_rng(1)
        starts = np.sort(rng.choice((len(Qw) - 64) // 64, n_waves, replace=False)) * 64
        cands, unres, util = [], [], []
        for st in starts:
            steps_l = []
            for w in Qw[st:st + 64]:
                fy, fz = np.floor(w[1] / h), np.floor(w[2] / h)
                keys, n, nst = [], 0, 0
                for dz in (-1, 0, 1):
                    for dy in (-1, 0, 1):
                        ylo, zlo = (fy + dy) * h, (fz + dz) * h
                        gy = max(0., ylo - w[1], w[1] - (ylo + h))
                        gz = max(0., zlo - w[2], w[2] - (zlo + h))
                        lb = gy * gy + gz * gz
                        rem = lim1 * (1 + 1e-5) - lb
                        if rem < 0:
                            continue
                        r = np.sqrt(rem)
                        sa, sb = int(np.floor((w[0] - r) * sxf)) - ox, int(np.floor((w[0] + r) * sxf)) - ox
                        base = ((int(fz + dz) - oz) * ny + (int(fy + dy) - oy)) * nx
                        a0 = np.searchsorted(L, base + sa)
                        b0 = np.searchsorted(L, base + sb + 1)
                        if b0 > a0:
                            d = ((P[a0:b0] - w) ** 2).sum(1)
                            keys += list(d)
                            n += b0 - a0
                            nst += -(-(b0 - a0) // RU)
                keys.sort()
                cands.append(n)
                unres.append(len(keys) < 5 or keys[4] > lim1)
                steps_l.append(nst)
            S = np.array(steps_l)
            util.append(S.mean() / max(S.max(), 1))
        print(f"h {h} sxf {sxf} lim1 {lim1:.4f}: candidates mean {np.mean(cands):.1f} p90 {np.percentile(cands, 90):.0f}, "
              f"unresolved {np.mean(unres):.3f}, flattened util {np.mean(util):.3f}")


def sorted_model(n_blocks=6):
    """Flattened per-pass walk on the current grid with each 256-query block's queries re-dealt to its 4 waves
    in order of their pass-1 step count (known after the row resolve): lane-loop utilisation."""
    wl = synth.make_workload("C5", n_scans=1)
    c = synth.CONFIGS["C5"]
    e, s, _, _ = oracle.extract(wl.scans[0], **c["extract"])
    gs = Grid(np.asarray(wl.surf_map))
    Qw = synth.transform_points(wl.guess[0], s)[:, :3]
    rng = np.random.default_rng(2)
    starts = np.sort(rng.choice((len(Qw) - 256) // 256, n_blocks, replace=False)) * 256
    u_plain, u_sorted, u_sorted_tot = [], [], []
    for st in starts:
        C = []
        for w in Qw[st:st + 256]:
            p1, p2 = walk(gs, w)
            C.append([-(-n // RU) for n in p1 + p2])
        C = np.array(C)
        s1, s2 = C[:, :9].sum(1), C[:, 9:].sum(1)

        def util(idx):
            tot_mean = tot_max = 0.0
            for wv in range(4):
                ii = idx[wv * 64:(wv + 1) * 64]
                tot_mean += s1[ii].mean() + s2[ii].mean()
                tot_max += s1[ii].max() + s2[ii].max()
            return tot_mean / tot_max
        u_plain.append(util(np.arange(256)))
        u_sorted.append(util(np.argsort(s1, kind="stable")))
        u_sorted_tot.append(util(np.argsort(s1 + s2, kind="stable")))
    print(f"flattened per pass: block order {np.mean(u_plain):.3f}, sorted by pass-1 steps {np.mean(u_sorted):.3f}, "
          f"sorted by all steps (bound) {np.mean(u_sorted_tot):.3f}")
