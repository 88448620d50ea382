"""Generate tests/golden/c1_small.npz: a small C1-shaped workload with the oracle's outputs and
independent numpy cross-checks.  The reference holds no golden vectors for this path (its only
known-answer test is commented out and reads absent PCDs), so these fixtures pin the CPU
restatement against regressions; numpy (eigh, lstsq) pins it against independent algorithms.

Run: python tests/golden/make_golden.py   (deterministic; seeds from SURVEY.md §8(d))
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "lmsf-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))

from lmsf import synth  # noqa: E402
import oracle  # noqa: E402


def main():
    oracle.build()
    oracle.set_threads(1)
    wl = synth.make_workload("C1", n_scans=1, map_points=40_000, n_cols=900, road_length=10.0, radius=30.0)
    scan = wl.scans[0]
    e, s, ei, si = oracle.extract(scan)
    reg = oracle.Registration()
    reg.set_map(1, wl.edge_map)
    reg.set_map(2, wl.surf_map)
    reg.set_scan(1, e)
    reg.set_scan(2, s)
    rec, nn = reg.match(wl.guess[0])
    reg.set_fixed_schedule(True)
    reg.set_max_iterations(5)
    x, tr, st = reg.solve(wl.guess[0])
    # numpy pins: principal direction of every edge match, plane residual of every surf match
    dots, perr = [], []
    for i in np.nonzero(rec["kind"] == 1)[0]:
        P = wl.edge_map[nn[i], :3].astype(np.float64)
        c = P.mean(0)
        _, V = np.linalg.eigh((P - c).T @ (P - c))
        d = (rec["v0"][i] - rec["v1"][i]) / 0.2
        dots.append(abs(d @ V[:, 2]))
    for i in np.nonzero(rec["kind"] == 2)[0]:
        A = wl.surf_map[nn[i], :3].astype(np.float64)
        xx, *_ = np.linalg.lstsq(A, -np.ones(5), rcond=None)
        n = xx / np.linalg.norm(xx)
        perr.append(1.0 - abs(n @ rec["v0"][i]))
    np.savez_compressed(
        os.path.join(HERE, "c1_small.npz"),
        scan=scan, edge_map=wl.edge_map, surf_map=wl.surf_map, guess=wl.guess[0], truth=wl.truth[0],
        edge_src=ei, surf_src=si, nn=nn, kind=rec["kind"], v0=rec["v0"], v1=rec["v1"], trace=tr,
        np_edge_dir_dot=np.array(dots), np_plane_err=np.array(perr))
    print(f"edges {len(e)} surfs {len(s)} matches {(rec['kind'] > 0).sum()} trace {tr.shape}")


if __name__ == "__main__":
    main()
