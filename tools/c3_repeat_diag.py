"""Repeat the C3 dual-LiDAR parity sequence (tests/test_gpu_parity.py::test_dual_lidar_refine_parity[4096]) N times
per option set on the GPU, against one oracle run, and report each repetition's first deviating frame and largest
pose difference -- a diagnostic for a deviation seen once in the GPU suite.  python tools/c3_repeat_diag.py [N]"""
import os
import sys
import time

import numpy as np

REPO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, os.path.join(REPO, "lmsf-slam_amd"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import torch  # noqa: E402,F401  (the HIP runtime first)
from lmsf import _lib as lib, dual, synth  # noqa: E402
import oracle as oracle_mod  # noqa: E402
import tracker as OT  # noqa: E402
from conftest import mat_err, pose_matrix  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ds = synth.make_dual_sequence(6, n_cols=4096, step=0.5)
X = pose_matrix(ds.extrinsic)
X0 = X @ pose_matrix(np.concatenate([synth.axis_angle_quat(np.radians([0.5, -0.5, 0.5])), [0.03, -0.02, 0.02]]))
ot = OT.Tracker()
ext = X0.copy()
ref = []
for i in range(len(ds.truth)):
    ep, sp, _, _ = oracle_mod.extract(ds.primary[i])
    es, ss, _, _ = oracle_mod.extract(ds.sub[i])
    _, typ, _ = ot.solve(ep, sp, 0.1 * i)
    prim_o = ot.curr.copy()
    sub_o, _ = ot._register({1: es, 2: ss}, dual.iso_mul(prim_o, ext))
    ext = dual.iso_mul(dual.iso_inv(prim_o), sub_o)
    ref.append((typ, prim_o, sub_o, ext.copy()))
print("oracle done", flush=True)

for name, loop, prefetch in (("default", 1, True), ("lm_loop_off", 0, True), ("no_prefetch", 1, False)):
    for rep in range(N):
        ctx = lib.Context(max_batch=4, max_scan_points=70000, max_features=70000)
        ctx.set_option(lib.OPT_LM_LOOP, loop)
        sysg = dual.DualLidarSystem(ctx, extrinsic=X0)
        worst, first = 0.0, -1
        for i in range(len(ds.truth)):
            nxt = (ds.primary[i + 1], ds.sub[i + 1]) if prefetch and i + 1 < len(ds.truth) else None
            prim_g, sub_g = sysg.process(ds.primary[i], ds.sub[i], 0.1 * i, next_frame=nxt)
            typ, prim_o, sub_o, ext_o = ref[i]
            d = max(max(mat_err(a, b)) for a, b in ((prim_g, prim_o), (sub_g, sub_o), (sysg.extrinsic, ext_o)))
            if sysg.last["primary_update"] != typ:
                d = max(d, 1.0)
            if d > 1e-4 and first < 0:
                first = i
            worst = max(worst, d)
        ks = ctx.kernel_stats()
        print(f"{name} rep {rep}: worst {worst:.3g} first_bad_frame {first} loop_recoveries {ks.loop_recoveries}",
              flush=True)
        sysg.close()
        ctx.close()
