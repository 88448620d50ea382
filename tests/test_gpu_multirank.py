"""The N-rank GPU data path pinned numerically on a one-GPU box.

`bench.py --gpus 2 --dist-backend gloo-gpu --config C4` runs the C4 configuration (BASELINE configs[3]) as two
ranks on the box's GPU: the launcher starts `torch.distributed.run` as a child process, rank 0 broadcasts the shared
prior map, and every step all-gathers (pose, update type, feature counts) and -- when a stream keyframes -- the
feature payloads, so both replicas append every stream's keyframes in rank order (lmsf/multi.py KeyframeExchange,
the protocol liblmsf_dist.so runs over RCCL on a multi-GPU node).  Each rank dumps its per-step poses and update
types (`--dump`); here two oracle trackers (oracle/tracker.py) consume the same two streams and the same keyframe
stream, and each rank's tracking must equal its oracle replica's: update decisions exactly, poses <= 1e-4 m / rad
(north_star) at every step.  RCCL itself only runs on the driver's 8-GPU node; gloo carries the collectives here.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
POSE_TOL = 1e-4


def test_c4_two_rank_rehearsal_matches_oracle_trackers(oracle_mod, tmp_path):
    import tracker as OT
    from conftest import mat_err
    sys.path.insert(0, REPO)
    import bench
    steps, warmup, map_points, cols = 3, 1, 500_000, 4096
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo-gpu", "--config",
           "C4", "--steps", str(steps), "--warmup", str(warmup), "--map-points", str(map_points), "--cols", str(cols),
           "--no-cpu", "--no-n27", "--workers", "1", "--dump", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1 and '"n_gpus": 2' in line[0] and "rehearsal" in line[0]
    dumps = [np.load(tmp_path / f"c4_rank{q}.npz") for q in range(2)]
    n = steps + warmup
    assert all(len(dm["poses"]) == n for dm in dumps)
    em, sm = bench.c4_map(map_points)
    streams = [bench.c4_stream(q, 2, n, cols) for q in range(2)]
    ots = []
    for q in range(2):
        ot = OT.Tracker(manual_map_update=True)
        T0 = np.eye(4)
        from lmsf import synth
        T0[:3, :3] = synth.quat_to_mat(streams[q][0][0][:4])
        T0[:3, 3] = streams[q][0][0][4:]
        ot.origin = T0.copy()
        ot.reg.set_fixed_schedule(True)
        ot.reg.set_max_iterations(5)
        ot.set_prior_map(1, em)
        ot.set_prior_map(2, sm)
        ots.append(ot)
    keyframes = 0
    for i in range(n):
        kfs = []
        for q in range(2):
            e, s, _, _ = oracle_mod.extract(streams[q][1][i])
            _, typ, _ = ots[q].solve(e, s, 0.1 * i)
            assert int(dumps[q]["types"][i]) == typ, (q, i)
            dt, dr = mat_err(dumps[q]["poses"][i], ots[q].curr)
            assert dt <= POSE_TOL and dr <= POSE_TOL, (q, i, dt, dr)
            if typ:
                kfs.append((e, s, ots[q].curr.copy()))
        for ot in ots:                            # every replica appends every stream's keyframes, in rank order
            for e, s, P in kfs:
                ot.add_keyframe(e, s, P)
            if kfs:
                ot.commit()
        keyframes += len(kfs)
    assert keyframes >= 2
