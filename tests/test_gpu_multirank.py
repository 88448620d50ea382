"""The N-rank GPU data path pinned numerically on a one-GPU box (C2 added in r05).

`bench.py --gpus 2 --dist-backend gloo-gpu --config C4` runs the C4 configuration (BASELINE configs[3]) as two
ranks on the box's GPU: the launcher starts `torch.distributed.run` as a child process, rank 0 broadcasts the shared
prior map, and every step all-gathers (pose, update type, feature counts) and -- when a stream keyframes -- the
feature payloads, so both replicas append every stream's keyframes in rank order.  Since r06 the exchanges run in
the shipped C library (liblmsf_dist.so, lmsf_group_exchange_keyframes / _broadcast_cloud / _allgather_poses / _max:
bench.py --dist-impl c, the default) -- over RCCL on a multi-GPU node, over its host transport on gloo here.  Each rank dumps its per-step poses and update
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
    assert '"dist_impl": "c-transport"' in line[0]      # the shipped C library's exchanges
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


def test_c2_two_rank_rehearsal_matches_oracle(oracle_mod, tmp_path):
    """The default configuration's N-rank path (scan-sharded C2, poses all-gathered after every step) as two gloo-gpu
    ranks on the box's GPU: each rank's own poses reach both ranks unchanged (the all-gather), and the first units of
    each rank -- its own scans (rank-dependent seeds) at its own guesses -- match the oracle's registration."""
    from conftest import pose_err
    sys.path.insert(0, REPO)
    import bench
    from lmsf import synth
    map_points, cols, batch, unique = 200_000, 1024, 8, 4
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--dist-backend", "gloo-gpu", "--config",
           "C2", "--steps", "2", "--warmup", "1", "--batch", str(batch), "--unique-scans", str(unique), "--streams", "1",
           "--map-points", str(map_points), "--cols", str(cols), "--no-cpu", "--no-n27", "--h2d", "off", "--workers",
           "1", "--dump", str(tmp_path)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1 and '"n_gpus": 2' in line[0] and "rehearsal" in line[0]
    assert '"dist_impl": "c-transport"' in line[0]      # the shipped C library's exchanges
    dumps = [np.load(tmp_path / f"c2_rank{q}.npz") for q in range(2)]
    for q in range(2):
        assert dumps[q]["gathered"].shape == (2, batch, 7)
        for o in range(2):
            assert np.array_equal(dumps[o]["gathered"][q], dumps[q]["poses"]), (q, o)
    c = synth.CONFIGS["C2"]
    k = c["k"]
    scene = synth.make_scene(1000 + k, road_length=80.0)
    em, sm = synth.make_map(scene, map_points, 1000 + k + 7, center_x=(0.0, 80.0), radius=c["radius"])
    for q in range(2):
        dm = dumps[q]
        for i in range(2):   # units 0 and 1: scans 0 and 1 of rank q
            u = int(dm["unit_scan"][i])
            scan = bench.make_scans([(1000 + k, dm["truth_u"][u], int(dm["seeds"][u]), cols, c["elev"])], 1)[0]
            e, s, _, _ = oracle_mod.extract(scan, **c["extract"])
            reg = oracle_mod.Registration()
            reg.set_map(1, em)
            reg.set_map(2, sm)
            reg.set_scan(1, e)
            reg.set_scan(2, s)
            reg.set_fixed_schedule(True)
            reg.set_max_iterations(5)
            ox, _, _ = reg.solve(dm["guesses"][i])
            dt, dr = pose_err(dm["poses"][i], ox)
            assert dt <= POSE_TOL and dr <= POSE_TOL, (q, i, dt, dr)


_RCCL_ONE_RANK = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "lmsf-slam_amd"))
import torch
import torch.distributed as dist
from lmsf import multi
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=sys.argv[2])
torch.cuda.set_device(0)
dev = torch.device("cuda", 0)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=dev)
coll = multi.CCollectives(1, dev, 0, rccl=True)
poses = np.arange(35, dtype=np.float64).reshape(5, 7)
g = coll.gather_poses(poses, torch.zeros((1, 5, 7), dtype=torch.float64, device=dev))
assert np.array_equal(g.cpu().numpy()[0], poses)
assert coll.max(3.5) == 3.5
rng = np.random.default_rng(1)
e0, s0 = rng.random((11, 4)).astype(np.float32), rng.random((23, 4)).astype(np.float32)
e, s = coll.broadcast_map(e0, s0)
assert e.device.type == "cuda" and e.cpu().numpy().tobytes() == e0.tobytes() and s.cpu().numpy().tobytes() == s0.tobytes()
assert coll.impl == "c-rccl"
coll.close()
dist.destroy_process_group()
print("rccl group ok")
"""


def test_rccl_group_in_python_one_rank():
    """bench.py's --dist-impl c on the nccl backend: multi.CCollectives creates liblmsf_dist.so's own RCCL
    communicator (rank 0's unique id broadcast over torch.distributed, lmsf_group_create on the rank's GPU) beside
    torch's, with torch's librccl serving both (one RCCL and one HIP runtime in the process), and runs the pose
    all-gather, the max and the device-memory map broadcast through it (one rank: the box has one GPU)."""
    import socket
    sk = socket.socket()
    sk.bind(("127.0.0.1", 0))
    port = sk.getsockname()[1]
    sk.close()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run([sys.executable, "-c", _RCCL_ONE_RANK, REPO, str(port)], capture_output=True, text=True,
                       timeout=180, env=env)
    assert r.returncode == 0 and "rccl group ok" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
