"""World-size-2 gloo rehearsal of the multi-GPU path: scans sharded across
ranks with no data-path collective, then the all-gather of 6-DoF poses and the max-over-ranks
timing that bench.py runs over RCCL on GPUs."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lmsf-slam_amd"))
    import torch
    import torch.distributed as dist
    from lmsf import multi
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    n_total, per = 10, None
    lo, hi = multi.shard_range(n_total, rank, world)
    local = np.stack([np.full(7, 100.0 * i + k) for i, k in enumerate(range(lo, hi))]) if hi > lo else np.zeros((0, 7))
    per = 5
    buf = torch.zeros((world, per, 7), dtype=torch.float64)
    multi.gather_poses(local, buf)
    t = multi.max_over_ranks(float(rank + 1))
    out_q.put((rank, lo, hi, buf.numpy().copy(), t))
    dist.destroy_process_group()


def test_shard_range_balanced():
    from lmsf import multi
    for n in (0, 1, 7, 64, 1000):
        for w in (1, 2, 3, 8):
            parts = [multi.shard_range(n, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == n
            assert all(parts[i][1] == parts[i + 1][0] for i in range(w - 1))
            sizes = [b - a for a, b in parts]
            assert max(sizes) - min(sizes) <= 1


def test_gloo_world2_pose_allgather():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    for rank, lo, hi, buf, t in res:
        assert t == 2.0                                   # max over ranks
        for r2, lo2, hi2, _, _ in res:                    # every rank sees every rank's poses
            expect = np.stack([np.full(7, 100.0 * i + k) for i, k in enumerate(range(lo2, hi2))])
            np.testing.assert_array_equal(buf[r2], expect)
