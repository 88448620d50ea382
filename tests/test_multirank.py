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


def _worker_c45(rank, world, port, out_q, impl="torch"):
    """C5 pair partition + padded pose gather; C4 map broadcast + keyframe exchange -- through torch.distributed or
    the shipped C library's protocol (multi.CCollectives over gloo host collectives: bench.py --dist-impl c)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lmsf-slam_amd"))
    import torch
    import torch.distributed as dist
    from lmsf import multi
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    coll = multi.make_collectives(impl, world)
    # C5: 7 pairs, rank r owns i = r, r + 2, ...; pose of pair i = i
    mine = multi.pair_partition(7, rank, world)
    allp = coll.gather_pair_poses(np.stack([np.full(7, float(i)) for i in mine]), 7)
    # C4: rank 0's map replicated
    rng = np.random.default_rng(0)
    e0 = rng.random((11, 4)).astype(np.float32)
    s0 = rng.random((23, 4)).astype(np.float32)
    et, st = coll.broadcast_map(e0 if rank == 0 else None, s0 if rank == 0 else None)
    # C4 keyframe exchange over 3 steps: step 0 both keyframe, step 1 none, step 2 only rank 1
    cap = 8
    xchg = coll.keyframe_exchange(cap)
    log = []
    for step, kf in enumerate([(1, 1), (0, 0), (0, 2)]):
        typ = kf[rank]
        ne, ns = 2 + rank, 3 + step
        feat = torch.zeros((2 * cap, 4), dtype=torch.float32)
        feat[:ne] = 10 * rank + step
        feat[cap:cap + ns] = -(10 * rank + step)
        pose = np.eye(4)
        pose[0, 3] = 100 * rank + step
        got = xchg.exchange(pose, typ, ne if typ else 0, ns if typ else 0, feat)
        log.append([(q, fe.numpy().copy(), fs.numpy().copy(), P.copy()) for q, fe, fs, P in got])
    # a count above a rank's capacity is refused on every rank alike, before any feature gather
    payload = xchg.payload_bytes
    try:
        xchg.exchange(np.eye(4), 1, 1, cap + 3 if rank == 1 else 1, torch.zeros((2 * cap, 4), dtype=torch.float32))
        refused = False
    except ValueError:
        refused = True
    out_q.put((rank, allp, et.numpy(), st.numpy(), log, payload, refused, coll.impl, coll.max(float(rank + 3))))
    coll.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("impl", ["torch", "c"])
def test_gloo_world2_pairs_map_and_keyframe_exchange(impl):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_c45, args=(r, 2, port, q, impl)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(0)
    e0 = rng.random((11, 4)).astype(np.float32)
    s0 = rng.random((23, 4)).astype(np.float32)
    assert all(r[6] for r in res)                 # both ranks refused the over-capacity exchange
    assert all(r[7] == ("c-transport" if impl == "c" else "torch") and r[8] == 4.0 for r in res)
    for rank, allp, et, st, log, payload, *_ in res:
        # features gathered at the keyframing ranks' largest counts: step 0 (3 + 3 rows), step 2 (3 + 5 rows),
        # 2 ranks x 16 B per row -- not 2 x 2 cap rows per exchange
        assert payload == 2 * (3 + 3) * 16 + 2 * (3 + 5) * 16
        np.testing.assert_array_equal(allp, np.stack([np.full(7, float(i)) for i in range(7)]))
        assert et.tobytes() == e0.tobytes() and st.tobytes() == s0.tobytes()
        assert [q for q, *_ in log[0]] == [0, 1] and log[1] == [] and [q for q, *_ in log[2]] == [1]
        for step, entries in enumerate(log):
            for qr, fe, fs, P in entries:
                assert fe.shape == (2 + qr, 4) and fs.shape == (3 + step, 4)
                assert (fe == 10 * qr + step).all() and (fs == -(10 * qr + step)).all()
                assert P[0, 3] == 100 * qr + step
    # both replicas append the same keyframes in the same order
    for a, b in zip(res[0][4], res[1][4]):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            assert x[0] == y[0] and x[1].tobytes() == y[1].tobytes() and x[2].tobytes() == y[2].tobytes()


def _worker_cdist(rank, world, port, out_q):
    """The C library's protocol (liblmsf_dist.so) over gloo: pose gather, map broadcast, 3 keyframe-exchange
    steps, error agreement (one rank passes a bad buffer: every rank gets the error, none hangs)."""
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "lmsf-slam_amd"))
    import torch.distributed as dist
    from lmsf import multi
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = multi.CGroup()
    res = {}
    res["poses"] = g.allgather_poses(np.stack([np.full(7, 10.0 * rank + i) for i in range(3)]))
    rng = np.random.default_rng(5)
    cloud = rng.random((13, 4)).astype(np.float32)
    buf = np.zeros((16, 4), np.float32)
    if rank == 0:
        buf[:13] = cloud
    res["bcast"] = (g.broadcast_cloud(0, buf, 13 if rank == 0 else 0), buf.copy())
    small = np.zeros((8 if rank == 1 else 16, 4), np.float32)   # rank 1 cannot hold 13 rows
    res["bcast_small"] = g.broadcast_cloud(0, small, 13 if rank == 0 else 0)
    cap = 8
    gathered = np.zeros((world, 2 * cap, 4), np.float32)
    replica = []                                                # the keyframes this replica appends, in order
    steps = []
    for step, kf in enumerate([(1, 1), (0, 0), (0, 2)]):
        typ = kf[rank]
        ne, ns = 2 + rank, 3 + step
        feat = np.zeros((2 * cap, 4), np.float32)
        feat[:ne] = 10 * rank + step
        feat[cap:cap + ns] = -(10 * rank + step)
        pose = np.eye(4)
        pose[0, 3] = 100 * rank + step
        n_calls = len(g.gather_bytes)
        rc, info, anyk, rows = g.exchange_keyframes(pose, typ, ne if typ else 0, ns if typ else 0, feat, cap,
                                                    gathered)
        steps.append((rc, info.copy(), anyk, rows, g.gather_bytes[n_calls + 1:]))   # the calls after the info row
        if rc == 0 and anyk:
            flat = gathered.reshape(-1, 4)
            for q in range(world):
                if info[q, 16] != 0:
                    ne_q, ns_q = int(info[q, 17]), int(info[q, 18])
                    e0, s0 = q * rows[0], world * rows[0] + q * rows[1]
                    replica.append((q, flat[e0:e0 + ne_q].copy(), flat[s0:s0 + ns_q].copy(),
                                    info[q, :16].reshape(4, 4).copy()))
    res["steps"] = steps
    res["replica"] = replica
    # rank 1 passes no gathered buffer while rank 0 keyframes: both must return LMSF_ERR_ARG (-1)
    feat = np.zeros((2 * cap, 4), np.float32)
    rc, _, anyk, _ = g.exchange_keyframes(np.eye(4), 1 if rank == 0 else 0, 1, 1, feat, cap,
                                          gathered if rank == 0 else None)
    res["bad_args"] = (rc, anyk)
    # rank 0 keyframes 6 rows while rank 1's buffer holds 4 per kind: the max count exceeds a rank's capacity
    small_cap = 4 if rank == 1 else cap
    feat = np.zeros((2 * small_cap, 4), np.float32)
    rc, _, anyk, _ = g.exchange_keyframes(np.eye(4), 1 if rank == 0 else 0, 6 if rank == 0 else 0,
                                          1 if rank == 0 else 0, feat, small_cap, gathered)
    res["over_cap"] = (rc, anyk)
    res["max"] = g.max(1.5 + rank)
    g.close()
    out_q.put((rank, res))
    dist.destroy_process_group()


def test_gloo_world2_c_library_protocol():
    """Verdict r02 item 7: the C library's keyframe-exchange protocol (lmsf_group_exchange_keyframes and the
    info / padded-buffer layout of include/lmsf/lmsf_dist.h) rehearsed on 2 CPU ranks through its own code,
    over a caller-supplied transport: identical keyframe order on both replicas, and every rank takes the
    same error path."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_cdist, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cloud = np.random.default_rng(5).random((13, 4)).astype(np.float32)
    for rank in (0, 1):
        r = res[rank]
        rc, poses = r["poses"]
        assert rc == 0
        for q2 in (0, 1):
            np.testing.assert_array_equal(poses[q2], np.stack([np.full(7, 10.0 * q2 + i) for i in range(3)]))
        (rc, rows), buf = r["bcast"]
        assert rc == 0 and rows == 13 and buf[:13].tobytes() == cloud.tobytes()
        assert r["bcast_small"] == (-4, 13)                      # LMSF_ERR_CAPACITY on both ranks
        assert [s[0] for s in r["steps"]] == [0, 0, 0]
        assert [s[2] for s in r["steps"]] == [1, 0, 1]
        # payload at the keyframing ranks' largest counts, not 2 cap = 16 rows per rank:
        # step 0 both keyframe (n_edge 2 / 3, n_surf 3 / 3), step 2 only rank 1 (3 edges, 5 surfs)
        assert [s[3] for s in r["steps"]] == [(3, 3), (0, 0), (3, 5)]
        assert r["steps"][0][4] == [3 * 16, 3 * 16] and r["steps"][1][4] == [] and r["steps"][2][4] == [3 * 16, 5 * 16]
        assert r["bad_args"] == (-1, 0)
        assert r["over_cap"] == (-1, 0)
        assert r["max"] == (0, 2.5)
        assert [q2 for q2, *_ in r["replica"]] == [0, 1, 1]
    for (rc0, i0, *_), (rc1, i1, *_) in zip(res[0]["steps"], res[1]["steps"]):
        assert i0.tobytes() == i1.tobytes()                      # the same info table on every rank
    for a, b in zip(res[0]["replica"], res[1]["replica"]):
        assert a[0] == b[0] and all(x.tobytes() == y.tobytes() for x, y in zip(a[1:], b[1:]))
    q2, fe, fs, P = res[0]["replica"][2]                          # step 2: rank 1's keyframe
    assert fe.shape == (3, 4) and (fe == 12).all() and fs.shape == (5, 4) and (fs == -12).all() and P[0, 3] == 102
