"""Multi-GPU plumbing: one process per GPU over RCCL (torch.distributed "nccl").
C2 batch path: scans sharded across ranks with no data-path collective, then one all-gather of the
6-DoF poses (7 doubles per scan).  C5: pairs partitioned i mod N, one padded pose all-gather.
C4: shared map broadcast once from rank 0; per tracking step a pose/keyframe-flag all-gather and,
when a stream keyframes, an all-gather of the features at the keyframing streams' largest counts
(KeyframeExchange).

The same functions run on CPU tensors with the gloo backend (tests/test_multirank.py).
"""
from __future__ import annotations

import numpy as np


def shard_range(n_total: int, rank: int, world: int):
    """Contiguous, balanced slice [lo, hi) of n_total items owned by `rank`."""
    base, rem = divmod(n_total, world)
    lo = rank * base + min(rank, rem)
    hi = lo + base + (1 if rank < rem else 0)
    return lo, hi


def gather_poses(local_poses: np.ndarray, out_tensor, device=None):
    """All-gather (B, 7) float64 poses from every rank into out_tensor (world, B, 7)."""
    import torch
    import torch.distributed as dist
    t = torch.from_numpy(np.ascontiguousarray(local_poses, dtype=np.float64))
    if device is not None:
        t = t.to(device, non_blocking=True)
    dist.all_gather_into_tensor(out_tensor, t.unsqueeze(0))
    return out_tensor


def max_over_ranks(value: float, device=None) -> float:
    import torch
    import torch.distributed as dist
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---- C5: loop-closure re-registration, pairs partitioned i mod N, one padded pose all-gather
def pair_partition(n_pairs: int, rank: int, world: int):
    """Global pair indices owned by `rank` (i mod world), SURVEY 8(e) C5."""
    return list(range(rank, n_pairs, world))


def gather_pair_poses(local_poses: np.ndarray, n_pairs: int, world: int, device=None) -> np.ndarray:
    """All-gather every rank's (len(pair_partition), 7) poses; returns (n_pairs, 7) in global pair order."""
    import torch
    per = -(-n_pairs // world)
    buf = np.zeros((per, 7))
    buf[:len(local_poses)] = local_poses
    out = torch.zeros((world, per, 7), dtype=torch.float64, device=device)
    gather_poses(buf, out, device)
    allp = out.cpu().numpy()
    res = np.zeros((n_pairs, 7))
    for r in range(world):
        idx = pair_partition(n_pairs, r, world)
        res[idx] = allp[r, :len(idx)]
    return res


# ---- C4: shared map replicated from rank 0, keyframe features exchanged between streams
def broadcast_map(edge, surf, device=None):
    """Rank 0's (n, 4) float32 edge / surf maps replicated on every rank (one broadcast each)."""
    import torch
    import torch.distributed as dist
    rank = dist.get_rank()
    if rank == 0:
        n = torch.tensor([len(edge), len(surf)], dtype=torch.int64, device=device)
    else:
        n = torch.zeros(2, dtype=torch.int64, device=device)
    dist.broadcast(n, 0)
    out = []
    for k, src in enumerate((edge, surf)):
        if rank == 0:
            t = torch.as_tensor(np.ascontiguousarray(src, dtype=np.float32)).to(device)
        else:
            t = torch.empty((int(n[k]), 4), dtype=torch.float32, device=device)
        dist.broadcast(t, 0)
        out.append(t)
    return out[0], out[1]


class KeyframeExchange:
    """Per tracking step: all-gather (pose 4x4, update type, edge count, surf count) of every
    stream, and -- only when some stream keyframed -- the feature buffers at the keyframing streams'
    largest counts (max n_edge rows of edges, then max n_surf rows of surfs per rank, not the padded
    capacity), so that every replica appends the same keyframes in rank order (SURVEY 8(e) C4:
    `ncclAllGather` of the pose every step, of the transformed-feature payload when a stream emits a
    keyframe).

    feat: (2 * cap, 4) float32 tensor on `device` holding this rank's [edges | surfs] (edges at 0,
    surfs at cap).  Returns [(rank, edge_view, surf_view, pose4x4)] for the keyframed streams (a replica adds
    its own entry from its context, lmsf_tracker_add_keyframe_extracted; with one stream the views are None
    and feat is not read).  payload_bytes / steps count what went over the wire."""

    def __init__(self, cap: int, world: int, device=None):
        import torch
        self.cap, self.world, self.device = cap, world, device
        self.info = torch.zeros((world, 20), dtype=torch.float64, device=device)
        self.own = torch.zeros(20, dtype=torch.float64, device=device)
        self.gbuf = torch.zeros(world * 2 * cap * 4, dtype=torch.float32, device=device)
        self.payload_bytes = 0      # feature bytes this rank received, summed over steps
        self.steps = 0

    def exchange(self, pose, update_type, n_edge, n_surf, feat):
        import torch.distributed as dist
        import torch
        vec = np.concatenate([np.asarray(pose, dtype=np.float64).ravel(), [update_type, n_edge, n_surf, self.cap]])
        self.steps += 1
        if self.world <= 1:   # one stream: nothing to exchange; the caller adds its own keyframe from its context
            return [(0, None, None, np.asarray(pose, dtype=np.float64).reshape(4, 4))] if update_type else []
        self.own.copy_(torch.from_numpy(vec))
        dist.all_gather_into_tensor(self.info, self.own.unsqueeze(0))
        allinfo = self.info.cpu().numpy()
        kf = allinfo[:, 16] > 0
        if not kf.any():
            return []
        me, ms = int(allinfo[kf, 17].max()), int(allinfo[kf, 18].max())
        # every rank sends me / ms rows of its own buffer: they must fit the smallest one, counts non-negative -- the
        # C library's all-rank check (lmsf_group_exchange_keyframes), raised alike on every rank from the same info
        if me > allinfo[:, 19].min() or ms > allinfo[:, 19].min() or (allinfo[kf, 17:19] < 0).any():
            raise ValueError(f"keyframe exchange: counts ({me}, {ms}) exceed the smallest rank capacity "
                             f"{int(allinfo[:, 19].min())} or are negative")
        W, cap = self.world, self.cap
        ge = self.gbuf[:W * me * 4].view(W, me, 4)
        gs = self.gbuf[W * me * 4:W * (me + ms) * 4].view(W, ms, 4)
        if me:
            dist.all_gather_into_tensor(ge.view(W * me, 4), feat[:me].contiguous())
        if ms:
            dist.all_gather_into_tensor(gs.view(W * ms, 4), feat[cap:cap + ms].contiguous())
        self.payload_bytes += W * (me + ms) * 16
        out = []
        for q in range(W):
            if kf[q]:
                ne, ns = int(allinfo[q, 17]), int(allinfo[q, 18])
                out.append((q, ge[q, :ne], gs[q, :ns], allinfo[q, :16].reshape(4, 4)))
        return out


# ---- the C library's protocol (liblmsf_dist.so, include/lmsf/lmsf_dist.h) over a torch.distributed group
class CGroup:
    """lmsf_group over caller-supplied host collectives (lmsf_group_create_transport) that run on the
    current torch.distributed process group (gloo on CPU): the C / C++ callers' exchange protocol --
    argument agreement, info layout, keyframe order -- executed by the same compiled code the RCCL
    groups use, without GPUs.  Buffers are host memory (numpy)."""

    _AG = None
    _BC = None

    def __init__(self, lib_path=None):
        import ctypes as C
        import os
        import torch.distributed as dist
        from . import _lib
        _lib._share_torch_hip_runtime()
        path = lib_path or os.path.join(_lib.PKG_ROOT, "liblmsf_dist.so")
        L = C.CDLL(path)
        P = C.c_void_p
        CGroup._AG = C.CFUNCTYPE(C.c_int32, P, P, P, C.c_size_t)
        CGroup._BC = C.CFUNCTYPE(C.c_int32, P, P, C.c_size_t, C.c_int32)

        class Transport(C.Structure):
            _fields_ = [("user", P), ("allgather", CGroup._AG), ("broadcast", CGroup._BC)]

        L.lmsf_group_create_transport.argtypes = [C.c_int32, C.c_int32, C.POINTER(Transport), C.POINTER(P)]
        L.lmsf_group_create_transport.restype = C.c_int32
        L.lmsf_group_destroy.argtypes = [P]
        L.lmsf_group_destroy.restype = None
        L.lmsf_group_allgather_poses.argtypes = [P, P, C.c_int32, P]
        L.lmsf_group_broadcast_cloud.argtypes = [P, C.c_int32, P, C.c_size_t, C.POINTER(C.c_size_t)]
        L.lmsf_group_exchange_keyframes.argtypes = [P, P, C.c_int32, C.c_int64, C.c_int64, P, C.c_size_t, P, P,
                                                    P, C.POINTER(C.c_int32)]
        L.lmsf_group_max.argtypes = [P, C.POINTER(C.c_double)]
        for f in ("lmsf_group_allgather_poses", "lmsf_group_broadcast_cloud", "lmsf_group_exchange_keyframes",
                  "lmsf_group_max"):
            getattr(L, f).restype = C.c_int32
        self.C, self.L = C, L
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.gather_bytes = []      # bytes per rank of every all-gather the library asked for (protocol tests)

        def allgather(user, send, recv, nbytes):
            self.gather_bytes.append(int(nbytes))
            try:
                import torch
                src = torch.frombuffer(bytearray(C.string_at(send, nbytes)), dtype=torch.uint8)
                outs = [torch.empty(nbytes, dtype=torch.uint8) for _ in range(self.world)]
                dist.all_gather(outs, src)
                cat = torch.cat(outs).numpy()
                C.memmove(recv, cat.ctypes.data, nbytes * self.world)
                return 0
            except Exception:   # noqa: BLE001 -- reported to the library as a transport failure
                return 1

        def broadcast(user, buf, nbytes, root):
            try:
                import torch
                t = torch.frombuffer(bytearray(C.string_at(buf, nbytes)), dtype=torch.uint8)
                dist.broadcast(t, int(root))
                C.memmove(buf, t.numpy().ctypes.data, nbytes)
                return 0
            except Exception:   # noqa: BLE001
                return 1

        self._cbs = (CGroup._AG(allgather), CGroup._BC(broadcast))   # kept alive with the group
        self._tp = Transport(None, self._cbs[0], self._cbs[1])
        h = P()
        rc = L.lmsf_group_create_transport(self.world, self.rank, C.byref(self._tp), C.byref(h))
        if rc != 0:
            raise RuntimeError(f"lmsf_group_create_transport: {rc}")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.L.lmsf_group_destroy(self.h)
            self.h = None

    def allgather_poses(self, poses):
        p = np.ascontiguousarray(poses, dtype=np.float64).reshape(-1, 7)
        out = np.zeros((self.world, len(p), 7))
        rc = self.L.lmsf_group_allgather_poses(self.h, p.ctypes.data, len(p), out.ctypes.data)
        return rc, out

    def broadcast_cloud(self, root, buf, n):
        """buf: (cap, 4) float32 numpy array (the root's holds n rows); returns (status, rows)."""
        nn = self.C.c_size_t(n)
        rc = self.L.lmsf_group_broadcast_cloud(self.h, root, buf.ctypes.data if buf is not None else None,
                                               0 if buf is None else len(buf), self.C.byref(nn))
        return rc, nn.value

    def exchange_keyframes(self, pose, update_type, n_edge, n_surf, feat, cap, gathered):
        """feat: (2 cap, 4) float32 or None; gathered: float32 of >= world * 2 cap rows or None.
        Returns (status, info (world, 19), any, (rows_edge, rows_surf)); rank r's edges are then rows
        [r rows_edge, + n_edge_r) of gathered and its surfs rows [world rows_edge + r rows_surf, + n_surf_r)."""
        info = np.zeros((self.world, 19))
        anyk = self.C.c_int32(-1)
        rows = np.zeros(2, np.int64)
        P = np.ascontiguousarray(pose, dtype=np.float64)
        rc = self.L.lmsf_group_exchange_keyframes(self.h, P.ctypes.data, int(update_type), int(n_edge), int(n_surf),
                                                  feat.ctypes.data if feat is not None else None, cap, info.ctypes.data,
                                                  gathered.ctypes.data if gathered is not None else None,
                                                  rows.ctypes.data, self.C.byref(anyk))
        return rc, info, anyk.value, (int(rows[0]), int(rows[1]))

    def max(self, v):
        d = self.C.c_double(v)
        rc = self.L.lmsf_group_max(self.h, self.C.byref(d))
        return rc, d.value


class RcclGroup(CGroup):
    """lmsf_group over RCCL (lmsf_group_create): the shipped C library's own communicator on this rank's GPU, the
    code a C / C++ caller of include/lmsf/lmsf_dist.h links.  Rank 0's unique id reaches the other ranks over the
    current torch.distributed group (one 128-byte broadcast before any collective of the library).  Cloud and
    keyframe buffers are device memory of that GPU (torch tensors' data pointers); poses and the max are host."""

    def __init__(self, device_index, lib_path=None):
        import ctypes as C
        import os
        import torch
        import torch.distributed as dist
        from . import _lib
        _lib._share_torch_hip_runtime()     # one HIP runtime and torch's RCCL (same SONAME) in the process
        L = C.CDLL(lib_path or os.path.join(_lib.PKG_ROOT, "liblmsf_dist.so"))
        P = C.c_void_p
        L.lmsf_group_unique_id.argtypes = [P]
        L.lmsf_group_create.argtypes = [C.c_int32, C.c_int32, C.c_int32, P, C.POINTER(P)]
        L.lmsf_group_destroy.argtypes = [P]
        L.lmsf_group_destroy.restype = None
        L.lmsf_group_allgather_poses.argtypes = [P, P, C.c_int32, P]
        L.lmsf_group_broadcast_cloud.argtypes = [P, C.c_int32, P, C.c_size_t, C.POINTER(C.c_size_t)]
        L.lmsf_group_exchange_keyframes.argtypes = [P, P, C.c_int32, C.c_int64, C.c_int64, P, C.c_size_t, P, P,
                                                    P, C.POINTER(C.c_int32)]
        L.lmsf_group_max.argtypes = [P, C.POINTER(C.c_double)]
        for f in ("lmsf_group_unique_id", "lmsf_group_create", "lmsf_group_allgather_poses", "lmsf_group_broadcast_cloud",
                  "lmsf_group_exchange_keyframes", "lmsf_group_max"):
            getattr(L, f).restype = C.c_int32
        self.C, self.L = C, L
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.gather_bytes = []
        uid = np.zeros(128, np.uint8)
        if self.rank == 0 and L.lmsf_group_unique_id(uid.ctypes.data) != 0:
            raise RuntimeError("lmsf_group_unique_id failed")
        bdev = torch.device("cuda", device_index) if dist.get_backend() == "nccl" else torch.device("cpu")
        t = torch.from_numpy(uid).to(bdev)
        dist.broadcast(t, 0)
        uid = np.ascontiguousarray(t.cpu().numpy())
        h = P()
        rc = L.lmsf_group_create(int(device_index), self.world, self.rank, uid.ctypes.data, C.byref(h))
        if rc != 0:
            raise RuntimeError(f"lmsf_group_create: {rc}")
        self.h = h


class Collectives:
    """The exchanges of the N-rank paths over torch.distributed (`impl` "torch": the functions
    above).  world <= 1: no collective at all."""

    impl = "torch"

    def __init__(self, world, device=None):
        self.world, self.device = world, device

    def gather_poses(self, poses, gathered):
        return gather_poses(poses, gathered, self.device)

    def gather_pair_poses(self, poses, n_pairs):
        return gather_pair_poses(poses, n_pairs, self.world, self.device)

    def max(self, v):
        return max_over_ranks(v, self.device)

    def broadcast_map(self, edge, surf):
        return broadcast_map(edge, surf, self.device)

    def keyframe_exchange(self, cap):
        return KeyframeExchange(cap, self.world, self.device)

    def close(self):
        pass


class CCollectives(Collectives):
    """The same exchanges through the shipped C library (liblmsf_dist.so, include/lmsf/lmsf_dist.h): its RCCL
    communicator on the rank's GPU ("c-rccl", device buffers), or -- ranks on gloo (the CPU and gloo-gpu
    rehearsals) -- its protocol over torch.distributed host collectives ("c-transport", host buffers).  Results
    are returned in the torch implementation's forms, so the bench paths do not depend on which one runs."""

    def __init__(self, world, device=None, device_index=None, rccl=True):
        super().__init__(world, device)
        self.rccl = rccl
        self.impl = "c-rccl" if rccl else "c-transport"
        self.g = RcclGroup(device_index) if rccl else CGroup()

    def _check(self, rc, what):
        if rc != 0:
            raise RuntimeError(f"{what}: lmsf status {rc}")

    def gather_poses(self, poses, gathered):
        rc, allp = self.g.allgather_poses(poses)
        self._check(rc, "lmsf_group_allgather_poses")
        import torch
        gathered.copy_(torch.from_numpy(allp))
        return gathered

    def gather_pair_poses(self, poses, n_pairs):
        per = -(-n_pairs // self.world)
        buf = np.zeros((per, 7))
        buf[:len(poses)] = poses
        rc, allp = self.g.allgather_poses(buf)
        self._check(rc, "lmsf_group_allgather_poses")
        res = np.zeros((n_pairs, 7))
        for r in range(self.world):
            idx = pair_partition(n_pairs, r, self.world)
            res[idx] = allp[r, :len(idx)]
        return res

    def max(self, v):
        rc, m = self.g.max(float(v))
        self._check(rc, "lmsf_group_max")
        return m

    def broadcast_map(self, edge, surf):
        """Rank 0's maps into every rank's buffers with lmsf_group_broadcast_cloud (row counts first, by
        lmsf_group_max, so every rank sizes its buffer)."""
        import torch
        out = []
        for src in (edge, surf):
            n = int(self.max(float(len(src)) if self.g.rank == 0 else 0.0))
            on = self.device if self.rccl else torch.device("cpu")
            if self.g.rank == 0:
                t = torch.as_tensor(np.ascontiguousarray(src, dtype=np.float32)).to(on).contiguous()
            else:
                t = torch.empty((n, 4), dtype=torch.float32, device=on)
            if self.rccl:
                torch.cuda.synchronize(self.device)   # torch's upload / allocation done before the library's stream reads
            self._check(self._bcast(t, n), "lmsf_group_broadcast_cloud")
            out.append(t.to(self.device) if self.device is not None else t)
        return out[0], out[1]

    def _bcast(self, t, n):
        C = self.g.C
        nn = C.c_size_t(n)
        if self.rccl:
            return self.g.L.lmsf_group_broadcast_cloud(self.g.h, 0, C.c_void_p(t.data_ptr()) if n else None, n,
                                                       C.byref(nn))
        a = t.numpy()
        rc, _ = self.g.broadcast_cloud(0, a if n else None, n)
        return rc

    def keyframe_exchange(self, cap):
        return CKeyframeExchange(self, cap)

    def close(self):
        self.g.close()


class CKeyframeExchange:
    """KeyframeExchange's interface on lmsf_group_exchange_keyframes: (pose, update type, counts) of every rank,
    then -- only when some rank keyframed -- the features at the keyframing ranks' largest counts; returns
    [(rank, edge_view, surf_view, pose4x4)] for the keyframed streams in rank order."""

    def __init__(self, coll, cap):
        import torch
        self.coll, self.cap, self.world = coll, cap, coll.world
        on = coll.device if coll.rccl else torch.device("cpu")
        self.gbuf = torch.zeros((coll.world * 2 * cap, 4), dtype=torch.float32, device=on)
        self.hfeat = None if coll.rccl else torch.zeros((2 * cap, 4), dtype=torch.float32)
        if coll.rccl:
            torch.cuda.synchronize(coll.device)       # the zeroed buffer before the library's stream writes it
        self.payload_bytes = 0
        self.steps = 0

    def exchange(self, pose, update_type, n_edge, n_surf, feat):
        self.steps += 1
        if self.world <= 1:
            return [(0, None, None, np.asarray(pose, dtype=np.float64).reshape(4, 4))] if update_type else []
        g = self.coll.g
        C = g.C
        P = np.ascontiguousarray(pose, dtype=np.float64).reshape(16)
        info = np.zeros((self.world, 19))
        rows = np.zeros(2, np.int64)
        anyk = C.c_int32(0)
        if self.coll.rccl:
            fptr, gptr = C.c_void_p(feat.data_ptr()), C.c_void_p(self.gbuf.data_ptr())
        else:
            if update_type:
                self.hfeat[:n_edge].copy_(feat[:n_edge])
                self.hfeat[self.cap:self.cap + n_surf].copy_(feat[self.cap:self.cap + n_surf])
            fptr, gptr = C.c_void_p(self.hfeat.data_ptr()), C.c_void_p(self.gbuf.data_ptr())
        rc = g.L.lmsf_group_exchange_keyframes(g.h, P.ctypes.data, int(update_type), int(n_edge), int(n_surf), fptr,
                                               self.cap, info.ctypes.data, gptr, rows.ctypes.data, C.byref(anyk))
        if rc != 0:
            raise ValueError(f"lmsf_group_exchange_keyframes: status {rc} (counts above the smallest rank capacity?)")
        if not anyk.value:
            return []
        W, re_, rs = self.world, int(rows[0]), int(rows[1])
        self.payload_bytes += W * (re_ + rs) * 16
        out = []
        for q in range(W):
            if info[q, 16] > 0:
                ne, ns = int(info[q, 17]), int(info[q, 18])
                e0, s0 = q * re_, W * re_ + q * rs
                out.append((q, self.gbuf[e0:e0 + ne], self.gbuf[s0:s0 + ns], info[q, :16].reshape(4, 4)))
        return out


def make_collectives(impl, world, device=None, device_index=None):
    """impl "torch" | "c" (the shipped C library: RCCL on the nccl backend, its host transport on gloo)."""
    if impl == "c" and world > 1:
        import torch.distributed as dist
        return CCollectives(world, device, device_index, rccl=dist.get_backend() == "nccl")
    return Collectives(world, device)
