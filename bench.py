"""Benchmark of the MI355X LOAM registration hot path (BASELINE.json configs).

Default (the driver's line): C2 -- LiDAR scans/s registered, ~64k-point VLP-16 scans vs a
1M-point feature map.  One step = one pass of the hot path over one batch of B synthetic scans per
GPU: LOAM feature extraction from the raw scans + scan-to-map registration (5 outer iterations of
5-NN matching, line/plane fits and a 4-iteration Ceres-equivalent LM), followed by the RCCL
all-gather of the resulting 6-DoF poses across ranks.  Inputs (raw scans, map index) are resident
in HBM before the timed region.  Weak scaling: B scans per GPU.

Other configurations (`--config`), each its own JSON line:
  C3  dual-LiDAR frames/s: per frame two 16-beam 4096-column scans (~2 x 63k points), primary
      tracker Solve + sub-LiDAR online extrinsic refine against the primary local map
      (MultiLidarSystem phase 1); one independent system per GPU (weak scaling).
  C4  tracking scans/s: one scan stream per GPU tracked against a shared 5M-point map (RCCL
      broadcast from rank 0) plus the stitched window of every stream's keyframes (RCCL
      all-gather of poses every step, of keyframe features when a stream keyframes).
  C5  scan pairs/s: 1,000 re-registrations of 128-beam 2048-column scans (~254k points) against a
      10M-point map, pairs partitioned i mod N, one all-gather of the poses (strong scaling).

Usage: python bench.py [--config C2|C3|C4|C5] [--gpus N --steps K --warmup W ...]
       With --gpus N > 1 outside torch.distributed.run, the bench starts
       `python -m torch.distributed.run --nproc-per-node N bench.py ...` as a child process (one rank
       per GPU) and exits with its return code; inside the ranks WORLD_SIZE must equal N.

Roofline (`roofline`): the dominant kernel's PMC-measured HBM bytes per launch (rocprofv3 FETCH_SIZE /
WRITE_SIZE passes committed under profiles/, `traffic`) over its live HIP-event launch time; the
SURVEY 8(d) byte model (counted over the queries that actually searched) is reported beside it as
`roofline.model`, flagged when it would exceed the HBM peak.
"""
import argparse
import collections
import json
import math
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "lmsf-slam_amd"))

HBM_PEAK_GBS = 8000.0   # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)

DEFAULTS = {   # per configuration: batch (scans per launch), map points, columns, steps, warmup
    # C2 defaults follow SURVEY 8(d) "Scans/s": 1,024 scans (4 x 256) after one warm-up step.  Batch 256
    # over 2 context streams of 128 (measured, r01, with the query memo: 128 x 1 stream 19.0k scans/s,
    # 128 x 2 19.8k, 256 x 2 20.9k; before it 64 x 1 17.3k, 64 x 2 17.8k; 4 streams lose): one launch
    # per context is ~12 ms of latency, well inside a 10 Hz LiDAR's 100 ms
    # 40 steps = ~0.9 s timed (a 4-step window is dominated by clock ramp / host jitter)
    # r02 (tools/gpu_ab_batch.sh, 128 slots per context): 256 x 2 streams 22.37-22.39k scans/s, 384 x 3
    # 22.84k, 512 x 4 23.06-23.13k, 768 x 6 23.07k, 1024 x 8 22.92k, 1024 x 4 (256 per context) 22.92k,
    # 512 x 8 (64 per context) 22.27k: four contexts of 128 fill the chip's gaps best (22 ms per step)
    # r05 (two boxes, alternating, 512 scans per step): 2 contexts of 256 28.35-28.38k / 27.91-28.11k scans/s, 4 of
    # 128 27.98-28.08k / 27.70-27.72k, 3 27.84-28.00k, 6 27.85-28.01k, 8 27.66-27.68k, 1 27.50-27.55k -- with the
    # r03-r05 per-launch savings (wave LM control, memo lists) two larger launches now overlap best
    "C2": dict(batch=512, map_points=1_000_000, cols=4096, steps=40, warmup=2, streams=2),
    "C3": dict(batch=1, map_points=0, cols=4096, steps=20, warmup=3),
    "C4": dict(batch=1, map_points=5_000_000, cols=4096, steps=20, warmup=3),
    # C5: launches of 125 taken in turn by 3 contexts (r04 A/B, two rounds each: 1 context 3,836 pairs/s, 2 4,104,
    # 3 4,114-4,169, 4 4,138-4,149, 8 4,083-4,108): a launch's LM-control phases overlap the next one's search.
    # r05 re-check: 2 4,264-4,270, 2 x 250 scans 4,287-4,300, 3 4,321-4,327, 4 4,341-4,356 -- 3 kept (4 within 0.5%)
    "C5": dict(batch=125, map_points=10_000_000, cols=2048, steps=2, warmup=1, pipeline=3),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C2", choices=sorted(DEFAULTS))
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--batch", type=int, default=None, help="scans per GPU per launch")
    ap.add_argument("--unique-scans", type=int, default=None, help="distinct synthetic scans per rank")
    ap.add_argument("--streams", type=int, default=None,
                    help="C2/C5: contexts per GPU (one HIP stream each) sharing a launch batch; their kernels "
                         "run concurrently, so the small solver / extraction launches of one fill the chip "
                         "beside the other's")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="C5: contexts per GPU taking whole launches of the pass in turn (launch j on context j mod "
                         "P, its previous launch waited for first), so one launch's solver phases overlap the "
                         "next one's search")
    ap.add_argument("--inflight", type=int, default=None,
                    help="C2: at most this many of the --streams contexts' launches in flight (the next one "
                         "launched when the oldest finishes; default: all)")
    ap.add_argument("--map-points", type=int, default=None)
    ap.add_argument("--cols", type=int, default=None)
    ap.add_argument("--outer", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=1000, help="C5: scan pairs in the whole job")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-lookahead", action="store_true",
                    help="C3 / C4: trackers without the keyframe lookahead (lmsf_tracker_config.keyframe_lookahead = 0, "
                         "event-ordered rebuilds) -- for PMC passes, whose serialised dispatches would stall its "
                         "device-side flag waits")
    ap.add_argument("--no-prefetch", action="store_true",
                    help="C3/C4: extract each scan only when its step starts (default: the next scan's extraction "
                         "runs beside the current registration, lmsf_prefetch_features)")
    ap.add_argument("--no-n27", action="store_true",
                    help="skip the untimed n27-counting step (PMC passes: every dispatch then runs as timed)")
    ap.add_argument("--traffic-json", default=None,
                    help="per-launch HBM bytes of the neighbour-search kernel from rocprofv3 PMC runs")
    ap.add_argument("--h2d", choices=("auto", "on", "off", "shadow"), default="auto",
                    help="C2: also time K steps that stream every step's scans from pinned host memory "
                         "(lmsf_batch_load_scans_async, overlapped with the previous launch) -- reported as "
                         "`h2d_inclusive` beside the HBM-resident headline")
    ap.add_argument("--workers", type=int, default=None, help="processes generating the synthetic scans")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=V",
                    help="context option (lmsf_set_option, e.g. MEMO_BOUND=2 or QUERY_MEMO=0) for A/B runs; the "
                         "line records it under config.options")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo", "gloo-gpu"),
                    help="torch.distributed backend of the ranks (nccl = RCCL); gloo: CPU rehearsal of the launcher; "
                         "gloo-gpu: rehearsal of the N-rank GPU path on a box with fewer GPUs (rank r on GPU r mod "
                         "the device count, gloo collectives on the GPU tensors; the line is marked as a rehearsal)")
    ap.add_argument("--dist-impl", default="auto", choices=("auto", "torch", "c"),
                    help="the N-rank exchanges: c = the shipped C library (liblmsf_dist.so: its RCCL communicator on "
                         "the nccl backend, its protocol over host collectives on gloo), torch = torch.distributed "
                         "(lmsf/multi.py); auto = c (VERDICT r05 #5: the code a C / C++ caller links)")
    ap.add_argument("--dump", default=None, metavar="DIR",
                    help="C4: each rank writes its per-step poses and update types to DIR/c4_rank<r>.npz (the multi-rank "
                         "parity test replays them against oracle trackers); C2: its units' scans (seeds, truth), "
                         "guesses, last-step poses and all-gathered poses to DIR/c2_rank<r>.npz")
    ap.add_argument("--launch-check", action="store_true",
                    help="no GPU work: ranks join the process group, run the C2 pose all-gather on CPU tensors and "
                         "print the line skeleton (CPU test of the --gpus launcher)")
    a = ap.parse_args(argv)
    for k, v in DEFAULTS[a.config].items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    if a.streams is None:
        a.streams = 1
    if a.pipeline is None:
        a.pipeline = 1
    if a.unique_scans is None:
        a.unique_scans = {"C2": a.batch, "C5": a.batch}.get(a.config, 1)   # one distinct scan per slot of a launch
    if a.traffic_json is None:
        a.traffic_json = os.path.join(REPO, "profiles", f"traffic_{a.config}.json")   # latest PMC summary (tools/traffic.py)
    return a


# ----------------------------------------------------------------------------- shared plumbing
def launch_ranks(argv, n):
    """--gpus N outside torch.distributed.run: one child process running the standard launcher with N
    ranks over this script (never exec: the parent must not have touched the GPU, and it waits for and
    forwards the child's return code)."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")   # dmabuf IPC only on this pool (RCCL)
    return subprocess.run(cmd, env=env).returncode


class Dist:
    def __init__(self, backend="nccl", impl="auto"):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.gpu = self.local                             # the device this rank registers on
        self.backend = backend
        self.impl = "c" if impl == "auto" else impl
        self.torch = self.dist = self.dev = self.coll = None

    def _collectives(self):
        from lmsf import multi
        self.coll = multi.make_collectives(self.impl, self.world, self.dev, self.gpu)
        return self

    def init(self):
        """Bind the GPU and join the process group (after the host-side input generation)."""
        import torch
        import torch.distributed as dist
        self.torch, self.dist = torch, dist
        if self.backend == "gloo-gpu":                    # N ranks sharing the box's GPUs, gloo collectives
            self.gpu = self.local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(self.gpu)
            self.dev = torch.device("cuda", self.gpu)
            if self.world > 1:
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                dist.init_process_group("gloo")
            return self._collectives()
        if self.backend != "nccl":                        # CPU rehearsal (gloo)
            self.dev = torch.device("cpu")
            if self.world > 1:
                os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
                dist.init_process_group(self.backend)
            return self._collectives()
        if self.world > 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            torch.cuda.set_device(self.local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", self.local))
        else:
            torch.cuda.set_device(0)
        self.dev = torch.device("cuda", self.local)
        return self._collectives()

    def sync(self):
        if self.dev is not None and self.dev.type == "cuda":
            self.torch.cuda.synchronize()

    def barrier(self):
        if self.world > 1:
            self.dist.barrier()

    def close(self):
        if self.coll is not None:
            self.coll.close()
        if self.world > 1 and self.dist is not None and self.dist.is_initialized():
            self.dist.destroy_process_group()


def timed(d, step, warmup, steps, ctxs, count_n27=True):
    """W untimed steps, then K steps between barrier + synchronize; max over ranks.  The last
    warmup step (or, with W = 0, one step after the timed region) runs with the n27 accounting on:
    it costs the search extra loads, so the timed launches run without it.  Returns the mean n27
    per query of that step with the elapsed time."""
    torch = d.torch

    def counted():
        for c in ctxs:
            c.kernel_stats_reset(timing=False, n27=True)
        step()
        ks = [c.kernel_stats() for c in ctxs]
        return sum(k.n27_sum for k in ks) / max(sum(k.queries for k in ks), 1)

    if not count_n27:
        for _ in range(warmup):
            step()
    else:
        for _ in range(warmup - 1):
            step()
    mean_n27 = (counted() if warmup > 0 else None) if count_n27 else 0.0
    for c in ctxs:
        c.kernel_stats_reset(timing=True)
    d.barrier()
    d.sync()
    t0 = time.perf_counter()
    out = None
    for _ in range(steps):
        out = step()
    d.sync()
    d.barrier()
    elapsed = time.perf_counter() - t0
    if d.world > 1:
        elapsed = d.coll.max(elapsed)
    if mean_n27 is None:
        stats = [c.kernel_stats() for c in ctxs]   # keep the timed launches' accounting
        mean_n27 = counted()
        for c, ks in zip(ctxs, stats):
            c._timed_stats = ks
    return elapsed, out, mean_n27


def timed_stats(ctx):
    """Neighbour-search accounting of the timed launches."""
    return getattr(ctx, "_timed_stats", None) or ctx.kernel_stats()


def sum_stats(stats):
    """Kernel accounting summed over contexts (launch time: each launch's own HIP-event span)."""
    import types
    return types.SimpleNamespace(**{f: sum(getattr(k, f) for k in stats)
                                    for f in ("launches", "total_ms", "queries", "n27_sum", "fused_launches",
                                              "reused_queries", "refit_queries")})


def shared_map(d, make):
    """Map generated on rank 0 and replicated to every GPU by an RCCL broadcast."""
    torch = d.torch
    if d.world == 1:
        e, s = make()
        return torch.from_numpy(e).to(d.dev), torch.from_numpy(s).to(d.dev)
    e, s = make() if d.rank == 0 else (None, None)
    return d.coll.broadcast_map(e, s)


def kernel_name(ks, dense=False):
    """The timed neighbour-search launch: the fused search + fit kernels (batch launches; on a dense map the two
    passes on the first-pass grid and the pass-2 fit) or the single-scan search."""
    if ks.launches and ks.fused_launches == ks.launches and dense:
        return ("dense_pass1_kernel + dense_pass2_kernel + dense_fit2_kernel (dense map: first pass on the 0.5 m "
                "first-pass grid with the fit of the queries it completes, bounded pass-2 walk of the listed rest, "
                "their fit; from outer iteration 3 match_memo_kernel first and dense_pass1_listed_kernel over its "
                "misses in place of the full first pass; one outer iteration)")
    if ks.launches and ks.fused_launches == ks.launches:
        return ("match_memo_kernel + match_fit_kernel (query memo pass from outer iteration 2, then the fused 5-NN "
                "search + line/plane fit + record write of the queries it lists; one outer iteration)")
    return "knn_kernel (8-lane 5-NN search with the slot memo; fit_eval_kernel follows)"


def load_traffic(traffic_json, **match):
    """PMC summary of the dominant kernel (tools/traffic.py) when it was measured on this workload."""
    if not traffic_json or not os.path.exists(traffic_json):
        return None
    try:
        tj = json.load(open(traffic_json))
    except (ValueError, OSError):
        return None
    for k, v in match.items():
        if tj.get(k) != v:
            return None
    return tj


def valu_pass(tj):
    """The committed VALU pass of the profile `tj` was taken from (`<profile>/valu_busy.txt`, tools/valu_busy.py:
    SQ_ACTIVE_INST_VALU x 4 / CUs over GRBM_GUI_ACTIVE / 8, lane utilisation from SQ_ACTIVE_INST_VALU vs thread
    counts): the rows of the kernels `tj` names, the busiest first."""
    if not tj or not tj.get("profile") or not tj.get("kernel"):
        return None
    path = os.path.join(REPO, tj["profile"], "valu_busy.txt")
    if not os.path.exists(path):
        return None
    names = [k.strip() for k in str(tj["kernel"]).split(",") if k.strip()]
    rows = []
    for ln in open(path).read().splitlines()[1:]:
        parts = ln.split()
        if len(parts) < 7:
            continue
        name = " ".join(parts[:-6]).split("::")[-1]
        if not any(name.startswith(n) for n in names):
            continue
        disp, busy, lane, vpw, wait = parts[-6:-1]
        rows.append({"kernel": name, "dispatches": int(disp), "valu_busy": float(busy), "lane_util": float(lane),
                     "valu_per_wave": int(vpw), "wait_any": float(wait)})
    if not rows:
        return None
    rows.sort(key=lambda r: -r["valu_busy"])
    return {"source": os.path.relpath(path, REPO), "kernels": rows}


def binding_roof(valu, frac):
    """What bounds the dominant kernel, from the committed counters: VALU issue when its busiest kernel keeps the
    CUs' VALU >= 75% busy (the f64 fit / key network), HBM when the PMC traffic is >= 60% of peak,
    else latency (waves waiting on dependent loads with the VALU idle: the single-scan launches)."""
    if valu and valu["kernels"][0]["valu_busy"] >= 0.75:
        return "valu"
    if frac is not None and frac >= 0.6:
        return "hbm"
    return "latency" if valu else "hbm"


def knn_roofline(ks, mean_n27, tj, elapsed_s, note, solo=None, dense=False):
    """Roofline of the dominant (neighbour-search) kernel.

    The launch time is `solo` when given: the HIP-stamped span of each search launch (memo pass + fused
    search) measured live in an untimed pass that runs the context streams one at a time, i.e. the kernel
    alone on the chip -- the condition of the committed rocprofv3 profile.  (The timed region runs several
    context streams at once; a launch's span there includes time it shares the chip with other streams'
    kernels, reported as `concurrent`.)  Without `solo` the timed launches' own spans are used (single-
    stream configurations).

    achieved = PMC-measured HBM bytes per launch (`traffic`: (2 FETCH_SIZE + WRITE_SIZE) KiB per outer
    iteration, MI355X_MICROARCH.md's gfx950 correction, from the committed rocprofv3 passes `tj`) / that
    launch time.  `rocprof` recomputes it with the profiler's own mean duration in the PMC run (the two
    agree when the profile is of the current library).  `model` is SURVEY 8(d)'s algorithmic figure over
    the same launch time: sum over the queries that searched of [16 (query) + 27*8 (cell ranges) +
    16 n27(q)] + 16 B per memo-reused query + 16 + 5*16 B per refitted query (its 5 neighbours gathered,
    no walk), n27 per searched query from the counted untimed step; it counts every candidate read as an
    HBM read while the 16 MB map + index stay in L2 / Infinity Cache."""
    t = solo if solo is not None else ks
    launches = max(int(t.launches), 1)
    avg_launch_ms = t.total_ms / launches
    reused = int(getattr(t, "reused_queries", 0))
    refit = int(getattr(t, "refit_queries", 0))
    searched = int(t.queries) - reused - refit
    model_bytes = (searched * (16 + 27 * 8 + 16 * mean_n27) + reused * 16 + refit * (16 + 5 * 16)) / launches
    model_gbs = model_bytes / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    model_wall_gbs = model_bytes * int(ks.launches) / elapsed_s / 1e9 if elapsed_s > 0 else 0.0
    traffic = int(tj["hbm_bytes_per_launch"]) if tj else None
    if traffic and avg_launch_ms > 0:
        achieved, basis = traffic / (avg_launch_ms * 1e-3) / 1e9, "pmc bytes / live " + ("solo" if solo else "timed") + \
            " launch span"
    elif traffic:
        achieved, basis = None, "untimed (no search-launch stamps in this build)"
    else:   # never the model: it counts cache-served candidate reads as HBM bytes
        achieved, basis = None, "unmeasured (no PMC profile of this workload under profiles/)"
    frac = round(achieved / HBM_PEAK_GBS, 4) if achieved is not None else None
    valu = valu_pass(tj)
    # every query priced as a full walk (the strict 8(d) sum): above the HBM peak it proves the timed kernels do not
    # do that work (memo reuse, pruned walks), so no 8(d) figure is a roofline then
    strict_bytes = int(t.queries) * (16 + 27 * 8 + 16 * mean_n27) / launches
    strict_gbs = strict_bytes / (avg_launch_ms * 1e-3) / 1e9 if avg_launch_ms > 0 else 0.0
    out = {"bound": binding_roof(valu, frac), "achieved": round(achieved, 1) if achieved is not None else None,
           "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": frac, "frac_basis": "HBM: PMC bytes over the live launch span",
           "traffic": traffic, "basis": basis, "valu": valu,
           "kernel": kernel_name(ks, dense), "avg_launch_ms": round(avg_launch_ms, 4), "launches": int(t.launches),
           "queries_per_launch": int(t.queries / launches),
           "reused_query_frac": round(reused / max(int(t.queries), 1), 4),
           "refit_query_frac": round(refit / max(int(t.queries), 1), 4),
           "l2_hit_rate": round(tj["l2_hit_rate"], 3) if tj and tj.get("l2_hit_rate") is not None else None,
           "model": {"bytes_per_launch": int(model_bytes), "searched_queries_per_launch": int(searched / launches),
                     "mean_n27": round(mean_n27, 1), "gbs": round(model_gbs, 1),
                     "frac": round(model_gbs / HBM_PEAK_GBS, 4), "gbs_over_timed_window": round(model_wall_gbs, 1),
                     "exceeds_peak": bool(model_gbs > HBM_PEAK_GBS or model_wall_gbs > HBM_PEAK_GBS),
                     "strict": {"bytes_per_launch": int(strict_bytes), "gbs": round(strict_gbs, 1),
                                "exceeds_peak": bool(strict_gbs > HBM_PEAK_GBS)}},
           "note": note}
    # a byte model above the HBM peak cannot be HBM traffic: the walk reads fewer candidates than n27 counts (the
    # pruned walk) or the reads are cache-served -- the model is then no roofline at all; nor is the
    # searched-only form once the strict all-query sum is above the peak (the work it prices is not the timed work)
    out["model"]["valid"] = not (out["model"]["exceeds_peak"] or out["model"]["strict"]["exceeds_peak"])
    if not out["model"]["valid"]:
        out["model"]["frac"] = None
        out["model"]["invalid_reason"] = (
            "the 8(d) byte model exceeds the HBM peak: it counts every candidate of the 27 cells as an HBM read; only "
            "the PMC traffic is a roofline here" if out["model"]["exceeds_peak"] else
            "the strict 8(d) sum over all queries exceeds the HBM peak: the memo / pruned walks skip most of the work "
            "it prices, so neither 8(d) form is a roofline; only the PMC traffic is")
    if solo is not None:
        span = ks.total_ms / max(int(ks.launches), 1)
        out["concurrent"] = {"avg_launch_ms": round(span, 4), "launches": int(ks.launches),
                             "note": "timed region: search-launch spans with the other context streams' kernels "
                                     "sharing the chip (not a kernel duration)"}
    if tj:
        mean_us = tj.get("rocprof_mean_us")
        out["rocprof"] = {"profile": tj.get("profile"), "mean_us": mean_us,
                          "frac": round(traffic / (mean_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4) if mean_us else None,
                          "model_frac": round(model_bytes / (mean_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)
                          if mean_us and out["model"]["valid"] else None,
                          "live_over_rocprof": round(avg_launch_ms * 1e3 / mean_us, 3) if mean_us else None,
                          "dispatches": tj.get("dispatches")}
    return out


def solo_launches(ctxs, guesses_of):
    """One untimed pass over the context streams one at a time (launch + wait each: the search kernels
    run alone on the chip, as in the rocprofv3 profile) with the launch stamps on; their summed accounting."""
    stats = []
    for i, c in enumerate(ctxs):
        g = guesses_of(i)
        if g is None:
            continue
        c.kernel_stats_reset(timing=True)
        c.batch_launch(g)
        c.batch_wait(len(g))
        stats.append(c.kernel_stats())
    return sum_stats(stats) if stats else None


def in_turn(n_units, chunk, P):
    """Launch / wait schedule of a pass whose launches of `chunk` units are taken in turn by P contexts (launch j
    on context j mod P, that context's previous launch waited for first; the rest waited oldest first at the
    end): a list of ("launch" | "wait", context, first unit, count)."""
    ev, busy, order = [], [None] * P, []
    for j, c0 in enumerate(range(0, n_units, chunk)):
        ci, nb = j % P, min(chunk, n_units - c0)
        if busy[ci] is not None:
            ev.append(("wait", ci) + busy[ci])
        ev.append(("launch", ci, c0, nb))
        busy[ci] = (c0, nb)
        order = [x for x in order if x != ci] + [ci]
    return ev + [("wait", ci) + busy[ci] for ci in order]


def apply_options(args, ctxs):
    """--opt NAME=V on every context (lmsf_set_option)."""
    from lmsf import _lib
    for o in args.opt:
        name, v = o.split("=", 1)
        for c in ctxs:
            c.set_option(getattr(_lib, "OPT_" + name.upper()), int(v))


def line(args, d, metric, value, unit, elapsed, scaling, workload, extra_cfg, roofline, cpu, **extra):
    if args.opt:
        extra_cfg = dict(extra_cfg, options=list(args.opt))
    if d.world > 1:               # which code ran the exchanges
        extra_cfg = dict(extra_cfg, dist_impl=d.coll.impl)
    if d.backend == "gloo-gpu":   # ranks share GPUs: a correctness rehearsal, not a scaling measurement
        extra_cfg = dict(extra_cfg, rehearsal=f"{d.world} ranks on {d.torch.cuda.device_count()} GPU(s), gloo")
    out = {"metric": metric, "value": round(value, 2), "unit": unit, "n_gpus": d.world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
           "scaling": scaling, "vs_baseline": None, "dtype": "f64", "data": "synthetic",
           "config": dict({"workload": workload}, **extra_cfg), "roofline": roofline, "cpu_baseline": cpu,
           # which throughput `value` is (the task contract's HBM-resident rate); SURVEY 8(d)'s
           # H2D-inclusive scans/s is `h2d_inclusive` where the configuration streams host scans
           "value_basis": "inputs resident in HBM when the timed region starts (bench contract)"
           + ("; SURVEY 8(d)'s H2D-inclusive figure is h2d_inclusive.value" if extra.get("h2d_inclusive") else "")}
    out.update(extra)
    print(json.dumps(out))


def cpu_oracle():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle
    oracle.set_threads(1)
    return oracle


def cpu_share(usable):
    """Host cores one GPU's CPU baseline may use: the job's per-GPU CPU share when the machine states one
    (OMP_NUM_THREADS, set to the per-GPU share on the GPU pool: 16), else the usable cores over the node's 8 GPUs."""
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        return max(1, min(int(omp), usable)), f"OMP_NUM_THREADS={omp}: the job's per-GPU CPU share"
    return max(1, usable // 8), f"{usable} usable host CPUs / 8 GPUs per node"


def mat_delta(A, B):
    """(translation m, rotation rad) between two 4x4 poses."""
    import numpy as np
    from lmsf import synth
    return float(np.linalg.norm(A[:3, 3] - B[:3, 3])), synth.rot_angle_of_matrix(A[:3, :3].T @ B[:3, :3])


def host_cpu():
    """Host CPU model (report the CPU the baseline ran on) and the cores this process may use."""
    model = "unknown"
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    return model, usable


def _scan_job(job):
    from lmsf import synth
    seed_scene, pose, seed, cols, elev = job
    return synth.make_scan(synth.make_scene(seed_scene, road_length=80.0), pose, seed, n_cols=cols, elev_deg=elev)


def under_profiler():
    """rocprofv3 preloads its tool library (and with --pmc initialises the GPU) before the program starts."""
    return "rocprof" in os.environ.get("LD_PRELOAD", "") or any(k.startswith("ROCPROF") for k in os.environ)


def make_scans(jobs, workers):
    """Synthetic scans generated in a process pool (before the rank touches the GPU: fork is safe), workers
    closed and joined (never signalled).  Serial under rocprofv3: a forked child would carry the profiler's
    tool state and signal handlers."""
    if workers <= 1 or len(jobs) < 4 or under_profiler():
        return [_scan_job(j) for j in jobs]
    import multiprocessing as mp
    pool = mp.get_context("fork").Pool(min(workers, len(jobs)))
    try:
        out = pool.map(_scan_job, jobs, chunksize=max(1, len(jobs) // (4 * workers)))
    finally:
        pool.close()
        pool.join()
    return out


def exchange_poses(cfg, poses, gathered, pairs, coll):
    """The C2 / C5 collective section: the RCCL all-gather of every rank's 6-DoF poses, through the
    shipped C library (lmsf_group_allgather_poses) or torch.distributed (--dist-impl)."""
    if coll.world <= 1:
        return poses
    if cfg == "C2":
        return coll.gather_poses(poses, gathered)
    return coll.gather_pair_poses(poses, pairs)


def run_launch_check(args, d):
    """--launch-check: the ranks of a `--gpus N` launch join the process group (gloo on CPU) and run the
    C2 pose all-gather; rank 0 prints the line skeleton (n_gpus = world size)."""
    import numpy as np
    import torch
    n = 4
    poses = np.stack([np.full(7, 1000.0 * d.rank + i) for i in range(n)])
    gathered = torch.zeros((d.world, n, 7), dtype=torch.float64)
    g = exchange_poses("C2", poses, gathered, 0, d.coll)
    g = g.numpy() if hasattr(g, "numpy") else np.asarray(g)[None]
    ok = all(np.array_equal(g[r], np.stack([np.full(7, 1000.0 * r + i) for i in range(n)])) for r in range(d.world))
    if d.world > 1:
        ok = d.coll.max(0.0 if ok else 1.0) == 0.0
    if d.rank == 0:
        print(json.dumps({"metric": "launch-check", "value": 0.0, "unit": "scans/s", "n_gpus": d.world,
                          "steps": args.steps, "warmup": args.warmup, "backend": d.backend, "gather_ok": bool(ok),
                          "dist_impl": d.coll.impl}))
    return 0 if ok else 4


# ----------------------------------------------------------------------------- C2 / C5: batch re-registration
def run_batch(args, d):
    import numpy as np
    from lmsf import multi, synth
    cfg = args.config
    c = synth.CONFIGS[cfg]
    k = c["k"]
    world, rank = d.world, d.rank
    U = max(1, min(args.unique_scans, args.batch))
    if cfg == "C5" and args.batch % U:
        args.batch -= args.batch % U          # slot j holds scan j % U in every chunk
    truth_u = synth.trajectory(U * world, 3000 + k, step=80.0 / max(U * world, 1))[rank * U:(rank + 1) * U]
    scans_u = make_scans([(1000 + k, truth_u[i], 2000 + k + 97 * (rank * U + i), args.cols, c["elev"])
                          for i in range(U)], args.workers)
    d.init()
    torch = d.torch
    from lmsf import _lib
    scene = synth.make_scene(1000 + k, road_length=80.0)
    em_t, sm_t = shared_map(d, lambda: synth.make_map(scene, args.map_points, 1000 + k + 7, center_x=(0.0, 80.0),
                                                      radius=c["radius"]))
    if cfg == "C2":
        n_units = args.batch                                   # scans this rank registers per step
        unit_scan = [i % U for i in range(n_units)]
        rng = np.random.default_rng(3000 + k + rank)
        guesses = np.stack([synth.perturb(truth_u[unit_scan[i]], rng) for i in range(n_units)])
    else:                                                      # C5: pairs i = rank, rank + N, ...
        mine = multi.pair_partition(args.pairs, rank, world)
        n_units = len(mine)
        unit_scan = [j % U for j in range(n_units)]
        guesses = np.stack([synth.perturb(truth_u[unit_scan[j]], np.random.default_rng(3000 + k + 7919 * i))
                            for j, i in enumerate(mine)])
    chunk = min(args.batch, n_units)
    P = max(1, args.pipeline) if cfg == "C5" and n_units > chunk else 1   # contexts taking launches in turn
    S = 1 if P > 1 else max(1, min(args.streams, chunk))    # contexts sharing one launch
    sub_b = -(-chunk // S)                                   # slots per context
    max_pts = max(len(s) for s in scans_u)
    ctxs = [_lib.Context(device=d.gpu, max_batch=sub_b, max_scan_points=max_pts + 64, max_features=max_pts + 64,
                         schedule=_lib.SCHEDULE_FIXED, max_iterations=args.outer, **c["extract"])
            for _ in range(max(S, P))]
    apply_options(args, ctxs)
    ctx_scans = [[scans_u[j % U] for j in range(i * sub_b, min((i + 1) * sub_b, chunk))] for i in range(S)]
    ctx_scans += [ctx_scans[0]] * (len(ctxs) - S)            # pipelined contexts: every launch holds the same slots
    for cx, sc in zip(ctxs, ctx_scans):
        cx.set_map(_lib.EDGE, em_t)
        cx.set_map(_lib.SURF, sm_t)
        cx.load_scans(sc)
    map_points = int(em_t.shape[0] + sm_t.shape[0])
    gathered = torch.zeros((world, n_units, 7), dtype=torch.float64, device=d.dev)
    poses = np.zeros((n_units, 7))
    matches = np.zeros(n_units, np.int64)                    # residual blocks of each unit's last outer iteration
    enqueue_s = []                                           # host time inside lmsf_batch_launch, per step
    coll_s = []                                              # host time of the pose all-gather section, per step
    stream_in = {"on": False, "shadow": None}
    host_bufs = []

    def pipelined_step():
        enq = 0.0
        for kind, ci, a, m in in_turn(n_units, chunk, P):
            if kind == "wait":
                poses[a:a + m], st = ctxs[ci].batch_wait(m)
                matches[a:a + m] = [s.edge_matches + s.surf_matches for s in st]
            else:
                t_enq = time.perf_counter()
                ctxs[ci].batch_launch(guesses[a:a + m])
                enq += time.perf_counter() - t_enq
        t_c = time.perf_counter()
        exchange_poses(cfg, poses, gathered, args.pairs, d.coll)
        coll_s.append(time.perf_counter() - t_c)
        enqueue_s.append(enq)
        return poses

    def step():
        if P > 1:
            return pipelined_step()
        enq = 0.0
        for c0 in range(0, n_units, chunk):
            nb = min(chunk, n_units - c0)
            parts = [(i, cx, c0 + i * sub_b, min(sub_b, nb - i * sub_b)) for i, cx in enumerate(ctxs) if nb > i * sub_b]
            W = len(parts) if not args.inflight else max(1, min(args.inflight, len(parts)))
            if W < len(parts):                               # a window of W launches in flight, oldest waited first
                for k2, (i, cx, a, m) in enumerate(parts):
                    if k2 >= W:
                        _, cw, aw, mw = parts[k2 - W]
                        poses[aw:aw + mw], st = cw.batch_wait(mw)
                        matches[aw:aw + mw] = [s.edge_matches + s.surf_matches for s in st]
                    t_enq = time.perf_counter()
                    cx.batch_launch(guesses[a:a + m])
                    enq += time.perf_counter() - t_enq
                for i, cx, a, m in parts[len(parts) - W:]:
                    poses[a:a + m], st = cx.batch_wait(m)
                    matches[a:a + m] = [s.edge_matches + s.surf_matches for s in st]
                continue
            for i, cx, a, m in parts:                        # every context's batch enqueued before any wait
                t_enq = time.perf_counter()
                cx.batch_launch(guesses[a:a + m])
                enq += time.perf_counter() - t_enq
                if stream_in["shadow"] is not None:          # diagnostics: the same DMA, nothing waits for it
                    dst, side, spans = stream_in["shadow"]
                    with torch.cuda.stream(side):
                        e0 = torch.cuda.Event(enable_timing=True)
                        e1 = torch.cuda.Event(enable_timing=True)
                        e0.record(side)
                        dst[i].copy_(host_bufs[i][0], non_blocking=True)
                        e1.record(side)
                        spans.append((e0, e1))
                elif stream_in["on"]:                        # next step's scans, overlapped with this launch
                    cx.load_scans_async(*host_bufs[i])
            for i, cx, a, m in parts:
                poses[a:a + m], st = cx.batch_wait(m)
                matches[a:a + m] = [s.edge_matches + s.surf_matches for s in st]
        t_c = time.perf_counter()
        exchange_poses(cfg, poses, gathered, args.pairs, d.coll)
        coll_s.append(time.perf_counter() - t_c)
        enqueue_s.append(enq)
        return poses

    elapsed, _, mean_n27 = timed(d, step, args.warmup, args.steps, ctxs, not args.no_n27)
    if args.dump and cfg == "C2":   # the multi-rank parity test (tests/test_gpu_multirank.py) replays these
        os.makedirs(args.dump, exist_ok=True)
        g = gathered.cpu().numpy() if world > 1 else poses[None].copy()
        np.savez(os.path.join(args.dump, f"c2_rank{rank}.npz"), poses=poses, gathered=g, guesses=guesses,
                 truth_u=truth_u, unit_scan=np.asarray(unit_scan),
                 seeds=np.asarray([2000 + k + 97 * (rank * U + i) for i in range(U)]), world=world, cols=args.cols,
                 map_points=args.map_points)
    enqueue_ms = float(np.median(enqueue_s)) * 1e3
    timed_coll = coll_s[args.warmup:args.warmup + args.steps]   # timed() runs the warmups first
    collective_ms = round(1e3 * float(np.mean(timed_coll)), 4) if timed_coll and world > 1 else 0.0
    ks = sum_stats([timed_stats(cx) for cx in ctxs])
    total_units = (args.batch * world if cfg == "C2" else args.pairs) * args.steps
    terr = [synth.pose_delta(poses[i], truth_u[unit_scan[i]]) for i in range(n_units)]
    tj = load_traffic(args.traffic_json, config=cfg, batch=sub_b, streams=1, map_points=map_points,
                      unique_scans=min(U, sub_b))
    solo = None
    if S > 1 or P > 1:   # kernel time alone on the chip (the profile's condition), live, after the timed region
        c0 = 0
        solo = solo_launches(ctxs, lambda i: guesses[c0 + i * sub_b:c0 + min((i + 1) * sub_b, chunk)]
                             if i * sub_b < chunk else None)
    roof = knn_roofline(ks, mean_n27, tj, elapsed,
                        "traffic: PMC bytes per outer iteration (memo pass + search) from a one-stream rocprofv3 run "
                        "of the same per-context batch (device-wide counters, profiles/); avg_launch_ms: device "
                        "wall-clock stamps around each search launch of a live untimed pass running one context "
                        "stream at a time", solo=solo, dense=cfg == "C5")
    h2d = None
    if cfg == "C2" and (args.h2d in ("on", "shadow") or (args.h2d == "auto" and U == n_units)):
        # SURVEY 8(d) "including ... H2D of the scan": the same K steps with every step's scans streamed
        # from page-locked host memory (one DMA per context, issued right after that context's launch so
        # it overlaps the registration; the copy waits for the launch's extraction to have read the slots)
        for sc in ctx_scans:
            counts = np.array([len(x) for x in sc], np.int64)
            buf = torch.from_numpy(np.concatenate(sc, 0)).pin_memory()
            host_bufs.append((buf, counts))
        if args.h2d == "shadow":   # diagnostics: uploads into scratch on a side stream, launches on resident scans
            lo, hi = torch.cuda.Stream.priority_range()
            stream_in["shadow"] = ([torch.empty_like(b, device=d.dev) for b, _ in host_bufs],
                                   torch.cuda.Stream(priority=hi), [])
        else:
            for cx, (buf, counts) in zip(ctxs, host_bufs):
                cx.load_scans_async(buf, counts)
        stream_in["on"] = True
        step()
        d.barrier()
        d.sync()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        d.sync()
        d.barrier()
        el2 = time.perf_counter() - t0
        if world > 1:
            el2 = d.coll.max(el2)
        stream_in["on"] = False
        copy_ms = None
        if stream_in["shadow"] is not None:   # DMA time of the uploads alone: ms per step (link-bound if ~ step)
            spans = stream_in["shadow"][2][len(host_bufs):]   # the timed steps (after the untimed one)
            copy_ms = round(sum(a.elapsed_time(b) for a, b in spans) / max(args.steps, 1), 3)
        stream_in["shadow"] = None
        up = sum(int(b.numel()) * 4 for b, _ in host_bufs)
        h2d = {"value": round(args.batch * world * args.steps / el2, 2), "unit": "scans/s",
               "ms_per_step": round(el2 / args.steps * 1e3, 3), "upload_bytes_per_step_per_gpu": up,
               "mode": args.h2d if args.h2d == "shadow" else "streamed",
               **({"upload_dma_ms_per_step": copy_ms} if copy_ms is not None else {}),
               "note": "every step's raw scans uploaded from pinned host memory inside the timed window "
                       "(lmsf_batch_load_scans_async on each context's copy stream, overlapped with the previous "
                       "launch); the headline `value` keeps the scans HBM-resident"}
    cpu, pose_dv = None, None
    if rank == 0 and world == 1 and not args.no_cpu:
        oracle = cpu_oracle()
        model, usable = host_cpu()
        reg = oracle.Registration()
        reg.set_map(1, em_t.cpu().numpy())           # the same broadcast map
        reg.set_map(2, sm_t.cpu().numpy())
        reg.set_fixed_schedule(True)
        reg.set_max_iterations(args.outer)
        n_done, worst_t, worst_r = 0, 0.0, 0.0
        t1 = time.perf_counter()
        while n_done < n_units and (n_done == 0 or time.perf_counter() - t1 < args.cpu_seconds):
            e, s, _, _ = oracle.extract(scans_u[unit_scan[n_done]], **c["extract"])
            reg.set_scan(1, e)
            reg.set_scan(2, s)
            ox, _, _ = reg.solve(guesses[n_done])
            dt, dr = synth.pose_delta(ox, poses[n_done])
            worst_t, worst_r = max(worst_t, dt), max(worst_r, dr)
            n_done += 1
        cpu_el = time.perf_counter() - t1
        unit = "scans/s" if cfg == "C2" else "pairs/s"
        cpu = {"value": round(n_done / cpu_el, 3), "unit": unit, "cores": 1, "kind": "port", "cpu_model": model,
               "sample": f"{n_done} {'scans' if cfg == 'C2' else 'pairs'} of the same {cfg} workload (extract + "
                         f"{args.outer} outer iterations, kd-tree 5-NN, Ceres-LM restatement; kd-tree build "
                         f"excluded), {cpu_el:.1f} s on 1 thread of a {model} ({os.cpu_count()} host CPUs, "
                         f"{usable} usable)"}
        pose_dv = {"scans": n_done, "max_m": worst_t, "max_rad": worst_r}
        # the same restatement with OpenMP over queries on one GPU's share of the host cores,
        # reported beside the single-thread baseline (cpu_share: the share and where it comes from)
        nt, share_basis = cpu_share(usable)
        oracle.set_threads(nt)
        m_done = 0
        t2 = time.perf_counter()
        while m_done < n_units and (m_done == 0 or time.perf_counter() - t2 < args.cpu_seconds / 3):
            e, s, _, _ = oracle.extract(scans_u[unit_scan[m_done]], **c["extract"])
            reg.set_scan(1, e)
            reg.set_scan(2, s)
            reg.solve(guesses[m_done])
            m_done += 1
        mt_el = time.perf_counter() - t2
        oracle.set_threads(1)
        cpu["multi_thread"] = {"value": round(m_done / mt_el, 3), "cores": nt, "cores_basis": share_basis,
                               "host_cpus": os.cpu_count(), "usable_cpus": usable,
                               "sample": f"{m_done} {'scans' if cfg == 'C2' else 'pairs'}, {mt_el:.1f} s, OpenMP "
                                         f"over queries"}
    if rank == 0:
        npts = int(np.mean([len(s) for s in scans_u]))
        if cfg == "C2":
            metric = "LiDAR scans/sec registered (64k-pt scan, 1M-pt map)"
            wl = (f"C2: VLP-16 16x{args.cols} scans (~{npts} pts) vs {map_points}-pt edge+surf map, "
                  f"{args.outer} outer iters x Ceres-LM(4), extraction included, batch {args.batch} scans/GPU "
                  f"({U} distinct) over {S} context stream(s), scans HBM-resident")
            extra = {"batch_per_gpu": args.batch, "distinct_scans_per_gpu": U, "map_points": map_points,
                     "outer_iterations": args.outer, "parallelism": f"scan-sharded x{world}"}
            if ks.launches and roof is not None:   # residual blocks the LM evaluations stream, over the features (queries) of the batch
                roof["matched_record_frac"] = round(float(matches.sum()) / (ks.queries / ks.launches * S), 4)
            extra["host_enqueue_ms_per_step"] = round(enqueue_ms, 3)   # lmsf_batch_launch calls, all contexts
            unit, scaling = "scans/s", "weak"
        else:
            metric = "LiDAR scan pairs/sec re-registered (128-beam 254k-pt scan, 10M-pt map, 1k pairs)"
            wl = (f"C5: 128x{args.cols} scans (~{npts} pts, {U} distinct per GPU) vs {map_points}-pt map, "
                  f"{args.pairs} pairs (i mod {world} per GPU, launches of {chunk}"
                  + (f", {P} contexts taking them in turn" if P > 1 else "") + f"), {args.outer} outer iters x "
                  f"Ceres-LM(4)")
            extra = {"pairs": args.pairs, "launch_batch": chunk, "pipelined_contexts": P,
                     "distinct_scans_per_gpu": U, "map_points": map_points,
                     "outer_iterations": args.outer, "parallelism": f"pair-sharded x{world}"}
            unit, scaling = "pairs/s", "strong"
        extra["collective_ms_per_step"] = collective_ms   # pose all-gather section (0: one rank, no collective)
        line(args, d, metric, total_units / elapsed, unit, elapsed, scaling, wl, extra, roof, cpu,
             h2d_inclusive=h2d, pose_delta_vs_cpu=pose_dv,
             pose_error_vs_truth={"max_m": max(t for t, _ in terr), "max_rad": max(r for _, r in terr)})
    for cx in ctxs:
        cx.close()


# ----------------------------------------------------------------------------- C4: stitched multi-stream tracking
def c4_stream(rank, world, n, cols, workers=1):
    """Rank `rank`'s C4 stream: ground truth and synthetic scans (8 m/s at 10 Hz, its own start on the road)."""
    from lmsf import synth
    c = synth.CONFIGS["C4"]
    k = c["k"]
    start = 8.0 * rank if world <= 8 else 64.0 * rank / world
    truth = synth.trajectory(n, 3000 + k + rank, step=0.8, start_x=start)
    scans = make_scans([(1000 + k, truth[i], 2000 + k + 97 * i + 7717 * rank, cols, c["elev"]) for i in range(n)], workers)
    return truth, scans


def c4_map(map_points):
    """The shared C4 prior map (generated on rank 0 and broadcast)."""
    from lmsf import synth
    c = synth.CONFIGS["C4"]
    k = c["k"]
    scene = synth.make_scene(1000 + k, road_length=80.0)
    return synth.make_map(scene, map_points, 1000 + k + 7, center_x=(0.0, 80.0), radius=c["radius"])


def run_streams(args, d):
    import numpy as np
    from lmsf import multi, synth
    world, rank = d.world, d.rank
    n = args.warmup + args.steps
    truth, scans = c4_stream(rank, world, n, args.cols, args.workers)
    d.init()
    torch = d.torch
    from lmsf import _lib
    scans_dev = [torch.from_numpy(s).to(d.dev) for s in scans]
    em_t, sm_t = shared_map(d, lambda: c4_map(args.map_points))
    max_pts = max(len(s) for s in scans)
    ctx = _lib.Context(device=d.gpu, max_batch=1, max_scan_points=max_pts + 64, max_features=max_pts + 64,
                       schedule=_lib.SCHEDULE_FIXED, max_iterations=args.outer)
    apply_options(args, [ctx])
    # keyframe lookahead (lmsf_tracker_config.keyframe_lookahead) only for one stream: with several, the keyframes of
    # lower ranks are appended before this rank's own and would undo it at every step
    tr = _lib.Tracker(ctx, manual_map_update=True, keyframe_lookahead=(world == 1 and not args.no_lookahead))
    T0 = np.eye(4)
    T0[:3, :3] = synth.quat_to_mat(truth[0][:4])
    T0[:3, 3] = truth[0][4:]
    tr.set_initial_pose(T0)
    tr.set_prior_map(_lib.EDGE, em_t)
    tr.set_prior_map(_lib.SURF, sm_t)
    map_points = int(em_t.shape[0] + sm_t.shape[0])
    cap = max_pts + 64
    fbuf = torch.zeros((2 * cap, 4), dtype=torch.float32, device=d.dev)       # [edges | surfs] of own scan
    xchg = d.coll.keyframe_exchange(cap)
    state = {"i": 0, "kf": 0, "err": [], "xchg_s": 0.0, "poses": [], "types": []}

    phases = collections.defaultdict(float) if os.environ.get("LMSF_BENCH_PHASES") else None

    def mark(name, t0):   # host time per call (diagnostics: LMSF_BENCH_PHASES=1 prints the means to stderr)
        t1 = time.perf_counter()
        if phases is not None:
            phases[name] += t1 - t0
        return t1

    def step():
        i = state["i"]
        t = time.perf_counter()
        ctx.extract(scans_dev[i])
        if not args.no_prefetch and i + 1 < n:
            ctx.prefetch(scans_dev[i + 1])   # the preprocess thread running one scan ahead
        t = mark("extract", t)
        _, r = tr.solve_extracted(0.1 * i)
        t = mark("solve", t)
        P = tr.pose()
        ne = ns = 0
        if r.update_type and world > 1:                               # the payload the other streams append
            ne = ctx.copy_features_into(_lib.EDGE, fbuf[:cap])
            ns = ctx.copy_features_into(_lib.SURF, fbuf[cap:])
        t = mark("copy_features", t)
        tx = time.perf_counter()
        kfs = xchg.exchange(P, r.update_type, ne, ns, fbuf)           # same list, same order everywhere
        state["xchg_s"] += time.perf_counter() - tx
        t = mark("exchange", t)
        for q, fe, fs, pose in kfs:
            if q == rank:                                             # own keyframe: from the context, no copies
                tr.add_keyframe_extracted(pose)
            else:
                tr.add_keyframe(fe, fs, pose)
        t = mark("add_keyframe", t)
        if kfs:
            tr.commit_map()
            state["kf"] += len(kfs)
        t = mark("commit", t)
        Tt = np.eye(4)
        Tt[:3, :3] = synth.quat_to_mat(truth[i][:4])
        Tt[:3, 3] = truth[i][4:]
        state["err"].append(float(np.linalg.norm(P[:3, 3] - Tt[:3, 3])))
        state["poses"].append(P.copy())
        state["types"].append(int(r.update_type))
        state["i"] += 1
        return P

    elapsed, _, mean_n27 = timed(d, step, args.warmup, args.steps, [ctx], not args.no_n27)
    if args.dump:   # every step of this rank, warm-up included (the stream from its first scan)
        os.makedirs(args.dump, exist_ok=True)
        np.savez(os.path.join(args.dump, f"c4_rank{rank}.npz"), poses=np.stack(state["poses"]),
                 types=np.asarray(state["types"]), world=world, cols=args.cols, map_points=args.map_points,
                 outer=args.outer)
    if phases is not None:
        nst = state["i"]
        print("phases ms/step: " + "  ".join(f"{k} {1e3 * v / nst:.3f}" for k, v in phases.items()), file=sys.stderr)
    ks = timed_stats(ctx)
    pose_dv = None
    roof = knn_roofline(ks, mean_n27, load_traffic(args.traffic_json, config="C4", batch=1, map_points=map_points),
                        elapsed, "one 63k-query scan per launch (8 lanes per query): latency-bound launches")
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        oracle = cpu_oracle()
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import tracker as OT
        ot = OT.Tracker(manual_map_update=True)
        ot.origin = T0.copy()
        ot.reg.set_fixed_schedule(True)
        ot.reg.set_max_iterations(args.outer)
        ot.set_prior_map(1, em_t.cpu().numpy())      # the same broadcast map
        ot.set_prior_map(2, sm_t.cpu().numpy())
        n_done = 0
        worst = [0.0, 0.0]
        t1 = time.perf_counter()
        while n_done < n and (n_done == 0 or time.perf_counter() - t1 < args.cpu_seconds):
            e, s, _, _ = oracle.extract(scans[n_done])
            _, typ, _ = ot.solve(e, s, 0.1 * n_done)
            if typ:
                ot.add_keyframe(e, s, ot.curr)
                ot.commit()
            dt, dr = mat_delta(state["poses"][n_done], ot.curr)   # the GPU tracker's pose of the same scan
            worst = [max(worst[0], dt), max(worst[1], dr)]
            n_done += 1
        cpu_el = time.perf_counter() - t1
        pose_dv = {"scans": n_done, "max_m": worst[0], "max_rad": worst[1]}
        cpu = {"value": round(n_done / cpu_el, 3), "unit": "scans/s", "cores": 1, "kind": "port",
               "cpu_model": host_cpu()[0],
               "sample": f"first {n_done} scans of the rank-0 stream (extract + tracker Solve with "
                         f"{args.outer} outer iterations + keyframe map rebuild incl. kd-tree over the 5M prior), "
                         f"{cpu_el:.1f} s on 1 thread of {os.cpu_count()} host cores"}
    if rank == 0:
        line(args, d, "LiDAR scans/sec tracked (64k-pt scan streams, shared 5M-pt map, one stream per GPU)",
             world * args.steps / elapsed, "scans/s", elapsed, "weak",
             f"C4: one VLP-16 16x{args.cols} stream per GPU (8 m/s, 10 Hz) tracked against a {map_points}-pt "
             f"shared map + stitched keyframe window (10 keyframes, voxel 0.2/0.4 m), {args.outer} outer iters",
             {"streams": world, "map_points": map_points, "outer_iterations": args.outer,
              "parallelism": f"stream-per-GPU x{world}", "extract_ahead": not args.no_prefetch}, roof, cpu,
             tracking_error_m={"rank0_max": max(state["err"]), "rank0_last": state["err"][-1]},
             keyframes_appended=state["kf"],
             # host time in the keyframe exchange per scan (the collectives at world > 1), over all steps run
             keyframe_exchange_ms_per_step=round(1e3 * state["xchg_s"] / max(state["i"], 1), 4),
             keyframe_payload_bytes_per_step=int(xchg.payload_bytes / max(xchg.steps, 1)),
             **({"pose_delta_vs_cpu": pose_dv} if cpu is not None else {}))
    tr.close()
    ctx.close()


# ----------------------------------------------------------------------------- C3: dual-LiDAR online refine
def run_dual(args, d):
    import numpy as np
    d.init()
    torch = d.torch
    from lmsf import _lib, dual, synth
    world, rank = d.world, d.rank
    n = args.warmup + args.steps
    ds = synth.make_dual_sequence(n, n_cols=args.cols, step=0.5, start_x=8.0 * rank if world <= 8 else 64.0 * rank / world)

    def mat(p):
        T = np.eye(4)
        T[:3, :3] = synth.quat_to_mat(p[:4])
        T[:3, 3] = p[4:]
        return T

    X = mat(ds.extrinsic)
    X0 = X @ mat(np.concatenate([synth.axis_angle_quat(np.radians([0.5, -0.5, 0.5])), [0.03, -0.02, 0.02]]))
    prim_dev = [torch.from_numpy(s).to(d.dev) for s in ds.primary]
    sub_dev = [torch.from_numpy(s).to(d.dev) for s in ds.sub]
    max_pts = max(max(len(s) for s in ds.primary), max(len(s) for s in ds.sub))
    ctx = _lib.Context(device=d.gpu, max_batch=1, max_scan_points=max_pts + 64, max_features=max_pts + 64)
    apply_options(args, [ctx])
    system = dual.DualLidarSystem(ctx, extrinsic=X0, keyframe_lookahead=not args.no_lookahead)
    state = {"i": 0, "poses": []}

    def step():
        i = state["i"]
        nxt = (prim_dev[i + 1], sub_dev[i + 1]) if not args.no_prefetch and i + 1 < len(prim_dev) else None
        out = system.process(prim_dev[i], sub_dev[i], 0.1 * i, next_frame=nxt)
        state["poses"].append((out[0].copy(), out[1].copy()))
        state["i"] += 1
        return out

    elapsed, _, mean_n27 = timed(d, step, args.warmup, args.steps, [ctx], not args.no_n27)
    ks = timed_stats(ctx)
    pose_dv = None
    roof = knn_roofline(ks, mean_n27, load_traffic(args.traffic_json, config="C3", batch=1), elapsed,
                        "one ~63k-query scan per launch (8 lanes per query) against the voxelised local map: "
                        "latency-bound launches")
    ext_err = [float(np.linalg.norm(system.extrinsic[:3, 3] - X[:3, 3])),
               synth.rot_angle_of_matrix(system.extrinsic[:3, :3].T @ X[:3, :3])]
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        oracle = cpu_oracle()
        sys.path.insert(0, os.path.join(REPO, "oracle"))
        import tracker as OT
        ot = OT.Tracker()
        ext = X0.copy()
        n_done = 0
        worst = [0.0, 0.0]
        t1 = time.perf_counter()
        while n_done < n and (n_done == 0 or time.perf_counter() - t1 < args.cpu_seconds):
            ep, sp, _, _ = oracle.extract(ds.primary[n_done])
            es, ss, _, _ = oracle.extract(ds.sub[n_done])
            ot.solve(ep, sp, 0.1 * n_done)
            prim = ot.curr.copy()
            sub, _ = ot._register({1: es, 2: ss}, dual.iso_mul(prim, ext))
            ext = dual.iso_mul(dual.iso_inv(prim), sub)
            for g, o in zip(state["poses"][n_done], (prim, sub)):   # the GPU's primary and refined sub poses
                dt, dr = mat_delta(g, o)
                worst = [max(worst[0], dt), max(worst[1], dr)]
            n_done += 1
        cpu_el = time.perf_counter() - t1
        pose_dv = {"frames": n_done, "max_m": worst[0], "max_rad": worst[1]}
        cpu = {"value": round(n_done / cpu_el, 3), "unit": "frames/s", "cores": 1, "kind": "port",
               "cpu_model": host_cpu()[0],
               "sample": f"first {n_done} frames of the same dual-LiDAR sequence (2 extractions, tracker Solve, "
                         f"sub-LiDAR refine, keyframe map rebuild), {cpu_el:.1f} s on 1 thread of "
                         f"{os.cpu_count()} host cores"}
    if rank == 0:
        npts = int(np.mean([len(s) for s in ds.primary]))
        line(args, d, "dual-LiDAR frames/sec (2x64k-pt scans, tracking + online extrinsic refine)",
             world * args.steps / elapsed, "frames/s", elapsed, "weak",
             f"C3: two VLP-16 16x{args.cols} LiDARs (~{npts} pts each) at the PS-Calib extrinsic, primary "
             f"tracking (reference decay schedule) + sub-LiDAR refine against the voxelised 10-keyframe local map",
             {"systems": world, "parallelism": f"system-per-GPU x{world}", "extract_ahead": not args.no_prefetch},
             roof, cpu,
             extrinsic_error={"m": ext_err[0], "rad": ext_err[1]},
             **({"pose_delta_vs_cpu": pose_dv} if cpu is not None else {}))
    system.close()
    ctx.close()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.workers is None:
        args.workers = max(1, min(16, (host_cpu()[1] or 1)))
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return launch_ranks(argv, args.gpus)          # before anything touches the GPU
    d = Dist(args.dist_backend, args.dist_impl)
    if d.world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={d.world}", file=sys.stderr)
        return 3
    if args.launch_check:
        d.init()
        rc = run_launch_check(args, d)
        d.close()
        return rc
    {"C2": run_batch, "C5": run_batch, "C4": run_streams, "C3": run_dual}[args.config](args, d)
    d.close()
    return 0


if __name__ == "__main__":
    sys.exit(main())
