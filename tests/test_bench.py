"""bench.py host logic on CPU: the --gpus N launcher (torch.distributed.run as a child process, the
ranks' world-size check, the C2 pose all-gather over gloo) and the roofline arithmetic."""
import json
import os
import subprocess
import sys
import types

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env=None, timeout=180):
    e = dict(os.environ)
    e.pop("WORLD_SIZE", None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True, timeout=timeout, env=e)


@pytest.mark.parametrize("impl,expect", [("auto", "c-transport"), ("torch", "torch")])
def test_gpus2_launches_two_ranks_and_gathers(impl, expect):
    """The launcher's ranks run the C2 pose all-gather and the max-over-ranks through the shipped C library
    (--dist-impl auto = c: liblmsf_dist.so's protocol, here over gloo host collectives; RCCL on the nccl backend)
    or torch.distributed; the line names which."""
    r = _run(["--gpus", "2", "--launch-check", "--dist-backend", "gloo", "--dist-impl", impl])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1                       # rank 0 only
    assert lines[0]["n_gpus"] == 2 and lines[0]["gather_ok"] is True and lines[0]["dist_impl"] == expect


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--launch-check", "--dist-backend", "gloo"], env={"WORLD_SIZE": "1"})
    assert r.returncode == 3 and "WORLD_SIZE=1" in r.stderr


def test_child_return_code_propagates():
    r = _run(["--gpus", "2", "--launch-check", "--dist-backend", "no-such-backend"])
    assert r.returncode != 0


def _bench_module():
    sys.path.insert(0, REPO)
    import bench
    return bench


def test_roofline_measured_and_model():
    bench = _bench_module()
    ks = types.SimpleNamespace(launches=10, total_ms=10.0, queries=1_000_000, reused_queries=400_000,
                               fused_launches=10, n27_sum=0)
    tj = {"hbm_bytes_per_launch": 1_000_000_000, "l2_hit_rate": 0.75, "rocprof_mean_us": 800.0,
          "profile": "profiles/x", "dispatches": 3}
    r = bench.knn_roofline(ks, 50.0, tj, 0.02, "n")
    # 1 GB per 1 ms launch = 1000 GB/s; rocprof: 1 GB / 0.8 ms
    assert r["basis"].startswith("pmc") and r["achieved"] == 1000.0 and r["frac"] == 0.125
    assert abs(r["rocprof"]["frac"] - 1e9 / 0.8e-3 / 1e9 / 8000) < 1e-4
    assert r["rocprof"]["live_over_rocprof"] == 1.25 and "concurrent" not in r
    # with a solo pass, achieved / model use its launch spans; the timed (concurrent) spans are reported beside
    solo = types.SimpleNamespace(**dict(vars(ks), total_ms=8.0))
    rs = bench.knn_roofline(ks, 50.0, tj, 0.02, "n", solo=solo)
    assert rs["achieved"] == 1250.0 and rs["avg_launch_ms"] == 0.8 and rs["concurrent"]["avg_launch_ms"] == 1.0
    assert rs["rocprof"]["live_over_rocprof"] == 1.0 and rs["model"]["frac"] == rs["rocprof"]["model_frac"]
    # model over the 600k searched queries per 10 launches + 16 B per reused query
    mb = (600_000 * (16 + 216 + 16 * 50) + 400_000 * 16) / 10
    assert r["model"]["bytes_per_launch"] == int(mb) and r["model"]["searched_queries_per_launch"] == 60_000
    assert r["model"]["exceeds_peak"] is False
    # a model figure above the HBM peak is flagged
    r2 = bench.knn_roofline(types.SimpleNamespace(**dict(vars(ks), total_ms=0.01)), 50.0, None, 0.02, "n")
    assert r2["basis"].startswith("unmeasured") and r2["achieved"] is None and r2["frac"] is None
    assert r2["model"]["exceeds_peak"] is True and r2["traffic"] is None
    assert r2["model"]["valid"] is False and r2["model"]["frac"] is None      # no roofline claim from it
    # a build without search stamps (no launch time): no achieved figure, no division by zero
    r3 = bench.knn_roofline(types.SimpleNamespace(**dict(vars(ks), total_ms=0.0)), 50.0, tj, 0.02, "n")
    assert r3["achieved"] is None and r3["frac"] is None and r3["basis"].startswith("untimed")


def test_roofline_bound_from_committed_valu_pass():
    """the line's `bound` is the roof the committed counters show -- VALU issue for the C2 / C5
    batch searches (busy >= 0.75), latency for the single-scan C3 / C4 launches -- with the VALU pass beside the
    HBM fraction; the 8(d) model is marked invalid once its strict all-query sum exceeds the HBM peak."""
    bench = _bench_module()
    ks = types.SimpleNamespace(launches=10, total_ms=10.0, queries=1_000_000, reused_queries=400_000,
                               fused_launches=10, n27_sum=0)
    for cfg, bound, kernel in (("C2", "valu", "match_fit_kernel"), ("C5", "valu", "dense_pass1_kernel"),
                               ("C4", "latency", "knn_kernel"), ("C3", "latency", "knn_kernel")):
        tj = bench.load_traffic(os.path.join(REPO, "profiles", f"traffic_{cfg}.json"), config=cfg)
        r = bench.knn_roofline(ks, 50.0, tj, 0.02, "n")
        assert r["bound"] == bound and r["valu"]["kernels"][0]["kernel"] == kernel, cfg
        assert r["frac_basis"].startswith("HBM") and r["frac"] is not None
        assert os.path.exists(os.path.join(REPO, r["valu"]["source"]))
    assert bench.binding_roof(None, 0.7) == "hbm" and bench.binding_roof(None, None) == "hbm"
    # slow launches: both 8(d) forms far below the peak, the model stands
    slow = types.SimpleNamespace(**dict(vars(ks), total_ms=1000.0))
    r = bench.knn_roofline(slow, 50.0, None, 0.02, "n")
    assert r["model"]["valid"] is True and r["model"]["strict"]["exceeds_peak"] is False
    # 99% memo reuse: 2.6 MB searched-only per 10-us launch fits, the strict 1M x 1,032 B = 103 MB (10 TB/s) does not
    mid = types.SimpleNamespace(**dict(vars(ks), total_ms=0.1, reused_queries=990_000))
    r = bench.knn_roofline(mid, 50.0, None, 10.0, "n")
    assert r["model"]["exceeds_peak"] is False and r["model"]["strict"]["exceeds_peak"] is True
    assert r["model"]["valid"] is False and r["model"]["frac"] is None and "strict" in r["model"]["invalid_reason"]


def test_load_traffic_matches_workload(tmp_path):
    bench = _bench_module()
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"config": "C2", "batch": 128, "map_points": 10, "hbm_bytes_per_launch": 5}))
    assert bench.load_traffic(str(p), config="C2", batch=128, map_points=10)["hbm_bytes_per_launch"] == 5
    assert bench.load_traffic(str(p), config="C2", batch=64, map_points=10) is None
    assert bench.load_traffic(str(tmp_path / "missing.json"), config="C2") is None


@pytest.mark.parametrize("n_units,chunk,P", [(1000, 125, 1), (1000, 125, 3), (1000, 125, 8), (1000, 125, 9),
                                              (7, 3, 2), (0, 125, 3)])
def test_in_turn_schedule(n_units, chunk, P):
    """C5's pipelined pass (bench.py --pipeline): every unit launched once, a context's launch waited for
    before it is reused and before the pass ends, at most P launches in flight."""
    ev = _bench_module().in_turn(n_units, chunk, P)
    launched, inflight = [], {}
    for kind, ci, a, m in ev:
        assert 0 <= ci < P
        if kind == "launch":
            assert ci not in inflight
            inflight[ci] = (a, m)
            launched.append((a, m))
            assert len(inflight) <= P
        else:
            assert inflight.pop(ci) == (a, m)
    assert not inflight
    covered = sorted(u for a, m in launched for u in range(a, a + m))
    assert covered == list(range(n_units))


def test_kernel_labels_and_cpu_share(monkeypatch):
    """the roofline names the kernels it timed (dense maps: the two first-pass-grid passes and the
    pass-2 fit; sparse batch maps: the memo pass + fused search; tracking: the single-scan search), and the
    multi-thread CPU baseline runs on a stated per-GPU share of the host cores."""
    bench = _bench_module()
    ks = types.SimpleNamespace(launches=10, total_ms=10.0, queries=1000, reused_queries=0, fused_launches=10, n27_sum=0)
    dense = bench.knn_roofline(ks, 50.0, None, 0.02, "n", dense=True)["kernel"]
    assert dense.startswith("dense_pass1_kernel + dense_pass2_kernel + dense_fit2_kernel")
    assert bench.knn_roofline(ks, 50.0, None, 0.02, "n")["kernel"].startswith("match_memo_kernel + match_fit_kernel")
    single = types.SimpleNamespace(**dict(vars(ks), fused_launches=0))
    assert "match_" not in bench.knn_roofline(single, 50.0, None, 0.02, "n")["kernel"]
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench.cpu_share(256) == (16, "OMP_NUM_THREADS=16: the job's per-GPU CPU share")
    assert bench.cpu_share(8)[0] == 8
    monkeypatch.delenv("OMP_NUM_THREADS")
    n, basis = bench.cpu_share(256)
    assert n == 32 and "/ 8 GPUs" in basis


def test_tracking_lines_carry_pose_delta():
    """The C3 / C4 lines report the GPU-vs-CPU pose difference over the frames the CPU baseline tracked
    (pose_delta_vs_cpu), as the C2 / C5 lines do; mat_delta is the 4x4 form of synth.pose_delta."""
    import numpy as np
    bench = _bench_module()
    src = open(BENCH).read()
    for fn in ("def run_streams", "def run_dual"):
        body = src[src.index(fn):]
        body = body[:body.index("\ndef ", 1)]
        assert '"pose_delta_vs_cpu": pose_dv' in body and "mat_delta(" in body, fn
    A = np.eye(4)
    B = np.eye(4)
    B[:3, 3] = (0.0, 3e-5, 4e-5)
    c, s = np.cos(1e-6), np.sin(1e-6)
    B[:2, :2] = [[c, -s], [s, c]]
    dt, dr = bench.mat_delta(A, B)
    assert abs(dt - 5e-5) < 1e-12 and abs(dr - 1e-6) < 1e-12
