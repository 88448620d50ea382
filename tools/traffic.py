"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes (MI355X_MICROARCH.md §HBM):

  bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024      (FETCH_SIZE reads 1/2 of 128-B requests on gfx950)

The FETCH_SIZE pass also carries --kernel-trace: the kernel's mean duration in that same run is kept
as rocprof_mean_us, so bench.py's roofline can be recomputed from the committed files alone.

Usage: python tools/traffic.py <fetch_dir> <write_dir> <hitmiss_dir> <kernels> <out.json> [k=v ...]
       kernels: comma-separated name substrings of the kernels one "launch" (one outer iteration of the
       neighbour search) runs, the first naming the kernel that runs exactly once per launch (e.g.
       match_fit_kernel,match_memo_kernel: the memo pass runs in outer iterations > 0 only); per-launch
       figures = sums over all their dispatches / dispatches of the first ("a|b": either name counts: the tracking
       search's outer iterations are knn_kernel<..., 0> launches, iteration 0 a prior pass <..., 1> beside the
       keyframe rebuild and a window pass <..., 2>, counted once).
       (k=v: the workload the passes ran -- config, batch, streams, map_points, unique_scans, profile)
"""
import csv
import glob
import json
import sys


def counter_rows(d):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    return list(csv.DictReader(open(f)))


def per_launch(d, kernels, counter):
    """(sum of `counter` over the dispatches of every kernel in `kernels`, dispatches of kernels[0])."""
    tot, first = 0.0, set()
    for r in counter_rows(d):
        if r["Counter_Name"] != counter or not any(k in r["Kernel_Name"] for k in kernels):
            continue
        tot += float(r["Counter_Value"])
        if any(k in r["Kernel_Name"] for k in kernels[0].split("|")):
            first.add(r["Dispatch_Id"])
    return tot, len(first)


def mean_duration_us(d, kernels):
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not files:
        return None
    tot, n = 0, 0
    for r in csv.DictReader(open(files[0])):
        if any(k in r["Kernel_Name"] for k in kernels):
            tot += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            n += any(k in r["Kernel_Name"] for k in kernels[0].split("|"))
    return tot / n / 1e3 if n else None


def main():
    fetch_dir, write_dir, hm_dir, kernel_list, out = sys.argv[1:6]
    kernels = kernel_list.split(",")
    extra = dict(a.split("=", 1) for a in sys.argv[6:])
    fe, n_fe = per_launch(fetch_dir, kernels, "FETCH_SIZE")
    wr, n_wr = per_launch(write_dir, kernels, "WRITE_SIZE")
    hit, _ = per_launch(hm_dir, kernels, "TCC_HIT_sum")
    miss, _ = per_launch(hm_dir, kernels, "TCC_MISS_sum")
    fetch_kb, write_kb = fe / n_fe, wr / n_wr
    res = {
        "kernel": kernel_list,
        "dispatches": n_fe,
        "fetch_size_kb_per_launch": fetch_kb,
        "write_size_kb_per_launch": write_kb,
        "hbm_bytes_per_launch": int((2 * fetch_kb + write_kb) * 1024),
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts 128-B requests at 64 B)",
        "l2_hit_rate": hit / max(hit + miss, 1.0),
        "rocprof_mean_us": mean_duration_us(fetch_dir, kernels),
    }
    for k, v in extra.items():
        res[k] = int(v) if v.isdigit() else v
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
