"""Per-launch HBM traffic of a kernel from rocprofv3 PMC passes (MI355X_MICROARCH.md §HBM):

  bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024      (FETCH_SIZE reads 1/2 of 128-B requests on gfx950)

The FETCH_SIZE pass also carries --kernel-trace: the kernel's mean duration in that same run is kept
as rocprof_mean_us, so bench.py's roofline can be recomputed from the committed files alone.

Usage: python tools/traffic.py <fetch_dir> <write_dir> <hitmiss_dir> <kernel-substring> <out.json> [k=v ...]
       (k=v: the workload the passes ran -- config, batch, streams, map_points, unique_scans, profile)
"""
import csv
import glob
import json
import sys


def per_dispatch(d, kernel):
    f = glob.glob(f"{d}/**/*counter_collection.csv", recursive=True)[0]
    vals = {}
    for r in csv.DictReader(open(f)):
        if kernel in r["Kernel_Name"]:
            key = (r["Dispatch_Id"], r["Counter_Name"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (disp, name), v in vals.items():
        out.setdefault(name, []).append(v)
    return out


def mean_duration_us(d, kernel):
    files = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not files:
        return None
    durs = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(files[0]))
            if kernel in r["Kernel_Name"]]
    return sum(durs) / len(durs) / 1e3 if durs else None


def main():
    fetch_dir, write_dir, hm_dir, kernel, out = sys.argv[1:6]
    extra = dict(a.split("=", 1) for a in sys.argv[6:])
    fe = per_dispatch(fetch_dir, kernel)["FETCH_SIZE"]
    wr = per_dispatch(write_dir, kernel)["WRITE_SIZE"]
    hm = per_dispatch(hm_dir, kernel)
    fetch_kb = sum(fe) / len(fe)
    write_kb = sum(wr) / len(wr)
    hit, miss = sum(hm["TCC_HIT_sum"]), sum(hm["TCC_MISS_sum"])
    res = {
        "kernel": kernel,
        "dispatches": len(fe),
        "fetch_size_kb_per_launch": fetch_kb,
        "write_size_kb_per_launch": write_kb,
        "hbm_bytes_per_launch": int((2 * fetch_kb + write_kb) * 1024),
        "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE counts 128-B requests at 64 B)",
        "l2_hit_rate": hit / max(hit + miss, 1.0),
        "rocprof_mean_us": mean_duration_us(fetch_dir, kernel),
    }
    for k, v in extra.items():
        res[k] = int(v) if v.isdigit() else v
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
