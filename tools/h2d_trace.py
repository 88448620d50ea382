"""H2D copies against the kernels of a rocprofv3 trace (tools/profile_h2d.sh): per large host-to-device copy
its start, duration, bytes and rate, the kernels of the same stream/queue around it, and per step how
much of the copy time overlapped kernel execution.  usage: h2d_trace.py TRACE_DIR [MIN_MB]"""
import csv
import glob
import os
import sys


def load(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


d = sys.argv[1]
min_bytes = float(sys.argv[2] if len(sys.argv) > 2 else 16) * 2 ** 20
kern = load(os.path.join(d, "**", "*kernel_trace.csv"))
copies = load(os.path.join(d, "**", "*memory_copy_trace.csv"))
if not copies:
    sys.exit(f"no memory_copy_trace.csv under {d}")
cols = list(copies[0].keys())
print("copy columns:", cols)
bkey = next(k for k in cols if "Size" in k or "Bytes" in k)
dkey = next(k for k in cols if k.lower() in ("direction", "kind", "operation")) if any(
    k.lower() in ("direction", "kind", "operation") for k in cols) else None
big = [c for c in copies if float(c[bkey]) >= min_bytes]
big.sort(key=lambda c: int(c["Start_Timestamp"]))
ks = sorted(((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"]) for k in kern))
if not big:
    sys.exit("no copy above the size threshold")
t0 = int(big[0]["Start_Timestamp"])
tot_b = tot_t = 0.0
for c in big:
    s, e, nb = int(c["Start_Timestamp"]), int(c["End_Timestamp"]), float(c[bkey])
    busy = 0   # kernel time overlapping this copy (union not needed for the ratio's sense: clipped sum)
    for a, b, _ in ks:
        if b <= s or a >= e:
            continue
        busy += min(b, e) - max(a, s)
    tot_b += nb
    tot_t += e - s
    print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:8.1f} us  {nb / 2**20:7.1f} MiB  {nb / max(e - s, 1):6.2f} GB/s  "
          f"kernel-time overlapped {busy / 1e3:9.1f} us  {c.get(dkey, '') if dkey else ''}")
print(f"{len(big)} copies, {tot_b / 2**20:.0f} MiB, mean rate {tot_b / max(tot_t, 1):.2f} GB/s (per copy, concurrent copies "
      f"share the link)")
span = int(big[-1]["End_Timestamp"]) - t0
print(f"first copy start -> last copy end {span / 1e3:.1f} us: {tot_b / max(span, 1):.2f} GB/s aggregate")
