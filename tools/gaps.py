"""Inter-kernel gaps of a rocprofv3 kernel trace (run_kernel_trace.csv): where the stream idles.
usage: gaps.py TRACE [FRACTION_FROM]  (default: the last 40% of dispatches, i.e. the timed steps)"""
import collections
import csv
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").split("::")[-1][:34]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
rows = rows[int(len(rows) * (float(sys.argv[2]) if len(sys.argv) > 2 else 0.6)):]
gaps, cnt = collections.defaultdict(float), collections.Counter()
tot_gap = 0
for a, b in zip(rows, rows[1:]):
    g = int(b["Start_Timestamp"]) - int(a["End_Timestamp"])
    if g > 0:
        k = (short(a["Kernel_Name"]), short(b["Kernel_Name"]))
        gaps[k] += g
        cnt[k] += 1
        tot_gap += g
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
span = int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])
print(f"span {span / 1e6:.3f} ms  kernels {busy / 1e6:.3f} ms  gaps {tot_gap / 1e6:.3f} ms")
for k, v in sorted(gaps.items(), key=lambda x: -x[1])[:20]:
    print(f"{v / 1e6:8.3f} ms {cnt[k]:5d} x {v / cnt[k] / 1e3:7.1f} us  {k[0]} -> {k[1]}")
