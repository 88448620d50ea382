"""Per-kernel duration medians of a rocprofv3 kernel trace directory: probe_stats.py DIR"""
import collections
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("lmsf::", "").split("(")[0][-28:]
    agg[(n, r["Grid_Size_X"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items()):
    v = sorted(v)
    print(f"{k[0]:30s} {k[1]:>8s} n={len(v):3d} med={v[len(v) // 2]:7.1f} min={v[0]:7.1f}")
