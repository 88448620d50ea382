"""One step of a rocprofv3 kernel trace (run_kernel_trace.csv) as a timeline: per dispatch its start
offset, gap before it and duration (us).  usage: timeline.py TRACE FIRST_KERNEL [STEP_INDEX]
(a step starts at each dispatch whose name contains FIRST_KERNEL; default: the 10th from the end)."""
import csv
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").split("::")[-1][:48]


rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
k = int(sys.argv[3]) if len(sys.argv) > 3 else -10
a, b = starts[k], starts[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
prev_end = t0
busy = 0
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    busy += e - s
    print(f"{(s - t0) / 1e3:9.1f} gap {(s - prev_end) / 1e3:7.1f} dur {(e - s) / 1e3:7.1f}  {short(r['Kernel_Name'])}")
    prev_end = max(prev_end, e)
print(f"step {(int(rows[b]['Start_Timestamp']) - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, {b - a} dispatches")
