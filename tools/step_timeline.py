"""One tracking step of a rocprofv3 kernel trace (run_kernel_trace.csv under DIR) as a timeline with queues, and
the step periods: step_timeline.py DIR [FIRST_KERNEL] [STEP]   (diagnostics: the C4 / C3 latency breakdown)"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
first = sys.argv[2] if len(sys.argv) > 2 else "ring_count_kernel"
k = int(sys.argv[3]) if len(sys.argv) > 3 else -6
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))


def short(n):
    n = n.replace("(anonymous namespace)::", "").replace("void ", "").replace("lmsf::", "")
    return n.split("(")[0][:34]


starts = [i for i, r in enumerate(rows) if first in r["Kernel_Name"]]
a, b = starts[k], starts[k + 1]
t0 = int(rows[a]["Start_Timestamp"])
for r in rows[a:b]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} q{r['Queue_Id']:>3} {(e - s) / 1e3:6.1f} {short(r['Kernel_Name'])} {r['Grid_Size_X']}")
print("step", (int(rows[b]["Start_Timestamp"]) - t0) / 1e3)
print("step periods", [round((int(rows[starts[i + 1]]["Start_Timestamp"]) - int(rows[starts[i]]["Start_Timestamp"])) / 1e3)
                       for i in range(len(starts) - 1)])
