"""Per outer iteration of the batch search: the memo pass and match_fit_kernel durations of each launch in
a one-stream rocprofv3 kernel trace (the PMC FETCH_SIZE pass), in dispatch order -- which outer iterations
cost what.  usage: iter_durations.py TRACE_DIR > out.csv"""
import csv
import glob
import sys

f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
print("launch,memo_us,fit_us,fit_variant,grid")
memo = None
k = 0
for r in rows:
    n = r["Kernel_Name"]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if "match_memo_kernel" in n:
        memo = d
    elif "match_fit_kernel" in n:
        var = n.split("<")[1].split(">")[0].replace(" ", "") if "<" in n else ""
        print(f"{k},{memo if memo is not None else 0:.1f},{d:.1f},{var},{r.get('Grid_Size_X', '')}")
        memo = None
        k += 1
