"""Summarise a rocprofv3 kernel_stats.csv: name, calls, avg us, total ms, share."""
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Name"].split("(")[0].replace("void ", "")[:48]
    print(f"{n:48s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:10.1f}us {float(r['TotalDurationNs'])/1e6:9.3f}ms {float(r['Percentage']):6.2f}%")
