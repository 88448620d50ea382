"""Per-kernel summary of one rocprofv3 --pmc pass: kernel,counter,dispatches,total,per_dispatch.

Usage: python tools/pmc_summary.py <pmc_dir> <out.csv>
"""
import csv
import glob
import sys


def main():
    d, out = sys.argv[1:3]
    f = glob.glob(f"{d}/*counter_collection.csv")[0]
    acc = {}
    for r in csv.DictReader(open(f)):
        k = (r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0], r["Counter_Name"])
        disp, tot = acc.get(k, (set(), 0.0))
        disp.add(r["Dispatch_Id"])
        acc[k] = (disp, tot + float(r["Counter_Value"]))
    with open(out, "w") as fo:
        fo.write("kernel,counter,dispatches,total,per_dispatch\n")
        for (kern, ctr), (disp, tot) in sorted(acc.items()):
            fo.write(f"{kern},{ctr},{len(disp)},{tot:.0f},{tot / len(disp):.1f}\n")


if __name__ == "__main__":
    main()
