#!/bin/bash
# Package one configuration's gpurun_out profile directory (tools/profile.sh output) into
# profiles/<round>/<CFG>/ and profiles/traffic_<CFG>.json:
#   tools/package_profiles.sh <src dir> <CFG> <round> <k=v ...>   (k=v: the PMC passes' workload)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
S=$1; CFG=$2; RND=$3; shift 3
O=$R/profiles/$RND/$CFG
mkdir -p $O
cp $S/trace/run_kernel_stats.csv $O/kernel_stats.csv
python3 $R/tools/kstats.py $O/kernel_stats.csv > $O/kernel_stats.txt
python3 $R/tools/gaps.py $S/trace/run_kernel_trace.csv > $O/gaps.txt
tail -1 $S/trace_bench.json > $O/bench_under_rocprof.json
for t in FETCH_SIZE WRITE_SIZE TCC_HIT_sum SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU; do
  [ -d $S/pmc_$t ] || continue
  d=$(dirname $(find $S/pmc_$t -name "*counter_collection.csv" | head -1))
  python3 $R/tools/pmc_summary.py $d $O/pmc_${t}_summary.csv
  tail -1 $S/pmc_$t.json > $O/pmc_${t}_bench.json
done
# per-kernel durations of the FETCH pass (the run the traffic figures come from)
python3 - $S/pmc_FETCH_SIZE $O/pmc_durations.csv <<'PY'
import collections, csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_trace.csv", recursive=True)[0]
agg = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    agg[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
with open(sys.argv[2], "w") as fo:
    fo.write("kernel,dispatches,mean_us,total_us\n")
    for k, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        fo.write(f"{k},{len(v)},{sum(v) / len(v) / 1e3:.1f},{sum(v) / 1e3:.1f}\n")
PY
python3 $R/tools/iter_durations.py $S/pmc_FETCH_SIZE > $O/pmc_iter_durations.csv
python3 $R/tools/traffic.py $S/pmc_FETCH_SIZE $S/pmc_WRITE_SIZE $S/pmc_TCC_HIT_sum "${KERNELS:-match_fit_kernel,match_memo_kernel}" $R/profiles/traffic_$CFG.json config=$CFG profile=profiles/$RND/$CFG round=${RND#r} "$@" > /dev/null
[ -d $S/pmc_SQ_ACTIVE_INST_VALU ] && python3 $R/tools/valu_busy.py $O > $O/valu_busy.txt
echo "packaged $CFG -> $O"
