# Alternating A/B of variant libraries (lmsf-slam_amd/ab/liblmsf_<v>.so), REPS rounds, one bench per run.
set -u
cd "$GRAFT_REPO_ROOT"
for r in $(seq 1 ${REPS:-2}); do
  for v in ${VARIANTS:-base}; do
    for cfg in ${CONFIGS:-C2}; do
      LMSF_LIB=$PWD/lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 python bench.py --config $cfg --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab_${v}_${cfg}_$r.log 2>&1
      rc=$?; echo "$v $cfg $r rc=$rc $(tail -1 gpurun_out/ab_${v}_${cfg}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_ms"])' 2>/dev/null)"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
