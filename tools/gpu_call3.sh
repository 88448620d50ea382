# GPU tests (subset by -k), then C4 / C3 benches alternating bench.py argument sets (ARGSETS, ';'-separated),
# then a C4 kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "${TESTS:-voxel or tracker or keyframe or dual or local_map or common or prefetch or extract}" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
IFS=';' read -ra SETS <<< "${ARGSETS:- ;--no-prefetch}"
for r in ${ROUNDS:-1 2}; do
  for cfg in ${CFGS:-C4 C3}; do
    j=0
    for a in "${SETS[@]}"; do
      j=$((j+1))
      LMSF_BENCH_PHASES=1 timeout -k 10 300 python bench.py --config $cfg --no-cpu $a > gpurun_out/w_${cfg}_${j}_r$r.json 2> gpurun_out/w_${cfg}_${j}_r$r.err
      rc=$?; echo "$cfg [$a] r$r rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/w_${cfg}_${j}_r$r.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null) $(grep phases gpurun_out/w_${cfg}_${j}_r$r.err)"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
[ -n "${NO_TRACE:-}" ] && exit 0
mkdir -p gpurun_out/r03 && cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/r03/trace_C4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --config C4 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/r03/trace_C4.json" 2>&1; echo "trace rc=$?"
