set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2 3; do
  for cfg in C4 C3; do
    LMSF_BENCH_PHASES=1 timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/w_${cfg}_r$r.json 2> gpurun_out/w_${cfg}_r$r.err
    rc=$?; echo "$cfg r$r rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/w_${cfg}_r$r.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null) $(grep phases gpurun_out/w_${cfg}_r$r.err)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
