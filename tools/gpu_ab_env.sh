# Parity tests, then alternating A/B of environment settings: ENVS="A=1 A=0" (one word per variant,
# comma-separated assignments inside a word), REPS rounds of bench.py --config CONFIG.
set -u
cd "$GRAFT_REPO_ROOT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread ${TESTS} ${TESTK:+-k "$TESTK"} > gpurun_out/ab_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/ab_tests.log
  case $rc in 0) ;; *) exit $rc;; esac
fi
for r in $(seq 1 ${REPS:-2}); do
  for v in ${ENVS}; do
    tag=$(echo $v | tr ',=' '__')
    env $(echo $v | tr ',' ' ') timeout -k 10 300 python bench.py --config ${CONFIG:-C2} --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab_${tag}_$r.log 2>&1
    rc=$?; echo "$v $r rc=$rc $(tail -1 gpurun_out/ab_${tag}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["roofline"]["avg_launch_ms"])' 2>/dev/null)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
