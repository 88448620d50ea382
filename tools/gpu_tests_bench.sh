# GPU parity suite, then the tracking configurations.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
for cfg in ${CONFIGS:-C2 C3 C4}; do
  timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
