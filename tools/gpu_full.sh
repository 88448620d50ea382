# Full round check: GPU parity suite, smoke, every bench configuration (with CPU baselines).
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
for cfg in C2 C3 C4 C5; do
  timeout -k 10 900 python bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
