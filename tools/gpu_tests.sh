# GPU test suite, smoke and the default bench line on the box (each step under its own limit; stop at the
# first failure).  Logs under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -rs --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
[ -n "${NO_BENCH:-}" ] && exit 0
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench_rc=$rc"; tail -c 600 gpurun_out/bench_default.log
