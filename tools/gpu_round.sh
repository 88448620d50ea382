# One GPU call: the -m gpu suite, smoke, then bench lines of the configurations named in CFGS (default: C2 C5),
# each step under its own limit, stopping at the first failure.  Logs under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "${NO_TESTS:-}" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -rs --timeout 300 --timeout-method thread \
  ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -1 gpurun_out/smoke.log
case $rc in 0) ;; *) exit $rc;; esac
fi
for cfg in ${CFGS:-C2 C5}; do
  timeout -k 10 600 python bench.py --config $cfg ${BENCH_ARGS:-} > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err
  rc=$?; echo "bench_${cfg}_rc=$rc"; tail -c 400 gpurun_out/bench_$cfg.json
  case $rc in 0) ;; *) exit $rc;; esac
done
