set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rs > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1
echo "bench_rc=$?"
