# r04 closing check at HEAD: GPU suite, smoke, the default bench line (C2).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final2
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/final2/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/final2/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final2/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -2 gpurun_out/final2/smoke.log; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 400 python -u bench.py > gpurun_out/final2/bench_C2.json 2> gpurun_out/final2/bench_C2.err
rc=$?; echo "bench C2 rc=$rc"; tail -c 300 gpurun_out/final2/bench_C2.json; echo
