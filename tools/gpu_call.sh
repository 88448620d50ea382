set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "batch_run_matches or c2_fullsize or memo_dense or streamed" > gpurun_out/gpu_tests2.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests2.log; case $rc in 0) ;; *) exit $rc;; esac
OPTS="- MEMO_BOUND=2" ROUNDS=2 bash tools/gpu_ab_opts.sh
