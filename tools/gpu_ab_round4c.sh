set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
CONFIGS=C5 VARIANTS="p2fine p2coarse sy4 nosplit" ROUNDS=1 bash tools/gpu_ab_lib.sh || exit $?
