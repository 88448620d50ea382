set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "extract or prefetch or ingest or c1 or smoke" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
NO_TESTS=1 VARIANTS="x00 x11" CFG=C5 OUT=xtrace5 bash tools/gpu_trace_variants.sh || exit $?
NO_TESTS=1 VARIANTS="x00 x11" CFG=C2 OUT=xtrace2 bash tools/gpu_trace_variants.sh || exit $?
ROUNDS=1 CONFIGS="C5 C2" VARIANTS="x00 x11" bash tools/gpu_ab_lib.sh || exit $?
