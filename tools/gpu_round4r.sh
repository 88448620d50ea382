# r04: buffer growth made stream-safe (voxel look-back scratch zeroed on its stream, device drained before growth
# frees) -- GPU suite, then the C4 / C3 profiles with the commit worker threads (the form that faulted under
# rocprofv3's PMC passes), the single-scan loop and extract-ahead as the bench runs them.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
ROUND=r04w CFGS="C4 C3" PMC_TIMEOUT=150 bash tools/gpu_profiles.sh || exit $?
