set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "voxel or tracker or keyframe or dual or local_map or common" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
MODES=0 bash tools/gpu_probe.sh
