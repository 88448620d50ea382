# Tracking iteration: GPU tests, C4 with per-phase host times, C3, then a C4 kernel trace.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -1 gpurun_out/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
LMSF_BENCH_PHASES=1 timeout -k 10 300 python bench.py --config C4 --no-cpu > gpurun_out/c4p.log 2>&1 || exit $?
LMSF_SPIN_SYNC=0 timeout -k 10 300 python bench.py --config C4 --no-cpu > gpurun_out/c4_nospin.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --config C3 --no-cpu > gpurun_out/c3.log 2>&1 || exit $?
CONFIGS=C4 bash tools/profile_tracking.sh
