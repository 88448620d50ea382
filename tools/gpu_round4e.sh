# r04: wave-cooperative LM control -- GPU suite, phase timing (stepprof), one-stream kernel trace, A/B vs the
# one-lane LDS form (mode2) and 256-thread lm_step (st256) on C2, C3 / C4 (single-scan loop) A/B.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
LMSF_LIB=lmsf-slam_amd/ab/liblmsf_stepprof.so timeout -k 10 300 python bench.py --config C2 --no-cpu --h2d off --streams 1 --batch 128 --steps 2 --warmup 1 > gpurun_out/stepprof.log 2>&1
rc=$?; echo "stepprof_rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
mkdir -p gpurun_out/ctltrace
for v in cur mode2; do
  LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ctltrace/$v -o run -- python3 bench.py --config C2 --no-cpu --h2d off --streams 1 --batch 128 --steps 2 --warmup 1 > gpurun_out/ctltrace/$v.log 2>&1
  rc=$?; echo "trace $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
CONFIGS=C2 VARIANTS="cur mode2 st256" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
CONFIGS="C4 C3" VARIANTS="cur mode2" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
