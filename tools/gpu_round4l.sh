# r04: memo lists by block atomics -- GPU suite, one-stream kernel traces, C2 A/B.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
mkdir -p gpurun_out/c2list2
for v in cur noatomic; do
  LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2list2/$v -o run --output-format csv -- python3 bench.py --config C2 --no-cpu --h2d off --streams 1 --batch 128 --steps 2 --warmup 1 > gpurun_out/c2list2/$v.json 2> gpurun_out/c2list2/$v.err
  rc=$?; echo "trace $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
CONFIGS=C2 VARIANTS="cur noatomic" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
