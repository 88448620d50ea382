# r04: row tails as straight-line code -- GPU suite, one-stream C2 traces, C2 / C5 A/B.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
mkdir -p gpurun_out/c2tail
for v in cur notail; do
  LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2tail/$v -o run --output-format csv -- python3 bench.py --config C2 --no-cpu --h2d off --streams 1 --batch 128 --steps 2 --warmup 1 > gpurun_out/c2tail/$v.json 2> gpurun_out/c2tail/$v.err
  rc=$?; echo "trace $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
CONFIGS=C2 VARIANTS="cur notail" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
CONFIGS=C5 VARIANTS="cur notail" ROUNDS=1 bash tools/gpu_ab_lib.sh || exit $?
