# r04: listed search on a reduced grid -- GPU suite, one-stream kernel traces, C2 A/B.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
mkdir -p gpurun_out/c2div
for v in cur div1; do
  LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2div/$v -o run --output-format csv -- python3 bench.py --config C2 --no-cpu --h2d off --streams 1 --batch 128 --steps 2 --warmup 1 > gpurun_out/c2div/$v.json 2> gpurun_out/c2div/$v.err
  rc=$?; echo "trace $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
CONFIGS=C2 VARIANTS="cur div1 div8" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
CONFIGS=C5 VARIANTS="p2s4 p2s0 p2s8" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
# diagnostic: the C4 PMC pass with the keyframe commit enqueued on the caller's thread (no worker threads)
mkdir -p gpurun_out/r04/C4diag
cd /tmp && export TMPDIR=/tmp
LMSF_LIB=$GRAFT_REPO_ROOT/lmsf-slam_amd/ab/liblmsf_inlinecommit.so LMSF_COMMIT_INLINE=1 timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/r04/C4diag/pmc_FETCH_SIZE -o pmc --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C4 --no-cpu --no-n27 --h2d off --steps 6 --warmup 2 --opt LM_LOOP=0 --no-prefetch > $GRAFT_REPO_ROOT/gpurun_out/r04/C4diag/pmc_FETCH_SIZE.json 2> $GRAFT_REPO_ROOT/gpurun_out/r04/C4diag/pmc_FETCH_SIZE.err
echo "c4diag rc=$?"
