set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/c5memo
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "dense or c5 or one_lane" > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
CFG=C5 ROUNDS=2 ARGS="-;--opt QUERY_MEMO=0" bash tools/gpu_ab_args.sh || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/c5memo/m1c -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --config C5 --no-cpu --steps 1 --warmup 1 --pipeline 1 > $GRAFT_REPO_ROOT/gpurun_out/c5memo/m1c.json 2> $GRAFT_REPO_ROOT/gpurun_out/c5memo/m1c.err
rc=$?; echo "trace rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
cd "$GRAFT_REPO_ROOT"
true

