# r04: GPU suite, one-stream C2 kernel trace (LM control reduction tail), default C2 bench line.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
mkdir -p gpurun_out/c2trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/c2trace/t -o run --output-format csv -- python3 bench.py --config C2 --no-cpu --h2d off --streams 1 --batch 128 --steps 2 --warmup 1 > gpurun_out/c2trace/t.json 2> gpurun_out/c2trace/t.err
rc=$?; echo "trace rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
rc=$?; echo "bench rc=$rc"; tail -c 600 gpurun_out/bench_default.json
