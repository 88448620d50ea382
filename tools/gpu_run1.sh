set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
timeout -k 10 600 python bench.py --steps 5 --warmup 1 > gpurun_out/bench1.log 2>&1
rc=$?; echo "bench_rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof1" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof1.log" 2>&1
echo "prof_rc=$?"
