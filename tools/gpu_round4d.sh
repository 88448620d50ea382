set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
LMSF_LIB=lmsf-slam_amd/ab/liblmsf_stepprof.so timeout -k 10 300 python bench.py --config C2 --no-cpu --h2d off --streams 1 --batch 128 --steps 2 --warmup 1 > gpurun_out/stepprof.log 2>&1
rc=$?; echo "stepprof_rc=$rc"; grep -c "lm_step" gpurun_out/stepprof.log; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python bench.py --config C5 --no-cpu > gpurun_out/bench_C5.json 2> gpurun_out/bench_C5.err
rc=$?; echo "bench_C5_rc=$rc"; tail -c 300 gpurun_out/bench_C5.json
