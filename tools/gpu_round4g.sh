# r04: C3 short run outside the profiler (the PMC pass faulted), GPU suite, C5 A/B of the pass-2 restructure.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 python -u bench.py --config C3 --no-cpu --no-n27 --h2d off --steps 6 --warmup 2 > gpurun_out/diag_c3.json 2> gpurun_out/diag_c3.err
rc=$?; echo "diag_c3_rc=$rc"; tail -c 400 gpurun_out/diag_c3.json; case $rc in 0) ;; *) tail -5 gpurun_out/diag_c3.err; exit $rc;; esac
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
CONFIGS=C5 VARIANTS="cur prevp2" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
