# r04 end-of-round evidence (1/2): GPU suite, smoke, the four configurations' bench lines at HEAD.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/final/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/final/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; echo "smoke_rc=$rc"; tail -2 gpurun_out/final/smoke.log; case $rc in 0) ;; *) exit $rc;; esac
for cfg in C2 C5 C4 C3; do
  a=""; [ $cfg = C2 ] || a="--config $cfg"
  timeout -k 10 400 python -u bench.py $a > gpurun_out/final/bench_$cfg.json 2> gpurun_out/final/bench_$cfg.err
  rc=$?; echo "bench $cfg rc=$rc"; tail -c 300 gpurun_out/final/bench_$cfg.json; echo; case $rc in 0) ;; *) exit $rc;; esac
done
