# Parity suite of the current build, then bench lines of $CONFIGS (no CPU leg).
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
for cfg in ${CONFIGS:-C2 C5}; do
  timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/ab_${TAG:-cur}_$cfg.log 2>&1
  rc=$?; echo "${TAG:-cur} $cfg rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
