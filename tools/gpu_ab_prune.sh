# knn pruning: parity tests of the current build, C2 + C5 benches, first-pass radius overrides on C5.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
for cfg in C2 C5; do
  timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/ab_cur_$cfg.log 2>&1
  rc=$?; echo "cur $cfg rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
for v in ${LIMS:-0.05 0.25}; do
  LMSF_KNN_LIM1=$v timeout -k 10 600 python bench.py --config C5 --no-cpu > gpurun_out/ab_lim1_${v}_C5.log 2>&1
  rc=$?; echo "lim1=$v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
