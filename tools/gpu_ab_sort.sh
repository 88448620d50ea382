# Parity suite, then A/B of the sector sort on the tracking configs and C2.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"
case $rc in 0) ;; *) exit $rc;; esac
for cfg in C3 C4 C2; do
  for m in rank bitonic; do
    LMSF_EXTRACT_SORT=$m timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/ab_${cfg}_$m.log 2>&1
    rc=$?; echo "$cfg $m rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
