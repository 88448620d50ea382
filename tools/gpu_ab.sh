set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
for team in 8 16 32; do for remap in 0 1; do
  LMSF_KNN_TEAM=$team LMSF_XCD_REMAP=$remap timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/ab_${team}_${remap}.log 2>&1
  rc=$?; echo "ab team=$team remap=$remap rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done; done
