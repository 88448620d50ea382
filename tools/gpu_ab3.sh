set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"
case $rc in 124|134|137|139) exit $rc;; esac
for team in 1 2; do for b in 64 128; do
  LMSF_KNN_TEAM=$team timeout -k 10 300 python bench.py --steps 5 --warmup 1 --no-cpu --batch $b > gpurun_out/ab3_t${team}_b${b}.log 2>&1
  rc=$?; echo "team=$team batch=$b rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done; done
cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof3" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu > "$GRAFT_REPO_ROOT/gpurun_out/prof3.log" 2>&1
echo "prof_rc=$?"
