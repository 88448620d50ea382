# Memo-refit change: the memo / full-size parity tests, then A/B of LMSF_MEMO_REFIT on the C2 bench (x2 each).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_refit.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests_refit.log
case $rc in 0) ;; *) exit $rc;; esac
ENVS="LMSF_MEMO_REFIT=0 - LMSF_MEMO_REFIT=0 -" bash tools/gpu_ab_env.sh
for i in 1 2 3 4; do python3 -c "import json;d=json.load(open('gpurun_out/ab_env_$i.json'));r=d['roofline'];print($i,d['value'],d['ms_per_step'],r['avg_launch_ms'],r['reused_query_frac'],r.get('refit_query_frac'))"; done
