# Memo change: full GPU suite, then A/B of LMSF_MEMO_EXACT / LMSF_MEMO_REFIT on C2, and of LMSF_MEMO_EXACT on C3 / C4.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
ENVS="LMSF_MEMO_EXACT=0 - LMSF_MEMO_REFIT=0 - LMSF_MEMO_EXACT=0 -" bash tools/gpu_ab_env.sh || exit $?
for i in 1 2 3 4 5 6; do python3 -c "import json;d=json.load(open('gpurun_out/ab_env_$i.json'));r=d['roofline'];print('C2',$i,d['value'],d['ms_per_step'],r['avg_launch_ms'],r['reused_query_frac'],r.get('refit_query_frac'))"; done
for cfg in C3 C4; do
  for e in LMSF_MEMO_EXACT=0 LMSF_MEMO_EXACT=1 LMSF_MEMO_EXACT=0 LMSF_MEMO_EXACT=1; do
    env $e timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/ab_$cfg.json 2> gpurun_out/ab_$cfg.err
    rc=$?; case $rc in 0) ;; *) echo "$cfg $e rc=$rc"; exit $rc;; esac
    python3 -c "import json;d=json.load(open('gpurun_out/ab_$cfg.json'));print('$cfg','$e',d['value'],d['ms_per_step'])"
  done
done
