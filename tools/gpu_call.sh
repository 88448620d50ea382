set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  for env in "-" "LMSF_LM_LOOP=0"; do
    e=$( [ "$env" = "-" ] && echo "" || echo "$env")
    tag=$(echo "${env}" | tr -c 'A-Za-z0-9\n' '_')
    for cfg in C4 C3; do
      env $e LMSF_LIB=lmsf-slam_amd/ab/liblmsf_cur.so timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/loop_${cfg}_${tag}_r$r.json 2> gpurun_out/loop_${cfg}_${tag}_r$r.err
      rc=$?; echo "$cfg $env r$r rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/loop_${cfg}_${tag}_r$r.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
