# GPU tests (subset), then bench runs of CFG alternating library variants (VARIANTS, lmsf-slam_amd/ab/) with
# ARGS, ROUNDS times; then optional extra runs (EXTRA: ';'-separated bench.py argument sets, shipped library).
set -u
cd "$GRAFT_REPO_ROOT"
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "$TESTS" > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests_rc=$rc"; tail -2 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
fi
for r in $(seq 1 ${ROUNDS:-2}); do
  for spec in ${VARIANTS:-prev cur}; do   # spec: variant[:ENV=V[,ENV=V]]
    v=${spec%%:*}; envs=$( [ "$spec" = "$v" ] && echo "" || echo "${spec#*:}" | tr ',' ' ')
    tag=$(echo "$spec" | tr ':,=' '___')
    env $envs LMSF_LIB=$PWD/lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 400 python bench.py --config ${CFG:-C2} --no-cpu ${ARGS:-} > gpurun_out/v_${tag}_r$r.json 2> gpurun_out/v_${tag}_r$r.err
    rc=$?; echo "${CFG:-C2} $spec r$r rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/v_${tag}_r$r.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], (d.get('h2d_inclusive') or {}).get('ms_per_step'))" 2>/dev/null)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
IFS=';' read -ra SETS <<< "${EXTRA:-}"
j=0
for a in "${SETS[@]}"; do
  j=$((j+1))
  timeout -k 10 400 python bench.py --no-cpu $a > gpurun_out/x_$j.json 2> gpurun_out/x_$j.err
  rc=$?; echo "extra [$a] rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/x_$j.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d.get('h2d_inclusive'))" 2>/dev/null)"
  case $rc in 0) ;; *) exit $rc;; esac
done
