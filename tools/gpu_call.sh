set -u
cd "$GRAFT_REPO_ROOT"
NO_BENCH=1 bash tools/gpu_tests.sh || exit $?
timeout -k 10 300 python bench.py --no-cpu --h2d on > gpurun_out/bench_c2.json 2> gpurun_out/bench_c2.err; echo "c2 rc=$?"
for cfg in C4 C3 C4 C3; do
  timeout -k 10 300 python bench.py --config $cfg --no-cpu > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err
  rc=$?; echo "$cfg rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bench_$cfg.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
  case $rc in 0) ;; *) exit $rc;; esac
done
python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bench_c2.json') if l.startswith('{')][-1]); print('C2', d['value'], d['ms_per_step'], d['h2d_inclusive']['ms_per_step'])"
