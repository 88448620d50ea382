# A/B of context options in one box session (bench.py --opt): each OPTS entry ("-" = defaults; "A=1,B=2"
# lists) runs the bench once per round, ROUNDS rounds alternating; one JSON line per run under
# gpurun_out/ab_opt_<round>_<i>.json.  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for o in ${OPTS:--}; do
    i=$((i+1))
    args=$( [ "$o" = "-" ] && echo "" || echo "$o" | tr ',' '\n' | sed 's/^/--opt /' | tr '\n' ' ')
    timeout -k 10 300 python bench.py --config ${CFG:-C2} --no-cpu --h2d off ${BENCH_ARGS:-} $args > gpurun_out/ab_opt_${r}_$i.json 2> gpurun_out/ab_opt_${r}_$i.err
    rc=$?; echo "round $r opt[$i]=$o rc=$rc $(python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_opt_${r}_$i.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['reused_query_frac'] if d.get('roofline') else '')" 2>/dev/null)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
