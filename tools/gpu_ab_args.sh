# A/B of bench.py argument sets in one box session: ARGS entries separated by ';' ("-" = defaults), ROUNDS
# rounds alternating; one JSON line per run under gpurun_out/ab_args_<round>_<i>.json.  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra SETS <<< "${ARGS:--}"
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for a in "${SETS[@]}"; do
    i=$((i+1))
    [ "$a" = "-" ] && a=""
    o=gpurun_out/ab_args_${r}_$i
    timeout -k 10 300 python bench.py --config ${CFG:-C2} --no-cpu --h2d off $a > $o.json 2> $o.err
    rc=$?; echo "round $r args[$i]=$a rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('$o.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
