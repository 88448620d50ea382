# A/B of environment knobs of an -DLMSF_AB build (LMSF_LIB, default lmsf-slam_amd/ab/liblmsf_cur.so): ROUNDS rounds,
# each running every CONFIGS entry at every VALUES entry in turn -- values of KNOB, or with KNOB=- comma lists of
# assignments ("A=1,B=0"; "-" = none); value / ms per step on stdout, the bench lines under
# gpurun_out/knob_<cfg>_<i>_r<round>.json.  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
export LMSF_LIB=${LMSF_LIB:-lmsf-slam_amd/ab/liblmsf_cur.so}
for r in $(seq 1 ${ROUNDS:-1}); do
  for cfg in ${CONFIGS:-C4}; do
    i=0
    for v in ${VALUES:-0 1}; do
      i=$((i+1))
      if [ "${KNOB:--}" = "-" ]; then envs=$( [ "$v" = "-" ] && echo "" || echo "$v" | tr ',' ' '); else envs="$KNOB=$v"; fi
      o=gpurun_out/knob_${cfg}_${i}_r$r
      env $envs timeout -k 10 300 python bench.py --config $cfg --no-cpu --h2d off ${BENCH_ARGS:-} > $o.json 2> $o.err
      rc=$?; echo "$cfg [$v] r$r rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('$o.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
