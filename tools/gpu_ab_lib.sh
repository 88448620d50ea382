# A/B of variant builds (lmsf-slam_amd/ab/liblmsf_<v>.so via LMSF_LIB): ROUNDS rounds, each running every
# CONFIGS entry with every VARIANTS entry in turn; one bench line gpurun_out/ablib_<cfg>_<v>_r<round>.json
# and its value / ms per step on stdout.  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
for r in $(seq 1 ${ROUNDS:-1}); do
  for cfg in ${CONFIGS:-C2}; do
    for v in ${VARIANTS:-old}; do
      o=gpurun_out/ablib_${cfg}_${v}_r$r
      LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 python bench.py --config $cfg --no-cpu --h2d off ${BENCH_ARGS:-} > $o.json 2> $o.err
      rc=$?; echo "$cfg $v r$r rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('$o.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
      case $rc in 0) ;; *) exit $rc;; esac
    done
  done
done
