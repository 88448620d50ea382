# A/B of the single-scan team size (LMSF_KNN_TEAM) on C4 / C3, alternating, one bench line each.
set -u
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for t in 8 4 16; do
    for cfg in C4 C3; do
      LMSF_KNN_TEAM=$t timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-n27 > gpurun_out/team_${cfg}_${t}_$rep.log 2>&1 || exit $?
      python -c "import json;l=[x for x in open('gpurun_out/team_${cfg}_${t}_$rep.log') if x.startswith('{')][-1];d=json.loads(l);print('$cfg team=$t', d['ms_per_step'], d['roofline']['avg_launch_ms'])"
    done
  done
done
