# A/B of the spin wait (LMSF_SPIN_SYNC) on the tracking configurations, alternating, two runs each.
set -u
cd "$GRAFT_REPO_ROOT"
for rep in 1 2; do
  for sp in 1 0; do
    for cfg in C4 C3; do
      LMSF_SPIN_SYNC=$sp timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-n27 > gpurun_out/spin_${cfg}_${sp}_$rep.log 2>&1 || exit $?
      python -c "import json,sys;l=[x for x in open('gpurun_out/spin_${cfg}_${sp}_$rep.log') if x.startswith('{')][-1];print('$cfg spin=$sp', json.loads(l)['ms_per_step'])"
    done
  done
done
