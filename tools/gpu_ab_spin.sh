# A/B of the host-side waits of the tracking step (one -DLMSF_AB build, env knobs): worker spin before sleeping,
# spinning stream waits.  C4 then C3 per setting, ROUNDS rounds.
set -u
cd "$GRAFT_REPO_ROOT"
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in ${ENVS:-"LMSF_WORKER_SPIN_US=0,LMSF_SPIN_SYNC=0" "LMSF_WORKER_SPIN_US=2000,LMSF_SPIN_SYNC=0"}; do
    envs=$(echo "$e" | tr ',' ' ')
    for cfg in C4 C3; do
      env LMSF_LIB=lmsf-slam_amd/ab/liblmsf_cur.so $envs timeout -k 10 300 python bench.py --config $cfg --no-cpu --steps 60 --warmup 12 > gpurun_out/spin_$cfg.json 2>/dev/null || exit $?
      echo "$cfg $e r$r $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/spin_$cfg.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
    done
  done
done
