# A/B of runtime switches in one box session: each ENVS entry (space-free "A=1,B=0" lists, "-" = none)
# runs the default C2 bench once; one JSON line per entry under gpurun_out/ab_env_<i>.json.  The knobs are read
# only by -DLMSF_AB builds (tools/build_variant.sh): set LMSF_LIB to one.
set -u
cd "$GRAFT_REPO_ROOT"
i=0
for e in ${ENVS:--}; do
  i=$((i+1))
  envs=$( [ "$e" = "-" ] && echo "" || echo "$e" | tr ',' ' ')
  env $envs timeout -k 10 300 python bench.py --no-cpu --h2d off ${BENCH_ARGS:-} > gpurun_out/ab_env_$i.json 2> gpurun_out/ab_env_$i.err
  rc=$?; echo "env[$i]=$e rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
