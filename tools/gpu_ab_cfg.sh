# A/B of runtime switches per configuration: for each CONFIGS entry and each ENVS entry ("A=1,B=0",
# "-" = none) one bench line gpurun_out/ab_<cfg>_<i>.json; stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
for cfg in ${CONFIGS:-C4 C3}; do
  i=0
  for e in ${ENVS:--}; do
    i=$((i+1))
    envs=$( [ "$e" = "-" ] && echo "" || echo "$e" | tr ',' ' ')
    env $envs timeout -k 10 300 python bench.py --config $cfg --no-cpu ${BENCH_ARGS:-} > gpurun_out/ab_${cfg}_$i.json 2> gpurun_out/ab_${cfg}_$i.err
    rc=$?; echo "$cfg env[$i]=$e rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  done
done
