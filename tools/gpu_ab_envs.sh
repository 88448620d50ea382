# A/B of environment settings on one config: ENVS="A=1,B=2 A=3" (comma-separated assignments per arm).
set -u
cd "$GRAFT_REPO_ROOT"
i=0
for arm in $ENVS; do
  i=$((i+1))
  env $(echo "$arm" | tr ',' ' ') timeout -k 10 600 python bench.py --config ${CFG:-C2} --no-cpu > gpurun_out/ab_env${i}_${CFG:-C2}.log 2>&1
  rc=$?; echo "arm $i ($arm) rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
