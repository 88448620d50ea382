# Several env A/B arms across configs: ARMS="CFG:VAR=val,VAR2=val ..." (X=0 = baseline arm).
set -u
cd "$GRAFT_REPO_ROOT"
i=0
for arm in $ARMS; do
  i=$((i+1))
  cfg=${arm%%:*}; envs=${arm#*:}
  env $(echo "$envs" | tr ',' ' ') timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/ab_m${i}_${cfg}.log 2>&1
  rc=$?; echo "arm $i ($arm) rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
