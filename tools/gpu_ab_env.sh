# A/B of an environment tunable: for each value of $VAR in $VALUES, the bench configs $CONFIGS.
set -u
cd "$GRAFT_REPO_ROOT"
for v in $VALUES; do
  for cfg in ${CONFIGS:-C2}; do
    env "$VAR=$v" timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/ab_${VAR}_${v}_$cfg.log 2>&1
    rc=$?; echo "$VAR=$v $cfg rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
