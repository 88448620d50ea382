set -u
cd "$GRAFT_REPO_ROOT"
for cfg in C3 C4; do
  for m in rank bitonic; do
    LMSF_EXTRACT_SORT=$m timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/ab_${cfg}_$m.log 2>&1
    rc=$?; echo "$cfg $m rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
