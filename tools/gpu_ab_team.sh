# A/B of the knn team size on single-scan (tracking) launches: C3 and C4, one process per setting.
set -u
cd "$GRAFT_REPO_ROOT"
for cfg in C4 C3; do
  for T in 1 2 4 8 16; do
    LMSF_KNN_TEAM=$T timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/ab_${cfg}_T$T.log 2>&1
    rc=$?; echo "$cfg T=$T rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
