# A/B of alternative builds of liblmsf_hip.so (lmsf-slam_amd/ab/liblmsf_<v>.so, selected by LMSF_LIB).
set -u
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-base}; do
  for cfg in ${CONFIGS:-C2 C5}; do
    LMSF_LIB=$PWD/lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 600 python bench.py --config $cfg --no-cpu > gpurun_out/ab_${TAG:-}${v}_$cfg.log 2>&1
    rc=$?; echo "$v $cfg rc=$rc"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
