# A/B of variant builds (lmsf-slam_amd/ab/liblmsf_<v>.so via LMSF_LIB): for each CONFIGS entry and each
# VARIANTS entry one bench line gpurun_out/ablib_<cfg>_<v>.json; stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
for cfg in ${CONFIGS:-C2}; do
  for v in ${VARIANTS:-old}; do
    LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 python bench.py --config $cfg --no-cpu --h2d off ${BENCH_ARGS:-} > gpurun_out/ablib_${cfg}_$v.json 2> gpurun_out/ablib_${cfg}_$v.err
    rc=$?; echo "$cfg $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  done
done
