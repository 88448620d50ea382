# A/B of variant builds, alternating, one indexed bench line each: gpurun_out/ablib2_<i>_<v>.json
set -u
cd "$GRAFT_REPO_ROOT"
i=0
for v in ${VARIANTS:-old new}; do
  i=$((i+1))
  LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 python bench.py --config ${CFG:-C2} --no-cpu --h2d off ${BENCH_ARGS:-} > gpurun_out/ablib2_${i}_$v.json 2> gpurun_out/ablib2_${i}_$v.err
  rc=$?; case $rc in 0) ;; *) echo "$v rc=$rc"; exit $rc;; esac
  python3 -c "import json;l=[x for x in open('gpurun_out/ablib2_${i}_$v.json') if x.startswith('{')][-1];print('$i $v', json.loads(l)['value'])"
done
