# lm_eval occupancy A/B: records per thread 4 (default, 4 waves) vs 2 (5 waves) vs 1 (6 waves), C2.
set -u
cd "$GRAFT_REPO_ROOT"
for v in def pt2 pt1 def pt2; do
  lib=""; [ $v = def ] || lib=lmsf-slam_amd/ab/liblmsf_$v.so
  LMSF_LIB=$lib timeout -k 10 300 python bench.py --no-cpu --h2d off > gpurun_out/ev_$v.json 2> gpurun_out/ev_$v.err
  rc=$?; echo "$v rc=$rc $(tail -1 gpurun_out/ev_$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  case $rc in 0) ;; *) exit $rc;; esac
done
