# GPU parity suite, then the memo A/B: consecutive-gap test (LMSF_MEMO_ORDER) and the memo pass's
# occupancy (variant libraries ab/liblmsf_w4 / w6 vs the default build), one C2 bench line each.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
run() {   # tag, env...
  tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --no-cpu --h2d off > gpurun_out/mo_$tag.json 2> gpurun_out/mo_$tag.err
  rc=$?; echo "$tag rc=$rc $(tail -1 gpurun_out/mo_$tag.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print(d["value"], d["ms_per_step"], r["reused_query_frac"], r["refit_query_frac"])')"
  case $rc in 0) ;; *) exit $rc;; esac
}
run def LMSF_MEMO_ORDER=1
run noorder LMSF_MEMO_ORDER=0
run w4 LMSF_LIB=lmsf-slam_amd/ab/liblmsf_w4.so
run w6 LMSF_LIB=lmsf-slam_amd/ab/liblmsf_w6.so
run def2 LMSF_MEMO_ORDER=1
