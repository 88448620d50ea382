# GPU parity suite, then the current library vs the previous commit's (ab/liblmsf_prev.so, built by
# `git stash; tools/build_variant.sh prev ""; git stash pop`) on each CONFIGS entry, alternating.
set -u
cd "$GRAFT_REPO_ROOT"
if [ -z "${SKIP_TESTS:-}" ]; then
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
fi
for cfg in ${CONFIGS:-C2 C4 C3}; do
  for v in new prev new prev; do
    lib=""; [ $v = new ] || lib=lmsf-slam_amd/ab/liblmsf_$v.so
    LMSF_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --no-cpu --h2d off > gpurun_out/abp_${cfg}_$v.json 2> gpurun_out/abp_${cfg}_$v.err
    rc=$?; echo "$cfg $v rc=$rc $(tail -1 gpurun_out/abp_${cfg}_$v.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
