set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py -k "tracker or c4 or deferred or lookback or sparse_point or dual or growth or shared_map" -v -p no:cacheprovider --timeout 400 --timeout-method thread > gpurun_out/pre_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/pre_tests.log; case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  for v in 1 0; do
    LMSF_LIB=lmsf-slam_amd/ab/liblmsf_cur.so LMSF_PRESEARCH=$v timeout -k 10 300 python bench.py --config C4 --no-cpu --steps 60 --warmup 12 > gpurun_out/c4pre_${v}_$r.json 2>/dev/null || exit $?
    echo "C4 presearch=$v r$r $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c4pre_${v}_$r.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])")"
    LMSF_LIB=lmsf-slam_amd/ab/liblmsf_cur.so LMSF_PRESEARCH=$v timeout -k 10 300 python bench.py --config C3 --no-cpu > gpurun_out/c3pre_${v}_$r.json 2>/dev/null || exit $?
    echo "C3 presearch=$v r$r $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/c3pre_${v}_$r.json') if l.startswith('{')][-1]); print(d['value'], d['ms_per_step'])")"
  done
done
