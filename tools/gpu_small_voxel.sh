# Small-cloud voxel kernel: its tests, then the full GPU suite, then C4 / C3 A/B (LMSF_SMALL_VOXEL).
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -k voxel --timeout 120 --timeout-method thread > gpurun_out/gpu_voxel.log 2>&1
rc=$?; echo "voxel_rc=$rc"; tail -1 gpurun_out/gpu_voxel.log; case $rc in 0) ;; *) exit $rc;; esac
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -1 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
for rep in 1 2; do
  for sv in 1 0; do
    for cfg in C4 C3; do
      LMSF_SMALL_VOXEL=$sv timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-n27 > gpurun_out/sv_${cfg}_${sv}_$rep.log 2>&1 || exit $?
      python -c "import json;l=[x for x in open('gpurun_out/sv_${cfg}_${sv}_$rep.log') if x.startswith('{')][-1];print('$cfg small=$sv', json.loads(l)['ms_per_step'])"
    done
  done
done
