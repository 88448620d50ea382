# Walk key min/max change: the GPU parity suite on the default library, then library A/B on C2 / C5
# (k0 = fmin/fmax, k1 = asm min/max, k2 = asm + packed d2), interleaved twice.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
[ -n "${SKIP_TESTS:-}" ] || timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log
case $rc in 0) ;; *) exit $rc;; esac
for r in 1 2; do
  CONFIGS="C2 C5" VARIANTS="k0 k1 k2" bash tools/gpu_ab_lib.sh || exit $?
  for cfg in C2 C5; do for v in k0 k1 k2; do
    python3 -c "import json;d=json.load(open('gpurun_out/ablib_${cfg}_$v.json'));r=d['roofline'];print('$r','$cfg','$v',d['value'],d['ms_per_step'],r['avg_launch_ms'])"
  done; done
done
