# One-stream rocprofv3 kernel traces of variant builds (lmsf-slam_amd/ab/liblmsf_<v>.so via LMSF_LIB):
#   VARIANTS="cur nofine" CFG=C2 OUT=c2fine [TRACE_ARGS="..."] bash tools/gpu_trace_variants.sh
# -> gpurun_out/$OUT/<v>/ (kernel_stats.csv of each), then optionally (AB_ROUNDS > 0) the same variants' bench
# lines through tools/gpu_ab_lib.sh.  TRACE_ARGS default: C2 one context of 128 scans, 2 steps (C5: 1 step).
# Runs the -m gpu suite first unless NO_TESTS is set.  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
if [ -z "${NO_TESTS:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "tests_rc=$rc"; tail -3 gpurun_out/gpu_tests.log; case $rc in 0) ;; *) exit $rc;; esac
fi
CFG=${CFG:-C2}
case $CFG in
  C2) DEF="--config C2 --no-cpu --h2d off --streams 1 --batch 128 --steps 2 --warmup 1";;
  C5) DEF="--config C5 --no-cpu --steps 1 --warmup 1";;
  *) DEF="--config $CFG --no-cpu --no-n27 --h2d off --steps 6 --warmup 2";;
esac
OUT=${OUT:-trace_$CFG}
for v in ${VARIANTS:-cur}; do
  mkdir -p gpurun_out/$OUT/$v
  LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$OUT/$v \
    -o run --output-format csv -- python3 bench.py ${TRACE_ARGS:-$DEF} > gpurun_out/$OUT/$v.json 2> gpurun_out/$OUT/$v.err
  rc=$?; echo "trace $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
if [ "${AB_ROUNDS:-0}" -gt 0 ]; then
  CONFIGS=$CFG VARIANTS="${VARIANTS:-cur}" ROUNDS=$AB_ROUNDS bash tools/gpu_ab_lib.sh || exit $?
fi
