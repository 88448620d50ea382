# Profiles (ROUND, default r05) of one bench configuration (CFG, default C2): kernel trace + stats of the bench
# command, then PMC passes (each counter set in a run of its own; --kernel-trace only beside --pmc):
# HBM traffic (FETCH_SIZE, WRITE_SIZE), L2 hit/miss, and an SQ pass (wave cycles, waits, instruction
# mix).  PMC runs use one context stream (device-wide counters) and skip the untimed n27 step.
set -u
R="$GRAFT_REPO_ROOT"
CFG=${CFG:-C2}
O="$R/gpurun_out/${ROUND:-r05}/$CFG"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
if [ -z "${SKIP_TRACE:-}" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --config $CFG --no-cpu --h2d off > "$O/trace_bench.json" 2> "$O/trace_bench.err"
rc=$?; echo "trace $CFG rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
fi
case $CFG in
  C2) PMC_ARGS="--steps 2 --warmup 1 --streams 1 --batch 256" ;;   # one context of the default launch (2 x 256)
  C5) PMC_ARGS="--steps 1 --warmup 1 --streams 1 --pipeline 1" ;;
  *)  PMC_ARGS="--steps 6 --warmup 2 --no-lookahead" ;;   # C3 / C4: PMC passes serialise dispatches (flag waits)
esac
PMC_ARGS="$PMC_ARGS ${PMC_EXTRA:-}"   # e.g. C3 / C4: --opt LM_LOOP=0 --no-prefetch (the r04 C3 PMC pass faulted with both on)
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES" "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT GRBM_GUI_ACTIVE"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL ${PMC_TIMEOUT:-300} rocprofv3 --pmc $ctr --kernel-trace -d "$O/pmc_$tag" -o pmc --output-format csv -- python3 "$R/bench.py" --config $CFG --no-cpu --no-n27 --h2d off $PMC_ARGS > "$O/pmc_$tag.json" 2> "$O/pmc_$tag.err"
  rc=$?; echo "pmc $CFG $tag rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
echo profiles-done
