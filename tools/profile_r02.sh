# Round-2 profiles of the default C2 bench: kernel trace + stats of the driver's command, then PMC
# passes (each counter set in a run of its own; --kernel-trace only beside --pmc) on one context stream
# of the per-context batch: HBM traffic (FETCH_SIZE, WRITE_SIZE), L2 hit/miss, and an SQ pass (wave
# cycles, waits, instruction mix) for match_fit_kernel and lm_eval_kernel.
set -u
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/r02"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
if [ -z "${SKIP_TRACE:-}" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu --h2d off > "$O/trace_bench.json" 2> "$O/trace_bench.err"
rc=$?; echo "trace rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
fi
PMC_ARGS="--steps 2 --warmup 1 --no-cpu --no-n27 --h2d off --streams 1 --batch 128 ${PMC_EXTRA:-}"
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum" "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 240 rocprofv3 --pmc $ctr --kernel-trace -d "$O/pmc_$tag" -o pmc --output-format csv -- python3 "$R/bench.py" $PMC_ARGS > "$O/pmc_$tag.json" 2> "$O/pmc_$tag.err"
  rc=$?; echo "pmc $tag rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
echo profiles-done
