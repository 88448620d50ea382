# Kernel-trace stats of C2 and C5, then one SQ counter pass on C2 (wave cycles / waits / instruction mix).
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for cfg in ${CONFIGS:-C2 C5}; do
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --no-cpu > "$R/gpurun_out/prof_$cfg.log" 2>&1
  rc=$?; echo "prof $cfg rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES --kernel-trace -d "$R/gpurun_out/pmc_sq" -o pmc --output-format csv -- python3 "$R/bench.py" --steps 2 --warmup 1 --no-cpu > "$R/gpurun_out/pmc_sq.log" 2>&1
rc=$?; echo "pmc sq rc=$rc"; exit $rc
