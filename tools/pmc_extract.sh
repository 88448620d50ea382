# SQ counter passes over the extraction kernels of the C2 bench (one context stream, batch 128):
# gpurun_out/pmc_ext_<tag>/ per pass.
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for ctr in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVES" "SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 200 rocprofv3 --pmc $ctr --kernel-trace ${KREGEX:+--kernel-include-regex "$KREGEX"} -d "$R/gpurun_out/pmc_ext_$tag" -o pmc --output-format csv -- python3 "$R/bench.py" --no-cpu --no-n27 --h2d off --steps 2 --warmup 1 --streams 1 --batch 128 > "$R/gpurun_out/pmc_ext_$tag.json" 2> "$R/gpurun_out/pmc_ext_$tag.err"
  rc=$?; echo "pmc $tag rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
