# Kernel trace of the C2 H2D-inclusive steps (--memory-copy-trace crashed rocprofv3 at process exit, r03) (verdict r02 item 4): kernel + memory-copy trace of a bench run
# with every step's scans streamed from pinned host memory.  No --pmc here (trace domains only).
set -u
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/${ROUND:-r03}/h2d"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
  python3 "$R/bench.py" --no-cpu --h2d on --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-} > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "h2d trace rc=$rc"; exit $rc
