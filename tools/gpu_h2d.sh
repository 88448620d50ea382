# H2D investigation: copy bandwidth probe, then a kernel trace of the C2
# bench whose last K steps stream every step's scans from pinned host memory.
set -u
cd "$GRAFT_REPO_ROOT"
if [ -z "${SKIP_PROBE:-}" ]; then
timeout -k 10 120 python tools/h2d_probe.py > gpurun_out/h2d_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
fi
mkdir -p gpurun_out/h2dtrace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/h2dtrace" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --steps 10 ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/h2dtrace.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/h2dtrace.err"
echo "trace rc=$?"
