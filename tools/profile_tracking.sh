# Kernel traces of the tracking configurations (C3 dual-LiDAR, C4 shared-map streams) for the per-scan
# latency breakdown (tools/gaps.py), each bench under its own limit.
set -u
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/${ROUND:-r03}"
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for cfg in ${CONFIGS:-C4 C3}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/trace_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --no-cpu > "$O/trace_$cfg.json" 2> "$O/trace_$cfg.err"
  rc=$?; echo "trace $cfg rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
