# Voxel filter kernel durations per A/B mode (tools/voxel_probe.py under rocprofv3 --kernel-trace --stats).
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-0 1 2 3}; do
  LIBENV=$( [ -n "${VAR:-}" ] && echo "LMSF_LIB=$R/lmsf-slam_amd/ab/liblmsf_$VAR.so" || echo "" )
  env $LIBENV LMSF_VR_MODE=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/probe_$m" -o run --output-format csv -- python3 "$R/tools/voxel_probe.py" > "$R/gpurun_out/probe_$m.log" 2>&1
  rc=$?; echo "mode $m rc=$rc $(grep -v '^W\|^E' $R/gpurun_out/probe_$m.log | tail -1)"; case $rc in 0) ;; *) exit $rc;; esac
done
