# Extraction ablation on the box: kernel trace + stats of a one-context C2 batch (128 scans) per library
# variant (VARIANTS; "default" = the in-tree library, else lmsf-slam_amd/ab/liblmsf_<v>.so), summaries under
# gpurun_out/xab/<v>/.  Stops at the first failure.
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for v in ${VARIANTS:-default}; do
  lib=$R/lmsf-slam_amd/liblmsf_hip.so
  [ "$v" = default ] || lib=$R/lmsf-slam_amd/ab/liblmsf_$v.so
  mkdir -p "$R/gpurun_out/xab/$v"
  LMSF_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/xab/$v" -o run --output-format csv -- python3 "$R/bench.py" --config C2 --no-cpu --no-n27 --h2d off --steps 3 --warmup 1 --streams 1 --batch 128 > "$R/gpurun_out/xab/$v/bench.json" 2> "$R/gpurun_out/xab/$v/bench.err"
  rc=$?; echo "xab $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  f=$(find "$R/gpurun_out/xab/$v" -name '*kernel_stats.csv' | head -1)
  python3 "$R/tools/kstats.py" "$f" | head -16
done
