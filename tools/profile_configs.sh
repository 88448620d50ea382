# Kernel-trace profiles of the non-default bench configurations (one rocprofv3 run each).
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for cfg in ${CONFIGS:-C3 C4 C5}; do
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --no-cpu > "$R/gpurun_out/prof_$cfg.log" 2>&1
  rc=$?; echo "prof $cfg rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
