# Parity suite, then $CONFIGS benches under rocprofv3 kernel-trace (kernel stats per config).
set -u
R="$GRAFT_REPO_ROOT"
cd "$R"
timeout -k 10 600 python -m pytest tests -m gpu -q -x -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
for cfg in ${CONFIGS:-C2}; do
  rm -rf "$R/gpurun_out/prof_$cfg"
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_$cfg" -o run --output-format csv -- python3 "$R/bench.py" --config $cfg --no-cpu > "$R/gpurun_out/ab_prof_$cfg.log" 2>&1
  rc=$?; echo "prof $cfg rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
