# Round-1 profiles: kernel trace of the default bench command + PMC passes for HBM traffic
# (each counter set in a pass of its own; no tracing domains beside --kernel-trace).
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_r01" -o bench --output-format csv -- python "$R/bench.py" > "$R/gpurun_out/prof_r01_bench.log" 2>&1
rc=$?; echo "trace_rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $ctr | tr ' ' '_')
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d "$R/gpurun_out/pmc_$tag" -o pmc --output-format csv -- python "$R/bench.py" --steps 2 --warmup 1 --no-cpu --streams 1 --batch 128 > "$R/gpurun_out/pmc_$tag.log" 2>&1
  rc=$?; echo "pmc $tag rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
