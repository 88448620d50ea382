# PMC passes (HBM traffic of the search kernel) for the C4 and C5 bench configurations, one counter
# set per pass, each under its own time limit.
set -u
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for cfg in ${PMC_CONFIGS:-C4 C5}; do
  case $cfg in C4) args="--steps 4 --warmup 2";; C5) args="--steps 1 --warmup 1 --pairs 250";; esac
  for ctr in FETCH_SIZE WRITE_SIZE "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $ctr | tr ' ' '_')
    timeout -s KILL 400 rocprofv3 --pmc $ctr --kernel-trace -d "$R/gpurun_out/pmc_${cfg}_$tag" -o pmc --output-format csv -- python "$R/bench.py" --config $cfg --no-cpu $args > "$R/gpurun_out/pmc_${cfg}_$tag.log" 2>&1
    rc=$?; echo "pmc $cfg $tag rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
  done
done
