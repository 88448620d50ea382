# All bench configurations on one GPU (each step under its own time limit; stop at the first failure).
set -u
cd "$GRAFT_REPO_ROOT"
for cfg in ${CONFIGS:-C2 C3 C4 C5}; do
  timeout -k 10 900 python bench.py --config $cfg > gpurun_out/bench_$cfg.log 2>&1
  rc=$?; echo "bench $cfg rc=$rc"
  case $rc in 0) ;; *) exit $rc;; esac
done
