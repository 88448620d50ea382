# C5 bench line at HEAD (3 pipelined contexts), then C2 A/B of the in-flight window (tools/gpu_ab_args.sh).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/final
timeout -k 10 400 python -u bench.py --config C5 > gpurun_out/final/bench_C5.json 2> gpurun_out/final/bench_C5.err
rc=$?; echo "bench C5 rc=$rc"; tail -c 300 gpurun_out/final/bench_C5.json; echo; case $rc in 0) ;; *) exit $rc;; esac
CFG=C2 ROUNDS=2 ARGS="-;--streams 8 --inflight 4;--streams 6 --inflight 4;--streams 8 --inflight 5" bash tools/gpu_ab_args.sh
