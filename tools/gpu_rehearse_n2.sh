# Two ranks on the box's one GPU over gloo (bench.py --dist-backend gloo-gpu): the N-rank data path of every
# configuration -- sharding, map broadcast, pose / keyframe exchanges, max-over-ranks timing -- on real devices.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/n2
for cfg in C2 C5 C4 C3; do
  timeout -k 10 420 python -u bench.py --config $cfg --gpus 2 --dist-backend gloo-gpu --steps 3 --warmup 1 \
    > gpurun_out/n2/bench_$cfg.json 2> gpurun_out/n2/bench_$cfg.err
  rc=$?; echo "n2 $cfg rc=$rc"; tail -c 400 gpurun_out/n2/bench_$cfg.json; echo; case $rc in 0) ;; *) tail -20 gpurun_out/n2/bench_$cfg.err; exit $rc;; esac
done
echo n2-done
