# Ablation timing of the fused search + fit (one context stream, batch 128, memo off so every outer
# iteration searches every query): avg HIP-event launch time per variant library.
set -u
cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-base nofit nowalk}; do
  LMSF_MEMO=0 LMSF_LIB=lmsf-slam_amd/ab/liblmsf_$v.so timeout -k 10 300 python bench.py --no-cpu --h2d off --streams 1 --batch 128 --steps 6 --warmup 1 > gpurun_out/ablate_$v.json 2> gpurun_out/ablate_$v.err
  rc=$?; echo "variant $v rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
