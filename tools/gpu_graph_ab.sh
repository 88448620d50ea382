# GPU parity suite, then the HIP-graph A/B (LMSF_GRAPH) on C2 / C4 / C3, one bench line per run.
set -u
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests_rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
for cfg in ${CONFIGS:-C2 C4 C3}; do
  for g in 1 0 1; do
    LMSF_GRAPH=$g timeout -k 10 300 python bench.py --config $cfg --no-cpu --h2d off > gpurun_out/gab_${cfg}_$g.json 2> gpurun_out/gab_${cfg}_$g.err
    rc=$?; echo "$cfg graph=$g rc=$rc $(tail -1 gpurun_out/gab_${cfg}_$g.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    case $rc in 0) ;; *) exit $rc;; esac
  done
done
