set -u
cd "$GRAFT_REPO_ROOT"
i=0
for a in ${CASES:-"--batch 256 --streams 2"}; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu --h2d off $(echo $a | tr , " ") > gpurun_out/abcfg_$i.json 2> gpurun_out/abcfg_$i.err
  rc=$?; echo "[$a] rc=$rc $(tail -1 gpurun_out/abcfg_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
  case $rc in 0) ;; *) exit $rc;; esac
done
