set -u
cd "$GRAFT_REPO_ROOT"
export LMSF_LIB=lmsf-slam_amd/ab/liblmsf_ab.so
for r in 1 2; do
for e in 2 3 4 99; do
for a in "--pipeline 1" "--pipeline 3"; do
LMSF_DENSE_MEMO_FROM=$e timeout -k 10 300 python bench.py --config C5 --no-cpu $a > gpurun_out/p.json 2> gpurun_out/p.err
rc=$?; echo "from $e [$a] r$r rc=$rc $(python3 -c "import json; d=json.loads([l for l in open('gpurun_out/p.json') if l.startswith('{')][-1]); print(d['value'], d['roofline']['avg_launch_ms'])")"
case $rc in 0) ;; *) exit $rc;; esac
done
done
done
