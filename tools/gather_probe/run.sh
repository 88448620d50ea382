# FETCH_SIZE calibration of 16-B gathers (gather_probe.hip): one rocprofv3 pass per counter set, then the summary.
set -u
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/${ROUND:-r04}/gather_probe"
mkdir -p "$O"
B="$R/tools/gather_probe/gather_probe"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 "$B" > "$O/bytes.json" || exit $?
for ctr in FETCH_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_HIT_sum TCC_MISS_sum"; do
  tag=$(echo $ctr | cut -d' ' -f1)
  timeout -s KILL 120 rocprofv3 --pmc $ctr --kernel-trace -d "$O/pmc_$tag" -o pmc --output-format csv -- "$B" > /dev/null 2> "$O/pmc_$tag.err"
  rc=$?; echo "pmc $tag rc=$rc"; case $rc in 0) ;; *) exit $rc;; esac
done
echo probe-done
