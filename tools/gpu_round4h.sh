# r04: C4 / C3 kernel traces + PMC passes at HEAD with the single-scan LM loop and extract-ahead off in the PMC runs
# (the C3 PMC pass with both on faulted under rocprofv3 on box A; the same run outside the profiler passes).
set -u
cd "$GRAFT_REPO_ROOT"
CFGS="C4 C3" PMC_EXTRA="--opt LM_LOOP=0 --no-prefetch" PMC_TIMEOUT=150 bash tools/gpu_profiles.sh || exit $?
