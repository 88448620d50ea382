set -u
cd "$GRAFT_REPO_ROOT"
CONFIGS=C5 VARIANTS="split nosplit nosort fine" ROUNDS=1 bash tools/gpu_ab_lib.sh || exit $?
CONFIGS=C2 VARIANTS="split ctl1" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
