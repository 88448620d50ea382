# r04: dense-walk deferred insertion A/B on C5 (cur / defer8 / defer4), then C3 / C4 profiles at HEAD.
set -u
cd "$GRAFT_REPO_ROOT"
CONFIGS=C5 VARIANTS="cur defer8 defer4 p2pipe" ROUNDS=2 bash tools/gpu_ab_lib.sh || exit $?
CFGS="C3 C4" bash tools/gpu_profiles.sh || exit $?
