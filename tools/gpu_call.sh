set -u
cd "$GRAFT_REPO_ROOT"
bash tools/profile_h2d.sh || exit $?
CONFIGS=C4 bash tools/profile_tracking.sh || exit $?
echo all-done
