# r04 end-of-round evidence (2/2): C2 and C5 kernel traces + PMC passes at HEAD (tools/profile.sh).
set -u
cd "$GRAFT_REPO_ROOT"
CFGS="C2 C5" bash tools/gpu_profiles.sh || exit $?
