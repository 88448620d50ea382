# Profiles of the configurations in CFGS (tools/profile.sh each: kernel trace + PMC passes) and, with PROBE=1, the
# FETCH_SIZE gather calibration (tools/gather_probe/run.sh).  Stops at the first failure.
set -u
cd "$GRAFT_REPO_ROOT"
if [ -n "${PROBE:-}" ]; then bash tools/gather_probe/run.sh || exit $?; fi
for cfg in ${CFGS:-C2}; do
  CFG=$cfg bash tools/profile.sh || exit $?
done
echo all-profiles-done
