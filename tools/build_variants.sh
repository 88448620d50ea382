# Variant builds for A/B runs: each VARIANTS entry "name:-DX=1,-DY=2" ("," separates flags) becomes
# lmsf-slam_amd/ab/liblmsf_<name>.so, built from the current sources with those extra flags
# (then tools/gpu_ab_lib.sh on the box with VARIANTS="<names>").  -DLMSF_AB: env overrides of the A/B knobs.
set -eu
cd "$(dirname "$0")/../lmsf-slam_amd"
mkdir -p ab
for v in ${VARIANTS:?}; do
  n=${v%%:*}; f=$( [ "$v" = "$n" ] && echo "" || echo "${v#*:}" | tr ',' ' ')
  make -s -j4 BUILD=build_ab/$n OUT=ab/liblmsf_$n.so EXTRA="-DLMSF_AB $f" ab/liblmsf_$n.so &
done
wait
ls -la ab
