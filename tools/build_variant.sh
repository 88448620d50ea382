#!/bin/bash
# Build an A/B variant of liblmsf_hip.so: tools/build_variant.sh <name> "<extra hipcc flags>"
# -> lmsf-slam_amd/ab/liblmsf_<name>.so (selected at run time by LMSF_LIB).  Built with -DLMSF_AB: the A/B
# knobs (ab_int in csrc/lmsf_internal.h) then take environment overrides, which the shipped library ignores.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/lmsf-slam_amd
B=$P/build_ab/$1
mkdir -p $B $P/ab
FL="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -w -DLMSF_AB -I$R/include -I$P/csrc $2"
ls $P/csrc/*.cpp $P/csrc/*.hip | grep -v /dist.cpp | xargs -P 8 -I{} sh -c "/opt/rocm/bin/hipcc $FL -x hip -c {} -o $B/\$(basename {}).o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o $P/ab/.tmp_$1.so $B/*.o && mv $P/ab/.tmp_$1.so $P/ab/liblmsf_$1.so
echo "built $P/ab/liblmsf_$1.so"
