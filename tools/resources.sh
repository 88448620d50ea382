#!/bin/bash
# VGPRs / scratch / occupancy of every kernel of one source: tools/resources.sh csrc/k_match.hip [extra flags]
cd "$(dirname "$0")/../lmsf-slam_amd"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -ffp-contract=off -w -I../include -Icsrc ${@:2} -x hip -c $1 -o /dev/null \
  -Rpass-analysis=kernel-resource-usage 2>&1 | python3 ../tools/resources.py
