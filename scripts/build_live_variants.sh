#!/usr/bin/env bash
# Build libpekf.so variants that differ only in the fused front-end + filter kernel's compile flags
# (csrc/pekf_live.hip: ring / queue / quorum macros, scheduler, occupancy), for same-box A/B with
# scripts/ab_live.sh.  Needs a built tree (make in csrc) for the other objects.
# usage: scripts/build_live_variants.sh name "<flags>" [name "<flags>" ...]   -> ab/live_<name>.so
# SRC=pekf_frontend builds variants of that source instead (-> ab/frontend_<name>.so).
set -eu
cd "$(dirname "$0")/../poseestimationkf_amd/csrc"
mkdir -p ../../ab
SRC=${SRC:-pekf_live}
TAG=${SRC#pekf_}
OTHERS=$(ls build/*.o | grep -v "$SRC.o")
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -I../../include \
      -fno-slp-vectorize -ffp-contract=on $flags -c $SRC.hip -o ../../ab/${TAG}_$name.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../ab/${TAG}_$name.so $OTHERS ../../ab/${TAG}_$name.o -ldl
  echo "ab/${TAG}_$name.so: $flags"
done
