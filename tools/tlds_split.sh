#!/bin/bash
# Build libniidmix variants with the LDS tile kernel's staging or position loop compiled out
# (NIIDMIX_TLDS_SPLIT=1: no position loop, 2: no staging) into tools/build/, for timing the
# kernel's phases with tools/exact_probe.py under NIIDMIX_LIB=<variant>.  CPU-side build step.
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
mkdir -p "$R/tools/build"
for v in ${SPLITS:-1 2 3 4 5}; do
  hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -ffp-contract=off -mcode-object-version=5 \
    -DNIIDMIX_TLDS_SPLIT=$v -I "$R/include" -o "$R/tools/build/libniidmix_split$v.so" \
    "$R/non-iid-topology-simulator_amd/csrc/niidmix.hip"
done
