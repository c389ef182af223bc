#!/bin/bash
# gateway-heavy stripes (8-GPU rank emulation): member-load flags, skew, tile variants
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s53; mkdir -p $O
timeout -k 10 500 python -u tools/stripe_probe.py --worlds 8,4 --steps 20 \
  --variant def: --variant nt0:NIIDMIX_CLIQUE_TILE=16x7x8x64x0x4 --variant rw0:NIIDMIX_CLIQUE_TILE=16x7x8x0x2x4 \
  --variant st16:NIIDMIX_CLIQUE_TILE=16x7x8x64x16x4 --variant skew8:NIIDMIX_CLIQUE_SKEW=8 --variant t813:NIIDMIX_CLIQUE_TILE=8x13x4x64x2x4 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
