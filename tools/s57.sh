#!/bin/bash
# batched overflow residual gathers (2 / 3 in flight) on gateway-heavy stripes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s57; mkdir -p $O
timeout -k 10 400 python -u tools/stripe_probe.py --worlds 8,4,1 --steps 20 --variant def: \
  --variant ovb2:NIIDMIX_CLIQUE_TILE=16x7x8x64x34x4 --variant ovb3:NIIDMIX_CLIQUE_TILE=16x7x8x64x66x4 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep world $O/probe.txt
