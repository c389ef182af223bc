#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s26
timeout -k 10 300 python tools/tune_inproc.py --reps 5 --steps 20 --variant def::clique \
  --variant nt:NIIDMIX_CLIQUE_TILE=16x7x8x64x2x4:clique --variant rw0:NIIDMIX_CLIQUE_TILE=16x7x8x0x0x4:clique \
  --variant b8:NIIDMIX_CLIQUE_TILE=8x13x4x64x0x4:clique > gpurun_out/s26/tune.txt 2>&1 || { tail -5 gpurun_out/s26/tune.txt; exit 1; }
cat gpurun_out/s26/tune.txt
timeout -k 10 200 ./tools/hbm_probe5 > gpurun_out/s26/probe5.txt 2>&1 || { tail -5 gpurun_out/s26/probe5.txt; exit 1; }
head -3 gpurun_out/s26/probe5.txt
