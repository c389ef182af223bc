#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s27
timeout -k 10 300 python tools/tune_inproc.py --reps 5 --steps 20 --variant def::clique \
  --variant nt:NIIDMIX_CLIQUE_TILE=16x7x8x64x2x4:clique --variant nt_nores:NIIDMIX_CLIQUE_TILE=16x7x8x64x6x4:clique \
  --variant nt_nored:NIIDMIX_CLIQUE_TILE=16x7x8x64x10x4:clique --variant nt_none:NIIDMIX_CLIQUE_TILE=16x7x8x64x14x4:clique > gpurun_out/s27/tune.txt 2>&1 || { tail -5 gpurun_out/s27/tune.txt; exit 1; }
cat gpurun_out/s27/tune.txt
timeout -k 10 200 ./tools/hbm_probe5 > gpurun_out/s27/probe5.txt 2>&1 || { tail -5 gpurun_out/s27/probe5.txt; exit 1; }
head -3 gpurun_out/s27/probe5.txt
