#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s31
PADS=0,128,256,512,768,256 PAD_REPS=3 timeout -k 10 300 python tools/alloc_probe.py > gpurun_out/s31/alloc.txt 2>&1 || { tail -5 gpurun_out/s31/alloc.txt; exit 1; }
cat gpurun_out/s31/alloc.txt
