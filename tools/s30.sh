#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s30
timeout -k 10 300 python tools/alloc_probe.py > gpurun_out/s30/alloc.txt 2>&1 || { tail -5 gpurun_out/s30/alloc.txt; exit 1; }
cat gpurun_out/s30/alloc.txt
