#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s24
timeout -k 10 300 python tools/blocked_probe.py > gpurun_out/s24/blocked.txt 2>&1 || { tail -20 gpurun_out/s24/blocked.txt; exit 1; }
cat gpurun_out/s24/blocked.txt
