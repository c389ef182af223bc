#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s35
timeout -k 10 150 ./tools/hbm_probe7 > gpurun_out/s35/probe7.txt 2>&1 || { tail -5 gpurun_out/s35/probe7.txt; exit 1; }
cat gpurun_out/s35/probe7.txt
