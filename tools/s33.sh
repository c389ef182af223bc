#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s33
cd tools && timeout -k 10 300 python xy_probe.py > ../gpurun_out/s33/xy.txt 2>&1 || { tail -5 ../gpurun_out/s33/xy.txt; exit 1; }
cat ../gpurun_out/s33/xy.txt
