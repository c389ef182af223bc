#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s25
timeout -k 10 200 ./tools/hbm_probe5 > gpurun_out/s25/probe5.txt 2>&1 || { tail -5 gpurun_out/s25/probe5.txt; exit 1; }
head -17 gpurun_out/s25/probe5.txt
timeout -k 10 300 python tools/tune_inproc.py --reps 3 --steps 10 --variant clique::clique > gpurun_out/s25/tune.txt 2>&1 || { tail -5 gpurun_out/s25/tune.txt; exit 1; }
cat gpurun_out/s25/tune.txt
