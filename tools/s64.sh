#!/bin/bash
# per-rank stripe round at N = 1, 2, 4, 8 (emulated one rank at a time on one GPU)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s64; mkdir -p $O
timeout -k 10 400 python -u tools/stripe_probe.py --worlds 1,2,4,8 --steps 20 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep -v amdgpu.ids $O/probe.txt | tail -20
