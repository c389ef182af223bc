#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s68; mkdir -p $O
timeout -k 10 200 python -u tools/ring_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep ring100 $O/probe.txt
timeout -k 10 200 python -u tools/ring_probe.py >> $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep ring100 $O/probe.txt | tail -1
