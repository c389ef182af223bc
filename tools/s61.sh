#!/bin/bash
# ring100 (configs[1]): every kernel variant on the same box, hipGraph, to pick the latency-bound config's kernel
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s61; mkdir -p $O
for k in csr-fast csr-exact tile-fast tile-exact tile-lds-fast tile-lds-exact staged-fast staged-exact; do
  timeout -k 10 200 python bench.py --config ring100 --kernel $k --steps 200 --warmup 20 --no-cpu-baseline > $O/ring_$k.json 2> $O/ring_$k.err || { tail -5 $O/ring_$k.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/ring_$k.json')); print('$k', d['ms_per_step'], d['config']['launch_ms'], d['roofline']['frac'])"
done
