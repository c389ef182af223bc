#!/bin/bash
# ring100: hipGraph on/off, CSR fast, 2 reps
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s67; mkdir -p $O
for rep in 1 2; do for g in on off; do
  timeout -k 10 200 python bench.py --config ring100 --kernel csr-fast --graph $g --steps 500 --warmup 50 --no-cpu-baseline > $O/ring_$g.json 2> $O/ring_$g.err || { tail -5 $O/ring_$g.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ring_$g.json')); print('graph $g', d['ms_per_step'], d['config']['launch_ms'], d['config']['stream_copy_GBs'], d['roofline']['frac'])"
done; done
