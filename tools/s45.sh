#!/bin/bash
# blocked layout block width sweep, 2 fresh processes each, same box
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s45; mkdir -p $O
for i in 1 2; do for b in 1024 2048 4096 8192 16384; do
  NIIDMIX_BLOCK_COLS=$b timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 > $O/b_${b}_$i.json 2> $O/b_${b}_$i.err || { tail -5 $O/b_${b}_$i.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_${b}_$i.json')); print($b, $i, d['ms_per_step'], d['roofline']['frac'], d['config']['slab_layout'], d['config']['stream_copy_GBs'])"
done; done
