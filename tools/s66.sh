#!/bin/bash
# ring100 with merged-order row tiles allowed (NIIDMIX_TILE_MIN_NNZ=1): tile kernels vs CSR, hipGraph
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s66; mkdir -p $O
export NIIDMIX_TILE_MIN_NNZ=1
for k in csr-fast tile-fast tile-lds-fast csr-exact tile-exact tile-lds-exact; do
  timeout -k 10 200 python bench.py --config ring100 --kernel $k --steps 500 --warmup 50 --no-cpu-baseline > $O/ring_$k.json 2> $O/ring_$k.err || { tail -5 $O/ring_$k.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ring_$k.json')); print('$k', d['ms_per_step'], d['config']['launch_ms'], d['roofline']['frac'])"
done
