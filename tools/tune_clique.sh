#!/bin/bash
# Sweep clique-kernel register tiles on the headline config (one GPU session).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
OUT=gpurun_out/${1:-tune}; mkdir -p "$OUT"
for tile in ${TILES:-default 16x7x4 16x7x8 8x13x4 8x13x6 16x8x8 16x8x4}; do
  if [ "$tile" = default ]; then unset NIIDMIX_CLIQUE_TILE; else export NIIDMIX_CLIQUE_TILE=$tile; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps ${STEPS:-50} --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench_$tile.json" 2> "$OUT/bench_$tile.err" || { echo "tile $tile failed"; tail -5 "$OUT/bench_$tile.err"; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/bench_$tile.json')); print('$tile', d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['config']['stream_copy_GBs'])"
done
