#!/bin/bash
# Exact-mode kernels (bit-identical paths) on the headline and the other configs, one GPU session.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
OUT=gpurun_out/${1:-exact}; mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -5 "$OUT/$name.err"; return 1; }; python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['config']['kernel'], d['roofline']['achieved'], d['roofline']['frac'], d['config']['stream_copy_GBs'])"; }
run headline --steps 20 || exit 1
for k in csr-exact tile-exact tile-lds-exact; do run headline_$k --steps 5 --kernel $k || exit 1; done
for rt in 8 32; do NIIDMIX_TILE_RT=$rt run headline_tile_rt$rt --steps 5 --kernel tile-exact || exit 1; done
run smallworld_tile --steps 5 --config dcliques1000-smallworld --kernel tile-exact || exit 1
run ring100 --steps 200 --config ring100 || exit 1
run ring100_exact --steps 200 --config ring100 --kernel csr-exact || exit 1
run fc1000 --steps 5 --config fc1000 || exit 1
run fc1000_tile --steps 2 --warmup 1 --config fc1000 --kernel tile-exact || exit 1
