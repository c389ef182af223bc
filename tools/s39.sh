#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s38; mkdir -p $O/cfg
run() { local name=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > "$O/cfg/$name.json" 2> "$O/cfg/$name.err" || { echo "$name failed"; tail -5 "$O/cfg/$name.err"; return 1; }; python -c "import json; d=json.load(open('$O/cfg/$name.json')); print('$name', d['ms_per_step'], d['value'], d['config']['kernel'], d['roofline']['achieved'], d['roofline']['unit'], d['roofline']['frac'])"; }
run fc1000_auto --steps 10 --config fc1000 || exit 1
run fc1000_dense --steps 3 --warmup 1 --config fc1000 --kernel dense || exit 1
run headline_tile_exact --steps 5 --kernel tile-exact || exit 1
run smallworld_exact --steps 5 --config dcliques1000-smallworld --kernel tile-lds-exact || exit 1
timeout -k 10 300 python bench.py --workload grad-clique --steps 20 --e2e > $O/grad.json 2> $O/grad.err || { tail -5 $O/grad.err; exit 1; }
cat $O/grad.json
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
