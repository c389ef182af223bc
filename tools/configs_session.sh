#!/bin/bash
# Measure the other BASELINE configs + the host-resident (E2E) round, one GPU session.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
OUT=gpurun_out/${1:-cfg}; mkdir -p "$OUT"
run() { local name=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > "$OUT/$name.json" 2> "$OUT/$name.err" || { echo "$name failed"; tail -5 "$OUT/$name.err"; return 1; }; python -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['ms_per_step'], d['value'], d['config']['kernel'], d['roofline']['achieved'], d['roofline']['unit'], d['roofline']['frac'], d.get('e2e'))"; }
run headline_e2e --steps 20 --e2e || exit 1
run headline_exact --steps 5 --kernel tile-lds-exact || exit 1
run headline_csr_exact --steps 5 --kernel csr-exact || exit 1
run smallworld --steps 20 --config dcliques1000-smallworld || exit 1
run ring100 --steps 200 --config ring100 || exit 1
run ring100_exact --steps 200 --config ring100 --kernel csr-exact || exit 1
run fc1000_dense --steps 3 --warmup 1 --config fc1000 --kernel dense || exit 1
