#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
OUT=gpurun_out/${1:-tune2}; mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -q -x > "$OUT/pytest.log" 2>&1; rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -ge 2 ] && exit $rc
for kv in wave block; do
  export NIIDMIX_CLIQUE_KERNEL=$kv
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 50 --warmup 5 ${BENCH_ARGS:-} > "$OUT/bench_$kv.json" 2> "$OUT/bench_$kv.err" || { echo "$kv failed"; tail -5 "$OUT/bench_$kv.err"; exit 1; }
  python -c "import json; d=json.load(open('$OUT/bench_$kv.json')); print('$kv', d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'], d['config']['stream_copy_GBs'])"
done
