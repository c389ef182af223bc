#!/bin/bash
# round 4 session Q: the strip kernel auto-selected on a 256-B row pitch (ring 100); full GPU suite
out=gpurun_out/r4q
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
timeout -k 10 300 python bench.py --config ring100 --steps 200 --no-cpu-baseline > $out/bench_ring.json 2> $out/bench_ring.err || exit 2
python -c "import json;d=json.load(open('$out/bench_ring.json'));print('ring', d['ms_per_step'], d['config']['kernel'], d['config']['slab_layout'], d['config'].get('cold_cache_round'))"
