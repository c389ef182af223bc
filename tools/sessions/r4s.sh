#!/bin/bash
# round 4 session S: pipelined two-half strip kernel (ring 100 on a 256-B row pitch): strip tests,
# the probe sweep against the one-piece kernel, the ring bench line
out=gpurun_out/r4s
mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_band.py -x -q --timeout 120 --timeout-method thread > $out/pytest_band.log 2>&1
rc=$?; tail -2 $out/pytest_band.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest_band.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
timeout -k 10 300 python tools/band_probe.py > $out/band_probe.txt 2>&1 || { tail $out/band_probe.txt; exit 2; }
cat $out/band_probe.txt
timeout -k 10 300 python bench.py --config ring100 --steps 200 --no-cpu-baseline > $out/bench_ring.json 2> $out/bench_ring.err || exit 3
python -c "import json;d=json.load(open('$out/bench_ring.json'));print('ring', d['ms_per_step'], d['config']['kernel'], d['config']['slab_layout'], d['config'].get('cold_cache_round'))"
