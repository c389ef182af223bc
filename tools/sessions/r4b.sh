#!/bin/bash
# round 4 session B: gpu tests (all), band probe, ring100 bench, whole-round E2E, 10k block widths,
# node shards under the smallworld interclique
out=gpurun_out/r4b
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -15 $out/pytest.log; ok $rc || { echo "pytest rc=$rc: stop"; exit $rc; }
timeout -k 10 300 python -u tools/band_probe.py > $out/band_probe.txt 2>&1 || { cat $out/band_probe.txt; exit 3; }
cat $out/band_probe.txt
timeout -k 10 300 python bench.py --config ring100 --no-cpu-baseline > $out/bench_ring.json 2> $out/bench_ring.err || exit 4
cat $out/bench_ring.json
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-step > $out/bench_e2e_step.json 2> $out/bench_e2e_step.err || exit 5
cat $out/bench_e2e_step.json
timeout -k 10 600 python -u tools/q_probe.py --n 10000 --blocks 64,128 --variants 8x13x4x13 --iters 10 --reps 3 > $out/q_probe_blocks.txt 2>&1 || exit 6
grep SUMMARY $out/q_probe_blocks.txt
timeout -k 10 600 python -u tools/shard_probe.py --interclique smallworld --n 10000 --worlds 2,4,8 > $out/shard_probe_smallworld.txt 2>&1 || exit 7
grep "predicted" $out/shard_probe_smallworld.txt
timeout -k 10 600 python -u tools/exact_probe.py --rts 16 --metas seg,mfma --mf-items 2,3,4 --reps 2 > $out/exact_mfitem.txt 2>&1 || exit 8
grep SUMMARY $out/exact_mfitem.txt
exit $rc
