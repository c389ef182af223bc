#!/bin/bash
# round 4 session F: walker-only kernel split from the matrix-core path (64 VGPRs), 12/8/4-row
# loops, 8-register-row kernel; full GPU suite, exact A/B, ring cold cache, gloo 2-rank rehearsal
out=gpurun_out/r4f
mkdir -p $out
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -4 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; echo "pytest rc=$rc: stop"; exit 1; }
timeout -k 10 400 python -u tools/exact_probe.py --rts 16 --metas seg,seg16,rem8,rem16 --reps 3 > $out/exact_probe.txt 2>&1 || { tail -5 $out/exact_probe.txt; exit 2; }
grep SUMMARY $out/exact_probe.txt
for v in auto16:1 small0:0; do
  tag=${v%%:*}; sm=${v##*:}
  NIIDMIX_TLDS_SMALL=$sm timeout -k 10 600 python bench.py --config dcliques10000 --kernel tile-lds-exact --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_exact10k_$tag.json 2> $out/bench_exact10k_$tag.err || exit 3
  python -c "import json;d=json.load(open('$out/bench_exact10k_$tag.json'));print('10k exact $tag', d['ms_per_step'], 'ms', d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --kernel tile-lds-exact --steps 20 --no-cpu-baseline > $out/bench_exact_headline.json 2> $out/bench_exact_headline.err || exit 4
python -c "import json;d=json.load(open('$out/bench_exact_headline.json'));print('headline exact', d['ms_per_step'], 'ms', d['roofline']['frac'])"
timeout -k 10 300 python bench.py --config ring100 --steps 200 --no-cpu-baseline > $out/bench_ring_cold.json 2> $out/bench_ring_cold.err || exit 5
python -c "import json;d=json.load(open('$out/bench_ring_cold.json'));print('ring', d['ms_per_step'], d['config'].get('cold_cache_round'))"
# the driver's default N > 1 command, rehearsed with gloo (both ranks on this one GPU; timings not meaningful)
NIIDMIX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $out/gloo2_default.json 2> $out/gloo2_default.err || { echo "gloo rehearsal failed"; tail -5 $out/gloo2_default.err; exit 6; }
python -c "import json;d=json.load(open('$out/gloo2_default.json'));print('gloo2', d['ms_per_step'], [(l['interclique'], l.get('ms_per_step'), l.get('error')) for l in d['config']['node_shards']])"
