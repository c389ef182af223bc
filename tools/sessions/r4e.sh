#!/bin/bash
# round 4 session E: register rows in the exact tiles (10 000 nodes): tests, then bench A/B
out=gpurun_out/r4e
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize_10k.py -k "register_rows or tile_lds_exact_rowmajor or tile_lds" -m gpu -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -4 $out/pytest.log; ok $rc || { echo "pytest rc=$rc: stop"; exit $rc; }
[ $rc -eq 0 ] || { grep FAILED $out/pytest.log | head; exit 1; }
for r in auto 0; do
  NIIDMIX_TLDS_REMOTE=$r timeout -k 10 600 python bench.py --config dcliques10000 --kernel tile-lds-exact --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_exact10k_remote_$r.json 2> $out/bench_exact10k_remote_$r.err || exit 5
  python -c "import json;d=json.load(open('$out/bench_exact10k_remote_$r.json'));print('remote=$r', d['ms_per_step'], 'ms', d['roofline']['frac'])"
done
timeout -k 10 300 python bench.py --kernel tile-lds-exact --steps 10 --no-cpu-baseline > $out/bench_exact_headline.json 2> $out/bench_exact_headline.err || exit 6
python -c "import json;d=json.load(open('$out/bench_exact_headline.json'));print('headline exact', d['ms_per_step'], 'ms', d['roofline']['frac'])"
NIIDMIX_TLDS_REMOTE=1 timeout -k 10 300 python bench.py --kernel tile-lds-exact --steps 10 --no-cpu-baseline > $out/bench_exact_headline_rem.json 2> $out/bench_exact_headline_rem.err || exit 7
python -c "import json;d=json.load(open('$out/bench_exact_headline_rem.json'));print('headline exact remote=1', d['ms_per_step'], 'ms', d['roofline']['frac'])"
timeout -k 10 300 python bench.py --config ring100 --steps 200 --no-cpu-baseline > $out/bench_ring_cold.json 2> $out/bench_ring_cold.err || exit 8
python -c "import json;d=json.load(open('$out/bench_ring_cold.json'));print('ring', d['ms_per_step'], d['config'].get('cold_cache_round'))"
# the driver's default N > 1 command, rehearsed with gloo (both ranks on this one GPU; timings not meaningful)
NIIDMIX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $out/gloo2_default.json 2> $out/gloo2_default.err || { echo "gloo rehearsal rc=$?"; tail -5 $out/gloo2_default.err; exit 9; }
python -c "import json;d=json.load(open('$out/gloo2_default.json'));print('gloo2', d['ms_per_step'], [(l['interclique'], l.get('ms_per_step'), l.get('error')) for l in d['config']['node_shards']])"
