#!/bin/bash
# round 4 session Y: the driver's default N > 1 command rehearsed with gloo on the final library
# (both ranks on this one GPU; timings not meaningful), plus --config dcliques10000 at N = 2
out=gpurun_out/r4y
mkdir -p $out
NIIDMIX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 > $out/gloo2_default.json 2> $out/gloo2_default.err || { echo "gloo rehearsal failed"; tail -5 $out/gloo2_default.err; exit 1; }
python -c "import json;d=json.loads([l for l in open('$out/gloo2_default.json') if l.startswith('{')][-1]);print('gloo2', d['n_gpus'], d['ms_per_step'], d['config']['lib_sha16'], [(l['interclique'], l.get('ms_per_step'), l.get('error')) for l in d['config']['node_shards']])"
