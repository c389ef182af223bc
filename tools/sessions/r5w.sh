#!/bin/bash
# Round 5: the driver's default N > 1 command rehearsed with gloo on the final library (both ranks
# on this one GPU; timings not meaningful): the stripes line, config.world, both node-shard legs
# with their xgmi (exchange-only) records.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5w}; mkdir -p $O; export TMPDIR=/tmp
NIIDMIX_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --steps 5 --warmup 2 > $O/gloo2_default.json 2> $O/gloo2_default.err || { echo "gloo rehearsal failed"; tail -5 $O/gloo2_default.err; exit 1; }
python -c "
import json
d = json.loads([l for l in open('$O/gloo2_default.json') if l.startswith('{')][-1])
w = d['config'].get('world', {})
print('gloo2', d['n_gpus'], d['ms_per_step'], d['config']['lib_sha16'], w.get('backend'), w.get('world_size'), w.get('distinct_devices'))
for l in d['config']['node_shards']:
    print(l['interclique'], l.get('ms_per_step'), l.get('error'), json.dumps(l.get('xgmi'))[:300])
"
