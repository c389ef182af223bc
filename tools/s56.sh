#!/bin/bash
# rehearse bench.py --gpus 2 (column stripes) as two ranks on the one GPU over gloo
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s56; mkdir -p $O
export NIIDMIX_BENCH_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 > $O/b2.json 2> $O/b2.err || { tail -20 $O/b2.err; exit 1; }
cat $O/b2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --steps 5 --warmup 2 --kernel tile-lds-exact > $O/b2e.json 2> $O/b2e.err || { tail -20 $O/b2e.err; exit 1; }
cat $O/b2e.json
