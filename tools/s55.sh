#!/bin/bash
# residual register queue 4 (FL & 32) on gateway-heavy stripes; dcliques10000 with the gateway hint
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s55; mkdir -p $O
timeout -k 10 400 python -u tools/stripe_probe.py --worlds 8,1 --steps 20 --variant def: \
  --variant rq4o8:NIIDMIX_CLIQUE_TILE=16x7x8x64x34x4 --variant rq4o4:NIIDMIX_CLIQUE_TILE=16x7x4x64x34x4 > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
grep world $O/probe.txt
timeout -k 10 300 python bench.py --config dcliques10000 --steps 10 --warmup 2 > $O/b10k.json 2> $O/b10k.err || { tail -5 $O/b10k.err; exit 1; }
python -c "import json; d=json.load(open('$O/b10k.json')); print('10k', d['ms_per_step'], d['roofline']['frac'])"
