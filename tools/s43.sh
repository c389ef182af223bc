#!/bin/bash
# 10000-node d-cliques on ONE GPU (2 x 42 GB slabs), headline bench, blocked vs rowmajor
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s43; mkdir -p $O
timeout -k 10 400 python bench.py --config dcliques10000 --steps 10 --warmup 2 > $O/d10k.json 2> $O/d10k.err || { tail -5 $O/d10k.err; exit 1; }
cat $O/d10k.json
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d['roofline'], d['config']['slab_layout'])"
timeout -k 10 300 python bench.py --no-cpu-baseline --workload grad-clique > $O/grad.json 2> $O/grad.err || { tail -5 $O/grad.err; exit 1; }
python -c "import json; d=json.load(open('$O/grad.json')); print(d['ms_per_step'], d['roofline'], d['config']['slab_layout'])"
