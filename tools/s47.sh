#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s47; mkdir -p $O
timeout -k 10 400 python bench.py --workload grad-clique --e2e --no-cpu-baseline --steps 5 > $O/grad_e2e.json 2> $O/grad_e2e.err || { tail -8 $O/grad_e2e.err; exit 1; }
python -c "import json; d=json.load(open('$O/grad_e2e.json')); print(d['ms_per_step'], d['e2e'])"
