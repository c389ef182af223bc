#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s41; mkdir -p $O
for w in 131072 65536 32768 16384 8192; do
  NIIDMIX_WINDOW=$w timeout -k 10 300 python bench.py --no-cpu-baseline --steps 3 --warmup 1 --e2e > $O/e2e_$w.json 2> $O/e2e_$w.err || { tail -5 $O/e2e_$w.err; exit 1; }
  python -c "import json; d=json.load(open('$O/e2e_$w.json')); print($w, d['e2e'])"
done
