#!/bin/bash
# one-pass big-clique kernel on column-blocked slabs: parity, FC-1000 bench (blocked default) and row-major
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s72; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bigclique or fc1000 or many_gateways" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for rep in 1 2; do for lay in blocked rowmajor; do
timeout -k 10 300 python bench.py --config fc1000 --layout $lay --no-cpu-baseline > $O/bench_fc_$lay.json 2> $O/bench_fc_$lay.err || { tail -5 $O/bench_fc_$lay.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_fc_$lay.json')); print('$lay', d['ms_per_step'], d['config']['slab_layout'], d['roofline']['frac'])"
done; done
