#!/bin/bash
# big-clique one-pass kernel: non-temporal vs plain row loads, blocked (bench) and row-major (A/B tool)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s76; mkdir -p $O
timeout -k 10 300 python -u tools/ab_clique.py --config fc1000 --env NIIDMIX_BIGREG_LOADS --variants nt,plain --reps 5 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -2 $O/ab.txt
for rep in 1 2; do for m in nt plain; do
NIIDMIX_BIGREG_LOADS=$m timeout -k 10 300 python bench.py --config fc1000 --no-cpu-baseline > $O/bench_fc_$m.json 2> $O/bench_fc_$m.err || { tail -5 $O/bench_fc_$m.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_fc_$m.json')); print('$m', d['ms_per_step'], d['config']['slab_layout'], d['roofline']['frac'])"
done; done
NIIDMIX_BIGREG_LOADS=plain timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bigclique or fc1000" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
