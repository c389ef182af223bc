#!/bin/bash
# after the per-layout item map: full GPU suite, smoke, FC-1000 bench (blocked), row-major A/B vs two-pass, headline bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s75; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py --config fc1000 > $O/bench_fc1000.json 2> $O/bench_fc1000.err || { tail -5 $O/bench_fc1000.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_fc1000.json')); print('fc1000', d['ms_per_step'], d['config']['slab_layout'], d['roofline'])"
timeout -k 10 300 python -u tools/ab_clique.py --config fc1000 --env NIIDMIX_BIG --variants reg,8x16 --reps 5 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -2 $O/ab.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
