#!/bin/bash
# full GPU suite + smoke + headline bench + ring100 / fc1000 bench lines after the big-clique and CSR-width changes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s70; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 200 python bench.py --config ring100 --steps 500 --warmup 50 > $O/bench_ring100.json 2> $O/bench_ring100.err || { tail -5 $O/bench_ring100.err; exit 1; }
cat $O/bench_ring100.json
timeout -k 10 300 python bench.py --config fc1000 > $O/bench_fc1000.json 2> $O/bench_fc1000.err || { tail -5 $O/bench_fc1000.err; exit 1; }
cat $O/bench_fc1000.json
