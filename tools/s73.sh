#!/bin/bash
# closing run: full GPU suite + smoke + headline bench + FC-1000 (blocked) bench and its profile passes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s73; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --config fc1000 > $O/bench_fc1000.json 2> $O/bench_fc1000.err || { tail -5 $O/bench_fc1000.err; exit 1; }
cat $O/bench_fc1000.json
BENCH_ARGS="--config fc1000" bash tools/profile_session.sh s73/fc || exit 1
