#!/bin/bash
# re-entry check after container re-creation: full GPU suite + smoke + headline bench + kernel-trace stats
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s59; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/$O/prof" -o run -- python3 "$R/bench.py" --steps 20 > "$R/$O/prof_bench.json" 2> "$R/$O/prof.err" || { tail -5 "$R/$O/prof.err"; exit 1; }
cat "$R/$O/prof_bench.json"
find "$R/$O/prof" -name '*kernel_stats.csv' | head -3
