#!/bin/bash
# one-pass register-resident big-clique kernel: parity, A/B vs the two-pass kernel on FC-1000, bench line
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s71; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "bigclique or fc1000 or many_gateways" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 300 python -u tools/ab_clique.py --config fc1000 --env NIIDMIX_BIG --variants reg,8x16 --reps 5 > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
tail -5 $O/ab.txt
timeout -k 10 400 python bench.py --config fc1000 --no-cpu-baseline > $O/bench_fc.json 2> $O/bench_fc.err || { tail -5 $O/bench_fc.err; exit 1; }
cat $O/bench_fc.json
