#!/bin/bash
# column-stripe multi-GPU partition: GPU parity + per-rank emulated round times
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s52; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 400 python -u tools/stripe_probe.py > $O/probe.txt 2>&1 || { tail -20 $O/probe.txt; exit 1; }
cat $O/probe.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err || { tail -5 $O/bench1.err; exit 1; }
cat $O/bench1.json
