#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/s13_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/s13_pytest.log; [ $rc -ge 1 ] && { grep -E "Error|assert|FAILED" gpurun_out/s13_pytest.log | head -20; exit $rc; }
for a in "--steps 5 --kernel staged-exact" "--steps 5 --kernel staged-fast" "--config fc1000 --steps 10" "--config fc1000 --steps 3 --warmup 1 --kernel dense" "--config ring100 --steps 200 --kernel staged-fast" "--steps 20"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/s13_b.json 2>gpurun_out/s13_b.err || { tail -5 gpurun_out/s13_b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s13_b.json')); print(d['config']['workload'][:30], d['config']['kernel'], d['config']['hipgraph'], d['ms_per_step'], d['value'], d['roofline']['achieved'], d['roofline']['frac'])"
done
