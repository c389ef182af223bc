#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_shard.py -q -x > gpurun_out/s9_pytest.log 2>&1; rc=$?; tail -4 gpurun_out/s9_pytest.log; [ $rc -ge 2 ] && exit $rc
for a in "--config ring100 --steps 200" "--config ring100 --steps 200 --kernel csr-exact" "--config ring100 --steps 200 --graph off" "--steps 20"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/s9_b.json 2>gpurun_out/s9_b.err || { tail -5 gpurun_out/s9_b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s9_b.json')); print(d['config']['kernel'], d['config']['hipgraph'], d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
