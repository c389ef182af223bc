#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/s16_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/s16_pytest.log; [ $rc -ge 1 ] && { grep -E "Error|assert|FAILED" gpurun_out/s16_pytest.log | head -20; exit $rc; }
for a in "--config ring100 --steps 200" "--config ring100 --steps 200 --kernel csr-exact" "--steps 5 --kernel csr-exact" "--steps 5 --kernel csr-fast" "--steps 20"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline $a > gpurun_out/s16_b.json 2>gpurun_out/s16_b.err || { tail -5 gpurun_out/s16_b.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/s16_b.json')); print(d['config']['workload'][:20], d['config']['kernel'], d['config']['hipgraph'], d['ms_per_step'], d['value'], d['roofline']['achieved'], d['roofline']['frac'])"
done
timeout -k 10 400 python tools/tune_inproc.py --reps 3 --variant def::clique --variant nt16:NIIDMIX_CLIQUE_TILE=16x7x8x0x2:clique --variant b8:NIIDMIX_CLIQUE_TILE=8x13x4x0x0:clique --variant nt8:NIIDMIX_CLIQUE_TILE=8x13x4x0x2:clique
