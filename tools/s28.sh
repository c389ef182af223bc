#!/bin/bash
# clique kernel: residual descriptors fetched with the member descriptors; NT member loads default
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s28
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s28/pytest.txt 2>&1 || { tail -30 gpurun_out/s28/pytest.txt; exit 1; }
tail -1 gpurun_out/s28/pytest.txt
timeout -k 10 300 python tools/tune_inproc.py --reps 5 --steps 20 --variant def::clique \
  --variant old_nont:NIIDMIX_CLIQUE_TILE=16x7x8x64x0x4:clique --variant nores:NIIDMIX_CLIQUE_TILE=16x7x8x64x6x4:clique > gpurun_out/s28/tune.txt 2>&1 || { tail -5 gpurun_out/s28/tune.txt; exit 1; }
cat gpurun_out/s28/tune.txt
timeout -k 10 300 python tools/tune_inproc.py --config dcliques1000-smallworld --reps 3 --steps 20 --variant def::clique \
  --variant nores:NIIDMIX_CLIQUE_TILE=16x7x8x64x6x4:clique > gpurun_out/s28/tune_sw.txt 2>&1 || { tail -5 gpurun_out/s28/tune_sw.txt; exit 1; }
cat gpurun_out/s28/tune_sw.txt
