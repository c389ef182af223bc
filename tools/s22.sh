#!/bin/bash
# LDS tile kernel v2 (lane-parallel uniform weights, double-buffered LDS reads): parity + timings
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s22
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tile_lds or auto_kernel" > gpurun_out/s22/pytest_lds.txt 2>&1 || { tail -30 gpurun_out/s22/pytest_lds.txt; exit 1; }
tail -1 gpurun_out/s22/pytest_lds.txt
timeout -k 10 400 python tools/tune_inproc.py --reps 3 --steps 5 \
  --variant l8:NIIDMIX_TILE_LDS_RT=8:tile-lds-exact --variant l16:NIIDMIX_TILE_LDS_RT=16:tile-lds-exact \
  --variant l32:NIIDMIX_TILE_LDS_RT=32:tile-lds-exact --variant l8f:NIIDMIX_TILE_LDS_RT=8:tile-lds-fast \
  --variant l16f:NIIDMIX_TILE_LDS_RT=16:tile-lds-fast \
  --variant t8:NIIDMIX_TILE_RT=8:tile-exact --variant clique::clique > gpurun_out/s22/tune.txt 2>&1 || { tail -20 gpurun_out/s22/tune.txt; exit 1; }
cat gpurun_out/s22/tune.txt
