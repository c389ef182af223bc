#!/bin/bash
# LDS tile kernel with a copy-free double buffer: parity + timings per tile height; gradient rounds
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s42
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dropin.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tile_lds or clique_gradient or training" > gpurun_out/s42/pytest.txt 2>&1 || { tail -30 gpurun_out/s42/pytest.txt; exit 1; }
tail -1 gpurun_out/s42/pytest.txt
timeout -k 10 400 python tools/tune_inproc.py --reps 3 --steps 5 --variant l8:NIIDMIX_TILE_LDS_RT=8:tile-lds-exact \
  --variant l16:NIIDMIX_TILE_LDS_RT=16:tile-lds-exact --variant l32:NIIDMIX_TILE_LDS_RT=32:tile-lds-exact > gpurun_out/s42/tune.txt 2>&1 || { tail -20 gpurun_out/s42/tune.txt; exit 1; }
cat gpurun_out/s42/tune.txt
