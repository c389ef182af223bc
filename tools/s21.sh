#!/bin/bash
# LDS-staged tile kernel: parity + exact-mode timings (tile vs tile-lds, tile heights)
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s21
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "tile_lds" > gpurun_out/s21/pytest_lds.txt 2>&1 || { tail -30 gpurun_out/s21/pytest_lds.txt; exit 1; }
tail -1 gpurun_out/s21/pytest_lds.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s21/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/s21/pytest.txt; [ $rc -ge 1 ] && { grep -E "Error|assert|FAILED" gpurun_out/s21/pytest.txt | head -30; exit $rc; }
timeout -k 10 400 python tools/tune_inproc.py --reps 3 --steps 5 \
  --variant l8:NIIDMIX_TILE_LDS_RT=8:tile-lds-exact --variant l16:NIIDMIX_TILE_LDS_RT=16:tile-lds-exact \
  --variant l32:NIIDMIX_TILE_LDS_RT=32:tile-lds-exact --variant l16f:NIIDMIX_TILE_LDS_RT=16:tile-lds-fast \
  --variant t8:NIIDMIX_TILE_RT=8:tile-exact --variant clique::clique > gpurun_out/s21/tune.txt 2>&1 || { tail -20 gpurun_out/s21/tune.txt; exit 1; }
cat gpurun_out/s21/tune.txt
timeout -k 10 400 python tools/tune_inproc.py --reps 3 --steps 5 --config dcliques1000-smallworld \
  --variant l8:NIIDMIX_TILE_LDS_RT=8:tile-lds-exact --variant l16:NIIDMIX_TILE_LDS_RT=16:tile-lds-exact \
  --variant t8:NIIDMIX_TILE_RT=8:tile-exact --variant clique::clique > gpurun_out/s21/tune_sw.txt 2>&1 || { tail -20 gpurun_out/s21/tune_sw.txt; exit 1; }
cat gpurun_out/s21/tune_sw.txt
