#!/bin/bash
# packed-math tile kernel with uniform-weight positions: parity + exact-mode timings
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s20
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s20/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/s20/pytest.txt; [ $rc -ge 1 ] && { grep -E "Error|assert|FAILED" gpurun_out/s20/pytest.txt | head -30; exit $rc; }
timeout -k 10 400 python tools/tune_inproc.py --reps 3 --steps 5 --variant t8:NIIDMIX_TILE_RT=8:tile-exact \
  --variant t16:NIIDMIX_TILE_RT=16:tile-exact --variant t32:NIIDMIX_TILE_RT=32:tile-exact \
  --variant t16n2:NIIDMIX_TILE_RT=16,NIIDMIX_TILE_NE=2:tile-exact --variant t8n2:NIIDMIX_TILE_RT=8,NIIDMIX_TILE_NE=2:tile-exact \
  --variant clique::clique > gpurun_out/s20/tune.txt 2>&1 || { tail -20 gpurun_out/s20/tune.txt; exit 1; }
cat gpurun_out/s20/tune.txt
timeout -k 10 400 python tools/tune_inproc.py --config fc1000 --reps 2 --steps 3 \
  --variant t16:NIIDMIX_TILE_RT=16:tile-exact --variant t32:NIIDMIX_TILE_RT=32:tile-exact > gpurun_out/s20/tune_fc.txt 2>&1 || { tail -20 gpurun_out/s20/tune_fc.txt; exit 1; }
cat gpurun_out/s20/tune_fc.txt
