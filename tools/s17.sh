#!/bin/bash
# tile kernel: GPU parity + first timings
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/s17_pytest.log 2>&1; rc=$?; tail -2 gpurun_out/s17_pytest.log; [ $rc -ge 1 ] && { grep -E "Error|assert|FAILED" gpurun_out/s17_pytest.log | head -30; exit $rc; }
timeout -k 10 400 python tools/tune_inproc.py --reps 3 --steps 5 --variant csr::csr-exact \
  --variant t8:NIIDMIX_TILE_RT=8:tile-exact --variant t16:NIIDMIX_TILE_RT=16:tile-exact \
  --variant t16n2:NIIDMIX_TILE_RT=16,NIIDMIX_TILE_NE=2:tile-exact --variant t32:NIIDMIX_TILE_RT=32:tile-exact \
  --variant t8n2:NIIDMIX_TILE_RT=8,NIIDMIX_TILE_NE=2:tile-exact \
  --variant t16f:NIIDMIX_TILE_RT=16:tile-fast --variant clique::clique || exit 1
timeout -k 10 400 python tools/tune_inproc.py --config fc1000 --reps 2 --steps 3 --variant csr::csr-exact \
  --variant t16:NIIDMIX_TILE_RT=16:tile-exact --variant t32:NIIDMIX_TILE_RT=32:tile-exact --variant dense::dense || exit 1
