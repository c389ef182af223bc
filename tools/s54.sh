#!/bin/bash
# gateway-row load hint (temporal loads for rows re-gathered as residual terms): A/B on stripes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s54; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_shard.py tests/test_gpu_memory.py -m gpu -x -q --timeout 120 --timeout-method thread -k "clique or stripe or blocked" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
V="--variant def: --variant nt0:NIIDMIX_CLIQUE_TILE=16x7x8x64x0x4"
timeout -k 10 400 python -u tools/stripe_probe.py --worlds 8,2,1 --steps 20 $V > $O/hint.txt 2>&1 || { tail -20 $O/hint.txt; exit 1; }
NIIDMIX_GATEWAY_HINT=0 timeout -k 10 400 python -u tools/stripe_probe.py --worlds 8,2,1 --steps 20 $V > $O/nohint.txt 2>&1 || { tail -20 $O/nohint.txt; exit 1; }
echo HINT; grep world $O/hint.txt; echo NOHINT; grep world $O/nohint.txt
