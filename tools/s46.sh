#!/bin/bash
# fused device round (gradient mean + SGD step + mixing): parity over training rounds
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s46; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_gradient.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
