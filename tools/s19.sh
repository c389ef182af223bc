#!/bin/bash
# gradient averaging on GPU: parity (all -m gpu tests) + grad-clique bench + headline bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s19
timeout -k 10 300 python -u -m pytest tests/test_gpu_gradient.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s19/pytest_grad.txt 2>&1 || { tail -30 gpurun_out/s19/pytest_grad.txt; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s19/pytest.txt 2>&1; rc=$?; tail -3 gpurun_out/s19/pytest.txt; [ $rc -ge 1 ] && { grep -E "Error|assert|FAILED" gpurun_out/s19/pytest.txt | head -30; exit $rc; }
timeout -k 10 300 python bench.py --workload grad-clique --steps 20 --e2e > gpurun_out/s19/grad.json 2>gpurun_out/s19/grad.err || { tail -5 gpurun_out/s19/grad.err; exit 1; }
cat gpurun_out/s19/grad.json
timeout -k 10 300 python bench.py > gpurun_out/s19/bench.json 2>gpurun_out/s19/bench.err || { tail -5 gpurun_out/s19/bench.err; exit 1; }
cat gpurun_out/s19/bench.json
