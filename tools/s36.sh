#!/bin/bash
# VMM-mapped slabs: tests, robustness over allocations, bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s36
timeout -k 10 200 python -u -m pytest tests/test_gpu_memory.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s36/pytest.txt 2>&1 || { tail -30 gpurun_out/s36/pytest.txt; exit 1; }
tail -1 gpurun_out/s36/pytest.txt
ALLOC_VMM=1 ALLOCS=10 timeout -k 10 300 python tools/alloc_probe.py > gpurun_out/s36/alloc_vmm.txt 2>&1 || { tail -5 gpurun_out/s36/alloc_vmm.txt; exit 1; }
cat gpurun_out/s36/alloc_vmm.txt
ALLOCS=4 timeout -k 10 300 python tools/alloc_probe.py > gpurun_out/s36/alloc_hip.txt 2>&1 || { tail -5 gpurun_out/s36/alloc_hip.txt; exit 1; }
cat gpurun_out/s36/alloc_hip.txt
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/s36/bench.json 2> gpurun_out/s36/bench.err || { tail -5 gpurun_out/s36/bench.err; exit 1; }
cat gpurun_out/s36/bench.json
