set -e
mkdir -p gpurun_out/s2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k tile > gpurun_out/s2/pytest_tile.log 2>&1; tail -3 gpurun_out/s2/pytest_tile.log
for pad in 0 64 256 1024; do timeout -k 10 120 ./tools/hbm_probe 1000 1048576 $pad > gpurun_out/s2/probe_pad$pad.txt; done
for pad in 0 64 256 1024 4096; do timeout -k 10 120 python bench.py --no-cpu-baseline --ld-pad $pad > gpurun_out/s2/bench_pad$pad.json; done
