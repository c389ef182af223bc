#!/bin/bash
# round 4 session P: column-strip kernel for few nodes (ring 100)
out=gpurun_out/r4p
mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_band.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
timeout -k 10 300 python -u tools/band_probe.py --rc 4,1:2,2 --steps 20 --reps 5 > $out/band_probe.txt 2>&1 || { tail -5 $out/band_probe.txt; exit 2; }
cat $out/band_probe.txt
