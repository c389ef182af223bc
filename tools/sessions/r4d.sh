#!/bin/bash
# round 4 session D: exact matrix-core path software-pipelined: bitwise tests, then A/B
out=gpurun_out/r4d
mkdir -p $out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "tile_lds" -m gpu -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -4 $out/pytest.log; ok $rc || { echo "pytest rc=$rc: stop"; exit $rc; }
[ $rc -eq 0 ] || { grep FAILED $out/pytest.log | head; exit 1; }
timeout -k 10 600 python -u tools/exact_probe.py --rts 16 --metas seg,mfma --mf-items 3,5,7 --reps 2 > $out/exact_mfma_pipelined.txt 2>&1 || exit 8
grep SUMMARY $out/exact_mfma_pipelined.txt
