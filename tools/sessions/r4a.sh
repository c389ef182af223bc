#!/bin/bash
# round 4 session A: gpu tests, default bench, ring100 (band kernel), whole-round E2E
out=gpurun_out/r4a
mkdir -p $out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -5 $out/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stop"; exit $rc; fi
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err || exit $?
cat $out/bench.json
timeout -k 10 300 python bench.py --config ring100 --no-cpu-baseline > $out/bench_ring.json 2> $out/bench_ring.err || exit $?
cat $out/bench_ring.json
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-step > $out/bench_e2e_step.json 2> $out/bench_e2e_step.err || exit $?
cat $out/bench_e2e_step.json
exit $rc
