#!/bin/bash
# round 4 session N: plain row-streamed round steps each node right after its backward
out=gpurun_out/r4n
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_dropin.py tests/test_gpu_gradient.py -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
timeout -k 10 900 python bench.py --no-cpu-baseline --e2e-step --steps 3 > $out/bench_e2e_step.json 2> $out/bench_e2e_step.err || { tail -5 $out/bench_e2e_step.err; exit 2; }
python -c "import json;d=json.load(open('$out/bench_e2e_step.json'));print(json.dumps(d['e2e']['next_step'], indent=0))"
