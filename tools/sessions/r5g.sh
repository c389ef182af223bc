#!/bin/bash
# Round 5: whole GPU suite on the current library, smoke, headline bench, then the whole-round E2E
# (row-streamed, paced write-back, logger costs).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5g}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "FAILED" $O/pytest_gpu.log | head
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_headline.json 2> $O/bench_headline.err || { echo bench failed; tail $O/bench_headline.err; exit 4; }
python -c "import json;d=json.load(open('$O/bench_headline.json'));print('headline', d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 900 python -u bench.py --no-cpu-baseline --e2e-step --steps 3 > $O/bench_e2e.json 2> $O/bench_e2e.err || { echo e2e failed; tail $O/bench_e2e.err; exit 6; }
python -c "import json;d=json.load(open('$O/bench_e2e.json'));print(json.dumps(d.get('e2e'), indent=1))"
echo done
