#!/bin/bash
# Round 5: the whole-round E2E alone (exposed cost against the pinned-slab CPU baseline).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5k}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u bench.py --no-cpu-baseline --e2e-step --steps 3 > $O/bench_e2e.json 2> $O/bench_e2e.err || { echo e2e failed; tail $O/bench_e2e.err; exit 6; }
python -c "import json;d=json.load(open('$O/bench_e2e.json'));print(json.dumps(d.get('e2e'), indent=1))"
echo done
