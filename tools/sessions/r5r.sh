#!/bin/bash
# Round 5: whole-round E2E with 16 vs 15 torch threads for the training (one core left to the HIP
# runtime), same box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5r}; mkdir -p $O; export TMPDIR=/tmp
for t in 16 15; do
  timeout -k 10 900 python -u bench.py --no-cpu-baseline --e2e-step --e2e-threads $t --steps 3 > $O/bench_e2e_t$t.json 2> $O/bench_e2e_t$t.err || { echo "e2e $t failed"; tail $O/bench_e2e_t$t.err; exit 6; }
  python -c "import json;d=json.load(open('$O/bench_e2e_t$t.json'))['e2e']['next_step'];print('t$t', d['threads'], {k: (v.get('round_ms'), v.get('exposed_ms'), v.get('host_blocked_ms')) for k, v in d.items() if isinstance(v, dict) and 'round_ms' in v})"
done
echo done
