#!/bin/bash
# Round 5: whole-round E2E with the copies on the SDMA engines (default) and on blit kernels
# (HSA_ENABLE_SDMA=0), same box, one after the other.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5n}; mkdir -p $O; export TMPDIR=/tmp
for v in sdma blit; do
  if [ $v = blit ]; then export HSA_ENABLE_SDMA=0; fi
  timeout -k 10 900 python -u bench.py --no-cpu-baseline --e2e-step --steps 3 > $O/bench_e2e_$v.json 2> $O/bench_e2e_$v.err || { echo "e2e $v failed"; tail $O/bench_e2e_$v.err; exit 6; }
  python -c "import json;d=json.load(open('$O/bench_e2e_$v.json'))['e2e']['next_step'];print('$v', {k: (v.get('round_ms'), v.get('exposed_ms'), v.get('host_blocked_ms')) for k, v in d.items() if isinstance(v, dict) and 'round_ms' in v})"
done
echo done
