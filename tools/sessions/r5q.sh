#!/bin/bash
# Round 5: clique-gradient mean, loads in flight per thread (NIIDMIX_GRAD_U 4 / 8 / 16), interleaved.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5q}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
for u in 8 16 4; do
  NIIDMIX_GRAD_U=$u timeout -k 10 300 python bench.py --no-cpu-baseline --workload grad-clique --steps 10 > $O/bench_u$u.json 2> $O/bench_u$u.err || { echo "bench u $u failed"; tail -5 $O/bench_u$u.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_u$u.json'));r=d['roofline'];print('u$u', d['ms_per_step'], r['frac'])"
done; done
echo done
