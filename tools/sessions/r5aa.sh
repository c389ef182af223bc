#!/bin/bash
# Round 5: clique-gradient mean with non-temporal member loads (NIIDMIX_GRAD_NT=1) vs default:
# gradient parity under both, interleaved bench A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5aa}; mkdir -p $O; export TMPDIR=/tmp
NIIDMIX_GRAD_NT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_gradient.py -m gpu -q --timeout 200 --timeout-method thread > $O/pytest_nt.log 2>&1 || { echo "pytest nt failed"; tail -20 $O/pytest_nt.log; exit 3; }
tail -1 $O/pytest_nt.log
for rep in 1 2 3; do
for v in 0 1; do
  NIIDMIX_GRAD_NT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --workload grad-clique --steps 10 > $O/bench_nt$v.json 2> $O/bench_nt$v.err || { echo "bench nt $v failed"; tail -5 $O/bench_nt$v.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_nt$v.json'));r=d['roofline'];print('nt$v', d['ms_per_step'], r['frac'])"
done; done
echo done
