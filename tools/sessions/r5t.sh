#!/bin/bash
# Round 5: bf16x6 dense, loop without the odd-step branch; SCHED 3 vs 5 (hand-ordered groups; loads pinned at
# the top of each K-step): parity under both, then interleaved bench A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5j}; mkdir -p $O; export TMPDIR=/tmp
for sc in 3 5; do
  NIIDMIX_DENSE_B6_SCHED=$sc timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dense" --timeout 200 --timeout-method thread > $O/pytest_sched$sc.log 2>&1 || { echo "pytest sched $sc failed"; tail -20 $O/pytest_sched$sc.log; exit 3; }
  tail -1 $O/pytest_sched$sc.log
done
for rep in 1 2; do
for sc in 3 5; do
  NIIDMIX_DENSE_B6_SCHED=$sc timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel dense --steps 5 --warmup 2 > $O/bench_sched$sc.json 2> $O/bench_sched$sc.err || { echo "bench sched $sc failed"; tail -5 $O/bench_sched$sc.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_sched$sc.json'));r=d['roofline'];print('sched$sc', d['ms_per_step'], r['frac'])"
done; done
echo done
