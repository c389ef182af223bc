#!/bin/bash
# Round 5: bf16x6 dense, one wave per SIMD (NIIDMIX_DENSE_B6_W1=1) vs the two-wave kernel:
# bitwise test and dense parity under both, then an interleaved bench A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5p}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "one_wave" --timeout 200 --timeout-method thread > $O/pytest_bitwise.log 2>&1 || { echo "bitwise test failed"; tail -30 $O/pytest_bitwise.log; exit 3; }
tail -1 $O/pytest_bitwise.log
NIIDMIX_DENSE_B6_W1=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dense" --timeout 200 --timeout-method thread > $O/pytest_w1.log 2>&1 || { echo "pytest w1 failed"; tail -20 $O/pytest_w1.log; exit 3; }
tail -1 $O/pytest_w1.log
for rep in 1 2; do
for v in 0 1; do
  NIIDMIX_DENSE_B6_W1=$v timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel dense --steps 5 --warmup 2 > $O/bench_w1_$v.json 2> $O/bench_w1_$v.err || { echo "bench w1 $v failed"; tail -5 $O/bench_w1_$v.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_w1_$v.json'));r=d['roofline'];print('w1=$v', d['ms_per_step'], r['frac'])"
done; done
echo done
