#!/bin/bash
# Round 5: the bf16x6 dense GEMM -- parity tests, then bench A/B against the fp32 MFMA kernel.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/r5b; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "dense" > $O/dense_tests.log 2>&1
rc=$?; echo "dense tests rc=$rc"; grep -E "PASS|FAIL|Error|assert" $O/dense_tests.log | tail -25
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
  tests/test_gpu_fullsize.py -k "dense" > $O/dense_full.log 2>&1
rc=$?; echo "dense fullsize rc=$rc"; tail -3 $O/dense_full.log
[ $rc -ne 0 ] && exit $rc
for k in dense dense-f32 dense; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel $k --steps 5 --warmup 2 > $O/bench_$k.json 2> $O/bench_$k.err || { echo "bench $k failed"; tail -5 $O/bench_$k.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_$k.json'));print('$k', d['ms_per_step'], d['roofline'])"
done
echo done
# 10 000 nodes, one GPU: 64-column blocks / 4-clique items (default) vs 32-column blocks / 8-clique
# items (a chunk of every row is 1.28 MB instead of 2.56 MB), interleaved
for v in d64 d32 d64 d32; do
  if [ $v = d32 ]; then export NIIDMIX_Q_BLOCK_COLS=32; else unset NIIDMIX_Q_BLOCK_COLS; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --config dcliques10000 --steps 5 --warmup 2 > $O/bench_10k_$v.json 2> $O/bench_10k_$v.err || { echo "bench 10k $v failed"; tail -5 $O/bench_10k_$v.err; exit 5; }
  python -c "import json;d=json.load(open('$O/bench_10k_$v.json'));print('10k $v', d['ms_per_step'], d['roofline']['frac'], d['config']['slab_layout'])"
done
unset NIIDMIX_Q_BLOCK_COLS
echo done2
