#!/bin/bash
# Round 5: bf16x6 dense GEMM with distance-2 prefetch -- parity, bench; 10k 32-column blocks A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5c}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "dense" > $O/dense_tests.log 2>&1
rc=$?; echo "dense tests rc=$rc"; tail -3 $O/dense_tests.log
[ $rc -ne 0 ] && exit $rc
for k in dense dense-f32 dense; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel $k --steps 5 --warmup 2 > $O/bench_$k.json 2> $O/bench_$k.err || { echo "bench $k failed"; tail -5 $O/bench_$k.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_$k.json'));r=d['roofline'];print('$k', d['ms_per_step'], r['frac'], r.get('fp32_equivalent_frac_of_fp32_mfma_peak'))"
done
for v in d64 d32 d64 d32; do
  if [ $v = d32 ]; then export NIIDMIX_Q_BLOCK_COLS=32; else unset NIIDMIX_Q_BLOCK_COLS; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --config dcliques10000 --steps 5 --warmup 2 > $O/bench_10k_$v.json 2> $O/bench_10k_$v.err || { echo "bench 10k $v failed"; tail -5 $O/bench_10k_$v.err; exit 5; }
  python -c "import json;d=json.load(open('$O/bench_10k_$v.json'));print('10k $v', d['ms_per_step'], d['roofline']['frac'], d['config']['slab_layout'])"
done
unset NIIDMIX_Q_BLOCK_COLS
echo done
