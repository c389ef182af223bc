#!/bin/bash
# Round 5: bf16x6 dense GEMM, 256 x 256 blocks (waves of 128 x 64, TM 4) vs 128 x 256 (TM 2).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5i}; mkdir -p $O; export TMPDIR=/tmp
for tm in 2 4; do
NIIDMIX_DENSE_B6_TM=$tm timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "dense" > $O/dense_tests_tm$tm.log 2>&1
rc=$?; echo "dense tests tm$tm rc=$rc"; tail -1 $O/dense_tests_tm$tm.log
[ $rc -ne 0 ] && exit $rc
done
for rep in 1 2 3; do
for tm in 2 4; do
  export NIIDMIX_DENSE_B6_TM=$tm
  timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel dense --steps 5 --warmup 2 > $O/bench_tm$tm.json 2> $O/bench_tm$tm.err || { echo "bench tm$tm failed"; tail -5 $O/bench_tm$tm.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_tm$tm.json'));r=d['roofline'];print('tm$tm', d['ms_per_step'], r['frac'], r.get('fp32_equivalent_frac_of_fp32_mfma_peak'))"
done; done
unset NIIDMIX_DENSE_B6_TM
echo done
