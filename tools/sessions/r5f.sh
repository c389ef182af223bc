#!/bin/bash
# Round 5: bf16x6 dense GEMM schedule / block-width A/B (interleaved, same box).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5f}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "dense" > $O/dense_tests.log 2>&1
rc=$?; echo "dense tests rc=$rc"; tail -1 $O/dense_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
for v in 4_0 4_1 2_0 2_1; do
  export NIIDMIX_DENSE_B6_WN=${v%_*} NIIDMIX_DENSE_B6_SCHED=${v#*_}
  timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel dense --steps 5 --warmup 2 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_$v.json'));r=d['roofline'];print('$v', d['ms_per_step'], r['frac'], r.get('fp32_equivalent_frac_of_fp32_mfma_peak'))"
done; done
echo done
