#!/bin/bash
# Round 5: bf16x6 dense epilogue by buffer stores: dense parity (incl. non-finite cases and the
# one-wave bitwise test), then an interleaved A/B against the previous library (tools/variants).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5z}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "dense" --timeout 200 --timeout-method thread > $O/pytest_dense.log 2>&1 || { echo "pytest dense failed"; tail -20 $O/pytest_dense.log; exit 3; }
tail -1 $O/pytest_dense.log
for rep in 1 2; do
for v in prev new; do
  if [ $v = prev ]; then L=tools/variants/libniidmix_prev.so; else L=""; fi
  NIIDMIX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel dense --steps 5 --warmup 2 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_$v.json'));r=d['roofline'];print('$v', d['ms_per_step'], r['frac'])"
done; done
echo done
