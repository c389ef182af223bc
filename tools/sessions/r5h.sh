#!/bin/bash
# Round 5: bf16x6 dense GEMM time split (ablation builds: no loads / no MFMA / no LDS operand reads).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5h}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2; do
for a in 0 1 2 3; do
  export NIIDMIX_DENSE_B6_ABL=$a
  timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel dense --steps 5 --warmup 2 > $O/bench_abl$a.json 2> $O/bench_abl$a.err || { echo "bench abl $a failed"; tail -5 $O/bench_abl$a.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_abl$a.json'));r=d['roofline'];print('abl$a', d['ms_per_step'], r['frac'])"
done; done
unset NIIDMIX_DENSE_B6_ABL
echo done
