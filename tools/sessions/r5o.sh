#!/bin/bash
# Round 5: bf16x6 dense, X as if pre-split (ABL 4: three 16-B pieces per thread and K-step, no
# split) against the same build's SCHED 3 kernel (ABL 5), interleaved; ablation library.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5o}; mkdir -p $O; export TMPDIR=/tmp
export NIIDMIX_LIB=tools/variants/libniidmix_abl.so
for rep in 1 2; do
for a in 5 4; do
  NIIDMIX_DENSE_B6_ABL=$a timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel dense --steps 5 --warmup 2 > $O/bench_abl$a.json 2> $O/bench_abl$a.err || { echo "bench abl $a failed"; tail -5 $O/bench_abl$a.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_abl$a.json'));r=d['roofline'];print('abl$a', d['ms_per_step'], r['frac'])"
done; done
echo done
