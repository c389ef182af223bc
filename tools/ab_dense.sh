#!/bin/bash
# Interleaved A/B of the bf16x6 dense GEMM variants on FC-1000 at P = 2^20 (one bench line each,
# REPS passes): the default kernel and k_mix_dense_b6d's NIIDMIX_DENSE_B6_DMA configurations.
set -u
O=${1:?out dir}; REPS=${REPS:-2}
mkdir -p "$O"
for rep in $(seq 1 $REPS); do
  for v in ${VARIANTS:-default 4,3 4,2 2,2}; do
    if [ $v = default ]; then unset NIIDMIX_DENSE_B6_DMA; else export NIIDMIX_DENSE_B6_DMA=$v; fi
    f=$O/bench_${v//,/_}_$rep.json
    timeout -k 10 120 python bench.py --no-cpu-baseline --config fc1000 --kernel dense --steps 10 --warmup 3 > $f 2> $f.err || { echo "bench $v failed"; tail -5 $f.err; exit 4; }
    python -c "import json;d=json.load(open('$f'));print('$v', d['ms_per_step'], d['roofline']['frac'])"
  done
done
