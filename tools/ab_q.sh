#!/bin/bash
# Interleaved A/B of the multi-clique tile variants on configs[4] on one GPU (10 000-node d-cliques,
# P = 2^20): the default tile and member-split tiles (NIIDMIX_CLIQUE_QM=W,R,OCC).
set -u
O=${1:?out dir}; REPS=${REPS:-2}
mkdir -p "$O"
for rep in $(seq 1 $REPS); do
  for v in ${VARIANTS:-default 8,4,4 8,7,4,2 16,4,4,2}; do
    if [ $v = default ]; then unset NIIDMIX_CLIQUE_QM; else export NIIDMIX_CLIQUE_QM=$v; fi
    f=$O/bench_${v//,/_}_$rep.json
    timeout -k 10 300 python bench.py --no-cpu-baseline --config dcliques10000 --steps 5 --warmup 2 > $f 2> $f.err || { echo "bench $v failed"; tail -5 $f.err; exit 4; }
    python -c "import json;d=json.load(open('$f'));print('$v', d['ms_per_step'], d['roofline']['frac'])"
  done
done
