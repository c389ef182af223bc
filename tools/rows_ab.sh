#!/bin/bash
# A/B of the rt-16 tile height (NIIDMIX_TILE_LDS_ROWS) on the exact kernel: tools/rows_ab.sh OUT CONFIG_ARGS -- ROWS...
# e.g. tools/rows_ab.sh gpurun_out/x "--config dcliques10000 --steps 3 --warmup 1" 16 10 12
set -u
O=${1:?}; A=${2:?}; shift 2; REPS=${REPS:-2}
mkdir -p "$O"
for rep in $(seq 1 $REPS); do
  for r in "$@"; do
    f=$O/bench_r${r}_$rep.json
    NIIDMIX_TILE_LDS_ROWS=$r timeout -k 10 400 python bench.py --no-cpu-baseline --kernel tile-lds-exact $A > $f 2> $f.err || { echo "bench rows $r failed"; tail -5 $f.err; exit 4; }
    python -c "import json;d=json.load(open('$f'));print('rows $r', d['ms_per_step'], d['roofline']['frac'])"
  done
done
