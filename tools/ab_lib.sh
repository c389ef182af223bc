#!/bin/bash
# Interleaved A/B of two libraries on one bench command: tools/ab_lib.sh OUT LIB_A LIB_B BENCH_ARGS...
set -u
O=${1:?}; A=${2:?}; B=${3:?}; shift 3; REPS=${REPS:-3}
mkdir -p "$O"
for rep in $(seq 1 $REPS); do
  for v in A B; do
    if [ $v = A ]; then L=$A; else L=$B; fi
    f=$O/bench_${v}_$rep.json
    NIIDMIX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $f 2> $f.err || { echo "bench $v failed"; tail -5 $f.err; exit 4; }
    python -c "import json;d=json.load(open('$f'));print('$v', d['config']['lib_sha16'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
