#!/bin/bash
# Interleaved A/B of environment settings on one bench command:
#   tools/env_ab.sh OUT "BENCH_ARGS" "ENV_A" "ENV_B" ...     (ENV: space-separated K=V, or "-" for none)
# e.g. tools/env_ab.sh gpurun_out/x "--config dcliques10000 --kernel tile-lds-exact --steps 3 --warmup 1" \
#        NIIDMIX_TLDS_REM2=0 NIIDMIX_TLDS_REM2=1
set -u
O=${1:?}; A=${2:?}; shift 2; REPS=${REPS:-2}
mkdir -p "$O"
for rep in $(seq 1 $REPS); do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    f=$O/bench_v${i}_$rep.json
    [ "$e" = "-" ] && e=""
    env $e timeout -k 10 400 python bench.py --no-cpu-baseline $A > $f 2> $f.err || { echo "bench [$e] failed"; tail -5 $f.err; exit 4; }
    python -c "import json;d=json.load(open('$f'));print('[$e]', d['ms_per_step'], d['roofline']['frac'])"
  done
done
