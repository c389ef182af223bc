#!/bin/bash
# round 4 session T: same-box A/B of the closing library against the previous closing library
# (063a27d9, built from commit 40892d4 into tools/build/libniidmix_063a.so) on the HBM-bound lines
# (headline clique, clique-gradient mean, fully-connected big clique), interleaved, 3 times each
out=gpurun_out/r4t
mkdir -p $out
R=${GRAFT_REPO_ROOT:-$(pwd)}
NEW=$R/non-iid-topology-simulator_amd/niidmix/libniidmix.so
OLD=$R/tools/build/libniidmix_063a.so
for i in 1 2 3; do
  for lib in new old; do
    L=$NEW; [ $lib = old ] && L=$OLD
    for cfg in headline grad fc1000; do
      a="--no-cpu-baseline --no-cold-cache --steps 20"
      [ $cfg = grad ] && a="$a --workload grad-clique"
      [ $cfg = fc1000 ] && a="$a --config fc1000"
      NIIDMIX_LIB=$L timeout -k 10 200 python bench.py $a > $out/${cfg}_${lib}_$i.json 2> $out/${cfg}_${lib}_$i.err || { echo "$cfg $lib failed"; tail -3 $out/${cfg}_${lib}_$i.err; exit 1; }
      python -c "import json;d=json.load(open('$out/${cfg}_${lib}_$i.json'));print('$cfg $lib $i', d['ms_per_step'], d['config']['lib_sha16'], d['config'].get('stream_copy_GBs'))"
    done
  done
done
