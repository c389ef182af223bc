#!/bin/bash
# FETCH_SIZE per launch of the multi-clique tile at 10 000 nodes, per variant (one PMC pass each).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=${1:?out dir}; mkdir -p "$O"
for v in ${VARIANTS:-default 8,4,4}; do
  if [ $v = default ]; then unset NIIDMIX_CLIQUE_QM; else export NIIDMIX_CLIQUE_QM=$v; fi
  d=$R/$O/pmc_${v//,/_}
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $d -o p -- python3 $R/bench.py --no-cpu-baseline --config dcliques10000 --steps 2 --warmup 1 > $d.log 2>&1 || { echo "pmc $v failed"; tail -5 $d.log; exit 5; }
  python3 -c "
import sys; sys.path.insert(0, '$R/tools')
from pmc_traffic import per_dispatch
import statistics
v = per_dispatch('$d', 'FETCH_SIZE', 'k_mix_clique_q')
r = 2 * statistics.median(v) * 1024
print('$v', 'reads', round(r / 1e9, 2), 'GB =', round(r / 41.943e9, 3), 'x algorithmic')"
done
