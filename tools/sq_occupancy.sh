#!/bin/bash
# SQ counters (one rocprofv3 --pmc pass each) of the exact tile kernel under tile-plan variants:
#   tools/sq_occupancy.sh OUT
# headline exact with 16-row tiles vs the balanced height; 10 000 nodes with the 16-register
# kernel vs the two-phase one.  Summaries: OUT/sq_<name>.txt (tools/sq_summary.py).
set -u
O=${1:?}; mkdir -p "$O"; export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
C=SQ_WAVES,SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_ACTIVE_INST_VALU,SQ_INSTS_VALU,SQ_WAIT_INST_LDS,SQ_WAIT_ANY
pass() {  # name env bench-args...
  n=$1; e=$2; shift 2
  env $e timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d "$R/$O/pmc_$n" -o p -- python3 "$R/bench.py" --no-cpu-baseline --no-cold-cache "$@" > "$O/pmc_$n.log" 2>&1 || { echo "pmc $n failed"; tail -5 "$O/pmc_$n.log"; return 1; }
  python tools/sq_summary.py k_mix_tile_lds "$O/pmc_$n" > "$O/sq_$n.txt" && echo "== $n ($e)" && cat "$O/sq_$n.txt"
}
pass head16 NIIDMIX_TILE_LDS_ROWS=16 --kernel tile-lds-exact --steps 5 || exit 1
pass headauto NIIDMIX_TILE_LDS_ROWS=auto --kernel tile-lds-exact --steps 5 || exit 1
pass d10k_reg16 NIIDMIX_TLDS_REM2=0 --config dcliques10000 --kernel tile-lds-exact --steps 2 --warmup 1 || exit 1
pass d10k_two NIIDMIX_TLDS_REM2=1 --config dcliques10000 --kernel tile-lds-exact --steps 2 --warmup 1 || exit 1
