#!/bin/bash
# SQ counter passes (two per kernel, each within the per-block limits) for the exact and dense kernels.
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r03sq; mkdir -p $O; export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
run() { n=$1; shift; i=1; for c in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $c --output-format csv -d $PWD/$O/${n}_p$i -o p -- python3 bench.py --no-cpu-baseline "$@" > $O/${n}_p$i.log 2>&1 || { echo "$n pass $i failed"; tail $O/${n}_p$i.log; exit 5; }
  i=$((i+1)); done; }
run exact --kernel tile-lds-exact --steps 2 --warmup 1
run dense --config fc1000 --kernel dense --p 262144 --steps 2 --warmup 1
echo ok
