#!/bin/bash
# round 4 session O: SQ counters of the final exact kernel (headline and 10 000 nodes)
out=gpurun_out/r4o
mkdir -p $out
export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
for cfg in headline d10k; do
  args="--kernel tile-lds-exact --steps 2 --warmup 1"; [ $cfg = d10k ] && args="$args --config dcliques10000"
  i=1
  for c in "$P1" "$P2"; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $PWD/$out/sq_${cfg}_p$i -o p -- python3 bench.py --no-cpu-baseline --no-cold-cache $args > $out/sq_${cfg}_p$i.log 2>&1 || { echo "sq $cfg pass $i failed"; tail -3 $out/sq_${cfg}_p$i.log; exit 4; }
    i=$((i+1))
  done
  python tools/sq_summary.py k_mix_tile_lds $out/sq_${cfg}_p1 $out/sq_${cfg}_p2 > $out/sq_${cfg}_summary.txt; echo "== $cfg"; cat $out/sq_${cfg}_summary.txt
done
