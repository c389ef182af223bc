#!/bin/bash
# Round 5: SQ counters of the final bf16x6 dense kernel (256 x 256 tiles, SCHED 3), FC-1000 at
# P = 2^18 (two passes within the per-block counter limits), plus a GRBM pass for the clock.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5y}; mkdir -p $O; export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
i=1
for c in "$P1" "$P2"; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/$O/dense_p$i -o p -- python3 $R/bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --p 262144 --steps 2 --warmup 1 > $O/dense_p$i.log 2>&1 || { echo "pass $i failed"; tail $O/dense_p$i.log; exit 5; }
  i=$((i+1))
done
python tools/sq_summary.py k_mix_dense_b6 $O/dense_p1 $O/dense_p2 > $O/sq_dense_b6_final.txt
cat $O/sq_dense_b6_final.txt
