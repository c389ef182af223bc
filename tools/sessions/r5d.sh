#!/bin/bash
# Round 5: SQ counters of the bf16x6 dense kernel vs the fp32 one (FC-1000 at P = 2^18).
set -u
cd ${GRAFT_REPO_ROOT:-$(pwd)}
O=gpurun_out/r5d; mkdir -p $O; export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
run() { n=$1; shift; i=1; for c in "$P1" "$P2" "FETCH_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $PWD/$O/${n}_p$i -o p -- python3 bench.py --no-cpu-baseline --no-cold-cache "$@" > $O/${n}_p$i.log 2>&1 || { echo "$n pass $i failed"; tail $O/${n}_p$i.log; exit 5; }
  i=$((i+1)); done; }
run b6 --config fc1000 --kernel dense --p 262144 --steps 2 --warmup 1
run f32 --config fc1000 --kernel dense-f32 --p 262144 --steps 2 --warmup 1
python tools/sq_summary.py k_mix_dense_b6 $O/b6_p1 $O/b6_p2 $O/b6_p3 > $O/sq_b6.txt
python tools/sq_summary.py "k_mix_dense<" $O/f32_p1 $O/f32_p2 $O/f32_p3 > $O/sq_f32.txt
paste $O/sq_b6.txt $O/sq_f32.txt
echo ok
