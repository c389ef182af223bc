#!/bin/bash
# Round 5: bf16x6 dense GEMM (unconditional loads, mask at the split) -- parity, bench, SQ pass.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5e}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "dense" > $O/dense_tests.log 2>&1
rc=$?; echo "dense tests rc=$rc"; tail -3 $O/dense_tests.log
[ $rc -ne 0 ] && exit $rc
NIIDMIX_DENSE_B6_WN=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_parity.py -k "dense" > $O/dense_tests_wn2.log 2>&1
rc=$?; echo "dense tests wn2 rc=$rc"; tail -3 $O/dense_tests_wn2.log
[ $rc -ne 0 ] && exit $rc
for v in wn4 wn2 f32 wn4 wn2; do
  k=dense; [ $v = f32 ] && k=dense-f32
  if [ $v = wn2 ]; then export NIIDMIX_DENSE_B6_WN=2; else unset NIIDMIX_DENSE_B6_WN; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --config fc1000 --kernel $k --steps 5 --warmup 2 > $O/bench_$v.json 2> $O/bench_$v.err || { echo "bench $v failed"; tail -5 $O/bench_$v.err; exit 4; }
  python -c "import json;d=json.load(open('$O/bench_$v.json'));r=d['roofline'];print('$v', d['ms_per_step'], r['frac'], r.get('fp32_equivalent_frac_of_fp32_mfma_peak'))"
done
unset NIIDMIX_DENSE_B6_WN
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_INSTS_VMEM GRBM_GUI_ACTIVE"
i=1; for c in "$P1" "$P2" "FETCH_SIZE"; do
  timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $PWD/$O/b6_p$i -o p -- python3 bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --p 262144 --steps 2 --warmup 1 > $O/b6_p$i.log 2>&1 || { echo "pass $i failed"; tail $O/b6_p$i.log; exit 5; }
  i=$((i+1)); done
python tools/sq_summary.py k_mix_dense_b6 $O/b6_p1 $O/b6_p2 $O/b6_p3 | tee $O/sq_b6.txt | tail -12
echo ok
