#!/bin/bash
# round 4 session J: walker weight select two positions ahead (A/B against the session-H build)
out=gpurun_out/r4j
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fullsize_10k.py tests/test_gpu_dropin.py -k "tile_lds or register_rows or exact or training or gradient" -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; echo "pytest rc=$rc: stop"; exit 1; }
for lib in cur prev cur prev; do
  L=$PWD/non-iid-topology-simulator_amd/niidmix/libniidmix.so; [ $lib = prev ] && L=$PWD/tools/build/libniidmix_prev.so
  NIIDMIX_LIB=$L timeout -k 10 300 python -u tools/exact_probe.py --rts 16 --metas rem8,rem16 --reps 2 > $out/exact_probe_$lib.txt 2>&1 || { tail -5 $out/exact_probe_$lib.txt; exit 2; }
  echo "lib $lib"; grep SUMMARY $out/exact_probe_$lib.txt
done
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $P1 --output-format csv -d $PWD/$out/sq_exact_p1 -o p -- python3 bench.py --no-cpu-baseline --kernel tile-lds-exact --steps 2 --warmup 1 > $out/sq_exact_p1.log 2>&1 || { echo "sq pass failed"; tail -3 $out/sq_exact_p1.log; exit 4; }
python tools/sq_summary.py k_mix_tile_lds $out/sq_exact_p1 > $out/sq_exact_summary.txt; cat $out/sq_exact_summary.txt
timeout -k 10 300 python bench.py --kernel tile-lds-exact --steps 20 --no-cpu-baseline > $out/bench_exact_headline.json 2> $out/bench_exact_headline.err || exit 5
python -c "import json;d=json.load(open('$out/bench_exact_headline.json'));print('headline exact', d['ms_per_step'], 'ms', d['roofline']['frac'])"
timeout -k 10 600 python bench.py --config dcliques10000 --kernel tile-lds-exact --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_exact10k.json 2> $out/bench_exact10k.err || exit 6
python -c "import json;d=json.load(open('$out/bench_exact10k.json'));print('10k exact', d['ms_per_step'], 'ms', d['roofline']['frac'])"
timeout -k 10 400 python -u tools/pinned_train_probe.py > $out/pinned_train_probe.txt 2>&1 || exit 7
cat $out/pinned_train_probe.txt
