#!/bin/bash
# round 4 session L: exact walker loops for every tile row count 9..16 (A/B against the final build)
out=gpurun_out/r4l
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_fullsize_10k.py -k "tile_lds or register_rows or exact" -m gpu -x -q --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $out/pytest.log | head; echo "pytest rc=$rc: stop"; exit 1; }
for lib in cur prev cur prev; do
  L=$PWD/non-iid-topology-simulator_amd/niidmix/libniidmix.so; [ $lib = prev ] && L=$PWD/tools/build/libniidmix_prev.so
  NIIDMIX_LIB=$L timeout -k 10 300 python -u tools/exact_probe.py --rts 16 --metas rem8,rem16,seg --reps 2 > $out/exact_probe_$lib.txt 2>&1 || { tail -5 $out/exact_probe_$lib.txt; exit 2; }
  echo "lib $lib"; grep SUMMARY $out/exact_probe_$lib.txt
done
for lib in cur prev; do
  L=$PWD/non-iid-topology-simulator_amd/niidmix/libniidmix.so; [ $lib = prev ] && L=$PWD/tools/build/libniidmix_prev.so
  NIIDMIX_LIB=$L timeout -k 10 600 python bench.py --config dcliques10000 --kernel tile-lds-exact --steps 5 --warmup 2 --no-cpu-baseline > $out/bench_exact10k_$lib.json 2> $out/bench_exact10k_$lib.err || exit 3
  python -c "import json;d=json.load(open('$out/bench_exact10k_$lib.json'));print('10k exact $lib', d['ms_per_step'], 'ms', d['roofline']['frac'])"
done
