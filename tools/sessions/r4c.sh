#!/bin/bash
# round 4 session C: re-run the fixed GPU tests, persistent multi-clique tile probe, round-robin
# whole-round E2E, dense MFMA busy counters
out=gpurun_out/r4c
mkdir -p $out
export TMPDIR=/tmp
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_band.py tests/test_gpu_dropin.py tests/test_gpu_parity.py -k "band or dropin or training or multi_clique_tile_auto or dsgd or sample or sparse or randomize or multi_device" -m gpu -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?; tail -6 $out/pytest.log; ok $rc || { echo "pytest rc=$rc: stop"; exit $rc; }
for k in 0 1 2; do
  NIIDMIX_Q_PERSIST=$k timeout -k 10 300 python -u tools/q_probe.py --n 10000 --blocks 64 --variants 8x13x4x13 --iters 10 --reps 3 > $out/q_persist$k.txt 2>&1 || exit 6
  echo "persist $k: $(grep SUMMARY $out/q_persist$k.txt)"
done
timeout -k 10 900 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --e2e-step > $out/bench_e2e_step.json 2> $out/bench_e2e_step.err || exit 5
python -c "import json;d=json.load(open('$out/bench_e2e_step.json'));print(json.dumps(d['e2e'],indent=1))"
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $PWD/$out/dense_pmc -o p -- python3 $PWD/bench.py --config fc1000 --kernel dense --p 262144 --steps 3 --warmup 1 --no-cpu-baseline > $out/dense_pmc.log 2>&1 || { tail -5 $out/dense_pmc.log; exit 7; }
ls -R $out/dense_pmc | head
exit $rc
