#!/bin/bash
# round 4 session V: dense MFMA K-step / occupancy sweep (BK 16 / 8, 3 / 4 waves per SIMD; the
# OCC=4 builds spill a few VGPRs), parity tests under BK=8, interleaved bench lines
out=gpurun_out/r4v
mkdir -p $out
NIIDMIX_DENSE_BK=8 timeout -k 10 300 python -u -m pytest tests -m gpu -k "dense" -x -q --timeout 200 --timeout-method thread > $out/pytest_dense_bk8.log 2>&1
rc=$?; tail -2 $out/pytest_dense_bk8.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest_dense_bk8.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
for i in 1 2; do
  for v in 16:3 8:3 8:4 16:4; do
    bk=${v%:*}; oc=${v#*:}
    NIIDMIX_DENSE_BK=$bk NIIDMIX_DENSE_OCC=$oc timeout -k 10 200 python bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --steps 5 --warmup 1 > $out/dense_${bk}_${oc}_$i.json 2> $out/dense_${bk}_${oc}_$i.err || { echo "bench $v failed"; tail -3 $out/dense_${bk}_${oc}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$out/dense_${bk}_${oc}_$i.json'));print('dense BK=$bk OCC=$oc', d['ms_per_step'], d['roofline']['frac'])"
  done
done
