#!/bin/bash
# round 4 session U: dense MFMA with K-steps of 16 (168 VGPRs, three blocks per CU) vs 32 (256
# VGPRs, two blocks): dense parity tests under the BK=16 kernel, then interleaved bench lines
out=gpurun_out/r4u
mkdir -p $out
NIIDMIX_DENSE_BK=16 timeout -k 10 300 python -u -m pytest tests -m gpu -k "dense" -x -q --timeout 200 --timeout-method thread > $out/pytest_dense_bk16.log 2>&1
rc=$?; tail -2 $out/pytest_dense_bk16.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest_dense_bk16.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
for i in 1 2; do
  for bk in 32 16; do
    NIIDMIX_DENSE_BK=$bk timeout -k 10 200 python bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --steps 5 --warmup 1 > $out/dense_bk${bk}_$i.json 2> $out/dense_bk${bk}_$i.err || { echo "bench bk$bk failed"; tail -3 $out/dense_bk${bk}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$out/dense_bk${bk}_$i.json'));print('dense BK=$bk', d['ms_per_step'], d['roofline']['frac'])"
  done
done
