#!/bin/bash
# round 4 session W: dense MFMA, BK=16 default with the interior fetch fast path (no per-lane
# bounds on interior tiles / K-steps) vs the previous build (tools/build/libniidmix_bk.so, BK=16
# via env); dense parity tests on the new default
out=gpurun_out/r4w
mkdir -p $out
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest tests -m gpu -k "dense" -x -q --timeout 200 --timeout-method thread > $out/pytest_dense.log 2>&1
rc=$?; tail -2 $out/pytest_dense.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest_dense.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
for i in 1 2; do
  for v in new prev; do
    L=$R/non-iid-topology-simulator_amd/niidmix/libniidmix.so; [ $v = prev ] && L=$R/tools/build/libniidmix_bk.so
    NIIDMIX_LIB=$L NIIDMIX_DENSE_BK=16 timeout -k 10 200 python bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --steps 5 --warmup 1 > $out/dense_${v}_$i.json 2> $out/dense_${v}_$i.err || { echo "bench $v failed"; tail -3 $out/dense_${v}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$out/dense_${v}_$i.json'));print('dense $v', d['ms_per_step'], d['roofline']['frac'], d['config']['lib_sha16'])"
  done
done
