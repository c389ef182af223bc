#!/bin/bash
# round 4 session AA: dense MFMA, persistent grids of 3 / 2 blocks per CU walking the tiles in step
# (so the tiles in flight on an XCD share W's K-slices in L2) vs one block per tile
out=gpurun_out/r4aa
mkdir -p $out
R=${GRAFT_REPO_ROOT:-$(pwd)}
NIIDMIX_DENSE_PERSIST=3 timeout -k 10 300 python -u -m pytest tests -m gpu -k "dense" -x -q --timeout 200 --timeout-method thread > $out/pytest_dense.log 2>&1
rc=$?; tail -2 $out/pytest_dense.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest_dense.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
for i in 1 2; do
  for v in 0 3 6; do
    NIIDMIX_DENSE_PERSIST=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --steps 5 --warmup 1 > $out/dense_p${v}_$i.json 2> $out/dense_p${v}_$i.err || { echo "bench $v failed"; tail -3 $out/dense_p${v}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$out/dense_p${v}_$i.json'));print('dense persist=$v', d['ms_per_step'], d['roofline']['frac'])"
  done
done
for v in 0 3; do
NIIDMIX_DENSE_PERSIST=$v timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$out/pmc_f$v -o p -- python3 $R/bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --steps 3 --warmup 1 > $out/pmc_f$v.log 2>&1 || { echo pmc failed; tail -3 $out/pmc_f$v.log; exit 3; }
done
python - <<'PY'
import csv,glob
for v in (0,3):
    rows=[r for f in glob.glob(f'gpurun_out/r4aa/pmc_f{v}/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f)) if 'k_mix_dense' in r.get('Kernel_Name','')]
    x=[float(r['Counter_Value']) for r in rows]
    print('persist', v, 'dense FETCH per launch GB (x2 correction):', 2*sum(x)/len(x)*1024/1e9 if x else None)
PY
