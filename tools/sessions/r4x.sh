#!/bin/bash
# round 4 session X: dense MFMA with X tiles loaded non-temporally (so W, read by every column tile,
# stays in L2) vs the closing library (tools/build/libniidmix_prev2.so): time and PMC traffic
out=gpurun_out/r4x
mkdir -p $out
R=${GRAFT_REPO_ROOT:-$(pwd)}
timeout -k 10 300 python -u -m pytest tests -m gpu -k "dense" -x -q --timeout 200 --timeout-method thread > $out/pytest_dense.log 2>&1
rc=$?; tail -2 $out/pytest_dense.log
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $out/pytest_dense.log | head -20; echo "pytest rc=$rc: stop"; exit 1; }
for i in 1 2; do
  for v in nt prev; do
    L=$R/non-iid-topology-simulator_amd/niidmix/libniidmix.so; [ $v = prev ] && L=$R/tools/build/libniidmix_prev2.so
    NIIDMIX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --steps 5 --warmup 1 > $out/dense_${v}_$i.json 2> $out/dense_${v}_$i.err || { echo "bench $v failed"; tail -3 $out/dense_${v}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$out/dense_${v}_$i.json'));print('dense $v', d['ms_per_step'], d['roofline']['frac'], d['config']['lib_sha16'])"
  done
done
NIIDMIX_LIB=$R/non-iid-topology-simulator_amd/niidmix/libniidmix.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $R/$out/pmc_f -o p -- python3 $R/bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --steps 3 --warmup 1 > $out/pmc_f.log 2>&1 || { echo pmc failed; tail -3 $out/pmc_f.log; exit 3; }
python - <<'PY'
import csv,glob
rows=[r for f in glob.glob('gpurun_out/r4x/pmc_f/**/*counter_collection.csv',recursive=True) for r in csv.DictReader(open(f)) if 'k_mix_dense' in r.get('Kernel_Name','')]
v=[float(r['Counter_Value']) for r in rows]
print('dense FETCH_SIZE per launch (KB, x2 gfx950 correction -> GB):', len(v), 2*sum(v)/len(v)*1024/1e9 if v else None)
PY
