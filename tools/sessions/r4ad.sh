#!/bin/bash
# round 4 session AD: ring 100 strip kernel with non-temporal LDS-DMA loads (cache policy nt,
# tools/build/libniidmix_aux2.so) vs the final library, interleaved bench lines
out=gpurun_out/r4ad
mkdir -p $out
R=${GRAFT_REPO_ROOT:-$(pwd)}
for i in 1 2 3; do
  for v in final aux2; do
    L=$R/non-iid-topology-simulator_amd/niidmix/libniidmix.so; [ $v = aux2 ] && L=$R/tools/build/libniidmix_aux2.so
    NIIDMIX_LIB=$L timeout -k 10 200 python bench.py --no-cpu-baseline --no-cold-cache --config ring100 --steps 400 > $out/ring_${v}_$i.json 2> $out/ring_${v}_$i.err || { echo "bench $v failed"; tail -3 $out/ring_${v}_$i.err; exit 2; }
    python -c "import json;d=json.load(open('$out/ring_${v}_$i.json'));print('ring $v', d['ms_per_step']*1000, 'us', d['config']['kernel'], d['config']['lib_sha16'])"
  done
done
NIIDMIX_LIB=$R/tools/build/libniidmix_aux2.so timeout -k 10 200 python -u -m pytest tests/test_gpu_band.py -k strip -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1; tail -1 $out/pytest.log
