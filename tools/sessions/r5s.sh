#!/bin/bash
# Round 5: same-box A/B of the library before the one-wave dense kernel (tools/variants, rebuilt
# from commit cb1a1d3) and the current one: headline and clique-gradient mean, interleaved.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5s}; mkdir -p $O; export TMPDIR=/tmp
for rep in 1 2 3; do
for v in old new; do
  if [ $v = old ]; then L=tools/variants/libniidmix_e527.so; else L=""; fi
  NIIDMIX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > $O/bench_head_$v.json 2> $O/bench_head_$v.err || { echo "bench $v failed"; tail -5 $O/bench_head_$v.err; exit 4; }
  NIIDMIX_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --workload grad-clique --steps 10 > $O/bench_grad_$v.json 2> $O/bench_grad_$v.err || { echo "grad $v failed"; tail -5 $O/bench_grad_$v.err; exit 4; }
  python -c "import json;a=json.load(open('$O/bench_head_$v.json'));b=json.load(open('$O/bench_grad_$v.json'));print('$v', a['config']['lib_sha16'], 'head', a['ms_per_step'], a['config']['frac_of_stream_copy'], 'grad', b['ms_per_step'])"
done; done
echo done
