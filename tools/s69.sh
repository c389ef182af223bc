#!/bin/bash
# ring100: CSR work-item width A/B (NIIDMIX_CSR_SPL), hipGraph bench lines
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s69; mkdir -p $O
for rep in 1 2; do
for spl in 1 2 4; do
  NIIDMIX_CSR_SPL=$spl timeout -k 10 200 python bench.py --config ring100 --kernel csr-fast --steps 500 --warmup 50 --no-cpu-baseline > $O/ring_$spl.json 2> $O/ring_$spl.err || { tail -5 $O/ring_$spl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/ring_$spl.json')); print('spl $spl', d['ms_per_step'], d['config']['launch_ms'], d['config']['stream_copy_GBs'], d['roofline']['frac'])"
done
done
