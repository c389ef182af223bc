#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; mkdir -p gpurun_out/s15; export TMPDIR=/tmp
for spl in 1 4; do
  NIIDMIX_CSR_SPL=$spl timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/s15/spl$spl" -o kt -- python3 "$R/bench.py" --no-cpu-baseline --config ring100 --steps 200 > gpurun_out/s15/spl$spl.log 2>&1 || { tail -5 gpurun_out/s15/spl$spl.log; exit 1; }
  grep -h '^{' gpurun_out/s15/spl$spl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('spl$spl', d['ms_per_step'])"
  grep k_mix_csr gpurun_out/s15/spl$spl/kt_kernel_stats.csv | cut -c1-60,200-400
done
timeout -k 10 300 python -m pytest tests/test_gpu_dropin.py -q -x -k consensus > gpurun_out/s15/pt.log 2>&1; tail -2 gpurun_out/s15/pt.log
