#!/bin/bash
# Round 5: non-temporal second reads: the multi-clique tile's gateway gathers (NIIDMIX_Q_GATHER_NT=1)
# and the exact walker's register rows (NIIDMIX_TLDS_REM_NT=1): parity under both, then 10 000-node
# fast / exact and headline exact, interleaved A/B.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-r5ab}; mkdir -p $O; export TMPDIR=/tmp
NIIDMIX_Q_GATHER_NT=1 NIIDMIX_TLDS_REM_NT=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -k "multi_clique or tile_lds or register" --timeout 200 --timeout-method thread > $O/pytest_nt.log 2>&1 || { echo "pytest nt failed"; tail -20 $O/pytest_nt.log; exit 3; }
tail -1 $O/pytest_nt.log
for rep in 1 2; do
for v in 0 1; do
  NIIDMIX_Q_GATHER_NT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --config dcliques10000 --steps 5 --warmup 2 > $O/bench_d10k_nt$v.json 2> $O/bench_d10k_nt$v.err || { echo "d10k $v failed"; tail -5 $O/bench_d10k_nt$v.err; exit 4; }
  NIIDMIX_TLDS_REM_NT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --config dcliques10000 --kernel tile-lds-exact --steps 3 --warmup 1 > $O/bench_d10kx_nt$v.json 2> $O/bench_d10kx_nt$v.err || { echo "d10k exact $v failed"; tail -5 $O/bench_d10kx_nt$v.err; exit 4; }
  NIIDMIX_TLDS_REM_NT=$v timeout -k 10 300 python bench.py --no-cpu-baseline --kernel tile-lds-exact --steps 10 > $O/bench_x_nt$v.json 2> $O/bench_x_nt$v.err || { echo "exact $v failed"; tail -5 $O/bench_x_nt$v.err; exit 4; }
  python -c "
import json
a=json.load(open('$O/bench_d10k_nt$v.json'));b=json.load(open('$O/bench_d10kx_nt$v.json'));c=json.load(open('$O/bench_x_nt$v.json'))
print('nt$v', 'd10k', a['ms_per_step'], 'd10k_exact', b['ms_per_step'], 'exact', c['ms_per_step'])"
done; done
echo done
