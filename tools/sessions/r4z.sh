#!/bin/bash
# round 4 session Z: MFMA utilisation of the final dense kernel (K-steps of 16), one counter pass
# and its kernel trace, as profiles/r04/dense_mfma_utilisation.txt did for the round-3 kernel
out=gpurun_out/r4z
mkdir -p $out
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace --stats --output-format csv -d $R/$out/mfma -o m -- python3 $R/bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --p 262144 --steps 3 --warmup 1 > $out/mfma.log 2>&1 || { echo "pmc failed"; tail -5 $out/mfma.log; exit 1; }
timeout -k 10 200 python bench.py --no-cpu-baseline --no-cold-cache --config fc1000 --kernel dense --p 262144 --steps 3 --warmup 1 > $out/bench_p262144.json 2> $out/bench_p262144.err || exit 2
ls -R $out/mfma | head
