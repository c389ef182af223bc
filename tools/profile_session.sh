#!/bin/bash
# rocprofv3 passes for the headline bench command: kernel-trace stats, then FETCH_SIZE and
# WRITE_SIZE in separate PMC passes (counters never combined with runtime/sys traces).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
OUT=gpurun_out/${1:-prof}; mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --steps ${STEPS:-10} --warmup 2 ${BENCH_ARGS:-}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/kt" -o kt -- python3 "$R/bench.py" $ARGS > "$OUT/kt.log" 2>&1 || { echo "kernel-trace failed"; tail -20 "$OUT/kt.log"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d "$R/$OUT/fetch" -o f -- python3 "$R/bench.py" $ARGS > "$OUT/fetch.log" 2>&1 || { echo "fetch pass failed"; tail -20 "$OUT/fetch.log"; exit 2; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d "$R/$OUT/write" -o w -- python3 "$R/bench.py" $ARGS > "$OUT/write.log" 2>&1 || { echo "write pass failed"; tail -20 "$OUT/write.log"; exit 3; }
grep -h "^{" "$OUT/kt.log" | tail -1
find "$OUT" -name "*kernel_stats.csv" | head -3
