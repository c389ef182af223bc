#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, kernel-trace profile.  Each GPU step has its own
# time limit; a crash/timeout/abort (rc >= 2 for pytest, any nonzero otherwise) stops the session.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
OUT=gpurun_out/${1:-session}
mkdir -p "$OUT"
export TMPDIR=/tmp
rocm-smi --showproductname > "$OUT/rocm_smi.txt" 2>&1 || true
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -rs --timeout 120 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 "$OUT/pytest_gpu.log"
if [ $rc -ge 2 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo smoke failed; cat "$OUT/smoke.log"; exit 3; }
cat "$OUT/smoke.log"
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { echo bench failed; tail -20 "$OUT/bench.err"; exit 4; }
cat "$OUT/bench.json"
if [ -n "${PROFILE:-1}" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$OUT/prof" -o kt -- python3 "$R/bench.py" --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/prof.log" 2>&1 || { echo profile failed; tail -20 "$OUT/prof.log"; exit 5; }
  find "$OUT/prof" -name "*stats*" | head
fi
