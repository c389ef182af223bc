#!/bin/bash
# One parameterised GPU-box session (replaces the round-4/5 one-off scripts under tools/sessions/).
#
#   tools/session.sh NAME STEP [STEP ...]
#
# Output goes to gpurun_out/NAME/.  Each STEP is KIND:ARGS and runs under its own time limit; the
# session stops at the first failing step (a test failure, a crash, an abort or a timeout), so no
# GPU work follows a fault.  Kinds:
#   pytest:ARGS      python -m pytest ARGS -m gpu (thread timeouts of 300 s per test)  -> pytest_K.log
#   bench:ARGS       python bench.py ARGS                                             -> bench_K.json
#   trace:ARGS       rocprofv3 --kernel-trace --stats over bench.py --no-cpu-baseline ARGS -> trace_K/
#   pmc:CTRS|ARGS    rocprofv3 --pmc CTRS (one pass) over bench.py --no-cpu-baseline ARGS -> pmc_K/
#   py:ARGS          python ARGS (a tool or probe script)                              -> py_K.log
#   smoke:           __graft_entry__.smoke()                                           -> smoke.log
#   sh:CMD           bash -c CMD (env settings, A/B loops)                              -> sh_K.log
# K is the step's index.  STEP_TIMEOUT (seconds, default 600) bounds each step.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
NAME=${1:?session name}
shift
O=gpurun_out/$NAME
mkdir -p "$O"
export TMPDIR=/tmp
T=${STEP_TIMEOUT:-600}
k=0
for step in "$@"; do
  k=$((k + 1))
  kind=${step%%:*}
  args=${step#*:}
  echo "[$k] $kind $args"
  case $kind in
    pytest)
      timeout -k 10 "$T" python -u -m pytest $args -m gpu -v -rs --timeout 300 --timeout-method thread \
        > "$O/pytest_$k.log" 2>&1
      rc=$?; tail -3 "$O/pytest_$k.log" ;;
    bench)
      timeout -k 10 "$T" python bench.py $args > "$O/bench_$k.json" 2> "$O/bench_$k.err"
      rc=$?; cat "$O/bench_$k.json"; [ $rc -ne 0 ] && tail -20 "$O/bench_$k.err" ;;
    trace)
      timeout -k 10 "$T" rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/trace_$k" -o kt \
        -- python3 "$R/bench.py" --no-cpu-baseline $args > "$O/trace_$k.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && tail -20 "$O/trace_$k.log" ;;
    pmc)
      ctrs=${args%%|*}; bargs=${args#*|}
      timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d "$R/$O/pmc_$k" -o pmc \
        -- python3 "$R/bench.py" --no-cpu-baseline $bargs > "$O/pmc_$k.log" 2>&1
      rc=$?; [ $rc -ne 0 ] && tail -20 "$O/pmc_$k.log" ;;
    py)
      timeout -k 10 "$T" python -u $args > "$O/py_$k.log" 2>&1
      rc=$?; tail -15 "$O/py_$k.log" ;;
    sh)
      timeout -k 10 "$T" bash -c "$args" > "$O/sh_$k.log" 2>&1
      rc=$?; tail -25 "$O/sh_$k.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1
      rc=$?; cat "$O/smoke.log" ;;
    *)
      echo "unknown step kind: $kind"; rc=2 ;;
  esac
  echo "[$k] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
echo "session $NAME done"
