#!/bin/bash
# Round 5, first GPU session: the new parity tests (ring100 at its timed shape, sharded ring auto
# kernel, read guard, logger hooks), then the whole GPU suite and smoke.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/r5a; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_fullsize.py -k "ring100" tests/test_gpu_shard.py::test_sharded_ring_auto_kernel_loopback \
  > $O/new_tests.log 2>&1
rc=$?; echo "new ring rc=$rc"; tail -3 $O/new_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread \
  tests/test_gpu_dropin.py -k "guard or logger or consensus" > $O/new_tests2.log 2>&1
rc=$?; echo "new dropin rc=$rc"; tail -3 $O/new_tests2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "FAILED" $O/pytest_gpu.log | head
[ $rc -ge 2 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 3; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_headline.json 2> $O/bench_headline.err || { echo bench failed; tail $O/bench_headline.err; exit 4; }
cat $O/bench_headline.json | head -c 600; echo
echo done
