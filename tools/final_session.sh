#!/bin/bash
# Closing GPU session of a round, with the final library, in parts that each fit one gpurun call:
#
#   tools/final_session.sh NAME tests     GPU test suite, smoke, the default bench line
#   tools/final_session.sh NAME cfgA      headline, exact, fully-connected, ring100, gradient mean
#   tools/final_session.sh NAME cfgB      10 000 nodes (fast, exact), dense bf16x6, dense fp32
#   tools/final_session.sh NAME e2e       the host-resident round (bench.py --e2e --e2e-step)
#
#   tools/final_session.sh NAME merge     (here, after the parts) stamps of every part -> profiles/traffic.json
#
# Per config: a bench line, a kernel trace (--stats) and two separate PMC passes (FETCH_SIZE,
# WRITE_SIZE) whose per-launch bytes are stamped with the library hash into $O/traffic_PART.json
# (seeded from profiles/traffic.json: each part runs on a fresh box, and one file per part keeps a
# later part's merge from overwriting an earlier part's stamps).  Every GPU step has its own time
# limit; a step that fails ends the session.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
O=gpurun_out/${1:-final}; PART=${2:-tests}; mkdir -p $O; export TMPDIR=/tmp
T=$O/traffic_$PART.json
[ "$PART" = merge ] || [ -f $T ] || cp profiles/traffic.json $T
one() {   # name kernel-substring alg-bytes bench-args...
  n=$1; k=$2; alg=$3; shift 3
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > $O/bench_$n.json 2> $O/bench_$n.err || { echo "bench $n failed"; tail -5 $O/bench_$n.err; return 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/kt_$n -o kt -- python3 $R/bench.py --no-cpu-baseline --no-cold-cache "$@" > $O/kt_$n.log 2>&1 || { echo "trace $n failed"; tail -5 $O/kt_$n.log; return 1; }
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $R/$O/pmc_${n}_$c -o p -- python3 $R/bench.py --no-cpu-baseline --no-cold-cache "$@" > $O/pmc_${n}_$c.log 2>&1 || { echo "pmc $n $c failed"; tail -5 $O/pmc_${n}_$c.log; return 1; }
  done
  python tools/pmc_traffic.py $O/pmc_${n}_FETCH_SIZE $O/pmc_${n}_WRITE_SIZE $k --alg-bytes $alg --key-from $O/bench_$n.json --out $T > $O/traffic_$n.txt || return 1
  python -c "import json;d=json.load(open('$O/bench_$n.json'));t=json.load(open('$O/traffic_$n.txt'));print('$n', d['ms_per_step'], 'ms', d['roofline']['frac'], 'traffic x', round(t['ratio_to_algorithmic'],4))"
}
case $PART in
  tests)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; grep -E "FAILED" $O/pytest_gpu.log | head
    [ $rc -ne 0 ] && exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; cat $O/smoke.log; exit 3; }
    tail -1 $O/smoke.log
    timeout -k 10 600 python bench.py > $O/bench_headline_default.json 2> $O/bench_headline_default.err || { echo bench failed; tail $O/bench_headline_default.err; exit 4; }
    cat $O/bench_headline_default.json ;;
  cfgA)
    one headline k_mix_clique 8388608000 --steps 20 || exit 5
    one exact k_mix_tile_lds 8388608000 --kernel tile-lds-exact --steps 10 || exit 5
    one fc1000 k_mix_bigclique 8388608000 --config fc1000 --steps 10 || exit 5
    one ring100 k_mix_strip 49604800 --config ring100 --steps 200 || exit 5
    one grad k_grad_segment_mean 8388608000 --workload grad-clique --steps 10 || exit 5 ;;
  cfgB)
    one d10k k_mix_clique 83886080000 --config dcliques10000 --steps 5 --warmup 2 || exit 5
    one d10k_exact k_mix_tile_lds 83886080000 --config dcliques10000 --kernel tile-lds-exact --steps 3 --warmup 1 || exit 5
    one dense k_mix_dense_b6 8388608000 --config fc1000 --kernel dense --steps 5 --warmup 2 || exit 5
    one dense_f32 "k_mix_dense<" 8388608000 --config fc1000 --kernel dense-f32 --steps 3 --warmup 1 || exit 5 ;;
  e2e)
    timeout -k 10 1000 python bench.py --no-cpu-baseline --e2e --e2e-step --steps 3 > $O/bench_e2e.json 2> $O/bench_e2e.err || { echo e2e failed; tail $O/bench_e2e.err; exit 6; }
    python -c "import json;d=json.load(open('$O/bench_e2e.json'));e=d['e2e']['next_step'];[print(k, v) for k, v in e.items() if isinstance(v, dict)]" ;;
  merge)
    python - "$O" <<'PY' || exit 7
import glob, json, sys
path = "profiles/traffic.json"
out = json.load(open(path))
# the library the parts measured (every bench line of the session carries its hash); a part's
# other entries are its seed, possibly older than another part's stamps
libs = {json.load(open(b))["config"]["lib_sha16"] for b in glob.glob(sys.argv[1] + "/bench_*.json")
        if "e2e" not in b}
assert len(libs) == 1, libs
lib = libs.pop()
for f in sorted(glob.glob(sys.argv[1] + "/traffic_*.json")):
    for k, v in json.load(open(f))["entries"].items():
        if v.get("lib_sha16") == lib and v != out["entries"].get(k):
            out["entries"][k] = v
            print("stamped", lib, k)
json.dump(out, open(path, "w"), indent=1, sort_keys=True)
PY
    ;;
  *) echo "unknown part $PART"; exit 2 ;;
esac
echo "part $PART done"
