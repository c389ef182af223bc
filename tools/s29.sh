#!/bin/bash
# Round-1 refresh: rocprof kernel-trace + PMC traffic of the headline, all configs, grad, final bench
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/${OUTDIR:-s29}; mkdir -p $O
bash tools/profile_session.sh ${OUTDIR:-s29}/prof || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_grad" -o kt -- python3 "$R/bench.py" --workload grad-clique --no-cpu-baseline --steps 10 --warmup 2 > $O/prof_grad.log 2>&1 || { echo "grad kt failed"; tail -5 $O/prof_grad.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_exact" -o kt -- python3 "$R/bench.py" --kernel tile-lds-exact --no-cpu-baseline --steps 5 --warmup 1 > $O/prof_exact.log 2>&1 || { echo "exact kt failed"; tail -5 $O/prof_exact.log; exit 1; }
bash tools/configs_session.sh ${OUTDIR:-s29}/cfg || exit 1
run() { local name=$1; shift; timeout -k 10 400 python bench.py --no-cpu-baseline "$@" > "$O/cfg/$name.json" 2> "$O/cfg/$name.err" || { echo "$name failed"; tail -5 "$O/cfg/$name.err"; return 1; }; python -c "import json; d=json.load(open('$O/cfg/$name.json')); print('$name', d['ms_per_step'], d['value'], d['config']['kernel'], d['roofline']['achieved'], d['roofline']['unit'], d['roofline']['frac'])"; }
run headline_tile_lds_exact --steps 5 --kernel tile-lds-exact || exit 1
run headline_tile_exact --steps 5 --kernel tile-exact || exit 1
run fc1000_auto --steps 10 --config fc1000 || exit 1
run smallworld_exact --steps 5 --config dcliques1000-smallworld --kernel tile-lds-exact || exit 1
timeout -k 10 300 python bench.py --workload grad-clique --steps 20 --e2e > $O/grad.json 2> $O/grad.err || { tail -5 $O/grad.err; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
cat $O/bench.json
