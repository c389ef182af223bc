#!/bin/bash
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s50; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/ring" -o kt -- python3 "$R/bench.py" --config ring100 --no-cpu-baseline --steps 200 --graph off > $O/ring.log 2>&1 || { tail -5 $O/ring.log; exit 1; }
python3 -c "
import csv,glob
for f in glob.glob('$O/ring/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        print(r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3, 'us', float(r['MinNs'])/1e3)
"
grep -h "^{" $O/ring.log | tail -1 | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['ms_per_step'], d['config']['launch_ms'])"
