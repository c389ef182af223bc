#!/bin/bash
# SQ counters of the exact-mode tile kernels (LDS vs global) and the clique kernel
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s23; mkdir -p $O
export TMPDIR=/tmp
for k in tile-lds-exact tile-exact; do
  A="--no-cpu-baseline --steps 3 --warmup 1 --kernel $k"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS --kernel-trace --output-format csv -d "$R/$O/$k-a" -o a -- python3 "$R/bench.py" $A > $O/$k-a.log 2>&1 || { echo "pass a $k failed"; tail -20 $O/$k-a.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --kernel-trace --output-format csv -d "$R/$O/$k-b" -o b -- python3 "$R/bench.py" $A > $O/$k-b.log 2>&1 || { echo "pass b $k failed"; tail -20 $O/$k-b.log; exit 1; }
done
python3 - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/s23/*/*counter_collection.csv")):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "tile" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[2], {k: "%.4g" % (sum(v) / len(v)) for k, v in acc.items()})
PY
