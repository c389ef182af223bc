#!/bin/bash
# column-blocked device layout: tests + bench (blocked vs rowmajor) on several fresh processes
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s37; mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_gpu_memory.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for i in 1 2 3 4; do
  for lay in blocked rowmajor; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --layout $lay > $O/b_${lay}_$i.json 2> $O/b_${lay}_$i.err || { tail -5 $O/b_${lay}_$i.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b_${lay}_$i.json')); print('$lay', $i, d['ms_per_step'], d['roofline']['frac'], d['config']['slab_layout'], d['config']['stream_copy_GBs'])"
  done
done
