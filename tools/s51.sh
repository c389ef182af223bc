#!/bin/bash
# blocked-layout gradient segment mean: parity + grad-clique bench blocked vs row-major
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s51; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_memory.py tests/test_gpu_gradient.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for lay in blocked rowmajor blocked rowmajor; do
  timeout -k 10 300 python bench.py --workload grad-clique --layout $lay --no-cpu-baseline > $O/b_$lay.json 2> $O/b_$lay.err || { tail -5 $O/b_$lay.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b_$lay.json')); print('$lay', d['ms_per_step'], d['roofline']['frac'], d['config'].get('slab_layout'))"
done
