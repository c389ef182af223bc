#!/bin/bash
# clique kernel with 128 residual entries lane-parallel: parity + 10 000-node single-GPU round
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/s44; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_memory.py tests/test_gpu_shard.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
timeout -k 10 400 python bench.py --config dcliques10000 --steps 10 --warmup 2 > $O/d10k.json 2> $O/d10k.err || { tail -5 $O/d10k.err; exit 1; }
python -c "import json; d=json.load(open('$O/d10k.json')); print('d10k', d['ms_per_step'], d['roofline']['frac'], d['config']['stream_copy_GBs'])"
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench.json')); print('headline', d['ms_per_step'], d['roofline']['frac'], d['config']['stream_copy_GBs'])"
