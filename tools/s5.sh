set -e
O=gpurun_out/s5; mkdir -p $O
timeout -k 10 100 ./tools/hbm_probe2 > $O/probe2.txt
for t in 16x7x8x0x0 16x7x8x0x2 8x13x4x0x0 8x13x4x0x2 16x7x8x0x0; do
  NIIDMIX_CLIQUE_TILE=$t timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 > $O/bench_$t.json
  echo $t $(python -c "import json;d=json.load(open('$O/bench_$t.json'));print(d['ms_per_step'],d['roofline']['achieved'])")
done
