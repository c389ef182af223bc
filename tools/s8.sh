set -e
O=gpurun_out/s8; mkdir -p $O
for pad in 0 256; do for t in 16x7x8x0x0 16x7x8x0x2 8x13x4x0x0 8x13x4x0x2; do
  NIIDMIX_CLIQUE_TILE=$t timeout -k 10 120 python bench.py --no-cpu-baseline --steps 40 --ld-pad $pad > $O/bench_${t}_$pad.json
  echo $t $pad $(python -c "import json;d=json.load(open('$O/bench_${t}_$pad.json'));print(d['ms_per_step'],d['roofline']['achieved'])")
done; done
timeout -k 10 100 ./tools/hbm_probe3 > $O/probe3.txt
