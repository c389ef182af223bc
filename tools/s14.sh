set -e
O=gpurun_out/s14; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
NIIDMIX_LIB=$PWD/tools/libniidmix_old.so timeout -k 10 100 python tools/ab_clique.py --variants 16x7x8x0x0,16x7x8x0x2 2>&1 | grep -v amdgpu.ids | sed 's/^/old /'
timeout -k 10 100 python tools/ab_clique.py --variants 16x7x8x64x0,16x7x8x64x2,16x7x8x0x0,8x13x4x64x0,8x13x4x64x2 2>&1 | grep -v amdgpu.ids | sed 's/^/new /'
done
timeout -k 10 60 ./tools/hbm_probe5 | head -3
