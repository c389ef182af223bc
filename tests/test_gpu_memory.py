"""VMM-mapped node-state slabs (niidmix.memory / niidmix_hbm_alloc): ordinary torch tensors that
the mixing kernels read and write bit-identically, freed and re-allocated through the MemPool."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


def test_slab_roundtrip_and_reuse(gpu):
    from niidmix import memory
    a = memory.empty_slab(1000, 1 << 16, gpu)
    assert a.is_cuda and a.shape == (1000, 1 << 16) and a.data_ptr() % (2 << 20) == 0
    src = torch.arange(a.numel(), dtype=torch.float32).view_as(a)
    a.copy_(src.to(gpu))
    assert torch.equal(a.cpu(), src)
    ptr = a.data_ptr()
    del a
    b = memory.empty_slab(1000, 1 << 16, gpu)                 # served again from the pool
    b.fill_(3.0)
    torch.cuda.synchronize()
    assert float(b.sum()) == 3.0 * b.numel()
    del b
    torch.cuda.synchronize()
    assert ptr != 0


def test_kernels_on_slab_memory_bitwise(gpu, oracle_mod):
    from niidmix import memory, ops
    g = load_golden("dcliques1000_fc_p64")
    m = ops.Mixer(csr=ops.csr_from_numpy(g["row_ptr"], g["col"], g["val"]), cliques=g["cliques"],
                  device=gpu)
    x = memory.empty_slab(1000, 64, gpu)
    x.copy_(torch.from_numpy(g["x"]).to(gpu))
    y = memory.empty_slab(1000, 64, gpu)
    m(x, out=y, mode="exact")
    assert oracle_mod.bitwise_equal(y.cpu().numpy(), g["y"])
    m(x, out=y, kernel="clique")
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(y.cpu().numpy(), g["y"], bound, rtol=1e-5)
    assert ok, worst
