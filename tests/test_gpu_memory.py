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


@pytest.mark.parametrize("p", [64, 4096, 10_000, 3 * 4096 + 256])
def test_blocked_clique_equals_rowmajor(p, gpu, oracle_mod):
    """The clique kernel on column-blocked slabs [K, N, B] gives bit-identical results to the
    row-major kernel (same arithmetic, different addresses), partial last block included."""
    from niidmix import memory, ops
    g = load_golden("dcliques1000_fc_p64")
    m = ops.Mixer(csr=ops.csr_from_numpy(g["row_ptr"], g["col"], g["val"]), cliques=g["cliques"],
                  device=gpu)
    gen = torch.Generator(device=gpu).manual_seed(p)
    x = torch.randn(1000, p, device=gpu, generator=gen)
    y_ref = m(x, kernel="clique")
    xb = memory.to_blocked(x)
    yb = memory.empty_blocked(1000, p, gpu)
    m.mix_blocked(xb, yb, p)
    y = memory.from_blocked(yb, p)
    assert torch.equal(y, y_ref)
    if p == 64:
        bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
        xg = memory.to_blocked(torch.from_numpy(g["x"]).to(gpu))
        m.mix_blocked(xg, yb, 64)
        ok, worst = oracle_mod.check_tolerance(memory.from_blocked(yb, 64).cpu().numpy(), g["y"],
                                               bound, rtol=1e-5)
        assert ok, worst


@pytest.mark.parametrize("p", [64, 10_000, 3 * 4096 + 256])
def test_blocked_grad_mean_equals_rowmajor(p, gpu, oracle_mod):
    """The clique-gradient segment mean on column-blocked slabs is bit-identical to the row-major
    kernel, and at p=64 to the reference's own averaged gradients (average_gradients,
    d_sgd.py:19-27)."""
    from conftest import load_grad
    from niidmix import gradient, memory
    d, topo, params = load_grad("grad_dcliques1000_fc_p64")
    plan = gradient.build_grad_plan(d["g"].shape[0], topo, params)
    gm = gradient.GradMean(plan, gpu)
    if p == 64:
        x = torch.from_numpy(d["g"]).to(gpu)
    else:
        x = torch.randn(plan.n, p, device=gpu, generator=torch.Generator(device=gpu).manual_seed(p))
    y_ref = gm(x)
    yb = memory.empty_blocked(plan.n, p, gpu)
    gm.mean_blocked(memory.to_blocked(x), yb, p)
    y = memory.from_blocked(yb, p)
    assert torch.equal(y, y_ref)
    if p == 64:
        stepped = np.zeros(plan.n, bool)
        stepped[plan.stepped] = True
        assert oracle_mod.bitwise_equal(y.cpu().numpy()[stepped], d["g_out"][stepped])
