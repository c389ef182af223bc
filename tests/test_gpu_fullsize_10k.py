"""Parity at BASELINE.json configs[4]'s sizes (10 000-node d-cliques, P = 2^20), through the same
layouts and launch paths as bench.py --config dcliques10000 and the multi-GPU stripes:

  * the single-GPU fast round exactly as benched: relabeled (clique-contiguous) rows, column-blocked
    VMM slabs [16384, 10000, 64] (the multi-clique tile's layout: a 64-column chunk of every row is
    one contiguous stretch), the clique kernel (k_mix_clique_q); EVERY element against the exact
    kernel's round of the same input (1e-5 condition-aware, tests/fullcheck.py), 32 random blocks
    plus the first and last against the oracle (the last starts 1.05e10 elements into the slab:
    past 2^31, 2^32 and 2^33), plus column-sum preservation over every block; and the same on the
    round-2 layout [4096, 10000, 256] (NIIDMIX_Q_BLOCK_COLS=256);
  * the exact default (tile-lds-exact: since round 4 each clique's 99 inter-clique sources are
    register rows, 100 staged rows -> 128-column items; NIIDMIX_TLDS_REMOTE=0 stages all 199 rows ->
    96-column items) on row-major [10000, 2^20] slabs, bitwise on windows that straddle item
    boundaries, the ragged last item, rows whose offsets exceed 2^33 elements and 16 random
    windows;
  * one rank of the 8000-node weak N=8 column-stripe shape (StripedMixer: 79 gateway terms per
    clique, B = 64), windows against the oracle and column sums over the whole stripe.

Columns of Θ' = Wᵀ Θ are independent (d_sgd.py:96-116 mixes every tensor element-wise), so a column
window of the oracle is the full computation restricted to those columns.  Reference topology:
random_cliques.py:43-44 (fully-connected interclique by default), interclique.py:57-75.
"""
import numpy as np
import pytest
import torch

from fullcheck import check_blocked_every_element

pytestmark = pytest.mark.gpu
RTOL = 1e-5
P_FULL = 1 << 20


@pytest.fixture(scope="module")
def dc10k():
    from niidmix.generate import dcliques_csr
    return dcliques_csr(10000, 100, "fully-connected", 1337)


def _free():
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _check_fast(oracle_mod, csr, xw, yw, what):
    ref = oracle_mod.mix_exact_c(xw, csr.row_ptr, csr.col, csr.val)
    bound = oracle_mod.condition_bound(xw, csr.row_ptr, csr.col, csr.val)
    ok, worst = oracle_mod.check_tolerance(yw, ref, bound, rtol=RTOL)
    assert ok, (what, worst)


def _blocked_colsum_gap(xb, yb):
    """max |colsum(x) - colsum(y)| over every column of two [K, N, B] slabs (fp64 sums)."""
    gap = 0.0
    for k0 in range(0, xb.shape[0], 256):
        sx = torch.sum(xb[k0:k0 + 256], dim=1, dtype=torch.float64)
        sy = torch.sum(yb[k0:k0 + 256], dim=1, dtype=torch.float64)
        gap = max(gap, torch.max(torch.abs(sx - sy)).item())
    return gap


@pytest.mark.parametrize("bc_env,qm", [("", ""), ("256", ""), ("", "8,4,4"), ("", "8,7,4,2"), ("", "16,4,4,2")])
def test_dcliques10000_single_gpu_as_benched(dc10k, gpu, oracle_mod, monkeypatch, bc_env, qm):
    """qm: the member-split multi-clique tile (NIIDMIX_CLIQUE_QM=W,R,OCC, round 6)."""
    from niidmix import memory, ops
    if bc_env:
        monkeypatch.setenv("NIIDMIX_Q_BLOCK_COLS", bc_env)
    if qm:
        monkeypatch.setenv("NIIDMIX_CLIQUE_QM", qm)
    csr, cliques = dc10k
    m = ops.Mixer(csr=csr, cliques=cliques, device=gpu)
    assert m.kernel_for("fast") == "clique" and m.plan.max_clique_res == 99
    perm, bc = m.device_layout()
    assert perm is not None and bc == (int(bc_env) if bc_env else 64)
    m = m.relabeled(perm)
    xb = memory.empty_blocked(10000, P_FULL, gpu, bc)
    kb = P_FULL // bc
    assert tuple(xb.shape) == (kb, 10000, bc)
    xb.normal_(generator=torch.Generator(device=gpu).manual_seed(10))
    yb = memory.empty_blocked(10000, P_FULL, gpu, bc)
    yb.fill_(float("nan"))                       # every output element must be written
    m.mix_blocked(xb, yb, P_FULL)
    torch.cuda.synchronize()
    assert (kb - 1) * xb.stride(0) > (1 << 33)
    assert not torch.isnan(yb).any().item()
    # every element against the exact kernel; 32 random blocks + first / last vs the oracle
    check_blocked_every_element(m, xb, yb, P_FULL, oracle_mod, seed=22 + len(bc_env))
    assert _blocked_colsum_gap(xb, yb) < 2e-3
    del xb, yb
    _free()


@pytest.mark.parametrize("remote", ["auto", "0"])
def test_dcliques10000_tile_lds_exact_rowmajor(remote, dc10k, gpu, oracle_mod, monkeypatch):
    from niidmix import memory, ops
    monkeypatch.setenv("NIIDMIX_TLDS_REMOTE", remote)
    csr, cliques = dc10k
    m = ops.Mixer(csr=csr, cliques=cliques, device=gpu)
    assert m.kernel_for("exact") == "tile-lds-exact"
    if remote == "auto":
        # up to 15 register rows per tile: 8 with the rest staged would not fit three blocks
        assert m.tlds.max_src == 100 and m.tlds.rem_rows is not None and m.tlds.rem_regs == 16
        cw = 128           # 102 x 128 x 4 B = 52 KB per block; P = 2^20 = 8192 x 128: exact items
    else:
        assert m.tlds.max_src == 199 and m.tlds.rem_rows is None
        cw = 96            # 199 x 96 x 4 B = 76 KB: two blocks per CU; 2^20 = 10922 x 96 + 64
    x = memory.empty_slab(10000, P_FULL, gpu)
    x.normal_(generator=torch.Generator(device=gpu).manual_seed(11))
    y = memory.empty_slab(10000, P_FULL, gpu)
    y.fill_(float("nan"))
    m(x, out=y, mode="exact")
    torch.cuda.synchronize()
    w = cw * 3
    rng = np.random.default_rng(23)
    picks = [int(c) for c in rng.integers(0, P_FULL - w, size=16)]
    for c0 in [0, cw * 5461 - 40, P_FULL - w] + picks:
        xw = x[:, c0:c0 + w].cpu().numpy()
        ref = oracle_mod.mix_exact_c(xw, csr.row_ptr, csr.col, csr.val)
        assert oracle_mod.bitwise_equal(y[:, c0:c0 + w].cpu().numpy(), ref), c0
    # every element written; column sums preserved over ALL columns
    assert not torch.isnan(y).any().item()
    sx = torch.zeros(P_FULL, dtype=torch.float64, device=gpu)
    sy = torch.zeros(P_FULL, dtype=torch.float64, device=gpu)
    for r0 in range(0, 10000, 1000):
        sx += torch.sum(x[r0:r0 + 1000], dim=0, dtype=torch.float64)
        sy += torch.sum(y[r0:r0 + 1000], dim=0, dtype=torch.float64)
    assert torch.max(torch.abs(sx - sy)).item() < 2e-3
    del x, y
    _free()


def test_dcliques8000_stripe_rank7(gpu, oracle_mod):
    """Weak-scaling N=8's per-rank shape: 8000 nodes (80 cliques, 79 gateway terms each, B = 64),
    rank 7's column stripe [917504, 1048576) of P = 2^20 through StripedMixer."""
    from niidmix.shard import StripedMixer
    sm = StripedMixer.dcliques(8000, 100, world=8, rank=7, interclique="fully-connected",
                               device=gpu, p=P_FULL)
    assert sm.blocked and sm.block_cols == 64 and sm.mixer.plan.max_clique_res == 79
    assert (sm.c0, sm.c1) == (7 * (P_FULL // 8), P_FULL)
    x = torch.randn(8000, sm.p_local, device=gpu, generator=torch.Generator(device=gpu).manual_seed(12))
    xb, yb = sm.to_layout(x), sm.empty()
    sm(xb, yb)
    y = sm.from_layout(yb)
    torch.cuda.synchronize()
    # the rank-order CSR (the stripe mixer runs the relabeled one)
    from niidmix.generate import dcliques_csr
    csr, _ = dcliques_csr(8000, 100, "fully-connected", 1337)
    w = 512
    for c0 in (0, sm.p_local // 2 - 200, sm.p_local - w):
        _check_fast(oracle_mod, csr, x[:, c0:c0 + w].cpu().numpy(), y[:, c0:c0 + w].cpu().numpy(), c0)
    gap = torch.max(torch.abs(torch.sum(x, 0, dtype=torch.float64) -
                              torch.sum(y, 0, dtype=torch.float64))).item()
    assert gap < 2e-3
    del x, xb, yb, y
    _free()
