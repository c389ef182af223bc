"""Every-element checks of the fast kernels at full size (VERDICT r05 #1a).

A fast-mode round at BASELINE sizes is checked on EVERY output element against the exact kernel's
output of the same input -- the exact kernel (tile-lds-exact) is bit-identical to the oracle
(tests/test_gpu_parity.py on the reference-run fixtures, and on sampled blocks at full size here) --
with the same condition-aware tolerance as oracle.check_tolerance: |y - y_exact| <= rtol *
(|W|^T |X|) + 1e-38, NaN where the exact round has NaN, the same infinities.  The bound |W|^T |X|
is itself computed on the GPU by the exact CSR kernel on |W| and |X| (fp32, the oracle's own
condition_bound restated on the device).  Sampled blocks of the fast output are checked against the
C oracle as well.  Test infrastructure only."""
import numpy as np
import torch


def abs_mixer(csr, device):
    """A Mixer over |W| (exact CSR kernel): the condition bound |W|^T |X| on the device."""
    from niidmix import ops
    a = ops.csr_from_numpy(csr.row_ptr, csr.col, np.abs(csr.val))
    return ops.Mixer(csr=a, device=device, factor=False)


def blocks_rowmajor(xb, k0, k1):
    """Column blocks [k0, k1) of a column-blocked slab [K, rows, B] as one row-major [rows, w]."""
    kw, rows, b = xb[k0:k1].shape
    return xb[k0:k1].permute(1, 0, 2).reshape(rows, kw * b)


def worst_vs_exact(m, ma, xw, yw, rtol=1e-5):
    """Worst |y - y_exact| / (rtol |W|^T|X| + 1e-38) * rtol over a row-major window xw -> yw (rows
    in m's order); asserts the non-finite patterns agree.  Returns (worst, y_exact)."""
    ye = m(xw, mode="exact")
    bd = ma(xw.abs(), mode="exact", kernel="csr-exact")
    nan_e = torch.isnan(ye)
    assert torch.equal(nan_e, torch.isnan(yw)), "NaN pattern differs from the exact round"
    inf_e = torch.isinf(ye)
    assert torch.equal(torch.isinf(yw), inf_e) and torch.equal(yw[inf_e], ye[inf_e]), \
        "infinities differ from the exact round"
    worst = 0.0
    fin = ~(nan_e | inf_e)
    for r0 in range(0, xw.shape[0], 1024):
        sl = slice(r0, r0 + 1024)
        d = (yw[sl].double() - ye[sl].double()).abs()
        lim = rtol * bd[sl].double() + 1e-38
        ratio = torch.where(fin[sl], d / lim, torch.zeros_like(d))
        worst = max(worst, float(ratio.max()) * rtol)
    return worst, ye


def check_blocked_every_element(m, xb, yb, p, oracle_mod, n_oracle=32, seed=0, win_cols=1 << 16,
                                rtol=1e-5):
    """Every element of a blocked fast round (xb -> yb, rows in m's order) against the exact kernel
    (tolerance), plus `n_oracle` randomly drawn column blocks against the C oracle (tolerance) and
    the exact kernel's output on those blocks against the oracle (bitwise).  Returns the worst
    ratio seen."""
    kb, rows, b = xb.shape
    assert kb * b >= p
    ma = abs_mixer(m.csr, xb.device)
    per = max(1, win_cols // b)
    rng = np.random.default_rng(seed)
    picks = set(int(k) for k in rng.choice(kb, size=min(n_oracle, kb), replace=False))
    picks |= {0, kb - 1}
    worst = 0.0
    for k0 in range(0, kb, per):
        k1 = min(kb, k0 + per)
        w = min(p, k1 * b) - k0 * b
        xw = blocks_rowmajor(xb, k0, k1)[:, :w].contiguous()
        yw = blocks_rowmajor(yb, k0, k1)[:, :w].contiguous()
        wr, ye = worst_vs_exact(m, ma, xw, yw, rtol)
        assert wr <= rtol, (k0, wr)
        worst = max(worst, wr)
        for k in sorted(kk for kk in picks if k0 <= kk < k1):
            c0, c1 = (k - k0) * b, min(w, (k - k0 + 1) * b)
            xn = xw[:, c0:c1].cpu().numpy()
            ref = oracle_mod.mix_exact_c(xn, m.csr.row_ptr, m.csr.col, m.csr.val)
            assert oracle_mod.bitwise_equal(ye[:, c0:c1].cpu().numpy(), ref), ("exact", k)
            bound = oracle_mod.condition_bound(xn, m.csr.row_ptr, m.csr.col, m.csr.val)
            ok, wo = oracle_mod.check_tolerance(yw[:, c0:c1].cpu().numpy(), ref, bound, rtol=rtol)
            assert ok, ("oracle", k, wo)
        del xw, yw, ye
    return worst


def check_rowmajor_every_element(m, x, y, oracle_mod, n_oracle=32, seed=0, win_cols=1 << 16,
                                 block=1024, rtol=1e-5):
    """check_blocked_every_element for a row-major fast round x -> y [rows, p]: column windows
    against the exact kernel, `n_oracle` random `block`-column windows against the C oracle."""
    rows, p = x.shape
    ma = abs_mixer(m.csr, x.device)
    nblk = -(-p // block)
    rng = np.random.default_rng(seed)
    picks = set(int(k) for k in rng.choice(nblk, size=min(n_oracle, nblk), replace=False))
    picks |= {0, nblk - 1}
    worst = 0.0
    for c0 in range(0, p, win_cols):
        c1 = min(p, c0 + win_cols)
        xw = x[:, c0:c1].contiguous()
        yw = y[:, c0:c1].contiguous()
        wr, ye = worst_vs_exact(m, ma, xw, yw, rtol)
        assert wr <= rtol, (c0, wr)
        worst = max(worst, wr)
        for k in sorted(kk for kk in picks if c0 <= kk * block < c1):
            a, b = k * block - c0, min(c1, (k + 1) * block) - c0
            xn = xw[:, a:b].cpu().numpy()
            ref = oracle_mod.mix_exact_c(xn, m.csr.row_ptr, m.csr.col, m.csr.val)
            assert oracle_mod.bitwise_equal(ye[:, a:b].cpu().numpy(), ref), ("exact", k)
            bound = oracle_mod.condition_bound(xn, m.csr.row_ptr, m.csr.col, m.csr.val)
            ok, wo = oracle_mod.check_tolerance(yw[:, a:b].cpu().numpy(), ref, bound, rtol=rtol)
            assert ok, ("oracle", k, wo)
        del xw, yw, ye
    return worst
