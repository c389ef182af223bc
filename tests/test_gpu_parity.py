"""GPU parity of the HIP kernels (libniidmix.so through the torch custom ops / C-ABI) against the
golden vectors (bit-exact mode) and the pinned oracle (fast modes, condition-aware 1e-5).

Tolerance for fast kernels (north star: "within 1e-5 relative fp32"): elementwise
|y - y_ref| <= 1e-5 * (|W|^T |Θ|)_ij — relative to the magnitude of the terms summed, because plain
elementwise relative error is ill-posed under cancellation.
"""
import numpy as np
import pytest
import torch

from conftest import golden_cases, load_golden

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def _ops():
    from niidmix import ops
    return ops


def _mixer(g, dev, **kw):
    ops = _ops()
    csr = ops.csr_from_numpy(g["row_ptr"], g["col"], g["val"])
    return ops.Mixer(csr=csr, cliques=g.get("cliques"), device=dev, **kw)


@pytest.mark.parametrize("name", golden_cases())
@pytest.mark.parametrize("kernel", ["csr-exact", "tile-exact", "ell-exact"])
def test_exact_kernel_bitwise_vs_golden(name, kernel, gpu, oracle_mod):
    g = load_golden(name)
    m = _mixer(g, gpu)
    if kernel == "tile-exact" and m.tile is None:
        m = _tile_mixer(g, gpu, 8)
    if kernel == "ell-exact" and m.ell is None:
        pytest.skip("a row has more than 8 entries")
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel=kernel).cpu().numpy()
    assert oracle_mod.bitwise_equal(y, g["y"]), name


@pytest.mark.parametrize("name", golden_cases())
@pytest.mark.parametrize("kernel", ["csr-fast", "clique", "dense", "dense-f32", "tile-fast",
                                    "ell-fast"])
def test_fast_kernels_tolerance_vs_golden(name, kernel, gpu, oracle_mod):
    """Every fast kernel on every golden case, non-finite fixtures included: NaN where the
    reference has NaN, the same inf where it has inf (the factored and GEMM kernels recompute
    non-finite outputs from the CSR, include/niidmix.h), finite outputs within 1e-5 of the
    condition bound."""
    g = load_golden(name)
    m = _mixer(g, gpu)
    p = g["x"].shape[1]
    if kernel == "clique" and (m.plan is None or p % 4):
        pytest.skip(f"no clique plan ({m.plan_reason}) or p % 4")
    if kernel == "tile-fast" and m.tile is None:
        m = _tile_mixer(g, gpu, 16)
    if kernel == "ell-fast" and m.ell is None:
        pytest.skip("a row has more than 8 entries")
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel=kernel).cpu().numpy()
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=RTOL)
    assert ok, f"{name}/{kernel}: worst {worst:.3g}"


def _tile_mixer(g, dev, rt):
    """A Mixer with a tile plan of height rt even for low-degree topologies (tests only)."""
    from niidmix import tile
    m = _mixer(g, dev)
    tp, why = tile.build_tile_plan(m.csr, g.get("cliques"), rt)
    assert tp is not None, why
    m.tile = tp
    m.t_sub_ptr = torch.from_numpy(tp.sub_ptr).to(dev)
    m.t_sub_rows = torch.from_numpy(tp.sub_rows).to(dev)
    m.t_sub_wself = torch.from_numpy(tp.sub_wself).to(dev)
    m.t_pos_src = torch.from_numpy(tp.pos_src).to(dev)
    m.t_pos_mask = torch.from_numpy(tp.pos_mask.view(np.int32)).to(dev)
    m.t_pos_w = torch.from_numpy(tp.pos_w).to(dev)
    return m


@pytest.mark.parametrize("rt", [8, 16, 32])
@pytest.mark.parametrize("name", ["dcliques1000_fc_p64", "dcliques300_fc_p37", "fc64_p33",
                                  "nonfinite_ring8_p16", "n2_ring_linear7850", "ring100_p257"])
def test_tile_exact_heights_bitwise(name, rt, gpu, oracle_mod):
    """Every tile height (8/16/32 rows; vector widths follow p) is bit-identical to the reference,
    including the average-only flag (setup.model.average alone)."""
    g = load_golden(name)
    m = _tile_mixer(g, gpu, rt)
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="tile-exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y, g["y"]), (name, rt)
    ops = _ops()
    out = torch.empty_like(x)
    ops.mix_tile(x, m.t_sub_ptr, m.t_sub_rows, m.t_sub_wself, m.t_pos_src, m.t_pos_mask,
                 m.t_pos_w, out, rt, ops.EXACT | ops.AVERAGE_ONLY)
    ref = oracle_mod.mix_exact_c(g["x"], g["row_ptr"], g["col"], g["val"], average_only=True)
    assert oracle_mod.bitwise_equal(out.cpu().numpy(), ref), (name, rt)


def _tile_lds_mixer(g, dev, rt):
    """A Mixer with an LDS tile plan of height rt for any golden topology (tests only): cliques
    as groups where the fixture has them, else consecutive row blocks."""
    from niidmix import tile
    m = _mixer(g, dev)
    cl = g.get("cliques")
    if not cl:
        span = rt * tile.LDS_MAX_WAVES[rt]
        cl = [list(range(s, min(s + span, m.n))) for s in range(0, m.n, span)]
    lp, why = tile.build_tile_lds_plan(m.csr, cl, rt)
    if lp is None:
        pytest.skip(why)
    ts = tile.build_tile_segments(lp) if rt == 16 else None
    m.set_tile_lds_plan(lp, ts, tile.build_tile_mfma_positions(lp) if ts is not None else None)
    return m


@pytest.mark.parametrize("rt", [8, 16, 32])
@pytest.mark.parametrize("name", golden_cases())
def test_tile_lds_bitwise(name, rt, gpu, oracle_mod):
    """The LDS-staged tile kernel (exact) is bit-identical to the reference on every golden case
    and tile height, average-only flag included; fast mode meets the 1e-5 condition-aware bound."""
    g = load_golden(name)
    if g["x"].shape[1] % 2:
        pytest.skip("odd p: the LDS tile kernel reads column pairs")
    m = _tile_lds_mixer(g, gpu, rt)
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="tile-lds-exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y, g["y"]), (name, rt)
    ops = _ops()
    lp = m.tlds
    out = torch.empty_like(x)
    ops.mix_tile_lds(x, m.l_sub_ptr, m.l_sub_rows, m.l_sub_slot, m.l_sub_wself, m.l_pos_slot,
                     m.l_pos_mask, m.l_pos_w, m.l_grp_tile_ptr, m.l_grp_src_ptr, m.l_grp_src_rows,
                     out, rt, lp.max_src, lp.max_tiles, ops.EXACT | ops.AVERAGE_ONLY)
    ref = oracle_mod.mix_exact_c(g["x"], g["row_ptr"], g["col"], g["val"], average_only=True)
    assert oracle_mod.bitwise_equal(out.cpu().numpy(), ref), (name, rt)
    if np.all(np.isfinite(g["x"])):
        yf = m(x, kernel="tile-lds-fast").cpu().numpy()
        bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
        ok, worst = oracle_mod.check_tolerance(yf, g["y"], bound, rtol=RTOL)
        assert ok, (name, rt, worst)


@pytest.mark.parametrize("rt", [8, 16])
@pytest.mark.parametrize("name", golden_cases())
def test_tile_lds_bitwise_full_height_tiles(name, rt, gpu, oracle_mod, monkeypatch):
    """Tiles of RT rows (no unused slot: NIIDMIX_TILE_LDS_PAD=0; the rt-16 default, whose
    hand-scheduled loop needs no pad), so rt 8's positions every row takes go through the
    per-position path instead of the save/restore of the pad slot: still bit-identical."""
    monkeypatch.setenv("NIIDMIX_TILE_LDS_PAD", "0")
    g = load_golden(name)
    if g["x"].shape[1] % 2:
        pytest.skip("odd p: the LDS tile kernel reads column pairs")
    m = _tile_lds_mixer(g, gpu, rt)
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="tile-lds-exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y, g["y"]), (name, rt)


@pytest.mark.parametrize("cols", ["120", "96"])
@pytest.mark.parametrize("name", golden_cases())
def test_tile_lds_narrow_items_bitwise(name, cols, gpu, oracle_mod, monkeypatch):
    """120- and 96-column items (the launcher's choice when that lets another block share a CU;
    forced here by NIIDMIX_TLDS_COLS) are bit-identical on every golden case with even p."""
    monkeypatch.setenv("NIIDMIX_TLDS_COLS", cols)
    g = load_golden(name)
    if g["x"].shape[1] % 2:
        pytest.skip("odd p: the LDS tile kernel reads column pairs")
    m = _tile_lds_mixer(g, gpu, 16)
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="tile-lds-exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y, g["y"]), (name, cols)


@pytest.mark.parametrize("name", golden_cases())
def test_tile_lds_segment_loop_bitwise(name, gpu, oracle_mod):
    """RT-16 LDS tiles with the segment loop (runs of consecutive slots at immediate offsets,
    MASKED entries for the rest; niidmix.tile.build_tile_segments) and with the per-position loop:
    both bit-identical to the reference, exact and average-only; fast within 1e-5."""
    g = load_golden(name)
    if g["x"].shape[1] % 2:
        pytest.skip("odd p: the LDS tile kernel reads column pairs")
    m = _tile_lds_mixer(g, gpu, 16)
    assert m.tseg is not None and m.tseg.lp is m.tlds
    x = torch.from_numpy(g["x"]).to(gpu)
    for seg in (True, False):
        m.use_segments = seg
        y = m(x, kernel="tile-lds-exact").cpu().numpy()
        assert oracle_mod.bitwise_equal(y, g["y"]), (name, seg)
    ops = _ops()
    lp = m.tlds
    out = torch.empty_like(x)
    ops.mix_tile_lds(x, m.l_sub_ptr, m.l_sub_rows, m.l_sub_slot, m.l_sub_wself, m.l_pos_slot,
                     m.l_pos_mask, m.l_pos_w, m.l_grp_tile_ptr, m.l_grp_src_ptr, m.l_grp_src_rows,
                     out, 16, lp.max_src, lp.max_tiles, ops.EXACT | ops.AVERAGE_ONLY, m.s_seg_ptr,
                     m.s_seg, m.s_seg_w)
    ref = oracle_mod.mix_exact_c(g["x"], g["row_ptr"], g["col"], g["val"], average_only=True)
    assert oracle_mod.bitwise_equal(out.cpu().numpy(), ref), name
    if np.all(np.isfinite(g["x"])):
        m.use_segments = True
        yf = m(x, kernel="tile-lds-fast").cpu().numpy()
        bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
        ok, worst = oracle_mod.check_tolerance(yf, g["y"], bound, rtol=RTOL)
        assert ok, (name, worst)


@pytest.mark.parametrize("mf_waves", ["", "3", "-3"])
@pytest.mark.parametrize("name", golden_cases())
def test_tile_lds_mfma_bitwise(name, mf_waves, gpu, oracle_mod, monkeypatch):
    """The exact matrix-core path (v_mfma_f32_16x16x4_f32 with 0/1 row masks; blocks whose staged
    rows hold a non-finite or tiny value fall back to the segment walker; Mixer.use_mfma, off by
    default) is bit-identical to the reference on every golden case, non-finite fixtures included,
    and to the walker."""
    g = load_golden(name)
    if g["x"].shape[1] % 2:
        pytest.skip("odd p: the LDS tile kernel reads column pairs")
    if mf_waves:      # "3": the first 3 waves of a block on the matrix cores, the rest walk
        # segments; "-3": every 3rd column chunk's blocks on the matrix cores, the others walk
        monkeypatch.setenv("NIIDMIX_TLDS_MF_WAVES", mf_waves)
    m = _tile_lds_mixer(g, gpu, 16)
    assert m.tmf is not None and m.tmf.lp is m.tlds
    x = torch.from_numpy(g["x"]).to(gpu)
    for use in (True, False):
        m.use_mfma = use
        y = m(x, kernel="tile-lds-exact").cpu().numpy()
        assert oracle_mod.bitwise_equal(y, g["y"]), (name, use)


@pytest.mark.parametrize("p", [1002, 1 << 16])
def test_tile_lds_mfma_random_and_fallback_blocks(p, gpu, oracle_mod):
    """1000-node d-cliques on random data: every block on the matrix cores; then zeros, -0.0, a
    subnormal, an inf and a NaN planted in a few column chunks, whose blocks take the walker while
    the rest stay on the MFMA path: bitwise the C oracle either way (ragged last item at p=1002)."""
    g = load_golden("dcliques1000_fc_p64")
    m = _tile_lds_mixer(g, gpu, 16)
    m.use_mfma = True
    rng = np.random.default_rng(p)
    x = (rng.standard_normal((1000, p)) * np.exp2(rng.integers(-20, 20, (1000, p)))).astype(np.float32)
    ref = oracle_mod.mix_exact_c(x, g["row_ptr"], g["col"], g["val"])
    y = m(torch.from_numpy(x).to(gpu), kernel="tile-lds-exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y, ref)
    x2 = x.copy()
    x2[3, 5] = 0.0
    x2[17, 130] = -0.0
    x2[400, 261] = np.float32(1e-42)
    x2[999, p - 1] = np.inf
    x2[250, p // 2] = np.nan
    ref2 = oracle_mod.mix_exact_c(x2, g["row_ptr"], g["col"], g["val"])
    y2 = m(torch.from_numpy(x2).to(gpu), kernel="tile-lds-exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y2, ref2)


@pytest.mark.parametrize("n,size,inter", [(1000, 10, "fully-connected"), (600, 30, "smallworld"),
                                          (2000, 100, "ring")])
def test_tile_lds_segment_loop_masked_heavy(n, size, inter, gpu, oracle_mod):
    """Topologies whose tiles are mostly MASKED entries (cliques of 10: most positions are one
    gateway row's inter-clique edge) or many-tile cliques (100 members, 7 tiles): the segment
    loop is bitwise the C oracle, with 120-column items and a ragged last item (p = 1002)."""
    from niidmix.generate import dcliques_csr
    csr, cl = dcliques_csr(n, size, inter, 1337)
    g = {"row_ptr": csr.row_ptr, "col": csr.col, "val": csr.val, "cliques": cl}
    m = _tile_lds_mixer(g, gpu, 16)
    assert m.tseg is not None
    x = np.random.default_rng(n).standard_normal((n, 1002)).astype(np.float32)
    y = m(torch.from_numpy(x).to(gpu), kernel="tile-lds-exact").cpu().numpy()
    ref = oracle_mod.mix_exact_c(x, csr.row_ptr, csr.col, csr.val)
    assert oracle_mod.bitwise_equal(y, ref), (n, size, inter)


@pytest.mark.parametrize("p", [1002, 256])
@pytest.mark.parametrize("mode", ["exact", "fast"])
@pytest.mark.parametrize("two", ["1", "0"])
@pytest.mark.parametrize("n", [2000, 3000])
def test_tile_lds_register_rows_two_phase(n, two, mode, p, gpu, oracle_mod, monkeypatch):
    """16 register rows per tile walked in two phases of 8 (rem_regs -16, NIIDMIX_TLDS_REM2):
    d-cliques of 100 with 20 / 30 cliques put 10-15 gateway rows -- register rows -- in a tile,
    so the walk reloads rows 8..15 mid-tile.  Exact: bitwise the C oracle, with -0.0, a
    subnormal and inf / NaN in register rows (they reach only the rows reading them); fast:
    within the tolerance.  two = "0": the 16-register kernel on the same plan."""
    from niidmix.generate import dcliques_csr
    monkeypatch.setenv("NIIDMIX_TLDS_REM2", two)
    csr, cl = dcliques_csr(n, 100, "fully-connected", 1337)
    g = {"row_ptr": csr.row_ptr, "col": csr.col, "val": csr.val, "cliques": cl}
    m = _mixer(g, gpu)
    lp = m.tlds
    assert lp is not None and lp.rem_rows is not None and lp.rem_regs == 16 and m.tlds_rem2
    assert int((lp.rem_rows.reshape(-1, 16) >= 0).sum(1).max()) > 8
    x = np.random.default_rng(n + p).standard_normal((n, p)).astype(np.float32)
    regs = np.unique(lp.rem_rows[lp.rem_rows >= 0])
    x[regs[0], 3] = -0.0
    x[regs[1], 5] = np.float32(1e-42)
    if mode == "exact":
        x[regs[-1], 7] = np.inf
        x[regs[-2], 9] = np.nan
    y = m(torch.from_numpy(x).to(gpu), kernel="tile-lds-" + mode).cpu().numpy()
    ref = oracle_mod.mix_exact_c(x, csr.row_ptr, csr.col, csr.val)
    if mode == "exact":
        assert oracle_mod.bitwise_equal(y, ref), (n, two)
        # every reader of the register row (its clique and its remote gateway) and no other; the
        # row's own output is NaN (x_self * 0)
        assert (~np.isfinite(y[:, 7])).sum() == (csr.col == regs[-1]).sum()
        assert np.isnan(y[regs[-1], 7]) and np.isinf(y[:, 7]).sum() == (csr.col == regs[-1]).sum() - 1
        assert np.isnan(y[:, 9]).sum() == (csr.col == regs[-2]).sum()
    else:
        bound = oracle_mod.condition_bound(x, csr.row_ptr, csr.col, csr.val)
        ok, worst = oracle_mod.check_tolerance(y, ref, bound, rtol=RTOL)
        assert ok, (n, two, worst)


@pytest.mark.parametrize("remote", ["0", "auto"])
def test_tile_lds_narrow_items_float2(remote, gpu, oracle_mod, monkeypatch):
    """The all-staged 1000-node d-cliques plan picks 120-column items by itself (109 staged
    rows); the default plan (8 register rows per tile, 101 staged) 128-column items; p = 1002
    (p % 4 == 2: float2 staging) ends in a ragged item.  Bitwise against the C oracle."""
    monkeypatch.setenv("NIIDMIX_TLDS_REMOTE", remote)
    g = load_golden("dcliques1000_fc_p64")
    x = np.random.default_rng(5).standard_normal((g["x"].shape[0], 1002)).astype(np.float32)
    x[3, 7] = -0.0
    x[11, 1001] = np.float32(1e-42)
    m = _mixer(g, gpu)                  # the Mixer's own plan choice (RT 16, segments)
    assert m.tlds is not None and m.tlds.tile.rt == 16 and m.tseg is not None
    if remote == "0":
        assert m.tlds.rem_rows is None
        assert m.tlds.max_src * 128 * 4 > 160 * 1024 // 3 >= m.tlds.max_src * 120 * 4
    else:
        assert m.tlds.rem_rows is not None and m.tlds.rem_regs == 8
        assert (m.tlds.max_src + 2) * 128 * 4 + 1024 <= 160 * 1024 // 3
    y = m(torch.from_numpy(x).to(gpu), kernel="tile-lds-exact").cpu().numpy()
    ref = oracle_mod.mix_exact_c(x, g["row_ptr"], g["col"], g["val"])
    assert oracle_mod.bitwise_equal(y, ref)


def test_tile_lds_strided_window(gpu, oracle_mod):
    """A column window of a wider slab (ld > p, p not a multiple of 128 or 4)."""
    g = load_golden("dcliques1000_fc_p64")
    m = _tile_lds_mixer(g, gpu, 16)
    gen = torch.Generator().manual_seed(3)
    full = torch.randn(1000, 1000, generator=gen)
    x = full.to(gpu)[:, 2:2 + 522]
    out = torch.zeros((1000, 1024), device=gpu)[:, 6:6 + 522]
    m(x, out=out, kernel="tile-lds-exact")
    ref = oracle_mod.mix_exact_c(full.numpy(), g["row_ptr"], g["col"], g["val"], cols=(2, 524))
    assert oracle_mod.bitwise_equal(out.cpu().numpy(), ref[:, 2:524])


def test_auto_kernel_choice(gpu):
    g = load_golden("dcliques1000_fc_p64")
    m = _mixer(g, gpu)
    assert m.kernel_for("fast") == "clique"
    assert m.kernel_for("exact") == "tile-lds-exact"
    g = load_golden("fc64_p33")
    assert _mixer(g, gpu).kernel_for("fast") == "clique"      # MH fully-connected = one clique
    ops = _ops()
    rng = np.random.default_rng(0)
    n = 128
    w = rng.random((n, n)).astype(np.float32)
    w /= w.sum(0, keepdims=True)                               # dense, column-stochastic, no structure
    csr = ops.csr_from_numpy(np.arange(0, n * n + 1, n),
                             np.concatenate([[i] + [j for j in range(n) if j != i] for i in range(n)]),
                             np.concatenate([[w[i, i]] + [w[j, i] for j in range(n) if j != i]
                                             for i in range(n)]))
    assert ops.Mixer(csr=csr, device=gpu).kernel_for("fast") == "dense"
    g = load_golden("ring100_p257")
    assert _mixer(g, gpu).kernel_for("fast") == "ell-fast"
    assert _mixer(g, gpu).kernel_for("exact") == "ell-exact"   # degree 2: no tile plan, ELL rows


def _dcliques_full(gpu, p, seed=0):
    g = load_golden("dcliques1000_fc_p64")
    m = _mixer(g, gpu)
    gen = torch.Generator(device=gpu).manual_seed(seed)
    x = torch.randn(m.n, p, device=gpu, generator=gen)
    return g, m, x


def _windows(p, w=2048):
    return [(0, w), (p // 2 - w // 2, p // 2 + w // 2), (p - w, p)]


@pytest.mark.parametrize("kernel", ["csr-exact", "tile-exact", "tile-lds-exact"])
def test_full_size_exact_windows(kernel, gpu, oracle_mod):
    """BASELINE configs[2] at full size (N=1000 d-cliques, P=2^20): exact kernels are bit-identical
    to the oracle on sampled column windows (columns are independent)."""
    p = 1 << 20
    g, m, x = _dcliques_full(gpu, p)
    y = m(x, kernel=kernel)
    for c0, c1 in _windows(p):
        xw = x[:, c0:c1].cpu().numpy()
        ref = oracle_mod.mix_exact_c(xw, g["row_ptr"], g["col"], g["val"])
        assert oracle_mod.bitwise_equal(y[:, c0:c1].cpu().numpy(), ref), (c0, c1)


def test_full_size_clique_windows_and_checksum(gpu, oracle_mod):
    """Headline kernel at full size on row-major slabs: EVERY element against the exact kernel's
    round of the same input (1e-5 condition-aware, tests/fullcheck.py), 32 random 1024-column
    windows plus the first and last against the oracle, and column sums over ALL columns (W is
    doubly stochastic) as an extra check."""
    from fullcheck import check_rowmajor_every_element
    p = 1 << 20
    g, m, x = _dcliques_full(gpu, p, seed=1)
    y = m(x, kernel="clique")
    check_rowmajor_every_element(m, x, y, oracle_mod, seed=21)
    cs_x = x.double().sum(0)
    cs_y = y.double().sum(0)
    # column sums agree to fp32 accumulation accuracy of ~1000 terms of O(1)
    assert torch.max(torch.abs(cs_x - cs_y)).item() < 1e-3


def test_rounds_converge_to_mean(gpu):
    """Repeated mixing (ping-pong slabs) converges every node to the global average: the
    consensus property D-SGD relies on, checked for the exact and the clique kernel."""
    g = load_golden("dcliques300_fc_p37")
    m = _mixer(g, gpu)
    x0 = torch.randn(m.n, 64, device=gpu)
    mean = x0.double().mean(0)
    for kernel in ["csr-exact", "clique"]:
        a, b = x0.clone(), torch.empty_like(x0)
        for _ in range(1000):
            m(a, out=b, kernel=kernel)
            a, b = b, a
        assert torch.max(torch.abs(a.double() - mean)).item() < 1e-4


def test_strided_slab_and_odd_p(gpu, oracle_mod):
    """ld > p (a column window of a wider slab) and p % 4 != 0 take the scalar path."""
    g = load_golden("ring100_p257")
    m = _mixer(g, gpu)
    big = torch.zeros(100, 300, device=gpu)
    big[:, 10:267] = torch.from_numpy(g["x"]).to(gpu)
    xv = big[:, 10:267]
    outbig = torch.full((100, 300), 7.0, device=gpu)
    out = outbig[:, 20:277]
    m(xv, out=out, mode="exact")
    assert oracle_mod.bitwise_equal(out.cpu().numpy(), g["y"])
    assert torch.all(outbig[:, :20] == 7.0) and torch.all(outbig[:, 277:] == 7.0)


def test_errors(gpu):
    ops = _ops()
    g = load_golden("ring100_p257")
    m = _mixer(g, gpu)
    x = torch.from_numpy(g["x"]).to(gpu)
    with pytest.raises(RuntimeError, match="overlap"):
        m(x, out=x, mode="exact")
    with pytest.raises(RuntimeError, match="HIP"):
        m(x.cpu(), mode="exact")
    with pytest.raises(RuntimeError, match="float32"):
        m(x.double(), mode="exact")
    with pytest.raises(RuntimeError):
        ops.mix_csr(x, m.row_ptr[:-1], m.col, m.val, torch.empty_like(x), 0)


def test_mean_rows_and_distance(gpu, oracle_mod):
    ops = _ops()
    d = np.load(__import__("conftest").GOLDEN + "/uniform_avg_k7_p100.npz")
    x = torch.from_numpy(d["x"]).to(gpu)
    mean = torch.empty(x.shape[1], device=gpu)
    dist2 = torch.empty(x.shape[0], device=gpu, dtype=torch.float64)
    ops.mean_rows(x, mean, dist2, ops.EXACT)
    assert oracle_mod.bitwise_equal(mean.cpu().numpy(), d["y"][0])
    ref = ((d["x"].astype(np.float64) - d["y"][0].astype(np.float64)) ** 2).sum(1)
    np.testing.assert_allclose(dist2.cpu().numpy(), ref, rtol=1e-12)
    big = torch.randn(1000, 100003, device=gpu)
    mean = torch.empty(big.shape[1], device=gpu)
    ops.mean_rows(big, mean, torch.empty(0, device=gpu, dtype=torch.float64), ops.EXACT)
    ref = oracle_mod.mean_rows_c(big[:, :4096].cpu().numpy())
    assert oracle_mod.bitwise_equal(mean[:4096].cpu().numpy(), ref)


@pytest.mark.parametrize("kernel", ["dense", "dense-f32", "clique"])
def test_fc1000_dense_and_factored(kernel, gpu, oracle_mod):
    """configs[3] shape (fully-connected N=1000, MH weights) at reduced P: the MFMA GEMM and the
    big-clique factored kernel (two-pass) both within the tolerance of the oracle."""
    from niidmix.topology import mh_csr
    n = 1000
    edges = {i: [j for j in range(n) if j != i] for i in range(n)}
    csr = mh_csr(n, edges)
    ops = _ops()
    m = ops.Mixer(csr=csr, device=gpu)
    assert m.plan is not None and m.plan.max_clique == 1000
    x = torch.randn(n, 4096 + 12, device=gpu)
    y = m(x, kernel=kernel).cpu().numpy()
    xn = x.cpu().numpy()
    ref = oracle_mod.mix_exact_c(xn, csr.row_ptr, csr.col, csr.val)
    bound = oracle_mod.condition_bound(xn, csr.row_ptr, csr.col, csr.val)
    ok, worst = oracle_mod.check_tolerance(y, ref, bound, rtol=RTOL)
    assert ok, worst


def test_dense_kstep_variants_agree(gpu, oracle_mod, monkeypatch):
    """The dense MFMA kernel's K-step / occupancy variants (16 shipped; 32 = round 3; 8 and four
    waves per SIMD: tuning switches) accumulate k in the same order, so on finite inputs their
    outputs are bitwise equal, and within the tolerance of the oracle; ragged M, K and P tiles
    (N = 1000, P = 4096 + 12), interior tiles through the unchecked fetch."""
    from niidmix.topology import mh_csr
    n = 1000
    edges = {i: [j for j in range(n) if j != i] for i in range(n)}
    csr = mh_csr(n, edges)
    ops = _ops()
    m = ops.Mixer(csr=csr, device=gpu)
    x = torch.randn(n, 4096 + 12, device=gpu)
    outs = {}
    for bk, occ in (("16", "3"), ("32", "0"), ("8", "3"), ("8", "4"), ("16", "4")):
        monkeypatch.setenv("NIIDMIX_DENSE_BK", bk)
        monkeypatch.setenv("NIIDMIX_DENSE_OCC", occ)
        outs[(bk, occ)] = m(x, kernel="dense-f32").cpu().numpy()
    base = outs[("16", "3")]
    for k, y in outs.items():
        assert oracle_mod.bitwise_equal(y, base), k
    xn = x.cpu().numpy()
    ref = oracle_mod.mix_exact_c(xn, csr.row_ptr, csr.col, csr.val)
    bound = oracle_mod.condition_bound(xn, csr.row_ptr, csr.col, csr.val)
    ok, worst = oracle_mod.check_tolerance(base, ref, bound, rtol=RTOL)
    assert ok, worst


@pytest.mark.gpu
def test_stream_copy(gpu):
    """The bench's copy-ceiling primitive copies exactly (ragged tail of the last block included)."""
    import ctypes
    from niidmix import _lib
    for n in (4, 1020, 1 << 20, (1 << 20) + 36):
        a = torch.randn(n, device=gpu)
        b = torch.zeros(n, device=gpu)
        s = ctypes.c_void_p(torch.cuda.current_stream(gpu).cuda_stream)
        _lib.check(_lib.lib.niidmix_stream_copy_f32(a.data_ptr(), b.data_ptr(), n, s))
        torch.cuda.synchronize()
        assert torch.equal(a, b)


@pytest.mark.parametrize("n", [3000, 10000])
def test_clique_many_gateways(n, gpu, oracle_mod):
    """Fully-connected interclique over many cliques: 29 / 99 gateway (residual) entries per
    clique, i.e. the 128-entry descriptor path at 10 000 nodes; row-major and blocked slabs."""
    from niidmix import memory, ops
    from niidmix.generate import dcliques_csr
    csr, cliques = dcliques_csr(n, 100, "fully-connected", 1337)
    m = ops.Mixer(csr=csr, cliques=cliques, device=gpu)
    assert m.plan is not None, m.plan_reason
    gen = torch.Generator().manual_seed(n)
    xh = torch.randn(n, 256, generator=gen)
    x = xh.to(gpu)
    y = m(x, kernel="clique").cpu().numpy()
    ref = oracle_mod.mix_exact_c(xh.numpy(), csr.row_ptr, csr.col, csr.val)
    bound = oracle_mod.condition_bound(xh.numpy(), csr.row_ptr, csr.col, csr.val)
    ok, worst = oracle_mod.check_tolerance(y, ref, bound, rtol=RTOL)
    assert ok, worst
    yb = memory.empty_blocked(n, 256, gpu)
    m.mix_blocked(memory.to_blocked(x), yb, 256)
    assert np.array_equal(memory.from_blocked(yb, 256).cpu().numpy(), y)


@pytest.mark.parametrize("n,size,inter,p", [(1200, 600, "ring", 4096 + 20), (900, 300, "fully-connected", 999),
                                            (1000, 1000, "ring", 33), (2000, 500, "smallworld", 250)])
def test_bigclique_one_pass(n, size, inter, p, gpu, oracle_mod, monkeypatch):
    """Big cliques (> 256 members): the one-pass register-resident kernel (k_mix_bigclique_reg,
    R = 16 and 32, one or more degree groups, gateway residual terms, ragged column tails) within
    the tolerance of the oracle, and equal to the two-pass kernel (NIIDMIX_BIG=8x16) up to the
    summation order."""
    from niidmix import ops
    from niidmix.generate import dcliques_csr
    csr, cliques = dcliques_csr(n, size, inter, 1337)
    m = ops.Mixer(csr=csr, cliques=cliques, device=gpu)
    assert m.plan is not None and m.plan.max_clique > 256, m.plan_reason
    gen = torch.Generator().manual_seed(p)
    xh = torch.randn(n, p, generator=gen)
    x = xh.to(gpu)
    monkeypatch.delenv("NIIDMIX_BIG", raising=False)
    y = m(x, kernel="clique").cpu().numpy()
    ref = oracle_mod.mix_exact_c(xh.numpy(), csr.row_ptr, csr.col, csr.val)
    bound = oracle_mod.condition_bound(xh.numpy(), csr.row_ptr, csr.col, csr.val)
    ok, worst = oracle_mod.check_tolerance(y, ref, bound, rtol=RTOL)
    assert ok, worst
    monkeypatch.setenv("NIIDMIX_BIG", "8x16")
    y2 = m(x, kernel="clique").cpu().numpy()
    ok, worst = oracle_mod.check_tolerance(y2, ref, bound, rtol=RTOL)
    assert ok, worst
    assert np.max(np.abs(y - y2)) <= 1e-5 * np.max(bound)


@pytest.mark.parametrize("n,size,inter", [(1000, 1000, "ring"), (1200, 600, "ring"), (2000, 500, "smallworld")])
def test_bigclique_blocked_layout(n, size, inter, gpu, oracle_mod, monkeypatch):
    """The one-pass big-clique kernel on column-blocked slabs [P/B, N, B] (B = 256 and 1024, a
    ragged last block): with 4-B lanes (NIIDMIX_BIGREG_V4=0) bit-identical to the same kernel on
    the row-major slab; with float4 lanes (k_mix_bigclique_v4, the default for one-group cliques
    on blocked slabs; =1 forces it for every group count) within the 1e-5 condition-aware
    tolerance of the oracle -- its column sums add in another order."""
    from niidmix import memory, ops
    from niidmix.generate import dcliques_csr
    csr, cliques = dcliques_csr(n, size, inter, 1337)
    m = ops.Mixer(csr=csr, cliques=cliques, device=gpu)
    assert m.plan is not None and m.plan.max_clique > 256, m.plan_reason
    for p, bc in ((1500, 256), (2048 + 96, 1024)):
        gen = torch.Generator().manual_seed(p)
        x = torch.randn(n, p, generator=gen).to(gpu)
        y = m(x, kernel="clique")
        xb = memory.to_blocked(x, bc)
        yb = memory.empty_blocked(n, p, gpu, bc)
        monkeypatch.setenv("NIIDMIX_BIGREG_V4", "0")
        m.mix_blocked(xb, yb, p)
        assert torch.equal(memory.from_blocked(yb, p), y)
        monkeypatch.setenv("NIIDMIX_BIGREG_V4", "1")
        yb.fill_(float("nan"))
        m.mix_blocked(xb, yb, p)
        y4 = memory.from_blocked(yb, p).cpu().numpy()
        xn = x.cpu().numpy()
        ref = oracle_mod.mix_exact_c(xn, csr.row_ptr, csr.col, csr.val)
        bound = oracle_mod.condition_bound(xn, csr.row_ptr, csr.col, csr.val)
        ok, worst = oracle_mod.check_tolerance(y4, ref, bound, rtol=RTOL)
        assert ok, (n, inter, p, worst)
    monkeypatch.delenv("NIIDMIX_BIGREG_V4")
    # partly overlapping blocked slabs in one allocation are refused (Jacobi, d_sgd.py:99-116)
    k, rows, b = yb.shape
    flat = torch.zeros(2 * k * rows * b, device=gpu)
    xo = flat[: k * rows * b].view(k, rows, b)
    oo = flat[k * rows * b // 2: k * rows * b // 2 + k * rows * b].view(k, rows, b)
    with pytest.raises(RuntimeError, match="overlap"):
        m.mix_blocked(xo, oo, p)


@pytest.mark.parametrize("tile", ["8x13x4x13", "16x7x8x2", "16x7x4x7", "16x7x4x7x8", "16x7x8x2x8"])
@pytest.mark.parametrize("name", golden_cases())
def test_multi_clique_tile_vs_golden(name, tile, gpu, oracle_mod, monkeypatch):
    """The multi-clique tile (k_mix_clique_q: 4 cliques x 64 columns per item, the default for
    >= 4096 member rows) forced on every golden clique case, non-finite fixtures included: row-major
    slabs (64-bit row offsets) and column-blocked slabs of 64 and 256 columns (32-bit offsets),
    within the tolerance, with the reference's inf / NaN pattern; blocked == row-major bitwise."""
    from niidmix import memory
    g = load_golden(name)
    m = _mixer(g, gpu)
    p = g["x"].shape[1]
    if m.plan is None or p % 4:
        pytest.skip("no clique plan / p % 4")
    monkeypatch.setenv("NIIDMIX_CLIQUE_Q", "4")
    monkeypatch.setenv("NIIDMIX_CLIQUE_QT", tile)
    if m.plan.max_clique > 112 or int(tile.split("x")[0]) * int(tile.split("x")[1]) < m.plan.max_clique:
        pytest.skip("clique larger than the tile")
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="clique").cpu().numpy()
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=RTOL)
    assert ok, (name, tile, worst)
    for bc in (64, 256):
        yb = memory.empty_blocked(m.n, p, gpu, bc)
        m.mix_blocked(memory.to_blocked(x, bc), yb, p)
        assert oracle_mod.bitwise_equal(memory.from_blocked(yb, p).cpu().numpy(), y), (name, tile, bc)


@pytest.mark.parametrize("qm", ["8,4,4", "8,7,4,2", "16,4,4,2"])
@pytest.mark.parametrize("name", golden_cases())
def test_member_split_tile_vs_golden(name, qm, gpu, oracle_mod, monkeypatch):
    """The member-split multi-clique tile (round 6, NIIDMIX_CLIQUE_QM: one clique per item, the
    lane quarters split its members) forced on every golden clique case, non-finite fixtures
    included: row-major and column-blocked slabs within the tolerance with the reference's inf /
    NaN pattern, blocked == row-major bitwise."""
    from niidmix import memory
    g = load_golden(name)
    m = _mixer(g, gpu)
    p = g["x"].shape[1]
    if m.plan is None or p % 4:
        pytest.skip("no clique plan / p % 4")
    f = [int(v) for v in qm.split(",")]
    w, r, ms = f[0], f[1], (f[3] if len(f) > 3 else 4)
    if m.plan.max_clique > 112 or ms * w * r < m.plan.max_clique:
        pytest.skip("clique larger than the tile")
    monkeypatch.setenv("NIIDMIX_CLIQUE_Q", "4")
    monkeypatch.setenv("NIIDMIX_CLIQUE_QM", qm)
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="clique").cpu().numpy()
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=RTOL)
    assert ok, (name, qm, worst)
    for bc in (64, 256):
        yb = memory.empty_blocked(m.n, p, gpu, bc)
        m.mix_blocked(memory.to_blocked(x, bc), yb, p)
        assert oracle_mod.bitwise_equal(memory.from_blocked(yb, p).cpu().numpy(), y), (name, qm, bc)


@pytest.mark.parametrize("n,inter,size", [(4000, "fully-connected", 100), (5000, "smallworld", 100),
                                          (4200, "ring", 100), (4400, "smallworld", 110),
                                          (4480, "fully-connected", 112)])
def test_multi_clique_tile_auto(n, inter, size, gpu, oracle_mod, monkeypatch):
    """Many cliques (>= 4096 member rows): the launcher picks the multi-clique tile by itself; a
    ragged column tail (p = 4100) and a clique count not divisible by 4 (42 cliques of 100); equal
    within the tolerance to the one-clique tile (NIIDMIX_CLIQUE_Q=1) and to the oracle."""
    from niidmix import memory, ops
    from niidmix.generate import dcliques_csr
    csr, cliques = dcliques_csr(n, size, inter, 1337)
    m = ops.Mixer(csr=csr, cliques=cliques, device=gpu)
    assert m.plan is not None, m.plan_reason
    assert m.plan.max_clique == size       # 105-112 members: the 16x7 tile on 64-column blocks
    p = 4100
    xh = torch.randn(n, p, generator=torch.Generator().manual_seed(n))
    x = xh.to(gpu)
    monkeypatch.delenv("NIIDMIX_CLIQUE_Q", raising=False)
    monkeypatch.delenv("NIIDMIX_CLIQUE_QT", raising=False)
    y = m(x, kernel="clique").cpu().numpy()
    ref = oracle_mod.mix_exact_c(xh.numpy(), csr.row_ptr, csr.col, csr.val)
    bound = oracle_mod.condition_bound(xh.numpy(), csr.row_ptr, csr.col, csr.val)
    ok, worst = oracle_mod.check_tolerance(y, ref, bound, rtol=RTOL)
    assert ok, worst
    monkeypatch.setenv("NIIDMIX_CLIQUE_Q", "1")
    y1 = m(x, kernel="clique").cpu().numpy()
    ok, worst = oracle_mod.check_tolerance(y1, ref, bound, rtol=RTOL)
    assert ok, worst
    # the 8 x 13 multi-clique tile sums in another order than the one-clique 16 x 7 tile; for
    # 105-112 members both are 16 waves x 7 rows, so the group sums come out bit-identical
    assert not np.array_equal(y, y1) or n < 4096 or size > 104
    monkeypatch.delenv("NIIDMIX_CLIQUE_Q")
    perm, bc = m.device_layout()
    mr = m.relabeled(perm)
    pt = torch.from_numpy(perm).to(gpu)
    xp = torch.empty_like(x)
    xp[pt] = x
    yb = memory.empty_blocked(n, p, gpu, bc)
    mr.mix_blocked(memory.to_blocked(xp, bc), yb, p)
    ok, worst = oracle_mod.check_tolerance(memory.from_blocked(yb, p)[pt].cpu().numpy(), ref, bound,
                                           rtol=RTOL)
    assert ok, worst


@pytest.mark.parametrize("mode", ["exact", "fast"])
@pytest.mark.parametrize("name,p", [("ring100_p257", 62006), ("grid49_p20", 4099), ("n2_ring_linear7850", 7850),
                                    ("nonfinite_ring8_p16", 16), ("expander64_p48", 1001)])
def test_ell_kernel_sizes_and_widths(name, p, mode, gpu, oracle_mod, monkeypatch):
    """The ELL low-degree kernel at ragged sizes (float4 / float2 / scalar paths by p), every chunk
    count per wave (NIIDMIX_ELL_CH), bitwise the C oracle in exact mode (and the average-only flag),
    within the tolerance in fast mode; the golden fixture's own x in the first columns."""
    g = load_golden(name)
    m = _mixer(g, gpu)
    if m.ell is None:
        pytest.skip("a row has more than 8 entries")
    rng = np.random.default_rng(p)
    xh = rng.standard_normal((m.n, p)).astype(np.float32)
    k0 = min(p, g["x"].shape[1])
    xh[:, :k0] = g["x"][:, :k0]
    x = torch.from_numpy(xh).to(gpu)
    ref = oracle_mod.mix_exact_c(xh, g["row_ptr"], g["col"], g["val"])
    bound = oracle_mod.condition_bound(xh, g["row_ptr"], g["col"], g["val"])
    for ch in ("1", "2", "4"):
        monkeypatch.setenv("NIIDMIX_ELL_CH", ch)
        y = m(x, kernel="ell-" + mode).cpu().numpy()
        if mode == "exact":
            assert oracle_mod.bitwise_equal(y, ref), ch
        else:
            ok, worst = oracle_mod.check_tolerance(y, ref, bound, rtol=RTOL)
            assert ok, (ch, worst)
    if mode == "exact":
        ops = _ops()
        out = torch.empty_like(x)
        ops.mix_ell(x, m.e_col, m.e_val, m.e_len, out, m.ell, ops.EXACT | ops.AVERAGE_ONLY)
        ref = oracle_mod.mix_exact_c(xh, g["row_ptr"], g["col"], g["val"], average_only=True)
        assert oracle_mod.bitwise_equal(out.cpu().numpy(), ref)


def test_blocked_overlap_checks_use_each_block_stride(gpu):
    """Column-blocked slabs whose block strides differ: out's block 1 IS x's block 1 (x's blocks
    at 2R and 3R, out's at 0 and 3R).  The overlap checks measure each slab with its own block
    stride, so the mixing op and the blocked gradient mean both refuse it (Jacobi, d_sgd.py:99-116;
    the mean is out-of-place, d_sgd.py:19-45)."""
    from niidmix import ops
    g = load_golden("dcliques300_fc_p37")
    m = _mixer(g, gpu)
    rows, bc = 300, 1024
    r_ = rows * bc
    flat = torch.zeros(6 * r_, device=gpu)
    x = flat[2 * r_:4 * r_].view(2, rows, bc)
    out = torch.as_strided(flat, (2, rows, bc), (3 * r_, bc, 1))
    assert out[1].data_ptr() == x[1].data_ptr()
    with pytest.raises(RuntimeError, match="overlap"):
        m.mix_blocked(x, out, 2 * bc)
    seg_ptr = torch.tensor([0, 2], dtype=torch.int32, device=gpu)
    seg_row = torch.tensor([0, 1], dtype=torch.int32, device=gpu)
    with pytest.raises(RuntimeError, match="overlap"):
        ops.grad_segment_mean_blocked(x, seg_ptr, seg_row, out, 2 * bc)
    # disjoint slabs with different block strides are accepted
    out_ok = torch.as_strided(flat, (2, rows, bc), (r_, bc, 1))[:, :, :]
    out_ok = torch.zeros(3 * r_, device=gpu).as_strided((2, rows, bc), (int(1.5 * r_), bc, 1))
    m.mix_blocked(x, out_ok, 2 * bc)


@pytest.mark.parametrize("regs", [8, 16])
@pytest.mark.parametrize("mode", ["exact", "fast"])
@pytest.mark.parametrize("name", golden_cases("dcliques"))
def test_tile_lds_register_rows_vs_golden(name, mode, regs, gpu, oracle_mod, monkeypatch):
    """Plans whose out-of-group sources only masked entries read keep them in registers
    (NIIDMIX_TLDS_REMOTE: build_tile_lds_plan(remote_regs=True), the 10 000-node default):
    bitwise the reference in exact mode (non-finite fixtures included: inf / NaN in a gateway's
    neighbour reach the output only through the register row), within the tolerance in fast
    mode; the stage holds fewer rows than the all-staged plan.  regs: the kernel with 8 register
    rows per tile (a plan capped at 8, the rest staged) and with 16 (on the same plan)."""
    g = load_golden(name)
    if g["x"].shape[1] % 2:
        pytest.skip("odd p: the LDS tile kernel reads column pairs")
    monkeypatch.setenv("NIIDMIX_TLDS_REMOTE", "0")
    m0 = _mixer(g, gpu)
    if m0.tlds is None:
        pytest.skip(m0.tlds_reason)
    monkeypatch.setenv("NIIDMIX_TLDS_REMOTE", "8")
    m = _mixer(g, gpu)
    if m.tlds.rem_rows is None:
        pytest.skip("no source qualifies for a register row")
    assert m.tlds.max_src < m0.tlds.max_src and m.tmf is None
    assert m.tlds.rem_regs == 8 and not (m.tlds.rem_rows.reshape(-1, 16)[:, 8:] >= 0).any()
    m.tlds.rem_regs = regs              # 16: the 16-register kernel reads the plan's -1 entries
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="tile-lds-" + mode).cpu().numpy()
    if mode == "exact":
        assert oracle_mod.bitwise_equal(y, g["y"]), name
    else:
        bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
        ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=RTOL)
        assert ok, (name, worst)


@pytest.mark.parametrize("rows", ["auto", "13", "10", "9"])
@pytest.mark.parametrize("mode", ["exact", "fast"])
@pytest.mark.parametrize("name", golden_cases("dcliques"))
def test_tile_lds_tile_rows_vs_golden(name, mode, rows, gpu, oracle_mod, monkeypatch):
    """Shorter rt-16 tiles (NIIDMIX_TILE_LDS_ROWS; "auto" = tile.balanced_tile_rows, the default):
    more tiles -- waves -- per group, up to 12, with the register-row plans and the 9..15-row
    walker loops: bitwise the reference in exact mode, within the tolerance in fast mode."""
    g = load_golden(name)
    if g["x"].shape[1] % 2:
        pytest.skip("odd p: the LDS tile kernel reads column pairs")
    monkeypatch.setenv("NIIDMIX_TILE_LDS_ROWS", rows)
    m = _mixer(g, gpu)
    if m.tlds is None:
        pytest.skip(m.tlds_reason)
    if rows != "auto":
        assert int(np.max(m.tlds.tile.sub_rows.reshape(-1, 16) >= 0, axis=0).sum()) <= int(rows)
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="tile-lds-" + mode).cpu().numpy()
    if mode == "exact":
        assert oracle_mod.bitwise_equal(y, g["y"]), name
    else:
        bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
        ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=RTOL)
        assert ok, (name, worst)


@pytest.mark.parametrize("n,p", [(1000, 4096 + 12), (64, 33), (130, 257), (257, 1030), (17, 5)])
def test_dense_b6_split_gemm(n, p, gpu, oracle_mod):
    """The bf16x6 dense GEMM (kernel "dense": three-term bf16 splits, six products on
    v_mfma_f32_32x32x16_bf16) on a dense column-stochastic W with no structure, ragged M, K and P
    (partial 128-row and 256-column tiles, K not a multiple of 16, odd P): within the 1e-5
    condition-aware tolerance of the oracle, and no worse than 4x the fp32 MFMA kernel's worst
    relative error on the same inputs (the split keeps fp32-level accuracy)."""
    ops = _ops()
    rng = np.random.default_rng(n + p)
    w = rng.random((n, n)).astype(np.float32) + np.float32(0.01)
    w /= w.sum(0, keepdims=True)
    csr = ops.csr_from_numpy(*_dense_csr(w))
    m = ops.Mixer(csr=csr, device=gpu)
    x = torch.from_numpy(rng.standard_normal((n, p)).astype(np.float32) * 3).to(gpu)
    xn = x.cpu().numpy()
    ref = oracle_mod.mix_exact_c(xn, csr.row_ptr, csr.col, csr.val)
    bound = oracle_mod.condition_bound(xn, csr.row_ptr, csr.col, csr.val)
    worst = {}
    for k in ("dense", "dense-f32"):
        y = m(x, kernel=k).cpu().numpy()
        ok, worst[k] = oracle_mod.check_tolerance(y, ref, bound, rtol=RTOL)
        assert ok, (k, worst[k])
    assert worst["dense"] <= 4 * max(worst["dense-f32"], 1e-7), worst


FLT_MAX = float(np.finfo(np.float32).max)


def _extreme_case(case, n, p, rng):
    """(W, X) of one extreme-magnitude case for the bf16x6 GEMM (VERDICT r05 #1b)."""
    w = rng.random((n, n)).astype(np.float32) + np.float32(0.01)
    x = rng.standard_normal((n, p))
    if case == "column-scales":
        # columns at 2^k, k in {-126, -120, -100, -60, 60, 100, 120} (2^-126 x N(0,1): subnormals)
        ks = np.array([-126, -120, -100, -60, 60, 100, 120])
        x = x * np.exp2(ks[np.arange(p) % len(ks)])[None, :]
    elif case == "mixed-rows":
        # every column mixes rows at 2^-100 and 2^100
        x = x * np.where(np.arange(n) % 2 == 0, 2.0 ** -100, 2.0 ** 100)[:, None]
    elif case == "near-flt-max":
        # every other row within 2^-8 of FLT_MAX (random sign): its bf16 head may round to inf
        big = FLT_MAX * (1.0 - rng.random((n, p)) * 2.0 ** -8) * np.sign(x)
        x = np.where((np.arange(n) % 2 == 0)[:, None], big, x)
    elif case == "tiny-w":
        # W entries spread over 1e-30 .. 1
        w = w * np.power(10.0, -30.0 * rng.random((n, n))).astype(np.float32)
    elif case == "tiny-w-tiny-x":
        w = w * np.power(10.0, -30.0 * rng.random((n, n))).astype(np.float32)
        x = x * 2.0 ** -60
    w = w / w.sum(0, keepdims=True)
    return w.astype(np.float32), x.astype(np.float32)


@pytest.mark.parametrize("case", ["column-scales", "mixed-rows", "near-flt-max", "tiny-w",
                                  "tiny-w-tiny-x"])
@pytest.mark.parametrize("n,p", [(257, 300), (1000, 1030)])
def test_dense_b6_extreme_inputs(case, n, p, gpu, oracle_mod):
    """The auto-selected bf16x6 GEMM (Mixer.kernel_for('fast') == 'dense' for a dense W with no
    clique structure) on inputs whose split residues are not representable as assumed by the
    well-scaled argument (niidmix.hip, k_mix_dense_b6 header): columns from 2^-126 (subnormal) to
    2^120, columns mixing 2^+-100 rows, values within 2^-8 of FLT_MAX (bf16 head -> inf: the
    non-finite guard carries the element), W entries down to 1e-30 (with and without tiny X);
    ragged M, K (n % 16 != 0) and P tiles.  Within the 1e-5 condition-aware tolerance of the
    oracle (the reference's fp32 loop, d_sgd.py:96-116 / model/__init__.py:19-24), like the fp32
    MFMA kernel on the same inputs."""
    ops = _ops()
    rng = np.random.default_rng(sum(map(ord, case)) + n)
    w, xn = _extreme_case(case, n, p, rng)
    csr = ops.csr_from_numpy(*_dense_csr(w))
    m = ops.Mixer(csr=csr, device=gpu)
    assert m.kernel_for("fast") == "dense"
    x = torch.from_numpy(xn).to(gpu)
    with np.errstate(over="ignore", invalid="ignore"):
        ref = oracle_mod.mix_exact_c(xn, csr.row_ptr, csr.col, csr.val)
        bound = oracle_mod.condition_bound(xn, csr.row_ptr, csr.col, csr.val)
    worst = {}
    for k in ("dense", "dense-f32"):
        y = m(x, kernel=k).cpu().numpy()
        ok, worst[k] = oracle_mod.check_tolerance(y, ref, bound, rtol=RTOL)
        assert ok, (case, k, worst[k])


def test_dense_b6_tail_rows_not_read(gpu):
    """on the last K-step the bf16x6 GEMM loads 16 rows from k0; rows past n must read
    as zeros (buffer range check), never the memory after x.  x is the first n rows (n % 16 != 0)
    of a buffer whose tail rows are NaN: the output must be bitwise that of the same x followed by
    zero rows (a NaN read would send elements through the CSR recompute, whose bits differ)."""
    ops = _ops()
    rng = np.random.default_rng(5)
    for n, p in ((257, 300), (1000, 1030)):
        w = rng.random((n, n)).astype(np.float32) + np.float32(0.01)
        w /= w.sum(0, keepdims=True)
        m = ops.Mixer(csr=ops.csr_from_numpy(*_dense_csr(w)), device=gpu)
        kpad = -(-n // 16) * 16 + 16
        xv = torch.from_numpy(rng.standard_normal((n, p)).astype(np.float32)).to(gpu)
        bufs = {}
        for tail in ("zero", "nan"):
            buf = torch.full((kpad, p), 0.0 if tail == "zero" else float("nan"), device=gpu)
            buf[:n] = xv
            bufs[tail] = m(buf[:n], kernel="dense").cpu().numpy()
        a, b = bufs["zero"], bufs["nan"]
        assert not np.isnan(b).any()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32)), n


@pytest.mark.parametrize("variant", [("NIIDMIX_DENSE_B6_W1", "1"), ("NIIDMIX_DENSE_B6_DMA", "4,3"),
                                     ("NIIDMIX_DENSE_B6_DMA", "4,2"), ("NIIDMIX_DENSE_B6_DMA", "2,2"),
                                     ("NIIDMIX_DENSE_B6_DMA", "4,2,3"), ("NIIDMIX_DENSE_B6_DMA", "2,2,3")])
@pytest.mark.parametrize("n,p", [(1000, 4096 + 12), (64, 33), (257, 1030), (300, 70000)])
def test_dense_b6_variants_bitwise(n, p, variant, gpu, monkeypatch):
    """The bf16x6 kernel's variants run the same products in the same K order through the same
    MFMA per output element as the default (8 waves of 128 x 64, W through registers), so their
    outputs are bit-identical, non-finite guard included: one wave per SIMD (k_mix_dense_b6w, 4
    waves of 128 x 128) and the W tiles by LDS-DMA (k_mix_dense_b6d, round 6: 256 x 256 with a
    three- or two-deep W ring, and 256 x 128 blocks two per CU; X three K-steps ahead)."""
    ops = _ops()
    rng = np.random.default_rng(7 * n + p)
    w = rng.random((n, n)).astype(np.float32) + np.float32(0.01)
    w /= w.sum(0, keepdims=True)
    m = ops.Mixer(csr=ops.csr_from_numpy(*_dense_csr(w)), device=gpu)
    xn = rng.standard_normal((n, p)).astype(np.float32)
    xn[n // 2, p // 3] = np.inf                       # a non-finite input: its column is recomputed
    x = torch.from_numpy(xn).to(gpu)
    monkeypatch.delenv("NIIDMIX_DENSE_B6_W1", raising=False)
    monkeypatch.delenv("NIIDMIX_DENSE_B6_DMA", raising=False)
    base = m(x, kernel="dense").cpu().numpy()
    monkeypatch.setenv(*variant)
    got = m(x, kernel="dense").cpu().numpy()
    assert np.array_equal(base.view(np.uint32), got.view(np.uint32))
    xn2 = rng.standard_normal((n, p)).astype(np.float32) * 3
    ref = oracle_c_tol(xn2, m, gpu)
    assert ref


def oracle_c_tol(xn, m, gpu):
    """m's current dense kernel on xn within the 1e-5 condition-aware tolerance of the C oracle."""
    from oracle import oracle
    csr = m.csr
    y = m(torch.from_numpy(xn).to(gpu), kernel="dense").cpu().numpy()
    ref = oracle.mix_exact_c(xn, csr.row_ptr, csr.col, csr.val)
    bound = oracle.condition_bound(xn, csr.row_ptr, csr.col, csr.val)
    ok, worst = oracle.check_tolerance(y, ref, bound, rtol=RTOL)
    return ok


def _dense_csr(w):
    """CSR of W^T rows (self first) of a dense [N, N] W (every entry an edge)."""
    n = w.shape[0]
    row_ptr = np.arange(n + 1, dtype=np.int64) * n
    col = np.concatenate([[i] + [j for j in range(n) if j != i] for i in range(n)]).astype(np.int32)
    val = w[col, np.repeat(np.arange(n), n)].astype(np.float32)
    return row_ptr, col, val
