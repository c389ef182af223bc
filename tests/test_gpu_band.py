"""k_mix_band (banded rows: a ring in its cycle order) against the reference's own outputs and the
C oracle: bitwise in exact mode, within the condition-aware tolerance in fast mode, at the float4,
float2 and scalar paths, both row-group shapes, cyclic wrap on tiny rings, the average-only flag,
and ring 100 at P = 62 006 inside a hipGraph as bench.py times it."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu
RTOL = 1e-5


def _relabeled(csr, dev):
    from niidmix import ops
    m = ops.Mixer(csr=csr, device=dev)
    perm, _ = m.device_layout()
    if perm is None:                      # already banded as stored (a 3-ring)
        assert m.band == 1
        perm = np.arange(csr.n)
    mr = m.relabeled(perm)
    assert mr.band == 1
    return mr, perm


@pytest.mark.parametrize("name", ["ring100_p257", "nonfinite_ring8_p16"])
def test_band_vs_reference_golden(name, gpu, oracle_mod):
    """The reference's own round (golden y), rows in the ring's cycle order on the device."""
    from niidmix.topology import MixCSR
    g = load_golden(name)
    csr = MixCSR(g["row_ptr"], g["col"], g["val"]).validate()
    mr, perm = _relabeled(csr, gpu)
    pt = torch.from_numpy(perm).to(gpu)
    x = torch.from_numpy(g["x"]).to(gpu)
    xp = torch.empty_like(x)
    xp[pt] = x
    p = x.shape[1]
    if p % 2:                             # ring100_p257: an odd P takes the ELL kernel ...
        assert mr.kernel_for("exact", xp) == "ell-exact"
        assert oracle_mod.bitwise_equal(mr(xp, mode="exact")[pt].cpu().numpy(), g["y"])
        p -= 1                            # ... and its first 256 columns the band kernel
    xe = xp[:, :p].contiguous()
    # p = 256: rows on a 256-B pitch, where the strip kernel is the auto choice (few nodes); the
    # band kernel is called explicitly below
    assert mr.kernel_for("exact", xe) in ("band-exact", "strip-exact")
    assert mr.kernel_for("fast", xe) in ("band-fast", "strip-fast")
    y = mr(xe, kernel="band-exact")[pt].cpu().numpy()
    assert oracle_mod.bitwise_equal(y, g["y"][:, :p])
    yf = mr(xe, kernel="band-fast")[pt].cpu().numpy()
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])[:, :p]
    ok, worst = oracle_mod.check_tolerance(yf, g["y"][:, :p], bound, rtol=RTOL)
    assert ok, worst


def _ring(n, seed):
    from niidmix.topology import mh_csr
    rng = np.random.default_rng(seed)
    order = rng.permutation(n)
    edges = {}
    for i in range(n):
        a, b = int(order[(i - 1) % n]), int(order[(i + 1) % n])
        edges[int(order[i])] = [a, b] if rng.random() < 0.5 else [b, a]
    return mh_csr(n, edges)


@pytest.mark.parametrize("rc", ["1,1", "1,2", "1,4", "2,1", "2,2", "4,1", "4,4", "8,2"])
@pytest.mark.parametrize("n,p", [(3, 1000), (4, 4098), (5, 62006), (17, 1000), (100, 62006),
                                 (100, 4098), (257, 2048)])
def test_band_sizes(n, p, rc, gpu, oracle_mod, monkeypatch):
    from niidmix import ops
    monkeypatch.setenv("NIIDMIX_BAND_RC", rc)
    mr, _ = _relabeled(_ring(n, n + p), gpu)
    c = mr.csr
    assert mr.kernel_for("exact") == "band-exact"
    xh = np.random.default_rng(p).standard_normal((n, p)).astype(np.float32)
    xh[0, 0], xh[n - 1, 1] = np.inf, np.nan
    x = torch.from_numpy(xh).to(gpu)
    ref = oracle_mod.mix_exact_c(xh, c.row_ptr, c.col, c.val)
    assert oracle_mod.bitwise_equal(mr(x, kernel="band-exact").cpu().numpy(), ref)
    bound = oracle_mod.condition_bound(xh, c.row_ptr, c.col, c.val)
    ok, worst = oracle_mod.check_tolerance(mr(x, kernel="band-fast").cpu().numpy(), ref, bound,
                                           rtol=RTOL)
    assert ok, worst
    out = torch.empty_like(x)
    ops.mix_band(x, mr.e_col, mr.e_val, mr.e_len, out, mr.ell, mr.band, ops.EXACT | ops.AVERAGE_ONLY)
    ref = oracle_mod.mix_exact_c(xh, c.row_ptr, c.col, c.val, average_only=True)
    assert oracle_mod.bitwise_equal(out.cpu().numpy(), ref)


def test_band2_lattice(gpu, oracle_mod):
    """ELL width 5, band 2 (every node linked to +-1 and +-2, lists in shuffled order); an odd p
    (scalar rows) falls back to the ELL kernel."""
    from niidmix import ops
    from niidmix.topology import mh_csr
    n, p = 37, 3000
    rng = np.random.default_rng(1)
    edges = {i: [int(v) for v in rng.permutation([(i + 1) % n, (i - 1) % n, (i + 2) % n, (i - 2) % n])]
             for i in range(n)}
    csr = mh_csr(n, edges)
    m = ops.Mixer(csr=csr, device=gpu)
    assert m.band == 2 and m.kernel_for("exact") == "band-exact"
    xh = rng.standard_normal((n, p)).astype(np.float32)
    y = m(torch.from_numpy(xh).to(gpu), mode="exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y, oracle_mod.mix_exact_c(xh, csr.row_ptr, csr.col, csr.val))
    xo = torch.from_numpy(xh[:, :2999].copy()).to(gpu)
    assert m.kernel_for("exact", xo) == "ell-exact"
    y = m(xo, mode="exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y, oracle_mod.mix_exact_c(xh[:, :2999].copy(), csr.row_ptr,
                                                               csr.col, csr.val))


@pytest.mark.parametrize("mode", ["fast", "exact"])
def test_ring100_band_hipgraph(mode, gpu, oracle_mod):
    """bench.py --config ring100 as timed: cycle-order rows, P = 62 006 (float2 path), the rounds
    captured in ONE hipGraph (two ping-pong rounds per replay), each round checked against the
    oracle applied to its own GPU input."""
    from niidmix import memory
    from niidmix.topology import MixCSR
    g = load_golden("ring100_p257")
    mr, _ = _relabeled(MixCSR(g["row_ptr"], g["col"], g["val"]).validate(), gpu)
    c = mr.csr
    p = 62006
    kernel = mr.kernel_for(mode)
    assert kernel == "band-" + mode
    a = memory.empty_slab(100, p, gpu)
    a.normal_(generator=torch.Generator(device=gpu).manual_seed(2))
    b = memory.empty_slab(100, p, gpu)
    mr(a, out=b, kernel=kernel, mode=mode)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        mr(a, out=b, kernel=kernel, mode=mode)
        mr(b, out=a, kernel=kernel, mode=mode)
    for _ in range(2):
        x0 = a.cpu().numpy()
        graph.replay()
        torch.cuda.synchronize()
        y1, y2 = b.cpu().numpy(), a.cpu().numpy()
        for xin, yout in ((x0, y1), (y1, y2)):
            ref = oracle_mod.mix_exact_c(xin, c.row_ptr, c.col, c.val)
            if mode == "exact":
                assert oracle_mod.bitwise_equal(yout, ref)
            else:
                bound = oracle_mod.condition_bound(xin, c.row_ptr, c.col, c.val)
                ok, worst = oracle_mod.check_tolerance(yout, ref, bound, rtol=RTOL)
                assert ok, worst


@pytest.mark.parametrize("name", ["ring100_p257", "nonfinite_ring8_p16", "n2_ring_linear7850"])
def test_strip_vs_reference_golden(name, gpu, oracle_mod):
    """k_mix_strip (column strips staged in LDS, few nodes): the reference's own round, bitwise in
    exact mode (odd P too: a strip is 64 columns of every row, lanes past P store nothing), within
    the tolerance in fast mode; rank order (the strip kernel reads any row order)."""
    from niidmix import ops
    from niidmix.topology import MixCSR
    g = load_golden(name)
    csr = MixCSR(g["row_ptr"], g["col"], g["val"]).validate()
    m = ops.Mixer(csr=csr, device=gpu)
    if m.ell is None:
        pytest.skip("a row has more than 8 entries")
    x = torch.from_numpy(g["x"]).to(gpu)
    y = m(x, kernel="strip-exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(y, g["y"])
    yf = m(x, kernel="strip-fast").cpu().numpy()
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(yf, g["y"], bound, rtol=RTOL)
    assert ok, worst


@pytest.mark.parametrize("n,k,p", [(3, 3, 64), (17, 3, 1000), (100, 3, 62006), (256, 3, 130),
                                   (64, 5, 333), (200, 8, 129)])
def test_strip_sizes_vs_ell(n, k, p, gpu, oracle_mod):
    """Strip kernel bitwise the C oracle (exact) on rings and random low-degree graphs of 3-256
    nodes, ELL widths 3 / 5 / 8, P not a multiple of 64, a strided window of a wider slab, the
    average-only flag; and the explicit limit (257 rows) is refused."""
    from niidmix import ops
    from niidmix.topology import mh_csr
    rng = np.random.default_rng(n * 7 + k)
    if k == 3:
        edges = {i: [(i + 1) % n, (i - 1) % n] if n > 2 else [(i + 1) % n] for i in range(n)}
    else:
        edges = {}
        for i in range(n):
            nb = rng.choice([j for j in range(n) if j != i], size=k - 1, replace=False)
            edges[i] = [int(j) for j in nb]
        for i in list(edges):                     # symmetric graph, at most k - 1 neighbours kept
            for j in edges[i]:
                if i not in edges[j]:
                    edges[j].append(i)
        edges = {i: v[:k - 1] for i, v in edges.items()}
        for i in edges:                           # re-symmetrise after the cut
            edges[i] = [j for j in edges[i] if i in edges[j]]
    csr = mh_csr(n, edges)
    m = ops.Mixer(csr=csr, device=gpu)
    assert m.ell is not None and m.ell <= 8
    wide = torch.from_numpy(rng.standard_normal((n, p + 6)).astype(np.float32)).to(gpu)
    x = wide[:, 3:3 + p]                          # ld = p + 6
    y = m(x, kernel="strip-exact").cpu().numpy()
    ref = oracle_mod.mix_exact_c(wide.cpu().numpy(), csr.row_ptr, csr.col, csr.val, cols=(3, 3 + p))
    assert oracle_mod.bitwise_equal(y, ref[:, 3:3 + p])
    # contiguous rows (float4 lanes when p % 4 == 0: 256-column strips), and a 16-B row pitch
    yc = m(x.contiguous(), kernel="strip-exact").cpu().numpy()
    assert oracle_mod.bitwise_equal(yc, ref[:, 3:3 + p])
    ld = -(-p // 64) * 64
    xp = torch.empty((n, ld), device=gpu)
    xp[:, :p].copy_(x)
    outp = torch.full((n, ld), 5.0, device=gpu)
    m(xp[:, :p], out=outp[:, :p], kernel="strip-exact")
    assert oracle_mod.bitwise_equal(outp[:, :p].cpu().numpy(), ref[:, 3:3 + p])
    assert bool((outp[:, p:] == 5.0).all())
    out = torch.empty((n, p), device=gpu)
    ops.mix_strip(x.contiguous(), m.e_col, m.e_val, m.e_len, out, m.ell, ops.EXACT | ops.AVERAGE_ONLY)
    ref_avg = torch.empty_like(out)
    ops.mix_ell(x.contiguous(), m.e_col, m.e_val, m.e_len, ref_avg, m.ell, ops.EXACT | ops.AVERAGE_ONLY)
    assert torch.equal(out, ref_avg)
    if n == 256:
        with pytest.raises(RuntimeError, match="strip kernel"):
            big = torch.zeros((257, 64), device=gpu)
            ops.mix_strip(big, torch.zeros(257 * 3, dtype=torch.int32, device=gpu),
                          torch.zeros(257 * 3, device=gpu), torch.ones(257, dtype=torch.int32, device=gpu),
                          torch.empty_like(big), 3, ops.EXACT)


def test_strip_auto_on_row_pitch(gpu):
    """Ring 100 at P = 62 006 as bench.py allocates it (rows on a 256-B pitch): the Mixer picks the
    strip kernel (on ld = P it keeps ELL / band), bitwise the ELL kernel over two ping-pong rounds
    captured in a hipGraph, and the padding columns are never written."""
    from bench import golden
    from niidmix import ops
    csr, _ = golden("ring100_p257")
    m = ops.Mixer(csr=csr, device=gpu)
    n, p, ld = csr.n, 62006, 62016
    pa = torch.full((n, ld), 7.0, device=gpu)
    pb = torch.full((n, ld), 7.0, device=gpu)
    xa, xb = pa[:, :p], pb[:, :p]
    xa.normal_(generator=torch.Generator(device=gpu).manual_seed(3))
    assert m.kernel_for("exact", xa, xb) == "strip-exact" and m.kernel_for("fast", xa, xb) == "strip-fast"
    assert m.kernel_for("exact", xa.contiguous()) in ("ell-exact", "band-exact")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        m(xa, out=xb, mode="exact")
        m(xb, out=xa, mode="exact")
    x0 = xa.clone()
    g.replay()
    torch.cuda.synchronize()
    ref = m(m(x0.contiguous(), kernel="ell-exact"), kernel="ell-exact")
    assert torch.equal(xa, ref)
    assert bool((pa[:, p:] == 7.0).all()) and bool((pb[:, p:] == 7.0).all())


def test_strip_wave_and_lane_variants(gpu, monkeypatch):
    """The strip kernel's tuning switches (4 / 8 / 16 waves per strip, one-float lanes forced) give
    the shipped kernel's result bitwise, exact and fast, on ring 100 at P = 62 006 on a 256-B row
    pitch (float4 lanes by default)."""
    from bench import golden
    from niidmix import ops
    csr, _ = golden("ring100_p257")
    m = ops.Mixer(csr=csr, device=gpu)
    n, p, ld = csr.n, 62006, 62016
    xp = torch.empty((n, ld), device=gpu)
    x = xp[:, :p]
    x.normal_(generator=torch.Generator(device=gpu).manual_seed(5))
    for kname in ("strip-exact", "strip-fast"):
        base = m(x, kernel=kname)
        for sw, sv in (("4", "4"), ("16", "4"), ("8", "1"), ("4", "1")):
            monkeypatch.setenv("NIIDMIX_STRIP_SW", sw)
            monkeypatch.setenv("NIIDMIX_STRIP_SV", sv)
            assert torch.equal(m(x, kernel=kname), base), (kname, sw, sv)
        monkeypatch.delenv("NIIDMIX_STRIP_SW")
        monkeypatch.delenv("NIIDMIX_STRIP_SV")
    ref = m(x.contiguous(), kernel="ell-exact")
    assert torch.equal(m(x, kernel="strip-exact"), ref)
