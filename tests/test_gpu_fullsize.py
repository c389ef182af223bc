"""Parity of the shipped paths at the sizes they actually run (BASELINE.json configs[1..3]), through
the same layouts and launch paths as bench.py and the drop-in:

  * headline (configs[2]): the column-blocked VMM slab [1024, 1000, 1024] (clique-contiguous rows)
    read directly by the clique kernel, checked block by block against the oracle (no row-major
    round trip);
  * fully-connected N=1000 (configs[3]): the one-pass big-clique kernel on [32768, 1000, 32] at
    P = 2^20;
  * ring N=100, P=62006 (configs[1]): the CSR kernel inside a hipGraph (bench.py's small-slab path),
    fast and exact, two ping-pong rounds per graph;
plus the non-finite guard on the blocked and two-pass layouts, and the consensus-distance event
against the reference Logger's own numbers (tests/golden/consensus_*.npz).

Columns of Θ' = Wᵀ Θ are independent (d_sgd.py:96-116 mixes every tensor element-wise), so any
column window of the oracle is the full computation restricted to those columns.
"""
import json

import numpy as np
import pytest
import torch

from conftest import GOLDEN, load_golden

pytestmark = pytest.mark.gpu
RTOL = 1e-5
P_FULL = 1 << 20


def _mixer(csr, cliques, dev):
    from niidmix import ops
    return ops.Mixer(csr=csr, cliques=cliques, device=dev)


def _golden_csr(name):
    from niidmix import ops
    g = load_golden(name)
    return g, ops.csr_from_numpy(g["row_ptr"], g["col"], g["val"])


def _check_block(oracle_mod, csr, xw, yw, what):
    ref = oracle_mod.mix_exact_c(xw, csr.row_ptr, csr.col, csr.val)
    bound = oracle_mod.condition_bound(xw, csr.row_ptr, csr.col, csr.val)
    ok, worst = oracle_mod.check_tolerance(yw, ref, bound, rtol=RTOL)
    assert ok, (what, worst)


def _blocked_colsums(xb):
    return torch.stack([xb[k].double().sum(0) for k in range(xb.shape[0])])


def test_headline_blocked_vmm_slab_direct(gpu, oracle_mod):
    """bench.py's headline round exactly as timed: the device layout Mixer.device_layout picks
    (clique-contiguous rows, VMM column-blocked slabs [1024, 1000, 1024]), mix_blocked
    (k_mix_clique<16,7,2,...>) on the relabeled operator, checked on EVERY element (all 1024
    blocks) against the exact kernel's round of the same input within the 1e-5 condition-aware
    tolerance (tests/fullcheck.py), on 32 randomly drawn blocks plus the first and last against the
    oracle (relabeled CSR: the same sums, stored at permuted rows; the exact kernel bitwise there);
    every block's column sums are preserved (W doubly stochastic) as an extra check."""
    from fullcheck import check_blocked_every_element
    from niidmix import memory
    g, csr = _golden_csr("dcliques1000_fc_p64")
    m = _mixer(csr, g["cliques"], gpu)
    perm, bc = m.device_layout()
    m = m.relabeled(perm)
    xb = memory.empty_blocked(1000, P_FULL, gpu, bc)
    assert tuple(xb.shape) == (1024, 1000, 1024)
    xb.normal_(generator=torch.Generator(device=gpu).manual_seed(0))
    yb = memory.empty_blocked(1000, P_FULL, gpu, bc)
    yb.fill_(float("nan"))                       # every output element must be written
    m.mix_blocked(xb, yb, P_FULL)
    torch.cuda.synchronize()
    worst = check_blocked_every_element(m, xb, yb, P_FULL, oracle_mod, seed=20)
    print("headline fast vs exact, every element: worst", worst)
    assert torch.max(torch.abs(_blocked_colsums(xb) - _blocked_colsums(yb))).item() < 1e-3


def test_fc1000_blocked_bigclique_fullsize(gpu, oracle_mod):
    """bench.py --config fc1000 exactly as timed: MH fully-connected N=1000 (one clique of 1000,
    W = a I + c 11^T), VMM column-blocked slabs, the one-pass register-resident big-clique kernel
    (k_mix_bigclique_reg) at P = 2^20; blocks 0, 600 and 1023 against the oracle."""
    from niidmix import memory
    from niidmix.topology import mh_csr
    n = 1000
    csr = mh_csr(n, {i: [j for j in range(n) if j != i] for i in range(n)})
    m = _mixer(csr, None, gpu)
    assert m.kernel_for("fast") == "clique" and m.plan.max_clique == 1000
    perm, bc = m.device_layout()
    assert perm is None and bc == 32                 # [32768, 1000, 32]: one 128 KB item per block
    xb = memory.empty_blocked(n, P_FULL, gpu, bc)
    xb.normal_(generator=torch.Generator(device=gpu).manual_seed(1))
    yb = memory.empty_blocked(n, P_FULL, gpu, bc)
    m.mix_blocked(xb, yb, P_FULL)
    torch.cuda.synchronize()
    for k in (0, 1, 17000, 32767):
        _check_block(oracle_mod, csr, xb[k].cpu().numpy(), yb[k].cpu().numpy(), k)
    assert torch.max(torch.abs(_blocked_colsums(xb) - _blocked_colsums(yb))).item() < 1e-3


@pytest.mark.parametrize("mode", ["fast", "exact"])
def test_ring100_p62006_timed_shape_hipgraph(mode, gpu, oracle_mod):
    """bench.py --config ring100 EXACTLY as it is timed (bench.py single-GPU branch): the golden
    ring's CSR relabeled into its cycle order (Mixer.device_layout -> band_layout), node state in
    VMM slabs on a 256-B row pitch (memory.empty_slab(100, 62016) viewed as [:, :62006]), the
    kernel Mixer.kernel_for picks on that slab -- k_mix_strip with float4 lanes and non-temporal
    LDS-DMA staging -- and two ping-pong rounds captured in ONE hipGraph.  Every round of two
    replays is checked against the C oracle on the relabeled CSR applied to that round's own GPU
    input: bitwise in exact mode, 1e-5 condition-aware in fast mode.  The 10 pitch-padding columns
    of both slabs carry a sentinel that must survive (the strip kernel never writes them)."""
    from niidmix import memory
    g, csr = _golden_csr("ring100_p257")
    m = _mixer(csr, None, gpu)
    perm, _ = m.device_layout()
    assert perm is not None                           # rank order is not banded: cycle order
    m = m.relabeled(perm)
    p, ld = 62006, 62016
    assert ld == -(-p // 64) * 64                     # bench.py's pitch rule for few-node graphs
    fa, fb = memory.empty_slab(100, ld, gpu), memory.empty_slab(100, ld, gpu)
    assert fa.stride(0) == ld and fb.stride(0) == ld
    fa.normal_(generator=torch.Generator(device=gpu).manual_seed(2))
    sentinel = -1234.5
    fa[:, p:] = sentinel
    fb.fill_(sentinel)
    a, b = fa[:, :p], fb[:, :p]
    kernel = m.kernel_for(mode, a, b)
    assert kernel == ("strip-fast" if mode == "fast" else "strip-exact")
    m(a, out=b, kernel=kernel, mode=mode)             # warm-up outside the capture
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        m(a, out=b, kernel=kernel, mode=mode)
        m(b, out=a, kernel=kernel, mode=mode)
    rp, col, val = m.csr.row_ptr, m.csr.col, m.csr.val
    for _ in range(2):
        x0 = a.cpu().numpy()
        graph.replay()
        torch.cuda.synchronize()
        y1, y2 = b.cpu().numpy(), a.cpu().numpy()
        for xin, yout in ((x0, y1), (y1, y2)):
            ref = oracle_mod.mix_exact_c(xin, rp, col, val)
            if mode == "exact":
                assert oracle_mod.bitwise_equal(yout, ref)
            else:
                bound = oracle_mod.condition_bound(xin, rp, col, val)
                ok, worst = oracle_mod.check_tolerance(yout, ref, bound, rtol=RTOL)
                assert ok, worst
    for f in (fa, fb):
        assert bool(torch.all(f[:, p:] == sentinel)), "pitch padding written"


@pytest.mark.parametrize("mode", ["fast", "exact"])
def test_ring100_p62006_rank_order_ell_fallback_hipgraph(mode, gpu, oracle_mod):
    """The ring-100 round on slabs the strip and band kernels do NOT take -- rank order, ld = P
    (rows at 216-B offsets) -- falls back to the ELL kernel (float2 path, 4 chunks per wave); two
    ping-pong rounds in ONE hipGraph, each checked against the oracle on that round's own GPU input
    (bitwise in exact mode).  (bench.py's timed ring100 shape: the test above.)"""
    g, csr = _golden_csr("ring100_p257")
    m = _mixer(csr, None, gpu)
    p = 62006
    kernel = m.kernel_for(mode)
    assert kernel == ("ell-fast" if mode == "fast" else "ell-exact")
    a = torch.randn(100, p, device=gpu, generator=torch.Generator(device=gpu).manual_seed(2))
    b = torch.empty_like(a)
    m(a, out=b, kernel=kernel, mode=mode)                   # warm-up outside the capture
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        m(a, out=b, kernel=kernel, mode=mode)
        m(b, out=a, kernel=kernel, mode=mode)
    for _ in range(2):
        x0 = a.cpu().numpy()
        graph.replay()
        torch.cuda.synchronize()
        y1, y2 = b.cpu().numpy(), a.cpu().numpy()
        for xin, yout in ((x0, y1), (y1, y2)):
            ref = oracle_mod.mix_exact_c(xin, csr.row_ptr, csr.col, csr.val)
            if mode == "exact":
                assert oracle_mod.bitwise_equal(yout, ref)
            else:
                bound = oracle_mod.condition_bound(xin, csr.row_ptr, csr.col, csr.val)
                ok, worst = oracle_mod.check_tolerance(yout, ref, bound, rtol=RTOL)
                assert ok, worst


@pytest.mark.parametrize("name", ["nonfinite_dcliques300_fc_p64", "nonfinite_fc300_p36",
                                  "nonfinite_dcliques200_fractal_rm5_p64"])
def test_nonfinite_blocked_layout(name, gpu, oracle_mod):
    """The non-finite guard on the device-resident layout: column-blocked slabs (block width 256)
    through the clique / one-pass big-clique kernels give the reference's inf / NaN pattern."""
    from niidmix import memory
    g, csr = _golden_csr(name)
    m = _mixer(csr, g.get("cliques"), gpu)
    assert m.plan is not None, m.plan_reason
    x = torch.from_numpy(g["x"]).to(gpu)
    p = x.shape[1]
    yb = memory.empty_blocked(m.n, p, gpu, 256)
    m.mix_blocked(memory.to_blocked(x, 256), yb, p)
    y = memory.from_blocked(yb, p).cpu().numpy()
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=RTOL)
    assert ok, worst


@pytest.mark.parametrize("kernel_env", ["reg", "8x16", "16x1"])
def test_nonfinite_bigclique_variants(kernel_env, gpu, oracle_mod, monkeypatch):
    """Complete graph N=300 with ±inf / NaN / overflowing sums: the one-pass kernel and the two-pass
    kernel (NIIDMIX_BIG=<waves>x<blocks per CU>) on row-major slabs, and the MFMA GEMM, all with the
    reference's non-finite pattern."""
    g, csr = _golden_csr("nonfinite_fc300_p36")
    m = _mixer(csr, None, gpu)
    monkeypatch.setenv("NIIDMIX_BIG", kernel_env)
    x = torch.from_numpy(g["x"]).to(gpu)
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    for kernel in ("clique", "dense"):
        y = m(x, kernel=kernel).cpu().numpy()
        ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=RTOL)
        assert ok, (kernel, worst)


def test_auto_avoids_cancelling_plans(gpu):
    """Removed clique edges: the factored plan exists but carries cancelling -c_g corrections, so
    the auto choice takes the LDS tiles (fast) instead; explicit kernel='clique' is still served."""
    g, csr = _golden_csr("dcliques200_fractal_rm5_p40")
    m = _mixer(csr, g["cliques"], gpu)
    assert m.plan is not None and m.plan.n_cancel > 0
    assert m.kernel_for("fast") == "tile-lds-fast"
    g, csr = _golden_csr("dcliques1000_fc_p64")
    assert _mixer(csr, g["cliques"], gpu).kernel_for("fast") == "clique"


@pytest.mark.parametrize("name", ["consensus_linear_n16", "consensus_n100_p4099"])
def test_consensus_event_vs_reference_logger(name, gpu):
    """niidmix.logger.consensus_distance_event against the event the reference's own
    Logger.log_consensus_distance wrote for the same models (tests/golden/make_golden.py
    --consensus).  The center is bit-identical (exact uniform average); distances are accumulated
    in fp64 here and in fp32 per tensor by the reference (logger.py:42-48), hence rtol 1e-5 on
    avg/max/min/norm and 1e-4 on std (a difference of nearly equal distances)."""
    from niidmix import logger as nl
    d = np.load(f"{GOLDEN}/{name}.npz")
    shapes = [tuple(s) for s in json.loads(str(d["shapes_json"]))]
    x = d["x"]
    nodes = []
    for r in range(x.shape[0]):
        mdl = torch.nn.Module()
        mdl.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(s)) for s in shapes])
        off = 0
        with torch.no_grad():
            for q in mdl.parameters():
                k = q.numel()
                q.copy_(torch.from_numpy(x[r, off:off + k].copy()).view_as(q))
                off += k
        nodes.append({"rank": r, "model": mdl})
    ev = nl.consensus_distance_event({"nodes": nodes, "step": 7})
    ref = json.loads(str(d["event_json"]))
    assert ev["type"] == ref["type"] and ev["step"] == ref["step"]
    got, want = ev["distance_to_center"]["global"], ref["distance_to_center"]["global"]
    for key in ("avg", "max", "min"):
        np.testing.assert_allclose(got[key], want[key], rtol=1e-5, err_msg=key)
    np.testing.assert_allclose(got["std"], want["std"], rtol=1e-4)
    np.testing.assert_allclose(ev["center"]["norm"], ref["center"]["norm"], rtol=1e-5)


@pytest.mark.parametrize("name", ["dcliques1000_fc_p64", "nonfinite_dcliques300_fc_p64"])
def test_device_layout_relabeled_bitwise(name, gpu, oracle_mod):
    """Mixer.device_layout (clique-contiguous rows, per-plan block width) + Mixer.relabeled: the
    round on the permuted, blocked slab is bitwise the rank-order round, row for row."""
    from niidmix import memory
    g, csr = _golden_csr(name)
    m = _mixer(csr, g["cliques"], gpu)
    perm, bc = m.device_layout()
    assert perm is not None and bc in (256, 1024)
    mr = m.relabeled(perm)
    p = 4096 + 256
    x = torch.randn(m.n, p, device=gpu, generator=torch.Generator(device=gpu).manual_seed(4))
    if "nonfinite" in name:
        x[:, :64] = torch.from_numpy(g["x"]).to(gpu)
    y = memory.empty_blocked(m.n, p, gpu)
    m.mix_blocked(memory.to_blocked(x), y, p)
    pt = torch.from_numpy(perm).to(gpu)
    xp = torch.empty_like(x)
    xp[pt] = x
    yp = memory.empty_blocked(m.n, p, gpu, bc)
    mr.mix_blocked(memory.to_blocked(xp, bc), yp, p)
    assert oracle_mod.bitwise_equal(memory.from_blocked(yp, p)[pt].cpu().numpy(),
                                    memory.from_blocked(y, p).cpu().numpy())   # NaN == NaN


def test_fc_block32_layout_bitwise(gpu):
    """Big cliques stream 32-column blocks ([P/32, N, 32]: an item is one contiguous 128 KB
    stretch); bitwise the 1024-column layout's result, ragged last block included."""
    from niidmix import memory
    from niidmix.topology import mh_csr
    n = 600
    csr = mh_csr(n, {i: [j for j in range(n) if j != i] for i in range(n)})
    m = _mixer(csr, None, gpu)
    perm, bc = m.device_layout()
    assert perm is None and bc == 32
    p = 3000 + 20
    x = torch.randn(n, p, device=gpu, generator=torch.Generator(device=gpu).manual_seed(5))
    y1 = memory.empty_blocked(n, p, gpu, 1024)
    m.mix_blocked(memory.to_blocked(x, 1024), y1, p)
    y2 = memory.empty_blocked(n, p, gpu, 32)
    m.mix_blocked(memory.to_blocked(x, 32), y2, p)
    assert torch.equal(memory.from_blocked(y1, p), memory.from_blocked(y2, p))


def test_fc1000_dense_mfma_fullsize_windows(gpu, oracle_mod):
    """configs[3] through the MFMA GEMM (bench.py --config fc1000 --kernel dense) at the P = 2^20 it
    is profiled at: column windows at the start, middle and end (the last 128-column tile) against
    the oracle within the tolerance, and column sums preserved over every column."""
    from niidmix import memory
    from niidmix.topology import mh_csr
    n = 1000
    csr = mh_csr(n, {i: [j for j in range(n) if j != i] for i in range(n)})
    m = _mixer(csr, None, gpu)
    x = memory.empty_slab(n, P_FULL, gpu)
    x.normal_(generator=torch.Generator(device=gpu).manual_seed(6))
    y = memory.empty_slab(n, P_FULL, gpu)
    m(x, out=y, kernel="dense")
    torch.cuda.synchronize()
    for c0 in (0, P_FULL // 2 - 64, P_FULL - 384):
        xw = x[:, c0:c0 + 384].cpu().numpy()
        _check_block(oracle_mod, csr, xw, y[:, c0:c0 + 384].cpu().numpy(), c0)
    gap = torch.max(torch.abs(torch.sum(x, 0, dtype=torch.float64) -
                              torch.sum(y, 0, dtype=torch.float64))).item()
    assert gap < 1e-3
