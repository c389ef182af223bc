"""Shard-local mixing on the GPU: each rank's kernels over [local | halo] rows (halo filled here as
the RCCL exchange would) reproduce the single-GPU round — bitwise for the exact kernel, within
tolerance for the clique kernel whose residual terms now read halo rows."""
import numpy as np
import pytest
import torch

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world", [2, 4, 8])
def test_shard_local_kernels(world, gpu, oracle_mod):
    from niidmix.generate import dcliques_csr
    from niidmix.ops import Mixer
    from niidmix.shard import ShardPlan
    csr, cliques = dcliques_csr(1000 * world // 2, 100, "fully-connected", 1337)
    p = 1024
    x = torch.randn(csr.n, p, device=gpu)
    plan = ShardPlan(csr, cliques, world)
    xn = x.cpu().numpy()
    for r in range(world):
        sh = plan.local(r)
        rows = torch.from_numpy(np.concatenate([sh.nodes, sh.halo]).astype(np.int64)).to(gpu)
        xin = x.index_select(0, rows)
        m = Mixer(csr=sh.csr, cliques=sh.cliques, device=gpu)
        assert m.plan is not None, m.plan_reason
        ref = oracle_mod.mix_exact_c(xin.cpu().numpy(), sh.csr.row_ptr, sh.csr.col, sh.csr.val)
        ye = m(xin, mode="exact").cpu().numpy()
        assert oracle_mod.bitwise_equal(ye, ref)
        yc = m(xin, kernel="clique").cpu().numpy()
        bound = oracle_mod.condition_bound(xin.cpu().numpy(), sh.csr.row_ptr, sh.csr.col, sh.csr.val)
        ok, worst = oracle_mod.check_tolerance(yc, ref, bound, rtol=1e-5)
        assert ok, worst


def test_sharded_mixer_world1_window_blocked(gpu, oracle_mod):
    """ShardedMixer's window-blocked round on one rank equals the plain round."""
    from niidmix.shard import ShardedMixer
    g = load_golden("dcliques1000_fc_p64")
    from niidmix.topology import MixCSR
    csr = MixCSR(g["row_ptr"], g["col"], g["val"]).validate()
    p = 3000
    sm = ShardedMixer(csr, g["cliques"], 1, 0, gpu, p, windows=3)
    x = sm.empty().normal_()
    y = sm.empty()
    sm(x, y, mode="exact", kernel="csr-exact")
    full = torch.cat([x[k, :, :min(sm.w, p - k * sm.w)] for k in range(sm.k)], dim=1)
    got = torch.cat([y[k, :sm.n_local, :min(sm.w, p - k * sm.w)] for k in range(sm.k)], dim=1)
    nodes = torch.from_numpy(sm.shard.nodes).to(gpu)
    # local order is clique-contiguous: map back to global ids
    glob = torch.empty_like(got)
    glob[nodes] = got
    xg = torch.empty_like(full)
    xg[nodes] = full
    ref = oracle_mod.mix_exact_c(xg.cpu().numpy(), g["row_ptr"], g["col"], g["val"])
    assert oracle_mod.bitwise_equal(glob.cpu().numpy(), ref)


@pytest.mark.parametrize("world,inter", [(4, "fully-connected"), (3, "smallworld")])
def test_sharded_rounds_loopback(world, inter, gpu, oracle_mod):
    """The whole multi-GPU round (windowed halo exchange on a comm stream, per-window waits,
    shard-local kernels) with the RCCL transport replaced by in-process copies: 3 rounds equal the
    single-GPU oracle bitwise (exact) / within tolerance (fast)."""
    from niidmix.generate import dcliques_csr
    from niidmix.shard import LoopbackTransport, ShardedMixer
    n = 300 * world
    csr, cliques = dcliques_csr(n, 100, inter, 1337)
    p = 2000
    for mode, kernel in (("exact", "csr-exact"), ("fast", "clique")):
        tr = LoopbackTransport()
        sms = [ShardedMixer(csr, cliques, world, r, gpu, p, windows=3, transport=tr)
               for r in range(world)]
        gen = torch.Generator(device=gpu).manual_seed(3)
        x0 = torch.randn(n, p, device=gpu, generator=gen)
        xs, ys = [], []
        for sm in sms:
            x = sm.empty().zero_()
            nodes = torch.from_numpy(sm.shard.nodes).to(gpu)
            for k in range(sm.k):
                cw = min(sm.w, p - k * sm.w)
                x[k, :sm.n_local, :cw] = x0.index_select(0, nodes)[:, k * sm.w:k * sm.w + cw]
            xs.append(x)
            ys.append(sm.empty())
        for _ in range(3):
            tr.inputs = {r: xs[r] for r in range(world)}
            for r, sm in enumerate(sms):
                sm(xs[r], ys[r], kernel=kernel, mode=mode)
            xs, ys = ys, xs
        torch.cuda.synchronize()
        full = torch.empty_like(x0)
        for r, sm in enumerate(sms):
            nodes = torch.from_numpy(sm.shard.nodes).to(gpu)
            full[nodes] = torch.cat([xs[r][k, :sm.n_local, :min(sm.w, p - k * sm.w)]
                                     for k in range(sm.k)], dim=1)
        ref = x0.cpu().numpy()
        for _ in range(3):
            ref = oracle_mod.mix_exact_c(ref, csr.row_ptr, csr.col, csr.val)
        got = full.cpu().numpy()
        if mode == "exact":
            assert oracle_mod.bitwise_equal(got, ref)
        else:
            assert np.max(np.abs(got - ref)) < 1e-5


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_ring_auto_kernel_loopback(world, gpu, oracle_mod):
    """A node shard of a low-degree graph (the golden ring 100) with kernel=None on 256-column
    windows (row stride a multiple of 64 floats, the strip kernel's pitch test passes): each rank's
    rows read halo rows past its own, so the auto choice must NOT be the strip kernel (it stages rows
    0..n_local-1 only); 3 rounds, exact and fast, against the single-GPU oracle."""
    from niidmix.ops import csr_from_numpy
    from niidmix.shard import LoopbackTransport, ShardedMixer
    g = load_golden("ring100_p257")
    csr = csr_from_numpy(g["row_ptr"], g["col"], g["val"])
    n, p = csr.n, 1536
    for mode in ("exact", "fast"):
        tr = LoopbackTransport()
        sms = [ShardedMixer(csr, None, world, r, gpu, p, windows=3, transport=tr)
               for r in range(world)]
        gen = torch.Generator(device=gpu).manual_seed(4)
        x0 = torch.randn(n, p, device=gpu, generator=gen)
        xs, ys = [], []
        for sm in sms:
            assert sm.shard.csr.n_in > sm.n_local            # every ring shard reads halo rows
            x = sm.empty().zero_()
            assert x[0].stride(0) % 64 == 0
            k_auto = sm.kernel_for(mode, x)
            assert not k_auto.startswith("strip"), k_auto
            nodes = torch.from_numpy(sm.shard.nodes).to(gpu)
            for k in range(sm.k):
                cw = min(sm.w, p - k * sm.w)
                x[k, :sm.n_local, :cw] = x0.index_select(0, nodes)[:, k * sm.w:k * sm.w + cw]
            xs.append(x)
            ys.append(sm.empty())
        for _ in range(3):
            tr.inputs = {r: xs[r] for r in range(world)}
            for r, sm in enumerate(sms):
                sm(xs[r], ys[r], kernel=None, mode=mode)
            xs, ys = ys, xs
        torch.cuda.synchronize()
        full = torch.empty_like(x0)
        for r, sm in enumerate(sms):
            nodes = torch.from_numpy(sm.shard.nodes).to(gpu)
            full[nodes] = torch.cat([xs[r][k, :sm.n_local, :min(sm.w, p - k * sm.w)]
                                     for k in range(sm.k)], dim=1)
        ref = x0.cpu().numpy()
        for _ in range(3):
            ref = oracle_mod.mix_exact_c(ref, csr.row_ptr, csr.col, csr.val)
        got = full.cpu().numpy()
        if mode == "exact":
            assert oracle_mod.bitwise_equal(got, ref)
        else:
            assert np.max(np.abs(got - ref)) < 1e-5


@pytest.mark.parametrize("world", [2, 8])
def test_striped_mixer_equals_single_gpu(world, gpu, oracle_mod):
    """Every rank's column stripe (blocked slab, clique kernel) is bitwise the single-GPU blocked
    round's columns; exact-mode stripes are bitwise the oracle."""
    from niidmix import memory
    from niidmix.generate import dcliques_csr
    from niidmix.ops import Mixer
    from niidmix.shard import StripedMixer
    csr, cliques = dcliques_csr(1000 * world // 2, 100, "fully-connected", 1337)
    p = world * 1024 + 512 if world == 2 else 7 * 1024 + 256
    x = torch.randn(csr.n, p, device=gpu, generator=torch.Generator(device=gpu).manual_seed(world))
    full = Mixer(csr=csr, cliques=cliques, device=gpu)
    yb = memory.empty_blocked(csr.n, p, gpu)
    full.mix_blocked(memory.to_blocked(x), yb, p)
    y_full = memory.from_blocked(yb, p)
    covered = 0
    for r in range(world):
        sm = StripedMixer(csr, cliques, world, r, gpu, p)
        if sm.p_local == 0:
            continue
        assert sm.blocked and sm.perm is not None      # clique-contiguous device rows
        xs = sm.to_layout(x[:, sm.c0:sm.c1].contiguous())
        ys = sm.empty()
        sm(xs, ys)
        assert torch.equal(sm.from_layout(ys), y_full[:, sm.c0:sm.c1]), r
        covered += sm.p_local
        if r == 0:
            se = StripedMixer(csr, cliques, world, r, gpu, p, mode="exact")
            assert not se.blocked
            xe = se.empty()
            xe.copy_(x[:, se.c0:se.c1])
            ye = se.empty()
            se(xe, ye)
            ref = oracle_mod.mix_exact_c(x[:, se.c0:se.c1].cpu().numpy(), csr.row_ptr, csr.col,
                                         csr.val)
            assert oracle_mod.bitwise_equal(ye.cpu().numpy(), ref)
    assert covered == p


def test_striped_mixer_bigclique_blocked(gpu):
    """Fully-connected topology (one clique of 600 > 256 members: the one-pass big-clique kernel on
    32-column blocks): every rank's blocked column stripe is bitwise the single-GPU blocked round's
    columns (stripes use the blocked layout up to the 1024-member limit)."""
    from niidmix import memory
    from niidmix.ops import Mixer
    from niidmix.shard import StripedMixer
    from niidmix.topology import mh_csr
    n, world, p = 600, 4, 4 * 2048 + 96
    csr = mh_csr(n, {i: [j for j in range(n) if j != i] for i in range(n)})
    x = torch.randn(n, p, device=gpu, generator=torch.Generator(device=gpu).manual_seed(5))
    full = Mixer(csr=csr, device=gpu)
    perm, bc = full.device_layout()
    assert bc == 32
    yb = memory.empty_blocked(n, p, gpu, bc)
    full.mix_blocked(memory.to_blocked(x, bc), yb, p)
    y_full = memory.from_blocked(yb, p)
    covered = 0
    for r in range(world):
        sm = StripedMixer(csr, None, world, r, gpu, p)
        if sm.p_local == 0:
            continue
        assert sm.blocked
        xs = sm.to_layout(x[:, sm.c0:sm.c1].contiguous())
        ys = sm.empty()
        sm(xs, ys)
        assert torch.equal(sm.from_layout(ys), y_full[:, sm.c0:sm.c1]), r
        covered += sm.p_local
    assert covered == p


@pytest.mark.parametrize("world", [1, 2, 3])
@pytest.mark.parametrize("p", [1000, 4096])
def test_local_sharded_round_c_abi(world, p, gpu, oracle_mod):
    """The C-ABI sharded round (niidmix_mix_sharded_f32 via niidmix.shard.LocalShardedRound):
    world 1 builds a real RCCL communicator (ncclCommInitAll over the one device, nothing to
    exchange); worlds 2 and 3 put every shard on this GPU, so the halo exchange runs as
    device-to-device copies (the same pack / exchange / per-shard CSR path as over RCCL).  Two
    exact rounds are bitwise the oracle applied twice; a fast round is within the tolerance."""
    from niidmix.shard import LocalShardedRound
    g = load_golden("dcliques1000_fc_p64")
    from niidmix.ops import csr_from_numpy
    csr = csr_from_numpy(g["row_ptr"], g["col"], g["val"])
    sr = LocalShardedRound(csr, g["cliques"], [gpu] * world, p)
    assert sr.loopback == (world > 1)
    if world > 1:
        assert all(len(h["peer"]) > 0 for h in sr.host)
    xh = torch.randn(1000, p, generator=torch.Generator().manual_seed(p + world))
    sr.scatter(xh.to(gpu))
    sr("exact")
    sr("exact")
    y = sr.gather().numpy()
    ref = xh.numpy()
    for _ in range(2):
        ref = oracle_mod.mix_exact_c(ref, g["row_ptr"], g["col"], g["val"])
    assert oracle_mod.bitwise_equal(y, ref)
    sr.scatter(xh.to(gpu))
    sr("fast")
    yf = sr.gather().numpy()
    r1 = oracle_mod.mix_exact_c(xh.numpy(), g["row_ptr"], g["col"], g["val"])
    bound = oracle_mod.condition_bound(xh.numpy(), g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(yf, r1, bound, rtol=1e-5)
    assert ok, worst


@pytest.mark.parametrize("world", [2, 4, 8])
def test_local_sharded_round_rccl_devices(world, gpu, oracle_mod):
    """The RCCL branch of niidmix_mix_sharded_f32: one shard per DISTINCT GPU (ncclCommInitAll
    over `world` devices, grouped ncclSend / ncclRecv of the halo rows), two exact rounds bitwise
    the oracle applied twice.  Needs `world` visible GPUs (skipped on the one-GPU pool boxes; the
    driver's 8-GPU node runs it)."""
    if torch.cuda.device_count() < world:
        pytest.skip(f"needs {world} GPUs, {torch.cuda.device_count()} visible")
    from niidmix.ops import csr_from_numpy
    from niidmix.shard import LocalShardedRound
    g = load_golden("dcliques1000_fc_p64")
    csr = csr_from_numpy(g["row_ptr"], g["col"], g["val"])
    devs = [torch.device("cuda", i) for i in range(world)]
    sr = LocalShardedRound(csr, g["cliques"], devs, 4096)
    assert not sr.loopback
    xh = torch.randn(1000, 4096, generator=torch.Generator().manual_seed(world))
    sr.scatter(xh.to(gpu))
    sr("exact")
    sr("exact")
    y = sr.gather().numpy()
    ref = xh.numpy()
    for _ in range(2):
        ref = oracle_mod.mix_exact_c(ref, g["row_ptr"], g["col"], g["val"])
    assert oracle_mod.bitwise_equal(y, ref)
