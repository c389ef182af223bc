"""Multi-GPU sharding logic on CPU: the clique-aligned partition, halo plan and RCCL-style exchange
(here over gloo, world size 2 and 4), with the oracle as each rank's local compute.  The sharded
round must equal the single-process round bit for bit (same operand order per row)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden
from niidmix.shard import ShardPlan, ShardedMixer, column_stripe, window_layout
from niidmix.topology import MixCSR


def _csr(g):
    return MixCSR(g["row_ptr"], g["col"], g["val"]).validate()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_plan_partition_and_halo(world, oracle_mod):
    g = load_golden("dcliques1000_fc_p64")
    csr = _csr(g)
    plan = ShardPlan(csr, g["cliques"], world)
    seen = np.concatenate(plan.nodes_of)
    assert sorted(seen.tolist()) == list(range(1000))
    for r in range(world):
        sh = plan.local(r)
        # whole cliques only
        assert sum(len(c) for c in sh.cliques) == sh.n_local
        # halo rows are exactly the remote sources the local rows read
        need = set()
        for gid in sh.nodes:
            need.update(int(c) for c in csr.col[csr.row_ptr[gid]:csr.row_ptr[gid + 1]]
                        if plan.owner[c] != r)
        assert set(sh.halo.tolist()) == need
        # local mixing over [local | halo] rows == global mixing of those rows, bit for bit
        x_in = g["x"][np.concatenate([sh.nodes, sh.halo]).astype(np.int64)]
        y = oracle_mod.mix_exact_c(x_in, sh.csr.row_ptr, sh.csr.col, sh.csr.val)
        assert oracle_mod.bitwise_equal(y, g["y"][sh.nodes])
        # what r sends to q is what q expects, in q's halo order
        for q, idx in sh.send.items():
            hq = plan.local(q)
            expect = hq.halo[hq.halo_owner == r]
            np.testing.assert_array_equal(sh.nodes[idx], expect)


def test_window_layout():
    assert window_layout(1 << 20, 8) == (8, 131072)
    k, w = window_layout(1000, 8)
    assert k * w >= 1000 and w % 256 == 0 and (k - 1) * w < 1000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, name, p, rounds, q, topo=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        if topo is None:
            g = load_golden(name)
        else:                                   # generated topology handed over by the parent
            g = dict(topo)
        csr = _csr(g)

        def compute(x2d, out2d, kernel=None, mode="exact"):
            sh = sm.shard
            out2d.copy_(torch.from_numpy(oracle.mix_exact_c(
                x2d.contiguous().numpy(), sh.csr.row_ptr, sh.csr.col, sh.csr.val)))

        sm = ShardedMixer(csr, g.get("cliques"), world, rank, "cpu", p, windows=3, compute=compute)
        x = sm.empty().zero_()
        gx = g["x"][:, :p]
        for k in range(sm.k):
            c0 = k * sm.w
            cw = min(sm.w, p - c0)
            x[k, :sm.n_local, :cw] = torch.from_numpy(gx[sm.shard.nodes, c0:c0 + cw])
        out = sm.empty().zero_()
        for _ in range(rounds):
            sm(x, out)
            x, out = out, x
        res = np.concatenate([x[k, :sm.n_local, :min(sm.w, p - k * sm.w)].numpy()
                              for k in range(sm.k)], axis=1)
        q.put((rank, sm.shard.nodes, res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name", [(2, "dcliques1000_fc_p64"), (2, "ring100_p257"),
                                        (4, "dcliques300_fc_p37")])
def test_gloo_sharded_rounds(world, name, oracle_mod):
    g = load_golden(name)
    p = min(g["x"].shape[1], 40)
    rounds = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, name, p, rounds, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    got = [q.get(timeout=240) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    ref = g["x"][:, :p].copy()
    for _ in range(rounds):
        ref = oracle_mod.mix_exact_c(ref, g["row_ptr"], g["col"], g["val"])
    full = np.zeros_like(ref)
    for rank, nodes, res in got:
        full[nodes] = res
    assert oracle_mod.bitwise_equal(full, ref)


@pytest.mark.parametrize("inter", ["fully-connected", "smallworld"])
def test_gloo_world8_dcliques10000(inter, oracle_mod):
    """BASELINE configs[4]'s problem: 10 000 d-cliques nodes (100 cliques of 100, the reference
    generator restated, seed 1337) over 8 node shards, halo rows exchanged over gloo (the same
    DistTransport code the RCCL path runs), 2 rounds: bitwise the single-process oracle rounds."""
    from niidmix.generate import dcliques_csr
    csr, cliques = dcliques_csr(10000, 100, inter, 1337)
    p, rounds, world = 12, 2, 8
    gen = np.random.default_rng(10000)
    x = gen.standard_normal((10000, p)).astype(np.float32)
    topo = {"row_ptr": csr.row_ptr, "col": csr.col, "val": csr.val, "cliques": cliques, "x": x}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, None, p, rounds, q, topo))
             for r in range(world)]
    for pr in procs:
        pr.start()
    got = [q.get(timeout=300) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    ref = x.copy()
    for _ in range(rounds):
        ref = oracle_mod.mix_exact_c(ref, csr.row_ptr, csr.col, csr.val)
    full = np.full_like(ref, np.nan)
    for rank, nodes, res in got:
        full[nodes] = res
    assert oracle_mod.bitwise_equal(full, ref)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
@pytest.mark.parametrize("p", [1, 1000, 1024, 4096 + 4, 1 << 20, 3 * 1024 + 512])
def test_column_stripes_partition(world, p):
    """Stripes tile [0, p) in rank order, start on block boundaries and are balanced to a block."""
    stripes = [column_stripe(p, world, r) for r in range(world)]
    assert stripes[0][0] == 0 and stripes[-1][1] == p
    for (a0, a1), (b0, b1) in zip(stripes, stripes[1:]):
        assert a1 == b0
    assert all((c0 % 1024 == 0 or c0 == p) and c0 <= c1 for c0, c1 in stripes)
    widths = [c1 - c0 for c0, c1 in stripes]
    assert max(widths) <= -(-p // world) + 1024        # block-granular balance
    with pytest.raises(ValueError):
        column_stripe(p, world, world)


def _stripe_worker(rank, world, port, name, p, rounds, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import oracle
        g = load_golden(name)
        c0, c1 = column_stripe(p, world, rank, align=16)
        x = np.ascontiguousarray(g["x"][:, c0:c1])
        for _ in range(rounds):             # no exchange: each stripe's rounds are independent
            x = oracle.mix_exact_c(x, g["row_ptr"], g["col"], g["val"])
        parts = [None] * world
        dist.all_gather_object(parts, (c0, c1, x))
        if rank == 0:
            q.put(parts)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,name", [(2, "dcliques1000_fc_p64"), (3, "ring100_p257")])
def test_gloo_striped_rounds(world, name, oracle_mod):
    """Column stripes over gloo: the gathered stripes of R rounds equal the single-process rounds
    bit for bit (the round is independent per parameter column)."""
    g = load_golden(name)
    p = g["x"].shape[1]
    rounds = 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_stripe_worker, args=(r, world, port, name, p, rounds, q))
             for r in range(world)]
    for pr in procs:
        pr.start()
    parts = q.get(timeout=240)
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    ref = g["x"].copy()
    for _ in range(rounds):
        ref = oracle_mod.mix_exact_c(ref, g["row_ptr"], g["col"], g["val"])
    got = np.concatenate([x for _, _, x in parts], axis=1)
    assert [c for c0, c1, _ in parts for c in (c0, c1)][0] == 0 and parts[-1][1] == p
    assert oracle_mod.bitwise_equal(got, ref)


@pytest.mark.parametrize("world", [2, 4])
def test_strip_kernel_never_chosen_for_halo_shards(world):
    """the column-strip kernel stages rows 0..n-1 only, so a node shard whose rows read
    halo rows (csr.n_in > n) must never auto-select it, even on a 64-float-multiple row stride;
    the unsharded ring on the same stride does take it (Mixer.kernel_for, host-side only)."""
    from niidmix.ops import Mixer
    csr = _csr(load_golden("ring100_p257"))
    whole = Mixer(csr=csr, device="cpu")
    assert whole.kernel_for("fast", torch.empty(csr.n, 512)) == "strip-fast"
    assert whole.kernel_for("exact", torch.empty(csr.n, 512)) == "strip-exact"
    plan = ShardPlan(csr, None, world)
    for r in range(world):
        sh = plan.local(r)
        assert sh.csr.n_in > sh.n_local
        m = Mixer(csr=sh.csr, device="cpu")
        x = torch.empty(sh.rows_in, 512)
        for mode in ("fast", "exact"):
            assert not m.kernel_for(mode, x).startswith("strip")
        with pytest.raises(RuntimeError, match="strip kernel"):
            m(x, out=torch.empty(sh.n_local, 512), kernel="strip-fast")
