"""bench.py's own timed loop (bench.timed_rounds: warm-up, barrier + synchronize, EXACTLY K timed
rounds, max over ranks) driving the node-shard partition (--shard nodes: ShardedMixer, halo rows
exchanged every round over torch.distributed point-to-point) in a 2-rank gloo world on the CPU,
with the oracle as each rank's local compute (checker only).  After warm-up + K rounds every rank's
rows equal the oracle applied W + K times, bit for bit, and the reported times are the same on
every rank (max-reduced)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import load_golden


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, q, steps, warmup):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from niidmix.shard import ShardedMixer
        from niidmix.topology import MixCSR
        from oracle import oracle
        g = load_golden("dcliques300_fc_p37")
        csr = MixCSR(g["row_ptr"], g["col"], g["val"]).validate()
        p = g["x"].shape[1]

        def compute(x2d, out2d, kernel=None, mode="exact"):
            sh = sm.shard
            out2d.copy_(torch.from_numpy(oracle.mix_exact_c(
                x2d.contiguous().numpy(), sh.csr.row_ptr, sh.csr.col, sh.csr.val)))

        sm = ShardedMixer(csr, g["cliques"], world, rank, "cpu", p, windows=2, compute=compute)
        xa, xb = sm.empty().zero_(), sm.empty().zero_()
        for k in range(sm.k):
            c0 = k * sm.w
            cw = min(sm.w, p - c0)
            xa[k, :sm.n_local, :cw] = torch.from_numpy(g["x"][sm.shard.nodes, c0:c0 + cw])

        def step(a, b, evs=None):                   # bench.main's multi-GPU step
            sm(a, b, kernel=None, mode="exact", events=evs)

        region_s, launch_ms, graph = bench.timed_rounds(step, xa, xb, steps, warmup,
                                                        torch.device("cpu"), dist, False, "gloo")
        last = xa if (steps + warmup) % 2 == 0 else xb
        res = np.concatenate([last[k, :sm.n_local, :min(sm.w, p - k * sm.w)].numpy()
                              for k in range(sm.k)], axis=1)
        q.put((rank, sm.shard.nodes, res, region_s, launch_ms, graph is None, sm.halo_rows))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("steps,warmup", [(3, 1), (2, 2)])
def test_bench_timed_rounds_node_shards_gloo(steps, warmup, oracle_mod):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, steps, warmup)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    g = load_golden("dcliques300_fc_p37")
    ref = g["x"]
    for _ in range(steps + warmup):
        ref = oracle_mod.mix_exact_c(ref, g["row_ptr"], g["col"], g["val"])
    times = set()
    for rank, nodes, res, region_s, launch_ms, no_graph, halo in out:
        assert oracle_mod.bitwise_equal(res, ref[nodes]), rank
        assert no_graph and region_s > 0 and launch_ms > 0 and halo > 0
        times.add((region_s, launch_ms))
    assert len(times) == 1                          # max-reduced over the ranks


# ------------------------------------------------------------------------------------------------
# bench.py's default N > 1 path: the stripes line, then one node-shard leg per interclique
# (bench.run_node_legs: LegWatchdog + guarded_leg + node_shard_leg), in a 2-rank gloo world on the
# CPU with the oracle as each rank's compute (checker only)
def _oracle_compute(sm_ref):
    from oracle import oracle

    def compute(x2d, out2d, kernel=None, mode="exact"):
        sh = sm_ref[0].shard
        out2d.copy_(torch.from_numpy(oracle.mix_exact_c(
            x2d.contiguous().numpy(), sh.csr.row_ptr, sh.csr.col, sh.csr.val)))
    return compute


class _Args:
    steps, warmup, seed, leg_timeout = 2, 1, 0, 120.0


def _legs_worker(rank, world, port, q, n, p):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        from niidmix.generate import dcliques_csr
        from niidmix.shard import ShardedMixer, column_stripe
        from oracle import oracle
        cpu = torch.device("cpu")
        topo = {ic: dcliques_csr(n, 100, ic, 1337) for ic in ("fully-connected", "smallworld")}
        x0 = np.random.default_rng(5).standard_normal((n, p)).astype(np.float32)

        # 1) the stripes leg: rank r mixes columns [c0, c1) of every node, no exchange
        csr, _ = topo["fully-connected"]
        c0, c1 = column_stripe(p, world, rank, align=8)
        xa = torch.from_numpy(np.ascontiguousarray(x0[:, c0:c1]))
        xb = torch.empty_like(xa)

        def stripe_step(a, b, evs=None):
            b.copy_(torch.from_numpy(oracle.mix_exact_c(a.numpy(), csr.row_ptr, csr.col, csr.val)))
        bench.timed_rounds(stripe_step, xa, xb, _Args.steps, _Args.warmup, cpu, dist, False, "gloo")
        stripe = (xa if (_Args.steps + _Args.warmup) % 2 == 0 else xb).numpy().copy()

        # 2) node-shard legs: every leg's rows bitwise the oracle, then the keys of the report
        finals = {}
        for ic, (csr_i, cl_i) in topo.items():
            ref = [None]

            def make(ic_, csr_i=csr_i, cl_i=cl_i, ref=ref):
                ref[0] = ShardedMixer(csr_i, cl_i, world, rank, "cpu", p, windows=2,
                                      compute=_oracle_compute(ref))
                return ref[0]

            def fill(sm, x):
                x.zero_()
                for k in range(sm.k):
                    cw = min(sm.w, p - k * sm.w)
                    x[k, :sm.n_local, :cw] = torch.from_numpy(x0[sm.shard.nodes, k * sm.w:k * sm.w + cw])
            info, last, sm = bench.node_shard_leg(make, ic, _Args.steps, _Args.warmup, cpu, dist,
                                                  "gloo", fill=fill, single_ms=1.0)
            rows = np.concatenate([last[k, :sm.n_local, :min(sm.w, p - k * sm.w)].numpy()
                                   for k in range(sm.k)], axis=1)
            finals[ic] = (sm.shard.nodes, rows, info)

        # 3) run_node_legs as main() calls it: one good leg, one leg whose mixer fails on every
        #    rank (error captured, reported by interclique), then guarded_leg with a failure on
        #    rank 1 only (no communication inside the leg)
        report = []

        def make2(ic):
            if ic == "smallworld":
                raise RuntimeError("injected failure")
            ref = [None]
            ref[0] = ShardedMixer(topo[ic][0], topo[ic][1], world, rank, "cpu", p, windows=2,
                                  compute=_oracle_compute(ref))
            return ref[0]
        bench.run_node_legs(make2, ["fully-connected", "smallworld"], _Args, world, rank, cpu,
                            dist, "gloo", None, False, report)

        def one_rank_fails():
            if rank == 1:
                raise ValueError("only rank 1")
            return {"ok": True}
        g_info, g_err = bench.guarded_leg(one_rank_fails, dist, world, rank)
        ident = bench.world_identity(cpu, dist, world, "gloo")
        q.put((rank, stripe, (c0, c1), finals, report, g_info, g_err, ident))
    finally:
        dist.destroy_process_group()


def test_bench_default_multi_gpu_path_gloo(oracle_mod):
    from niidmix.generate import dcliques_csr
    world, n, p = 2, 300, 20
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_legs_worker, args=(r, world, port, q, n, p)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = [q.get(timeout=300) for _ in range(world)]
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    x0 = np.random.default_rng(5).standard_normal((n, p)).astype(np.float32)
    rounds = _Args.steps + _Args.warmup
    refs = {}
    for ic in ("fully-connected", "smallworld"):
        csr, _ = dcliques_csr(n, 100, ic, 1337)
        ref = x0
        for _ in range(rounds):
            ref = oracle_mod.mix_exact_c(ref, csr.row_ptr, csr.col, csr.val)
        refs[ic] = ref
    covered = np.zeros(p, bool)
    for rank, stripe, (c0, c1), finals, report, g_info, g_err, ident in out:
        # the self-describing N>1 record: backend, world size, distinct devices all-gathered
        assert ident["backend"] == "gloo" and ident["world_size"] == world
        assert ident["distinct_devices"] == world and len(ident["devices"]) == world
        assert ident["rccl_version"] is None
        # stripes: bitwise the oracle's columns
        assert oracle_mod.bitwise_equal(stripe, refs["fully-connected"][:, c0:c1]), rank
        covered[c0:c1] = True
        for ic, (nodes, rows, info) in finals.items():
            assert oracle_mod.bitwise_equal(rows, refs[ic][nodes]), (rank, ic)
            for key in ("interclique", "ms_per_step", "value_GBs", "launch_ms", "windows",
                        "halo_rows_max", "halo_GB_recv_max", "halo_GB_send_max",
                        "weak_efficiency_vs_1gpu"):
                assert key in info, key
            assert info["interclique"] == ic and info["halo_rows_max"] > 0
            xg = info["xgmi"]                 # the exchange alone, per rank
            assert len(xg["recv_GBs_per_rank"]) == world and len(xg["ms_per_round"]) == world
            assert all(v is not None and v > 0 for v in xg["recv_GBs_per_rank"])
        assert [e["interclique"] for e in report] == ["fully-connected", "smallworld"]
        assert "error" not in report[0] and report[0]["ms_per_step"] > 0
        assert report[1]["error"].startswith("failed on rank(s) [0, 1]")
        assert "injected failure" in report[1]["error"]
        assert g_info is None and g_err.startswith("failed on rank(s) [1]")
        if rank == 1:
            assert "only rank 1" in g_err
    assert covered.all()
    # the max-reduced halo figures agree across ranks
    assert out[0][3]["smallworld"][2]["halo_rows_max"] == out[1][3]["smallworld"][2]["halo_rows_max"]


def test_leg_watchdog_fires_and_cancels():
    import time
    import bench
    fired, exits = [], []
    with bench.LegWatchdog(0.2, lambda: fired.append(1), exit_fn=exits.append):
        time.sleep(0.6)
    assert fired == [1] and exits == [0]
    fired2, exits2 = [], []
    with bench.LegWatchdog(5.0, lambda: fired2.append(1), exit_fn=exits2.append) as wd:
        pass
    time.sleep(0.1)
    assert not wd.fired and fired2 == [] and exits2 == []


def test_node_leg_intercliques():
    import bench
    assert bench.node_leg_intercliques("auto", "fully-connected") == ["fully-connected", "smallworld"]
    assert bench.node_leg_intercliques("auto", "smallworld") == ["smallworld"]
    assert bench.node_leg_intercliques("off", "fully-connected") == []
    assert bench.node_leg_intercliques("ring, smallworld", "x") == ["ring", "smallworld"]
    with pytest.raises(SystemExit):
        bench.node_leg_intercliques("mesh", "x")


@pytest.mark.gpu
def test_world_identity_on_the_gpu():
    """bench.world_identity on a real GPU (the N > 1 line's config.world): the device's UUID and
    PCI address, and the RCCL version torch links, are readable on this image."""
    import bench
    w = bench.world_identity(torch.device("cuda:0"), None, 1, "nccl")
    assert w["backend"] == "nccl" and w["world_size"] == 1 and w["distinct_devices"] == 1
    d = w["devices"][0]
    assert d["uuid"] and d["pci"] and d["name"]
    assert w["rccl_version"] and not str(w["rccl_version"]).startswith("unavailable"), w
