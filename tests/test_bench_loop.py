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
