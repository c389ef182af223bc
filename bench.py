#!/usr/bin/env python
"""Benchmark: device-resident D-SGD neighbour mixing (one round = one step) on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config dcliques1000] [--kernel auto]
    torchrun --nproc-per-node N bench.py --gpus N ...      (N > 1, one process per GPU over RCCL)

Metric (BASELINE.json): "param-GB/s mixed (device-resident), 1000-node d-cliques, P=1M fp32"
  value = (nodes mixed by all ranks) * P * 4 B / (time per round)   [GB/s, higher is better]
A step is one full mixing round Θ' = Wᵀ Θ over every node (d_sgd.average, d_sgd.py:96-116), input
already resident in HBM, ping-pong slabs.  Timed with HIP events on the stream the kernels run on
(torch's current stream), K steps between a barrier + synchronize on both sides, max over ranks.

roofline: the dominant kernel's algorithmic bytes per launch (read Θ once + write Θ' once =
2*N*P*4; gathers of neighbour rows are NOT counted) / its average launch duration (HIP events
around every launch in the timed region), against the 8.0 TB/s HBM3E peak (MI355X_MICROARCH.md).
Dense W (fully-connected) is priced in FLOPs: kernel "dense" (bf16 splits) as 6 x 2*N^2*P bf16
FLOPs against the ~2.5 PF bf16 MFMA peak, kernel "dense-f32" as 2*N^2*P against the 157.3 TF fp32
MFMA peak.
traffic: HBM bytes per launch from rocprofv3 PMC counters (FETCH_SIZE x2 on gfx950 + WRITE_SIZE)
read from --traffic-json (tools/pmc_traffic.py, keyed by config.traffic_key), reported only when the
entry was measured with the library this run loaded (config.lib_sha16), else null.

cpu_baseline (rank 0, N=1): the reference loop restated faithfully in torch CPU
(oracle.reference_loop_average: per-node deepcopy / mul_(0) / add_(w*p), then update_models) timed
on this host's cores for one full round of the same topology at the same P.

Multi-GPU (N > 1), two problem sizes:
  default (--config dcliques1000): WEAK scaling over a d-cliques topology of 1000*N nodes (see
      --interclique), per-GPU bytes those of the N=1 headline round;
  --config dcliques10000: BASELINE configs[4], the FIXED 10 000-node problem (100 cliques of 100)
      split over N GPUs (STRONG scaling); rank 0 then also times the whole problem alone on its own
      GPU (--single-ref, default on) and reports speedup_vs_1gpu.
Two partitions:
  --shard stripes (default): rank r mixes parameter columns [c0, c1) of EVERY node (P/N columns
      each, block-aligned; the round is independent per column): no data-path collective
      (niidmix.shard.StripedMixer);
  --shard nodes: each rank owns whole cliques of nodes and the cross-shard edges' rows are
      exchanged over RCCL (xGMI) every round, pipelined over column windows with the mixing kernel
      (niidmix.shard.ShardedMixer); halo bytes per rank are reported.
"""
import argparse
import ctypes
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.join(REPO, "non-iid-topology-simulator_amd")
for _p in (REPO, PKG_ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "param-GB/s mixed (device-resident), 1000-node d-cliques, P=1M fp32"
GRAD_METRIC = "gradient-GB/s averaged (device-resident), 1000-node d-cliques --clique-gradient, P=1M fp32"
HBM_PEAK_GBS = 8000.0
FP32_PEAK_TFLOPS = 157.3
# dense bf16 MFMA peak (MI355X_MICROARCH.md: ~2.5 PF dense, 16x the fp32-input MFMA rate)
BF16_PEAK_TFLOPS = 2500.0
B6_PRODUCTS = 6          # bf16 products per fp32 product in the split GEMM (kernel "dense")


def parse():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawTextHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="dcliques1000",
                    choices=["dcliques1000", "ring100", "fc1000", "dcliques1000-smallworld",
                             "dcliques10000"])
    ap.add_argument("--p", type=int, default=None, help="parameters per node (default per config)")
    ap.add_argument("--kernel", default="auto",
                    choices=["auto", "csr-exact", "csr-fast", "ell-exact", "ell-fast", "band-exact",
                             "band-fast", "clique", "dense", "dense-f32", "tile-exact",
                             "tile-fast", "tile-lds-exact", "tile-lds-fast"])
    ap.add_argument("--interclique", default="fully-connected",
                    choices=["fully-connected", "smallworld", "ring"],
                    help="multi-GPU global d-cliques interclique topology")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-cold-cache", action="store_true",
                    help="skip the cold-cache single-round timing of graph-replayed configs")
    ap.add_argument("--cpu-sample-nodes", type=int, default=0,
                    help="bound the CPU baseline to the first K nodes' averages (0 = full round)")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic.json"))
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--graph", default="auto", choices=["auto", "on", "off"],
                    help="capture the K timed rounds in one hipGraph (auto: slabs < 256 MiB, where a "
                         "round is launch-bound rather than HBM-bound)")
    ap.add_argument("--e2e", action="store_true",
                    help="also time the host-resident round (pinned [N,P] host slab -> H2D -> mix -> "
                         "D2H, pipelined over column windows: the drop-in's per-round cost)")
    ap.add_argument("--e2e-step", action="store_true",
                    help="also time the drop-in's WHOLE round (d_sgd.next_step: CPU training of every "
                         "node, optimizer steps, mixing) with and without the mixing, and report the "
                         "mixing's exposed cost per round (row-streamed / windowed)")
    ap.add_argument("--e2e-rounds", type=int, default=5,
                    help="--e2e-step: timed rounds per variant (after one warm-up round)")
    ap.add_argument("--e2e-variants", type=str, default="",
                    help="--e2e-step: comma-separated subset of the variants (cpu_only_slab, the "
                         "baseline, is always run)")
    ap.add_argument("--e2e-threads", type=int, default=0,
                    help="--e2e-step: torch CPU threads for the training (default: torch's own count)")
    ap.add_argument("--layout", default="blocked", choices=["blocked", "blocked-rank", "rowmajor"],
                    help="single GPU, clique kernel: device-resident slabs column-blocked [P/B, N, B] "
                         "with clique-contiguous rows and B per plan (Mixer.device_layout, default), "
                         "column-blocked [P/1024, N, 1024] in rank order, or row-major [N, P]")
    ap.add_argument("--hipmalloc-slabs", action="store_true",
                    help="single GPU: allocate the slabs with torch's default (hipMalloc) allocator "
                         "instead of the VMM-mapped slab pool")
    ap.add_argument("--ld-pad", type=int, default=-1,
                    help="single GPU: pad every slab row by this many floats (ld = P + pad); "
                         "default: a 256-B row pitch for few-node low-degree graphs (ring 100), "
                         "none otherwise")
    ap.add_argument("--workload", default="mix", choices=["mix", "grad-clique"],
                    help="mix: the headline neighbour mixing round; grad-clique: the --clique-gradient "
                         "gradient mean (k_grad_segment_mean) over the same 1000-node d-cliques "
                         "topology (single GPU)")
    ap.add_argument("--nodes-per-gpu", type=int, default=1000,
                    help="multi-GPU weak scaling: nodes per rank (nodes x GPUs a multiple of 100; 1250 at "
                         "--gpus 8 gives BASELINE configs[4], 10000 nodes)")
    ap.add_argument("--shard", default="stripes", choices=["stripes", "nodes"],
                    help="multi-GPU partition: parameter-column stripes of every node (no exchange) "
                         "or node shards with an RCCL halo exchange")
    ap.add_argument("--windows", type=int, default=8,
                    help="multi-GPU: column windows the halo exchange is pipelined over")
    ap.add_argument("--single-ref", default="auto", choices=["auto", "on", "off"],
                    help="multi-GPU: rank 0 also times the N=1 point on its own GPU in the same run "
                         "(--config dcliques10000: the whole fixed problem -> speedup_vs_1gpu; "
                         "weak line: nodes_per_gpu nodes -> weak_efficiency_vs_1gpu) (auto: on)")
    ap.add_argument("--node-legs", default="auto",
                    help="multi-GPU with --shard stripes: after the stripes line, also time the "
                         "NODE-SHARD partition (RCCL halo exchange) on the same problem, one leg per "
                         "interclique in this comma list (auto: --interclique, then smallworld; "
                         "off: none).  Results go to config.node_shards; a failed or timed-out leg "
                         "records its error there and the stripes line is still printed")
    ap.add_argument("--leg-timeout", type=float, default=240.0,
                    help="multi-GPU: seconds one node-shard leg may take before every rank gives up "
                         "(rank 0 prints the line with the error, then all ranks exit 0)")
    ap.add_argument("--pg-timeout", type=float, default=900.0,
                    help="multi-GPU: torch.distributed collective timeout (seconds), above "
                         "--leg-timeout so the leg watchdog fires first")
    return ap.parse_args()


def golden(name):
    d = np.load(os.path.join(REPO, "tests", "golden", name + ".npz"))
    cl = None
    if "cliques_flat" in d:
        f, p = d["cliques_flat"], d["cliques_ptr"]
        cl = [f[p[i]:p[i + 1]].tolist() for i in range(len(p) - 1)]
    from niidmix.topology import MixCSR
    return MixCSR(d["row_ptr"], d["col"], d["val"]).validate(), cl


def single_gpu_topology(cfg):
    """(csr, cliques, default P, workload description)."""
    from niidmix.topology import mh_csr
    if cfg == "dcliques1000":
        csr, cl = golden("dcliques1000_fc_p64")
        return csr, cl, 1 << 20, ("d-cliques N=1000 (10 cliques x 100, fully-connected interclique, "
                                  "MH weights; topology generated by the reference, seed 1337)")
    if cfg == "dcliques1000-smallworld":
        csr, cl = golden("dcliques1000_smallworld_p16")
        return csr, cl, 1 << 20, "d-cliques N=1000 (10x100, smallworld interclique, MH)"
    if cfg == "ring100":
        csr, cl = golden("ring100_p257")
        return csr, cl, 62006, "ring N=100 (MH 1/3), P=62006 (LeNet-size)"
    if cfg == "dcliques10000":
        from niidmix.generate import dcliques_csr
        csr, cl = dcliques_csr(10000, 100, "fully-connected", 1337)
        return csr, cl, 1 << 20, ("d-cliques N=10000 (100 cliques x 100, fully-connected interclique, "
                                  "MH; the reference's generator restated, seed 1337) on ONE GPU: "
                                  "2 x 42 GB slabs resident in HBM")
    if cfg == "fc1000":
        n = 1000
        csr = mh_csr(n, {i: [j for j in range(n) if j != i] for i in range(n)})
        return csr, None, 1 << 20, "fully-connected N=1000 (MH weights, dense W)"
    raise ValueError(cfg)


def stream_copy_probe(numel, dev, iters=10):
    """This GPU's own HBM copy ceiling: libniidmix's streaming copy (nt float4 loads + stores,
    linear order) of a slab of the same size, 2*bytes per copy.  Boxes differ by up to ~20 %."""
    from niidmix import _lib
    numel -= numel % 4
    a = torch.zeros(numel, device=dev)
    b = torch.empty_like(a)
    strm = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)

    def cp():
        _lib.check(_lib.lib.niidmix_stream_copy_f32(a.data_ptr(), b.data_ptr(), numel, strm),
                   "stream copy")
    cp()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        cp()
    e.record()
    torch.cuda.synchronize()
    del a, b
    return 2 * numel * 4 * iters / (s.elapsed_time(e) / 1e3) / 1e9


def cold_cache_rounds(step, xa, xb, dev, rounds=10, flush_bytes=1 << 30):
    """a cache-resident config (the ring's 24.8 MB slab lives in the 256 MB MALL
    between graph-replayed rounds) is also timed once cold.  Before each round a 1 GiB scratch
    buffer is read and written (evicting the MALL and every XCD's L2), then ONE round is timed
    alone with HIP events on the launch stream; the same single-round timing without the flush is
    reported beside it (eager launches, so both include one launch's gap, unlike the graph).  The
    GPU is kept busy while the round is enqueued (the flush, or a short spin for the warm round), so
    the events time the GPU's work, not the host's enqueue of it."""
    scratch = torch.zeros(flush_bytes // 4, dtype=torch.float32, device=dev)
    stream = torch.cuda.current_stream(dev)
    spin = getattr(torch.cuda, "_sleep", None)
    res = {}
    for name, flush in (("warm_eager_us", False), ("cold_us", True)):
        ts = []
        for _ in range(rounds):
            if flush:
                scratch.add_(1.0)
            elif spin is not None:
                spin(1 << 20)                           # ~0.5 ms of GPU spin, touches no memory
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            step(xa, xb)
            e1.record(stream)
            torch.cuda.synchronize(dev)
            ts.append(e0.elapsed_time(e1) * 1e3)
            xa, xb = xb, xa
        res[name] = round(float(np.median(ts)), 2)
    del scratch
    torch.cuda.empty_cache()
    res["flush"] = f"{flush_bytes >> 20} MiB read+written before each cold round; median of {rounds}"
    return res


def e2e_rounds(mixer, n, p, dev, rounds=3):
    """Host-resident round as the drop-in runs it (niidmix.slab.SlabMixer): pinned host slab,
    H2D / mix / D2H pipelined over 32K-column windows on three streams."""
    from niidmix.slab import SlabMixer
    host = torch.empty((n, p), dtype=torch.float32, pin_memory=True)
    host.normal_()
    runner = SlabMixer(mixer, n, p, dev, window=int(os.environ.get("NIIDMIX_WINDOW", 1 << 15)))
    res = {}
    for mode in ("fast", "exact"):
        runner.mix(host, mode=mode)                     # warm-up
        ts = []
        for _ in range(rounds):
            runner.mix(host, mode=mode, timing=True)
            ts.append(runner.last_timing["round_s"])
        t = float(np.median(ts))
        res[mode] = {"round_ms": round(t * 1e3, 2), "GBs": round(n * p * 4 / t / 1e9, 1)}
    # the 'sample' topology's round (d_sgd.py:235-250) as the drop-in runs it (d_sgd.sample_average:
    # SampleAverage streamed over the same pinned slab): average of k active rows, then
    # update_models of every row; k = n / 10 rows drawn like get_sample's Random(42)
    from random import Random
    from niidmix.slab import SampleAverage
    k = max(1, n // 10)
    active = Random(42).sample(range(n), k)
    op = SampleAverage(dev)
    op.set_active(active, [1 / k] * k)
    srun = SlabMixer(op, n, p, dev, window=runner.window)
    srun.mix(host, mode="exact")
    ts = []
    for _ in range(rounds):
        srun.mix(host, mode="exact", timing=True)
        ts.append(srun.last_timing["round_s"])
    t = float(np.median(ts))
    res["sample"] = {"round_ms": round(t * 1e3, 2), "GBs": round(n * p * 4 / t / 1e9, 1),
                     "active_rows": k}
    del srun
    # PCIe reference: one plain pinned H2D and D2H of the whole slab
    d = torch.empty((n, p), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter(); d.copy_(host, non_blocking=True); torch.cuda.synchronize()
    h2d = time.perf_counter() - t0
    t0 = time.perf_counter(); host.copy_(d, non_blocking=True); torch.cuda.synchronize()
    d2h = time.perf_counter() - t0
    res["pcie_h2d_GBs"] = round(n * p * 4 / h2d / 1e9, 1)
    res["pcie_d2h_GBs"] = round(n * p * 4 / d2h / 1e9, 1)
    res["window_cols"] = runner.window
    return res


def e2e_fused_rounds(grad_op, plan, csr, cliques, n, p, dev, rounds=3):
    """Host-resident drop-in round WITH gradient averaging (--clique-gradient): the fused device
    round (niidmix.slab.FusedRoundRunner: H2D params + grads, gradient mean -> SGD step -> mixing,
    D2H params) against the unfused one (gradient slab round trip, CPU-side nothing, then the
    mixing slab round trip; the optimizer step itself is not timed there)."""
    from niidmix import ops
    from niidmix.slab import FusedRoundRunner, SlabMixer
    hp = torch.empty((n, p), dtype=torch.float32, pin_memory=True)
    hg = torch.empty((n, p), dtype=torch.float32, pin_memory=True)
    hp.normal_()
    hg.normal_()
    mixer = ops.Mixer(csr=csr, cliques=cliques, device=dev)
    w = int(os.environ.get("NIIDMIX_WINDOW", 1 << 15))
    fused = FusedRoundRunner(grad_op, plan.stepped, 0.1, mixer, n, p, dev, window=w)
    res = {}
    for mode in ("fast", "exact"):
        fused.run(hp, hg, mode=mode)
        ts = []
        for _ in range(rounds):
            fused.run(hp, hg, mode=mode, timing=True)
            ts.append(fused.last_timing["round_s"])
        res[f"fused_{mode}_round_ms"] = round(float(np.median(ts)) * 1e3, 2)
    del fused
    g_run = SlabMixer(grad_op, n, p, dev, window=w)
    m_run = SlabMixer(mixer, n, p, dev, window=w)
    g_run.mix(hg)
    m_run.mix(hp, mode="exact")
    ts = []
    for _ in range(rounds):
        t0 = time.perf_counter()
        g_run.mix(hg)
        m_run.mix(hp, mode="exact")
        ts.append(time.perf_counter() - t0)
    res["unfused_exact_round_ms"] = round(float(np.median(ts)) * 1e3, 2)
    res["window_cols"] = w
    return res


def e2e_next_step(csr, cliques, dev, rounds=5, mode="exact", only=None):
    """The drop-in's whole round, d_sgd.next_step (d_sgd.py:178-254) on the same topology: N nodes
    training on the CPU (synthetic data, a Linear(1023, 1024) model = 2^20 fp32 parameters, batch
    16), each node's optimizer.step(), then the mixing.  Variants, all built first and then run
    round-robin (round k of every variant before round k + 1 of any, so that drifts of the host's
    speed hit all of them alike), each timed over `rounds` rounds after one warm-up round:
      cpu_only            the same rounds with the mixing removed (the CPU part of the round);
      cpu_only_slab       the same with the parameters in the drop-in's pinned host slab (the
                          baseline exposed_ms is taken against: that memory alone changes the
                          CPU's training speed on some hosts);
      row_streamed        the plugin's default: the optimizer step on the device (round 6:
                          each node's gradient row goes H2D right after its backward(), the
                          parameters stay resident in HBM between rounds), the mixed rows come
                          back while the next round trains (deferred write-back);
      row_streamed_cpu_step  the round-4/5 default: the CPU steps, parameter rows go H2D right
                          after their optimizer.step() (NIIDMIX_DEVICE_STEP=0);
      row_streamed_paced  the same with the write-back paced (NIIDMIX_D2H_PACE=8: row blocks go D2H
                          8 ahead of the training that needs them, not all at once);
      row_streamed_sync   the same, but next_step waits for every mixed row before returning;
      windowed            the synchronous windowed round of rounds 1-3 (NIIDMIX_RESIDENT=0);
      fused_*             the same two with --clique-gradient (gradient mean + SGD step + mixing
                          on the device; parameter and gradient rows go up after each backward).
    exposed_ms = median round - median cpu_only_slab round (the mixing's cost the round still pays);
    host_blocked_ms = the time next_step itself spent waiting for rows or enqueueing copies and
    kernels (d_sgd.round_stats), the part of exposed_ms the plugin controls."""
    from niidmix import d_sgd
    n = csr.n
    edges = csr.edges()
    topo = {"edges": edges, "weights": torch.from_numpy(csr.dense())}
    if cliques:
        topo["cliques"] = cliques
    in_f, out_f, batch = 1023, 1024, 16
    g = torch.Generator().manual_seed(11)
    data = [(torch.randn(in_f, generator=g), int(torch.randint(0, out_f, (1,), generator=g)))
            for _ in range(batch * (rounds + 3))]

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = torch.nn.Linear(in_f, out_f)

        def forward(self, x, params):
            return torch.nn.functional.log_softmax(self.fc(x), dim=1)

    variants = ["cpu_only", "cpu_only_slab", "row_streamed", "row_streamed_cpu_step",
                "row_streamed_paced", "row_streamed_sync", "windowed"]
    if cliques:
        variants += ["fused_row_streamed", "fused_windowed"]
    if only:
        variants = [v for v in variants if v in only or v.startswith("cpu_only")]
    orig, orig_rs = d_sgd.average, d_sgd._row_streamed
    env_res = os.environ.get("NIIDMIX_RESIDENT")

    def make(v):
        fused = v.startswith("fused")
        params = {"meta": {"log": "WARNING", "seed": 1337}, "topology": {"name": "d-cliques"},
                  "logger": {"accuracy-logging-interval": 0, "accuracy-logging-interval-steps": 0,
                             "log-consensus-distance": False},
                  "algorithm": {"learning-rate": 0.1, "learning-momentum": 0.0, "batch-size": batch,
                                "initial-averaging": False, "clique-gradient": fused,
                                "unbiased-gradient": False, "mixing-mode": mode,
                                "deferred-writeback": v in ("row_streamed", "row_streamed_paced",
                                                            "row_streamed_cpu_step",
                                                            "fused_row_streamed")}}
        torch.manual_seed(3)
        nodes = []
        for r in range(n):
            mdl = Net()
            nodes.append({"rank": r, "epoch": 0, "train-set": data, "model": mdl,
                          "optimizer": d_sgd.optimizer(mdl, params)})
        st = {"params": params, "nodes": nodes, "ts": [], "blocked": 0.0, "wait": 0.0}
        if v == "cpu_only_slab":
            # the CPU part with the models' parameters in the drop-in's pinned host slab (its
            # memory trains at its own speed on some hosts), and no mixing
            from niidmix.slab import NodeSlab
            st["slab"] = NodeSlab([nd["model"] for nd in nodes])
        return st

    def step(v, st, k):
        if v.startswith("cpu_only"):
            d_sgd.average = lambda nds, t, p: None
            d_sgd._row_streamed = lambda p: False
        if v.endswith("windowed"):
            os.environ["NIIDMIX_RESIDENT"] = "0"          # read when the engine is built
        # paced write-back (niidmix.slab.ResidentRound, NIIDMIX_D2H_PACE): 8 row blocks ahead
        pace_env = os.environ.pop("NIIDMIX_D2H_PACE", None)
        if v == "row_streamed_paced":
            os.environ["NIIDMIX_D2H_PACE"] = "8"
        step_env = os.environ.pop("NIIDMIX_DEVICE_STEP", None)
        if v == "row_streamed_cpu_step":
            os.environ["NIIDMIX_DEVICE_STEP"] = "0"
        try:
            for key in ("wait_s", "enqueue_s"):
                d_sgd.round_stats[key] = 0.0
            t0 = time.perf_counter()
            if k < 0:
                st["state"], _, _ = d_sgd.init(st["nodes"], topo, st["params"])
            else:
                st["state"], _, _, _ = d_sgd.next_step(st["state"], st["params"], None)
            dt = time.perf_counter() - t0
            if k >= 1:
                st["ts"].append(dt)
                st["blocked"] += d_sgd.round_stats["wait_s"] + d_sgd.round_stats["enqueue_s"]
                st["wait"] += d_sgd.round_stats["wait_s"]
        finally:
            d_sgd.average, d_sgd._row_streamed = orig, orig_rs
            os.environ.pop("NIIDMIX_D2H_PACE", None)
            if pace_env is not None:
                os.environ["NIIDMIX_D2H_PACE"] = pace_env
            os.environ.pop("NIIDMIX_DEVICE_STEP", None)
            if step_env is not None:
                os.environ["NIIDMIX_DEVICE_STEP"] = step_env
            if env_res is None:
                os.environ.pop("NIIDMIX_RESIDENT", None)
            else:
                os.environ["NIIDMIX_RESIDENT"] = env_res

    d_sgd.MAX_ENGINES = max(d_sgd.MAX_ENGINES, len(variants))
    sts = {v: make(v) for v in variants}
    for k in range(-1, rounds + 1):                     # init, one warm-up round, timed rounds
        for v in variants:
            step(v, sts[v], k)
        print(f"[bench --e2e-step] round {k} done", file=sys.stderr, flush=True)
    d_sgd.synchronize()
    res = {"nodes": n, "p": in_f * out_f + out_f, "model": f"Linear({in_f}, {out_f})",
           "batch": batch, "rounds_timed": rounds, "mode": mode, "threads": torch.get_num_threads(),
           "order": "round-robin over the variants"}
    base = float(np.median(sts["cpu_only"]["ts"]))
    base_slab = float(np.median(sts["cpu_only_slab"]["ts"]))
    res["exposed_vs"] = ("cpu_only_slab: the same CPU rounds with the parameters in the pinned "
                         "slab and no mixing (exposed_ms_vs_plain_models: against models whose "
                         "parameters are plain allocations)")
    for v in variants:
        st = sts[v]
        out = {"round_ms": round(float(np.median(st["ts"])) * 1e3, 1),
               "round_ms_min": round(min(st["ts"]) * 1e3, 1)}
        if not v.startswith("cpu_only"):
            out["exposed_ms"] = round((float(np.median(st["ts"])) - base_slab) * 1e3, 1)
            out["exposed_ms_vs_plain_models"] = round((float(np.median(st["ts"])) - base) * 1e3, 1)
            out["host_blocked_ms"] = round(st["blocked"] / rounds * 1e3, 2)
            out["host_wait_ms"] = round(st["wait"] / rounds * 1e3, 2)
        res[v] = out
    if "row_streamed" in sts:
        res["logger"] = e2e_logger_costs([nd["model"] for nd in sts["row_streamed"]["nodes"]])
    d_sgd._engines.clear()
    d_sgd._fused_engines.clear()
    del sts
    torch.cuda.empty_cache()
    return res


def e2e_logger_costs(models, reps=3, cpu_sample=50):
    """What run.py's logging costs after a round at this size, with the hooks
    niidmix.d_sgd.init installs (niidmix.logger): the consensus-distance statistics and the global
    model (setup.model.average over every node) read from the resident output slab; the consensus
    statistics again from the pinned host slab (one H2D, the path before the first round or after a
    guarded write); and the reference's CPU arithmetic (logger.py:257-284: fp32 centre, one
    model_distance per model) timed on the first `cpu_sample` models and scaled to all of them."""
    from niidmix import guard
    from niidmix import logger as nl
    hit = guard.resident_rows(models)
    if hit is None or not hit[0].fresh:
        return {"error": "no fresh resident slab after the rounds"}
    rr = hit[0]

    def med(fn):
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        return round(float(np.median(ts)) * 1e3, 2)
    out = {"consensus_resident_ms": med(lambda: nl.consensus_statistics(models)),
           "consensus_source": nl.last_source["consensus"],
           "global_average_resident_ms": med(lambda: nl.average(models)),
           "average_source": nl.last_source["average"]}
    rr.fresh = False
    try:
        out["consensus_host_slab_ms"] = med(lambda: nl.consensus_statistics(models))
        out["host_slab_source"] = nl.last_source["consensus"]
    finally:
        rr.fresh = True
    sample = models[:cpu_sample]
    t0 = time.perf_counter()
    with torch.no_grad():
        flat = [torch.cat([q.detach().reshape(-1) for q in m.parameters()]) for m in sample]
        w = float(1. / len(models))
        center = flat[0] * 0
        for f in flat:
            center = center + w * f
        _ = [float(torch.sum((center - f) ** 2)) for f in flat]
    out["consensus_cpu_reference_ms_scaled"] = round((time.perf_counter() - t0) * 1e3 *
                                                     len(models) / len(sample), 1)
    out["cpu_sample_models"] = len(sample)
    return out


def traffic_key(args, kernel, p, slab_layout):
    return f"{args.config}/{args.workload}/{kernel}/p{p}/{slab_layout}"


def timed_rounds(step, xa, xb, steps, warmup, dev, dist=None, use_graph=False, backend="nccl"):
    """The timed region (the driver's contract): `warmup` untimed rounds, then EXACTLY `steps`
    rounds bracketed by a barrier + device synchronize on both sides; the region time and the
    mean per-launch time (HIP events around every launch on the launch stream, or the replayed
    hipGraph's region / steps) are max-reduced over ranks.  step(a, b, evs) runs one round a -> b
    (ping-pong).  On a CPU device (gloo tests of this loop) host timers replace the HIP events.
    Returns (region_s, launch_ms, graph)."""
    cpu = dev.type == "cpu"
    for _ in range(warmup):
        step(xa, xb)
        xa, xb = xb, xa
    graph = None
    if use_graph and not cpu:
        # the K timed rounds as ONE hipGraph (ping-pong unrolled); replayed once in the timed region
        graph = torch.cuda.CUDAGraph()
        a, b = xa, xb
        with torch.cuda.graph(graph):
            for _ in range(steps):
                step(a, b)
                a, b = b, a
        graph.replay()                                   # warm replay
        torch.cuda.synchronize(dev)
    if cpu:
        if dist:
            dist.barrier()
        t0 = time.perf_counter()
        launches = []
        for _ in range(steps):
            t1 = time.perf_counter()
            step(xa, xb)
            launches.append(time.perf_counter() - t1)
            xa, xb = xb, xa
        region_s = time.perf_counter() - t0
        if dist:
            dist.barrier()
        launch_ms = float(np.mean(launches)) * 1e3
    else:
        stream = torch.cuda.current_stream(dev)
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
              for _ in range(steps)]
        t_start, t_end = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if dist:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t_start.record(stream)
        if graph is not None:
            graph.replay()
        else:
            for i in range(steps):
                step(xa, xb, ev[i])
                xa, xb = xb, xa
        t_end.record(stream)
        torch.cuda.synchronize(dev)
        if dist:
            dist.barrier()
        region_s = t_start.elapsed_time(t_end) / 1e3
        if graph is not None:
            launch_ms = region_s * 1e3 / steps           # kernels back to back inside the graph
        else:
            launch_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if dist:
        tt = torch.tensor([region_s, launch_ms], dtype=torch.float64,
                          device=dev if (backend == "nccl" and not cpu) else "cpu")
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        region_s, launch_ms = tt.tolist()
    return region_s, launch_ms, graph


class LegWatchdog:
    """Deadline for one multi-GPU leg.  A point-to-point exchange that one rank never joins leaves
    its peers waiting inside RCCL (no exception reaches Python), so a timer thread ends the run
    instead: on_fire() (rank 0 prints the line measured so far, with the leg's error) and then
    exit_fn(0) -- os._exit, the process ends in place (no exec, no retry)."""

    def __init__(self, seconds, on_fire, exit_fn=None):
        import threading
        self.on_fire = on_fire
        self.exit_fn = exit_fn or os._exit
        self.fired = False
        self.timer = threading.Timer(seconds, self._fire)
        self.timer.daemon = True

    def _fire(self):
        self.fired = True
        try:
            self.on_fire()
        finally:
            self.exit_fn(0)

    def __enter__(self):
        self.timer.start()
        return self

    def __exit__(self, *exc):
        self.timer.cancel()
        return False


def guarded_leg(fn, dist, world, rank, flag_device="cpu"):
    """Run one leg on every rank; an exception is captured, not raised.  Every rank then learns
    which ranks failed (one SUM all-reduce of a per-rank flag), so all ranks leave the leg
    together.  Returns (info, error): info = fn()'s result, or None with error = a string naming
    the failed ranks and this rank's own exception (if any)."""
    info, err = None, None
    try:
        info = fn()
    except Exception as e:                               # noqa: BLE001 - recorded in the line
        err = f"{type(e).__name__}: {e}"
        print(f"[bench rank {rank}] node-shard leg failed: {err}", file=sys.stderr, flush=True)
    flags = torch.zeros(world, dtype=torch.float64, device=flag_device)
    flags[rank] = 1.0 if err else 0.0
    if dist is not None and world > 1:
        dist.all_reduce(flags, op=dist.ReduceOp.SUM)
    failed = [r for r in range(world) if flags[r].item() > 0]
    if failed:
        return None, f"failed on rank(s) {failed}" + (f": {err}" if err else "")
    return info, None


def world_identity(dev, dist, world, backend):
    """What the N>1 run actually ran on: the backend, the RCCL version torch
    links, the world size the process group reports, and each rank's device identity (GPU UUID and
    PCI domain:bus:device, or the host process for the CPU rehearsals) all-gathered, so the line
    itself shows N ranks on N distinct GPUs."""
    import socket
    if dev.type == "cuda":
        pr = torch.cuda.get_device_properties(dev)
        ident = {"uuid": str(getattr(pr, "uuid", "")),
                 "pci": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}",
                 "host": socket.gethostname(), "name": pr.name}
    else:
        ident = {"uuid": None, "pci": None, "host": socket.gethostname(),
                 "name": f"cpu pid {os.getpid()}"}
    ids = [None] * world
    if dist is not None and world > 1:
        dist.all_gather_object(ids, ident)
    else:
        ids = [ident]
    keys = [(d["host"], d["uuid"], d["pci"]) if d["uuid"] else (d["host"], d["name"]) for d in ids]
    version = None
    if backend == "nccl":
        try:
            v = torch.cuda.nccl.version()
            version = ".".join(str(x) for x in v) if isinstance(v, tuple) else str(v)
        except Exception as e:                       # noqa: BLE001 - recorded, not fatal
            version = f"unavailable: {e}"
    return {"backend": backend, "rccl_version": version,
            "world_size": dist.get_world_size() if dist is not None and world > 1 else 1,
            "distinct_devices": len(set(keys)), "devices": ids}


def exchange_rate(sm, x, rounds, dev, dist, backend):
    """The node-shard halo exchange ALONE (no mixing): `rounds` rounds of every window's grouped
    send/recv, timed on the host between device synchronisations and barriers.  Per rank: bytes
    received and sent per round, seconds per round, and the achieved rate (received bytes / time)
    all-gathered -- the xGMI GB/s each rank's links delivered."""
    world = sm.world
    cuda = dev.type == "cuda"
    if world < 2:
        return None
    if cuda:
        torch.cuda.synchronize(dev)
    dist.barrier()
    t0 = time.perf_counter()
    for _ in range(rounds):
        if cuda:
            with torch.cuda.stream(sm.comm_stream):
                pend = [sm.transport.exchange(sm, k, x[k]) for k in range(sm.k)]
                for h in pend:
                    sm.transport.wait(h)
        else:
            pend = [sm.transport.exchange(sm, k, x[k]) for k in range(sm.k)]
            for h in pend:
                sm.transport.wait(h)
    if cuda:
        torch.cuda.synchronize(dev)
    sec = (time.perf_counter() - t0) / rounds
    dist.barrier()
    mine = torch.tensor([sm.halo_bytes, sm.send_bytes, sec], dtype=torch.float64,
                        device=dev if (backend == "nccl" and cuda) else "cpu")
    allr = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(allr, mine)
    rows = [t.tolist() for t in allr]
    return {"rounds": rounds,
            "ms_per_round": [round(r[2] * 1e3, 4) for r in rows],
            "recv_GB": [float(f"{r[0] / 1e9:.4g}") for r in rows],
            "send_GB": [float(f"{r[1] / 1e9:.4g}") for r in rows],
            "recv_GBs_per_rank": [float(f"{r[0] / r[2] / 1e9:.4g}") if r[2] > 0 else None
                                  for r in rows],
            "method": "exchange only (no mixing), host clock between device synchronisations"}


def node_shard_leg(make, interclique, steps, warmup, dev, dist, backend, seed=0, single_ms=None,
                   fixed=False, fill=None):
    """Time the NODE-SHARD partition on one interclique with bench's own timed loop: `make(ic)`
    returns this rank's ShardedMixer (whole cliques per rank; every round the rows other ranks read
    go out and the rows this rank reads come in by grouped point-to-point, batch_isend_irecv =
    grouped ncclSend / ncclRecv over xGMI, pipelined with the mixing over column windows).  The
    reference's only exchange design is the same per-edge push (v1 gossip: isend(theta * W) /
    recv per edge, tools/v1/simulate.py:1570-1602).  fill(sm, x) sets the initial local rows
    (default: seeded N(0, 1)).  Returns (info, last output slab, mixer)."""
    sm = make(interclique)
    xa = sm.empty()
    if fill is None:
        gen = torch.Generator(device=dev).manual_seed(seed + 1000 * (sm.rank + 1))
        xa.normal_(generator=gen)
    else:
        fill(sm, xa)
    xb = sm.empty()
    kernel = sm.kernel_for("fast", xa)
    mode = "exact" if str(kernel).endswith("exact") else "fast"

    def step(a, b, evs=None):
        sm(a, b, kernel=kernel, mode=mode, events=evs)
    region_s, launch_ms, _ = timed_rounds(step, xa, xb, steps, warmup, dev, dist, False, backend)
    hb = torch.tensor([sm.halo_bytes, sm.send_bytes, sm.halo_rows], dtype=torch.float64,
                      device=dev if (backend == "nccl" and dev.type == "cuda") else "cpu")
    if dist is not None:
        dist.all_reduce(hb, op=dist.ReduceOp.MAX)
    ms = region_s * 1e3 / steps
    info = {"interclique": interclique, "ms_per_step": round(ms, 4),
            "value_GBs": round(sm.n_total * sm.p * 4 / (ms / 1e3) / 1e9, 2),
            "launch_ms": round(launch_ms, 4), "kernel": kernel, "mode": mode,
            "windows": sm.k, "window_cols": sm.w,
            "halo_rows_max": int(hb[2].item()),
            "halo_GB_recv_max": round(hb[0].item() / 1e9, 3),
            "halo_GB_send_max": round(hb[1].item() / 1e9, 3),
            "exchange": ("per column window: pack rows several peers read (index_select), "
                         "batch_isend_irecv with every peer (grouped ncclSend/ncclRecv) on a comm "
                         "stream; the compute stream waits only for that window")}
    if single_ms:
        key = "speedup_vs_1gpu" if fixed else "weak_efficiency_vs_1gpu"
        info[key] = round(single_ms / ms, 3)
    last = xa if (steps + warmup) % 2 == 0 else xb
    if dist is not None and sm.world > 1:
        # after the timed rounds, on the slab that is not the result: the exchange alone
        info["xgmi"] = exchange_rate(sm, xb if last is xa else xa, max(2, steps // 2), dev, dist,
                                     backend)
    return info, last, sm


def node_leg_intercliques(spec, interclique):
    if spec == "off":
        return []
    if spec == "auto":
        return [interclique] + (["smallworld"] if interclique != "smallworld" else [])
    out = [s.strip() for s in spec.split(",") if s.strip()]
    bad = [s for s in out if s not in ("fully-connected", "smallworld", "ring")]
    if bad:
        raise SystemExit(f"--node-legs: unknown interclique(s) {bad}")
    return out


def run_node_legs(make, intercliques, args, world, rank, dev, dist, backend, single_ms, fixed,
                  report, on_timeout=None, exit_fn=None):
    """Every node-shard leg, each under its own LegWatchdog and guarded_leg.  `report` is the list
    the results go into (rank 0's line holds it as config.node_shards); on a timeout the leg's
    error is appended and on_timeout() (rank 0: print the line as it stands) runs before exit."""
    flag_dev = dev if (backend == "nccl" and dev.type == "cuda") else "cpu"
    for ic in intercliques:
        pending = {"interclique": ic, "error": f"timed out after {args.leg_timeout:.0f} s"}

        def fire():
            report.append(pending)
            if on_timeout is not None:
                on_timeout()
        if rank == 0:
            print(f"[bench] node-shard leg {ic}: start", file=sys.stderr, flush=True)
        with LegWatchdog(args.leg_timeout, fire, exit_fn):
            info, err = guarded_leg(
                lambda: node_shard_leg(make, ic, args.steps, args.warmup, dev, dist, backend,
                                       args.seed, single_ms, fixed)[0],
                dist, world, rank, flag_dev)
        report.append(info if err is None else {"interclique": ic, "error": err})
        if rank == 0:
            print(f"[bench] node-shard leg {ic}: {'ok' if err is None else err}",
                  file=sys.stderr, flush=True)
        if dev.type == "cuda":
            torch.cuda.empty_cache()
    return report


def single_gpu_round_ms(n, p, interclique, dev, steps, warmup):
    """One GPU, the whole d-cliques problem of n nodes: the headline kernel on column-blocked VMM
    slabs (2 x n*p*4 bytes), mean of `steps` rounds after `warmup`."""
    from niidmix import memory, ops
    from niidmix.generate import dcliques_csr
    csr, cliques = dcliques_csr(n, 100, interclique, 1337)
    m = ops.Mixer(csr=csr, cliques=cliques, device=dev)
    perm, bc = m.device_layout()
    m = m.relabeled(perm)
    xa = memory.empty_blocked(n, p, dev, bc)
    xa.normal_(generator=torch.Generator(device=dev).manual_seed(7))
    xb = memory.empty_blocked(n, p, dev, bc)
    for _ in range(warmup):
        m.mix_blocked(xa, xb, p)
        xa, xb = xb, xa
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    s.record()
    for _ in range(steps):
        m.mix_blocked(xa, xb, p)
        xa, xb = xb, xa
    e.record()
    torch.cuda.synchronize(dev)
    ms = s.elapsed_time(e) / steps
    del xa, xb
    torch.cuda.empty_cache()
    return ms


def load_traffic(path, key, lib_sha):
    """PMC bytes per launch for `key` from profiles/traffic.json (tools/pmc_traffic.py), only if the
    entry was measured with THIS library (lib_sha16 stamp); else (None, why)."""
    try:
        with open(path) as f:
            e = json.load(f).get("entries", {}).get(key)
    except (OSError, ValueError):
        return None, "no traffic file"
    if e is None:
        return None, f"no PMC entry for {key}"
    if e.get("lib_sha16") != lib_sha:
        return None, f"PMC entry stale (measured with library {e.get('lib_sha16')}, loaded {lib_sha})"
    return float(e["bytes"]), "PMC (FETCH_SIZE x2 + WRITE_SIZE) of this library, profiles/traffic.json"



def cpu_baseline(csr, p, sample_nodes):
    """Faithful restatement of the reference loop on this host (oracle, checker/baseline only)."""
    from oracle import oracle
    n = csr.n
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    torch.set_num_threads(threads)
    W = torch.from_numpy(csr.dense())
    edges = csr.edges()
    g = torch.Generator().manual_seed(1)
    nodes = []
    for r in range(n):
        m = torch.nn.Module()
        m.w = torch.nn.Parameter(torch.randn(p, generator=g))
        nodes.append({"rank": r, "model": m})
    todo = nodes if not sample_nodes else nodes[:sample_nodes]
    # warm-up on two tiny models (allocator, thread pool)
    tiny = [{"rank": i, "model": torch.nn.Linear(4, 1)} for i in range(2)]
    oracle.reference_loop_average(tiny, {"weights": torch.tensor([[.5, .5], [.5, .5]]),
                                         "edges": {0: [1], 1: [0]}})

    # time the averages of `todo` (all nodes = one full round incl. update_models)
    t0 = time.perf_counter()
    if len(todo) == n:
        oracle.reference_loop_average(nodes, {"weights": W, "edges": edges})
    else:
        sub = {"weights": W, "edges": edges}
        # restrict the outer loop to the sampled nodes; neighbours still read the full node list
        _reference_partial(oracle, nodes, todo, sub)
    t = time.perf_counter() - t0
    k = len(todo)
    return {"value": k * p * 4 / t / 1e9, "unit": "GB/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"one round of the reference loop (oracle.reference_loop_average) over "
                      f"{k} of {n} nodes at P={p}, torch {torch.__version__} CPU, "
                      f"{torch.get_num_threads()} threads: {t:.2f} s"}


def cpu_baseline_grad(cliques, n, p):
    """The reference's clique-gradient loop restated (oracle.reference_loop_clique_gradient), timed
    on this host over the first clique (a bounded sample; every clique costs the same)."""
    from oracle import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or len(os.sched_getaffinity(0))
    torch.set_num_threads(threads)
    g = torch.Generator().manual_seed(1)
    clique = cliques[0]
    nodes = {}
    for r in clique:
        m = torch.nn.Module()
        m.w = torch.nn.Parameter(torch.zeros(p))
        m.w.grad = torch.randn(p, generator=g)
        nodes[r] = {"rank": r, "model": m}
    reps = 0
    t0 = time.perf_counter()
    while True:                       # repeat the clique until ~5 s of CPU work (a single clique
        oracle.reference_loop_clique_gradient(nodes, [clique])  # takes only ~10 ms at P = 2^20)
        reps += 1
        if time.perf_counter() - t0 > 5.0:
            break
    t = (time.perf_counter() - t0) / reps
    k = len(clique)
    return {"value": k * p * 4 / t / 1e9, "unit": "GB/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"the reference clique-gradient loop (oracle.reference_loop_clique_gradient) "
                      f"over clique 0 ({k} of {n} nodes) at P={p}, torch {torch.__version__} CPU, "
                      f"{torch.get_num_threads()} threads: {t * 1e3:.1f} ms per clique "
                      f"(mean of {reps} repetitions)"}


def _reference_partial(oracle, nodes, todo, topo):
    import copy
    W, edges = topo["weights"], topo["edges"]
    with torch.no_grad():
        res = {}
        for nd in todo:
            r = nd["rank"]
            grp = [nd["model"]] + [nodes[s]["model"] for s in edges[r]]
            cf = [W[r, r]] + [W[s, r] for s in edges[r]]
            c = copy.deepcopy(grp[0])
            for cp in c.parameters():
                cp.mul_(0)
            for mdl, w in zip(grp, cf):
                for cp, mp in zip(c.parameters(), mdl.parameters()):
                    cp.add_(w * mp)
            res[r] = c
        for nd in todo:
            for mp, newp in zip(nd["model"].parameters(), res[nd["rank"]].parameters()):
                mp.mul_(0.)
                mp.add_(newp)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # NIIDMIX_BENCH_BACKEND=gloo: rehearse the N-rank path with every rank on the visible GPU(s)
    # (one-GPU box; timing not meaningful).  The driver's runs use RCCL, one GPU per rank.
    backend = os.environ.get("NIIDMIX_BENCH_BACKEND", "nccl")
    gpu = local_rank if backend == "nccl" else local_rank % torch.cuda.device_count()
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist
        import datetime
        pg_timeout = datetime.timedelta(seconds=args.pg_timeout)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, timeout=pg_timeout)
        else:
            dist.init_process_group(backend, timeout=pg_timeout)

    from niidmix import memory, ops
    ident = world_identity(dev, dist, world, backend) if world > 1 else None
    if args.workload != "mix" and world > 1:
        raise SystemExit("--workload grad-clique is single-GPU")
    fixed = world > 1 and args.config == "dcliques10000"       # BASELINE configs[4]: strong scaling
    if world > 1 and args.config not in ("dcliques1000", "dcliques10000"):
        raise SystemExit("multi-GPU: --config dcliques1000 (weak, 1000 nodes per GPU) or dcliques10000")
    n_multi = 10000 if fixed else args.nodes_per_gpu * world
    if world == 1:
        csr, cliques, p_default, desc = single_gpu_topology(args.config)
        p = args.p or p_default
        if args.workload == "grad-clique":
            from niidmix.gradient import GradMean, build_grad_plan
            if not cliques:
                raise SystemExit(f"--workload grad-clique needs a clique topology, not {args.config}")
            plan = build_grad_plan(csr.n, {"cliques": cliques, "edges": csr.edges()},
                                   {"algorithm": {"clique-gradient": True}})
            mixer = GradMean(plan, dev)
            mixer.kernel_for = lambda mode, x=None: "grad-segment-mean"
            desc = "clique gradient mean (--clique-gradient, d_sgd.py:56-65) over " + desc
        else:
            mixer = ops.Mixer(csr=csr, cliques=cliques, device=dev)
        n_local = n_total = csr.n
        parallelism = "single GPU"
        gen = torch.Generator(device=dev).manual_seed(args.seed)
        # few nodes with ELL rows (ring 100): rows on a 256-B pitch, where the column-strip kernel
        # (Mixer.kernel_for) stores whole cache lines (--ld-pad N: ld = p + N instead)
        few = args.workload == "mix" and mixer.n <= ops.STRIP_MAX_ROWS and mixer.ell is not None
        ld = p + args.ld_pad if args.ld_pad >= 0 else (-(-p // 64) * 64 if few else p)
        # node-state slabs in VMM-mapped HBM (niidmix.memory); --hipmalloc-slabs:
        # torch's default allocator instead (placement-dependent speed, for comparison)
        alloc = (lambda: torch.empty(n_local, ld, device=dev)) if args.hipmalloc_slabs else \
            (lambda: memory.empty_slab(n_local, ld, dev))
        k0 = args.kernel
        if k0 == "auto":
            k0 = mixer.kernel_for("fast") if args.workload == "mix" else "grad-segment-mean"
        row_order = "rank"
        if args.layout == "blocked" and args.workload == "mix" and args.kernel in ("auto", "band-fast",
                                                                                 "band-exact"):
            perm, _ = mixer.device_layout() if mixer.plan is None else (None, None)
            if perm is not None:
                # a ring in its cycle order: every row's neighbours are the rows next to it, so the
                # band kernel reads them without descriptors (Mixer.device_layout)
                mixer = mixer.relabeled(perm)
                row_order = "ring cycle order"
                k0 = mixer.kernel_for("fast")
        if (args.layout in ("blocked", "blocked-rank") and not args.hipmalloc_slabs and p % 4 == 0
                and ((k0 == "clique" and args.workload == "mix" and mixer.plan.max_clique <= 1024)
                     or args.workload == "grad-clique")):
            # device-resident node state in the column-blocked layout [K, N, B],
            # with the row order and block width the factored kernel streams best
            # (Mixer.device_layout: clique-contiguous rows; B = 1024, 256 or 32 per plan)
            bc = memory.BLOCK_COLS
            if args.workload == "mix" and args.layout == "blocked":
                perm, bc = mixer.device_layout()
                if perm is not None:
                    mixer = mixer.relabeled(perm)
                    row_order = "clique-contiguous"
            xa = memory.empty_blocked(n_local, p, dev, bc)
            xa.normal_(generator=gen)
            xb = memory.empty_blocked(n_local, p, dev, bc)
        else:
            xa = alloc()
            xa.normal_(generator=gen)
            xa = xa[:, :p]
            xb = alloc()[:, :p]
        halo = 0
        cols_local = p
    elif args.shard == "stripes":
        from niidmix.shard import StripedMixer
        p = args.p or (1 << 20)
        mixer = StripedMixer.dcliques(n_total=n_multi, clique_size=100, world=world,
                                      rank=rank, interclique=args.interclique, device=dev, p=p,
                                      mode="exact" if args.kernel.endswith("exact") else "fast")
        n_local, n_total = mixer.n_local, mixer.n_total
        cols_local, halo = mixer.p_local, 0
        row_order = "clique-contiguous" if mixer.perm is not None else "rank"
        desc = (f"d-cliques N={n_total} ({n_total // 100} cliques x 100, {args.interclique} "
                f"interclique, MH), P={p} split in {world} column stripes")
        parallelism = (f"{world} parameter-column stripes of all {n_total} nodes (columns "
                       f"[{mixer.c0}, {mixer.c1}) on rank {rank}); no data-path collective")
        csr = None
        gen = torch.Generator(device=dev).manual_seed(args.seed + rank)
        xa = mixer.empty()
        xa.normal_(generator=gen)
        xb = mixer.empty()
    else:
        row_order = "shard-local (whole cliques)"
        from niidmix.shard import ShardedMixer
        p = args.p or (1 << 20)
        mixer = ShardedMixer.dcliques(n_total=n_multi, clique_size=100, world=world, rank=rank,
                                      interclique=args.interclique, device=dev, p=p,
                                      windows=args.windows)
        n_local, n_total = mixer.n_local, mixer.n_total
        halo = mixer.halo_rows
        cols_local = p
        desc = (f"d-cliques N={n_total} ({n_total // 100} cliques x 100, {args.interclique} "
                f"interclique, MH), {n_total // world} nodes per GPU on average; halo rows over RCCL")
        parallelism = (f"{world} clique-aligned node shards, RCCL (xGMI) halo exchange pipelined "
                       f"over {mixer.k} column windows")
        csr = None
        gen = torch.Generator(device=dev).manual_seed(args.seed + rank)
        xa = mixer.empty()
        xa.normal_(generator=gen)
        xb = mixer.empty()
    kernel = args.kernel if args.kernel != "auto" else mixer.kernel_for("fast", xa)
    mode = "exact" if kernel.endswith("exact") else "fast"

    blocked = world == 1 and xa.dim() == 3
    if blocked and args.workload == "mix":
        kernel = "clique"

    def step(a, b, evs=None):
        if world == 1:
            if evs is not None:
                evs[0].record(torch.cuda.current_stream(dev))
            if blocked and args.workload == "grad-clique":
                mixer.mean_blocked(a, b, p)
            elif blocked:
                mixer.mix_blocked(a, b, p)
            else:
                mixer(a, out=b, kernel=kernel, mode=mode)
            if evs is not None:
                evs[1].record(torch.cuda.current_stream(dev))
        else:
            mixer(a, b, kernel=kernel, mode=mode, events=evs)

    use_graph = world == 1 and (args.graph == "on" or
                                (args.graph == "auto" and n_local * cols_local * 4 < (256 << 20)))
    region_s, launch_ms, graph = timed_rounds(step, xa, xb, args.steps, args.warmup, dev, dist,
                                              use_graph, backend)
    step_s = region_s / args.steps
    value = n_total * p * 4 / step_s / 1e9
    slab_layout = (f"column-blocked [{xa.shape[0]}, {xa.shape[1]}, {xa.shape[2]}], "
                   f"{row_order} rows" if xa.dim() == 3 and (blocked or args.shard == "stripes") else
                   "window-blocked [K, rows_in, w]" if xa.dim() == 3 else
                   "row-major [N, P]" + (f" on a {xa.stride(0) * 4}-B row pitch"
                                         if xa.dim() == 2 and xa.stride(0) != p else "")
                   + (f", {row_order} rows" if row_order != "rank" else ""))
    single = None
    if world > 1 and args.single_ref != "off":
        # the N=1 point of this line, measured in the same run on rank 0's GPU with the same
        # kernel and layout (the other ranks wait): the fixed problem alone (strong scaling), or
        # one GPU's share of the weak line (nodes_per_gpu nodes, the same P)
        del xa, xb
        torch.cuda.empty_cache()
        if rank == 0:
            n1 = n_total if fixed else args.nodes_per_gpu
            single = single_gpu_round_ms(n1, p, args.interclique, dev, args.steps, args.warmup)
        dist.barrier()
    copy_gbs = stream_copy_probe(n_local * cols_local, dev)
    cold = (cold_cache_rounds(step, xa, xb, dev)
            if world == 1 and graph is not None and not args.no_cold_cache else None)

    out = None
    if rank == 0:
        # PMC traffic is profiled per single-GPU config and library build (profiles/traffic.json)
        from niidmix import _lib
        lib_sha = _lib.lib_sha16()
        traffic, traffic_src = (load_traffic(args.traffic_json, traffic_key(args, kernel, p,
                                                                            slab_layout), lib_sha)
                                if world == 1 else (None, "multi-GPU: not profiled"))
        if kernel == "dense":
            # the fp32 GEMM carried by bf16 splits: the matrix pipe executes B6_PRODUCTS bf16
            # products per algorithmic fp32 one, priced against the bf16 MFMA peak; the
            # algorithmic fp32 rate is reported beside it against the fp32 MFMA peak
            flops = 2.0 * n_local * n_local * cols_local
            fp32_rate = flops / (launch_ms / 1e3) / 1e12
            achieved = B6_PRODUCTS * fp32_rate
            roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": BF16_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved / BF16_PEAK_TFLOPS, 4),
                    "traffic": traffic,
                    "executed": f"{B6_PRODUCTS} bf16 products per fp32 product "
                                "(v_mfma_f32_32x32x16_bf16, three-term splits)",
                    "fp32_equivalent_TFLOPs": round(fp32_rate, 2),
                    "fp32_equivalent_frac_of_fp32_mfma_peak": round(fp32_rate / FP32_PEAK_TFLOPS, 4)}
        elif kernel == "dense-f32":
            flops = 2.0 * n_local * n_local * cols_local
            achieved = flops / (launch_ms / 1e3) / 1e12
            roof = {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP32_PEAK_TFLOPS,
                    "unit": "TFLOP/s", "frac": round(achieved / FP32_PEAK_TFLOPS, 4),
                    "traffic": traffic}
        else:
            alg = 2.0 * n_local * cols_local * 4
            achieved = alg / (launch_ms / 1e3) / 1e9
            roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                    "traffic": traffic}
            if cold is not None and 2 * n_local * cols_local * 4 < (256 << 20):
                # the slab pair lives in the 256 MB MALL between graph-replayed rounds: `frac` is a
                # cache-resident rate priced against the HBM peak; the cold round (MALL and L2
                # flushed first, one eager launch) priced the same way beside it
                roof["residency"] = "MALL-resident (slab pair < 256 MB): frac is not an HBM rate"
                if cold.get("cold_us"):
                    roof["cold_achieved"] = round(alg / (cold["cold_us"] / 1e6) / 1e9, 1)
                    roof["cold_frac"] = round(roof["cold_achieved"] / HBM_PEAK_GBS, 4)
        e2e = None
        if world == 1 and args.e2e and args.workload == "grad-clique":
            del xa, xb
            torch.cuda.empty_cache()
            e2e = e2e_fused_rounds(mixer, plan, csr, cliques, n_local, p, dev)
        elif world == 1 and args.e2e:
            e2e = e2e_rounds(mixer, n_local, p, dev)
        if world == 1 and args.e2e_step and csr is not None:
            xa = xb = None                              # noqa: F841 (free the device slabs)
            torch.cuda.empty_cache()
            e2e = dict(e2e or {})
            if args.e2e_threads > 0:
                torch.set_num_threads(args.e2e_threads)
            e2e["next_step"] = e2e_next_step(
                csr, cliques, dev, rounds=args.e2e_rounds,
                only=set(v for v in args.e2e_variants.split(",") if v) or None)
        cpu = None
        if world == 1 and not args.no_cpu_baseline and args.config != "dcliques10000":
            if args.workload == "grad-clique":
                cpu = cpu_baseline_grad(cliques, csr.n, p)
            else:
                cpu = cpu_baseline(csr, p, args.cpu_sample_nodes)
        out = {
            "metric": METRIC if args.workload == "mix" else GRAD_METRIC, "value": round(value, 2), "unit": "GB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(step_s * 1e3, 4),
            "higher_is_better": True, "scaling": "strong" if fixed else "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (seeded N(0,1) [N,P] fp32 slab resident in HBM; topology from the "
                    "reference's generators)",
            "config": {"workload": desc, "n_nodes": n_total, "p": p, "kernel": kernel,
                       "mode": mode, "parallelism": parallelism,
                       "launch_ms": round(launch_ms, 4), "halo_rows_rank0": halo,
                       "hipgraph": graph is not None,
                       "slab_memory": ("hipMalloc" if args.hipmalloc_slabs or
                                       (world > 1 and args.shard == "nodes")
                                       else "VMM 2 MiB chunks (niidmix_hbm_alloc)"),
                       "slab_layout": slab_layout,
                       "lib_sha16": lib_sha, "traffic_source": traffic_src,
                       "traffic_key": traffic_key(args, kernel, p, slab_layout),
                       "stream_copy_GBs": round(copy_gbs, 1),
                       "frac_of_stream_copy": (round(roof["achieved"] / copy_gbs, 4)
                                               if roof["unit"] == "GB/s" else None)},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if e2e is not None:
            out["e2e"] = e2e
        if cold is not None:
            # the slab pair fits the MALL, so the graph-replayed rounds run cache-resident
            out["config"]["cache_resident"] = 2 * n_local * cols_local * 4 < (256 << 20)
            out["config"]["cold_cache_round"] = cold
        if ident is not None:
            out["config"]["world"] = ident
        if world > 1 and args.shard == "nodes":
            out["config"]["halo_GB_recv_rank0"] = round(mixer.halo_bytes / 1e9, 3)
            out["config"]["halo_GB_send_rank0"] = round(mixer.send_bytes / 1e9, 3)
        if single is not None:
            out["config"]["single_gpu_ms"] = round(single, 4)
            if fixed:
                out["config"]["speedup_vs_1gpu"] = round(single / (step_s * 1e3), 3)
            else:       # weak: each GPU's work equals the N=1 round's
                out["config"]["single_gpu_nodes"] = args.nodes_per_gpu
                out["config"]["weak_efficiency_vs_1gpu"] = round(single / (step_s * 1e3), 3)
    node_legs = (node_leg_intercliques(args.node_legs, args.interclique)
                 if world > 1 and args.shard == "stripes" else [])
    import threading
    print_lock, printed = threading.Lock(), [False]

    def emit():
        with print_lock:
            if out is not None and not printed[0]:
                printed[0] = True
                print(json.dumps(out), flush=True)
    if node_legs:
        # the same problem again as NODE SHARDS: whole cliques per rank, cross-shard edges' rows
        # exchanged over RCCL every round; never changes the stripes `value`
        from niidmix.shard import ShardedMixer
        legs = []
        if out is not None:
            out["config"]["node_shards"] = legs

        def make(ic):
            return ShardedMixer.dcliques(n_total=n_multi, clique_size=100, world=world, rank=rank,
                                         interclique=ic, device=dev, p=p, windows=args.windows)
        run_node_legs(make, node_legs, args, world, rank, dev, dist, backend, single, fixed, legs,
                      on_timeout=emit)
    emit()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
