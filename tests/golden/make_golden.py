#!/usr/bin/env python
"""Generate the golden mixing fixtures by running the REFERENCE simulator's own code.

Run in the development container only (it needs /root/reference; the GPU box never runs it):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

What it does, per case:
  1. builds a topology with the reference generator (tools/setup/topology/*.py,
     tools/setup/topology/d_cliques/*.py) and its Metropolis-Hastings weights
     (tools/setup/topology/weights.py:3-32),
  2. writes topology.json exactly like the generators do (json.dump of
     {'edges', 'weights', 'cliques'?}) and reads it back with the reference
     loader `setup.topology.load` (tools/setup/topology/__init__.py:4-12),
  3. builds one node dict per rank whose 'model' holds seeded fp32 parameters,
  4. calls the reference hot path `simulate.algorithm.d_sgd.average`
     (tools/simulate/algorithm/d_sgd.py:96-116) and reads the parameters back.

Saved per case (tests/golden/<case>.npz):
  x, y           fp32 [N, P] slabs before / after one round (flattening = model.parameters() order)
  row_ptr, col, val   CSR of W^T in the reference's accumulation order: row i = [i] + edges[i],
                      val = W[i,i], W[src,i] ...   (d_sgd.py:105-110)
  cliques_flat, cliques_ptr   (d-cliques cases only)
  shapes_json    parameter shapes of the model (multi-tensor case)
Gradient cases (tests/golden/grad_<case>.npz) run the reference's `d_sgd.gradient`
(d_sgd.py:47-94: --clique-gradient with and without removed clique edges, --unbiased-gradient)
on nodes whose models carry seeded parameters AND seeded .grad tensors, with the reference's own
optimizer (d_sgd.optimizer: SGD lr 0.1, momentum 0), and store
  x, g           fp32 [N, P] parameters / gradients before
  y, g_out       fp32 [N, P] parameters / gradients after
  topology_json  {"edges", "cliques"?, "neighbourhoods"?} (no weights: gradient() never reads them)
  params_json    the 'algorithm' and 'topology' params passed
Non-finite cases (--nonfinite): d-cliques with and without removed clique edges and a complete graph
with ±inf, NaN, overflowing clique sums, -0.0 and subnormals.  Consensus cases (--consensus,
tests/golden/consensus_*.npz): the reference's Logger.log_consensus_distance run on seeded models;
x, shapes_json, the event (event_json) and stats = [avg, std, max, min, center norm].
Small cases additionally keep the raw topology.json (tests/golden/<case>.topology.json) so the
build's own reader can be checked against the reference loader's output.

The torchvision import in the reference's import chain (d_sgd -> setup.model -> linear ->
setup.dataset -> torchvision) is satisfied with an empty stub: torchvision is only used for
datasets, never by the mixing code.  Nothing from the reference is copied into this repo:
only inputs and outputs (data) are stored.
"""
import io
import json
import os
import sys
import tempfile
import types

import numpy as np
import torch

REF = os.environ.get("NIID_REFERENCE", "/root/reference")
OUT = os.path.dirname(os.path.abspath(__file__))


def _import_reference():
    for name in ["torchvision", "torchvision.datasets", "torchvision.transforms", "torchvision.utils"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["torchvision"].datasets = sys.modules["torchvision.datasets"]
    sys.modules["torchvision"].transforms = sys.modules["torchvision.transforms"]
    sys.path.insert(0, os.path.join(REF, "tools"))
    sys.path.insert(0, os.path.join(REF, "tools", "setup", "topology", "d_cliques"))
    import importlib
    mods = types.SimpleNamespace()
    mods.d_sgd = importlib.import_module("simulate.algorithm.d_sgd")
    mods.model = importlib.import_module("setup.model")
    mods.linear = importlib.import_module("setup.model.linear")
    mods.topo = importlib.import_module("setup.topology")
    mods.weights = importlib.import_module("setup.topology.weights")
    mods.metrics = importlib.import_module("setup.topology.metrics")
    mods.ring = importlib.import_module("setup.topology.ring")
    mods.fc = importlib.import_module("setup.topology.fully-connected")
    mods.expander = importlib.import_module("setup.topology.expander")
    mods.grid = importlib.import_module("setup.topology.grid")
    mods.random_graph = importlib.import_module("setup.topology.random_graph")
    mods.random_cliques = importlib.import_module("random_cliques")
    mods.interclique = importlib.import_module("interclique")
    mods.dc_utils = importlib.import_module("utils")
    return mods


R = _import_reference()
MH = {"weights": "metropolis-hasting"}


class FlatModel(torch.nn.Module):
    """A node model whose parameters have the given shapes (registration order = flattening order)."""

    def __init__(self, shapes):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(s)) for s in shapes])


def _nodes(n):
    return [{"rank": r, "classes": [0.1] * 10} for r in range(n)]


def _roundtrip(edges, weights, cliques=None):
    """topology.json exactly as the generators write it, read back by setup.topology.load."""
    topo = {"edges": {rank: list(edges[rank]) for rank in edges}, "weights": weights}
    if cliques is not None:
        topo["cliques"] = cliques
    text = json.dumps(topo)
    with tempfile.TemporaryDirectory() as d:
        with open(os.path.join(d, "topology.json"), "w") as f:
            f.write(text)
        loaded = R.topo.load(d)
    return text, loaded


def _csr(loaded, n):
    W = loaded["weights"]
    edges = loaded["edges"]
    row_ptr = [0]
    col, val = [], []
    for rank in range(n):
        srcs = [rank] + list(edges[rank])
        col += srcs
        val += [W[rank, rank].item()] + [W[s, rank].item() for s in edges[rank]]
        row_ptr.append(len(col))
    return (np.asarray(row_ptr, np.int64), np.asarray(col, np.int32), np.asarray(val, np.float32))


def _run_average(loaded, x, shapes):
    n = x.shape[0]
    nodes = []
    for rank in range(n):
        m = FlatModel(shapes) if shapes is not None else None
        flat = torch.from_numpy(x[rank].copy())
        with torch.no_grad():
            off = 0
            for p in m.parameters():
                k = p.numel()
                p.copy_(flat[off:off + k].view_as(p))
                off += k
        nodes.append({"rank": rank, "model": m})
    R.d_sgd.average(nodes, loaded, {})
    out = np.stack([torch.cat([p.detach().reshape(-1) for p in nd["model"].parameters()]).numpy()
                    for nd in nodes])
    return out


def save_case(name, edges, n, p, seed=0, cliques=None, shapes=None, x=None, keep_json=False,
              weights=None):
    if weights is None:
        weights = R.weights.compute_weights(_nodes(n), edges, MH)
    text, loaded = _roundtrip(edges, weights, cliques)
    if shapes is None:
        shapes = [(p,)]
    assert sum(int(np.prod(s)) for s in shapes) == p
    if x is None:
        g = torch.Generator().manual_seed(seed)
        x = torch.randn(n, p, generator=g, dtype=torch.float32).numpy()
    y = _run_average(loaded, x, shapes)
    row_ptr, col, val = _csr(loaded, n)
    extra = {}
    if cliques is not None:
        extra["cliques_flat"] = np.asarray([r for c in cliques for r in c], np.int32)
        extra["cliques_ptr"] = np.cumsum([0] + [len(c) for c in cliques]).astype(np.int64)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), x=x, y=y, row_ptr=row_ptr, col=col,
                        val=val, shapes_json=np.asarray(json.dumps([list(s) for s in shapes])),
                        **extra)
    if keep_json:
        with open(os.path.join(OUT, name + ".topology.json"), "w") as f:
            f.write(text)
    print(f"{name}: N={n} P={p} nnz={len(col)}")


def dcliques(n, size, interclique, seed=1337, remove=0):
    params = {"topology": {"max-clique-size": size, "remove-clique-edges": remove,
                           "interclique-topology": interclique},
              "meta": {"seed": seed}, "dataset": {"nb-classes": 10}}
    cl, intra = R.random_cliques.cliques(_nodes(n), params)
    edges = R.interclique.get(interclique)(cl, intra, params)
    if remove > 0:
        edges, cl = R.dc_utils.remove_clique_edges(edges, cl, params)
    return {rank: list(edges[rank]) for rank in edges}, [list(c) for c in cl]


def _flat(nodes, attr):
    out = []
    for nd in nodes:
        ts = [p.grad if attr == "grad" else p for p in nd["model"].parameters()]
        out.append(torch.cat([t.detach().reshape(-1) for t in ts]).numpy())
    return np.stack(out)


def save_grad_case(name, n, p, topo, alg, remove=0, shapes=None, seed=0, special=False):
    """Run the reference's d_sgd.gradient on seeded parameters + gradients (see module doc)."""
    shapes = shapes or [(p,)]
    assert sum(int(np.prod(s)) for s in shapes) == p
    gen = torch.Generator().manual_seed(seed)
    x = torch.randn(n, p, generator=gen).numpy()
    g = torch.randn(n, p, generator=gen).numpy()
    if special:
        g[0, 0] = np.inf; g[1, 1] = -np.inf; g[2, 2] = np.nan
        g[:, 3] = -0.0; g[0, 4] = -0.0; g[1, 5] = 3.0e38; g[2, 5] = 3.0e38; g[3, 6] = 1e-45
        x[:, 3] = -0.0
    params = {"algorithm": {"clique-gradient": alg == "clique", "unbiased-gradient": alg == "unbiased",
                            "learning-rate": 0.1, "learning-momentum": 0.0},
              "topology": {"remove-clique-edges": remove}}
    nodes = []
    for rank in range(n):
        m = FlatModel(shapes)
        off = 0
        with torch.no_grad():
            for q in m.parameters():
                k = q.numel()
                q.copy_(torch.from_numpy(x[rank, off:off + k].copy()).view_as(q))
                q.grad = torch.from_numpy(g[rank, off:off + k].copy()).view_as(q).clone()
                off += k
        nodes.append({"rank": rank, "model": m, "optimizer": R.d_sgd.optimizer(m, params)})
    text = json.dumps(topo)
    loaded = json.loads(text)
    loaded["edges"] = {int(r): loaded["edges"][r] for r in loaded["edges"]}
    if "neighbourhoods" in loaded:
        loaded["neighbourhoods"] = {int(r): loaded["neighbourhoods"][r] for r in loaded["neighbourhoods"]}
    R.d_sgd.gradient(nodes, loaded, params)
    np.savez_compressed(os.path.join(OUT, "grad_" + name + ".npz"), x=x, g=g, y=_flat(nodes, "data"),
                        g_out=_flat(nodes, "grad"), topology_json=np.asarray(text),
                        params_json=np.asarray(json.dumps(params)),
                        shapes_json=np.asarray(json.dumps([list(s) for s in shapes])))
    print(f"grad_{name}: N={n} P={p} {alg} remove={remove}")


def grad_cases():
    e, cl = dcliques(300, 30, "fully-connected")
    save_grad_case("dcliques300_fc_p37", 300, 37, {"edges": e, "cliques": cl}, "clique")
    e, cl = dcliques(1000, 100, "fully-connected")
    save_grad_case("dcliques1000_fc_p64", 1000, 64, {"edges": e, "cliques": cl}, "clique", seed=1)
    e, cl = dcliques(200, 20, "fractal", remove=5)
    save_grad_case("dcliques200_fractal_rm5_p40", 200, 40, {"edges": e, "cliques": cl}, "clique",
                   remove=5, seed=2)
    e, cl = dcliques(40, 10, "ring")
    save_grad_case("dcliques40_ring_special_p16", 40, 16, {"edges": e, "cliques": cl}, "clique",
                   seed=3, special=True)
    save_grad_case("dcliques40_ring_rm3_special_p16", 40, 16,
                   {"edges": dcliques(40, 10, "ring", remove=3)[0],
                    "cliques": dcliques(40, 10, "ring", remove=3)[1]}, "clique", remove=3, seed=4,
                   special=True)
    # 2 cliques of 2 with the linear MNIST model ([10,784] + [10]): flattening order of gradients
    save_grad_case("cliques4_linear7850", 4, 7850, {"edges": {0: [1], 1: [0, 2], 2: [3, 1], 3: [2]},
                                                   "cliques": [[1, 0], [2, 3]]}, "clique",
                   shapes=[(10, 784), (10,)], seed=5)
    # unbiased gradient: neighbourhoods of 1..9 nodes in shuffled order (incl. the node itself or
    # not), over a ring; the reference generators of this repo version do not emit neighbourhoods
    import random
    rnd = random.Random(1337)
    n = 100
    edges = R.ring.create(_nodes(n), R.metrics.random({"seed": 1337}))
    hoods = {}
    for r in range(n):
        k = rnd.randint(1, 9)
        hoods[r] = rnd.sample(range(n), k)
    save_grad_case("unbiased_ring100_p257", n, 257,
                   {"edges": {r: list(edges[r]) for r in edges}, "neighbourhoods": hoods},
                   "unbiased", seed=6)
    hoods8 = {r: rnd.sample(range(8), rnd.randint(1, 8)) for r in range(8)}
    save_grad_case("unbiased_n8_special_p16", 8, 16,
                   {"edges": {r: [(r + 1) % 8, (r - 1) % 8] for r in range(8)},
                    "neighbourhoods": hoods8}, "unbiased", seed=7, special=True)


def nonfinite_cases():
    """±inf / NaN / overflow / -0.0 / subnormals through clique topologies (the factored kernels'
    non-finite guard, include/niidmix.h) and a complete graph (big-clique and GEMM kernels)."""
    def sprinkle(x, n, members, gateways, cl):
        m0, m1 = members[0], members[1]
        x[m0, 0] = np.inf                          # a plain member: its clique reads +inf
        x[gateways[0], 1] = -np.inf                # a gateway: its clique and remote readers
        x[members[2], 2] = np.nan
        x[m0, 3] = np.inf; x[m1, 3] = -np.inf      # +inf and -inf in one clique -> NaN there
        x[cl[1][0], 4] = np.inf                    # another clique, column 4
        for r in cl[2][:5]:
            x[r, 5] = 3.4e38                       # 5 x 3.4e38: the clique SUM overflows, the
        x[:, 6] = -0.0                             # reference's w*x terms do not
        x[cl[3][0], 7] = 1e-45
        x[cl[3][1], 7] = -1e-45
        return x

    def gateways_of(edges, cl):
        clique_of = {r: i for i, c in enumerate(cl) for r in c}
        return [r for r in range(len(clique_of)) if any(clique_of[s] != clique_of[r] for s in edges[r])]

    e, cl = dcliques(300, 30, "fully-connected")
    g = torch.Generator().manual_seed(21)
    x = torch.randn(300, 64, generator=g).numpy()
    gw = gateways_of(e, cl)
    plain = [r for r in cl[0] if r not in gw]
    x = sprinkle(x, 300, plain, [r for r in cl[0] if r in gw] or gw, cl)
    save_case("nonfinite_dcliques300_fc_p64", e, 300, 64, cliques=cl, x=x)

    # removed clique edges (fractal interclique, 5 removed per clique): an inf at a node must not
    # reach the clique members whose edge to it was removed (the factored form's -c*x correction)
    e, cl = dcliques(200, 20, "fractal", remove=5)
    g = torch.Generator().manual_seed(22)
    x = torch.randn(200, 64, generator=g).numpy()
    gw = gateways_of(e, cl)
    x = sprinkle(x, 200, [r for r in cl[0] if r not in gw], [r for r in cl[0] if r in gw] or gw, cl)
    for c in cl[4:10]:                             # columns 8..13: one inf per clique 4..9
        x[c[0], 8 + cl.index(c) - 4] = np.inf if cl.index(c) % 2 else -np.inf
    save_case("nonfinite_dcliques200_fractal_rm5_p64", e, 200, 64, cliques=cl, x=x)

    # complete graph N=300 (one clique of 300 > 256: the one-pass big-clique kernel; dense W)
    edges = R.fc.create(_nodes(300))
    g = torch.Generator().manual_seed(23)
    x = torch.randn(300, 36, generator=g).numpy()
    x[5, 0] = np.inf; x[7, 1] = -np.inf; x[9, 2] = np.nan
    x[11, 3] = np.inf; x[12, 3] = -np.inf
    for r in range(0, 300, 60):
        x[r, 4] = 3.4e38
    x[:, 5] = -0.0
    save_case("nonfinite_fc300_p36", edges, 300, 36, x=x)


def consensus_cases():
    """Logger.log_consensus_distance (tools/simulate/logger.py:257-284) run on seeded models with a
    stub Logger instance (only .global_events is read); the event's numbers are stored."""
    import importlib
    logger = importlib.import_module("simulate.logger")
    for name, n, shapes, seed, offset in (("consensus_linear_n16", 16, [(10, 784), (10,)], 31, 0.0),
                                          ("consensus_n100_p4099", 100, [(4099,)], 32, 3.0)):
        p = sum(int(np.prod(s)) for s in shapes)
        g = torch.Generator().manual_seed(seed)
        x = (torch.randn(n, p, generator=g) + offset).numpy()
        nodes = []
        for rank in range(n):
            m = FlatModel(shapes)
            with torch.no_grad():
                off = 0
                for q in m.parameters():
                    k = q.numel()
                    q.copy_(torch.from_numpy(x[rank, off:off + k].copy()).view_as(q))
                    off += k
            nodes.append({"rank": rank, "model": m})
        with tempfile.TemporaryDirectory() as d:
            stub = types.SimpleNamespace(global_events=os.path.join(d, "global.jsonlines"))
            logger.Logger.log_consensus_distance(stub, {"nodes": nodes, "step": 7})
            ev = json.loads(open(stub.global_events).read().strip())
        gl = ev["distance_to_center"]["global"]
        np.savez_compressed(os.path.join(OUT, name + ".npz"), x=x,
                            shapes_json=np.asarray(json.dumps([list(s) for s in shapes])),
                            event_json=np.asarray(json.dumps(ev)),
                            stats=np.asarray([gl["avg"], gl["std"], gl["max"], gl["min"],
                                              ev["center"]["norm"]], np.float64))
        print(f"{name}: N={n} P={p} avg={gl['avg']:.6g} norm={ev['center']['norm']:.6g}")


def main():
    # 1) ring N=100, P=257 (odd tail), random metric, MH weights 1/3
    edges = R.ring.create(_nodes(100), R.metrics.random({"seed": 1337}))
    save_case("ring100_p257", edges, 100, 257, keep_json=True)

    # 2) d-cliques N=1000: 10 cliques of 100, fully-connected interclique (reference default),
    #    MH.  This is also the topology of the headline benchmark (BASELINE.json configs[2]).
    e, cl = dcliques(1000, 100, "fully-connected")
    save_case("dcliques1000_fc_p64", e, 1000, 64, cliques=cl)
    e, cl = dcliques(1000, 100, "smallworld")
    save_case("dcliques1000_smallworld_p16", e, 1000, 16, cliques=cl)
    e, cl = dcliques(1000, 100, "ring")
    save_case("dcliques1000_ring_p16", e, 1000, 16, cliques=cl)
    # reference default clique size (30), 10 cliques, FC interclique
    e, cl = dcliques(300, 30, "fully-connected")
    save_case("dcliques300_fc_p37", e, 300, 37, cliques=cl, keep_json=True)
    # clique edges removed (breaks the pure clique structure; exercises residual terms)
    e, cl = dcliques(200, 20, "fractal", remove=5)
    save_case("dcliques200_fractal_rm5_p40", e, 200, 40, cliques=cl, keep_json=True)

    # 3) fully-connected N=64, P=33
    edges = R.fc.create(_nodes(64))
    save_case("fc64_p33", edges, 64, 33, keep_json=True)

    # other sparse generators
    save_case("expander64_p48", R.expander.create(_nodes(64), {}), 64, 48, keep_json=True)
    save_case("grid49_p20", R.grid.create(_nodes(49), R.metrics.random({"seed": 1337})), 49, 20,
              keep_json=True)
    rg = R.random_graph.create(_nodes(50), {"topology": {"topology-seed": 1, "nb-neighbours": 5}})
    save_case("randomgraph50_p24", rg, 50, 24, keep_json=True)

    # 4) N=1 (W=[[1]], no edges) with signed zeros and non-finite values
    x1 = np.array([[0.0, -0.0, 1.5, -2.25, np.inf, -np.inf, np.nan, 1e-40, -1e-40, 3.0e38, -3.0e38]],
                  np.float32)
    save_case("n1_special", {0: []}, 1, x1.shape[1], x=x1, keep_json=True)
    #    N=2 ring (tools/tests/basic.sh shape: W = 1/2) with the linear MNIST model (7850 = [10,784]+[10])
    edges = R.ring.create(_nodes(2), R.metrics.random({"seed": 1337}))
    save_case("n2_ring_linear7850", edges, 2, 7850, shapes=[(10, 784), (10,)], keep_json=True)

    # 5) non-finite / signed zero propagation through neighbours
    edges = R.ring.create(_nodes(8), R.metrics.random({"seed": 1337}))
    g = torch.Generator().manual_seed(5)
    x = torch.randn(8, 16, generator=g).numpy()
    x[0, 0] = np.inf; x[1, 1] = -np.inf; x[2, 2] = np.nan; x[3, 3] = -0.0; x[3, 4] = 0.0
    x[4, 5] = -0.0; x[5, 5] = -0.0; x[6, 5] = -0.0; x[7, 5] = -0.0; x[0, 5] = -0.0
    x[1, 5] = -0.0; x[2, 5] = -0.0; x[3, 5] = -0.0
    x[:, 6] = -0.0
    x[5, 7] = np.inf; x[6, 7] = -np.inf
    x[4, 8] = 1e-45; x[4, 9] = 3.4e38; x[5, 9] = 3.4e38
    save_case("nonfinite_ring8_p16", edges, 8, 16, x=x, keep_json=True)

    # 6) uniform global average setup.model.average(models) (weights=None -> python-float 1/K),
    #    the primitive under d_sgd.init / logger consensus distance (model/__init__.py:15-25)
    K, P = 7, 100
    g = torch.Generator().manual_seed(3)
    xu = torch.randn(K, P, generator=g).numpy()
    models = []
    for k in range(K):
        m = FlatModel([(P,)])
        with torch.no_grad():
            m.ps[0].copy_(torch.from_numpy(xu[k]))
        models.append(m)
    c = R.model.average(models)
    yu = c.ps[0].detach().numpy()[None, :]
    np.savez_compressed(os.path.join(OUT, "uniform_avg_k7_p100.npz"), x=xu, y=yu)
    print("uniform_avg_k7_p100")


def logger_round_cases():
    """One reference mixing round (d_sgd.average, d_sgd.py:96-116) on seeded models, then what
    run.py's logging reads from the mixed models: Logger.log_consensus_distance
    (logger.py:257-284, stub instance) and Logger.state's global model setup.model.average
    (logger.py:112) over every node, over a subset of them (nodes_to_log) and over node 0 alone
    (fully-connected / sample).  Stored: x (pre-round), y (post-round), the CSR of W^T, cliques,
    the event and its stats, and the three averaged models flattened."""
    import importlib
    logger = importlib.import_module("simulate.logger")
    name, n, shapes, seed = "logger_round_dcliques300_p520", 300, [(10, 51), (10,)], 41
    p = sum(int(np.prod(s)) for s in shapes)
    e, cl = dcliques(n, 100, "fully-connected")
    weights = R.weights.compute_weights(_nodes(n), e, MH)
    _, loaded = _roundtrip(e, weights, cl)
    g = torch.Generator().manual_seed(seed)
    x = (torch.randn(n, p, generator=g) + 0.5).numpy()
    nodes = []
    for rank in range(n):
        m = FlatModel(shapes)
        with torch.no_grad():
            off = 0
            for q in m.parameters():
                k = q.numel()
                q.copy_(torch.from_numpy(x[rank, off:off + k].copy()).view_as(q))
                off += k
        nodes.append({"rank": rank, "model": m})
    R.d_sgd.average(nodes, loaded, {})
    y = _flat(nodes, "param")
    with tempfile.TemporaryDirectory() as d:
        stub = types.SimpleNamespace(global_events=os.path.join(d, "global.jsonlines"))
        logger.Logger.log_consensus_distance(stub, {"nodes": nodes, "step": 3})
        ev = json.loads(open(stub.global_events).read().strip())
    gl = ev["distance_to_center"]["global"]
    subset = list(range(3, 13)) + [150, 299]
    centers = {}
    for key, sel in (("center_all", list(range(n))), ("center_subset", subset),
                     ("center_node0", [0])):
        c = R.model.average([nodes[r]["model"] for r in sel])
        centers[key] = torch.cat([q.detach().reshape(-1) for q in c.parameters()]).numpy()
    row_ptr, col, val = _csr(loaded, n)
    np.savez_compressed(os.path.join(OUT, name + ".npz"), x=x, y=y, row_ptr=row_ptr, col=col,
                        val=val, shapes_json=np.asarray(json.dumps([list(s) for s in shapes])),
                        cliques_flat=np.asarray([r for c in cl for r in c], np.int32),
                        cliques_ptr=np.cumsum([0] + [len(c) for c in cl]).astype(np.int64),
                        event_json=np.asarray(json.dumps(ev)),
                        stats=np.asarray([gl["avg"], gl["std"], gl["max"], gl["min"],
                                          ev["center"]["norm"]], np.float64),
                        subset=np.asarray(subset, np.int64), **centers)
    print(f"{name}: N={n} P={p} avg={gl['avg']:.6g} norm={ev['center']['norm']:.6g}")


if __name__ == "__main__":
    if "--logger" in sys.argv:
        logger_round_cases()
    elif "--grad" in sys.argv:
        grad_cases()
    elif "--nonfinite" in sys.argv:
        nonfinite_cases()
    elif "--consensus" in sys.argv:
        consensus_cases()
    else:
        main()
        grad_cases()
        nonfinite_cases()
        consensus_cases()
        logger_round_cases()
