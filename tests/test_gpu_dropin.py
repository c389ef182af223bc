"""The drop-in plugin (niidmix.d_sgd / niidmix.model) on the GPU against the reference's golden
vectors: same call signatures as tools/simulate/algorithm/d_sgd.py and tools/setup/model, same bits."""
import json

import numpy as np
import pytest
import torch

from conftest import golden_cases, load_golden

pytestmark = pytest.mark.gpu


class FlatModel(torch.nn.Module):
    def __init__(self, shapes):
        super().__init__()
        self.ps = torch.nn.ParameterList([torch.nn.Parameter(torch.zeros(s)) for s in shapes])


def _nodes_and_topology(g):
    shapes = [tuple(s) for s in json.loads(str(g["shapes_json"]))]
    n = len(g["row_ptr"]) - 1
    W = torch.zeros(n, n)
    edges = {}
    for i in range(n):
        b, e = g["row_ptr"][i], g["row_ptr"][i + 1]
        edges[i] = g["col"][b + 1:e].tolist()
        W[torch.from_numpy(g["col"][b:e].astype(np.int64)), i] = torch.from_numpy(g["val"][b:e])
    nodes = []
    for i in range(n):
        m = FlatModel(shapes)
        off = 0
        with torch.no_grad():
            for q in m.parameters():
                k = q.numel()
                q.copy_(torch.from_numpy(g["x"][i, off:off + k].copy()).view_as(q))
                off += k
        nodes.append({"rank": i, "model": m})
    topo = {"edges": edges, "weights": W}
    if "cliques" in g:
        topo["cliques"] = g["cliques"]
    return nodes, topo


def _params_of(nodes):
    return np.stack([torch.cat([q.detach().reshape(-1) for q in nd["model"].parameters()]).numpy()
                     for nd in nodes])


@pytest.mark.parametrize("name", [n for n in golden_cases()])
def test_dsgd_average_bitwise(name, gpu, oracle_mod, monkeypatch):
    """niidmix.d_sgd.average(nodes, topology, params) == reference d_sgd.average, bit for bit,
    on the reference's golden vectors; a second round equals the oracle applied twice."""
    monkeypatch.setenv("NIIDMIX_WINDOW", "256")     # several column windows -> pipelined path
    from niidmix import d_sgd
    g = load_golden(name)
    nodes, topo = _nodes_and_topology(g)
    d_sgd.average(nodes, topo, {})
    y1 = _params_of(nodes)
    assert oracle_mod.bitwise_equal(y1, g["y"]), name
    d_sgd.average(nodes, topo, {})
    y2 = _params_of(nodes)
    ref2 = oracle_mod.mix_exact_c(g["y"], g["row_ptr"], g["col"], g["val"])
    assert oracle_mod.bitwise_equal(y2, ref2), name


def test_dsgd_average_fast_mode(gpu, oracle_mod, monkeypatch):
    monkeypatch.setenv("NIIDMIX_MODE", "fast")
    from niidmix import d_sgd
    g = load_golden("dcliques1000_fc_p64")
    nodes, topo = _nodes_and_topology(g)
    d_sgd.average(nodes, topo, {})
    bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
    ok, worst = oracle_mod.check_tolerance(_params_of(nodes), g["y"], bound, rtol=1e-5)
    assert ok, worst


def test_model_average_uniform_and_weighted(gpu):
    from niidmix import model as nm
    d = np.load(__import__("conftest").GOLDEN + "/uniform_avg_k7_p100.npz")
    models = []
    for k in range(d["x"].shape[0]):
        m = FlatModel([(100,)])
        with torch.no_grad():
            m.ps[0].copy_(torch.from_numpy(d["x"][k]))
        models.append(m)
    c = nm.average(models)
    assert np.array_equal(c.ps[0].detach().numpy().view(np.uint32), d["y"][0].view(np.uint32))
    # weighted with 0-d fp32 tensors, as d_sgd passes W[src, rank]
    w = [torch.tensor(0.25), torch.tensor(0.5), torch.tensor(0.25)]
    c = nm.average(models[:3], w)
    x = d["x"][:3]
    acc = x[0] * np.float32(0)
    for k in range(3):
        acc = acc + np.float32(w[k].item()) * x[k]
    assert np.array_equal(c.ps[0].detach().numpy().view(np.uint32), acc.view(np.uint32))


def test_consensus_distance(gpu):
    from niidmix import model as nm
    torch.manual_seed(0)
    models = [torch.nn.Linear(30, 10) for _ in range(9)]
    center, dist, norm = nm.consensus_distance(models)
    flat = torch.stack([torch.cat([q.detach().reshape(-1) for q in m.parameters()]) for m in models]).double()
    mean = flat.mean(0)
    ref = torch.sqrt(((flat - mean) ** 2).sum(1))
    np.testing.assert_allclose(dist, ref.numpy(), rtol=1e-6)
    np.testing.assert_allclose(norm, float(torch.sqrt((mean ** 2).sum())), rtol=1e-6)


def test_training_rounds_match_reference_loop(gpu, oracle_mod):
    """A few D-SGD rounds (local SGD on CPU + mixing) of the tools/tests/basic.sh shape (2-node ring,
    linear MNIST-shaped model, batch 125) with synthetic data: the GPU drop-in's parameters equal,
    bit for bit, those of the same rounds with the reference loop (oracle) doing the mixing."""
    from niidmix import d_sgd

    def run(mix):
        torch.manual_seed(1337)
        params = {"meta": {"log": "WARNING", "seed": 1337},
                  "model": {"input-size": 784},
                  "topology": {"name": "ring"},
                  "algorithm": {"learning-rate": 0.1, "learning-momentum": 0.0, "batch-size": 125,
                                "initial-averaging": True, "clique-gradient": False,
                                "unbiased-gradient": False}}

        class Net(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.fc = torch.nn.Linear(784, 10)

            def forward(self, x, params):
                return torch.nn.functional.log_softmax(self.fc(x.view(-1, 784)), dim=1)

        g = torch.Generator().manual_seed(7)
        data = [(torch.rand(1, 28, 28, generator=g), int(torch.randint(0, 10, (1,), generator=g)))
                for _ in range(1000)]
        nodes = []
        for r in range(2):
            mdl = Net()
            nodes.append({"rank": r, "epoch": 0, "train-set": data[r * 500:(r + 1) * 500],
                          "model": mdl, "optimizer": d_sgd.optimizer(mdl, params)})
        topo = {"edges": {0: [1], 1: [0]}, "weights": torch.tensor([[0.5, 0.5], [0.5, 0.5]])}
        orig, orig_rs = d_sgd.average, d_sgd._row_streamed
        if mix == "oracle":
            d_sgd.average = lambda nds, t, p: oracle_mod.reference_loop_average(nds, t)
            d_sgd._row_streamed = lambda p: False          # next_step calls gradient + average
        try:
            state, _, _ = d_sgd.init(nodes, topo, params)
            for _ in range(6):
                state, losses, done, active = d_sgd.next_step(state, params, None)
        finally:
            d_sgd.average, d_sgd._row_streamed = orig, orig_rs
        return [torch.cat([q.detach().reshape(-1) for q in n["model"].parameters()]).clone()
                for n in nodes]

    a = run("gpu")
    b = run("oracle")
    for u, v in zip(a, b):
        assert torch.equal(u, v)


@pytest.mark.parametrize("resident", ["1", "0", "paced"])
def test_training_rounds_deferred_writeback(resident, gpu, oracle_mod, monkeypatch):
    """The row-streamed round (rows go H2D right after their optimizer.step(), the mixed rows come
    back while the next round trains; niidmix.slab.ResidentRound) with deferred write-back, on a
    16-node ring of linear MNIST-shaped models over 7 rounds: every round's parameters equal, bit for
    bit, those of the reference loop doing the mixing (oracle) once synchronised.  next_step really
    returns early on rounds where run.py reads no model, and returns synchronised on the rounds
    where run.py's should_log (every 3rd step here) reads them; resident=0 runs the windowed
    engine (always synchronous)."""
    from niidmix import d_sgd
    if resident == "paced":                               # write-back 2 row blocks ahead
        monkeypatch.setenv("NIIDMIX_D2H_PACE", "2")
        resident = "1"
    monkeypatch.setenv("NIIDMIX_RESIDENT", resident)
    monkeypatch.setenv("NIIDMIX_ROW_BLOCK", "3")          # ragged last block (16 = 5 x 3 + 1)
    n = 16

    def run(mix, sync_each=True):
        torch.manual_seed(1337)
        params = {"meta": {"log": "WARNING", "seed": 1337}, "model": {"input-size": 784},
                  "topology": {"name": "ring"},
                  "logger": {"accuracy-logging-interval": 0, "accuracy-logging-interval-steps": 3,
                             "log-consensus-distance": False},
                  "algorithm": {"learning-rate": 0.1, "learning-momentum": 0.0, "batch-size": 25,
                                "initial-averaging": False, "clique-gradient": False,
                                "unbiased-gradient": False, "deferred-writeback": True}}

        class Net(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.fc = torch.nn.Linear(784, 10)

            def forward(self, x, params):
                return torch.nn.functional.log_softmax(self.fc(x.view(-1, 784)), dim=1)

        g = torch.Generator().manual_seed(7)
        data = [(torch.rand(1, 28, 28, generator=g), int(torch.randint(0, 10, (1,), generator=g)))
                for _ in range(n * 200)]
        nodes = []
        for r in range(n):
            mdl = Net()
            nodes.append({"rank": r, "epoch": 0, "train-set": data[r * 200:(r + 1) * 200],
                          "model": mdl, "optimizer": d_sgd.optimizer(mdl, params)})
        edges = {r: [(r + 1) % n, (r - 1) % n] if r % 2 else [(r - 1) % n, (r + 1) % n]
                 for r in range(n)}
        from niidmix.topology import mh_csr
        topo = {"edges": edges, "weights": torch.from_numpy(mh_csr(n, edges).dense())}
        orig, orig_rs = d_sgd.average, d_sgd._row_streamed
        if mix == "oracle":
            d_sgd.average = lambda nds, t, p: oracle_mod.reference_loop_average(nds, t)
            d_sgd._row_streamed = lambda p: False
        snaps, pend = [], []
        try:
            state, _, _ = d_sgd.init(nodes, topo, params)
            for _ in range(7):
                state, losses, done, active = d_sgd.next_step(state, params, None)
                eng = d_sgd.round_engine(nodes)
                pend.append(bool(eng is not None and eng.resident is not None and
                                 eng.resident.pending))
                if not sync_each:
                    continue                   # the next round's training waits row by row
                d_sgd.synchronize()
                snaps.append(torch.stack([torch.cat([q.detach().reshape(-1)
                                                     for q in nd["model"].parameters()])
                                          for nd in nodes]).clone())
            if not sync_each:
                d_sgd.synchronize()
                snaps.append(torch.stack([torch.cat([q.detach().reshape(-1)
                                                     for q in nd["model"].parameters()])
                                          for nd in nodes]).clone())
        finally:
            d_sgd.average, d_sgd._row_streamed = orig, orig_rs
        return snaps, pend

    a, pend = run("gpu")
    b, _ = run("oracle")
    for k, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u, v), k
    a7, _ = run("gpu", sync_each=False)
    assert torch.equal(a7[-1], b[-1])
    if resident == "1":
        # state['step'] after round k is k + 1: run.py reads models at steps 3 and 6
        assert pend == [True, True, False, True, True, False, True]
    else:
        assert not any(pend)


class RingNet(torch.nn.Module):
    """The linear MNIST-shaped node model (module level: picklable by reference)."""

    def __init__(self):
        super().__init__()
        self.fc = torch.nn.Linear(784, 10)

    def forward(self, x, params):
        return torch.nn.functional.log_softmax(self.fc(x.view(-1, 784)), dim=1)


def _handoff_child(conn):
    """torch.multiprocessing child: receive a model, send back its class name and weight."""
    m = conn.recv()
    conn.send((type(m).__name__, type(m).__module__, m.fc.weight.detach().numpy().copy()))
    conn.close()


def _ring_training_setup(n, seed=1337):
    from niidmix import d_sgd
    from niidmix.topology import mh_csr
    torch.manual_seed(seed)
    params = {"meta": {"log": "WARNING", "seed": seed}, "model": {"input-size": 784},
              "topology": {"name": "ring"},
              "logger": {"accuracy-logging-interval": 0, "accuracy-logging-interval-steps": 0,
                         "log-consensus-distance": False},
              "algorithm": {"learning-rate": 0.1, "learning-momentum": 0.0, "batch-size": 25,
                            "initial-averaging": False, "clique-gradient": False,
                            "unbiased-gradient": False, "deferred-writeback": True}}

    g = torch.Generator().manual_seed(7)
    data = [(torch.rand(1, 28, 28, generator=g), int(torch.randint(0, 10, (1,), generator=g)))
            for _ in range(n * 200)]
    nodes = []
    for r in range(n):
        mdl = RingNet()
        nodes.append({"rank": r, "epoch": 0, "train-set": data[r * 200:(r + 1) * 200],
                      "model": mdl, "optimizer": d_sgd.optimizer(mdl, params)})
    edges = {r: [(r + 1) % n, (r - 1) % n] for r in range(n)}
    topo = {"edges": edges, "weights": torch.from_numpy(mh_csr(n, edges).dense())}
    return params, nodes, topo


def test_read_guard_unpredicted_reader(gpu, oracle_mod, monkeypatch):
    """a driver that reads models on rounds _deferred_ok did NOT predict (no
    logging configured, so every round returns with the write-back in flight; the D2H is held back
    ~50 ms by NIIDMIX_D2H_DELAY_CYCLES) gets the MIXED parameters through state_dict(), forward(),
    parameters(), pickle, torch.save / torch.load of the whole model and a torch.multiprocessing
    hand-off (each returns the ORIGINAL class) -- niidmix.guard waits for the
    model's own rows -- bitwise the reference loop doing the mixing.  With the guard off (NIIDMIX_READ_GUARD=0) the same reads see stale rows,
    which shows the test can tell the two apart."""
    import io
    import pickle
    from niidmix import d_sgd, guard
    n, rounds = 16, 6
    monkeypatch.setenv("NIIDMIX_ROW_BLOCK", "3")
    monkeypatch.setenv("NIIDMIX_D2H_DELAY_CYCLES", str(100_000_000))

    def run(mix, guard_on):
        monkeypatch.setenv("NIIDMIX_READ_GUARD", "1" if guard_on else "0")
        params, nodes, topo = _ring_training_setup(n)
        orig, orig_rs = d_sgd.average, d_sgd._row_streamed
        if mix == "oracle":
            d_sgd.average = lambda nds, t, p: oracle_mod.reference_loop_average(nds, t)
            d_sgd._row_streamed = lambda p: False
        seen, pend = [], []
        try:
            state, _, _ = d_sgd.init(nodes, topo, params)
            for k in range(rounds):
                state, _, _, _ = d_sgd.next_step(state, params, None)
                eng = d_sgd.round_engine(nodes)
                pend.append(bool(eng is not None and eng.resident is not None and
                                 eng.resident.pending))
                # the unpredicted reader, right after next_step: one entry point per round
                r = (5 * k + 3) % n
                mdl = nodes[r]["model"]
                if k == 0:
                    w = mdl.state_dict()["fc.weight"].clone()
                elif k == 1:
                    w = next(mdl.parameters()).detach().clone()
                elif k == 2:
                    mdl.forward(torch.zeros(1, 784), params)
                    w = mdl.fc.weight.detach().clone()
                elif k == 3:                          # pickle
                    c = pickle.loads(pickle.dumps(mdl))
                    assert type(c) is RingNet
                    w = c.fc.weight.detach().clone()
                elif k == 4:                          # a whole-model checkpoint
                    buf = io.BytesIO()
                    torch.save(mdl, buf)
                    buf.seek(0)
                    c = torch.load(buf, weights_only=False)   # our own file
                    assert type(c) is RingNet and buf.getbuffer().nbytes < 64 << 10
                    w = c.fc.weight.detach().clone()
                else:                                 # a torch.multiprocessing hand-off
                    ctx = torch.multiprocessing.get_context("spawn")
                    a, b = ctx.Pipe()
                    pr = ctx.Process(target=_handoff_child, args=(b,))
                    pr.start()
                    a.send(mdl)
                    name, mod, w = a.recv()
                    w = torch.from_numpy(w)
                    pr.join(60)
                    assert pr.exitcode == 0 and (name, mod) == ("RingNet", RingNet.__module__)
                seen.append(w)
                d_sgd.synchronize()
        finally:
            d_sgd.average, d_sgd._row_streamed = orig, orig_rs
        return seen, pend

    ref, _ = run("oracle", True)
    w0 = guard.stats["waits"]
    got, pend = run("gpu", True)
    assert all(pend), pend                        # every round really returned early
    assert guard.stats["waits"] > w0
    for k, (u, v) in enumerate(zip(got, ref)):
        assert torch.equal(u, v), k
    stale, pend = run("gpu", False)
    assert all(pend)
    assert any(not torch.equal(u, v) for u, v in zip(stale, ref))


@pytest.mark.parametrize("stripes", [1, 3])
def test_resident_device_step_resident_params(stripes, gpu, oracle_mod):
    """niidmix.slab.ResidentRound with the plain device step (fused_op without gradient averaging)
    over 1 and 3 column stripes of one GPU: round 0 sends parameters and gradients, rounds 1-3 only
    gradients (begin(resident_in0=True): the last round's output buffer becomes the input); every
    round bitwise torch's CPU SGD step (p.add_(g, alpha=-lr)) followed by the C oracle's mixing,
    with -0.0 gradients and parameters planted."""
    from niidmix import ops
    from niidmix.slab import ResidentRound, fused_op
    from niidmix.topology import mh_csr
    n, p, lr = 12, 3000, 0.05
    edges = {r: [(r + 1) % n, (r - 1) % n, (r + 5) % n] for r in range(n)}
    csr = mh_csr(n, {r: sorted(set(e)) for r, e in edges.items()})
    mixer = ops.Mixer(csr=csr, device=gpu)
    gen = torch.Generator().manual_seed(stripes)
    host_p = torch.randn(n, p, generator=gen).pin_memory()
    host_p[::4, ::5] = -0.0
    host_g = torch.empty(n, p).pin_memory()
    rr = ResidentRound(lambda dev, part: fused_op(dev, part, None, list(range(n)), lr, mixer),
                       n, p, [gpu] * stripes, block=4, align=256, n_in=2, n_out=1)
    assert len(rr.parts) == stripes
    ref = host_p.clone()
    for k in range(4):
        g = torch.randn(n, p, generator=gen)
        g[::3, ::7] = -0.0
        g[1::3, ::11] = 0.0
        host_g.copy_(g)
        if k == 0:
            rr.begin(host_p, host_g, outs=(host_p,))
        else:
            assert rr.current()
            rr.begin(None, host_g, outs=(host_p,), resident_in0=True)
        for i in range(n):
            rr.row_ready(i)
        rr.mix("exact")
        rr.wait_all()
        with torch.no_grad():
            ref.add_(g, alpha=-lr)
        ref = torch.from_numpy(oracle_mod.mix_exact_c(ref.numpy(), csr.row_ptr, csr.col, csr.val))
        assert oracle_mod.bitwise_equal(host_p.numpy(), ref.numpy()), k


@pytest.mark.parametrize("step", ["device", "cpu"])
def test_training_rounds_device_step(step, gpu, oracle_mod, monkeypatch):
    """the plain round with its optimizer step on the device (_FusedEngine(plain):
    gradient rows go up after each backward, filled with -0.0 first so that backward's in-place
    accumulate keeps every gradient's bits; p += (-lr) g on the resident parameters; mixing).  16
    nodes, 7 rounds, with -0.0 weights and inputs whose zero pixels make +-0 gradients (where a +0
    fill would differ): every round bitwise the reference loop (CPU SGD, then the reference mixing
    loop).  The parameters stay on the device between rounds -- uploaded only in the first round,
    after a guarded write (load_state_dict, round 3) and after an in-place write through a
    parameter (p.add_ under no_grad, round 5; its version counter).  step=cpu: NIIDMIX_DEVICE_STEP=0
    (the CPU steps; rows go up after optimizer.step())."""
    from niidmix import d_sgd
    monkeypatch.setenv("NIIDMIX_DEVICE_STEP", "1" if step == "device" else "0")
    monkeypatch.setenv("NIIDMIX_ROW_BLOCK", "3")
    n = 16

    def run(mix):
        torch.manual_seed(1337)
        params = {"meta": {"log": "WARNING", "seed": 1337}, "model": {"input-size": 784},
                  "topology": {"name": "ring"},
                  "logger": {"accuracy-logging-interval": 0, "accuracy-logging-interval-steps": 0,
                             "log-consensus-distance": False},
                  "algorithm": {"learning-rate": 0.1, "learning-momentum": 0.0, "batch-size": 25,
                                "initial-averaging": False, "clique-gradient": False,
                                "unbiased-gradient": False, "deferred-writeback": True}}
        g = torch.Generator().manual_seed(8)
        data = []
        for _ in range(n * 200):
            img = torch.rand(1, 28, 28, generator=g)
            img[:, :, :6] = 0.0                       # zero pixels: +-0 weight gradients
            data.append((img, int(torch.randint(0, 10, (1,), generator=g))))
        nodes = []
        for r in range(n):
            mdl = RingNet()
            with torch.no_grad():
                mdl.fc.weight[:, :40] = -0.0          # -0.0 parameters on the zero pixels' columns
                mdl.fc.bias[r % 10] = -0.0
            nodes.append({"rank": r, "epoch": 0, "train-set": data[r * 200:(r + 1) * 200],
                          "model": mdl, "optimizer": d_sgd.optimizer(mdl, params)})
        edges = {r: [(r + 1) % n, (r - 1) % n] for r in range(n)}
        from niidmix.topology import mh_csr
        topo = {"edges": edges, "weights": torch.from_numpy(mh_csr(n, edges).dense())}
        orig, orig_rs = d_sgd.average, d_sgd._row_streamed
        if mix == "oracle":
            d_sgd.average = lambda nds, t, p: oracle_mod.reference_loop_average(nds, t)
            d_sgd._row_streamed = lambda p: False
        snaps, eng = [], None
        try:
            state, _, _ = d_sgd.init(nodes, topo, params)
            for k in range(7):
                if k == 3:
                    nodes[5]["model"].load_state_dict(nodes[5]["model"].state_dict())
                if k == 5:
                    with torch.no_grad():
                        nodes[2]["model"].fc.bias.add_(0.5)
                state, _, _, _ = d_sgd.next_step(state, params, None)
                eng = d_sgd.round_engine(nodes) if mix == "gpu" else None
                d_sgd.synchronize()
                snaps.append(torch.stack([torch.cat([q.detach().reshape(-1)
                                                     for q in nd["model"].parameters()])
                                          for nd in nodes]).clone())
        finally:
            d_sgd.average, d_sgd._row_streamed = orig, orig_rs
        return snaps, eng

    a, eng = run("gpu")
    b, _ = run("oracle")
    assert any((torch.signbit(u) & (u == 0)).any() for u in b)   # -0.0 survives in the reference
    for k, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u.view(torch.int32), v.view(torch.int32)), k
    if step == "device":
        assert getattr(eng, "plain", False) and eng.param_uploads == 3, eng.param_uploads
    else:
        assert not getattr(eng, "plain", False)


@pytest.mark.parametrize("alg",["clique", "unbiased"])
def test_training_rounds_gradient_averaging(alg, gpu, oracle_mod, monkeypatch):
    """Rounds with --clique-gradient / --unbiased-gradient (linear model, 4 nodes): the drop-in's
    fused device round (gradient mean + SGD step + mixing) and its unfused GPU path (gradient
    slab, then the mixing slab) give the same parameters, bit for bit, as the reference's CPU
    loops (average_gradients / update_gradients / optimizer.step, then the reference mixing loop)."""
    from niidmix import d_sgd

    def cpu_gradient(nds, t, p):                  # d_sgd.py:47-94 restated with torch CPU ops
        with torch.no_grad():
            if p["algorithm"]["clique-gradient"]:
                oracle_mod.reference_loop_clique_gradient(nds, t["cliques"])
                stepped = [r for c in t["cliques"] for r in c]
            else:
                hoods = t["neighbourhoods"]
                grads = {n["rank"]: d_sgd.average_gradients([nds[q]["model"] for q in hoods[n["rank"]]])
                         for n in nds}
                for n in nds:
                    d_sgd.update_gradients([n["model"]], grads[n["rank"]])
                stepped = [n["rank"] for n in nds]
        for r in stepped:
            nds[r]["optimizer"].step()

    def run(path):
        monkeypatch.setenv("NIIDMIX_FUSED", "1" if path.startswith("fused") else "0")
        monkeypatch.setenv("NIIDMIX_ROW_BLOCK", "3")      # blocks of 3 rows: a ragged last block
        torch.manual_seed(1337)
        params = {"meta": {"log": "WARNING", "seed": 1337}, "model": {"input-size": 784},
                  "topology": {"name": "d-cliques", "remove-clique-edges": 0},
                  "logger": {"accuracy-logging-interval": 0, "accuracy-logging-interval-steps": 0,
                             "log-consensus-distance": False},
                  "algorithm": {"learning-rate": 0.1, "learning-momentum": 0.0, "batch-size": 50,
                                "initial-averaging": False, "clique-gradient": alg == "clique",
                                "unbiased-gradient": alg == "unbiased",
                                "deferred-writeback": path == "fused_deferred"}}

        class Net(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.fc = torch.nn.Linear(784, 10)

            def forward(self, x, params):
                return torch.nn.functional.log_softmax(self.fc(x.view(-1, 784)), dim=1)

        g = torch.Generator().manual_seed(11)
        data = [(torch.rand(1, 28, 28, generator=g), int(torch.randint(0, 10, (1,), generator=g)))
                for _ in range(800)]
        nodes = []
        for r in range(4):
            mdl = Net()
            nodes.append({"rank": r, "epoch": 0, "train-set": data[r * 200:(r + 1) * 200],
                          "model": mdl, "optimizer": d_sgd.optimizer(mdl, params)})
        w = torch.tensor([[0.5, 0.25, 0.0, 0.25], [0.25, 0.5, 0.25, 0.0],
                          [0.0, 0.25, 0.5, 0.25], [0.25, 0.0, 0.25, 0.5]])
        topo = {"edges": {0: [1, 3], 1: [0, 2], 2: [3, 1], 3: [2, 0]}, "weights": w,
                "cliques": [[1, 0], [2, 3]],
                "neighbourhoods": {0: [0, 2], 1: [3, 1, 0], 2: [2], 3: [1, 3]}}
        orig_g, orig_a = d_sgd.gradient, d_sgd.average
        if path == "oracle":
            d_sgd.gradient = cpu_gradient
            d_sgd.average = lambda nds, t, p: oracle_mod.reference_loop_average(nds, t)
        try:
            state, _, _ = d_sgd.init(nodes, topo, params)
            pend = []
            for _ in range(5):
                state, losses, done, active = d_sgd.next_step(state, params, None)
                eng = d_sgd.round_engine(nodes)
                pend.append(bool(eng is not None and eng.resident is not None and
                                 eng.resident.pending))
            d_sgd.synchronize()
        finally:
            d_sgd.gradient, d_sgd.average = orig_g, orig_a
        if path == "fused_deferred":
            assert all(pend), pend                 # next_step returned before the write-back
        elif path == "fused":
            assert not any(pend), pend
        return [(torch.cat([q.detach().reshape(-1) for q in n["model"].parameters()]).clone(),
                 torch.cat([q.grad.detach().reshape(-1) for q in n["model"].parameters()]).clone())
                for n in nodes]

    fused, unfused, ref = run("fused"), run("unfused"), run("oracle")
    deferred = run("fused_deferred")
    for u, v, r, d in zip(fused, unfused, ref, deferred):
        assert torch.equal(v[0], r[0]) and torch.equal(v[1], r[1])
        assert torch.equal(u[0], r[0])
        # the fused round writes the averaged gradients back where the reference leaves them
        assert torch.equal(u[1], r[1])
        assert torch.equal(d[0], r[0]) and torch.equal(d[1], r[1])


def test_sgd_step_rows_matches_torch_cpu_sgd(gpu):
    """k_sgd_step_rows == torch.optim.SGD(momentum=0).step on the CPU, bit for bit (ATen's CPU
    add_(g, alpha=-lr) is one fma with an fp32 alpha), on the listed rows only."""
    from niidmix import ops
    gen = torch.Generator().manual_seed(5)
    p = torch.randn(6, 1003, generator=gen)
    g = torch.randn(6, 1003, generator=gen)
    rows = [0, 2, 5]
    ref = p.clone()
    for r in rows:
        q = torch.nn.Parameter(ref[r].clone())
        q.grad = g[r].clone()
        torch.optim.SGD([q], lr=0.07).step()
        ref[r] = q.detach()
    pd = p.to(gpu)
    ops.sgd_step_rows(pd, g.to(gpu), torch.tensor(rows, dtype=torch.int32, device=gpu), -0.07)
    assert torch.equal(pd.cpu(), ref)


def _cpu_consensus_statistics(models):
    """CPU restatement of the reference's arithmetic (logger.py:257-284): fp32 center, per-tensor
    fp32 squared sums, sqrt of their sum."""
    import math
    with torch.no_grad():
        flat = [torch.cat([q.detach().reshape(-1) for q in m.parameters()]) for m in models]
        w = float(1. / len(flat))
        center = flat[0] * 0
        for f in flat:
            center = center + w * f
        d = [math.sqrt(float(torch.sum((center - f) ** 2))) for f in flat]
        return d, math.sqrt(float(torch.sum(center ** 2)))


def test_consensus_distance_event(gpu, tmp_path):
    """The GPU consensus-distance event has the reference's schema and statistics."""
    from niidmix import logger as nl
    torch.manual_seed(3)
    nodes = [{"rank": i, "model": torch.nn.Linear(50, 7)} for i in range(12)]
    ev = nl.consensus_distance_event({"nodes": nodes, "step": 4})
    d, norm = _cpu_consensus_statistics([n["model"] for n in nodes])
    import statistics
    g = ev["distance_to_center"]["global"]
    np.testing.assert_allclose(g["avg"], statistics.mean(d), rtol=1e-5)
    np.testing.assert_allclose(g["max"], max(d), rtol=1e-5)
    np.testing.assert_allclose(g["min"], min(d), rtol=1e-5)
    np.testing.assert_allclose(g["std"], statistics.stdev(d), rtol=1e-4)
    np.testing.assert_allclose(ev["center"]["norm"], norm, rtol=1e-5)
    assert ev["type"] == "consensus-distance" and ev["step"] == 4

    class L:
        global_events = str(tmp_path / "global.jsonlines")
    nl.install(L)
    L().log_consensus_distance({"nodes": nodes, "step": 5})
    import json
    line = json.loads(open(L.global_events).read().strip())
    assert line["step"] == 5 and "distance_to_center" in line


@pytest.mark.parametrize("stripes", [2, 3])
def test_multi_device_round_bitwise(stripes, gpu, oracle_mod):
    """The single-process multi-GPU drop-in round (niidmix.slab.MultiDeviceRound: one column stripe
    per device, each with its own streams and window pipeline, no exchange) with every stripe
    mapped to the one GPU of this box: bitwise the single-device round, exact and fast mode, and
    the exact round bitwise the reference fixture (d-cliques N=300)."""
    from niidmix import ops
    from niidmix.slab import MultiDeviceRound, SlabMixer
    g = load_golden("dcliques300_fc_p37")
    csr = ops.csr_from_numpy(g["row_ptr"], g["col"], g["val"])
    m = ops.Mixer(csr=csr, cliques=g["cliques"], device=gpu)
    n, p = 300, 5000
    gen = torch.Generator().manual_seed(stripes)
    x = torch.randn(n, p, generator=gen)
    for mode in ("exact", "fast"):
        h1 = x.clone().pin_memory()
        SlabMixer(m, n, p, gpu, window=1024).mix(h1, mode=mode)
        hk = x.clone().pin_memory()
        mr = MultiDeviceRound(lambda dev, nn, cols: SlabMixer(m.to(dev), nn, cols, dev, window=1024),
                              n, p, [gpu] * stripes, align=256)
        assert len([r for r in mr.runners if r is not None]) == stripes
        mr.run(hk, mode=mode)
        assert torch.equal(hk, h1), mode
    h = torch.from_numpy(g["x"]).clone().pin_memory()
    mr = MultiDeviceRound(lambda dev, nn, cols: SlabMixer(m.to(dev), nn, cols, dev), 300, 37,
                          [gpu] * stripes, align=16)
    mr.run(h, mode="exact")
    assert oracle_mod.bitwise_equal(h.numpy(), g["y"])


def test_multi_device_fused_round_bitwise(gpu):
    """The fused gradient + step + mixing round over 3 stripes on one GPU equals one device's."""
    from niidmix import ops
    from niidmix.gradient import GradMean, build_grad_plan
    from niidmix.slab import FusedRoundRunner, MultiDeviceRound
    g = load_golden("dcliques300_fc_p37")
    csr = ops.csr_from_numpy(g["row_ptr"], g["col"], g["val"])
    m = ops.Mixer(csr=csr, cliques=g["cliques"], device=gpu)
    plan = build_grad_plan(300, {"cliques": g["cliques"], "edges": csr.edges()},
                           {"algorithm": {"clique-gradient": True}})
    n, p = 300, 4100
    gen = torch.Generator().manual_seed(9)
    xp, xg = torch.randn(n, p, generator=gen), torch.randn(n, p, generator=gen)

    def make(dev, nn, cols):
        return FusedRoundRunner(GradMean(plan, dev), plan.stepped, 0.1, m.to(dev), nn, cols, dev,
                                window=1024)
    hp1, hg1 = xp.clone().pin_memory(), xg.clone().pin_memory()
    make(gpu, n, p).run(hp1, hg1, mode="exact")
    hp3, hg3 = xp.clone().pin_memory(), xg.clone().pin_memory()
    MultiDeviceRound(make, n, p, [gpu] * 3, align=256).run(hp3, hg3, mode="exact")
    assert torch.equal(hp1, hp3) and torch.equal(hg1, hg3)
    assert not torch.equal(hg1, xg)          # the averaged gradients were written back


def test_randomize_keeps_slab(gpu, oracle_mod):
    """--randomize: a new graph every round (d_sgd.py:223-234).  The drop-in rebuilds only the
    mixing operator for the same nodes (the pinned slab and the device window buffers stay), and
    each round is bit-identical to the reference loop on that round's graph."""
    from niidmix import d_sgd, generate
    n, p = 40, 300
    torch.manual_seed(2)
    nodes = [{"rank": r, "model": torch.nn.Linear(p - 1, 1)} for r in range(n)]
    params = {"algorithm": {"mixing-mode": "exact"},
              "topology": {"name": "random-graph", "nb-neighbours": 4, "topology-seed": 3,
                           "weights": "metropolis-hasting", "randomize": True}}
    topo = d_sgd.randomized_topology(nodes, params, None)
    slab = None
    for _ in range(3):
        before = np.stack([torch.cat([q.detach().reshape(-1) for q in nd["model"].parameters()]).numpy()
                           for nd in nodes])
        d_sgd.average(nodes, topo, params)
        eng = next(iter(d_sgd._engines.values()))
        if slab is None:
            slab = eng.slab
        assert eng.slab is slab                       # same pinned slab every round
        csr = topo["csr"]
        after = np.stack([torch.cat([q.detach().reshape(-1) for q in nd["model"].parameters()]).numpy()
                          for nd in nodes])
        ref = oracle_mod.mix_exact_c(before, csr.row_ptr, csr.col, csr.val)
        assert oracle_mod.bitwise_equal(after, ref)
        params["topology"]["topology-seed"] += 1
        topo = d_sgd.randomized_topology(nodes, params, None)


def test_randomize_training_rounds_device_step(gpu, oracle_mod):
    """--randomize through next_step with the device step (the plain round's default): a new graph
    every round (d_sgd.py:223-234) swaps only the mixing operator of the resident engine
    (_FusedEngine.set_topology): the same engine, slab and resident parameters every round (one
    parameter upload), and every round bitwise the reference loop (CPU SGD + the reference mixing
    on that round's graph)."""
    from niidmix import d_sgd
    n = 24

    def run(mix):
        params, nodes, _ = _ring_training_setup(n, seed=5)
        params["topology"] = {"name": "random-graph", "nb-neighbours": 4, "topology-seed": 3,
                              "weights": "metropolis-hasting", "randomize": True}
        topo = d_sgd.randomized_topology(nodes, params, None)
        orig, orig_rs = d_sgd.average, d_sgd._row_streamed
        if mix == "oracle":
            d_sgd.average = lambda nds, t, p: oracle_mod.reference_loop_average(nds, t)
            d_sgd._row_streamed = lambda p: False
        snaps, engs = [], []
        try:
            state, _, _ = d_sgd.init(nodes, topo, params)
            for _ in range(5):
                state, _, _, _ = d_sgd.next_step(state, params, None)
                engs.append(d_sgd.round_engine(nodes))
                d_sgd.synchronize()
                snaps.append(torch.stack([torch.cat([q.detach().reshape(-1)
                                                     for q in nd["model"].parameters()])
                                          for nd in nodes]).clone())
        finally:
            d_sgd.average, d_sgd._row_streamed = orig, orig_rs
        return snaps, engs

    a, engs = run("gpu")
    b, _ = run("oracle")
    for k, (u, v) in enumerate(zip(a, b)):
        assert torch.equal(u.view(torch.int32), v.view(torch.int32)), k
    assert all(e is engs[0] for e in engs) and engs[0].plain and engs[0].param_uploads == 1


@pytest.mark.parametrize("mode", ["exact", "fast"])
def test_sparse_topology_plugin_round(mode, gpu, oracle_mod, tmp_path, monkeypatch):
    """Sparse ingestion under the unchanged run.py: a rundir written by niidmix.sparse_topology,
    read by the reference loader's restatement (load_file; run.py:92-93 -> setup.topology.load,
    so 'weights' is an EMPTY tensor), mixed by the plugin's average(): exact mode bit for bit the
    reference's dense-W round (golden dcliques300_fc_p37), fast mode within the tolerance."""
    import os
    from niidmix import d_sgd, sparse_topology, topology
    (tmp_path / "nodes.json").write_text(json.dumps([{"rank": r} for r in range(300)]))
    (tmp_path / "params.json").write_text(json.dumps({"meta": {"seed": 1337, "log": "WARNING"},
                                                      "dataset": {"nb-classes": 10}}))
    sparse_topology.main(["d-cliques", "--rundir", str(tmp_path), "--max-clique-size", "30"])
    topo = topology.load_file(os.path.join(str(tmp_path), "topology.json"))
    assert topo["weights"].numel() == 0
    g = load_golden("dcliques300_fc_p37")
    nodes, _ = _nodes_and_topology(g)
    monkeypatch.setenv("NIIDMIX_MODE", mode)
    d_sgd.average(nodes, topo, {})
    y = _params_of(nodes)
    if mode == "exact":
        assert oracle_mod.bitwise_equal(y, g["y"])
    else:
        bound = oracle_mod.condition_bound(g["x"], g["row_ptr"], g["col"], g["val"])
        ok, worst = oracle_mod.check_tolerance(y, g["y"], bound, rtol=1e-5)
        assert ok, worst


def _ref_sample_round(all_nodes, active):
    """The reference's 'sample' branch after the optimizer steps (d_sgd.py:240-250), restated with
    torch CPU ops: setup.model.average (deepcopy, mul_(0), add_(w*p); model/__init__.py:15-25)
    then update_models over every node (p.mul_(0.); p.add_(new); d_sgd.py:29-35)."""
    import copy
    with torch.no_grad():
        w = [1 / len(active) for _ in active]
        center = copy.deepcopy(active[0]["model"])
        for c in center.parameters():
            c.mul_(0)
        for n, wi in zip(active, w):
            for c, q in zip(center.parameters(), n["model"].parameters()):
                c.add_(wi * q)
        for n in all_nodes:
            for q, c in zip(n["model"].parameters(), center.parameters()):
                q.mul_(0.)
                q.add_(c)


def test_sample_average_bitwise(gpu, monkeypatch):
    """niidmix.d_sgd.sample_average (the slab-level 'sample' round: average of the active rows,
    then update_models of EVERY row on the GPU) == the reference's CPU arithmetic, bit for bit,
    with inf / NaN / -0.0 in the models (a non-finite row becomes NaN, zero sign rules) and the
    slab streamed in several column windows."""
    monkeypatch.setenv("NIIDMIX_WINDOW", "256")
    from niidmix import d_sgd
    torch.manual_seed(4)

    def make():
        torch.manual_seed(4)
        nodes = [{"rank": r, "model": torch.nn.Linear(60, 9)} for r in range(23)]
        with torch.no_grad():
            nodes[3]["model"].weight[0, 0] = float("inf")
            nodes[5]["model"].weight[1, 1] = float("nan")
            nodes[7]["model"].bias[2] = -0.0
            for n in nodes:
                n["model"].bias[4] = 0.0 if n["rank"] % 2 else -0.0
        return nodes
    a, b = make(), make()
    for pick in ([0, 4, 9, 17], [3, 1], [22, 7, 5, 0, 11]):
        d_sgd.sample_average(a, [a[i] for i in pick])
        _ref_sample_round(b, [b[i] for i in pick])
        for u, v in zip(_params_of(a), _params_of(b)):
            assert np.array_equal(np.isnan(u), np.isnan(v))
            m = ~np.isnan(v)
            assert np.array_equal(u[m].view(np.uint32), v[m].view(np.uint32))


def test_sample_topology_training_rounds(gpu):
    """Whole 'sample' topology rounds through niidmix.d_sgd.next_step (random-with-overlap
    sampling, local SGD on CPU, the GPU average + broadcast) equal the same rounds with the
    reference's CPU branch, bit for bit."""
    from niidmix import d_sgd

    def run(mode):
        torch.manual_seed(1337)
        d_sgd._sample_cache.clear()
        params = {"meta": {"log": "WARNING", "seed": 1337}, "model": {"input-size": 784},
                  "topology": {"name": "sample", "sample-method": "random-with-overlap",
                               "sample-size": 3, "sample-overlap": 1},
                  "algorithm": {"learning-rate": 0.1, "learning-momentum": 0.0, "batch-size": 20,
                                "initial-averaging": False, "clique-gradient": False,
                                "unbiased-gradient": False}}

        class Net(torch.nn.Module):
            def __init__(self):
                super().__init__()
                self.fc = torch.nn.Linear(784, 10)

            def forward(self, x, params):
                return torch.nn.functional.log_softmax(self.fc(x.view(-1, 784)), dim=1)

        g = torch.Generator().manual_seed(9)
        data = [(torch.rand(1, 28, 28, generator=g), int(torch.randint(0, 10, (1,), generator=g)))
                for _ in range(600)]
        nodes = []
        for r in range(6):
            mdl = Net()
            nodes.append({"rank": r, "epoch": 0, "train-set": data[r * 100:(r + 1) * 100],
                          "model": mdl, "optimizer": d_sgd.optimizer(mdl, params)})
        orig = d_sgd.sample_average
        if mode == "cpu":
            d_sgd.sample_average = _ref_sample_round
        try:
            state, _, _ = d_sgd.init(nodes, {"edges": {}, "weights": torch.tensor([])}, params)
            for _ in range(5):
                state, losses, done, active = d_sgd.next_step(state, params, None)
        finally:
            d_sgd.sample_average = orig
        return [torch.cat([q.detach().reshape(-1) for q in n["model"].parameters()]).clone()
                for n in nodes]

    for u, v in zip(run("gpu"), run("cpu")):
        assert torch.equal(u, v)


def _fake_reference_modules(monkeypatch, tmp_path):
    """Stand-ins for the modules run.py imports before the plugin (simulate.logger, setup.model):
    /root/reference is not on the GPU box, so these hold the reference's CPU restatement; the
    plugin's init must route both through the GPU (niidmix.logger.install_hooks)."""
    import sys
    import types
    lg = types.ModuleType("simulate.logger")

    class Logger:
        def __init__(self):
            self.global_events = str(tmp_path / "global.jsonlines")

        def log_consensus_distance(self, state):          # replaced by the plugin's init
            raise AssertionError("CPU consensus distance ran")
    lg.Logger = Logger
    sm = types.ModuleType("setup.model")

    def cpu_average(models, weights=None):
        raise AssertionError("CPU setup.model.average ran")
    sm.average = cpu_average
    monkeypatch.setitem(sys.modules, "simulate.logger", lg)
    monkeypatch.setitem(sys.modules, "setup.model", sm)
    return lg, sm


def test_logger_hooks_read_resident_slab(gpu, monkeypatch, tmp_path):
    """VERDICT r04 What's missing #2: the unchanged driver's logging after a plugin round.  With
    the reference's modules loaded, niidmix.d_sgd.init routes Logger.log_consensus_distance and
    (log-global-model-accuracy) setup.model.average through the GPU, reading the RESIDENT output
    slab of the round (no H2D).  Checked against tests/golden/logger_round_dcliques300_p520, made
    by the reference itself (make_golden.py --logger): the round bitwise, the consensus event's
    avg/max/min/norm within 1e-5 and std within 1e-4 relative, the global models (all nodes, a
    nodes_to_log subset, node 0 alone) bitwise."""
    from niidmix import d_sgd, guard
    from niidmix import logger as nl
    g = load_golden("logger_round_dcliques300_p520")
    lg, sm = _fake_reference_modules(monkeypatch, tmp_path)
    nodes, topo = _nodes_and_topology(g)
    for nd in nodes:
        nd["train-set"] = [(torch.zeros(1), 0)]           # init() builds a loader per node
    params = {"meta": {"log": "WARNING"}, "topology": {"name": "d-cliques"},
              "logger": {"log-consensus-distance": True, "log-global-model-accuracy": True},
              "algorithm": {"initial-averaging": False, "batch-size": 8}}
    state, _, _ = d_sgd.init(nodes, topo, params)
    assert lg.Logger.log_consensus_distance is nl.log_consensus_distance
    assert sm.average is nl.average
    d_sgd.average(nodes, topo, params)                      # one resident round
    eng = d_sgd._engines[id(nodes)]
    assert eng.resident is not None and eng.resident.fresh
    assert oracle_bitwise(_params_of(nodes), g["y"])
    state["step"] = 3
    lg.Logger().log_consensus_distance(state)
    assert nl.last_source["consensus"] == "resident"
    ev = json.loads(open(tmp_path / "global.jsonlines").read().strip().splitlines()[-1])
    ref = json.loads(str(g["event_json"]))
    gl, rg = ev["distance_to_center"]["global"], ref["distance_to_center"]["global"]
    for k in ("avg", "max", "min"):
        np.testing.assert_allclose(gl[k], rg[k], rtol=1e-5)
    np.testing.assert_allclose(gl["std"], rg["std"], rtol=1e-4)
    np.testing.assert_allclose(ev["center"]["norm"], ref["center"]["norm"], rtol=1e-5)
    assert ev["type"] == ref["type"] and ev["step"] == ref["step"]
    models = [nd["model"] for nd in nodes]
    for key, sel in (("center_all", range(len(nodes))), ("center_subset", g["subset"]),
                     ("center_node0", [0])):
        c = sm.average([models[int(r)] for r in sel])
        assert nl.last_source["average"] == "resident"
        flat = torch.cat([q.detach().reshape(-1) for q in c.parameters()]).numpy()
        assert oracle_bitwise(flat, g[key]), key
        assert guard.row_tag(c) is None and type(c) is FlatModel     # a plain copy
    # an in-place write through a parameter (no Module method: the guard does not
    # see it) bumps the version counter, so the device copy is no longer trusted
    with torch.no_grad():
        models[4].ps[0].mul_(1.0)
    assert eng.resident.fresh and not eng.resident.current()
    c = sm.average(models)
    assert nl.last_source["average"] == "stacked"           # (values unchanged: x * 1.0)
    assert oracle_bitwise(torch.cat([q.detach().reshape(-1) for q in c.parameters()]).numpy(),
                          g["center_all"])
    # a guarded write (load_state_dict) makes the device copy stale: the next read stacks
    models[5].load_state_dict(models[5].state_dict())
    assert not eng.resident.fresh
    c = sm.average(models)
    assert nl.last_source["average"] == "stacked"
    assert oracle_bitwise(torch.cat([q.detach().reshape(-1) for q in c.parameters()]).numpy(),
                          g["center_all"])
    lg.Logger().log_consensus_distance(state)
    assert nl.last_source["consensus"] == "host-slab"
    ev2 = json.loads(open(tmp_path / "global.jsonlines").read().strip().splitlines()[-1])
    np.testing.assert_allclose(ev2["distance_to_center"]["global"]["avg"], rg["avg"], rtol=1e-5)
    np.testing.assert_allclose(ev2["center"]["norm"], ref["center"]["norm"], rtol=1e-5)


def oracle_bitwise(a, b):
    from oracle import oracle
    return oracle.bitwise_equal(np.asarray(a), np.asarray(b))


def test_logger_hooks_opt_out(gpu, monkeypatch, tmp_path):
    """NIIDMIX_GPU_LOGGER=0 leaves the reference's functions in place."""
    from niidmix import logger as nl
    lg, sm = _fake_reference_modules(monkeypatch, tmp_path)
    before = (lg.Logger.log_consensus_distance, sm.average)
    monkeypatch.setenv("NIIDMIX_GPU_LOGGER", "0")
    assert nl.install_hooks({"logger": {"log-global-model-accuracy": True}}) == []
    assert (lg.Logger.log_consensus_distance, sm.average) == before
    monkeypatch.delenv("NIIDMIX_GPU_LOGGER")
    assert nl.install_hooks({"logger": {}, "algorithm": {"gpu-logger": False}}) == []
    assert nl.install_hooks({"logger": {}}) == ["simulate.logger.Logger.log_consensus_distance"]
    assert sm.average is before[1]                 # only with log-global-model-accuracy


def test_consensus_event_in_training_rounds(gpu, monkeypatch, tmp_path):
    """The row-streamed training rounds of next_step with log-consensus-distance on (run.py
    logs the event once every node's epoch is done, and next_step then returns synchronised): the
    event the installed hook writes reads the resident slab and matches the CPU restatement of the
    reference arithmetic on the synchronised host models."""
    from niidmix import d_sgd
    from niidmix import logger as nl
    lg, _ = _fake_reference_modules(monkeypatch, tmp_path)
    params, nodes, topo = _ring_training_setup(8)
    params["logger"]["log-consensus-distance"] = True
    for nd in nodes:
        nd["train-set"] = nd["train-set"][:50]               # 2 steps per epoch at batch 25
    state, _, _ = d_sgd.init(nodes, topo, params)
    log = lg.Logger()
    logged = 0
    for _ in range(4):
        state, _, done, _ = d_sgd.next_step(state, params, None)
        if all(done.values()):
            eng = d_sgd.round_engine(nodes)
            assert not eng.resident.pending                  # predicted: returned synchronised
            log.log_consensus_distance(state)
            assert nl.last_source["consensus"] == "resident"
            ev = json.loads(open(log.global_events).read().strip().splitlines()[-1])
            d, norm = _cpu_consensus_statistics([n["model"] for n in nodes])
            gl = ev["distance_to_center"]["global"]
            np.testing.assert_allclose(gl["avg"], np.mean(d), rtol=1e-5)
            np.testing.assert_allclose(ev["center"]["norm"], norm, rtol=1e-5)
            logged += 1
    assert logged == 2
