"""Drop-in host logic on CPU: NodeSlab views, meta/CLI registration."""
import json
import os
import sys

import torch

from niidmix import meta
from niidmix.slab import NodeSlab


def test_nodeslab_views_and_optimizer():
    torch.manual_seed(0)
    models = [torch.nn.Linear(7, 3) for _ in range(4)]
    before = [torch.cat([q.detach().reshape(-1).clone() for q in mm.parameters()]) for mm in models]
    opts = [torch.optim.SGD(mm.parameters(), lr=0.1) for mm in models]
    slab = NodeSlab(models, pin=False)
    assert slab.host.shape == (4, 7 * 3 + 3)
    for i in range(4):
        assert torch.equal(slab.host[i], before[i])
    # optimizer steps write straight into the slab
    x = torch.randn(5, 7)
    models[2](x).sum().backward()
    opts[2].step()
    flat = torch.cat([q.detach().reshape(-1) for q in models[2].parameters()])
    assert torch.equal(slab.host[2], flat)
    assert not torch.equal(slab.host[2], before[2])
    assert slab.owns(models) and not slab.owns(models[::-1])


def test_meta_extend_refuses_overwrite(tmp_path):
    d = str(tmp_path)
    meta.extend(d, "meta", {"seed": 1})
    assert meta.params(d, "meta") == {"seed": 1}
    try:
        meta.extend(d, "meta", {"seed": 2})
        raise RuntimeError("should have refused")
    except AssertionError:
        pass


def test_cli_registers_plugin(tmp_path):
    d = str(tmp_path)
    topo = {"edges": {"0": [1], "1": [0]}, "weights": [[0.5, 0.5], [0.5, 0.5]]}
    with open(os.path.join(d, "topology.json"), "w") as f:
        json.dump(topo, f)
    meta.extend(d, "topology", {"name": "ring"})
    from niidmix import d_sgd
    d_sgd.main(["--rundir", d, "--batch-size", "125"])
    alg = meta.params(d, "algorithm")
    assert alg["module"] == "niidmix.d_sgd" and alg["batch-size"] == 125
    assert alg["mixing-mode"] == "exact"


def test_blocked_layout_roundtrip_cpu():
    """niidmix.memory.to_blocked / from_blocked: [rows, p] <-> [ceil(p/B), rows, B]."""
    import torch
    from niidmix import memory
    x = torch.arange(5 * 9000, dtype=torch.float32).view(5, 9000)
    xb = memory.to_blocked(x, block_cols=4096)
    assert xb.shape == (3, 5, 4096)
    assert torch.equal(xb[1, 2, :10], x[2, 4096:4106])
    assert float(xb[2, :, 9000 - 8192:].abs().sum()) == 0.0
    assert torch.equal(memory.from_blocked(xb, 9000), x)


def test_mixing_devices_policy(monkeypatch):
    """One GPU per 64K parameter columns at most, NIIDMIX_DEVICES selects (no GPU needed)."""
    import torch
    from niidmix.slab import MIN_STRIPE_COLS, mixing_devices
    devs = [torch.device("cuda", i) for i in range(8)]
    assert mixing_devices(7850, devs) == devs[:1]                 # linear MNIST model
    assert mixing_devices(62006, devs) == devs[:1]                # LeNet size
    assert mixing_devices(1 << 20, devs) == devs                  # 1M parameters: all 8
    assert mixing_devices(3 * MIN_STRIPE_COLS, devs) == devs[:3]
    monkeypatch.setenv("NIIDMIX_DEVICES", "2,5")
    assert mixing_devices(1 << 20) == [torch.device("cuda", 2), torch.device("cuda", 5)]


def _run_py_reads_models(params, state, epoch_done, active):
    """Which of run.py's post-next_step branches (tools/simulate/run.py:105-119) read a model:
    log.state of the nodes its should_log (run.py:19-25) picks -- node 0 alone for fully-connected
    / sample when node 0 should log, else every active node that should -- and
    log_consensus_distance once every node finished its epoch."""
    lg = params["logger"]

    def should_log(node, done):
        if lg["accuracy-logging-interval"] and done and \
                node["epoch"] % lg["accuracy-logging-interval"] == 0:
            return True
        return bool(lg["accuracy-logging-interval-steps"]) and \
            state["step"] % lg["accuracy-logging-interval-steps"] == 0

    logged = []
    if params["topology"]["name"] in ("fully-connected", "sample") and \
            should_log(state["nodes"][0], epoch_done.get(0, False)):
        logged = [state["nodes"][0]]
    else:
        logged = [n for n in active if should_log(n, epoch_done[n["rank"]])]
    return bool(logged) or bool(all(epoch_done.values()) and lg["log-consensus-distance"])


def test_deferred_ok_mirrors_run_py_branches(monkeypatch):
    """niidmix.d_sgd._deferred_ok (may next_step return with the write-back in flight?) against
    run.py's own branch structure, over topologies, logging intervals, steps, per-node epochs and
    epoch-done patterns -- including the fully-connected case where node 0 does not log but another
    node whose epoch just ended does."""
    import itertools
    from niidmix import d_sgd
    monkeypatch.delenv("NIIDMIX_DEFERRED_WRITEBACK", raising=False)
    n = 4
    checked = 0
    for topo, ivl, ivl_steps, cons, step, epochs, done_bits in itertools.product(
            ("ring", "fully-connected", "sample", "d-cliques"), (0, 1, 2), (0, 3), (False, True),
            (1, 3, 6, 7), ((1, 1, 1, 1), (2, 1, 2, 3)), range(16)):
        nodes = [{"rank": r, "epoch": epochs[r]} for r in range(n)]
        state = {"nodes": nodes, "step": step}
        epoch_done = {r: bool(done_bits >> r & 1) for r in range(n)}
        params = {"topology": {"name": topo},
                  "logger": {"accuracy-logging-interval": ivl,
                             "accuracy-logging-interval-steps": ivl_steps,
                             "log-consensus-distance": cons},
                  "algorithm": {"deferred-writeback": True}}
        for active in (nodes, nodes[1:3]):
            ep = {nd["rank"]: epoch_done[nd["rank"]] for nd in active} if topo == "sample" \
                else epoch_done
            got = d_sgd._deferred_ok(params, state, ep, active)
            assert got == (not _run_py_reads_models(params, state, ep, active)), \
                (topo, ivl, ivl_steps, cons, step, epochs, done_bits, len(active))
            checked += 1
    assert checked > 1000
    params["algorithm"]["deferred-writeback"] = False
    assert not d_sgd._deferred_ok(params, state, epoch_done, nodes)


def test_read_guard_waits_for_own_row(monkeypatch):
    """niidmix.guard: every Module entry point that reads or writes a guarded model's parameters
    waits for that model's own row block while a round is pending (and only then); deepcopy and
    isinstance keep working; suspended() and NIIDMIX_READ_GUARD=0 turn it off."""
    import copy
    from niidmix import guard

    class FakeRound:
        pending = True

        def __init__(self):
            self.waited = []

        def wait_row(self, i):
            self.waited.append(i)

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.fc = torch.nn.Linear(3, 2)

        def forward(self, x, params=None):
            return self.fc(x)

    monkeypatch.delenv("NIIDMIX_READ_GUARD", raising=False)
    models = [Net() for _ in range(3)]
    eng = FakeRound()
    guard.install(models, eng)
    m = models[2]
    assert isinstance(m, Net) and type(m).__name__ == "Net" and type(models[0]) is type(m)
    x = torch.zeros(1, 3)
    for read in (lambda: m.forward(x, None), lambda: m(x), lambda: list(m.parameters()),
                 lambda: list(m.named_parameters()), lambda: m.state_dict(),
                 lambda: m.load_state_dict(models[1].state_dict()), lambda: m.to(torch.float32)):
        eng.waited.clear()
        read()
        assert 2 in eng.waited and set(eng.waited) <= {1, 2}
    eng.waited.clear()
    c = copy.deepcopy(models[0])
    assert isinstance(c, Net) and torch.equal(c.fc.weight, models[0].fc.weight)
    eng.pending = False
    eng.waited.clear()
    models[0](x)
    list(models[1].parameters())
    assert eng.waited == []                          # nothing pending: no wait at all
    eng.pending = True
    with guard.suspended():
        list(models[0].parameters())
    assert eng.waited == []
    monkeypatch.setenv("NIIDMIX_READ_GUARD", "0")
    plain = [Net()]
    guard.install(plain, eng)
    assert type(plain[0]) is Net


def _handoff_child(conn):
    """torch.multiprocessing child: receive a model, send back its class and flat parameters."""
    m = conn.recv()
    # numpy, not a tensor: a tensor would go back through a shared-memory fd that this process,
    # about to exit, could no longer serve
    conn.send((type(m), torch.cat([q.detach().reshape(-1) for q in m.parameters()]).numpy()))
    conn.close()


class _Round:
    pending = True

    def __init__(self):
        self.waited = []

    def wait_row(self, i):
        self.waited.append(i)


def test_slab_models_pickle_compact():
    """A NodeSlab-backed model's parameters each have a storage of their own size: the reference
    logger's pickle.dumps(model.state_dict()) (logger.py:139,254) and torch.save(model) write that
    model only, not the whole [N, P] slab (a plain view would serialise its whole storage); the
    tensors still alias the slab (an in-place update lands in it)."""
    import io
    import pickle
    torch.manual_seed(3)
    models = [torch.nn.Linear(100, 10) for _ in range(64)]
    slab = NodeSlab(models, pin=False)
    one = 1010 * 4
    assert slab.host.numel() * 4 > 60 * one
    m = models[17]
    blob = pickle.dumps(m.state_dict())
    assert len(blob) < 2 * one + 2048
    sd = pickle.loads(blob)
    assert torch.equal(sd["weight"], m.weight.detach()) and torch.equal(sd["bias"], m.bias.detach())
    buf = io.BytesIO()
    torch.save(m, buf)
    assert buf.tell() < 2 * one + 4096
    v0 = slab.version()
    with torch.no_grad():
        m.bias.add_(1.0)
    assert torch.equal(slab.host[17, 1000:], m.bias.detach())
    assert slab.owns(models)
    assert slab.version() == v0 + 1          # in-place writes through a parameter are counted
    slab.host[3].fill_(0.5)                  # raw slab writes (the D2H write-back) are not
    assert slab.version() == v0 + 1


def test_guarded_model_pickles_as_base_class(monkeypatch):
    """VERDICT r05 #5 / ADVICE r05: a guarded, slab-tagged model pickles -- pickle, torch.save /
    torch.load, deepcopy, a torch.multiprocessing hand-off -- as its ORIGINAL class holding its
    current values, after waiting for its own row while a round is pending; no tag travels with
    the copy.  A hand-off moves the sent parameters to shared memory (torch.multiprocessing's own
    semantics): the slab no longer owns the model, so the drop-in rebuilds its engine."""
    import copy
    import io
    import pickle
    from niidmix import guard
    monkeypatch.delenv("NIIDMIX_READ_GUARD", raising=False)
    torch.manual_seed(4)
    models = [torch.nn.Linear(6, 4) for _ in range(5)]
    slab = NodeSlab(models, pin=False)
    eng = _Round()
    guard.install(models, eng)
    m = models[3]
    assert type(m) is not torch.nn.Linear and isinstance(m, torch.nn.Linear)
    assert guard.row_tag(m)[1] == 3 and guard.slab_rows(models)[1] == [0, 1, 2, 3, 4]
    flat = slab.host[3].clone()

    def check(c):
        assert type(c) is torch.nn.Linear
        assert torch.equal(torch.cat([c.weight.detach().reshape(-1), c.bias.detach()]), flat)
        assert guard.row_tag(c) is None and guard.slab_rows([c]) is None

    for rt in (lambda: pickle.loads(pickle.dumps(m)),
               lambda: pickle.loads(pickle.dumps(m, protocol=1)),
               lambda: copy.deepcopy(m), lambda: copy.copy(m)):
        eng.waited.clear()
        check(rt())
        assert eng.waited == [3]
    buf = io.BytesIO()
    eng.waited.clear()
    torch.save(m, buf)
    assert eng.waited == [3]
    buf.seek(0)
    check(torch.load(buf, weights_only=False))     # a file this test wrote
    eng.pending = False
    eng.waited.clear()
    check(pickle.loads(pickle.dumps(m)))
    assert eng.waited == []
    eng.pending = True
    ctx = torch.multiprocessing.get_context("spawn")
    a, b = ctx.Pipe()
    pr = ctx.Process(target=_handoff_child, args=(b,))
    pr.start()
    eng.waited.clear()
    a.send(m)
    cls, got = a.recv()
    pr.join(60)
    assert pr.exitcode == 0 and cls is torch.nn.Linear and torch.equal(torch.from_numpy(got), flat)
    assert eng.waited == [3]
    assert not slab.owns(models) and guard.resident_rows(models) is None


def test_logger_install_hooks_cpu(monkeypatch, tmp_path):
    """niidmix.logger.install_hooks (called by niidmix.d_sgd.init) routes the reference driver's
    Logger.log_consensus_distance always, and setup.model.average only with
    log-global-model-accuracy; idempotent; NIIDMIX_GPU_LOGGER=0 / algorithm.gpu-logger false opt
    out; nothing is touched when the reference's modules are not loaded."""
    import types
    from niidmix import logger as nl
    monkeypatch.delitem(sys.modules, "simulate.logger", raising=False)
    monkeypatch.delitem(sys.modules, "setup.model", raising=False)
    assert nl.install_hooks({"logger": {"log-global-model-accuracy": True}}) == []
    lg = types.ModuleType("simulate.logger")

    class Logger:
        def log_consensus_distance(self, state):
            raise AssertionError("reference CPU version")
    lg.Logger = Logger
    sm = types.ModuleType("setup.model")
    ref_avg = lambda models, weights=None: None   # noqa: E731
    sm.average = ref_avg
    monkeypatch.setitem(sys.modules, "simulate.logger", lg)
    monkeypatch.setitem(sys.modules, "setup.model", sm)
    monkeypatch.setenv("NIIDMIX_GPU_LOGGER", "0")
    assert nl.install_hooks({"logger": {"log-global-model-accuracy": True}}) == []
    monkeypatch.delenv("NIIDMIX_GPU_LOGGER")
    assert nl.install_hooks({"logger": {}, "algorithm": {"gpu-logger": False}}) == []
    assert nl.install_hooks({"logger": {}}) == ["simulate.logger.Logger.log_consensus_distance"]
    assert Logger.log_consensus_distance is nl.log_consensus_distance and sm.average is ref_avg
    done = nl.install_hooks({"logger": {"log-global-model-accuracy": True}})
    assert done == ["simulate.logger.Logger.log_consensus_distance", "setup.model.average"]
    assert sm.average is nl.average
    assert nl.install_hooks({"logger": {"log-global-model-accuracy": True}}) == done


def test_device_step_eligibility(monkeypatch):
    """niidmix.d_sgd._device_step_ok: the plain round's optimizer step moves to the device only for
    the plugin's plain SGD (momentum, dampening, weight decay 0, no Nesterov / maximize) at
    params' learning rate over exactly the model's parameters; NIIDMIX_DEVICE_STEP=0 and
    NIIDMIX_RESIDENT=0 turn it off (no GPU needed)."""
    from niidmix import d_sgd
    monkeypatch.delenv("NIIDMIX_DEVICE_STEP", raising=False)
    monkeypatch.delenv("NIIDMIX_RESIDENT", raising=False)
    params = {"algorithm": {"learning-rate": 0.1, "learning-momentum": 0.0}}

    def nodes_with(**kw):
        out = []
        for r in range(3):
            m = torch.nn.Linear(4, 2)
            opt = d_sgd.optimizer(m, params) if not kw else torch.optim.SGD(m.parameters(), **kw)
            out.append({"rank": r, "model": m, "optimizer": opt})
        return out

    assert d_sgd._device_step_ok(params, nodes_with())
    assert not d_sgd._device_step_ok(params, nodes_with(lr=0.1, momentum=0.9))
    assert not d_sgd._device_step_ok(params, nodes_with(lr=0.1, weight_decay=1e-4))
    assert not d_sgd._device_step_ok(params, nodes_with(lr=0.2))
    assert not d_sgd._device_step_ok(params, nodes_with(lr=0.1, momentum=0.9, nesterov=True))
    nd = nodes_with()
    nd[1]["optimizer"] = torch.optim.SGD([next(nd[1]["model"].parameters())], lr=0.1)
    assert not d_sgd._device_step_ok(params, nd)          # not every parameter
    nd = nodes_with()
    nd[2]["optimizer"] = torch.optim.Adam(nd[2]["model"].parameters(), lr=0.1)
    assert not d_sgd._device_step_ok(params, nd)
    nd = nodes_with()
    nd[0]["model"].bias.requires_grad_(False)
    assert not d_sgd._device_step_ok(params, nd)          # a frozen parameter
    monkeypatch.setenv("NIIDMIX_DEVICE_STEP", "0")
    assert not d_sgd._device_step_ok(params, nodes_with())
    monkeypatch.delenv("NIIDMIX_DEVICE_STEP")
    monkeypatch.setenv("NIIDMIX_RESIDENT", "0")
    assert not d_sgd._device_step_ok(params, nodes_with())
