#!/usr/bin/env python
"""Drop-in D-SGD algorithm plugin whose per-round neighbour mixing runs on MI355X.

Same plugin API as the reference module tools/simulate/algorithm/d_sgd.py, so tools/simulate/run.py
(`algo = import_module(params['algorithm']['module'])`, run.py:50) and the tools/tests/*.sh
pipelines use it unchanged once params.algorithm.module = 'niidmix.d_sgd':

  optimizer(model, params)                  -> torch.optim.SGD            (d_sgd.py:118-122)
  init(nodes, topology, params)             -> (state, 0, False)          (d_sgd.py:124-143)
  next_step(state, params, rundir)          -> (state, losses, epoch_done, active_nodes)  (:178-254)
  average(nodes, topology, params)          -> None, Jacobi mixing of every node's model  (:96-116)
  update_models / average_gradients / update_gradients / gradient       (:19-94)

Only the mixing changes implementation (average(), and the sample topology's uniform average):
the nodes' models become views of one pinned host slab (niidmix.slab.NodeSlab), each round streams
that slab through HBM in column windows and the HIP kernels mix it (niidmix.ops.Mixer).  Mixing mode (params['algorithm']['mixing-mode'], or the
NIIDMIX_MODE environment variable):
  'exact' (default)  bit-identical to the reference loop (tests/test_gpu_dropin.py)
  'fast'             clique-factored / MFMA kernels, within 1e-5 condition-aware relative
Gradient averaging (--clique-gradient, --unbiased-gradient) also runs on the GPU, bit-identical
(niidmix.gradient); local training, optimizer steps and sampling stay on the CPU as in the reference.
"""
import argparse
import itertools
import json
import logging
import os
import time
import weakref
from random import Random

import torch
import torch.nn.functional as F

from . import guard
from . import logger as nl
from . import meta as m
from . import model as nm
from .topology import load as load_topology, to_csr

MODULE = "niidmix.d_sgd"


# ------------------------------------------------------------------------------------------------
# gradient helpers: the reference module's CPU functions, kept for API compatibility (callers that
# import them directly); gradient() below runs the averaged variants on the GPU
def average_gradients(models):
    """Mean of the models' gradients (d_sgd.py:19-27): zeros, add every grad, divide by count."""
    with torch.no_grad():
        acc = [torch.zeros_like(q.grad.data) for q in models[0].parameters()]
        for mdl in models:
            for a, q in zip(acc, mdl.parameters()):
                a.add_(q.grad.data)
        for a in acc:
            a.div_(len(models))
        return acc


def update_models(models, new_model):
    """p.mul_(0.); p.add_(new_p) for every parameter (d_sgd.py:29-35)."""
    with torch.no_grad():
        for mdl in models:
            for q, nq in zip(mdl.parameters(), new_model.parameters()):
                q.mul_(0.)
                q.add_(nq)
    return models


def update_gradients(models, gradients):
    """Overwrite every model's gradients (d_sgd.py:37-45)."""
    with torch.no_grad():
        for mdl in models:
            for g, q in zip(gradients, mdl.parameters()):
                if q.grad is None:
                    q.grad = torch.zeros_like(q)
                q.grad.data.zero_()
                q.grad.data.add_(g)
    return models


def _averages_gradients(params):
    alg = params["algorithm"]
    return bool(alg.get("clique-gradient") or alg.get("unbiased-gradient"))


class _GradEngine:
    """Gradient NodeSlab + GradMean + SlabMixer for one (node list, topology, flags) triple."""

    def __init__(self, nodes, topology, params, device):
        from .gradient import GradMean, build_grad_plan
        from .slab import NodeSlab, SlabMixer
        self.topology = topology
        self.key = _grad_key(params)
        self.plan = build_grad_plan(len(nodes), topology, params)
        self.slab = NodeSlab([n["model"] for n in nodes], grads=True)
        self.op = GradMean(self.plan, device)
        self.runner = SlabMixer(self.op, self.slab.n, self.slab.p, device,
                                window=int(os.environ.get("NIIDMIX_WINDOW", 1 << 15)))

    def valid_for(self, nodes, topology, params):
        return (topology is self.topology and _grad_key(params) == self.key
                and self.slab.owns([n["model"] for n in nodes]))


def _grad_key(params):
    alg = params["algorithm"]
    return (bool(alg.get("clique-gradient")), bool(alg.get("unbiased-gradient")),
            params.get("topology", {}).get("remove-clique-edges", 0))


_grad_engines = {}


class _SampleEngine:
    """NodeSlab of EVERY node + SampleAverage streamed by SlabMixer (one column stripe per GPU)."""

    def __init__(self, nodes, devices):
        from .slab import MultiDeviceRound, NodeSlab, SampleAverage, SlabMixer
        self.slab = NodeSlab([n["model"] for n in nodes])
        self.ops = []

        def make(dev, n, cols):
            op = SampleAverage(dev)
            self.ops.append(op)
            return SlabMixer(op, n, cols, dev, window=_window())
        self.runner = MultiDeviceRound(make, self.slab.n, self.slab.p, devices)

    def run(self, ranks, weights):
        for op in self.ops:
            op.set_active(ranks, weights)
        self.runner.run(self.slab.host, mode="exact")

    def owns(self, nodes):
        return self.slab.owns([n["model"] for n in nodes])


_sample_engines = {}


def sample_average(all_nodes, active):
    """The 'sample' topology's round after the active nodes' optimizer steps (d_sgd.py:240-250):
    avg = setup.model.average([active models], [1/len(active)]*len(active)), then
    update_models([every model], avg) — one device round over the pinned slab of every node
    (niidmix.slab.SampleAverage), bit for bit the reference's CPU arithmetic."""
    synchronize()
    key = id(all_nodes)
    eng = _sample_engines.get(key)
    if eng is None or not eng.owns(all_nodes):
        eng = _SampleEngine(all_nodes, _devices(all_nodes))
        _sample_engines.clear()
        _sample_engines[key] = eng
    pos = {id(n): i for i, n in enumerate(all_nodes)}
    logging.info("  computing average model of sample consisting of %d nodes (GPU)", len(active))
    eng.run([pos[id(n)] for n in active], [1 / len(active) for _ in active])


def gradient(nodes, topology, params):
    """Apply the local, clique-averaged or unbiased gradient, then step (d_sgd.py:47-94).

    The averaged variants run on the GPU: the nodes' gradients are views of one pinned host slab
    (NodeSlab(grads=True)), streamed through HBM in column windows and averaged by
    k_grad_segment_mean (whole cliques) or k_mix_csr | NIIDMIX_FLAG_MEAN (removed clique edges,
    neighbourhoods), bit-identical to average_gradients + update_gradients; the optimizer steps stay
    on the CPU, on the nodes the reference steps (niidmix.gradient.GradPlan.stepped)."""
    logging.info("  applying gradients")
    synchronize()
    if not _averages_gradients(params):
        for n in nodes:
            n["optimizer"].step()
        return
    key = id(nodes)
    eng = _grad_engines.get(key)
    if eng is None or not eng.valid_for(nodes, topology, params):
        dev = torch.device("cuda", torch.cuda.current_device())
        eng = _GradEngine(nodes, topology, params, dev)
        _grad_engines.clear()
        _grad_engines[key] = eng
    logging.info("  averaging gradients (GPU, %s)", eng.plan.kind)
    eng.runner.mix(eng.slab.host)
    for r in eng.plan.stepped:
        nodes[r]["optimizer"].step()


# optimizer -> weakref of the model whose parameters it was checked to cover (no strong refs: a
# dropped node list is not kept alive here)
_sgd_checked = weakref.WeakKeyDictionary()
# node lists whose device-step buffers did not fit in HBM (the CPU steps them): id -> weakref of
# the list's first model (an id reused by another list is not taken for it)
_no_device_step = {}


def _device_step_ok(params, nodes):
    """The plain round's optimizer step may run on the device (_FusedEngine(plain=True)): every
    node's optimizer is the plugin's plain SGD (optimizer() above, momentum 0: no state, p += -lr g)
    over exactly its model's parameters, all trainable, at params' learning rate;
    NIIDMIX_DEVICE_STEP=0 disables it (the CPU steps, as rounds 1-5 did).  The device steps every
    parameter: one the forward does not use (its gradient stays the -0.0 fill, where torch leaves
    None and the optimizer skips it) ends the step unchanged except that a -0.0 becomes +0.0."""
    if os.environ.get("NIIDMIX_DEVICE_STEP", "1") == "0" or not _resident_ok():
        return False
    hit = _no_device_step.get(id(nodes))
    if hit is not None and nodes and hit() is nodes[0]["model"]:
        return False
    lr = float(params["algorithm"]["learning-rate"])
    for nd in nodes:
        opt = nd.get("optimizer")
        if type(opt) is not torch.optim.SGD or len(opt.param_groups) != 1:
            return False
        g = opt.param_groups[0]
        if (float(g["lr"]) != lr or g["momentum"] != 0 or g["dampening"] != 0 or
                g["weight_decay"] != 0 or g["nesterov"] or g.get("maximize", False)):
            return False
        hit = _sgd_checked.get(opt)
        if hit is None or hit() is not nd["model"]:
            with guard.suspended():
                mine = list(nd["model"].parameters())
            if len(g["params"]) != len(mine) or any(a is not b for a, b in zip(g["params"], mine)):
                return False
            if not all(q.requires_grad for q in mine):     # a frozen parameter gets no gradient:
                return False                               # the CPU optimizer skips it
            _sgd_checked[opt] = weakref.ref(nd["model"])
    return True


def _fused_ok(params):
    """The fused device round applies when gradients are averaged and the optimizer step is plain
    SGD (momentum 0: the reference's default, d_sgd.py:262-263); NIIDMIX_FUSED=0 disables it."""
    alg = params["algorithm"]
    return (_averages_gradients(params) and float(alg.get("learning-momentum", 0.0)) == 0.0
            and os.environ.get("NIIDMIX_FUSED", "1") != "0")


class _FusedEngine:
    """Parameter slab + gradient slab + GradMean + Mixer, run either row-streamed and resident
    (niidmix.slab.ResidentRound with fused_op: each node's parameter and gradient rows go to the
    GPU right after its backward(), the mixed parameters and averaged gradients come back while
    the next round trains) or windowed (FusedRoundRunner); one column stripe per GPU when several
    are visible (niidmix.slab.MultiDeviceRound).

    plain=True: the plain D-SGD round with its optimizer step on the device (no gradient
    averaging; resident engine only): each node's gradient row goes up right after its backward(),
    the SGD step p += (-lr) g (d_sgd.py:51-52, bitwise torch's CPU SGD) runs on the device-resident
    parameters, then the mixing.  The gradients are views of a pinned slab filled with -0.0 before
    each backward (accumulate_grad adds in place: -0 + g = g bit for bit, every g, where a +0 fill
    would turn a -0 gradient into +0).  While the models were not written between rounds (the
    resident round's `fresh` flag, guarded writes, and the parameters' version counters) the
    parameters stay on the device: only gradients go H2D; otherwise they go up with them."""

    def __init__(self, nodes, topology, params, devices, plain=False):
        from .gradient import GradMean, build_grad_plan
        from .ops import Mixer
        from .slab import FusedRoundRunner, MultiDeviceRound, NodeSlab, ResidentRound, fused_op
        self.topology = topology
        self.weights_id = id(topology.get("weights"))
        self.plain = plain
        self.key = _grad_key(params) + (float(params["algorithm"]["learning-rate"]), plain)
        models = [n["model"] for n in nodes]
        self.slab = NodeSlab(models)
        self.gslab = NodeSlab(models, grads=True)
        self.plan = None if plain else build_grad_plan(len(nodes), topology, params)
        stepped = list(range(len(nodes))) if plain else self.plan.stepped
        csr = to_csr(topology)
        if csr.n != self.slab.n:
            raise ValueError(f"topology has {csr.n} nodes, {self.slab.n} models given")
        self.mixer = Mixer(csr=csr, cliques=topology.get("cliques"), device=devices[0])
        lr = params["algorithm"]["learning-rate"]

        n, p = self.slab.n, self.slab.p
        # the plain round's gradients are the nodes' own: nothing to write back
        wb = not plain and os.environ.get("NIIDMIX_GRAD_WRITEBACK", "1") != "0"
        self.resident = None
        self.runner = None
        self.param_uploads = 0          # rounds whose parameters went H2D (tests)
        if _resident_ok() and ResidentRound.fits(n, p, devices, buffers=4 if wb else 3):
            self.resident = ResidentRound(
                lambda dev, part: fused_op(dev, part, None if plain else GradMean(self.plan, dev),
                                           stepped, lr,
                                           self.mixer if dev == devices[0] else self.mixer.to(dev)),
                n, p, devices, block=_row_block(), n_in=2, n_out=2 if wb else 1)
            self.outs = (self.slab.host, self.gslab.host) if wb else (self.slab.host,)
            self.resident.version_of = self.slab.version
            guard.install(models, self.resident)
        elif not plain:
            def make(dev, n, cols):
                mixer = self.mixer if dev == devices[0] else self.mixer.to(dev)
                return FusedRoundRunner(GradMean(self.plan, dev), self.plan.stepped, lr, mixer, n,
                                        cols, dev, window=_window())
            self.runner = MultiDeviceRound(make, n, p, devices)

    @property
    def kind(self):
        return "own gradient" if self.plain else self.plan.kind

    def params_resident(self):
        """The device holds the models' current parameters: the last round's mixed output, with no
        write to the models since (guarded writes clear `fresh`; the version counters catch writes
        through the parameters, e.g. an optimizer step or p.add_ under no_grad)."""
        return self.resident is not None and self.resident.current()

    def clear_grad_row(self, i):
        """Before node i's backward: its gradient views to -0.0 (see the class docstring)."""
        self.gslab.host[i].fill_(-0.0)

    # the row-streamed round (resident engine only)
    def begin_round(self):
        if self.resident is not None:
            if self.params_resident():
                self.resident.begin(None, self.gslab.host, outs=self.outs, resident_in0=True)
            else:
                self.param_uploads += 1
                self.resident.begin(self.slab.host, self.gslab.host, outs=self.outs)

    def row_ready(self, i):
        if self.resident is not None:
            self.resident.row_ready(i)

    def wait_row(self, i):
        if self.resident is not None:
            self.resident.wait_row(i)

    def wait_all(self):
        if self.resident is not None:
            self.resident.wait_all()

    def run(self, mode, timing=False, defer=False):
        if self.resident is not None:
            if self.resident.hosts is None:
                self.begin_round()                    # nothing streamed: every row goes up now
            self.resident.mix(mode, timing=timing)
            if not defer:
                self.resident.wait_all()
                return self.resident.last_timing
            return None
        self.runner.run(self.slab.host, self.gslab.host, mode=mode, timing=timing)
        return self.runner.last_timing

    def same_models(self, nodes, params):
        models = [n["model"] for n in nodes]
        return (_grad_key(params) + (float(params["algorithm"]["learning-rate"]), self.plain)
                == self.key and self.slab.owns(models) and self.gslab.owns(models))

    def valid_for(self, nodes, topology, params):
        return (topology is self.topology and id(topology.get("weights")) == self.weights_id
                and self.same_models(nodes, params))

    def set_topology(self, topology):
        """A new graph for the same nodes (plain rounds, random-graph --randomize): only the
        mixing operator changes; the slabs and the resident device buffers are kept."""
        from .ops import Mixer
        csr = to_csr(topology)
        if csr.n != self.slab.n:
            raise ValueError(f"topology has {csr.n} nodes, {self.slab.n} models given")
        self.wait_all()                  # the last round's kernel may still read the old Mixer
        dev0 = self.resident.parts[0]["dev"]
        self.mixer = Mixer(csr=csr, cliques=topology.get("cliques"), device=dev0)
        for pt in self.resident.parts:
            pt["mixer"] = self.mixer if pt["dev"] == dev0 else self.mixer.to(pt["dev"])
        self.topology = topology
        self.weights_id = id(topology.get("weights"))


_fused_engines = {}


def fused_round(nodes, topology, params):
    """gradient(nodes, topology, params) followed by average(nodes, topology, params), as one
    device round: gradient mean, SGD step and mixing on each column window, one H2D of parameters
    and gradients and one D2H of the mixed parameters (niidmix.slab.FusedRoundRunner)."""
    synchronize()
    eng = _fused_engine(nodes, topology, params)
    logging.info("  fused gradient %s + SGD step + mixing (GPU, %s)", eng.plan.kind, _mode(params))
    t = eng.run(_mode(params), timing=logging.getLogger().isEnabledFor(logging.INFO))
    if t:
        logging.info("  fused round: %s", t)


def _fused_engine(nodes, topology, params, plain=False):
    key = (id(nodes), plain)
    eng = _fused_engines.get(key)
    if plain and eng is not None and not eng.valid_for(nodes, topology, params) and \
            eng.same_models(nodes, params):
        eng.set_topology(topology)                   # same nodes, new graph (--randomize)
    if eng is None or not eng.valid_for(nodes, topology, params):
        synchronize()
        eng = _FusedEngine(nodes, topology, params, _devices(nodes), plain=plain)
        _fused_engines.pop(key, None)
        _fused_engines[key] = eng
        while len(_fused_engines) > MAX_ENGINES:
            _fused_engines.pop(next(iter(_fused_engines)))
    return eng


# ------------------------------------------------------------------------------------------------
# the GPU mixing step
def _window():
    return int(os.environ.get("NIIDMIX_WINDOW", 1 << 15))


def _resident_ok():
    """The row-streamed resident rounds (niidmix.slab.ResidentRound); NIIDMIX_RESIDENT=0: the
    windowed rounds of rounds 1-3."""
    return os.environ.get("NIIDMIX_RESIDENT", "1") != "0"


def _row_block():
    return int(os.environ.get("NIIDMIX_ROW_BLOCK", 8))


class _Engine:
    """NodeSlab + Mixer + the round runner for one (node list, topology) pair.

    Resident (default when the two [N, P] buffers fit in HBM, NIIDMIX_RESIDENT=0 disables): the
    slab stays in HBM and the PCIe copies overlap the CPU part of the round
    (niidmix.slab.ResidentRound: rows go up right after their optimizer.step(), the mixed rows come
    back block by block while the next round trains).  Otherwise a windowed round
    (niidmix.slab.SlabMixer: H2D / mix / D2H pipelined over column windows).  With several GPUs
    visible (niidmix.slab.mixing_devices) either is split into parameter-column stripes, one per GPU
    and PCIe link; bitwise the same."""

    def __init__(self, nodes, topology, devices):
        from .ops import Mixer
        from .slab import MultiDeviceRound, NodeSlab, ResidentRound, SlabMixer  # noqa: F401
        self.topology = topology
        self.weights_id = id(topology.get("weights"))
        self.slab = NodeSlab([n["model"] for n in nodes])
        csr = to_csr(topology)
        if csr.n != self.slab.n:
            raise ValueError(f"topology has {csr.n} nodes, {self.slab.n} models given")
        self.devices = devices
        self.mixer = Mixer(csr=csr, cliques=topology.get("cliques"), device=devices[0])
        n, p = self.slab.n, self.slab.p
        self.resident = None
        self.runner = None
        if _resident_ok() and ResidentRound.fits(n, p, devices):
            from .slab import mixing_op
            self.resident = ResidentRound(
                lambda dev, part: mixing_op(dev, part, self.mixer if dev == devices[0]
                                            else self.mixer.to(dev)),
                n, p, devices, block=_row_block())
            self.resident.version_of = self.slab.version
            guard.install(self.slab.models, self.resident)
        else:
            self.runner = MultiDeviceRound(
                lambda dev, n, cols: SlabMixer(self.mixer if dev == devices[0] else self.mixer.to(dev),
                                               n, cols, dev, window=_window()), n, p, devices)

    # the row-streamed round (resident engine only)
    def begin_round(self):
        if self.resident is not None:
            self.resident.begin(self.slab.host)

    def row_ready(self, i):
        if self.resident is not None:
            self.resident.row_ready(i)

    def wait_row(self, i):
        if self.resident is not None:
            self.resident.wait_row(i)

    def wait_all(self):
        if self.resident is not None:
            self.resident.wait_all()

    def mix(self, mode, timing, defer=False):
        """One mixing round of every node.  defer=True (resident engine, next_step only): return
        with the mixed rows still streaming back (wait_row / wait_all before reading them)."""
        if self.resident is not None:
            if self.resident.host is None:
                self.resident.begin(self.slab.host)    # no row streamed: all of them go up now
            self.resident.mix(mode, timing=timing)
            if not defer:
                self.resident.wait_all()
                return self.resident.last_timing
            return None
        self.runner.run(self.slab.host, mode=mode, timing=timing)
        return self.runner.last_timing

    def owns(self, nodes):
        return self.slab.owns([n["model"] for n in nodes])

    def valid_for(self, nodes, topology):
        return (topology is self.topology and id(topology.get("weights")) == self.weights_id
                and self.owns(nodes))

    def set_topology(self, topology):
        """A new topology for the same nodes (random-graph --randomize, d_sgd.py:223-234): only the
        mixing operator is rebuilt; the pinned slab (the models' parameters) and the device window
        buffers are kept."""
        from .ops import Mixer
        csr = to_csr(topology)
        if csr.n != self.slab.n:
            raise ValueError(f"topology has {csr.n} nodes, {self.slab.n} models given")
        # the previous (deferred) round's kernel may still read the old Mixer's device descriptors
        # on the resident s_mix stream: drain it before they are freed
        self.wait_all()
        self.mixer = Mixer(csr=csr, cliques=topology.get("cliques"), device=self.devices[0])
        if self.resident is not None:
            for pt in self.resident.parts:
                pt["mixer"] = self.mixer if pt["dev"] == self.devices[0] else self.mixer.to(pt["dev"])
        else:
            for runner in self.runner.runners:
                if runner is not None:
                    runner.mixer = self.mixer if runner.device == self.devices[0] else \
                        self.mixer.to(runner.device)
        self.topology = topology
        self.weights_id = id(topology.get("weights"))



_engines = {}
# the engine that ran the last row-streamed next_step round of a node list (round_engine), held
# weakly: an engine evicted from the caches frees its HBM buffers
_last_round = {}
# engines (pinned slab + device buffers) kept per node list, the most recent ones
MAX_ENGINES = int(os.environ.get("NIIDMIX_MAX_ENGINES", 4))


def _mode(params):
    mode = os.environ.get("NIIDMIX_MODE") or params.get("algorithm", {}).get("mixing-mode", "exact")
    if mode not in ("exact", "fast"):
        raise ValueError(f"unknown mixing mode {mode!r}")
    return mode


def invalidate(nodes=None):
    """Declare the models of `nodes` (default: every node list) written behind the plugin's back
    (p.data.copy_, a raw pointer): the next round uploads their parameters again and the logger
    hooks stop reading the device copy."""
    for eng in list(_engines.values()) + list(_fused_engines.values()):
        rr = getattr(eng, "resident", None)
        if rr is not None and (nodes is None or eng.slab.owns([n["model"] for n in nodes])):
            rr.fresh = False


def round_engine(nodes):
    """The engine (_Engine or _FusedEngine, with .resident) whose row-streamed round last ran for
    this node list in next_step, or None."""
    ref = _last_round.get(id(nodes))
    return ref() if ref is not None else None


def synchronize():
    """Wait until the mixed parameters of the last round are all back in the nodes' models.
    next_step may return while they stream back (deferred write-back, _deferred_ok); everything in
    this module that reads or writes the models waits first, and so must any other reader."""
    for eng in list(_engines.values()) + list(_fused_engines.values()):
        eng.wait_all()


def _engine(nodes, topology):
    key = id(nodes)
    eng = _engines.get(key)
    if eng is not None and not eng.valid_for(nodes, topology) and eng.owns(nodes):
        eng.set_topology(topology)                   # same nodes, new graph: keep the slab
    if eng is None or not eng.valid_for(nodes, topology):
        synchronize()
        eng = _Engine(nodes, topology, _devices(nodes))
        _engines.pop(key, None)
        _engines[key] = eng
        while len(_engines) > MAX_ENGINES:               # oldest node lists first
            _engines.pop(next(iter(_engines)))
    return eng


def average(nodes, topology, params):
    """Every node's model <- sum_j W[j, rank] model_j over [self] + edges[rank], computed from the
    pre-round models (Jacobi) then written back (update_models), as d_sgd.py:96-116 — one GPU pass
    over the whole [N, P] slab instead of N*(deg+1)*n_tensors ATen calls.  Returns with every model
    updated."""
    logging.info("  computing averages of models (GPU, %s)", _mode(params))
    eng = _engine(nodes, topology)
    t = eng.mix(_mode(params), logging.getLogger().isEnabledFor(logging.INFO))
    if t:
        logging.info("  mixing round: %s", t)


# seconds the CPU spent on the mixing in the row-streamed rounds (bench.py --e2e-step): waiting for
# rows (wait_row / wait_all) and enqueueing copies and kernels (row_ready / mix)
round_stats = {"wait_s": 0.0, "enqueue_s": 0.0, "rounds": 0}


def _row_streamed(params):
    """Plain D-SGD rounds run row-streamed (next_step drives the resident engine itself instead of
    gradient() + average(); NIIDMIX_ROW_STREAM=0 restores the two calls)."""
    return os.environ.get("NIIDMIX_ROW_STREAM", "1") != "0"


def _should_log(node, epoch_done, params, state):
    """run.py:19-25, the driver's test for reading a node's model after next_step."""
    lg = params.get("logger", {})
    if lg.get("accuracy-logging-interval") and epoch_done and \
            node["epoch"] % lg["accuracy-logging-interval"] == 0:
        return True
    if lg.get("accuracy-logging-interval-steps") and \
            state["step"] % lg["accuracy-logging-interval-steps"] == 0:
        return True
    return False


def _deferred_ok(params, state, epoch_done, active):
    """May next_step return before the mixed rows are back on the host?  Only when the plugin was
    registered with deferred write-back (params.algorithm.deferred-writeback, the CLI default;
    NIIDMIX_DEFERRED_WRITEBACK=0/1 overrides) AND the driver reads no model before the next
    next_step: run.py:105-119 reads models only through log.state (should_log, run.py:19-25, per
    active node or node 0 for fully-connected / sample) and log_consensus_distance (every node
    epoch-done), both predicted here from the same params and state.  The next round's training
    waits for each node's own rows (wait_row) before its forward."""
    env = os.environ.get("NIIDMIX_DEFERRED_WRITEBACK")
    on = (env != "0") if env is not None else bool(params["algorithm"].get("deferred-writeback"))
    if not on:
        return False
    lg = params.get("logger", {})
    if lg.get("log-consensus-distance") and epoch_done and all(epoch_done.values()):
        return False
    # run.py:107-116: fully-connected / sample log node 0 when IT should log; otherwise (and for
    # every other topology) each active node that should log -- e.g. a node whose epoch ended when
    # node 0's did not
    if params["topology"]["name"] in ("fully-connected", "sample") and \
            _should_log(state["nodes"][0], epoch_done.get(0, False), params, state):
        return False
    return not any(_should_log(n, epoch_done[n["rank"]], params, state) for n in active)


def _devices(nodes):
    """GPUs the host-resident round uses (niidmix.slab.mixing_devices; NIIDMIX_DEVICES selects),
    the current device first."""
    from .slab import mixing_devices
    p = sum(q.numel() for q in nodes[0]["model"].parameters())
    cur = torch.cuda.current_device()
    devs = mixing_devices(p)
    if not os.environ.get("NIIDMIX_DEVICES"):
        order = [cur] + [d.index for d in devs if d.index != cur]
        devs = [torch.device("cuda", i) for i in order[:len(devs)]]
    return devs


# ------------------------------------------------------------------------------------------------
# plugin API
def optimizer(model, params):
    return torch.optim.SGD(model.parameters(), lr=params["algorithm"]["learning-rate"],
                           momentum=params["algorithm"]["learning-momentum"])


def _loader(node, params):
    return iter(torch.utils.data.DataLoader(node["train-set"],
                                            batch_size=int(params["algorithm"]["batch-size"]),
                                            shuffle=True))


def init(nodes, topology, params):
    logging.basicConfig(level=getattr(logging, params["meta"]["log"].upper(), None))
    synchronize()
    state = {"nodes": nodes, "topology": topology, "step": 0}
    # the reference driver's logging of the models on the GPU (niidmix.logger.install_hooks:
    # Logger.log_consensus_distance, and setup.model.average under log-global-model-accuracy)
    nl.install_hooks(params)
    for n in nodes:
        n["train-iterator"] = _loader(n, params)
    if params["algorithm"]["initial-averaging"]:
        center = nm.average([nodes[r]["model"] for r in range(len(nodes))])
        for r in range(len(nodes)):
            update_models([nodes[r]["model"]], center)
    return (state, 0, False)


def _peek(iterator):
    try:
        first = next(iterator)
    except StopIteration:
        return None
    return itertools.chain([first], iterator)


_sample_cache = {}


def get_sample(state, params, step):
    """Active nodes of the 'sample' topology (d_sgd.py:157-175)."""
    if step in _sample_cache:
        return _sample_cache[step]
    rnd = Random(42 + step)
    method = params["topology"]["sample-method"]
    size = params["topology"]["sample-size"]
    if method == "random":
        return rnd.sample(state["nodes"], size)
    if method == "random-with-overlap":
        if step == 0:
            return rnd.sample(state["nodes"], size)
        previous = get_sample(state, params, step - 1)
        active = rnd.sample(previous, params["topology"]["sample-overlap"])
        rest = [n for n in state["nodes"] if n not in active]
        active += rnd.sample(rest, size - params["topology"]["sample-overlap"])
        _sample_cache[step] = active
        return active


DENSE_JSON_MAX = int(os.environ.get("NIIDMIX_DENSE_JSON_MAX", 1024))


def randomized_topology(nodes, params, rundir):
    """The next round's random graph (d_sgd.py:223-234: random_graph.generate_topology with the
    incremented topology-seed), built SPARSE: the edge lists by the restated generator
    (niidmix.generate.random_graph, same RNG order, hence the same graph) and the MH weights as a
    CSR (topology.mh_csr, bit-identical to compute_weights) -- O(N k) storage instead of the dense
    N x N matrix (the diagonal keeps the reference's O(N^2) fp32 row sums, batched).  Every round the rundir gets topology.json (d_sgd.py:229-230), always readable
    by the reference's loader: up to NIIDMIX_DENSE_JSON_MAX nodes (default 1024) with the dense
    weights the reference writes, above it in the sparse form (niidmix.topology.sparse_json:
    'weights': [] + the CSR in topology.csr.npz), so the file never lags the graph the round used.
    The returned topology carries the weights as the reference's does (a dense tensor, or the
    empty tensor the loader makes of the sparse form) plus the CSR under 'csr'."""
    from .generate import random_graph_csr
    from .topology import sparse_json, save_csr
    t = params["topology"]
    weights = t.get("weights", "metropolis-hasting")
    if weights != "metropolis-hasting":
        raise ValueError(f"--weights {weights}: only metropolis-hasting is supported (the "
                         "reference's equal-clique-probability indexes sets, weights.py:5-14)")
    n = len(nodes)
    assert [nd["rank"] for nd in nodes] == list(range(n)), "nodes must be listed in rank order"
    csr, edges = random_graph_csr(n, t["nb-neighbours"], t["topology-seed"])
    dense = n <= DENSE_JSON_MAX
    w = csr.dense() if dense else None
    if rundir is not None:
        save_csr(os.path.join(rundir, "topology.csr.npz"), csr)
        with open(os.path.join(rundir, "topology.json"), "w+") as f:
            json.dump({"edges": {r: edges[r] for r in edges}, "weights": w.tolist()} if dense
                      else sparse_json(edges), f)
    return {"edges": edges, "csr": csr,
            "weights": torch.from_numpy(w) if dense else torch.tensor([])}


def next_step(state, params, rundir):
    sample = params["topology"]["name"] == "sample"
    active = get_sample(state, params, state["step"]) if sample else state["nodes"]
    topology = state["topology"]
    # plain D-SGD (own gradient, then mixing): the row-streamed round — each node's rows go to the
    # GPU right after its optimizer.step() and come back while the next round trains
    streamed = not sample and not _averages_gradients(params) and _row_streamed(params)
    feng = None
    if streamed and _device_step_ok(params, active):
        # ... with the optimizer step on the device: each node's gradient row goes up right after
        # its backward(), the parameters stay resident (_FusedEngine(plain=True))
        feng = _fused_engine(active, topology, params, plain=True)
        if feng.resident is None:                 # the buffers do not fit: CPU step, windowed
            _fused_engines.pop((id(active), True), None)
            _no_device_step[id(active)] = weakref.ref(active[0]["model"])
            feng = None
    eng = _engine(active, topology) if streamed and feng is None else None
    # gradient averaging, momentum 0: the fused device round, row-streamed too — each node's
    # parameter and gradient rows go up right after its backward()
    if feng is None and not sample and _fused_ok(params) and _row_streamed(params):
        feng = _fused_engine(active, topology, params)
    if eng is None and feng is None:
        synchronize()
    if feng is not None:
        feng.begin_round()
    weng = eng if eng is not None else feng
    losses, epoch_done = {}, {}
    clock = time.perf_counter
    for i, node in enumerate(active):                     # local training (CPU)
        if weng is not None:
            t0 = clock()
            weng.wait_row(i)                              # this node's mixed rows are back
            round_stats["wait_s"] += clock() - t0
        data, target = next(node["train-iterator"])
        # gradient averaging keeps .grad as views of the pinned gradient slab: zero in place (the
        # reference's torch 1.7.1 zero_grad behaviour) so backward accumulates into the views
        if feng is not None and feng.plain:
            feng.clear_grad_row(i)                        # -0.0: backward adds g bit for bit
        else:
            node["optimizer"].zero_grad(set_to_none=not _averages_gradients(params))
        loss = F.nll_loss(node["model"].forward(data, params), target)
        loss.backward()
        losses[node["rank"]] = loss.tolist()
        if feng is not None:
            t0 = clock()
            feng.row_ready(i)                             # its parameters and gradients are final
            round_stats["enqueue_s"] += clock() - t0
        rest = _peek(node["train-iterator"])
        done = rest is None
        if done:
            node["epoch"] += 1
            node["train-iterator"] = _loader(node, params)
        else:
            node["train-iterator"] = rest
        epoch_done[node["rank"]] = done
    defer = False
    if weng is not None:
        _last_round.clear()
        _last_round[id(active)] = weakref.ref(weng)
    if not sample:
        if feng is not None:
            t0 = clock()
            feng.wait_all()
            logging.info("  gradient (%s) + SGD step + mixing (GPU, %s, row-streamed)",
                         feng.kind, _mode(params))
            feng.run(_mode(params), defer=True)           # ★ GPU: gradient + step + mixing
            round_stats["enqueue_s"] += clock() - t0
            round_stats["rounds"] += 1
            eng, defer = feng, True
        elif _fused_ok(params):
            fused_round(active, topology, params)         # ★ GPU: gradient + step + mixing
        elif eng is not None:
            t0 = clock()
            eng.wait_all()                                # (every node trained: nothing pending)
            eng.begin_round()
            round_stats["wait_s"] += clock() - t0
            logging.info("  applying own gradient")
            for i, n in enumerate(active):                # d_sgd.py:51-52, rows sent as they
                n["optimizer"].step()                     # become final
                t0 = clock()
                eng.row_ready(i)
                round_stats["enqueue_s"] += clock() - t0
            logging.info("  computing averages of models (GPU, %s, row-streamed)", _mode(params))
            t0 = clock()
            eng.mix(_mode(params), False, defer=True)     # ★ GPU
            round_stats["enqueue_s"] += clock() - t0
            round_stats["rounds"] += 1
            defer = True
        else:
            gradient(active, topology, params)
            average(active, topology, params)             # ★ GPU
        if params["topology"]["name"] == "random-graph" and params["topology"]["randomize"]:
            params["topology"]["topology-seed"] += 1
            state["topology"] = randomized_topology(state["nodes"], params, rundir)
    else:
        for n in active:
            n["optimizer"].step()
        sample_average(state["nodes"], active)            # ★ GPU: average + update_models
    state["step"] += 1
    if defer and not _deferred_ok(params, state, epoch_done, active):
        t0 = clock()
        eng.wait_all()                                    # the driver reads models next
        round_stats["wait_s"] += clock() - t0
    return state, losses, epoch_done, active


def main(argv=None):
    ap = argparse.ArgumentParser(description="Provide Options for D-SGD (MI355X mixing).")
    ap.add_argument("--rundir", type=str, default=None)
    ap.add_argument("--learning-rate", type=float, default=0.1)
    ap.add_argument("--learning-momentum", type=float, default=0.0)
    ap.add_argument("--batch-size", type=int, default=128)
    ap.add_argument("--initial-averaging", action="store_const", const=True, default=False)
    ap.add_argument("--clique-gradient", action="store_const", const=True, default=False)
    ap.add_argument("--unbiased-gradient", action="store_const", const=True, default=False)
    ap.add_argument("--mixing-mode", choices=["exact", "fast"], default="exact",
                    help="exact: bit-identical to the reference loop; fast: clique/MFMA kernels")
    ap.add_argument("--no-deferred-writeback", dest="deferred_writeback", action="store_false",
                    help="next_step returns only once every mixed row is back in the models (by "
                         "default it returns while they stream back, whenever the driver reads no "
                         "model before the next round: run.py's logging is predicted)")
    args = ap.parse_args(argv)
    rundir = m.rundir(args)
    params = m.params(rundir)
    topology = load_topology(rundir)
    if args.clique_gradient:
        assert "cliques" in topology, \
            "Invalid --clique-gradient with {} topology, no 'cliques' found in topology.json.".format(
                params["topology"]["name"])
    if args.unbiased_gradient:
        assert "neighbourhoods" in topology, \
            "Invalid --unbiased-gradient with {} topology, no 'neighbourhoods' found in topology.json.".format(
                params["topology"]["name"])
    m.extend(rundir, "algorithm", {
        "name": "d-sgd", "module": MODULE,
        "learning-rate": args.learning_rate, "learning-momentum": args.learning_momentum,
        "batch-size": args.batch_size, "initial-averaging": args.initial_averaging,
        "clique-gradient": args.clique_gradient, "unbiased-gradient": args.unbiased_gradient,
        "mixing-mode": args.mixing_mode, "deferred-writeback": args.deferred_writeback,
    })
    if args.rundir is None:
        print(rundir)


if __name__ == "__main__":
    main()
