"""What run.py's logging reads from the models, on the GPU.

The reference driver logs, after next_step (tools/simulate/run.py:102-119):
  * Logger.log_consensus_distance (tools/simulate/logger.py:257-284): the uniform average of every
    node's model (setup.model.average) and each model's L2 distance to it -> one
    "consensus-distance" event in events/global.jsonlines;
  * Logger.state with log-global-model-accuracy (logger.py:97-112): setup.model.average over the
    nodes it logs, pickled for the accuracy workers.

Both are O(N P) host loops in the reference (N model_distance() calls, N*n_tensors ATen adds).
Here they read the mixed parameters where they already are: the resident round's output slab in
HBM (niidmix.slab.ResidentRound keeps it there after every round; `fresh` says it still equals the
models), one kernel pass per GPU stripe, no H2D.  Without a fresh resident slab, the models' pinned
host slab (niidmix.slab.NodeSlab) streams through the GPU in column windows (one H2D); models
that are not slab-backed are stacked (niidmix.model).

  install_hooks(params)          called by niidmix.d_sgd.init: routes the reference Logger's
                                 log_consensus_distance (when simulate.logger is imported) and,
                                 with log-global-model-accuracy, setup.model.average through here.
                                 Opt out: NIIDMIX_GPU_LOGGER=0 or params.algorithm.gpu-logger false
  consensus_distance_event(state)   the event dict, reference schema (doc/experiment.md)
  log_consensus_distance(logger, state)
  average(models, weights=None)  setup.model.average (tools/setup/model/__init__.py:15-25),
                                 bit-identical, reading the resident slab when it can

The uniform average is bit-identical to setup.model.average(models) (exact kernel); distances are
accumulated in fp64 (the reference accumulates fp32 per tensor), so they agree to ~1e-6 relative.
"""
import copy
import json
import os
import statistics
import sys
import time

import numpy as np
import torch

from . import guard, ops

# what the last call read: "resident" (HBM output slab), "host-slab" (pinned slab, one H2D) or
# "stacked" (models stacked, niidmix.model); tests check it
last_source = {"consensus": None, "average": None}


def _fresh_resident(models):
    """(ResidentRound, rows) when the models are rows of a resident round whose device outputs
    still hold their values, else None."""
    hit = guard.resident_rows(models)
    if hit is None:
        return None
    rr, rows = hit
    if not hasattr(rr, "parts") or not rr.current():
        return None
    return rr, rows


def _host_slab(models):
    """(NodeSlab, rows) when the models are rows of one pinned NodeSlab (niidmix.slab), else
    None."""
    hit = guard.slab_rows(models)
    return hit


def _stats_resident(rr):
    """Per-row squared distances to the uniform average and the average's squared norm, from the
    resident output slab: each GPU stripe on its own mixing stream (ordered after the round's op,
    before the next round's), fp64 partial sums added on the host."""
    d2, nrm = [], []
    for pt in rr.parts:
        x = pt["outs"][0]
        with torch.cuda.device(pt["dev"]), torch.cuda.stream(pt["s_mix"]):
            mean = torch.empty(x.shape[1], dtype=torch.float32, device=pt["dev"])
            dist2 = torch.empty(x.shape[0], dtype=torch.float64, device=pt["dev"])
            ops.mean_rows(x, mean, dist2, ops.EXACT)
            sq = torch.sum(mean.double() ** 2)
            # read back on the same (non-blocking) stream: a copy on the default stream would not
            # wait for the statistics
            d2.append(dist2.cpu())
            nrm.append(float(sq.cpu()))
    return sum(d2).numpy(), float(sum(nrm))


def _stats_host_slab(host, device, window=1 << 18):
    """The same statistics streaming a pinned host slab [N, P] through one GPU in column windows
    (the columns are independent: the average is per column, the distances sum over columns)."""
    from .slab import _copy2d
    n, p = host.shape
    w = min(window, p)
    buf = torch.empty((n, w), dtype=torch.float32, device=device)
    mean = torch.empty(w, dtype=torch.float32, device=device)
    dist2 = torch.empty(n, dtype=torch.float64, device=device)
    acc = torch.zeros(n, dtype=torch.float64, device=device)
    nrm = torch.zeros((), dtype=torch.float64, device=device)
    s = torch.cuda.current_stream(device)
    for c0 in range(0, p, w):
        cw = min(w, p - c0)
        _copy2d(buf.data_ptr(), w * 4, host.data_ptr() + c0 * 4, host.stride(0) * 4, cw * 4, n, 0, s)
        ops.mean_rows(buf[:, :cw], mean[:cw], dist2, ops.EXACT)
        acc += dist2
        nrm += torch.sum(mean[:cw].double() ** 2)
    return acc.cpu().numpy(), float(nrm.cpu())


def consensus_statistics(models, device=None):
    """(distances list, center norm) of Logger.log_consensus_distance for `models`."""
    models = list(models)
    res = _fresh_resident(models)
    if res is not None and res[1] == list(range(res[0].n)):
        d2, nrm = _stats_resident(res[0])
        last_source["consensus"] = "resident"
    else:
        dev = torch.device(device) if device is not None else \
            torch.device("cuda", torch.cuda.current_device())
        hs = _host_slab(models)
        from .d_sgd import synchronize
        synchronize()                      # the host slab must hold the last round's rows
        if hs is not None and hs[1] == list(range(hs[0].n)) and hs[0].host.is_pinned():
            d2, nrm = _stats_host_slab(hs[0].host, dev)
            last_source["consensus"] = "host-slab"
        else:
            from .model import consensus_distance
            _, d, norm = consensus_distance(models, device=dev)
            last_source["consensus"] = "stacked"
            return d, norm
    return np.sqrt(d2).tolist(), float(np.sqrt(nrm))


def consensus_distance_event(state):
    distances, norm = consensus_statistics([n["model"] for n in state["nodes"]])
    return {
        "type": "consensus-distance",
        "step": state["step"],
        "distance_to_center": {
            "global": {
                "avg": statistics.mean(distances),
                "std": statistics.stdev(distances) if len(distances) > 1 else 0.,
                "max": max(distances),
                "min": min(distances),
            }
        },
        "center": {"norm": norm},
        "timestamp": time.strftime("%Y-%m-%d-%H:%M:%S-%Z"),
    }


def log_consensus_distance(logger, state):
    """Logger.log_consensus_distance(self, state) on the GPU (same event, same file)."""
    ev = consensus_distance_event(state)
    with open(logger.global_events, "a") as events:
        events.write(json.dumps(ev) + "\n")


def install(logger_class):
    """Route a reference Logger class's log_consensus_distance through the GPU."""
    logger_class.log_consensus_distance = log_consensus_distance
    return logger_class


def _weights32(k, weights):
    if weights is None:
        weights = [float(1. / k) for _ in range(k)]   # model/__init__.py:17-18
    return np.asarray([float(v) for v in weights], np.float64).astype(np.float32)


def average(models, weights=None):
    """setup.model.average(models, weights) (tools/setup/model/__init__.py:15-25), bit for bit: a
    new model (deepcopy of models[0]) holding fl(..fl(models[0]*0 + w0*m0) + .. + w_{K-1}*m_{K-1}).
    Reads the resident output slab when the models are its rows (one AVERAGE_ONLY CSR row per GPU
    stripe, col = the models' rows, models[0] first), else stacks them (niidmix.model.average)."""
    models = list(models)
    if not models:
        raise ValueError("average() of no models")
    res = _fresh_resident(models)
    if res is None:
        from . import model as nm
        from .d_sgd import synchronize
        synchronize()
        last_source["average"] = "stacked"
        return guard.strip(nm.average(models, weights))
    rr, rows = res
    k = len(rows)
    w = _weights32(k, weights)
    flat = torch.empty(rr.p, dtype=torch.float32, pin_memory=True)
    evs = []
    for pt in rr.parts:
        x = pt["outs"][0]
        dev = pt["dev"]
        with torch.cuda.device(dev), torch.cuda.stream(pt["s_mix"]):
            out = torch.empty((1, x.shape[1]), dtype=torch.float32, device=dev)
            ops.mix_csr(x, torch.tensor([0, k], dtype=torch.int64, device=dev),
                        torch.tensor(rows, dtype=torch.int32, device=dev),
                        torch.from_numpy(w).to(dev), out, ops.EXACT | ops.AVERAGE_ONLY)
            flat[pt["c0"]:pt["c0"] + pt["w"]].copy_(out[0], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(pt["s_mix"])
            evs.append(ev)
    for ev in evs:
        ev.synchronize()
    last_source["average"] = "resident"
    from .model import unflatten_into
    center = guard.strip(copy.deepcopy(models[0]))
    return unflatten_into(center, flat)


def _enabled(params):
    if os.environ.get("NIIDMIX_GPU_LOGGER", "1") == "0":
        return False
    return params.get("algorithm", {}).get("gpu-logger", True) is not False


def install_hooks(params):
    """Called by niidmix.d_sgd.init.  When the reference driver's modules are loaded (run.py imports
    simulate.logger and setup.model before it imports the plugin), route
      Logger.log_consensus_distance            -> log_consensus_distance (always), and
      setup.model.average (Logger.state, :112) -> average (with log-global-model-accuracy).
    Returns the names patched.  Idempotent."""
    if not _enabled(params):
        return []
    done = []
    lg = sys.modules.get("simulate.logger")
    cls = getattr(lg, "Logger", None) if lg is not None else None
    if isinstance(cls, type):
        if cls.log_consensus_distance is not log_consensus_distance:
            install(cls)
        done.append("simulate.logger.Logger.log_consensus_distance")
    sm = sys.modules.get("setup.model")
    if params.get("logger", {}).get("log-global-model-accuracy") and sm is not None and \
            callable(getattr(sm, "average", None)):
        if sm.average is not average:
            sm.average = average
        done.append("setup.model.average")
    return done
