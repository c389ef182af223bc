"""Drop-in for setup.model.average (tools/setup/model/__init__.py:15-25) on the GPU.

average(models, weights=None) -> a new model (deepcopy of models[0]) holding
    fl(...fl(fl(models[0]*0) + fl(w_0*models[0])) + ... + fl(w_{K-1}*models[K-1]))
bit for bit, like the reference's deepcopy / mul_(0) / add_(w*p) loop.  weights=None means
float(1./len(models)) each, applied as an fp32 multiply (what ATen does with a Python scalar).
The K models are flattened (model.parameters() order) into a [K, P] device slab and reduced by the
exact CSR kernel with one output row (self = models[0] first, NIIDMIX_FLAG_AVERAGE_ONLY).
"""
import copy

import numpy as np
import torch

from . import ops


def flatten(models, device):
    rows = [torch.cat([q.detach().reshape(-1) for q in m.parameters()]) for m in models]
    return torch.stack(rows).to(device=device, dtype=torch.float32).contiguous()


def unflatten_into(model, flat):
    off = 0
    with torch.no_grad():
        for q in model.parameters():
            k = q.numel()
            q.copy_(flat[off:off + k].view_as(q))
            off += k
    return model


def average(models, weights=None, device=None):
    models = list(models)
    k = len(models)
    if k == 0:
        raise ValueError("average() of no models")
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if weights is None:
        weights = [float(1. / k) for _ in range(k)]
    w = np.asarray([float(v) for v in weights], np.float64).astype(np.float32)
    x = flatten(models, dev)
    out = torch.empty((1, x.shape[1]), dtype=torch.float32, device=dev)
    row_ptr = torch.tensor([0, k], dtype=torch.int64, device=dev)
    col = torch.arange(k, dtype=torch.int32, device=dev)
    val = torch.from_numpy(w).to(dev)
    ops.mix_csr(x, row_ptr, col, val, out, ops.EXACT | ops.AVERAGE_ONLY)
    center = copy.deepcopy(models[0])
    return unflatten_into(center, out[0].cpu())


def consensus_distance(models, device=None):
    """Logger.log_consensus_distance (logger.py:257-284) statistics on the GPU: the uniform average
    (exact kernel) and every model's L2 distance to it (fp64 accumulation).  Returns
    (center_flat_cpu, distances list, center_norm)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    x = flatten(models, dev)
    mean = torch.empty(x.shape[1], dtype=torch.float32, device=dev)
    dist2 = torch.empty(x.shape[0], dtype=torch.float64, device=dev)
    ops.mean_rows(x, mean, dist2, ops.EXACT)
    d = torch.sqrt(dist2).cpu().tolist()
    norm = float(torch.sqrt(torch.sum(mean.double() ** 2)).item())
    return mean.cpu(), d, norm
