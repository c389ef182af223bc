"""Node-state slab memory in HBM.

The [N, P] node slabs that stay resident in HBM are allocated by libniidmix's VMM allocator
(niidmix_hbm_alloc: a reserved VA range mapped from 2 MiB physical chunks) through a torch MemPool
with a pluggable allocator, so they are ordinary torch tensors.  The clique kernel's access pattern
(the rows of a clique at one column chunk, every clique of the chunk in flight together) measured
1.32 ms per headline round on every such slab, against 1.35-1.64 ms on hipMalloc'ed slabs
depending on where the driver placed them physically (tools/hbm_probe7.hip); linear copies are
unaffected.  Everything else keeps torch's default allocator.
"""
import contextlib
import ctypes

import torch

from . import _lib

_pools = {}


def slab_pool(device):
    """The MemPool of VMM-backed slabs on `device` (one per device, created on first use)."""
    device = torch.device(device)
    idx = device.index if device.index is not None else torch.cuda.current_device()
    pool = _pools.get(idx)
    if pool is None:
        alloc = torch.cuda.memory.CUDAPluggableAllocator(_lib.LIB_PATH, "niidmix_hbm_alloc",
                                                         "niidmix_hbm_free")
        pool = torch.cuda.MemPool(alloc.allocator())
        # process-lifetime objects: an extra reference that is never dropped, so neither is torn
        # down during interpreter shutdown while slab tensors (whose frees call into the allocator)
        # may still be alive; the driver reclaims the mappings at process exit
        for obj in (alloc, pool):
            ctypes.pythonapi.Py_IncRef(ctypes.py_object(obj))
        _pools[idx] = pool
    return pool


@contextlib.contextmanager
def slabs(device):
    """Allocations of torch tensors inside this context come from the slab pool of `device`."""
    with torch.cuda.device(torch.device(device)), torch.cuda.use_mem_pool(slab_pool(device)):
        yield


def empty_slab(rows, cols, device, dtype=torch.float32):
    """An uninitialised [rows, cols] tensor in VMM-backed slab memory on `device`."""
    with slabs(device):
        return torch.empty((rows, cols), dtype=dtype, device=device)


import os

BLOCK_COLS = int(os.environ.get("NIIDMIX_BLOCK_COLS", 1024))   # power of two >= 256


def empty_blocked(rows, p, device, block_cols=BLOCK_COLS):
    """An uninitialised COLUMN-BLOCKED slab [K, rows, block_cols] (K = ceil(p / block_cols)) in
    VMM-backed slab memory: the device-resident layout of node state for the clique kernel.
    Element (r, c) of the logical [rows, p] slab is x[c // block_cols, r, c % block_cols].  A
    clique's member rows are block_cols*4 bytes apart instead of p*4, which measured robust to the
    slab's physical placement (tools/hbm_probe7.hip)."""
    k = (p + block_cols - 1) // block_cols
    with slabs(device):
        return torch.empty((k, rows, block_cols), dtype=torch.float32, device=device)


def to_blocked(x, block_cols=BLOCK_COLS, out=None):
    """Row-major [rows, p] -> column-blocked [K, rows, block_cols] (padding columns zeroed)."""
    rows, p = x.shape
    if out is None:
        out = empty_blocked(rows, p, x.device, block_cols) if x.is_cuda else \
            torch.empty(((p + block_cols - 1) // block_cols, rows, block_cols), dtype=x.dtype)
    k = out.shape[0]
    for i in range(k):
        c0, c1 = i * block_cols, min(p, (i + 1) * block_cols)
        out[i, :, :c1 - c0].copy_(x[:, c0:c1])
        if c1 - c0 < block_cols:
            out[i, :, c1 - c0:].zero_()
    return out


def from_blocked(xb, p, out=None):
    """Column-blocked [K, rows, B] -> row-major [rows, p]."""
    k, rows, b = xb.shape
    if out is None:
        out = torch.empty((rows, p), dtype=xb.dtype, device=xb.device)
    for i in range(k):
        c0, c1 = i * b, min(p, (i + 1) * b)
        out[:, c0:c1].copy_(xb[i, :, :c1 - c0])
    return out
