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
