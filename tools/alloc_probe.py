#!/usr/bin/env python
"""Measurement tool (not product): does the clique kernel's time depend on the slab ALLOCATION
(physical placement) rather than the box?  Times the headline kernel on several fresh
allocations of x/y in one process, and on row-padded slabs (ld = P + pad)."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "non-iid-topology-simulator_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def timeit(m, x, y, steps=20, skew=None, tile=None):
    if skew is not None:
        os.environ["NIIDMIX_CLIQUE_SKEW"] = str(skew)
    if tile is not None:
        if tile:
            os.environ["NIIDMIX_CLIQUE_TILE"] = tile
        else:
            os.environ.pop("NIIDMIX_CLIQUE_TILE", None)
    for _ in range(3):
        m(x, out=y, kernel="clique")
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(steps):
        m(x, out=y, kernel="clique")
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / steps


def main():
    from niidmix import ops
    dev = torch.device("cuda:0")
    csr, cl, p, _ = bench.single_gpu_topology("dcliques1000")
    m = ops.Mixer(csr=csr, cliques=cl, device=dev)
    n = csr.n
    keep = []
    from niidmix import memory
    vmm = bool(os.environ.get("ALLOC_VMM"))
    for i in range(int(os.environ.get("ALLOCS", "4"))):
        if vmm:
            x = memory.empty_slab(n, p, dev)
            x.normal_()
            y = memory.empty_slab(n, p, dev)
        else:
            x = torch.randn(n, p, device=dev)
            y = torch.empty_like(x)
        for sk in [int(v) for v in os.environ.get("SKEWS", "0").split(",")]:
            for tl in os.environ.get("TILES", "").split(","):
                t = [timeit(m, x, y, skew=sk, tile=tl) for _ in range(3)]
                print(f"alloc {i} skew {sk:5d} tile {tl or 'default':18s}: x at {x.data_ptr():#x}  "
                      f"median {statistics.median(t):.4f} ms", flush=True)
        keep.append((x, y))                 # keep alive: the next allocation lands elsewhere
        if i == 1:
            keep = keep[-1:]
    del keep
    torch.cuda.empty_cache()
    pads = [int(v) for v in os.environ.get("PADS", "").split(",") if v]
    for rep in range(int(os.environ.get("PAD_REPS", "1"))):
        hold = []
        for pad in pads:
            x = torch.randn(n, p + pad, device=dev)[:, :p]
            y = torch.empty(n, p + pad, device=dev)[:, :p]
            t = [timeit(m, x, y) for _ in range(3)]
            print(f"rep {rep} pad {pad:6d}: median {statistics.median(t):.4f} ms  {t}", flush=True)
            hold.append((x, y))             # keep alive: fresh physical placement every time
            if len(hold) > 2:
                hold.pop(0)
        del hold
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
