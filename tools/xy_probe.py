#!/usr/bin/env python
"""Measurement tool (not product): which buffer's placement (input x or output y) decides the
clique kernel's speed?  Crosses 3 input and 3 output allocations in one process."""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "non-iid-topology-simulator_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from alloc_probe import timeit  # noqa: E402


def main():
    from niidmix import ops
    dev = torch.device("cuda:0")
    csr, cl, p, _ = bench.single_gpu_topology("dcliques1000")
    m = ops.Mixer(csr=csr, cliques=cl, device=dev)
    n = csr.n
    xs = [torch.randn(n, p, device=dev) for _ in range(3)]
    ys = [torch.empty(n, p, device=dev) for _ in range(3)]
    for i, x in enumerate(xs):
        row = []
        for j, y in enumerate(ys):
            row.append(statistics.median([timeit(m, x, y) for _ in range(3)]))
        print(f"x{i}: " + "  ".join(f"y{j} {t:.4f}" for j, t in enumerate(row)), flush=True)
    # copy rate of each buffer as source and destination (plain torch copy)
    for i, x in enumerate(xs):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ys[0].copy_(x)
        torch.cuda.synchronize()
        s.record()
        for _ in range(10):
            ys[0].copy_(x)
        e.record()
        torch.cuda.synchronize()
        print(f"copy x{i}->y0: {s.elapsed_time(e) / 10:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
