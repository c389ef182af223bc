#!/usr/bin/env python
"""Measurement tool (not product): the clique kernel on a column-BLOCKED device slab.

Layout [K, N, B] (K = P / B column blocks, each a row-major [N, B] slab with ld = B): a clique item
then reads its 100 member rows at a B*4-byte stride instead of P*4 = 4 MiB, so one item touches
far fewer (2 MiB) pages.  Times K back-to-back launches (one per block) against the plain
row-major [N, P] launch, interleaved, same process.
"""
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "non-iid-topology-simulator_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    from niidmix import ops
    dev = torch.device("cuda:0")
    csr, cl, p, _ = bench.single_gpu_topology(sys.argv[1] if len(sys.argv) > 1 else "dcliques1000")
    m = ops.Mixer(csr=csr, cliques=cl, device=dev)
    n = csr.n
    x = torch.randn(n * p, device=dev)
    y = torch.empty_like(x)
    steps = 10
    res = {}
    for rep in range(3):
        for b in [p, p >> 2, p >> 4, p >> 6, p >> 8]:
            k = p // b
            xs = [x[i * n * b:(i + 1) * n * b].view(n, b) for i in range(k)]
            ys = [y[i * n * b:(i + 1) * n * b].view(n, b) for i in range(k)]
            for _ in range(2):
                for i in range(k):
                    m(xs[i], out=ys[i], kernel="clique")
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(steps):
                for i in range(k):
                    m(xs[i], out=ys[i], kernel="clique")
            e.record()
            torch.cuda.synchronize()
            res.setdefault(b, []).append(s.elapsed_time(e) / steps)
    alg = 2 * n * p * 4
    for b, t in res.items():
        med = statistics.median(t)
        print(f"B={b:8d} K={p // b:4d}  median {med:.4f} ms  {alg / med / 1e6:.1f} GB/s  "
              f"frac {alg / med / 1e6 / 8000:.4f}  [{', '.join(f'{v:.4f}' for v in t)}]", flush=True)


if __name__ == "__main__":
    main()
