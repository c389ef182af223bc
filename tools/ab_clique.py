"""A/B timing of k_mix_clique tile variants on ONE box, interleaved (measurement tool).

    python tools/ab_clique.py [--reps 5] [--iters 20] [--variants 16x7x8x0x0,16x7x8x0x2 ...]

Builds the headline topology (1000-node d-cliques, P = 2^20), then for each repetition times every
variant (NIIDMIX_CLIQUE_TILE, read by the library at each launch) over `iters` back-to-back
launches with HIP events, so box-to-box HBM variance cancels out of the comparison.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "non-iid-topology-simulator_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from niidmix import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--config", default="dcliques1000")
    ap.add_argument("--variants", default="16x7x8x0x0,16x7x8x0x2")
    ap.add_argument("--ld-pad", type=int, default=0)
    ap.add_argument("--env", default="NIIDMIX_CLIQUE_TILE",
                    help="environment variable the variants are assigned to (NIIDMIX_BIG for the "
                         "big-clique kernel)")
    ap.add_argument("--no-res", action="store_true",
                    help="timing experiment only (WRONG results): drop the residual terms")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    csr, cliques, p, _ = bench.single_gpu_topology(a.config)
    m = ops.Mixer(csr=csr, cliques=cliques, device=dev)
    n = csr.n
    if a.no_res:
        m.p_res_ptr.zero_()
    ld = p + a.ld_pad
    x = torch.randn(n, ld, device=dev)[:, :p]
    y = torch.empty(n, ld, device=dev)[:, :p]
    variants = a.variants.split(",")
    res = {v: [] for v in variants}
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for _ in range(a.reps):
        for v in variants:
            os.environ[a.env] = v
            for _ in range(3):
                m(x, out=y, kernel="clique")
            torch.cuda.synchronize()
            s.record()
            for i in range(a.iters):
                if i % 2 == 0:
                    m(x, out=y, kernel="clique")
                else:
                    m(y, out=x, kernel="clique")
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.iters
            res[v].append(ms)
    alg = 2.0 * n * p * 4
    for v in variants:
        t = np.array(res[v])
        print(f"{v:>16}  median {np.median(t):.4f} ms  min {t.min():.4f}  max {t.max():.4f}  "
              f"{alg / np.median(t) / 1e6:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
