#!/usr/bin/env python
"""Device-resident layout A/B for the factored kernels (tuning tool, not the bench): one process,
variants interleaved, HIP-event timing of mix_blocked on VMM column-blocked slabs.

  --config fc1000      big-clique kernel, block widths (--blocks 32,64,128,256,1024)
  --config dcliques1000  register-tile clique kernel, block widths x row order (rank order vs
                       clique-contiguous rows: MixCSR.relabel)

    python tools/layout_probe.py --config fc1000 --blocks 32,128,1024 --reps 3
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "non-iid-topology-simulator_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="fc1000")
    ap.add_argument("--blocks", default="32,64,128,256,1024")
    ap.add_argument("--orders", default="rank,clique")
    ap.add_argument("--p", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    from niidmix import memory, ops
    from niidmix.topology import mh_csr
    dev = torch.device("cuda:0")
    if a.config == "fc1000":
        n = 1000
        csr = mh_csr(n, {i: [j for j in range(n) if j != i] for i in range(n)})
        cliques = None
        orders = ["rank"]
    elif a.config == "dcliques10000":
        from niidmix.generate import dcliques_csr
        csr, cliques = dcliques_csr(10000, 100, "fully-connected", 1337)
        n = csr.n
        orders = a.orders.split(",")
    else:
        g = np.load(os.path.join(REPO, "tests", "golden", "dcliques1000_fc_p64.npz"))
        csr = ops.csr_from_numpy(g["row_ptr"], g["col"], g["val"])
        f, cp = g["cliques_flat"], g["cliques_ptr"]
        cliques = [f[cp[i]:cp[i + 1]].tolist() for i in range(len(cp) - 1)]
        n = csr.n
        orders = a.orders.split(",")
    variants = []
    for order in orders:
        if order == "rank":
            c2, cl2 = csr, cliques
        else:                                    # clique-contiguous rows
            flat = [r for c in cliques for r in c]
            perm = np.empty(n, np.int64)
            perm[np.asarray(flat)] = np.arange(n)
            c2 = csr.relabel(perm)
            cl2 = [[int(perm[r]) for r in c] for c in cliques]
        m = ops.Mixer(csr=c2, cliques=cl2, device=dev)
        for b in map(int, a.blocks.split(",")):
            if m.plan.max_clique <= 256 and b < 64:
                continue
            variants.append((f"{order}/B{b}", m, b))
    res = {name: [] for name, _, _ in variants}
    for rep in range(a.reps):
        for name, m, b in variants:
            xa = memory.empty_blocked(n, a.p, dev, b)
            xa.normal_()
            xb = memory.empty_blocked(n, a.p, dev, b)
            for _ in range(3):
                m.mix_blocked(xa, xb, a.p)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.steps):
                m.mix_blocked(xa, xb, a.p)
                xa, xb = xb, xa
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.steps
            res[name].append(ms)
            print(f"rep {rep} {a.config} {name}: {ms:.4f} ms  frac {2 * n * a.p * 4 / ms / 1e6 / 8000:.4f}",
                  flush=True)
            del xa, xb
            torch.cuda.empty_cache()
    for name, v in res.items():
        print(f"SUMMARY {a.config} {name}: min {min(v):.4f} ms  mean {np.mean(v):.4f} ms", flush=True)


if __name__ == "__main__":
    main()
