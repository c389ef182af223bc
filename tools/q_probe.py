#!/usr/bin/env python
"""A/B of the multi-clique tile (k_mix_clique_q) against the one-clique register tile
(k_mix_clique) on many-clique d-cliques topologies (tuning tool, one process, interleaved).

    python tools/q_probe.py --n 10000 --p 1048576 --blocks 256,64 --variants old,8x13x4x13,16x7x8x2

Device layout as bench.py: clique-contiguous rows (Mixer.device_layout / relabeled), VMM
column-blocked slabs [P/B, N, B].  Variants: 'old' = NIIDMIX_CLIQUE_Q=1 (k_mix_clique), else a
NIIDMIX_CLIQUE_QT tile.  Every variant's output is compared with the first variant's (fast mode:
within 1e-5 of the |W|^T|X| bound on sampled blocks).
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "non-iid-topology-simulator_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def set_variant(v):
    if v == "old":
        os.environ["NIIDMIX_CLIQUE_Q"] = "1"
        os.environ.pop("NIIDMIX_CLIQUE_QT", None)
    else:
        os.environ["NIIDMIX_CLIQUE_Q"] = "4"
        os.environ["NIIDMIX_CLIQUE_QT"] = v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--p", type=int, default=1 << 20)
    ap.add_argument("--blocks", default="256")
    ap.add_argument("--variants", default="old,8x13x4x13")
    ap.add_argument("--interclique", default="fully-connected")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    from niidmix import memory, ops
    from niidmix.generate import dcliques_csr
    dev = torch.device("cuda:0")
    csr, cliques = dcliques_csr(a.n, 100, a.interclique, 1337)
    m = ops.Mixer(csr=csr, cliques=cliques, device=dev)
    perm, _ = m.device_layout()
    m = m.relabeled(perm)
    print(f"n={a.n} p={a.p} groups={m.plan.coef.shape[1] - 1} max_res={m.plan.max_clique_res}",
          flush=True)
    bound_w = np.abs(m.csr.val)
    for bc in [int(b) for b in a.blocks.split(",")]:
        xb = memory.empty_blocked(a.n, a.p, dev, bc)
        xb.normal_(generator=torch.Generator(device=dev).manual_seed(3))
        yb = memory.empty_blocked(a.n, a.p, dev, bc)
        ref = None
        times = {v: [] for v in a.variants.split(",")}
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        for rep in range(a.reps):
            for v in times:
                if v == "old" and bc < 256:
                    continue
                set_variant(v)
                m.mix_blocked(xb, yb, a.p)
                torch.cuda.synchronize()
                if rep == 0:
                    ks = [0, xb.shape[0] // 2, xb.shape[0] - 1]
                    got = [yb[k].cpu().numpy() for k in ks]
                    if ref is None:
                        ref = got
                        from oracle import oracle
                        for k, g in zip(ks, got):
                            xw = xb[k].cpu().numpy()
                            r = oracle.mix_exact_c(xw, m.csr.row_ptr, m.csr.col, m.csr.val)
                            bd = oracle.condition_bound(xw, m.csr.row_ptr, m.csr.col, bound_w)
                            ok, worst = oracle.check_tolerance(g, r, bd, rtol=1e-5)
                            print(f"  B={bc} {v} block {k} vs oracle: ok={ok} worst={worst:.2e}", flush=True)
                    else:
                        for g, r in zip(got, ref):
                            d = float(np.max(np.abs(g.astype(np.float64) - r)))
                            print(f"  B={bc} {v} vs first: max|diff| {d:.3e}", flush=True)
                s.record()
                for _ in range(a.iters):
                    m.mix_blocked(xb, yb, a.p)
                e.record()
                torch.cuda.synchronize()
                times[v].append(s.elapsed_time(e) / a.iters)
        alg = 2 * a.n * a.p * 4
        for v, ts in times.items():
            if ts:
                t = min(ts)
                gbs = alg / (t / 1e3) / 1e9                       # t in ms
                print(f"SUMMARY n={a.n} B={bc} {v}: min {t:.3f} ms mean {np.mean(ts):.3f} ms "
                      f"= {gbs:.0f} GB/s = {gbs / 8000:.3f} of 8 TB/s", flush=True)
        del xb, yb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
