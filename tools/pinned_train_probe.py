#!/usr/bin/env python
"""Host-side probe (tuning tool, not the bench): does the CPU part of a D-SGD round train slower
when the models' parameters are views of one PINNED [N, P] host slab (the drop-in's NodeSlab) than
when they are separate tensors or views of a pageable slab?  N nodes train a Linear(1023, 1024)
(P = 2^20) for one batch-16 step each, rounds interleaved over the three layouts.

    python tools/pinned_train_probe.py [--nodes 1000] [--rounds 4]
"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nodes", type=int, default=1000)
    ap.add_argument("--rounds", type=int, default=4)
    a = ap.parse_args()
    torch.manual_seed(0)
    n, in_f, out_f, batch = a.nodes, 1023, 1024, 16
    p = in_f * out_f + out_f
    x, y = torch.randn(batch, in_f), torch.randint(0, out_f, (batch,))

    def models(slab):
        out = []
        for i in range(n):
            m = torch.nn.Linear(in_f, out_f)
            if slab is not None:
                off = 0
                for q in m.parameters():
                    v = slab[i, off:off + q.numel()].view_as(q)
                    v.copy_(q.detach())
                    q.data = v
                    off += q.numel()
            out.append((m, torch.optim.SGD(m.parameters(), lr=0.1)))
        return out

    layouts = {"separate": models(None),
               "pageable_slab": models(torch.empty(n, p)),
               "pinned_slab": models(torch.empty(n, p, pin_memory=True))}

    def rnd(ms):
        t = time.perf_counter()
        for m, opt in ms:
            opt.zero_grad()
            torch.nn.functional.cross_entropy(m(x), y).backward()
            opt.step()
        return time.perf_counter() - t

    res = {k: [] for k in layouts}
    for r in range(a.rounds + 1):
        for k, ms in layouts.items():
            t = rnd(ms)
            if r:
                res[k].append(t)
    print(f"threads {torch.get_num_threads()}, {n} nodes, P = {p}")
    for k, v in res.items():
        print(f"{k:14s} round median {sorted(v)[len(v) // 2] * 1e3:.1f} ms  min {min(v) * 1e3:.1f} ms")


if __name__ == "__main__":
    main()
