#!/usr/bin/env python
"""Per-rank round time of the column-stripe partition (niidmix.shard.StripedMixer) for N-GPU weak
scaling, emulated one rank at a time on ONE GPU (tuning tool, not the bench): for each world size,
rank r's stripe of the 1000*N-node d-cliques round, timed with HIP events.

    python tools/stripe_probe.py [--worlds 1,2,4,8] [--steps 20] [--interclique fully-connected]
                                 [--fixed 10000]    (strong scaling: the same N for every world)
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "non-iid-topology-simulator_amd"))
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--p", type=int, default=1 << 20)
    ap.add_argument("--interclique", default="fully-connected")
    ap.add_argument("--fixed", type=int, default=0, help="fixed node count (strong scaling)")
    ap.add_argument("--variant", action="append", default=[],
                    help="name:ENV=VAL,ENV2=VAL2 (kernel-library tuning env, interleaved per rank)")
    a = ap.parse_args()
    from niidmix.shard import StripedMixer
    dev = torch.device("cuda:0")
    for world in map(int, a.worlds.split(",")):
        for rank in sorted({0, world - 1}):
            sm = StripedMixer.dcliques(a.fixed or 1000 * world, 100, world, rank, a.interclique,
                                       dev, a.p)
            x = sm.empty().normal_()
            y = sm.empty()
            for rep in range(2 if a.variant else 1):
                for name, envd in [(n, dict(kv.split("=") for kv in e.split(",") if kv))
                                   for n, e in (v.split(":", 1) for v in a.variant)] or [("", {})]:
                    saved = {k: os.environ.get(k) for k in envd}
                    os.environ.update(envd)
                    for _ in range(3):
                        sm(x, y)
                    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    torch.cuda.synchronize()
                    s.record()
                    for _ in range(a.steps):
                        sm(x, y)
                        x, y = y, x
                    e.record()
                    torch.cuda.synchronize()
                    for k, v in saved.items():
                        if v is None:
                            os.environ.pop(k, None)
                        else:
                            os.environ[k] = v
                    ms = s.elapsed_time(e) / a.steps
                    alg = 2 * sm.n_total * sm.p_local * 4
                    print(f"world {world} rank {rank} {name}: N={sm.n_total} cols [{sm.c0},{sm.c1}) "
                          f"res/clique max {sm.mixer.plan.max_clique_res}  {ms:.4f} ms  "
                          f"{alg / ms / 1e6:.0f} GB/s  frac {alg / ms / 1e6 / 8000:.4f}", flush=True)
            del x, y, sm
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
