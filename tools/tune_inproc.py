#!/usr/bin/env python
"""In-process A/B timing of mixing-kernel variants on one slab (tuning tool, not product).

    python tools/tune_inproc.py [--config dcliques1000] [--p P] [--reps 3] [--steps 30]
        --variant name:ENV=VAL,ENV2=VAL2:kernel  ...

Variants are interleaved per repetition (rule: compare A/B in one process, interleaved) and the
median ms per round is printed with the HBM roofline fraction (2*N*P*4 bytes per round).
"""
import argparse
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "non-iid-topology-simulator_amd"))
import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="dcliques1000")
    ap.add_argument("--p", type=int, default=None)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--variant", action="append", default=[])
    a = ap.parse_args()
    from niidmix import ops
    dev = torch.device("cuda:0")
    csr, cl, p0, desc = bench.single_gpu_topology(a.config)
    p = a.p or p0
    m = ops.Mixer(csr=csr, cliques=cl, device=dev)
    from niidmix import memory
    if os.environ.get("TUNE_HIPMALLOC"):
        x = torch.randn(csr.n, p, device=dev)
        y = torch.empty_like(x)
    else:
        x = memory.empty_slab(csr.n, p, dev)
        x.normal_()
        y = memory.empty_slab(csr.n, p, dev)
    variants = []
    for v in a.variant or ["wave::clique"]:
        name, env, kernel = v.split(":")
        envd = dict(kv.split("=") for kv in env.split(",") if kv)
        variants.append((name, envd, kernel))
    mixers = {}

    plan_env = ("NIIDMIX_TILE_RT", "NIIDMIX_TILE_LDS_RT")

    def mixer_for(envd):
        key = tuple(envd.get(k) for k in plan_env)
        if all(v is None for v in key):
            return m
        if key not in mixers:
            saved = {k: os.environ.get(k) for k in plan_env}
            for k in plan_env:
                if envd.get(k) is not None:
                    os.environ[k] = envd[k]
            mixers[key] = ops.Mixer(csr=csr, cliques=cl, device=dev)
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
            t = mixers[key].tile
            if t is not None and key[0] is not None:
                print(f"tile rt={key[0]}: {t.n_sub} tiles, {t.n_pos} positions, density {t.density:.3f}")
            t = mixers[key].tlds
            if t is not None and key[1] is not None:
                print(f"lds tile rt={key[1]}: {t.tile.n_sub} tiles, {t.tile.n_pos} positions, "
                      f"density {t.tile.density:.3f}, max_src {t.max_src}, max_tiles {t.max_tiles}")
        return mixers[key]

    res = {n: [] for n, _, _ in variants}
    res["copy"] = []
    for rep in range(a.reps):
        for name, envd, kernel in variants:
            mm = mixer_for(envd)
            saved = {k: os.environ.get(k) for k in envd}
            os.environ.update(envd)
            for _ in range(3):
                mm(x, out=y, kernel=kernel)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.steps):
                mm(x, out=y, kernel=kernel)
            e.record()
            torch.cuda.synchronize()
            res[name].append(s.elapsed_time(e) / a.steps)
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v
        res["copy"].append(2 * x.numel() * 4 / (bench.stream_copy_probe(x.numel(), dev) * 1e9) * 1e3)
    alg = 2 * csr.n * p * 4
    print(f"config {a.config} N={csr.n} P={p}  ({desc})")
    for name, t in res.items():
        med = statistics.median(t)
        print(f"{name:24s} median {med:.4f} ms  [{', '.join(f'{v:.4f}' for v in t)}]  "
              f"{alg / med / 1e6:.1f} GB/s  frac {alg / med / 1e6 / 8000:.4f}")


if __name__ == "__main__":
    main()
