#!/usr/bin/env python
"""ring100 (P = 62 006) round time per band-kernel shape (rows x column chunks per wave), the ELL
kernel, the column-strip kernel and the stream copy of the same slab, each as bench.py times it: K rounds in ONE hipGraph,
replayed (tuning tool).

    python tools/band_probe.py [--rc 1,1:1,2:2,2:4,4] [--steps 20] [--reps 5]
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "non-iid-topology-simulator_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def graph_round_us(step, a, b, steps, reps):
    step(a, b)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        x, y = a, b
        for _ in range(steps):
            step(x, y)
            x, y = y, x
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        g.replay()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / steps)
    return min(ts), float(np.median(ts))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rc", default="1,1:1,2:1,4:2,1:2,2:4,1:4,4:8,2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--p", type=int, default=62006)
    a = ap.parse_args()
    from bench import golden
    from niidmix import _lib, memory, ops
    dev = torch.device("cuda:0")
    csr, _ = golden("ring100_p257")
    m = ops.Mixer(csr=csr, device=dev)
    perm, _ = m.device_layout()
    mr = m.relabeled(perm)
    n, p = csr.n, a.p
    xa = memory.empty_slab(n, p, dev)
    xa.normal_(generator=torch.Generator(device=dev).manual_seed(1))
    xb = memory.empty_slab(n, p, dev)
    print(f"ring {n} x P={p}, {a.steps} rounds per hipGraph replay, min / median of {a.reps} replays")
    for rc in a.rc.split(":"):
        os.environ["NIIDMIX_BAND_RC"] = rc
        us = graph_round_us(lambda x, y: mr(x, out=y, kernel="band-fast"), xa, xb, a.steps, a.reps)
        print(f"band R,CH={rc:4s}  {us[0]:7.2f} / {us[1]:7.2f} us per round")
    os.environ.pop("NIIDMIX_BAND_RC", None)
    for ch in ("1", "2", "4"):
        os.environ["NIIDMIX_ELL_CH"] = ch
        us = graph_round_us(lambda x, y: m(x, out=y, kernel="ell-fast"), xa, xb, a.steps, a.reps)
        print(f"ell CH={ch}         {us[0]:7.2f} / {us[1]:7.2f} us per round (rank order)")
    os.environ.pop("NIIDMIX_ELL_CH", None)
    for mode, kname in (("fast", "strip-fast"), ("exact", "strip-exact")):
        us = graph_round_us(lambda x, y: mr(x, out=y, kernel=kname), xa, xb, a.steps, a.reps)
        print(f"strip {mode:5s}       {us[0]:7.2f} / {us[1]:7.2f} us per round (column strips in LDS)")
    # rows on a 256-B pitch (ld = p rounded up to 64 floats): every wave's 256-B row piece is then
    # whole cache lines (ld = p = 62 006 floats puts row r at 216 r mod 256 B)
    ldp = -(-p // 64) * 64
    pa = torch.empty((n, ldp), device=dev)
    pa[:, :p].copy_(xa)
    pb = torch.empty((n, ldp), device=dev)
    va, vb = pa[:, :p], pb[:, :p]
    for kname in ("strip-fast", "band-fast", "ell-fast"):
        mm = m if kname == "ell-fast" else mr
        us = graph_round_us(lambda x, y: mm(x, out=y, kernel=kname), va, vb, a.steps, a.reps)
        print(f"{kname:10s} ld={ldp} {us[0]:7.2f} / {us[1]:7.2f} us per round (256-B row pitch)")
    for sv in ("4", "1"):
        for sw in ("4", "8", "16"):
            os.environ["NIIDMIX_STRIP_SV"], os.environ["NIIDMIX_STRIP_SW"] = sv, sw
            us = graph_round_us(lambda x, y: mr(x, out=y, kernel="strip-fast"), va, vb, a.steps,
                                a.reps)
            print(f"strip SV={sv} SW={sw:2s} ld={ldp} {us[0]:7.2f} / {us[1]:7.2f} us per round")
    os.environ.pop("NIIDMIX_STRIP_SV")
    os.environ.pop("NIIDMIX_STRIP_SW")
    # the strip kernel's result against the band kernel's (exact: bitwise)
    ya, yb = torch.empty_like(xa), torch.empty_like(xa)
    mr(xa, out=ya, kernel="band-exact")
    mr(xa, out=yb, kernel="strip-exact")
    torch.cuda.synchronize()
    print("strip-exact == band-exact:", bool(torch.equal(ya, yb)))
    numel = n * p - (n * p) % 4
    fa, fb = xa.view(-1)[:numel], xb.view(-1)[:numel]

    def cp(x, y):
        _lib.check(_lib.lib.niidmix_stream_copy_f32(x.data_ptr(), y.data_ptr(), numel,
                   ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "copy")
    us = graph_round_us(cp, fa, fb, a.steps, a.reps)
    print(f"stream copy       {us[0]:7.2f} / {us[1]:7.2f} us per copy of the slab")


if __name__ == "__main__":
    main()
