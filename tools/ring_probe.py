#!/usr/bin/env python
"""ring100 launch-path probe (measurement tool): the CSR round launched (a) through ctypes with
pre-bound arguments back to back, (b) through the Mixer (validation + dispatch per call) back to
back, (c) through the Mixer captured in a hipGraph, and (d) the stream copy of the same slab.

    python tools/ring_probe.py [--iters 500]
"""
import argparse
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "non-iid-topology-simulator_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from niidmix import _lib, ops  # noqa: E402


def timed(fn, iters):
    for _ in range(20):
        fn(0)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for i in range(iters):
        fn(i)
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=500)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    csr, cl, p, _ = bench.single_gpu_topology("ring100")
    m = ops.Mixer(csr=csr, cliques=cl, device=dev)
    n = csr.n
    x = torch.randn(n, p, device=dev)
    y = torch.empty_like(x)
    strm = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    f = _lib.lib.niidmix_mix_csr_f32
    mode = ops.FAST | ops.LOW_DEGREE
    args = [(x.data_ptr(), p, y.data_ptr(), p, n, p, m.row_ptr.data_ptr(), m.col.data_ptr(),
             m.val.data_ptr(), mode, strm),
            (y.data_ptr(), p, x.data_ptr(), p, n, p, m.row_ptr.data_ptr(), m.col.data_ptr(),
             m.val.data_ptr(), mode, strm)]
    t_raw = timed(lambda i: f(*args[i & 1]), a.iters)
    t_mixer = timed(lambda i: m(x, out=y, kernel="csr-fast") if i % 2 == 0 else m(y, out=x, kernel="csr-fast"), a.iters)
    t_graph = {}
    for kern in ("csr-fast", "ell-fast", "csr-exact", "ell-exact"):
        for ch in (["4", "2", "1"] if kern.startswith("ell") else [""]):
            os.environ["NIIDMIX_ELL_CH"] = ch or "4"
            g = torch.cuda.CUDAGraph()
            m(x, out=y, kernel=kern)
            torch.cuda.synchronize()
            with torch.cuda.graph(g):
                for i in range(50):
                    if i % 2 == 0:
                        m(x, out=y, kernel=kern)
                    else:
                        m(y, out=x, kernel=kern)
            t_graph[kern + (f"/ch{ch}" if ch else "")] = timed(lambda i: g.replay(), max(1, a.iters // 50)) / 50
    # the LDS-staged tiles on the ring (groups of consecutive rows, each source row staged once per
    # group instead of gathered by ~3 waves)
    os.environ["NIIDMIX_TLDS_ANY_DEGREE"] = "1"
    m2 = ops.Mixer(csr=csr, cliques=cl, device=dev)
    assert m2.tlds is not None, m2.tlds_reason
    for kern in ("tile-lds-fast", "tile-lds-exact"):
        g = torch.cuda.CUDAGraph()
        m2(x, out=y, kernel=kern)
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            for i in range(50):
                if i % 2 == 0:
                    m2(x, out=y, kernel=kern)
                else:
                    m2(y, out=x, kernel=kern)
        t_graph[kern] = timed(lambda i: g.replay(), max(1, a.iters // 50)) / 50
    numel = n * p - (n * p) % 4
    xa, ya = x.view(-1)[:numel], y.view(-1)[:numel]
    cp = _lib.lib.niidmix_stream_copy_f32
    t_copy = timed(lambda i: cp(xa.data_ptr(), ya.data_ptr(), numel, strm), a.iters)
    print(f"ring100 N={n} P={p}: raw ctypes csr {t_raw:.2f} us  mixer csr {t_mixer:.2f} us  "
          f"stream copy {t_copy:.2f} us")
    for k, v in t_graph.items():
        print(f"  hipGraph {k}: {v:.2f} us per round")


if __name__ == "__main__":
    main()
