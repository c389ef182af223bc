#!/usr/bin/env python
"""Node-shard partition (niidmix.shard.ShardedMixer) of the fixed 10 000-node d-cliques problem,
emulated one rank at a time on ONE GPU (tuning tool, not the bench): per rank, the shard-local
mixing kernels over its K column windows (what the compute stream runs), and the halo volume the
RCCL exchange would carry; the xGMI time is predicted from the volume (7 links per GPU).

    python tools/shard_probe.py [--worlds 2,4,8] [--n 10000] [--interclique fully-connected]
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
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--n", type=int, default=10000)
    ap.add_argument("--p", type=int, default=1 << 20)
    ap.add_argument("--windows", type=int, default=8)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--interclique", default="fully-connected")
    ap.add_argument("--link-GBs", type=float, default=100.0,
                    help="assumed achievable xGMI bandwidth per link and direction")
    a = ap.parse_args()
    from niidmix.generate import dcliques_csr
    from niidmix.ops import Mixer
    from niidmix.shard import ShardPlan, window_layout
    dev = torch.device("cuda:0")
    csr, cliques = dcliques_csr(a.n, 100, a.interclique, 1337)
    k, w = window_layout(a.p, a.windows)
    for world in map(int, a.worlds.split(",")):
        plan = ShardPlan(csr, cliques, world)
        worst = None
        for rank in range(world):
            sh = plan.local(rank)
            m = Mixer(csr=sh.csr, cliques=sh.cliques, device=dev)
            x = torch.empty((k, sh.rows_in, w), device=dev).normal_()
            y = torch.empty((k, sh.rows_in, w), device=dev)
            kern = m.kernel_for("fast", x[0])

            def rnd():
                for kk in range(k):
                    cw = min(w, a.p - kk * w)
                    m(x[kk][:, :cw], out=y[kk][:sh.n_local, :cw], kernel=kern)
            rnd()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(a.steps):
                rnd()
            e.record()
            torch.cuda.synchronize()
            ms = s.elapsed_time(e) / a.steps
            recv = len(sh.halo) * a.p * 4
            per_peer = {}
            for q in sh.halo_owner.tolist():
                per_peer[q] = per_peer.get(q, 0) + a.p * 4
            link_ms = max(per_peer.values()) / (a.link_GBs * 1e9) * 1e3 if per_peer else 0.0
            print(f"world {world} rank {rank}: {sh.n_local} nodes + {len(sh.halo)} halo rows, "
                  f"kernel {kern} {ms:.3f} ms, halo recv {recv / 1e9:.2f} GB (max {max(per_peer.values(), default=0) / 1e9:.2f} GB "
                  f"from one peer -> {link_ms:.2f} ms at {a.link_GBs:.0f} GB/s per link)", flush=True)
            t = max(ms, link_ms)
            worst = t if worst is None else max(worst, t)
            del x, y, m
            torch.cuda.empty_cache()
        print(f"world {world}: predicted round max over ranks {worst:.3f} ms "
              f"(max of compute and per-link exchange, perfect overlap)", flush=True)


if __name__ == "__main__":
    main()
