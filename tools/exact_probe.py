#!/usr/bin/env python
"""Exact-mode (bit-identical) round A/B on the headline topology (tuning tool, not the bench): the
LDS-staged merged-order tile kernel at tile heights --rts (RT 16: matrix-core path "mfma", segment
walker "seg" and per-position loop "pos"), interleaved in one process; results of
every variant are checked bitwise against the first (--no-check for the phase-split builds of
tools/tlds_split.sh, whose results are not the mix).

    python tools/exact_probe.py [--rts 8,16] [--reps 2] [--order clique|rank]
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
    ap.add_argument("--rts", default="8,16")
    ap.add_argument("--p", type=int, default=1 << 20)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--order", default="clique", choices=["rank", "clique"])
    ap.add_argument("--no-check", action="store_true", help="phase-split builds: results are not the mix")
    ap.add_argument("--mf-items", default="",
                    help="comma list of k: also time the matrix-core path on every k-th column "
                         "chunk (NIIDMIX_TLDS_MF_WAVES=-k), the segment walker on the others")
    ap.add_argument("--metas", default="mfma,seg,pos",
                    help="RT 16 variants to time: mfma, seg (segment walker), seg16 (walker without "
                         "its 8- / 4-row loops, NIIDMIX_TLDS_SMALL=0), pos (per-position loop), "
                         "rem8 / rem16 (walker with register rows, 8 / 16 per tile)")
    ap.add_argument("--lds-rows", type=int, default=0,
                    help="occupancy probe: reserve LDS for this many staged rows (max_src) per block")
    a = ap.parse_args()
    from niidmix import memory, ops
    dev = torch.device("cuda:0")
    g = np.load(os.path.join(REPO, "tests", "golden", "dcliques1000_fc_p64.npz"))
    csr = ops.csr_from_numpy(g["row_ptr"], g["col"], g["val"])
    f, cp = g["cliques_flat"], g["cliques_ptr"]
    cliques = [f[cp[i]:cp[i + 1]].tolist() for i in range(len(cp) - 1)]
    base = ops.Mixer(csr=csr, cliques=cliques, device=dev)
    if a.order == "clique":
        perm, _ = base.device_layout()
        csr = csr.relabel(perm)
        cliques = [[int(perm[r]) for r in c] for c in cliques]
    mixers = {}
    rem_mixer, rem_natural = None, 16
    for rt in a.rts.split(","):
        os.environ["NIIDMIX_TILE_LDS_RT"] = rt
        os.environ["NIIDMIX_TLDS_REMOTE"] = "0"          # all staged; rem8 / rem16 below
        m = ops.Mixer(csr=csr, cliques=cliques, device=dev)
        assert m.tlds is not None, m.tlds_reason
        os.environ.pop("NIIDMIX_TLDS_REMOTE")
        if a.lds_rows:
            m.tlds.max_src = max(m.tlds.max_src, a.lds_rows)
        mixers[int(rt)] = m
        if rt == "16" and any(k.startswith("rem") for k in a.metas.split(",")):
            os.environ["NIIDMIX_TLDS_REMOTE"] = "1"
            mr = ops.Mixer(csr=csr, cliques=cliques, device=dev)
            assert mr.tlds is not None and mr.tlds.rem_rows is not None, mr.tlds_reason
            os.environ.pop("NIIDMIX_TLDS_REMOTE")
            print(f"register-row plan: {mr.tlds.max_src} staged rows (all staged: {m.tlds.max_src}), "
                  f"rem_regs {mr.tlds.rem_regs}", flush=True)
            rem_mixer, rem_natural = mr, mr.tlds.rem_regs
    n = csr.n
    x = memory.empty_slab(n, a.p, dev)
    x.normal_(generator=torch.Generator(device=dev).manual_seed(0))
    y = memory.empty_slab(n, a.p, dev)
    ref = None
    res = {}
    for rep in range(a.reps):
        for rt, m in mixers.items():
            metas = a.metas.split(",") + [f"mfitem{k}" for k in a.mf_items.split(",") if k]
            for meta in (metas if rt == 16 else ("pos",)):
                if meta.startswith("rem"):
                    m = rem_mixer
                    if int(meta[3:]) < rem_natural:
                        continue                          # the plan has tiles with more rows
                    m.tlds.rem_regs = int(meta[3:])      # 16: the 16-register kernel on the same plan
                else:
                    m = mixers[rt]
                m.use_segments = meta != "pos"
                m.use_mfma = meta.startswith("mf")
                if meta.startswith("mfitem"):
                    os.environ["NIIDMIX_TLDS_MF_WAVES"] = "-" + meta[6:]
                else:
                    os.environ.pop("NIIDMIX_TLDS_MF_WAVES", None)
                if meta == "seg16":
                    os.environ["NIIDMIX_TLDS_SMALL"] = "0"
                else:
                    os.environ.pop("NIIDMIX_TLDS_SMALL", None)
                m(x, out=y, kernel="tile-lds-exact")
                torch.cuda.synchronize()
                if ref is None:
                    ref = y[:, :65536].clone()
                elif not a.no_check:
                    assert torch.equal(y[:, :65536], ref), (rt, meta)
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(a.steps):
                    m(x, out=y, kernel="tile-lds-exact")
                e.record()
                torch.cuda.synchronize()
                ms = s.elapsed_time(e) / a.steps
                res.setdefault(f"rt{rt}/{meta}", []).append(ms)
                print(f"rep {rep} rt {rt} meta {meta}: {ms:.3f} ms", flush=True)
    for k, v in res.items():
        print(f"SUMMARY exact {a.order} {k}: min {min(v):.3f} ms mean {np.mean(v):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
