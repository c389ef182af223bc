#!/usr/bin/env python
"""Digest fixtures of BASELINE configs[4]'s topology, made by the REFERENCE generator itself.

Run in the development container only (it imports /root/reference; the GPU box never runs it):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_digests.py

For each case the reference's own code builds the d-cliques topology:
  random_cliques.cliques   (tools/setup/topology/d_cliques/random_cliques.py:18-37, seed 1337)
  interclique.get(name)    (interclique.py:57-75 fully-connected, :81-119 smallworld)
  weights.compute_weights  (tools/setup/topology/weights.py:3-32, Metropolis-Hastings, fp32)
and the CSR of W^T in d_sgd.average's operand order (row i = [i] + edges[i], value W[src, i],
d_sgd.py:105-110) is hashed with tests/golden/topo_digest.py.  At 10 000 nodes the dense
topology.json would be ~1 GB, so only the SHA-256 digests are committed
(tests/golden/dcliques_digests.json); tests/test_generate.py recomputes them from
niidmix.generate.dcliques_csr.  compute_weights' output goes into the CSR as the loader would
read it (json floats of fp32 values -> torch fp32: exact), without the JSON round trip.
"""
import json
import os
import sys
import time

import numpy as np

OUT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, OUT)

CASES = [
    # (n, clique size, interclique): configs[4] (10 000 nodes, the reference default interclique),
    # the weak N=8 line's 8 000 nodes, and configs[4] under smallworld
    (10000, 100, "fully-connected"),
    (8000, 100, "fully-connected"),
    (10000, 100, "smallworld"),
]


def main():
    import make_golden as G
    from topo_digest import digest
    out = {"generator": "reference random_cliques.cliques + interclique.get + "
                        "weights.compute_weights (metropolis-hasting), seed 1337",
           "cases": {}}
    for n, size, inter in CASES:
        t0 = time.time()
        edges, cliques = G.dcliques(n, size, inter)
        W = G.R.weights.compute_weights(G._nodes(n), edges, G.MH)     # list[N][N] of fp32 values
        row_ptr = [0]
        val = []
        for r in range(n):
            srcs = [r] + list(edges[r])
            val += [W[s][r] for s in srcs]
            row_ptr.append(len(val))
        del W
        d = digest(cliques, edges, np.asarray(row_ptr, np.int64), np.asarray(val, np.float32))
        out["cases"][f"dcliques{n}_{size}_{inter}"] = dict(d, clique_size=size, interclique=inter,
                                                           seed=1337)
        print(f"n={n} {inter}: nnz={d['nnz']} ({time.time() - t0:.0f} s)", flush=True)
    with open(os.path.join(OUT, "dcliques_digests.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
