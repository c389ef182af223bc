"""SHA-256 digests of a d-cliques topology (shared by make_digests.py, which applies it to the
REFERENCE generator's output, and tests/test_generate.py, which applies it to niidmix.generate).

A digest covers what the mixing round consumes, without storing it:
  cliques   the clique member lists in order (json)
  edges     edges[rank] for rank = 0..N-1, each list in its own order (json)
  row_ptr   int64 CSR row pointers of W^T, row i = [i] + edges[i]   (d_sgd.py:105-110)
  val       the fp32 bits of W[src, i] over that CSR (little-endian uint32)
"""
import hashlib
import json

import numpy as np


def _sha(b):
    return hashlib.sha256(b).hexdigest()


def digest(cliques, edges, row_ptr, val):
    n = len(edges)
    return {
        "n": n,
        "nnz": int(row_ptr[-1]),
        "cliques": _sha(json.dumps([[int(v) for v in c] for c in cliques]).encode()),
        "edges": _sha(json.dumps([[int(v) for v in edges[r]] for r in range(n)]).encode()),
        "row_ptr": _sha(np.ascontiguousarray(row_ptr, dtype="<i8").tobytes()),
        "val": _sha(np.ascontiguousarray(val, dtype="<f4").view("<u4").tobytes()),
    }
