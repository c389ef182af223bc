"""Topology boundary: topology.json -> the CSR of W^T that the mixing kernels consume.

Mirrors the reference reader and weight builder:
  load(rundir)          setup.topology.load      tools/setup/topology/__init__.py:4-12
  metropolis_hastings   compute_weights (MH)     tools/setup/topology/weights.py:3-32
and adds what the GPU path needs:
  MixCSR / to_csr       row i = [i] + edges[i] with values W[i,i], W[src,i] — exactly the operand
                        order d_sgd.average feeds setup.model.average (d_sgd.py:105-106), so the
                        exact kernel reproduces the reference's summation order.
  mh_csr                sparse Metropolis-Hastings straight to CSR (no dense N x N JSON; §8(f) row 4),
                        bit-identical to compute_weights.
  save_csr / load_csr   a sparse companion file for large N (topology.csr.npz).

topology.json format (doc/experiment.md, ring.py:52-58): {"edges": {"<rank>": [int...]},
"weights": [[float]*N]*N, "cliques"?: [[int]], "neighbourhoods"?: {"<rank>": [int]}}.
"""
import json
import os
from dataclasses import dataclass

import numpy as np
import torch


def load_file(path):
    """Read a topology.json file with setup.topology.load's conversions (topology/__init__.py:4-12):
    edge keys -> int (list order preserved), weights -> fp32 torch tensor [N, N], neighbourhood keys
    -> int."""
    with open(path, "r") as f:
        topology = json.load(f)
    edges = topology["edges"]
    topology["edges"] = {int(rank): edges[rank] for rank in edges}
    topology["weights"] = torch.tensor(topology["weights"])
    if "neighbourhoods" in topology:
        ns = topology["neighbourhoods"]
        topology["neighbourhoods"] = {int(rank): ns[rank] for rank in ns}
    return topology


def load(rundir):
    """Drop-in for setup.topology.load(rundir).  If the rundir holds a sparse companion
    (topology.csr.npz, written by save_csr / niidmix.sparse_topology) that is newer than
    topology.json (or there is no topology.json), the sparse form is returned under
    topology['csr'] (weights None) with 'edges' rebuilt from it."""
    path = os.path.join(rundir, "topology.json")
    sparse = os.path.join(rundir, "topology.csr.npz")
    if os.path.exists(path) and not (os.path.exists(sparse) and
                                     os.path.getmtime(sparse) > os.path.getmtime(path)):
        return load_file(path)
    if os.path.exists(sparse):
        csr, cliques = load_csr(sparse)
        topo = {"edges": csr.edges(), "csr": csr, "weights": None}
        if cliques is not None:
            topo["cliques"] = cliques
        return topo
    raise FileNotFoundError(path)


@dataclass
class MixCSR:
    """CSR of W^T rows: row i lists (src, W[src, i]) with the node itself first, then edges[i] in
    list order.  row_ptr int64 [N+1], col int32 [nnz], val fp32 [nnz].  n_in (default N) is the
    number of input rows the columns index: a node shard's CSR also reads halo rows >= N."""
    row_ptr: np.ndarray
    col: np.ndarray
    val: np.ndarray
    n_in: int = None

    def __post_init__(self):
        if self.n_in is None:
            self.n_in = len(self.row_ptr) - 1

    @property
    def n(self):
        return len(self.row_ptr) - 1

    @property
    def nnz(self):
        return int(self.row_ptr[-1])

    def degrees(self):
        """len(edges[i]) for every node (self entry excluded)."""
        return np.diff(self.row_ptr) - 1

    def edges(self):
        out = {}
        for i in range(self.n):
            b, e = int(self.row_ptr[i]), int(self.row_ptr[i + 1])
            out[i] = [int(c) for c in self.col[b + 1:e]]
        return out

    def dense(self):
        """W as the reference stores it: dense[src, dst] (fp32), [n_in, n]."""
        n = self.n
        w = np.zeros((self.n_in, n), np.float32)
        dst = np.repeat(np.arange(n), np.diff(self.row_ptr))
        w[self.col, dst] = self.val
        return w

    def relabel(self, perm):
        """The same operator with node i stored at slab row perm[i] (a device-resident row order,
        e.g. clique-contiguous): row perm[i] of the result lists (perm[src], W[src, i]) in the same
        operand order, so every output is computed exactly as before, only stored elsewhere."""
        perm = np.asarray(perm, np.int64)
        n = self.n
        if self.n_in != n or sorted(perm.tolist()) != list(range(n)):
            raise ValueError("relabel needs a permutation of the N rows (no halo rows)")
        inv = np.empty(n, np.int64)
        inv[perm] = np.arange(n)
        lens = np.diff(self.row_ptr)[inv]
        row_ptr = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
        idx = np.concatenate([np.arange(self.row_ptr[i], self.row_ptr[i + 1]) for i in inv]) \
            if n else np.zeros(0, np.int64)
        return MixCSR(row_ptr, perm[self.col[idx]].astype(np.int32), self.val[idx].copy()).validate()

    def validate(self):
        n = self.n
        if self.row_ptr[0] != 0 or np.any(np.diff(self.row_ptr) < 1):
            raise ValueError("every CSR row must start with the node itself")
        if len(self.col) != self.nnz or len(self.val) != self.nnz:
            raise ValueError("col/val length != row_ptr[-1]")
        if np.any(self.col[self.row_ptr[:-1]] != np.arange(n)):
            raise ValueError("first entry of row i must be i (the reference's models[0] = self)")
        if self.nnz and (self.col.min() < 0 or self.col.max() >= self.n_in):
            raise ValueError("column index out of range")
        return self


def to_csr(topology):
    """CSR of W^T in d_sgd.average's operand order (d_sgd.py:105-106)."""
    if "csr" in topology and topology.get("weights") is None:
        return topology["csr"]
    W = topology["weights"]
    Wn = W.numpy() if isinstance(W, torch.Tensor) else np.asarray(W, np.float32)
    Wn = np.asarray(Wn, np.float32)
    edges = topology["edges"]
    n = Wn.shape[0]
    counts = np.empty(n, np.int64)
    cols = []
    for rank in range(n):
        e = edges[rank]                      # KeyError for a missing rank, as the reference
        counts[rank] = 1 + len(e)
        cols.append(np.asarray([rank] + list(e), np.int64))
    col = np.concatenate(cols) if cols else np.zeros(0, np.int64)
    dst = np.repeat(np.arange(n), counts)
    val = Wn[col, dst].astype(np.float32)
    row_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    return MixCSR(row_ptr, col.astype(np.int32), val).validate()


def metropolis_hastings(n, edges):
    """compute_weights(..., {'weights': 'metropolis-hasting'}) (weights.py:15-25), dense fp32 [N,N],
    bit-identical: off-diagonals 1./(max(d_i, d_j)+1) rounded to fp32, then W[i,i] = 1. - W[i,:].sum()
    with the same torch fp32 row reduction."""
    w = torch.zeros((n, n))
    deg = [len(edges[i]) for i in range(n)]
    for i in range(n):
        for j in edges[i]:
            if j != i:
                w[i, j] = 1. / (max(deg[i], deg[j]) + 1)
    for i in range(n):
        w[i, i] = 1. - w[i, :].sum()
    _check_stochastic(w)
    return w


def _check_stochastic(w):
    # weights.py:28-30 (one-sided, as in the reference)
    eps = torch.finfo(torch.float32).eps
    assert all((w.sum(axis=0) - 1.0) < 10 * eps), \
        "Weights should sum to 1. Sum is off by {}".format(w.sum(axis=0) - 1.0)
    assert all((w.sum(axis=1) - 1.0) < 10 * eps), \
        "Weights should sum to 1. Sum is off by {}".format(w.sum(axis=1) - 1.0)


def mh_csr(n, edges):
    """Sparse Metropolis-Hastings straight to the mixing CSR, without materialising the N x N JSON.
    Values are bit-identical to compute_weights: each off-diagonal is the same fp32 rounding of
    1./(max(d_i,d_j)+1); the diagonal repeats the reference's fp32 reduction of the dense row
    W[i,:] (a zero row buffer with the row's entries scattered in, then torch .sum()), so the
    summation order - and hence every bit - matches weights.py:25.  MH weights are symmetric
    (W[j,i] = W[i,j]), so row i of W^T holds the same values as row i of W."""
    deg = np.asarray([len(edges[i]) for i in range(n)], np.int64)
    sets = [set(edges[i]) for i in range(n)]
    row = torch.zeros(n)
    counts = np.empty(n, np.int64)
    cols, vals = [], []
    for i in range(n):
        nb = np.asarray([j for j in edges[i] if j != i], np.int64)
        off = (1.0 / (np.maximum(deg[i], deg[nb]) + 1)).astype(np.float32) if len(nb) else \
            np.zeros(0, np.float32)
        if len(nb):
            idx = torch.from_numpy(nb)
            row[idx] = torch.from_numpy(off)
        diag = (1. - row.sum()).item()
        if len(nb):
            row[idx] = 0.0
        # W[src, i] for src in edges[i] (edges order): row src of W holds i iff i in edges[src]
        e = list(edges[i])
        ev = np.asarray([np.float32(diag) if j == i else
                         (1.0 / (max(deg[i], deg[j]) + 1) if i in sets[j] else 0.0)
                         for j in e], np.float64).astype(np.float32)
        cols.append(np.asarray([i] + e, np.int64))
        vals.append(np.concatenate([np.asarray([diag], np.float32), ev]))
        counts[i] = 1 + len(e)
    row_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    col = np.concatenate(cols).astype(np.int32) if n else np.zeros(0, np.int32)
    val = np.concatenate(vals).astype(np.float32) if n else np.zeros(0, np.float32)
    return MixCSR(row_ptr, col, val).validate()


def save_csr(path, csr, cliques=None):
    extra = {}
    if cliques is not None:
        extra["cliques_flat"] = np.asarray([r for c in cliques for r in c], np.int32)
        extra["cliques_ptr"] = np.cumsum([0] + [len(c) for c in cliques]).astype(np.int64)
    np.savez(path, row_ptr=csr.row_ptr, col=csr.col, val=csr.val, **extra)


def load_csr(path):
    d = np.load(path)
    csr = MixCSR(d["row_ptr"].astype(np.int64), d["col"].astype(np.int32),
                 d["val"].astype(np.float32)).validate()
    cliques = None
    if "cliques_flat" in d:
        f, p = d["cliques_flat"], d["cliques_ptr"]
        cliques = [f[p[i]:p[i + 1]].tolist() for i in range(len(p) - 1)]
    return csr, cliques
