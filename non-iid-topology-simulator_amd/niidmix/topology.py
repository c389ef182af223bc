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


SPARSE_KIND = "metropolis-hasting"     # the only weights a sparse topology.json stands for
CSR_FILE = "topology.csr.npz"


def sparse_json(edges, cliques=None, csr_file=CSR_FILE, extra=None):
    """topology.json content for a topology whose weights are NOT stored densely: the reference
    loader (setup.topology.load, topology/__init__.py:4-12) reads it unchanged -- 'edges' as usual,
    'weights': [] becomes an empty tensor -- and every reference consumer other than d_sgd.average
    (which the plugin replaces) reads only edges / cliques (analyze/topology.py).  The mixing
    weights are the Metropolis-Hastings weights of the edges ('weights-kind'; to_csr rebuilds them
    bit for bit with mh_csr) and the same CSR sits next to the file ('weights-csr')."""
    topo = {"edges": {str(r): [int(j) for j in edges[r]] for r in edges}, "weights": [],
            "weights-kind": SPARSE_KIND, "weights-csr": csr_file}
    if cliques is not None:
        topo["cliques"] = [[int(r) for r in c] for c in cliques]
    if extra:
        topo.update(extra)
    return topo


def write_sparse(rundir, csr, edges=None, cliques=None):
    """Write a sparse topology into `rundir`: topology.csr.npz first, then a topology.json the
    reference loader reads (sparse_json), so the unchanged run.py:92-93 (setup.topology.load)
    hands the plugin a topology it can mix."""
    save_csr(os.path.join(rundir, CSR_FILE), csr, cliques)
    with open(os.path.join(rundir, "topology.json"), "w+") as f:
        json.dump(sparse_json(edges if edges is not None else csr.edges(), cliques), f)


def _empty_weights(w):
    if w is None:
        return True
    if isinstance(w, torch.Tensor):
        return w.numel() == 0
    return len(w) == 0


def load(rundir):
    """Drop-in for setup.topology.load(rundir).  A sparse topology.json (sparse_json: empty
    'weights') gets its companion CSR attached as topology['csr'] when the rundir holds it; a
    rundir with only topology.csr.npz (or a companion newer than a dense topology.json, as older
    --randomize rundirs left them) is read from the CSR with 'edges' rebuilt from it."""
    path = os.path.join(rundir, "topology.json")
    sparse = os.path.join(rundir, CSR_FILE)
    if os.path.exists(path):
        topo = load_file(path)
        if _empty_weights(topo["weights"]) and topo["edges"]:
            comp = os.path.join(rundir, topo.get("weights-csr", CSR_FILE))
            if os.path.exists(comp):
                csr, _ = load_csr(comp)
                if _csr_matches_edges(csr, topo["edges"]):
                    topo["csr"] = csr
            return topo
        if not (os.path.exists(sparse) and os.path.getmtime(sparse) > os.path.getmtime(path)):
            return topo
    if os.path.exists(sparse):
        csr, cliques = load_csr(sparse)
        topo = {"edges": csr.edges(), "csr": csr, "weights": None}
        if cliques is not None:
            topo["cliques"] = cliques
        return topo
    raise FileNotFoundError(path)


def _csr_matches_edges(csr, edges, spot=64):
    """A companion CSR belongs to these edge lists: same N, nnz = N + sum(len(edges[r])), and the
    column lists of up to `spot` rows (first, last, evenly spaced) equal [r] + edges[r].  A stale
    companion (e.g. an interrupted write_sparse / --randomize, which write the CSR before the
    JSON) is then ignored and to_csr rebuilds the weights from the edges (mh_csr)."""
    n = len(edges)
    if csr.n != n or sorted(edges) != list(range(n)):
        return False
    if csr.nnz != n + sum(len(edges[r]) for r in range(n)):
        return False
    rows = np.unique(np.linspace(0, n - 1, min(n, spot)).astype(np.int64)) if n else []
    for r in rows:
        b, e = int(csr.row_ptr[r]), int(csr.row_ptr[r + 1])
        if csr.col[b:e].tolist() != [int(r)] + [int(c) for c in edges[int(r)]]:
            return False
    return True


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
    """CSR of W^T in d_sgd.average's operand order (d_sgd.py:105-106).

    Sparse topologies: with no dense weights (None, or the empty tensor the reference loader makes
    of a sparse topology.json's 'weights': []) the CSR comes from topology['csr'] when present,
    else it is rebuilt from the edges with mh_csr (bitwise compute_weights' Metropolis-Hastings
    weights; 'weights-kind' must say so)."""
    W = topology.get("weights")
    if _empty_weights(W):
        if "csr" in topology:
            return topology["csr"]
        edges = topology["edges"]
        if not edges:
            return MixCSR(np.zeros(1, np.int64), np.zeros(0, np.int32), np.zeros(0, np.float32))
        kind = topology.get("weights-kind")
        if kind != SPARSE_KIND:
            raise ValueError(f"topology has no weights and weights-kind {kind!r}: only "
                             f"{SPARSE_KIND!r} weights are rebuilt from the edges")
        n = len(edges)
        if sorted(edges) != list(range(n)):
            raise ValueError("sparse topology: edges must list every rank 0..N-1")
        return mh_csr(n, edges)
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


# below this many nodes a dense row is reduced by one thread either way (ATen's GRAIN_SIZE), so a
# batched 2-D row sum has the 1-D reduction's order; at or above it mh_csr sums row by row
ROWSUM_BATCH_MAX = 32768


def mh_csr(n, edges):
    """Sparse Metropolis-Hastings straight to the mixing CSR, without materialising the N x N JSON.
    Values are bit-identical to compute_weights (weights.py:15-25):
      * each off-diagonal W[i, j] (j in edges[i], j != i) is the fp32 rounding of the double
        1./(max(d_i, d_j) + 1), d = len(edges[.]);
      * the diagonal repeats the reference's fp32 reduction of the dense row W[i, :]: rows are
        scattered into a zero [B, N] buffer and reduced with torch's row sum, which is the same
        per-row reduction as the reference's 1-D W[i, :].sum() (the summation order, and hence
        every bit; tests/test_topology.py pins it on every golden topology);
      * entry (row i, src) of the CSR is W[src, i]: 1./(max(d_i, d_src) + 1) if i in edges[src],
        else 0 (the reference sets W[src, i] only along src's own edge list).
    Cost: O(N * degree) vectorised host work for the CSR, plus the diagonal's reduction over the
    dense rows, O(N^2) fp32 adds in [B, N] batches (the price of bitwise equality with the dense
    reduction: 10 000 nodes ~0.1 s)."""
    lens = np.asarray([len(edges[i]) for i in range(n)], np.int64)
    deg = lens
    src_of = np.repeat(np.arange(n, dtype=np.int64), lens)                 # row owning the entry
    dst = np.fromiter((j for i in range(n) for j in edges[i]), np.int64, int(lens.sum()))
    if dst.size and (dst.min() < 0 or dst.max() >= n):
        raise ValueError("edge endpoint out of range")
    off_mask = dst != src_of
    # W[i, j] for the reference's edge list of i (self entries skipped, weights.py:18-20)
    wi, wj = src_of[off_mask], dst[off_mask]
    wv = (1.0 / (np.maximum(deg[wi], deg[wj]) + 1)).astype(np.float32)
    diag = np.empty(n, np.float32)
    bsz = int(max(1, min(n, (1 << 25) // max(n, 1))))
    if n:
        starts = np.searchsorted(wi, np.arange(0, n, bsz))
        starts = np.append(starts, wi.size)
        buf = torch.zeros((bsz, n))
        for k, r0 in enumerate(range(0, n, bsz)):
            r1 = min(n, r0 + bsz)
            a, b = starts[k], starts[k + 1]
            ri = torch.from_numpy(wi[a:b] - r0)
            ci = torch.from_numpy(wj[a:b])
            buf[ri, ci] = torch.from_numpy(wv[a:b])
            if n < ROWSUM_BATCH_MAX:
                diag[r0:r1] = (1. - buf[:r1 - r0].sum(1)).numpy()
            else:
                # ATen splits a 1-D reduction of >= GRAIN_SIZE (32768) elements over its threads,
                # so the batched row sum (one thread per row) would order the adds differently:
                # reduce every dense row on its own, as the reference's W[i, :].sum() does
                for i in range(r1 - r0):
                    diag[r0 + i] = float(1. - buf[i].sum())
            buf[ri, ci] = 0.0
    # CSR of W^T in d_sgd.average's operand order: row i = [i] + edges[i]; value W[src, i]
    keys = np.unique(wi * n + wj) if wi.size else np.zeros(0, np.int64)   # W[a, b] != 0 pairs
    rows, srcs = src_of, dst                                              # entry (row i, src)
    has = np.isin(srcs * n + rows, keys) if keys.size else np.zeros(rows.size, bool)
    ev = np.where(has, 1.0 / (np.maximum(deg[rows], deg[srcs]) + 1), 0.0).astype(np.float32)
    self_ent = srcs == rows
    ev[self_ent] = diag[rows[self_ent]]
    counts = 1 + lens
    row_ptr = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    col = np.empty(int(row_ptr[-1]), np.int64)
    val = np.empty(int(row_ptr[-1]), np.float32)
    heads = row_ptr[:-1]
    col[heads] = np.arange(n)
    val[heads] = diag
    body = np.ones(int(row_ptr[-1]), bool)
    body[heads] = False
    col[body] = srcs
    val[body] = ev
    return MixCSR(row_ptr, col.astype(np.int32), val).validate()


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
