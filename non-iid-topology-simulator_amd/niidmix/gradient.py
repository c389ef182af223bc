"""Gradient averaging on the GPU: --clique-gradient and --unbiased-gradient.

Reference: tools/simulate/algorithm/d_sgd.py:47-94 (`gradient`), with average_gradients (:19-27:
zeros_like, add_ every member's grad in list order, div_(len)) and update_gradients (:37-45:
grad.zero_(); grad.add_(mean)).  Every node's new gradient is computed from the pre-update
gradients (the reference computes all means of a clique / of all nodes before writing any, and
cliques are disjoint), so the whole step is one Jacobi pass over a [N, P] gradient slab:

  clique-gradient, no removed edges (:56-65)   every member of a clique receives the mean over the
      clique, in clique order  ->  segments, k_grad_segment_mean (one read + one write per row)
  clique-gradient, removed edges (:66-78)      node r averages [q for q in clique if q == r or
      q in edges[r]]  ->  per-row CSR, k_mix_csr with NIIDMIX_FLAG_MEAN
  unbiased-gradient (:79-90)                   node r averages topology['neighbourhoods'][r] in list
      order  ->  per-row CSR, k_mix_csr with NIIDMIX_FLAG_MEAN

`stepped` lists the nodes whose optimizer the reference steps afterwards (every clique member, or
every node for unbiased-gradient).  A node in no clique is not stepped by the reference and its
gradient is left alone; here it gets a one-member segment / row (its own gradient, +0 + g/1, which
only differs from "untouched" by turning a -0.0 entry into +0.0 — a gradient that is never
applied).  Overlapping cliques (which no reference generator produces) would make the reference's
clique loop order-dependent and are refused.
"""
from dataclasses import dataclass

import numpy as np
import torch


@dataclass
class GradPlan:
    kind: str                       # "clique" | "clique-removed" | "unbiased"
    n: int
    row_ptr: np.ndarray = None      # int64 [n+1]   (CSR kinds)
    col: np.ndarray = None          # int32 [nnz]
    seg_ptr: np.ndarray = None      # int32 [S+1]   (segment kind)
    seg_row: np.ndarray = None      # int32 [M]
    stepped: list = None            # ranks whose optimizer steps afterwards, in the reference's order


def _csr(rows):
    row_ptr = np.zeros(len(rows) + 1, np.int64)
    row_ptr[1:] = np.cumsum([len(r) for r in rows])
    col = np.asarray([c for r in rows for c in r], np.int32)
    return row_ptr, col


def _check_cliques(cliques, n):
    seen = np.zeros(n, bool)
    for c in cliques:
        for r in c:
            if not 0 <= r < n:
                raise ValueError(f"clique member {r} outside 0..{n - 1}")
            if seen[r]:
                raise ValueError(f"node {r} is in more than one clique: the reference's clique loop "
                                 "(d_sgd.py:56-78) is order-dependent then; not supported")
            seen[r] = True
    return seen


def build_grad_plan(n, topology, params):
    """The averaging lists of d_sgd.gradient (d_sgd.py:47-94) for nodes 0..n-1 (positional, as the
    reference's nodes[rank]).  Returns None when no gradient averaging is configured."""
    alg = params["algorithm"]
    if alg.get("clique-gradient"):
        cliques = [list(map(int, c)) for c in topology["cliques"]]
        member = _check_cliques(cliques, n)
        removed = params.get("topology", {}).get("remove-clique-edges", 0)
        stepped = [r for c in cliques for r in c]
        loners = [r for r in range(n) if not member[r]]
        if not removed:
            segs = cliques + [[r] for r in loners]
            seg_ptr = np.zeros(len(segs) + 1, np.int32)
            seg_ptr[1:] = np.cumsum([len(s) for s in segs])
            seg_row = np.asarray([r for s in segs for r in s], np.int32)
            return GradPlan("clique", n, seg_ptr=seg_ptr, seg_row=seg_row, stepped=stepped)
        edges = topology["edges"]
        rows = [[r] for r in range(n)]
        for c in cliques:
            for r in c:
                adj = set(edges[r])
                rows[r] = [q for q in c if q == r or q in adj]
        row_ptr, col = _csr(rows)
        return GradPlan("clique-removed", n, row_ptr=row_ptr, col=col, stepped=stepped)
    if alg.get("unbiased-gradient"):
        hoods = topology["neighbourhoods"]
        rows = []
        for r in range(n):
            h = [int(q) for q in hoods[r]]
            if not h:
                raise ValueError(f"node {r} has an empty neighbourhood (the reference divides by 0)")
            if min(h) < 0 or max(h) >= n:
                raise ValueError(f"neighbourhood of node {r} names a node outside 0..{n - 1}")
            rows.append(h)
        row_ptr, col = _csr(rows)
        return GradPlan("unbiased", n, row_ptr=row_ptr, col=col, stepped=list(range(n)))
    return None


class GradMean:
    """Device operator g' = per-node gradient mean for one GradPlan (callable like ops.Mixer, so
    slab.SlabMixer can stream a host gradient slab through it)."""

    def __init__(self, plan, device):
        from . import ops
        self.ops = ops
        self.plan = plan
        self.n = plan.n
        dev = torch.device(device)
        if plan.seg_ptr is not None:
            self.seg_ptr = torch.from_numpy(plan.seg_ptr).to(dev)
            self.seg_row = torch.from_numpy(plan.seg_row).to(dev)
        else:
            self.row_ptr = torch.from_numpy(plan.row_ptr).to(dev)
            self.col = torch.from_numpy(plan.col).to(dev)
            self.val = torch.ones(len(plan.col), dtype=torch.float32, device=dev)
            self.hint = self.ops.LOW_DEGREE if len(plan.col) <= 4 * max(self.n, 1) else 0

    def mean_blocked(self, g, out, p):
        """Segment mean on column-blocked slabs [K, rows, B] (device-resident layout)."""
        if self.plan.seg_ptr is None:
            raise RuntimeError("blocked slabs: only the clique-gradient segment mean")
        self.ops.grad_segment_mean_blocked(g, self.seg_ptr, self.seg_row, out, int(p))
        return out

    def __call__(self, g, out=None, mode=None, kernel=None):
        """mode / kernel are accepted for SlabMixer compatibility: the mean is exact in every mode
        (w = 1: fma(1, g, acc) == fl(acc + g))."""
        if out is None:
            out = torch.empty((self.n, g.shape[1]), dtype=torch.float32, device=g.device)
        if self.plan.seg_ptr is not None:
            self.ops.grad_segment_mean(g, self.seg_ptr, self.seg_row, out)
        else:
            self.ops.mix_csr(g, self.row_ptr, self.col, self.val, out,
                             self.ops.EXACT | self.ops.MEAN | self.hint)
        return out
