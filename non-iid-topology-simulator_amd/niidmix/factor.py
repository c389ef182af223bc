"""Clique-factored form of a mixing matrix (host side, built once per topology).

D-Cliques topologies (tools/setup/topology/d_cliques/random_cliques.py:18-37 + interclique.py) are
cliques of c nodes plus a few inter-clique edges, weighted by Metropolis-Hastings
W[j,i] = 1/(max(d_i, d_j) + 1) (weights.py:15-25).  Inside a clique, W[j,i] therefore depends on j
only through j's degree, so for every member i

    y_i = sum_j W[j,i] x_j
        = a_i x_i + sum_g c_{i,g} S_g + sum_{(j,w) in R_i} w x_j

with S_g the sum of x over the clique members of degree class g, c_{i,g} the common in-clique
weight of class g seen from i, a_i = W[i,i] - c_{i,g(i)}, and R_i a short residual list (the
inter-clique "gateway" edges, plus corrections for removed clique edges).  One HBM read and one
write per parameter then suffice (k_mix_clique in csrc/niidmix.hip), instead of (degree+1) gathers.

The plan is derived from the LOADED W, never assumed: every coefficient is taken from W itself and
`effective_weights()` reproduces W (tests/test_factor.py checks this on every golden topology).  If
the structure does not hold (too many degree classes, a clique too large for the register tile,
too many residual terms) build_clique_plan returns None and the caller uses the generic kernels.
"""
from dataclasses import dataclass

import numpy as np

MAX_GROUPS = 4          # template limit of k_mix_clique
MAX_CLIQUE = 1 << 20    # <= 256: register-tiled k_mix_clique; larger: two-pass k_mix_bigclique


@dataclass
class CliquePlan:
    n: int
    n_groups: int
    max_clique: int
    max_clique_res: int
    clique_ptr: np.ndarray     # int32 [C+1]
    member_row: np.ndarray     # int32 [M]
    member_group: np.ndarray   # int32 [M]
    coef: np.ndarray           # fp32 [M, 1+G]: a_m, c_{m,0..G-1}
    res_ptr: np.ndarray        # int32 [M+1]
    res_col: np.ndarray        # int32 [R]
    res_val: np.ndarray        # fp32 [R]
    res_member: np.ndarray = None   # int32 [R]: the entry's member index within its clique
    n_cancel: int = 0          # residual terms that cancel (most of) a class value: removed clique
                               # edges (-c_g) or in-clique weights far below their class value.
                               # Their rounding error is not bounded by the row's own terms, so
                               # Mixer's auto choice avoids the factored kernel when n_cancel > 0.

    @property
    def n_cliques(self):
        return len(self.clique_ptr) - 1

    @property
    def n_members(self):
        return len(self.member_row)

    @property
    def n_res(self):
        return len(self.res_col)

    def effective_weights(self, n_in=None):
        """W_eff[src, dst] (float64) implied by the plan; equals W up to the fp32 rounding of a_i
        and of residual corrections."""
        n, G = self.n, self.n_groups
        W = np.zeros((n_in or n, n), np.float64)
        for c in range(self.n_cliques):
            mem = self.member_row[self.clique_ptr[c]:self.clique_ptr[c + 1]]
            grp = self.member_group[self.clique_ptr[c]:self.clique_ptr[c + 1]]
            for k, i in enumerate(mem):
                m = self.clique_ptr[c] + k
                W[i, i] += self.coef[m, 0]
                for g in range(G):
                    W[mem[grp == g], i] += self.coef[m, 1 + g]
                for q in range(self.res_ptr[m], self.res_ptr[m + 1]):
                    W[self.res_col[q], i] += self.res_val[q]
        return W

    def apply_np(self, x):
        """float64 evaluation of the factored formula (test helper)."""
        x = np.asarray(x, np.float64)
        y = np.zeros_like(x)
        for c in range(self.n_cliques):
            sl = slice(self.clique_ptr[c], self.clique_ptr[c + 1])
            mem, grp = self.member_row[sl], self.member_group[sl]
            S = [x[mem[grp == g]].sum(axis=0) for g in range(self.n_groups)]
            for k, i in enumerate(mem):
                m = self.clique_ptr[c] + k
                acc = self.coef[m, 0] * x[i]
                for g in range(self.n_groups):
                    acc = acc + self.coef[m, 1 + g] * S[g]
                for q in range(self.res_ptr[m], self.res_ptr[m + 1]):
                    acc = acc + self.res_val[q] * x[self.res_col[q]]
                y[i] = acc
        return y


def _mode(values, n_zero):
    """Most frequent value among `values` plus n_zero implicit zeros (ties -> smallest)."""
    if len(values) == 0:
        return 0.0
    u, cnt = np.unique(values, return_counts=True)
    if n_zero:
        z = np.searchsorted(u, 0.0)
        if z < len(u) and u[z] == 0.0:
            cnt[z] += n_zero
        else:
            u = np.insert(u, z, 0.0)
            cnt = np.insert(cnt, z, n_zero)
    return float(u[np.argmax(cnt)])


def build_clique_plan(csr, cliques, max_res_per_node=1.0, max_groups=MAX_GROUPS,
                      max_clique=MAX_CLIQUE):
    """Factor `csr` (MixCSR) over `cliques` (list of lists of ranks, topology.json 'cliques').
    Returns (plan, None) or (None, reason)."""
    n = csr.n
    if not cliques:
        return None, "no cliques"
    flat = np.asarray([r for c in cliques for r in c], np.int64)
    if len(flat) != n or not np.array_equal(np.sort(flat), np.arange(n)):
        return None, "cliques do not partition the nodes"
    biggest = max(len(c) for c in cliques)
    if biggest > max_clique:
        return None, f"clique of {biggest} members > {max_clique}"
    deg = csr.degrees()
    n_in = max(csr.n_in, n)                 # a shard's CSR also reads halo rows >= n
    clique_of = np.full(n_in, -1, np.int64)
    group_of = np.full(n_in, -1, np.int64)
    groups_per_clique = []
    for ci, c in enumerate(cliques):
        c = np.asarray(c, np.int64)
        clique_of[c] = ci
        classes = np.unique(deg[c])
        if len(classes) > max_groups:
            return None, f"clique {ci} has {len(classes)} degree classes > {max_groups}"
        group_of[c] = np.searchsorted(classes, deg[c])
        groups_per_clique.append([c[group_of[c] == g] for g in range(len(classes))])
    G = max(len(g) for g in groups_per_clique)

    M = n
    coef = np.zeros((M, 1 + G), np.float32)
    res_ptr = np.zeros(M + 1, np.int64)
    res_cols, res_vals, res_member = [], [], []
    n_cancel = 0
    member_row = flat.astype(np.int32)
    member_group = group_of[flat].astype(np.int32)
    clique_ptr = np.cumsum([0] + [len(c) for c in cliques]).astype(np.int32)
    for m, i in enumerate(flat):
        b, e = int(csr.row_ptr[i]), int(csr.row_ptr[i + 1])
        cols = csr.col[b:e].astype(np.int64)
        vals = csr.val[b:e]
        w_self = float(vals[0])
        cols, vals = cols[1:], vals[1:]
        ci = clique_of[i]
        same = (clique_of[cols] == ci) & (cols != i)
        groups = groups_per_clique[ci]
        cs = np.zeros(G, np.float64)
        for g, gm in enumerate(groups):
            sel = same & (group_of[cols] == g)
            present = vals[sel]
            others = len(gm) - (1 if group_of[i] == g else 0)
            cs[g] = _mode(present.astype(np.float64), others - int(sel.sum()))
        coef[m, 1:] = cs.astype(np.float32)
        coef[m, 0] = np.float32(w_self - float(np.float32(cs[group_of[i]])))
        rc, rv = [], []
        # inter-clique terms (zero weights kept: the reference still multiplies them, so a
        # non-finite source gives NaN there, and the kernel's non-finite guard must see that row)
        out = ~same & (cols != i)
        for j, w in zip(cols[out], vals[out]):
            rc.append(j); rv.append(float(w))
        # in-clique corrections (weights that differ from their class value); one that cancels
        # most of its class value (|w| < |c|/64) loses the fp32 accuracy of the term it replaces
        for j, w in zip(cols[same], vals[same]):
            c_j = float(np.float32(cs[group_of[j]]))
            if float(w) != c_j:
                rc.append(j); rv.append(float(w) - c_j)
                if abs(float(w)) * 64.0 < abs(c_j):
                    n_cancel += 1
        # in-clique members with no edge (W = 0) whose class value is not 0: a removed clique edge
        # (d_cliques/utils.py remove_clique_edges), corrected by -c_g (a cancelling term)
        present_set = set(cols[same].tolist())
        for g, gm in enumerate(groups):
            c_g = float(np.float32(cs[g]))
            if c_g == 0.0:
                continue
            for j in gm:
                if j != i and j not in present_set:
                    rc.append(int(j)); rv.append(-c_g)
                    n_cancel += 1
        res_cols.extend(rc)
        res_vals.extend(rv)
        res_member.extend([m - int(clique_ptr[ci])] * len(rc))
        res_ptr[m + 1] = res_ptr[m] + len(rc)
    n_res = int(res_ptr[-1])
    if n_res > max_res_per_node * n:
        return None, f"{n_res} residual terms > {max_res_per_node} per node"
    per_clique = res_ptr[clique_ptr[1:]] - res_ptr[clique_ptr[:-1]]
    max_cr = int(per_clique.max()) if len(per_clique) else 0
    plan = CliquePlan(n=n, n_groups=G, max_clique=biggest, max_clique_res=max_cr,
                      clique_ptr=clique_ptr,
                      member_row=member_row, member_group=member_group, coef=coef,
                      res_ptr=res_ptr.astype(np.int32),
                      res_col=np.asarray(res_cols, np.int32),
                      res_val=np.asarray(res_vals, np.float64).astype(np.float32),
                      res_member=np.asarray(res_member, np.int32), n_cancel=n_cancel)
    return plan, None
