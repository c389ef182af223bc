"""Merged-order row tiles for k_mix_tile (host side, once per topology).

The exact rule gives every output row its own operand order: self first, then edges[rank] in list
order (d_sgd.py:105-106, model/__init__.py:23-24).  Rows of one clique read almost the same source
rows, but the reference's edge lists are Python-set iteration orders that do not agree across rows,
so there is no single order for a clique.  A tile of rt rows gets a MERGED position list instead:
a short common supersequence of its rows' lists (LCS-guided insertion, _supersequence).  A source two rows order differently simply appears twice.
The kernel walks the positions in order, loads each position's source row once and applies it to
every row whose mask bit is set — each row sees exactly its own list, in its own order.

Density = entries / (rt * positions) is the fraction of useful (row, position) work; the Mixer only
picks the tile kernel when it is high (cliques: ~0.8-0.9; a ring: ~0.1 -> CSR gather instead).
"""
import bisect
from dataclasses import dataclass

import numpy as np

TILE_ROWS = (8, 16, 32)


@dataclass
class TilePlan:
    rt: int
    sub_ptr: np.ndarray     # int64 [T+1] offsets into the position arrays
    sub_rows: np.ndarray    # int32 [T*rt], -1 = unused slot
    sub_wself: np.ndarray   # fp32 [T*rt]
    pos_src: np.ndarray     # int32 [L]
    pos_mask: np.ndarray    # uint32 [L]
    pos_w: np.ndarray       # fp32 [L*rt]
    nnz: int                # off-diagonal entries covered

    @property
    def n_sub(self):
        return len(self.sub_ptr) - 1

    @property
    def n_pos(self):
        return int(self.sub_ptr[-1])

    @property
    def density(self):
        return self.nnz / max(1, self.rt * self.n_pos)

    def row_lists(self):
        """{row: [(src, w), ...]} as the kernel will apply them (self entry first) — for checks."""
        out = {}
        for t in range(self.n_sub):
            b, e = int(self.sub_ptr[t]), int(self.sub_ptr[t + 1])
            for r in range(self.rt):
                row = int(self.sub_rows[t * self.rt + r])
                if row < 0:
                    continue
                lst = [(row, np.float32(self.sub_wself[t * self.rt + r]))]
                for k in range(b, e):
                    if (int(self.pos_mask[k]) >> r) & 1:
                        lst.append((int(self.pos_src[k]), np.float32(self.pos_w[k * self.rt + r])))
                out[row] = lst
        return out


def _supersequence(seqs):
    """A common supersequence of the int sequences, built by insertion: each next sequence is
    matched against the current merge along a longest common subsequence (Hunt-Szymanski: LCS as a
    longest strictly increasing run of match positions), and only its unmatched elements are
    inserted, each right after the merge position of its last matched predecessor.  Inserting never
    breaks the earlier sequences' embeddings.  Rows whose orders agree except for a few swaps cost
    a few duplicates."""
    M = []
    for cols in seqs:
        if not M:
            M = list(cols)
            continue
        occ = {}
        for i, v in enumerate(M):
            occ.setdefault(v, []).append(i)
        seq = [(pos, k) for k, v in enumerate(cols) for pos in reversed(occ.get(v, ()))]
        tails, tails_at, prev = [], [], [-1] * len(seq)
        for s, (pos, _) in enumerate(seq):
            j = bisect.bisect_left(tails, pos)
            if j == len(tails):
                tails.append(pos)
                tails_at.append(s)
            else:
                tails[j] = pos
                tails_at[j] = s
            prev[s] = tails_at[j - 1] if j else -1
        matched = {}
        s = tails_at[-1] if tails_at else -1
        while s >= 0:
            matched[seq[s][1]] = seq[s][0]
            s = prev[s]
        inserts, last = {}, -1
        for k, v in enumerate(cols):
            if k in matched:
                last = matched[k]
            else:
                inserts.setdefault(last, []).append(v)
        out = list(inserts.get(-1, ()))
        for i, v in enumerate(M):
            out.append(v)
            out.extend(inserts.get(i, ()))
        M = out
    return M


def _merge(lists):
    """Entry lists [(cols, vals)] -> positions [(src, mask, {r: w})]: every list embedded (greedy
    leftmost) in one common supersequence."""
    seqs = [[int(c) for c in cols] for cols, _ in lists]
    M = _supersequence(seqs)
    masks = [0] * len(M)
    ws = [dict() for _ in M]
    for r, (seq, (_, vals)) in enumerate(zip(seqs, lists)):
        i = 0
        for k, v in enumerate(seq):
            while M[i] != v:
                i += 1
            masks[i] |= 1 << r
            ws[i][r] = vals[k]
            i += 1
    return [(c, m, w) for c, m, w in zip(M, masks, ws) if m]


def _split(rows, rt):
    """Cut a row group into ceil(len/rt) balanced consecutive parts."""
    k = -(-len(rows) // rt)
    base, extra = divmod(len(rows), k)
    parts, s = [], 0
    for i in range(k):
        m = base + (1 if i < extra else 0)
        parts.append(rows[s:s + m])
        s += m
    return parts


def build_tile_plan(csr, groups=None, rt=16):
    """(plan, None) or (None, reason).  groups: row lists (e.g. the cliques) cut into tiles of <= rt
    rows; None -> consecutive rows.  Every CSR row must belong to exactly one group."""
    if rt not in TILE_ROWS:
        return None, f"rt={rt} not in {TILE_ROWS}"
    n = csr.n
    if groups is None:
        groups = [list(range(s, min(s + rt, n))) for s in range(0, n, rt)]
    flat = np.asarray([r for g in groups for r in g], np.int64)
    if len(flat) != n or not np.array_equal(np.sort(flat), np.arange(n)):
        return None, "groups do not partition the rows"
    rp, col, val = csr.row_ptr, csr.col, csr.val
    full = (1 << rt) - 1
    sub_ptr, sub_rows, sub_wself = [0], [], []
    pos_src, pos_mask, pos_w = [], [], []
    for g in groups:
        for part in _split(list(g), rt):
            lists = [(col[rp[r] + 1:rp[r + 1]], val[rp[r] + 1:rp[r + 1]]) for r in part]
            pad = full & ~((1 << len(part)) - 1)
            for c, mask, ws in _merge(lists):
                w = np.zeros(rt, np.float32)
                for r, v in ws.items():
                    w[r] = v
                pos_src.append(c)
                pos_mask.append(mask | pad)
                pos_w.append(w)
            sub_ptr.append(len(pos_src))
            sub_rows.extend(list(part) + [-1] * (rt - len(part)))
            sub_wself.extend([val[rp[r]] for r in part] + [0.0] * (rt - len(part)))
    L = len(pos_src)
    return TilePlan(
        rt=rt, sub_ptr=np.asarray(sub_ptr, np.int64),
        sub_rows=np.asarray(sub_rows, np.int32), sub_wself=np.asarray(sub_wself, np.float32),
        pos_src=np.asarray(pos_src, np.int32).reshape(L),
        pos_mask=np.asarray(pos_mask, np.uint64).astype(np.uint32).reshape(L),
        pos_w=(np.stack(pos_w) if L else np.zeros((0, rt), np.float32)).reshape(L * rt),
        nnz=int(csr.nnz - csr.n)), None


def apply_np(plan, x, exact=True, average_only=False):
    """numpy model of k_mix_tile (same per-row order and roundings) — for CPU tests."""
    x = np.asarray(x, np.float32)
    rows = plan.row_lists()
    y = np.zeros((max(rows) + 1 if rows else 0, x.shape[1]), np.float32)
    for row, lst in rows.items():
        z = x[row] * np.float32(0)
        acc = z.copy()
        for src, w in lst:
            if exact:
                acc = acc + np.float32(w) * x[src]
            else:
                acc = (np.float64(w) * x[src].astype(np.float64) + acc).astype(np.float32)
        y[row] = acc if average_only else z + acc
    return y
