"""Block-staged plan for k_mix_staged (host side, once per topology).

Output rows are grouped into blocks — the topology's cliques when it has them, else runs of
consecutive rows — and each block lists the distinct input rows its rows read (its members plus
remote neighbours).  The kernel stages those rows of one column chunk in LDS once and serves every
CSR gather from LDS; each row still accumulates its entries in the reference's operand order, so
the exact mode stays bit-identical to k_mix_csr / the reference loop.
"""
from dataclasses import dataclass

import numpy as np

MAX_SRC = 256     # LDS slots per block (256 x 64 floats x 4 B = 64 KiB at one float per lane)


@dataclass
class StagedPlan:
    blk_ptr: np.ndarray    # int32 [B+1] into blk_rows
    blk_rows: np.ndarray   # int32 [n]
    src_ptr: np.ndarray    # int32 [B+1] into src_rows
    src_rows: np.ndarray   # int32 [S]
    scol: np.ndarray       # int32 [nnz]: slot of each CSR entry's source within its row's block
    max_src: int

    @property
    def n_blocks(self):
        return len(self.blk_ptr) - 1


def build_staged_plan(csr, blocks=None, block_rows=64, max_src=MAX_SRC):
    """(plan, None) or (None, reason).  blocks: list of row lists (e.g. cliques) or None."""
    n = csr.n
    if blocks is None:
        blocks = [list(range(s, min(s + block_rows, n))) for s in range(0, n, block_rows)]
    flat = np.asarray([r for b in blocks for r in b], np.int64)
    if len(flat) != n or not np.array_equal(np.sort(flat), np.arange(n)):
        return None, "blocks do not partition the rows"
    rp, col = csr.row_ptr, csr.col
    scol = np.empty(len(col), np.int32)
    src_lists = []
    for b in blocks:
        slots = {}
        order = []
        for r in b:                               # members first, in block order
            if r not in slots:
                slots[r] = len(order); order.append(r)
        for r in b:
            for k in range(rp[r], rp[r + 1]):
                c = int(col[k])
                if c not in slots:
                    slots[c] = len(order); order.append(c)
                scol[k] = slots[c]
        if len(order) > max_src:
            return None, f"a block reads {len(order)} rows > {max_src}"
        src_lists.append(order)
    return StagedPlan(
        blk_ptr=np.cumsum([0] + [len(b) for b in blocks]).astype(np.int32),
        blk_rows=flat.astype(np.int32),
        src_ptr=np.cumsum([0] + [len(s) for s in src_lists]).astype(np.int32),
        src_rows=np.asarray([r for s in src_lists for r in s], np.int32),
        scol=scol, max_src=max(len(s) for s in src_lists)), None
