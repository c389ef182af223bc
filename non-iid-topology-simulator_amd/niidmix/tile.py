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
import os
from dataclasses import dataclass

import numpy as np

TILE_ROWS = (8, 16, 32)
POS_UNIFORM = 1 << 30          # pos_src flag: every tile row's weight at this position is equal


@dataclass
class TilePlan:
    rt: int
    sub_ptr: np.ndarray     # int64 [T+1] offsets into the position arrays
    sub_rows: np.ndarray    # int32 [T*rt], -1 = unused slot
    sub_wself: np.ndarray   # fp32 [T*rt]
    pos_src: np.ndarray     # int32 [L] source row | POS_UNIFORM
    pos_mask: np.ndarray    # uint32 [L]
    pos_w: np.ndarray       # fp32 [L*rt]
    nnz: int                # off-diagonal entries covered
    grp_tile_ptr: np.ndarray = None   # int32 [G+1]: tiles of each input group

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
                        lst.append((int(self.pos_src[k]) & (POS_UNIFORM - 1),
                                    np.float32(self.pos_w[k * self.rt + r])))
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


def _list_rank(group, rp, col):
    """{row: median index of the row in the other group rows' in-group edge lists}: the order the
    group's lists roughly agree on (the reference's set iteration order)."""
    g = np.asarray(group, np.int64)
    if len(g) == 0:
        return {}
    inside = np.zeros(int(g.max()) + 1, bool)
    inside[g] = True
    pos = {int(r): [] for r in g}
    for r in g:
        c = col[rp[r] + 1:rp[r + 1]].astype(np.int64)
        c = c[c < len(inside)]
        for i, m in enumerate(c[inside[c]].tolist()):
            pos[m].append(i)
    return {m: (float(np.median(v)) if v else 0.0) for m, v in pos.items()}


def _class_tiles(group, rp, col, val, rt, max_rows=None):
    """Tiles of a row group: rows ordered by degree — under Metropolis-Hastings the weight
    W[j, i] = 1/(max(d_i, d_j) + 1) a source j carries into row i depends on i only through d_i —
    and each degree class cut on its own, so a source's weight is the same across a tile's rows
    (POS_UNIFORM; checked on the actual values) — e.g. the gateway rows of a D-Clique form their own
    tile.  Classes of fewer than max(2, rt/2) rows are merged into a neighbouring class (their
    positions are then weighted per row).

    Inside a class the rows follow the group's common list order (_list_rank) before the cut.  A
    tile row skips only its own position, so a tile of rows adjacent in that order has its skips in
    one run, and every row takes all its other positions (the kernel's cheapest form).  On the
    1000-node d-cliques topology the share of 4-position groups that every row takes rises from
    54 % to 77 %.  Results do not change: each row keeps its own list."""
    key = lambda r: int(rp[r + 1] - rp[r])
    rank = _list_rank(group, rp, col)
    rows = sorted(group, key=lambda r: (key(r), rank[int(r)]))
    runs = []
    for r in rows:
        if runs and key(runs[-1][-1]) == key(r):
            runs[-1].append(r)
        else:
            runs.append([r])
    small = max(2, rt // 2)                 # a class this small would waste a mostly empty tile
    merged = []
    for run in runs:
        if merged and len(merged[-1]) < small:
            merged[-1].extend(run)
        else:
            merged.append(list(run))
    if len(merged) > 1 and len(merged[-1]) < small:
        merged[-2].extend(merged.pop())
    return [part for run in merged for part in _split(run, max_rows or rt)]


def build_tile_plan(csr, groups=None, rt=16, max_rows=None):
    """(plan, None) or (None, reason).  groups: row lists (e.g. the cliques) cut into tiles of <= rt
    rows; None -> consecutive rows.  Every CSR row must belong to exactly one group.

    Inside a group rows are ordered by their self weight, then degree (stable) before the cut, so a
    tile holds rows of one Metropolis-Hastings degree class (D-Cliques: the gateway rows together):
    the weights a source carries into a tile's rows are then equal, the position is flagged
    POS_UNIFORM and the exact kernel forms each product once for the whole tile (its weight is
    replicated into every slot of pos_w).  max_rows (<= rt) caps the rows a tile holds."""
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
    grp_tile_ptr = [0]
    for g in groups:
        for part in _class_tiles(g, rp, col, val, rt, max_rows):
            lists = [(col[rp[r] + 1:rp[r + 1]], val[rp[r] + 1:rp[r + 1]]) for r in part]
            pad = full & ~((1 << len(part)) - 1)
            for c, mask, ws in _merge(lists):
                w = np.zeros(rt, np.float32)
                vals = np.asarray(list(ws.values()), np.float32)
                if len(vals) and np.all(vals.view(np.uint32) == vals[:1].view(np.uint32)):
                    w[:] = vals[0]
                    c = int(c) | POS_UNIFORM
                else:
                    for r, v in ws.items():
                        w[r] = v
                pos_src.append(c)
                pos_mask.append(mask | pad)
                pos_w.append(w)
            sub_ptr.append(len(pos_src))
            sub_rows.extend(list(part) + [-1] * (rt - len(part)))
            sub_wself.extend([val[rp[r]] for r in part] + [0.0] * (rt - len(part)))
        grp_tile_ptr.append(len(sub_ptr) - 1)
    L = len(pos_src)
    return TilePlan(
        rt=rt, sub_ptr=np.asarray(sub_ptr, np.int64),
        sub_rows=np.asarray(sub_rows, np.int32), sub_wself=np.asarray(sub_wself, np.float32),
        pos_src=np.asarray(pos_src, np.int32).reshape(L),
        pos_mask=np.asarray(pos_mask, np.uint64).astype(np.uint32).reshape(L),
        pos_w=(np.stack(pos_w) if L else np.zeros((0, rt), np.float32)).reshape(L * rt),
        nnz=int(csr.nnz - csr.n), grp_tile_ptr=np.asarray(grp_tile_ptr, np.int32)), None


LDS_MAX_SRC = 256
LDS_MAX_WAVES = {8: 16, 16: 8, 32: 4}     # waves (tiles) of a block: the span of row groups
MAX_TILES = {8: 16, 16: 12, 32: 4}        # tiles a group may have (k_mix_tile_lds launch bounds)
POS_REMOTE = 1 << 29           # pos_slot flag: the source is one of the tile's register rows
REM_MAX = 16                   # register rows per tile (rem_rows[t * REM_MAX + i])


@dataclass
class TileLdsPlan:
    """A TilePlan regrouped for k_mix_tile_lds: each group (clique) stages its distinct source rows
    in LDS; positions and tile rows refer to LDS slots."""
    tile: TilePlan
    pos_slot: np.ndarray      # int32 [L] slot | POS_UNIFORM
    sub_slot: np.ndarray      # int32 [T*rt]
    grp_tile_ptr: np.ndarray  # int32 [G+1]
    grp_src_ptr: np.ndarray   # int32 [G+1]
    grp_src_rows: np.ndarray  # int32 [sum of group source counts]
    max_src: int
    max_tiles: int
    rem_rows: np.ndarray = None   # int32 [T * REM_MAX] register rows per tile (-1: none), or None
    rem_regs: int = 0             # register rows the kernel loads per tile: 8 if no tile has more, 16

    @property
    def n_grp(self):
        return len(self.grp_tile_ptr) - 1


def _register_sources(tp, t0, t1, srcs, members, row_mask, cap=None):
    """{tile: [source rows]} of a group's sources kept in REGISTERS instead of the LDS stage: a
    source outside the group (a gateway row's inter-clique neighbour) whose every position is
    taken by at most all-but-two rows of its tile -- so the segment builder can never make it part
    of a run (runs read consecutive LDS slots) -- at most `cap` (REM_MAX) per tile, in list order.  At
    10 000 d-cliques nodes each clique reads 99 such rows, one per gateway member: staging them
    doubled the stage (199 rows), left room for 96-column items only, and each is read once."""
    rt = tp.rt
    ok = {int(v) for v in srcs if int(v) not in members}
    per_tile = {}
    for t in range(t0, t1):
        real = 0
        for r in range(rt):
            if tp.sub_rows[t * rt + r] >= 0:
                real |= 1 << r
        n_real = bin(real).count("1")
        for k in range(int(tp.sub_ptr[t]), int(tp.sub_ptr[t + 1])):
            v = int(tp.pos_src[k]) & row_mask
            if v in ok and bin(int(tp.pos_mask[k]) & real).count("1") > n_real - 2:
                ok.discard(v)
    for t in range(t0, t1):
        lst = []
        for k in range(int(tp.sub_ptr[t]), int(tp.sub_ptr[t + 1])):
            v = int(tp.pos_src[k]) & row_mask
            if v in ok and v not in lst:
                lst.append(v)
        per_tile[t] = lst
    # a source two tiles read, or a tile with too many, stays staged
    seen = {}
    for t, lst in per_tile.items():
        for v in lst:
            seen[v] = seen.get(v, 0) + 1
    for t in per_tile:
        lst = [v for v in per_tile[t] if seen[v] == 1]
        per_tile[t] = lst[:cap or REM_MAX]
    return per_tile


def balanced_tile_rows(csr, groups, rt=16):
    """Rows per rt-16 tile for k_mix_tile_lds: 16, unless the groups cut into 4k - 1 tiles (a
    100-row clique: 7), whose block then leaves one of the CU's four SIMDs a wave short in every
    block (7 waves: 2, 2, 2, 1): then the largest height that cuts one tile more (8 waves, two per
    SIMD; 1000-node d-cliques: 13-row tiles, three blocks x 8 waves = the 6 waves per SIMD its 80
    VGPRs allow).  Same box, headline exact round: 2.75 vs 2.81 ms (profiles/r06/tile_rows/)."""
    if rt != 16 or not groups:
        return rt
    rp, col, val = csr.row_ptr, csr.col, csr.val
    tiles = lambda r: max(len(_class_tiles(g, rp, col, val, rt, r)) for g in groups)
    t16 = tiles(rt)
    if t16 % 4 != 3 or t16 + 1 > MAX_TILES[rt]:
        return rt
    for r in range(rt - 1, rt // 2, -1):
        t = tiles(r)
        if t == t16 + 1:
            return r
        if t > t16 + 1:
            break
    return rt


def build_tile_lds_plan(csr, groups=None, rt=8, remote_regs=False, rem_cap=REM_MAX, tile_rows=None):
    """(plan, None) or (None, reason): build_tile_plan over `groups`, then per group the sorted list
    of distinct source rows (every row its tiles read, self rows included) and the slot indices.
    remote_regs (RT 16, segment walker only): sources outside a group that only MASKED entries
    read (_register_sources) are loaded into registers per tile (rem_rows) instead of staged, at
    most rem_cap (8 or 16) per tile; the rest stay staged.  tile_rows (RT 16): at most that many
    rows per tile (more, shorter tiles: more waves per block, up to MAX_TILES)."""
    if rem_cap not in (8, REM_MAX):
        raise ValueError(f"rem_cap {rem_cap} (8 or {REM_MAX})")
    if rt not in LDS_MAX_WAVES:
        return None, f"rt={rt} not in {tuple(LDS_MAX_WAVES)}"
    if groups:
        # cheap rejection before the merged-order tiles are built: a group reading more distinct
        # rows than the LDS stage holds (e.g. a fully-connected graph) can never build
        rp, col = csr.row_ptr, csr.col
        for gi, g in enumerate(groups):
            if len(g) > LDS_MAX_SRC:
                return None, f"group {gi} has {len(g)} rows (> {LDS_MAX_SRC})"
            g = np.asarray(g, np.int64)
            idx = np.concatenate([np.arange(rp[r], rp[r + 1]) for r in g]) if len(g) else g
            n_src = len(np.unique(np.concatenate([col[idx], g])))
            if n_src > LDS_MAX_SRC:
                return None, f"group {gi} reads {n_src} distinct rows (> {LDS_MAX_SRC})"
    # tiles of at most rt-1 rows leave slot rt-1 unused: the rt 8 / 32 loops skip that pad slot at
    # positions every row takes (k_mix_tile_lds, "simple" chunks); when that costs more tiles than
    # a group may have, full-height tiles (correct, slower).  The rt 16 loop (tlds16_run) needs no
    # pad: full-height tiles, one tile fewer per 1000-node d-clique (7 instead of 8).
    pad_default = "0" if rt == 16 else "1"
    max_rows = rt - 1 if os.environ.get("NIIDMIX_TILE_LDS_PAD", pad_default) == "1" else rt
    if rt == 16 and tile_rows is not None:
        max_rows = min(max_rows, int(tile_rows))
    if max_rows < rt and groups and any(len(_class_tiles(g, csr.row_ptr, csr.col, csr.val, rt, max_rows)) > MAX_TILES[rt]
                      for g in groups):
        max_rows = rt
    tp, why = build_tile_plan(csr, groups, rt, max_rows)
    if tp is None:
        return None, why
    row_mask = POS_UNIFORM - 1
    gtp = tp.grp_tile_ptr
    pos_slot = np.empty_like(tp.pos_src)
    sub_slot = np.zeros_like(tp.sub_rows)
    src_ptr, src_rows = [0], []
    max_src = max_tiles = 0
    remote = remote_regs and rt == 16
    rem_rows = np.full(tp.n_sub * REM_MAX, -1, np.int32) if remote else None
    for gi in range(len(gtp) - 1):
        t0, t1 = int(gtp[gi]), int(gtp[gi + 1])
        p0, p1 = int(tp.sub_ptr[t0]), int(tp.sub_ptr[t1])
        rows = tp.sub_rows[t0 * rt:t1 * rt]
        # slots numbered in list order (first appearance): consecutive positions then mostly read
        # consecutive slots, which k_mix_tile_lds reads from one address with immediate offsets
        seq = np.concatenate([tp.pos_src[p0:p1] & row_mask, rows[rows >= 0]])
        _, first = np.unique(seq, return_index=True)
        srcs = seq[np.sort(first)]
        reg_of = {}                                   # (tile, source) -> register index
        if remote:
            per_tile = _register_sources(tp, t0, t1, srcs, {int(r) for r in rows[rows >= 0]},
                                         row_mask, rem_cap)
            in_regs = set()
            for t, lst in per_tile.items():
                for i, v in enumerate(lst):
                    reg_of[(t, v)] = i
                    rem_rows[t * REM_MAX + i] = v
                    in_regs.add(v)
            srcs = np.asarray([v for v in srcs if int(v) not in in_regs], srcs.dtype)
        if len(srcs) > LDS_MAX_SRC:
            return None, f"group {gi} reads {len(srcs)} distinct rows (> {LDS_MAX_SRC})"
        if t1 - t0 > MAX_TILES[rt]:
            return None, f"group {gi} has {t1 - t0} tiles of {rt} rows (> {MAX_TILES[rt]})"
        slot_of = {int(r): i for i, r in enumerate(srcs)}
        for t in range(t0, t1):
            for k in range(int(tp.sub_ptr[t]), int(tp.sub_ptr[t + 1])):
                v = int(tp.pos_src[k])
                ri = reg_of.get((t, v & row_mask))
                pos_slot[k] = (POS_REMOTE | ri if ri is not None else slot_of[v & row_mask]) | \
                    (v & POS_UNIFORM)
        for k in range(t0 * rt, t1 * rt):
            r = int(tp.sub_rows[k])
            sub_slot[k] = slot_of[r] if r >= 0 else 0
        src_rows.extend(int(r) for r in srcs)
        src_ptr.append(len(src_rows))
        max_src = max(max_src, len(srcs))
        max_tiles = max(max_tiles, t1 - t0)
    rem_regs = 0
    if remote and not np.any(rem_rows >= 0):
        rem_rows = None                               # nothing to keep in registers
    elif remote:
        # 8 register rows cost 16 VGPRs fewer than 16 (k_mix_tile_lds NREM: 80 vs 96, three 7-wave
        # blocks per CU instead of two)
        rem_regs = 8 if not np.any(rem_rows.reshape(-1, REM_MAX)[:, 8:] >= 0) else 16
    return TileLdsPlan(tile=tp, pos_slot=pos_slot, sub_slot=sub_slot,
                       grp_tile_ptr=np.asarray(gtp, np.int32),
                       grp_src_ptr=np.asarray(src_ptr, np.int32),
                       grp_src_rows=np.asarray(src_rows, np.int32),
                       max_src=max(max_src, 1), max_tiles=max(max_tiles, 1),
                       rem_rows=rem_rows, rem_regs=rem_regs), None


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


SEG_HARD = 1 << 30           # seg word 0 flag: a MASKED position (rows in word 1, weight in word 2)
SEG_REMOTE = 1 << 29         # with SEG_HARD: the source is register row (word 0 & SEG_SLOT)
SEG_WORDS = 4
SEG_SLOT = 0xfff             # slot field of word 0


@dataclass
class TileSegments:
    """The positions of an RT-16 LDS tile plan cut into SEGMENTS for k_mix_tile_lds's segment loop
    (include/niidmix.h, niidmix_tile_lds_plan.seg*).  A fast segment is a run of positions that
      * read CONSECUTIVE LDS slots s0, s0+1, ... (slots are numbered in list order, so a tile's
        positions mostly do): the kernel reads position i at one base address + i * row bytes, an
        immediate offset, with no per-position descriptor;
      * carry a uniform weight, one of the tile's two (w0, w1 in seg_w; bit i of wsel picks w1);
      * are taken by every tile row, or by all rows but one (bit i of skip), where the k-th such
        position of the segment skips tile row r0 + k (a tile's rows follow the list order, so
        their own positions come in that order).
    Any other position becomes MASKED entries (word 0 = slot | SEG_HARD, word 1 = the rows taking it,
    word 2 = the weight's fp32 bits), one per weight class of its rows: each row still takes the
    position once, at this point of its own order, so exact results are unchanged.
    seg [S, 4] int32: runs s0 | L << 12 | r0 << 20, wsel bits, skip bits, 0 (slots < 4096,
    L <= 32); None when a group stages 4096 rows or more (never: LDS holds ~400).
    seg_ptr [T+1] int32 (segments of tile t), seg_w [T, 2] fp32."""
    seg_ptr: np.ndarray
    seg: np.ndarray
    seg_w: np.ndarray
    lp: object = None            # the TileLdsPlan these segments cut

    @property
    def n_seg(self):
        return len(self.seg)


def build_tile_segments(lp, max_len=32):
    """TileSegments of a TileLdsPlan (RT 16 tiles; any RT works, the kernel uses them at RT 16)."""
    tp = lp.tile
    rt = tp.rt
    full = (1 << rt) - 1
    if lp.max_src + 2 > SEG_SLOT:
        return None
    slots = (lp.pos_slot & (POS_REMOTE - 1)).astype(np.int64)
    remote = (lp.pos_slot & POS_REMOTE) != 0
    uni = (lp.pos_slot & POS_UNIFORM) != 0
    mask = tp.pos_mask.astype(np.int64)
    w0s = tp.pos_w.reshape(-1, rt)[:, 0] if tp.n_pos else np.zeros(0, np.float32)
    seg_ptr, segs, seg_w = [0], [], []
    for t in range(tp.n_sub):
        b, e = int(tp.sub_ptr[t]), int(tp.sub_ptr[t + 1])
        real = 0
        for r in range(rt):
            if tp.sub_rows[t * rt + r] >= 0:
                real |= 1 << r
        ws = []
        for k in range(b, e):                       # the tile's first two uniform weights
            if uni[k] and w0s[k] not in ws:
                ws.append(w0s[k])
                if len(ws) == 2:
                    break
        while len(ws) < 2:
            ws.append(np.float32(0.0))
        wbits = [np.float32(v).view(np.uint32) for v in ws]
        cur = None
        for k in range(b, e):
            miss = int(~mask[k] & full)
            wk = np.float32(w0s[k]).view(np.uint32)
            easy = bool(uni[k]) and (miss & (miss - 1)) == 0 and wk in wbits
            if remote[k]:
                assert not easy, "a register row must be a masked entry (_register_sources)"
            if not easy:
                if cur is not None:
                    segs.append(cur)
                    cur = None
                # MASKED entries: the rows that take the position, one entry per weight class
                # (each row still takes the position once, at this point of its own order)
                m = int(tp.pos_mask[k]) & real
                wr = tp.pos_w[k * rt:(k + 1) * rt]
                classes = {}
                for r in range(rt):
                    if (m >> r) & 1:
                        classes.setdefault(int(np.float32(wr[r]).view(np.uint32)), 0)
                        classes[int(np.float32(wr[r]).view(np.uint32))] |= 1 << r
                for wb, cm in classes.items():
                    segs.append(["M", int(slots[k]) | (SEG_REMOTE if remote[k] else 0), cm, wb])
                continue
            skip = miss.bit_length() - 1 if miss else -1
            sel = 1 if (wk == wbits[1] and wk != wbits[0]) else 0
            ok = (cur is not None and slots[k] == cur[0] + cur[1] and cur[1] < max_len and
                  (skip < 0 or cur[8] is None or cur[8] == skip))
            if not ok:
                if cur is not None:
                    segs.append(cur)
                cur = [int(slots[k]), 0, 0, 0, 0, 0, 0, k, None]
            i = cur[1]
            if sel:
                if i < 32:
                    cur[2] |= 1 << i
                else:
                    cur[3] |= 1 << (i - 32)
            if skip >= 0:
                if cur[8] is None:
                    cur[6] = skip                       # r0: the first skipped row
                if i < 32:
                    cur[4] |= 1 << i
                else:
                    cur[5] |= 1 << (i - 32)
                cur[8] = skip + 1
            cur[1] += 1
        if cur is not None:
            segs.append(cur)
        seg_ptr.append(len(segs))
        seg_w.append(ws)
    arr = np.zeros((len(segs), SEG_WORDS), np.int64)
    for i, sg in enumerate(segs):
        if sg[0] == "M":
            _, slot, cm, wb = sg
            arr[i] = [slot | SEG_HARD, cm, wb, 0]
        else:
            s0, ln, wlo, _, klo, _, r0 = sg[:7]
            arr[i] = [s0 | (ln << 12) | (r0 << 20), wlo, klo, 0]
    arr = (arr & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    return TileSegments(seg_ptr=np.asarray(seg_ptr, np.int32), seg=arr.reshape(-1, SEG_WORDS),
                        seg_w=np.asarray(seg_w, np.float32).reshape(-1, 2), lp=lp)


def rem_two_phase(lp, ts):
    """May k_mix_tile_lds walk this plan's register rows in two phases of 8 (rem_regs -16: 80 VGPRs
    instead of 96)?  Every tile must read register rows 0..7 only before its first segment that
    reads one of 8..15: the kernel loads 0..7 before the walk and 8..15 into the same registers
    there.  rem_rows lists a tile's register rows in first-use order and each is read by one
    masked entry, so d-cliques plans qualify."""
    if lp.rem_rows is None or ts is None or ts.lp is not lp:
        return False
    w0 = np.asarray(ts.seg)[:, 0].astype(np.int64)
    rem = ((w0 & SEG_HARD) != 0) & ((w0 & SEG_REMOTE) != 0)
    high = rem & ((w0 & SEG_SLOT) >= 8)
    low = rem & ((w0 & SEG_SLOT) < 8)
    for t in range(lp.tile.n_sub):
        b, e = int(ts.seg_ptr[t]), int(ts.seg_ptr[t + 1])
        h = np.flatnonzero(high[b:e])
        if len(h) and np.any(low[b + h[0]:e]):
            return False
    return True


def segments_row_lists(lp, ts):
    """{row: [(src, w), ...]} as the segment loop applies them (self first) -- for checks."""
    tp = lp.tile
    rt = tp.rt
    src_rows = lp.grp_src_rows
    gtp = lp.grp_tile_ptr
    grp_of = np.zeros(tp.n_sub, np.int64)
    for gi in range(len(gtp) - 1):
        grp_of[gtp[gi]:gtp[gi + 1]] = gi
    out = {}
    seg = ts.seg.view(np.uint32).astype(np.int64)
    for t in range(tp.n_sub):
        base = int(lp.grp_src_ptr[grp_of[t]])
        rows = tp.sub_rows[t * rt:(t + 1) * rt]
        lists = {r: [(int(rows[r]), np.float32(tp.sub_wself[t * rt + r]))]
                 for r in range(rt) if rows[r] >= 0}
        w0, w1 = ts.seg_w[t]
        for s in seg[ts.seg_ptr[t]:ts.seg_ptr[t + 1]]:
            hd = int(s[0])
            if hd & SEG_HARD:
                if hd & SEG_REMOTE:
                    src = int(lp.rem_rows[t * REM_MAX + (hd & SEG_SLOT)])
                else:
                    src = int(src_rows[base + (hd & SEG_SLOT)])
                m, w = int(s[1]), np.uint32(s[2]).view(np.float32)
                for r in lists:
                    if (m >> r) & 1:
                        lists[r].append((src, np.float32(w)))
                continue
            s0, ln, r_skip = hd & SEG_SLOT, (hd >> 12) & 0xff, (hd >> 20) & 0xff
            wsel, skip = int(s[1]), int(s[2])
            for i in range(ln):
                src = int(src_rows[base + s0 + i])
                w = w1 if (wsel >> i) & 1 else w0
                skipped = -1
                if (skip >> i) & 1:
                    skipped = r_skip
                    r_skip += 1
                for r in lists:
                    if r != skipped:
                        lists[r].append((src, np.float32(w)))
        for r, lst in lists.items():
            out[int(rows[r])] = lst
    return out


@dataclass
class TileMfmaPositions:
    """The positions of an RT-16 LDS tile plan as MFMA position lists (k_mix_tile_lds's matrix-core
    path, exact mode; include/niidmix.h niidmix_tile_lds_plan.mf*).

    v_mfma_f32_16x16x4_f32 is bit for bit a k-ordered chain of fp32 fmas, one rounding each
    (tools/mfma_exact_probe.hip: 0 mismatches in 2.7e8 chained outputs).  With A[col][k] =
    fl(w_k * x_{slot k}[col]) and B[k][row] = 1 when the tile row takes position k, else 0, each step
    is fl(acc + fl(w x)) for the rows that take it -- the reference's add_(w*p) -- and acc + (+-0)
    for the others, which leaves acc unchanged unless acc is -0 (the kernel's per-block check makes
    sure it never is: every staged value is finite and at least 1e-30 in magnitude, so each row's
    accumulator is non-zero after its self term; else the block takes the segment walker).
    A position whose rows carry different weights becomes one entry per weight class (each row
    still takes it once, at this point of its own order).  Tiles are padded to a multiple of 4
    entries with (slot 0, weight 0, no rows).
      mf_ptr [T+1] int32: entries of tile t;  mf [E, 4] int32: slot, weight (fp32 bits), row mask, 0"""
    mf_ptr: np.ndarray
    mf: np.ndarray
    lp: object = None

    @property
    def n_entries(self):
        return len(self.mf)


def build_tile_mfma_positions(lp):
    """TileMfmaPositions of a TileLdsPlan (RT 16 tiles)."""
    tp = lp.tile
    rt = tp.rt
    if rt != 16 or lp.rem_rows is not None:      # the matrix-core path reads every source from LDS
        return None
    slots = (lp.pos_slot & (POS_UNIFORM - 1)).astype(np.int64)
    uni = (lp.pos_slot & POS_UNIFORM) != 0
    ptr, ent = [0], []
    for t in range(tp.n_sub):
        real = 0
        for r in range(rt):
            if tp.sub_rows[t * rt + r] >= 0:
                real |= 1 << r
        n0 = len(ent)
        for k in range(int(tp.sub_ptr[t]), int(tp.sub_ptr[t + 1])):
            m = int(tp.pos_mask[k]) & real
            if m == 0:
                continue
            wr = tp.pos_w[k * rt:(k + 1) * rt]
            if uni[k]:
                ent.append((int(slots[k]), int(np.float32(wr[0]).view(np.uint32)), m))
                continue
            classes = {}
            for r in range(rt):
                if (m >> r) & 1:
                    wb = int(np.float32(wr[r]).view(np.uint32))
                    classes[wb] = classes.get(wb, 0) | (1 << r)
            for wb, cm in classes.items():
                ent.append((int(slots[k]), wb, cm))
        while (len(ent) - n0) % 4:
            ent.append((0, 0, 0))
        ptr.append(len(ent))
    arr = np.zeros((len(ent), 4), np.int64)
    if ent:
        arr[:, :3] = np.asarray(ent, np.int64)
    arr = (arr & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
    return TileMfmaPositions(mf_ptr=np.asarray(ptr, np.int32), mf=arr.reshape(-1, 4), lp=lp)


def mfma_row_lists(lp, tm):
    """{row: [(src, w), ...]} as the MFMA path applies them (self first) -- for checks."""
    tp = lp.tile
    rt = tp.rt
    gtp = lp.grp_tile_ptr
    grp_of = np.zeros(tp.n_sub, np.int64)
    for gi in range(len(gtp) - 1):
        grp_of[gtp[gi]:gtp[gi + 1]] = gi
    out = {}
    mf = tm.mf.view(np.uint32).astype(np.int64)
    for t in range(tp.n_sub):
        base = int(lp.grp_src_ptr[grp_of[t]])
        rows = tp.sub_rows[t * rt:(t + 1) * rt]
        lists = {r: [(int(rows[r]), np.float32(tp.sub_wself[t * rt + r]))]
                 for r in range(rt) if rows[r] >= 0}
        for e in mf[tm.mf_ptr[t]:tm.mf_ptr[t + 1]]:
            slot, wb, m = int(e[0]), np.uint32(e[1]).view(np.float32), int(e[2])
            for r in lists:
                if (m >> r) & 1:
                    lists[r].append((int(lp.grp_src_rows[base + slot]), np.float32(wb)))
        for r, lst in lists.items():
            out[int(rows[r])] = lst
    return out
