"""PyTorch-ROCm custom ops over libniidmix.so, and the Mixer that picks a kernel per topology.

Ops (registered in the `niidmix` namespace, usable as torch.ops.niidmix.*):
  mix_csr(x, row_ptr, col, val, out, mode)          k_mix_csr    exact (bit-exact) or fast
  mix_ell(x, ell_col, ell_val, ell_len, out, k, mode)  k_mix_ell  the same, low-degree graphs
  mix_band(x, ell_col, ell_val, ell_len, out, k, band, mode)
                                                    k_mix_band   the same, banded rows (a ring in
                                                    its cycle order, band_layout)
  mix_clique(x, clique_ptr, member_row, member_group, coef, res_ptr, res_col, res_val, res_member,
             row_ptr, col, val, out, max_clique, max_clique_res)
                                                    k_mix_clique (fast, HBM-bound; the CSR is the
                                                    non-finite guard, include/niidmix.h)
  mix_clique_blocked(..., out, p, ...)              the same on column-blocked slabs
  mix_tile_lds(x, <tile lds plan tensors>, out, rt, max_src, max_tiles, mode)
                                                    k_mix_tile_lds (exact default, LDS-staged)
  mix_dense(x, w, row_ptr, col, val, out)           k_mix_dense  (fp32 MFMA; CSR = non-finite guard)
  mix_dense_b6(x, wp, row_ptr, col, val, out)       k_mix_dense_b6 (bf16 MFMA, fp32-accurate splits)
  mean_rows(x, mean, dist2, mode)                   k_mean_cols + k_row_dist2
  grad_segment_mean(g, seg_ptr, seg_row, out)       k_grad_segment_mean (clique gradient mean)
  sgd_step_rows(p, g, rows, neg_lr)                 k_sgd_step_rows (the optimizer step, fused round)
  mix_csr(..., mode | MEAN)                         per-row gradient mean (unbiased / removed edges)
All ops launch on torch's current HIP stream of the input's device, never synchronise, and raise
RuntimeError (TORCH_CHECK-style) on bad arguments.  They accept HIP tensors only: there is no CPU
implementation and no fallback.
"""
import ctypes
import os
from typing import Optional

import numpy as np
import torch

from . import _lib
from .factor import build_clique_plan
from .tile import (LDS_MAX_WAVES, balanced_tile_rows, build_tile_lds_plan, build_tile_mfma_positions,
                   build_tile_plan, build_tile_segments, rem_two_phase)
from .topology import MixCSR, to_csr

EXACT, FAST = _lib.MODE_EXACT, _lib.MODE_FAST
AVERAGE_ONLY = 2
LOW_DEGREE = 4
MEAN = 8
MEMBER_GATEWAY = 256        # member_group hint bit (include/niidmix.h NIIDMIX_MEMBER_GATEWAY)


def _stream(t):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _req(cond, msg):
    if not cond:
        raise RuntimeError(msg)


def _slab(name, t, rows=None, cols=None):
    _req(isinstance(t, torch.Tensor), f"{name}: expected a tensor")
    _req(t.is_cuda, f"{name}: expected a HIP (cuda) tensor, got {t.device} (no CPU fallback)")
    _req(t.dtype == torch.float32, f"{name}: expected float32, got {t.dtype}")
    _req(t.dim() == 2, f"{name}: expected a 2-D [rows, p] slab")
    _req(t.stride(1) == 1 or t.shape[1] <= 1, f"{name}: rows must be contiguous (stride(1) == 1)")
    if rows is not None:
        _req(t.shape[0] == rows, f"{name}: expected {rows} rows, got {t.shape[0]}")
    if cols is not None:
        _req(t.shape[1] == cols, f"{name}: expected {cols} columns, got {t.shape[1]}")


def _vec(name, t, dtype, device, n=None):
    _req(t.device == device, f"{name}: must be on {device}")
    _req(t.dtype == dtype, f"{name}: expected {dtype}, got {t.dtype}")
    _req(t.dim() == 1 and t.is_contiguous(), f"{name}: expected a contiguous 1-D tensor")
    if n is not None:
        _req(t.numel() == n, f"{name}: expected {n} elements, got {t.numel()}")


def _no_overlap(a, b):
    if a.numel() == 0 or b.numel() == 0:
        return
    sa, sb = a.untyped_storage(), b.untyped_storage()
    if sa.data_ptr() != sb.data_ptr():
        return
    a0, b0 = a.data_ptr(), b.data_ptr()
    a1 = a0 + ((a.shape[0] - 1) * a.stride(0) + a.shape[1]) * 4
    b1 = b0 + ((b.shape[0] - 1) * b.stride(0) + b.shape[1]) * 4
    _req(a1 <= b0 or b1 <= a0, "x and out overlap: mixing is out-of-place (Jacobi, d_sgd.py:99-116)")


def _blocked_no_overlap(a, b, msg):
    """Two column-blocked [K, rows, B] slabs must not share a byte: each one's extent from its OWN
    block and row strides (the two may differ in block stride)."""
    if a.numel() == 0 or b.numel() == 0:
        return
    if a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr():
        return

    def ext(t):
        k, rows, bc = t.shape
        return ((k - 1) * t.stride(0) + (rows - 1) * t.stride(1) + bc) * 4
    a0, b0 = a.data_ptr(), b.data_ptr()
    _req(a0 + ext(a) <= b0 or b0 + ext(b) <= a0, msg)


def _ld(t):
    return t.stride(0) if t.shape[0] > 1 else max(t.shape[1], 1)


@torch.library.custom_op("niidmix::mix_csr", mutates_args=("out",))
def mix_csr(x: torch.Tensor, row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor,
            out: torch.Tensor, mode: int) -> None:
    _slab("x", x)
    _slab("out", out, cols=x.shape[1])
    _req(out.device == x.device, "x and out must be on the same device")
    n = out.shape[0]
    _vec("row_ptr", row_ptr, torch.int64, x.device, n + 1)
    _vec("col", col, torch.int32, x.device)
    _vec("val", val, torch.float32, x.device, col.numel())
    _no_overlap(x, out)
    rc = _lib.lib.niidmix_mix_csr_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out), n, x.shape[1],
                                      row_ptr.data_ptr(), col.data_ptr(), val.data_ptr(), int(mode),
                                      _stream(x))
    _lib.check(rc, "niidmix::mix_csr")


@torch.library.custom_op("niidmix::mix_ell", mutates_args=("out",))
def mix_ell(x: torch.Tensor, ell_col: torch.Tensor, ell_val: torch.Tensor, ell_len: torch.Tensor,
            out: torch.Tensor, k: int, mode: int) -> None:
    """mix_csr over the ELL layout of the same rows (low-degree graphs; include/niidmix.h)."""
    _slab("x", x)
    _slab("out", out, cols=x.shape[1])
    _req(out.device == x.device, "x and out must be on the same device")
    n = out.shape[0]
    # the kernel reads x[row] (the row's own entry) for every output row before its descriptors
    _req(x.shape[0] >= n, f"x has {x.shape[0]} rows, fewer than the {n} output rows")
    _vec("ell_col", ell_col, torch.int32, x.device, n * k)
    _vec("ell_val", ell_val, torch.float32, x.device, n * k)
    _vec("ell_len", ell_len, torch.int32, x.device, n)
    _no_overlap(x, out)
    rc = _lib.lib.niidmix_mix_ell_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out), n, x.shape[1],
                                      int(k), ell_col.data_ptr(), ell_val.data_ptr(),
                                      ell_len.data_ptr(), int(mode), _stream(x))
    _lib.check(rc, "niidmix::mix_ell")


def ell_layout(csr):
    """(k, col [N*k], val [N*k], len [N]) of the CSR's rows, padded to k in {3, 5, 8} entries, or
    None when a row has more than 8 entries.  Padding repeats the row's self entry (never summed:
    the kernel stops at len)."""
    lens = np.diff(csr.row_ptr)
    if csr.n == 0 or lens.max() > 8:
        return None
    k = 3 if lens.max() <= 3 else 5 if lens.max() <= 5 else 8
    n = csr.n
    col = np.repeat(np.arange(n, dtype=np.int32), k).reshape(n, k)
    val = np.zeros((n, k), np.float32)
    j = np.arange(int(csr.row_ptr[-1])) - np.repeat(csr.row_ptr[:-1], lens)
    r = np.repeat(np.arange(n), lens)
    col[r, j] = csr.col
    val[r, j] = csr.val
    return k, col.reshape(-1), val.reshape(-1), lens.astype(np.int32)


@torch.library.custom_op("niidmix::mix_band", mutates_args=("out",))
def mix_band(x: torch.Tensor, ell_col: torch.Tensor, ell_val: torch.Tensor, ell_len: torch.Tensor,
             out: torch.Tensor, k: int, band: int, mode: int) -> None:
    """mix_ell over rows whose entries all lie within +-band rows (cyclic; include/niidmix.h
    niidmix_mix_band_f32).  The band itself is the caller's contract (Mixer checks it once per
    topology, band_of)."""
    _slab("x", x)
    _slab("out", out, cols=x.shape[1])
    _req(out.device == x.device, "x and out must be on the same device")
    n = out.shape[0]
    _req(x.shape[0] == n, f"x has {x.shape[0]} rows, the band kernel reads exactly the {n} output rows")
    _vec("ell_col", ell_col, torch.int32, x.device, n * k)
    _vec("ell_val", ell_val, torch.float32, x.device, n * k)
    _vec("ell_len", ell_len, torch.int32, x.device, n)
    _no_overlap(x, out)
    rc = _lib.lib.niidmix_mix_band_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out), n,
                                       x.shape[1], int(k), int(band), ell_col.data_ptr(),
                                       ell_val.data_ptr(), ell_len.data_ptr(), int(mode), _stream(x))
    _lib.check(rc, "niidmix::mix_band")


@torch.library.custom_op("niidmix::mix_strip", mutates_args=("out",))
def mix_strip(x: torch.Tensor, ell_col: torch.Tensor, ell_val: torch.Tensor, ell_len: torch.Tensor,
              out: torch.Tensor, k: int, mode: int) -> None:
    """mix_ell for few nodes (<= STRIP_MAX_ROWS) by column strips staged in LDS (include/niidmix.h
    niidmix_mix_strip_f32): each element of x is read once; any row order."""
    _slab("x", x)
    _slab("out", out, cols=x.shape[1])
    _req(out.device == x.device, "x and out must be on the same device")
    n = out.shape[0]
    _req(n <= STRIP_MAX_ROWS, f"strip kernel: {n} rows (<= {STRIP_MAX_ROWS})")
    _req(x.shape[0] >= n, f"x has {x.shape[0]} rows, fewer than the {n} output rows")
    _vec("ell_col", ell_col, torch.int32, x.device, n * k)
    _vec("ell_val", ell_val, torch.float32, x.device, n * k)
    _vec("ell_len", ell_len, torch.int32, x.device, n)
    _no_overlap(x, out)
    rc = _lib.lib.niidmix_mix_strip_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out), n,
                                        x.shape[1], int(k), ell_col.data_ptr(), ell_val.data_ptr(),
                                        ell_len.data_ptr(), int(mode), _stream(x))
    _lib.check(rc, "niidmix::mix_strip")


STRIP_MAX_ROWS = 256

# (ELL width, band) pairs the band kernel is built for
BAND_OF_K = {3: 1, 5: 2}


def band_of(csr, k):
    """The band B of k_mix_band for this CSR at ELL width k (B = BAND_OF_K[k]) if every entry of row
    r reads a row r + d (mod N) with |d| <= B, else None.  Needs N >= 2B + 1 and no halo rows."""
    b = BAND_OF_K.get(k)
    n = csr.n
    if b is None or csr.n_in != n or n < 2 * b + 1:
        return None
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(csr.row_ptr))
    d = (csr.col.astype(np.int64) - rows) % n
    return b if bool(np.all((d <= b) | (d >= n - b))) else None


def band_layout(csr):
    """Row order that makes a RING banded (band 1): perm[i] = position of node i along its cycle,
    starting at node 0 (the reference's ring.create orders nodes by a metric, ring.py:12-27, so the
    rank order is not the cycle order).  None unless every node has exactly two distinct
    neighbours, both ways, forming one cycle."""
    n = csr.n
    if n < 3 or csr.n_in != n or not np.all(np.diff(csr.row_ptr) == 3):
        return None
    nb = csr.col.reshape(n, 3)[:, 1:].astype(np.int64)
    if np.any(nb[:, 0] == nb[:, 1]) or np.any(nb == np.arange(n)[:, None]):
        return None
    order = [0]
    prev, cur = -1, 0
    for _ in range(n - 1):
        a, b = int(nb[cur, 0]), int(nb[cur, 1])
        nxt = a if a != prev else b
        if cur not in (int(nb[nxt, 0]), int(nb[nxt, 1])):
            return None                       # not symmetric
        prev, cur = cur, nxt
        order.append(cur)
    if len(set(order)) != n or 0 not in (int(nb[cur, 0]), int(nb[cur, 1])):
        return None
    perm = np.empty(n, np.int64)
    perm[np.asarray(order, np.int64)] = np.arange(n)
    return perm


@torch.library.custom_op("niidmix::mix_clique", mutates_args=("out",))
def mix_clique(x: torch.Tensor, clique_ptr: torch.Tensor, member_row: torch.Tensor,
               member_group: torch.Tensor, coef: torch.Tensor, res_ptr: torch.Tensor,
               res_col: torch.Tensor, res_val: torch.Tensor, res_member: torch.Tensor,
               row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor,
               out: torch.Tensor, max_clique: int, max_clique_res: int) -> None:
    _slab("x", x)
    _slab("out", out, cols=x.shape[1])
    _req(member_row.device == x.device, "plan and slabs must be on the same device")
    _no_overlap(x, out)
    plan = _clique_plan_c(clique_ptr, member_row, member_group, coef, res_ptr, res_col, res_val,
                          res_member, row_ptr, col, val, max_clique, max_clique_res)
    rc = _lib.lib.niidmix_mix_clique_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out), x.shape[1],
                                         ctypes.byref(plan), _stream(x))
    _lib.check(rc, "niidmix::mix_clique")


def _clique_plan_c(clique_ptr, member_row, member_group, coef, res_ptr, res_col, res_val,
                   res_member, row_ptr, col, val, max_clique, max_clique_res):
    dev = member_row.device
    _vec("row_ptr", row_ptr, torch.int64, dev, member_row.numel() + 1)
    _vec("col", col, torch.int32, dev)
    _vec("val", val, torch.float32, dev, col.numel())
    _vec("clique_ptr", clique_ptr, torch.int32, dev)
    m = member_row.numel()
    _vec("member_row", member_row, torch.int32, dev)
    _vec("member_group", member_group, torch.int32, dev, m)
    _req(coef.device == dev and coef.dtype == torch.float32 and coef.dim() == 2 and
         coef.shape[0] == m and coef.is_contiguous(), "coef: expected contiguous fp32 [M, 1+G]")
    g = coef.shape[1] - 1
    _req(1 <= g <= 4, "coef: 1..4 groups supported")
    _vec("res_ptr", res_ptr, torch.int32, dev, m + 1)
    _vec("res_col", res_col, torch.int32, dev)
    _vec("res_val", res_val, torch.float32, dev, res_col.numel())
    _vec("res_member", res_member, torch.int32, dev, res_col.numel())
    return _lib.CliquePlanC(clique_ptr.numel() - 1, m, g, int(max_clique), int(max_clique_res),
                            clique_ptr.data_ptr(),
                            member_row.data_ptr(), member_group.data_ptr(), coef.data_ptr(),
                            res_ptr.data_ptr(), res_col.data_ptr() if res_col.numel() else
                            res_ptr.data_ptr(), res_val.data_ptr() if res_val.numel() else
                            coef.data_ptr(), res_member.data_ptr() if res_member.numel() else
                            res_ptr.data_ptr(), row_ptr.data_ptr(), col.data_ptr(), val.data_ptr())


@torch.library.custom_op("niidmix::mix_clique_blocked", mutates_args=("out",))
def mix_clique_blocked(x: torch.Tensor, clique_ptr: torch.Tensor, member_row: torch.Tensor,
                       member_group: torch.Tensor, coef: torch.Tensor, res_ptr: torch.Tensor,
                       res_col: torch.Tensor, res_val: torch.Tensor, res_member: torch.Tensor,
                       row_ptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor,
                       out: torch.Tensor, p: int, max_clique: int, max_clique_res: int) -> None:
    """Clique-factored round on column-blocked slabs x, out: [K, rows, B] (niidmix.memory)."""
    for name, t in (("x", x), ("out", out)):
        _req(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and
             t.dim() == 3 and t.stride(2) == 1,
             f"{name}: expected a HIP fp32 [K, rows, B] blocked slab with unit column stride")
    _req(x.shape == out.shape and x.stride(1) == out.stride(1), "x and out: same blocked geometry")
    k, rows, b = x.shape
    _req(0 <= p <= k * b and (k == 0 or p > (k - 1) * b), f"p={p} does not fit {k} blocks of {b}")
    _req(member_row.device == x.device, "plan and slabs must be on the same device")
    _blocked_no_overlap(x, out, "x and out overlap: mixing is out-of-place")
    plan = _clique_plan_c(clique_ptr, member_row, member_group, coef, res_ptr, res_col, res_val,
                          res_member, row_ptr, col, val, max_clique, max_clique_res)
    rc = _lib.lib.niidmix_mix_clique_blocked_f32(x.data_ptr(), out.data_ptr(), int(p), x.stride(1),
                                                 b, x.stride(0), out.stride(0),
                                                 ctypes.byref(plan), _stream(x))
    _lib.check(rc, "niidmix::mix_clique_blocked")


@torch.library.custom_op("niidmix::mix_tile", mutates_args=("out",))
def mix_tile(x: torch.Tensor, sub_ptr: torch.Tensor, sub_rows: torch.Tensor,
             sub_wself: torch.Tensor, pos_src: torch.Tensor, pos_mask: torch.Tensor,
             pos_w: torch.Tensor, out: torch.Tensor, rt: int, mode: int) -> None:
    _slab("x", x)
    _slab("out", out, cols=x.shape[1])
    dev = x.device
    t = sub_ptr.numel() - 1
    _vec("sub_ptr", sub_ptr, torch.int64, dev)
    _vec("sub_rows", sub_rows, torch.int32, dev, t * rt)
    _vec("sub_wself", sub_wself, torch.float32, dev, t * rt)
    _vec("pos_src", pos_src, torch.int32, dev)
    _vec("pos_mask", pos_mask, torch.int32, dev, pos_src.numel())      # uint32 bits
    _vec("pos_w", pos_w, torch.float32, dev, pos_src.numel() * rt)
    _no_overlap(x, out)
    # a plan without positions (every row reads only itself, e.g. N = 1) still passes valid
    # pointers: the C-ABI refuses NULL, and the kernel reads pos_* only inside sub_ptr ranges
    some = sub_ptr.data_ptr()
    plan = _lib.TilePlanC(t, int(rt), 0, sub_ptr.data_ptr(), sub_rows.data_ptr(),
                          sub_wself.data_ptr(), pos_src.data_ptr() or some,
                          pos_mask.data_ptr() or some, pos_w.data_ptr() or some)
    rc = _lib.lib.niidmix_mix_tile_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out), out.shape[0],
                                       x.shape[1], ctypes.byref(plan), int(mode), _stream(x))
    _lib.check(rc, "niidmix::mix_tile")


@torch.library.custom_op("niidmix::mix_tile_lds", mutates_args=("out",))
def mix_tile_lds(x: torch.Tensor, sub_ptr: torch.Tensor, sub_rows: torch.Tensor,
                 sub_slot: torch.Tensor, sub_wself: torch.Tensor, pos_slot: torch.Tensor,
                 pos_mask: torch.Tensor, pos_w: torch.Tensor, grp_tile_ptr: torch.Tensor,
                 grp_src_ptr: torch.Tensor, grp_src_rows: torch.Tensor, out: torch.Tensor, rt: int,
                 max_src: int, max_tiles: int, mode: int, seg_ptr: Optional[torch.Tensor] = None,
                 seg: Optional[torch.Tensor] = None, seg_w: Optional[torch.Tensor] = None,
                 mf_ptr: Optional[torch.Tensor] = None, mf: Optional[torch.Tensor] = None,
                 rem_rows: Optional[torch.Tensor] = None, rem_regs: int = 16) -> None:
    """seg_ptr / seg / seg_w: the plan's segments (niidmix.tile.build_tile_segments, RT 16 only):
    the kernel's segment loop instead of the per-position loop; bit-identical results.
    mf_ptr / mf: its MFMA position lists (niidmix.tile.build_tile_mfma_positions; needs the
    segments, exact mode): the matrix-core path, bit-identical, the walker its per-block fallback.
    rem_rows: the plan's register rows (build_tile_lds_plan(remote_regs=True); segments only);
    rem_regs: how many of each tile's 16 entries the kernel loads (8 when no tile has more, else 16;
    TileLdsPlan.rem_regs), or -16: all 16 in two phases of 8 (tile.rem_two_phase plans only)."""
    _slab("x", x)
    _slab("out", out, cols=x.shape[1])
    dev = x.device
    t = sub_ptr.numel() - 1
    g = grp_tile_ptr.numel() - 1
    _vec("sub_ptr", sub_ptr, torch.int64, dev)
    _vec("sub_rows", sub_rows, torch.int32, dev, t * rt)
    _vec("sub_slot", sub_slot, torch.int32, dev, t * rt)
    _vec("sub_wself", sub_wself, torch.float32, dev, t * rt)
    _vec("pos_slot", pos_slot, torch.int32, dev)
    _vec("pos_mask", pos_mask, torch.int32, dev, pos_slot.numel())      # uint32 bits
    _vec("pos_w", pos_w, torch.float32, dev, pos_slot.numel() * rt)
    _vec("grp_tile_ptr", grp_tile_ptr, torch.int32, dev)
    _vec("grp_src_ptr", grp_src_ptr, torch.int32, dev, g + 1)
    _vec("grp_src_rows", grp_src_rows, torch.int32, dev)
    segs = (None, None, None)
    if seg_ptr is not None:
        _req(rt == 16 and seg is not None and seg_w is not None,
             "segments: RT 16 plans, with seg_ptr, seg and seg_w")
        _vec("seg_ptr", seg_ptr, torch.int32, dev, t + 1)
        _vec("seg", seg, torch.int32, dev)
        _req(seg.numel() % 4 == 0 and seg.data_ptr() % 16 == 0, "seg: [S, 4] int32, 16-B aligned")
        _vec("seg_w", seg_w, torch.float32, dev, 2 * t)
        segs = (seg_ptr.data_ptr(), seg.data_ptr(), seg_w.data_ptr())
    mfs = (None, None)
    if mf_ptr is not None:
        _req(seg_ptr is not None and mf is not None, "MFMA position lists: with the segments, mf_ptr and mf")
        _vec("mf_ptr", mf_ptr, torch.int32, dev, t + 1)
        _vec("mf", mf, torch.int32, dev)
        _req(mf.numel() % 4 == 0 and mf.data_ptr() % 16 == 0, "mf: [E, 4] int32, 16-B aligned")
        mfs = (mf_ptr.data_ptr(), mf.data_ptr() if mf.numel() else mf_ptr.data_ptr())
    rem = None
    if rem_rows is not None:
        _req(seg_ptr is not None and mf_ptr is None,
             "register rows: with the segments and without the MFMA position lists")
        _vec("rem_rows", rem_rows, torch.int32, dev, t * 16)       # rows < x.shape[0]: the plan's
        _req(rem_regs in (8, 16, -16), f"rem_regs {rem_regs} (8, 16 or -16)")
        rem = rem_rows.data_ptr()
    _no_overlap(x, out)
    some = sub_ptr.data_ptr()
    plan = _lib.TileLdsPlanC(t, int(rt), g, int(max_src), int(max_tiles), sub_ptr.data_ptr(),
                             sub_rows.data_ptr(), sub_slot.data_ptr(), sub_wself.data_ptr(),
                             pos_slot.data_ptr() or some, pos_mask.data_ptr() or some,
                             pos_w.data_ptr() or some, grp_tile_ptr.data_ptr(),
                             grp_src_ptr.data_ptr(), grp_src_rows.data_ptr(), *segs, *mfs, rem,
                             int(rem_regs) if rem is not None else 0)
    rc = _lib.lib.niidmix_mix_tile_lds_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out),
                                           out.shape[0], x.shape[1], ctypes.byref(plan), int(mode),
                                           _stream(x))
    _lib.check(rc, "niidmix::mix_tile_lds")


@torch.library.custom_op("niidmix::mix_dense", mutates_args=("out",))
def mix_dense(x: torch.Tensor, w: torch.Tensor, row_ptr: torch.Tensor, col: torch.Tensor,
              val: torch.Tensor, out: torch.Tensor) -> None:
    _slab("x", x)
    n = x.shape[0]
    _slab("out", out, rows=n, cols=x.shape[1])
    _req(w.device == x.device and w.dtype == torch.float32 and w.shape == (n, n) and
         w.is_contiguous(), "w: expected contiguous fp32 [N, N] (W[src, dst])")
    _vec("row_ptr", row_ptr, torch.int64, x.device, n + 1)
    _vec("col", col, torch.int32, x.device)
    _vec("val", val, torch.float32, x.device, col.numel())
    _no_overlap(x, out)
    rc = _lib.lib.niidmix_mix_dense_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out), n,
                                        x.shape[1], w.data_ptr(), row_ptr.data_ptr(),
                                        col.data_ptr(), val.data_ptr(), _stream(x))
    _lib.check(rc, "niidmix::mix_dense")


def dense_split_w(w: torch.Tensor) -> torch.Tensor:
    """W^T split into three bf16 planes for mix_dense_b6 (niidmix_dense_split_w): uint16 storage of
    niidmix_dense_split_elems(n) elements on w's device, made once per topology."""
    _req(w.is_cuda and w.dtype == torch.float32 and w.dim() == 2 and w.shape[0] == w.shape[1]
         and w.is_contiguous(), "w: expected contiguous fp32 [N, N] on a HIP device")
    n = w.shape[0]
    wp = torch.empty(int(_lib.lib.niidmix_dense_split_elems(n)), dtype=torch.int16, device=w.device)
    rc = _lib.lib.niidmix_dense_split_w(w.data_ptr(), n, wp.data_ptr(), _stream(w))
    _lib.check(rc, "niidmix::dense_split_w")
    return wp


@torch.library.custom_op("niidmix::mix_dense_b6", mutates_args=("out",))
def mix_dense_b6(x: torch.Tensor, wp: torch.Tensor, row_ptr: torch.Tensor, col: torch.Tensor,
                 val: torch.Tensor, out: torch.Tensor) -> None:
    """Y = W^T X on the bf16 matrix cores with fp32 accuracy (three-term splits, six products;
    include/niidmix.h niidmix_mix_dense_bf16x6_f32); wp from dense_split_w."""
    _slab("x", x)
    n = x.shape[0]
    _slab("out", out, rows=n, cols=x.shape[1])
    _req(wp.device == x.device and wp.dtype == torch.int16 and wp.is_contiguous() and
         wp.numel() == int(_lib.lib.niidmix_dense_split_elems(n)),
         "wp: expected the dense_split_w planes of an [N, N] W")
    _vec("row_ptr", row_ptr, torch.int64, x.device, n + 1)
    _vec("col", col, torch.int32, x.device)
    _vec("val", val, torch.float32, x.device, col.numel())
    _no_overlap(x, out)
    rc = _lib.lib.niidmix_mix_dense_bf16x6_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out), n,
                                               x.shape[1], wp.data_ptr(), row_ptr.data_ptr(),
                                               col.data_ptr(), val.data_ptr(), _stream(x))
    _lib.check(rc, "niidmix::mix_dense_b6")


@torch.library.custom_op("niidmix::mean_rows", mutates_args=("mean", "dist2"))
def mean_rows(x: torch.Tensor, mean: torch.Tensor, dist2: torch.Tensor, mode: int) -> None:
    _slab("x", x)
    _req(mean.device == x.device and mean.dtype == torch.float32 and mean.numel() == x.shape[1]
         and mean.is_contiguous(), "mean: expected contiguous fp32 [p]")
    want_d = dist2.numel() > 0
    if want_d:
        _req(dist2.device == x.device and dist2.dtype == torch.float64 and
             dist2.numel() == x.shape[0], "dist2: expected fp64 [n] (or empty)")
    rc = _lib.lib.niidmix_mean_rows_f32(x.data_ptr(), _ld(x), x.shape[0], x.shape[1],
                                        mean.data_ptr(), dist2.data_ptr() if want_d else None,
                                        int(mode), _stream(x))
    _lib.check(rc, "niidmix::mean_rows")


@torch.library.custom_op("niidmix::grad_segment_mean", mutates_args=("out",))
def grad_segment_mean(g: torch.Tensor, seg_ptr: torch.Tensor, seg_row: torch.Tensor,
                      out: torch.Tensor) -> None:
    _slab("g", g)
    _slab("out", out, cols=g.shape[1])
    dev = g.device
    _req(out.device == dev, "g and out must be on the same device")
    _vec("seg_ptr", seg_ptr, torch.int32, dev)
    _vec("seg_row", seg_row, torch.int32, dev)
    _no_overlap(g, out)
    _req(out.shape[0] == g.shape[0], "g and out: same rows")
    rc = _lib.lib.niidmix_grad_segment_mean_f32(g.data_ptr(), _ld(g), out.data_ptr(), _ld(out),
                                                g.shape[0], g.shape[1], seg_ptr.numel() - 1,
                                                seg_ptr.data_ptr(), seg_row.data_ptr(), _stream(g))
    _lib.check(rc, "niidmix::grad_segment_mean")


@torch.library.custom_op("niidmix::grad_segment_mean_blocked", mutates_args=("out",))
def grad_segment_mean_blocked(g: torch.Tensor, seg_ptr: torch.Tensor, seg_row: torch.Tensor,
                              out: torch.Tensor, p: int) -> None:
    """grad_segment_mean on column-blocked slabs g, out: [K, rows, B] (niidmix.memory)."""
    for name, t in (("g", g), ("out", out)):
        _req(isinstance(t, torch.Tensor) and t.is_cuda and t.dtype == torch.float32 and
             t.dim() == 3 and t.stride(2) == 1,
             f"{name}: expected a HIP fp32 [K, rows, B] blocked slab with unit column stride")
    _req(g.shape == out.shape and g.stride(1) == out.stride(1), "g and out: same blocked geometry")
    k, rows, b = g.shape
    _req(0 <= p <= k * b and (k == 0 or p > (k - 1) * b), f"p={p} does not fit {k} blocks of {b}")
    _vec("seg_ptr", seg_ptr, torch.int32, g.device)
    _vec("seg_row", seg_row, torch.int32, g.device)
    _blocked_no_overlap(g, out, "g and out overlap: the mean is out-of-place")
    rc = _lib.lib.niidmix_grad_segment_mean_blocked_f32(
        g.data_ptr(), out.data_ptr(), rows, int(p), g.stride(1), b, g.stride(0), out.stride(0),
        seg_ptr.numel() - 1, seg_ptr.data_ptr(), seg_row.data_ptr(), _stream(g))
    _lib.check(rc, "niidmix::grad_segment_mean_blocked")


@torch.library.custom_op("niidmix::update_rows", mutates_args=("out",))
def update_rows(x: torch.Tensor, avg: torch.Tensor, out: torch.Tensor) -> None:
    """out[i] = fl(fl(x[i] * 0) + avg) for every row (out may be x itself): update_models(all_models,
    avg) of the 'sample' topology's round (d_sgd.py:246-250, :29-35)."""
    _slab("x", x)
    _slab("out", out, rows=x.shape[0], cols=x.shape[1])
    _req(avg.device == x.device and out.device == x.device and avg.dtype == torch.float32 and
         avg.dim() == 1 and avg.numel() == x.shape[1] and avg.is_contiguous(),
         "avg: expected contiguous fp32 [p] on the slab's device")
    if not (out.data_ptr() == x.data_ptr() and _ld(out) == _ld(x)):
        _no_overlap(x, out)
    rc = _lib.lib.niidmix_update_rows_f32(x.data_ptr(), _ld(x), out.data_ptr(), _ld(out),
                                          x.shape[0], x.shape[1], avg.data_ptr(), _stream(x))
    _lib.check(rc, "niidmix::update_rows")


@torch.library.custom_op("niidmix::sgd_step_rows", mutates_args=("p",))
def sgd_step_rows(p: torch.Tensor, g: torch.Tensor, rows: torch.Tensor, neg_lr: float) -> None:
    """p[rows] = fma(neg_lr, g[rows], p[rows]) in place (torch.optim.SGD, momentum 0)."""
    _slab("p", p)
    _slab("g", g, rows=p.shape[0], cols=p.shape[1])
    _req(g.device == p.device, "p and g must be on the same device")
    _vec("rows", rows, torch.int32, p.device)
    rc = _lib.lib.niidmix_sgd_step_rows_f32(p.data_ptr(), _ld(p), g.data_ptr(), _ld(g), p.shape[1],
                                            rows.data_ptr(), rows.numel(), float(neg_lr), _stream(p))
    _lib.check(rc, "niidmix::sgd_step_rows")


# ------------------------------------------------------------------------------------------------
# Mixer attributes built on first use (plan group -> attributes it sets)
_LAZY = {
    "plan": "clique", "plan_reason": "clique", "p_clique_ptr": "clique", "p_member_row": "clique",
    "p_member_group": "clique", "p_coef": "clique", "p_res_ptr": "clique", "p_res_col": "clique",
    "p_res_val": "clique", "p_res_member": "clique",
    "tile": "tile", "tile_reason": "tile", "t_sub_ptr": "tile", "t_sub_rows": "tile",
    "t_sub_wself": "tile", "t_pos_src": "tile", "t_pos_mask": "tile", "t_pos_w": "tile",
    "tlds": "tlds", "tlds_reason": "tlds", "l_sub_ptr": "tlds", "l_sub_rows": "tlds",
    "l_sub_slot": "tlds", "l_sub_wself": "tlds", "l_pos_slot": "tlds", "l_pos_mask": "tlds",
    "l_pos_w": "tlds", "l_grp_tile_ptr": "tlds", "l_grp_src_ptr": "tlds", "l_grp_src_rows": "tlds",
    "tseg": "tlds", "s_seg_ptr": "tlds", "s_seg": "tlds", "s_seg_w": "tlds",
    "tmf": "tlds", "m_mf_ptr": "tlds", "m_mf": "tlds", "l_rem_rows": "tlds", "tlds_rem2": "tlds",
    "w_dense": "dense", "w_split": "dense",
    "ell": "ell", "e_col": "ell", "e_val": "ell", "e_len": "ell", "band": "ell",
}


class _Scratch:
    """Attribute sink for a Mixer plan builder: reads fall through to the Mixer."""

    def __init__(self, owner):
        self._owner = owner

    def __getattr__(self, name):
        return getattr(self._owner, name)


class Mixer:
    """One topology's mixing operator on one device: Θ' = Wᵀ Θ for a [N, P] fp32 slab.

    kernel='auto' picks (fast mode):  clique-factored if W factors exactly over its cliques
    (factor.py; a fully-connected topology counts as one clique) without cancelling correction
    terms, else dense MFMA if W is a genuinely dense GEMM (nnz >= dense_threshold * N^2), else the
    LDS-staged tiles where the plan has cancelling corrections (removed clique edges), else the CSR
    gather.  mode='exact' uses the LDS-staged merged-order tiles where they build, else the global
    tiles, else the CSR gather; all follow the reference's operand order bit for bit.

    Plans are built on first use of the kernel that needs them (a random-graph round that only
    mixes in exact mode never builds the clique plan or a dense W).
    """

    def __init__(self, topology=None, *, csr=None, cliques=None, device="cuda",
                 dense_threshold=0.25, factor=True):
        if csr is None:
            csr = to_csr(topology)
        if cliques is None and topology is not None:
            cliques = topology.get("cliques")
        self.csr = csr
        self.n = csr.n
        self.cliques = cliques
        self.device = torch.device(device)
        self.factor = factor
        dev = self.device
        # the CSR is always on the device: the gather kernels read it and the factored / GEMM
        # kernels recompute non-finite outputs from it (include/niidmix.h)
        self.row_ptr = torch.from_numpy(csr.row_ptr).to(dev)
        self.col = torch.from_numpy(csr.col).to(dev)
        self.val = torch.from_numpy(csr.val).to(dev)
        self.dense_threshold = dense_threshold
        self.dense = (csr.n_in == csr.n and csr.nnz >= dense_threshold * self.n * self.n
                      and self.n >= 64)
        self._host = {}           # host-side plans, shared with the Mixers .to() makes
        self.use_segments = True  # RT-16 LDS tiles: segment loop where segments built
        # exact RT-16 LDS tiles: the matrix-core path (bit-identical, but 4.3 vs 3.2 ms on the
        # headline: DESIGN §3) only on request, NIIDMIX_TLDS_MFMA=1
        self.use_mfma = os.environ.get("NIIDMIX_TLDS_MFMA", "0") == "1"

    def to(self, device):
        """The same operator on another device, sharing the host-side plans (built once)."""
        m = Mixer(csr=self.csr, cliques=self.cliques, device=device,
                  dense_threshold=self.dense_threshold, factor=self.factor)
        m._host = self._host
        return m

    def _hosted(self, key, build):
        if key not in self._host:
            self._host[key] = build()
        return self._host[key]

    def __getattr__(self, name):
        group = _LAZY.get(name)
        if group is None:
            raise AttributeError(f"{type(self).__name__!s} has no attribute {name!r}")
        # build the group on a scratch object, then fill only what is not set yet: a caller (or a
        # test) that installed its own plan keeps it
        scratch = _Scratch(self)
        getattr(type(self), "_build_" + group)(scratch)
        for k, v in scratch.__dict__.items():
            if k != "_owner" and k not in self.__dict__:
                self.__dict__[k] = v
        return self.__dict__[name]

    def _build_clique(self):
        csr, dev = self.csr, self.device
        self.plan, self.plan_reason = (None, "factorisation disabled")
        fcl = self.cliques
        if not fcl and csr.n_in == csr.n and csr.nnz == csr.n * csr.n:
            fcl = [list(range(csr.n))]          # fully-connected: one clique (W = a I + c 11^T under MH)
        if self.factor:
            self.plan, self.plan_reason = self._hosted("clique", lambda: build_clique_plan(csr, fcl))
        if self.plan is None:
            return
        p = self.plan
        self.p_clique_ptr = torch.from_numpy(p.clique_ptr).to(dev)
        self.p_member_row = torch.from_numpy(p.member_row).to(dev)
        grp = p.member_group.copy()
        if os.environ.get("NIIDMIX_GATEWAY_HINT", "1") != "0" and len(p.res_col):
            # rows gathered as residual terms: loaded temporally by their own clique's item
            grp[np.isin(p.member_row, p.res_col)] |= MEMBER_GATEWAY
        self.p_member_group = torch.from_numpy(grp).to(dev)
        self.p_coef = torch.from_numpy(np.ascontiguousarray(p.coef)).to(dev)
        self.p_res_ptr = torch.from_numpy(p.res_ptr).to(dev)
        self.p_res_col = torch.from_numpy(p.res_col).to(dev)
        self.p_res_val = torch.from_numpy(p.res_val).to(dev)
        self.p_res_member = torch.from_numpy(p.res_member).to(dev)

    def _build_tile(self):
        # merged-order row tiles from global memory: only worth building when rows read many
        # sources (avg degree >= 8); NIIDMIX_TILE_RT=8|16|32 picks the tile height
        csr, dev = self.csr, self.device
        self.tile, self.tile_reason = (None, "average degree < 8")
        if csr.nnz >= 9 * max(csr.n, 1):
            rt = int(os.environ.get("NIIDMIX_TILE_RT", "8"))
            self.tile, self.tile_reason = self._hosted(
                ("tile", rt), lambda: build_tile_plan(csr, self.cliques, rt))
        if self.tile is None:
            return
        tp = self.tile
        self.t_sub_ptr = torch.from_numpy(tp.sub_ptr).to(dev)
        self.t_sub_rows = torch.from_numpy(tp.sub_rows).to(dev)
        self.t_sub_wself = torch.from_numpy(tp.sub_wself).to(dev)
        self.t_pos_src = torch.from_numpy(tp.pos_src).to(dev)
        self.t_pos_mask = torch.from_numpy(tp.pos_mask.view(np.int32)).to(dev)
        self.t_pos_w = torch.from_numpy(tp.pos_w).to(dev)

    def _build_tlds(self):
        # LDS-staged tiles (exact mode's default where they build: every group's distinct source
        # rows fit the LDS stage); NIIDMIX_TILE_LDS_RT=8|16|32 picks the tile height
        csr, dev = self.csr, self.device
        self.tlds, self.tlds_reason = (None, "average degree < 8")
        # NIIDMIX_TLDS_ANY_DEGREE=1 builds them for low-degree graphs too (ring / grid probes)
        if csr.nnz >= 9 * max(csr.n, 1) or os.environ.get("NIIDMIX_TLDS_ANY_DEGREE") == "1":
            rt = int(os.environ.get("NIIDMIX_TILE_LDS_RT", "16"))
            grp = self.cliques
            if not grp:
                span = rt * LDS_MAX_WAVES.get(rt, 1)
                grp = [list(range(s, min(s + span, csr.n))) for s in range(0, csr.n, span)]
            # rows per rt-16 tile: balanced_tile_rows (an even wave count per SIMD);
            # NIIDMIX_TILE_LDS_ROWS fixes it (tuning A/B)
            trows = os.environ.get("NIIDMIX_TILE_LDS_ROWS", "auto")
            trows = (self._hosted(("tlds_rows", rt), lambda: balanced_tile_rows(csr, grp, rt))
                     if trows == "auto" else int(trows))
            self.tlds, self.tlds_reason = self._hosted(
                ("tlds", rt, trows), lambda: build_tile_lds_plan(csr, grp, rt, tile_rows=trows))
            # register rows for sources outside a group that only masked entries read (a gateway
            # row's inter-clique neighbour): the stage shrinks to the group's own rows (10 000
            # d-cliques nodes: 199 staged rows -> 100, 128-column items instead of 96; 1000 nodes:
            # 111 -> 101, 128 instead of 120).  At most 8 per tile when the rows past the 8th,
            # staged, still leave three 128-column blocks per CU (80 VGPRs; 16 register rows take
            # 96: two blocks).  Same-box A/B, 1000 nodes: 2.92 (8) / 3.03 (16) vs 3.11 ms all
            # staged (profiles/r04/exact_register_rows_ab.txt).  NIIDMIX_TLDS_REMOTE=0 turns it
            # off; 8 / 16 fix the cap
            rem = os.environ.get("NIIDMIX_TLDS_REMOTE", "auto")
            lp0 = self.tlds
            if lp0 is not None and rt == 16 and rem != "0":
                lr, _ = self._hosted(("tlds_rem", rt, trows),
                                     lambda: build_tile_lds_plan(csr, grp, rt, remote_regs=True,
                                                                 tile_rows=trows))
                if lr is not None and lr.rem_rows is not None and lr.rem_regs == 16 and rem != "16" \
                        and (rem == "8" or self._rem8_fits(lr)):
                    l8, _ = self._hosted(("tlds_rem8", rt, trows), lambda: build_tile_lds_plan(
                        csr, grp, rt, remote_regs=True, rem_cap=8, tile_rows=trows))
                    if l8 is not None and l8.rem_rows is not None:
                        lr = l8
                if lr is not None and lr.rem_rows is not None:
                    self.tlds = lr
        if self.tlds is None:
            return
        lp = self.tlds
        # segment loop (RT 16): runs of consecutive LDS slots read at immediate offsets
        # (niidmix.tile.build_tile_segments); NIIDMIX_TLDS_SEG=0 keeps the per-position loop
        ts = tm = None
        if lp.tile.rt == 16 and os.environ.get("NIIDMIX_TLDS_SEG", "1") != "0":
            ts = self._hosted(("tseg", lp.tile.rt), lambda: build_tile_segments(lp))
            # position lists of the matrix-core exact path (used when Mixer.use_mfma)
            if ts is not None:
                tm = self._hosted(("tmf", lp.tile.rt), lambda: build_tile_mfma_positions(lp))
        # unbound: `self` may be the lazy builder's scratch object, whose attribute lookups (bound
        # methods included) fall through to the Mixer
        Mixer.set_tile_lds_plan(self, lp, ts, tm)

    @staticmethod
    def _rem8_fits(lr):
        """Would a plan with at most 8 register rows per tile (the rest staged) still stage few
        enough rows for three 128-column blocks per CU?  Counted from the 16-row plan lr."""
        n_reg = (lr.rem_rows.reshape(-1, 16) >= 0).sum(1)
        extra = np.maximum(n_reg - 8, 0)
        gtp = lr.grp_tile_ptr
        src = np.diff(lr.grp_src_ptr)
        most = max(int(src[g]) + int(extra[gtp[g]:gtp[g + 1]].sum()) for g in range(len(src)))
        return (most + 2) * 512 + 1024 <= (160 * 1024) // 3

    def set_tile_lds_plan(self, lp, ts=None, tm=None):
        """Upload an LDS tile plan (niidmix.tile.build_tile_lds_plan), its segments (or None: the
        per-position loop) and its MFMA position lists (or None: the segment walker) to this
        Mixer's device."""
        dev = self.device
        tp = lp.tile
        self.tlds = lp
        self.l_sub_ptr = torch.from_numpy(tp.sub_ptr).to(dev)
        self.l_sub_rows = torch.from_numpy(tp.sub_rows).to(dev)
        self.l_sub_slot = torch.from_numpy(lp.sub_slot).to(dev)
        self.l_sub_wself = torch.from_numpy(tp.sub_wself).to(dev)
        self.l_pos_slot = torch.from_numpy(lp.pos_slot).to(dev)
        self.l_pos_mask = torch.from_numpy(tp.pos_mask.view(np.int32)).to(dev)
        self.l_pos_w = torch.from_numpy(tp.pos_w).to(dev)
        self.l_grp_tile_ptr = torch.from_numpy(lp.grp_tile_ptr).to(dev)
        self.l_grp_src_ptr = torch.from_numpy(lp.grp_src_ptr).to(dev)
        self.l_grp_src_rows = torch.from_numpy(lp.grp_src_rows).to(dev)
        self.tseg = ts
        if ts is not None:
            # flat 1-D device arrays: seg [S*4] int32 (16-B rows), seg_w [T*2] fp32
            self.s_seg_ptr = torch.from_numpy(ts.seg_ptr).to(dev)
            self.s_seg = torch.from_numpy(np.ascontiguousarray(ts.seg).reshape(-1)).to(dev)
            self.s_seg_w = torch.from_numpy(np.ascontiguousarray(ts.seg_w).reshape(-1)).to(dev)
        self.l_rem_rows = (torch.from_numpy(lp.rem_rows).to(dev) if lp.rem_rows is not None
                           else None)
        # 16 register rows walked in two phases of 8 (80 VGPRs: as many blocks per CU as the LDS
        # allows instead of two)
        self.tlds_rem2 = lp.rem_regs == 16 and ts is not None and rem_two_phase(lp, ts)
        self.tmf = tm if ts is not None else None
        if self.tmf is not None:
            self.m_mf_ptr = torch.from_numpy(tm.mf_ptr).to(dev)
            self.m_mf = torch.from_numpy(np.ascontiguousarray(tm.mf).reshape(-1)).to(dev)

    def _build_ell(self):
        lay = self._hosted("ell", lambda: ell_layout(self.csr))
        self.ell = None if lay is None else lay[0]
        # the band kernel where the rows are banded as stored (a ring relabeled by band_layout)
        self.band = None if lay is None else self._hosted("band", lambda: band_of(self.csr, lay[0]))
        if lay is not None:
            k, col, val, ln = lay
            self.e_col = torch.from_numpy(col).to(self.device)
            self.e_val = torch.from_numpy(val).to(self.device)
            self.e_len = torch.from_numpy(ln).to(self.device)

    def _build_dense(self):
        self.w_dense = torch.from_numpy(self.csr.dense()).to(self.device)
        # W^T split into bf16 planes once per topology (the bf16x6 GEMM, kernel "dense"), when
        # the split fits the GEMM's 32-bit offsets (else the fp32 GEMM serves the graph)
        self.w_split = dense_split_w(self.w_dense) \
            if self.w_dense.is_cuda and b6_fits(self.n) else None

    def device_layout(self):
        """(perm, block_cols): the device-resident layout the factored kernels stream best, measured
        on MI355X (tools/layout_probe.py):
          rows: clique-contiguous (node i at slab row perm[i], cliques in plan order) — a
                clique's member rows of a column block are then one contiguous stretch
                (1000-node d-cliques 1.345 vs 1.375 ms, 10 000 nodes 15.8 vs 16.3 ms);
          columns: blocks of 1024 (register tile), 64 for many cliques (>= 4096 member rows: the
                multi-clique tile's chunk of every row contiguous), 256 for > 64 gateway terms, or
                32 for big cliques
                (> 256 members, 32-column items: an item is then one contiguous 128 KB stretch;
                fully-connected 1000 nodes 1.43 vs 1.77 ms).
        perm is None when the rows are already clique-contiguous.  Without a clique plan, a ring is
        put in its cycle order (band_layout: k_mix_band reads it; ring 100 at P = 62 006)."""
        if self.plan is None:
            perm = band_layout(self.csr) if self.ell is not None and self.band is None else None
            return perm, memory_block_cols()
        order = self.plan.member_row.astype(np.int64)
        perm = np.empty(self.n, np.int64)
        perm[order] = np.arange(self.n)
        if np.array_equal(perm, np.arange(self.n)) or self.csr.n_in != self.n:
            perm = None
        if self.plan.max_clique > 256:
            bc = 32
        elif self.plan.max_clique <= 112 and len(self.plan.member_row) >= Q_ROWS_MIN:
            # many cliques (k_mix_clique_q's 64-column items, 10 000 nodes): 64-column blocks, so a
            # column chunk of every row is ONE contiguous N x 256 B stretch.  With 256-column
            # blocks its rows sat 1 KiB apart and mapped onto a quarter of the L2's sets: the
            # gateway gathers (one per member) missed the XCD's L2 (PMC reads 1.44 x algorithmic)
            bc = int(os.environ.get("NIIDMIX_Q_BLOCK_COLS", "64"))
        else:
            bc = 256 if self.plan.max_clique_res > 64 else memory_block_cols()
        return perm, bc

    def relabeled(self, perm):
        """The same operator over a slab whose row perm[i] holds node i (MixCSR.relabel): every
        output is computed with the same operands in the same order, so the results are bitwise
        those of this operator, stored at the permuted rows."""
        if perm is None:
            return self
        perm = np.asarray(perm, np.int64)
        cl = None if self.cliques is None else [[int(perm[r]) for r in c] for c in self.cliques]
        return Mixer(csr=self.csr.relabel(perm), cliques=cl, device=self.device,
                     dense_threshold=self.dense_threshold, factor=self.factor)

    @property
    def factored_safe(self):
        """A clique plan exists and has no cancelling corrections (factor.CliquePlan.n_cancel)."""
        return self.plan is not None and self.plan.n_cancel == 0

    def _clique_args(self):
        return (self.p_clique_ptr, self.p_member_row, self.p_member_group, self.p_coef,
                self.p_res_ptr, self.p_res_col, self.p_res_val, self.p_res_member, self.row_ptr,
                self.col, self.val)

    def mix_blocked(self, x, out, p, mode="fast", kernel=None):
        """One round on column-blocked slabs [K, rows, B] (niidmix.memory.empty_blocked): the
        clique-factored kernel (the device-resident fast path)."""
        _req(mode == "fast" and kernel in (None, "clique"),
             "blocked slabs: only the clique kernel (fast mode) reads the blocked layout")
        _req(self.plan is not None, f"no clique plan: {self.plan_reason}")
        _req(self.plan.max_clique <= 1024, "blocked slabs: cliques of <= 1024 members (register "
             "tile, or the one-pass big-clique kernel); a bigger clique uses the two-pass kernel "
             "on [N, P] slabs")
        mix_clique_blocked(x, *self._clique_args(), out, int(p), self.plan.max_clique,
                           self.plan.max_clique_res)
        return out

    def _strip_ok(self, x, out):
        """The column-strip kernel (few nodes, ELL rows) on slabs whose rows sit on a 256-B pitch:
        ring 100 at P = 62 006 11.0 us per round vs 14.8 for the band kernel on the same pitch; on
        ld = P (rows at 216-B offsets) the kernels are equal, 15.6-16 us (tools/band_probe.py).
        The kernel stages rows 0..n-1 only, so every ELL column must index one of them: a node
        shard whose rows read halo rows (csr.n_in > n) is never a strip round."""
        return (self.ell is not None and self.n <= STRIP_MAX_ROWS and x is not None and
                self.csr.n_in == self.n and x.dim() == 2 and x.shape[0] == self.n and
                x.stride(0) % 64 == 0 and
                (out is None or (out.dim() == 2 and out.stride(0) % 64 == 0)))

    def kernel_for(self, mode="fast", x=None, out=None):
        if mode == "exact":
            # measured on the 1000-node d-cliques round (P = 2^20): LDS-staged tiles 4.8 ms, global
            # tiles 7.2 ms, CSR gather 23.1 ms; tile plans exist only for graphs with average
            # degree >= 8 (ring / grid rows read 2-4 sources: CSR gather)
            if self.tlds is not None and (x is None or _lds_ok(x)) and (out is None or _lds_ok(out)):
                return "tile-lds-exact"
            if self.tile is not None:
                return "tile-exact"
            if self._strip_ok(x, out):
                return "strip-exact"
            if self.band is not None and (x is None or (x.shape[0] == self.n and _lds_ok(x))) \
                    and (out is None or _lds_ok(out)):
                return "band-exact"
            return "ell-exact" if self.ell is not None else "csr-exact"
        if self.factored_safe and (x is None or _clique_ok(x)) and (out is None or _clique_ok(out)):
            return "clique"
        if self.dense:
            return "dense" if b6_fits(self.n, x) else "dense-f32"
        if self.plan is not None and self.tlds is not None and (x is None or _lds_ok(x)) and \
                (out is None or _lds_ok(out)):
            return "tile-lds-fast"               # clique graph with removed edges
        if self._strip_ok(x, out):
            return "strip-fast"
        if self.band is not None and (x is None or (x.shape[0] == self.n and _lds_ok(x))) \
                and (out is None or _lds_ok(out)):
            return "band-fast"
        return "ell-fast" if self.ell is not None else "csr-fast"

    def __call__(self, x, out=None, mode="fast", kernel=None):
        if out is None:
            out = torch.empty((self.n, x.shape[1]), dtype=torch.float32, device=x.device)
        k = kernel or self.kernel_for(mode, x, out)
        hint = LOW_DEGREE if self.csr.nnz <= 4 * max(self.n, 1) else 0
        if k == "csr-exact":
            mix_csr(x, self.row_ptr, self.col, self.val, out, EXACT | hint)
        elif k == "csr-fast":
            mix_csr(x, self.row_ptr, self.col, self.val, out, FAST | hint)
        elif k in ("ell-exact", "ell-fast"):
            _req(self.ell is not None, "no ELL layout: a row has more than 8 entries")
            mix_ell(x, self.e_col, self.e_val, self.e_len, out, self.ell,
                    EXACT if k == "ell-exact" else FAST)
        elif k in ("strip-exact", "strip-fast"):
            _req(self.ell is not None, "no ELL layout: a row has more than 8 entries")
            _req(self.csr.n_in == self.n and x.shape[0] == self.n,
                 "strip kernel: rows read sources past the slab's own rows (halo rows of a node "
                 "shard); the strip stages only rows 0..n-1 (use ell-*)")
            mix_strip(x, self.e_col, self.e_val, self.e_len, out, self.ell,
                      EXACT if k == "strip-exact" else FAST)
        elif k in ("band-exact", "band-fast"):
            _req(self.band is not None, "no band layout: rows are not banded as stored "
                 "(Mixer.device_layout / band_layout gives a ring's cycle order)")
            mix_band(x, self.e_col, self.e_val, self.e_len, out, self.ell, self.band,
                     EXACT if k == "band-exact" else FAST)
        elif k in ("tile-exact", "tile-fast"):
            _req(self.tile is not None, f"no tile plan: {self.tile_reason}")
            mix_tile(x, self.t_sub_ptr, self.t_sub_rows, self.t_sub_wself, self.t_pos_src,
                     self.t_pos_mask, self.t_pos_w, out, self.tile.rt,
                     EXACT if k == "tile-exact" else FAST)
        elif k in ("tile-lds-exact", "tile-lds-fast"):
            _req(self.tlds is not None, f"no LDS tile plan: {self.tlds_reason}")
            lp = self.tlds
            ts = self.tseg
            segs = (self.s_seg_ptr, self.s_seg, self.s_seg_w) if \
                self.use_segments and ts is not None and ts.lp is lp else ()
            rem = None
            if lp.rem_rows is not None:
                _req(bool(segs), "a plan with register rows needs the segment walker "
                     "(use_segments; NIIDMIX_TLDS_REMOTE=0 builds a plan without them)")
                rem = self.l_rem_rows
            if segs and rem is None and k == "tile-lds-exact" and self.use_mfma and \
                    self.tmf is not None and self.tmf.lp is lp:
                segs = segs + (self.m_mf_ptr, self.m_mf)
            if rem is not None:
                # two phases of 8 register rows (80 VGPRs: three 8-wave blocks per CU instead of
                # two) where the plan allows it; 10 000 nodes 31.3 vs 32.4 ms
                # (profiles/r06/tile_rows/); NIIDMIX_TLDS_REM2=0: the 16-register kernel
                two = self.tlds_rem2 and os.environ.get("NIIDMIX_TLDS_REM2", "1") == "1"
                segs = segs + (None, None, rem, -16 if two else lp.rem_regs)
            mix_tile_lds(x, self.l_sub_ptr, self.l_sub_rows, self.l_sub_slot, self.l_sub_wself,
                         self.l_pos_slot, self.l_pos_mask, self.l_pos_w, self.l_grp_tile_ptr,
                         self.l_grp_src_ptr, self.l_grp_src_rows, out, lp.tile.rt, lp.max_src,
                         lp.max_tiles, EXACT if k == "tile-lds-exact" else FAST, *segs)
        elif k == "clique":
            _req(self.plan is not None, f"no clique plan: {self.plan_reason}")
            mix_clique(x, *self._clique_args(), out, self.plan.max_clique,
                       self.plan.max_clique_res)
        elif k == "dense":
            # bf16 matrix cores, fp32-accurate by three-term splits: 2.7x the fp32 MFMA's rate
            _req(b6_fits(self.n, x), "kernel 'dense' (bf16x6): 16 rows of the slab or the "
                 "split W exceed 2^31 B; use 'dense-f32'")
            mix_dense_b6(x, self.w_split, self.row_ptr, self.col, self.val, out)
        elif k == "dense-f32":
            mix_dense(x, self.w_dense, self.row_ptr, self.col, self.val, out)
        else:
            raise ValueError(f"unknown kernel {k!r}")
        return out


def b6_fits(n, x=None):
    """The bf16x6 GEMM's limits (niidmix_mix_dense_bf16x6_f32, niidmix.hip:4428): the split W
    (2 B x niidmix_dense_split_elems(n)) and 16 rows of x's leading dimension below 2^31 B.  Host
    arithmetic only (no GPU call)."""
    lim = 0x7fffffff
    if 2 * int(_lib.lib.niidmix_dense_split_elems(int(n))) >= lim:
        return False
    return x is None or 16 * _ld(x) * 4 < lim


# member rows from which the launcher picks the multi-clique tile (niidmix.hip kQRowsMin)
Q_ROWS_MIN = 4096


def memory_block_cols():
    from .memory import BLOCK_COLS
    return BLOCK_COLS


def _clique_ok(x):
    """k_mix_clique streams float4 columns: p and ld multiples of 4, 16-B aligned base."""
    return x.shape[1] % 4 == 0 and _ld(x) % 4 == 0 and x.data_ptr() % 16 == 0


def _lds_ok(x):
    """k_mix_tile_lds reads column pairs: even p and ld, 8-B aligned base."""
    return x.shape[1] % 2 == 0 and _ld(x) % 2 == 0 and x.data_ptr() % 8 == 0


def csr_from_numpy(row_ptr, col, val):
    return MixCSR(np.asarray(row_ptr, np.int64), np.asarray(col, np.int32),
                  np.asarray(val, np.float32)).validate()
