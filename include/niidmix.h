/*
 * niidmix.h — C-ABI of the MI355X (gfx950) neighbour parameter-mixing library (libniidmix.so).
 *
 * The reference hot path is D-SGD's per-round Jacobi mixing
 *     theta'_i = sum_{j in {i} u E(i)} W[j, i] * theta_j
 * implemented in Python/ATen by
 *     d_sgd.average           /root/reference/tools/simulate/algorithm/d_sgd.py:96-116
 *     setup.model.average     /root/reference/tools/setup/model/__init__.py:15-25
 *     d_sgd.update_models     /root/reference/tools/simulate/algorithm/d_sgd.py:29-35
 * over the topology produced by setup.topology.load
 *     /root/reference/tools/setup/topology/__init__.py:4-12 (edges {int: list}, weights fp32 [N,N]).
 *
 * The reference has no FFI of its own (it is pure Python); the binding a maintainer adds is a ctypes
 * stub.  Every entry point below:
 *   - takes plain device pointers and sizes (no torch types), caller-owned buffers;
 *   - is stream-ordered on the given hipStream_t (passed as void*; NULL = default stream), never
 *     synchronises the host, never allocates;
 *   - returns NIIDMIX_OK or an error code; niidmix_last_error() gives a thread-local message.
 * Slabs are row-major fp32 [rows, p] with leading dimension ld (elements).  One row = the flattened
 * parameters of one simulated node in model.parameters() order.
 * Jacobi semantics: every output row is computed from the pre-round input, so x and y must not
 * overlap.  Every entry point that reads one slab and writes another gets the row count and checks
 * the full extents of both (NIIDMIX_EALIAS), each slab with its own strides.
 *
 * ABI 5 (this header): niidmix_dense_split_elems / niidmix_dense_split_w /
 * niidmix_mix_dense_bf16x6_f32 added (the dense GEMM on the bf16 matrix cores, fp32-accurate by
 * three-term splitting); niidmix_mix_strip_f32 refuses a strip that does not fit the device's LDS.
 * ABI 4: niidmix_mix_band_f32 added (banded low-degree graphs, e.g. a ring in its
 * cycle order), niidmix_mix_strip_f32 (column strips for few nodes), register rows in the LDS
 * tile plan.
 * ABI 3: n_rows added to niidmix_mix_tile_f32, niidmix_mix_tile_lds_f32,
 * niidmix_grad_segment_mean_f32 and niidmix_grad_segment_mean_blocked_f32 (full extent checks);
 * niidmix_update_rows_f32 added (the 'sample' topology's broadcast); niidmix_mix_ell_f32 added
 * (low-degree graphs); niidmix_sharded_* / niidmix_mix_sharded_f32 added (sharded round over
 * several GPUs of one process, RCCL); cliques of <= 112 members
 * accept 64-column blocks (the multi-clique tile).
 */
#ifndef NIIDMIX_H
#define NIIDMIX_H

#include <stdint.h>
#include <sys/types.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NIIDMIX_ABI_VERSION 5

enum niidmix_status {
    NIIDMIX_OK = 0,
    NIIDMIX_EINVAL = 1,       /* bad size / pointer / mode argument */
    NIIDMIX_EALIAS = 2,       /* input and output slabs overlap (Jacobi semantics violated) */
    NIIDMIX_EHIP = 3,         /* a HIP runtime call failed (launch error) */
    NIIDMIX_EUNSUPPORTED = 4  /* the plan exceeds what the kernel supports (e.g. clique too large) */
};

enum niidmix_mode {
    /* Bit-exact with the reference loop: for each row, z = x_self*0, acc = z, then in CSR order
     * acc = fl(acc + fl(w*x_j)) (no FMA), finally y = fl(z + acc).  This is setup.model.average's
     * deepcopy/mul_(0)/add_(w*p) (model/__init__.py:19-24) followed by update_models'
     * p.mul_(0.); p.add_(new) (d_sgd.py:31-34). */
    NIIDMIX_MODE_EXACT = 0,
    /* Same terms, fused multiply-add, any association: within the north-star's 1e-5 relative
     * (condition-aware) tolerance, not bitwise. */
    NIIDMIX_MODE_FAST = 1
};

/* OR-ed into `mode`: write the averaged model itself (setup.model.average's return value,
 * model/__init__.py:25) instead of the update_models epilogue fl(x_self*0 + avg).  The two differ
 * only in the sign of an exactly-zero result. */
#define NIIDMIX_FLAG_AVERAGE_ONLY 2

/* OR-ed into `mode` of niidmix_mix_csr_f32: performance hint, the graph's average row length
 * (in-degree + 1) is <= 4 (ring, grid): fewer speculative gathers per batch.  Results unchanged. */
#define NIIDMIX_FLAG_LOW_DEGREE 4

/* OR-ed into `mode` of niidmix_mix_csr_f32: gradient mean instead of parameter mixing.  Row r's
 * entries list the nodes whose gradients it averages (val must be 1.0f), in the reference's order:
 *   acc = +0; acc = fl(acc + g_j) for each entry;  y_r = fl(+0 + fl(acc / row length))
 * = average_gradients (d_sgd.py:19-27: zeros_like, add_, div_(len(models))) followed by
 * update_gradients (d_sgd.py:37-45: grad.zero_(); grad.add_(g)).  Used by --clique-gradient (the
 * clique's members, clique order; with removed clique edges only the members adjacent to the node,
 * d_sgd.py:56-78) and --unbiased-gradient (topology['neighbourhoods'][rank] order, d_sgd.py:79-90).
 * Identical results in EXACT and FAST mode (w = 1: fma(1, g, acc) == fl(acc + g)).  Exclusive with
 * NIIDMIX_FLAG_AVERAGE_ONLY. */
#define NIIDMIX_FLAG_MEAN 8

/* ABI version (NIIDMIX_ABI_VERSION). */
int niidmix_abi_version(void);

/* Thread-local description of the last error returned on this thread ("" if none). */
const char *niidmix_last_error(void);

/* Sparse mixing over a CSR of W^T rows, in the reference's accumulation order.
 * Replaces d_sgd.average (d_sgd.py:96-116) + setup.model.average (model/__init__.py:15-25)
 * + update_models (d_sgd.py:29-35) for all nodes of one round.
 *   x        [>= max(col)+1, ld_x] input slab (device)
 *   y        [n_rows, ld_y] output slab (device), must not overlap x
 *   row_ptr  [n_rows+1] int64 (device); row r's entries are [row_ptr[r], row_ptr[r+1])
 *   col      [nnz] int32 input-row indices (device); the FIRST entry of each row is the node itself
 *            (the reference's models[0] = self, d_sgd.py:105)
 *   val      [nnz] fp32 weights (device): val = W[src, rank] (d_sgd.py:106), self weight first
 *   mode     NIIDMIX_MODE_EXACT or NIIDMIX_MODE_FAST, optionally | NIIDMIX_FLAG_AVERAGE_ONLY
 *            | NIIDMIX_FLAG_LOW_DEGREE | NIIDMIX_FLAG_MEAN
 * Rows with no entries are written as +0. */
int niidmix_mix_csr_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                        int64_t p, const int64_t *row_ptr, const int32_t *col, const float *val,
                        int mode, void *stream);

/* The same round over an ELL layout of the same W^T rows, for low-degree graphs (ring, grid,
 * random regular): row r's entries are ell_col / ell_val[r*k .. r*k + ell_len[r]) in the CSR's
 * order (self first), padded to k entries (the padding is never read as a term).  k: 3, 5 or 8.
 *   x  [>= max(n_rows, max(col)+1), ld_x]: row r's own data (its first entry, normally r itself) is
 *      loaded before its descriptors arrive, so x must hold at least n_rows rows
 * The descriptors are scalar loads (one row per wave) and a wave streams several column chunks of
 * its row.  mode as niidmix_mix_csr_f32 (EXACT / FAST, | NIIDMIX_FLAG_AVERAGE_ONLY); bit-identical
 * to it in EXACT mode. */
int niidmix_mix_ell_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                        int64_t p, int k, const int32_t *ell_col, const float *ell_val,
                        const int32_t *ell_len, int mode, void *stream);

/* The same round for BANDED rows: every entry of row r reads row r + d (mod n_rows) with
 * |d| <= band (a ring in its cycle order: band 1; niidmix.ops.band_layout finds that order and
 * MixCSR.relabel puts the slab in it).  The descriptors are the ELL arrays of niidmix_mix_ell_f32
 * (absolute columns, self first, padded to k); the caller guarantees the band (the kernel folds
 * (col - r) mod n_rows into [-band, band]; an entry outside the band reads a wrong row).  A wave
 * loads its output rows and the band rows around them before any descriptor arrives, so a round is
 * one memory round trip per wave and each row is loaded about once instead of k times.
 * (k, band): (3, 1) or (5, 2); n_rows >= 2 band + 1; p and both ld even, 8-B aligned slabs
 * (NIIDMIX_EUNSUPPORTED otherwise: use niidmix_mix_ell_f32).  x and y: [n_rows, ld].  mode as
 * niidmix_mix_ell_f32; bit-identical to it (and to niidmix_mix_csr_f32) in EXACT mode. */
int niidmix_mix_band_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                         int64_t p, int k, int band, const int32_t *ell_col, const float *ell_val,
                         const int32_t *ell_len, int mode, void *stream);

/* The same round (d_sgd.average, tools/simulate/algorithm/d_sgd.py:96-116) for FEW nodes
 * (n_rows <= 256; ring 100, BASELINE configs[1], tools/setup/topology/ring.py:12-27) by column
 * strips: a block of 8 waves owns a strip of every row -- 256 columns (float4 lanes) when x and y
 * are 16-B aligned, both ld are multiples of 4, ld_x >= p rounded up to 4 and n_rows <= 156, else
 * 64 columns -- stages it in LDS by LDS-DMA and combines each output row from there in its ELL
 * order, so each element of x is read from memory once.  Any row order.  Descriptors: the ELL arrays of
 * niidmix_mix_ell_f32 (k = 3, 5 or 8).  Contract: every ell_col entry is < n_rows -- only rows
 * 0..n_rows-1 are staged, so x must hold exactly the rows the outputs read (a node shard whose
 * rows read halo rows past its own is NOT a strip round: use niidmix_mix_ell_f32); the descriptors
 * are device arrays and are not checked here (niidmix.ops.Mixer checks them once per topology).
 * NIIDMIX_EUNSUPPORTED when the strip does not fit the device's per-block LDS.
 * x 4-B aligned; x and y: [n_rows, ld].  mode as
 * niidmix_mix_ell_f32; bit-identical to it (and to niidmix_mix_csr_f32) in EXACT mode.  Round 4
 * (ABI 4). */
int niidmix_mix_strip_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                          int64_t p, int k, const int32_t *ell_col, const float *ell_val,
                          const int32_t *ell_len, int mode, void *stream);

/* Clique-factored mixing (fast mode only).  For each member m of clique c:
 *   y_m = a_m * x_m + sum_{g < n_groups} c_{m,g} * S_{c,g} + sum_r res_val[r] * x[res_col[r]]
 * with S_{c,g} = sum of x over the members of clique c in group g.  The host derives the plan from
 * the loaded W (topology.json 'cliques', d_cliques/random_cliques.py:18-37 + weights.py:15-25) and
 * verifies that it reproduces every W entry; see DESIGN.md.  All arrays are device pointers.
 *   clique_ptr   [n_cliques+1] int32 offsets into the member arrays
 *   member_row   [n_members] int32 row index (input row == output row)
 *   member_group [n_members] int32 group id in [0, n_groups), optionally OR-ed with
 *                NIIDMIX_MEMBER_GATEWAY when the member's row is also some residual entry's source
 *                (res_col): a load-policy hint only (that row is loaded temporally so the gather
 *                hits L2), never changes results
 *   coef         [n_members * (1 + n_groups)] fp32: a_m, then c_{m,0..n_groups-1}
 *   res_ptr      [n_members+1] int32 offsets into res_col/res_val (residual sparse terms)
 *   res_col      [n_res] int32 input rows, res_val [n_res] fp32
 *   res_member   [n_res] int32 index, within its clique, of the member each residual entry belongs
 *                to (the register tile fetches a clique's residual entries lane-parallel together
 *                with the member descriptors, so the gateway-row gathers issue right behind the
 *                member-row loads)
 *   max_clique   largest clique size: <= 256 selects a register tile (one HBM read per
 *                parameter); 257..1024 (e.g. fully-connected = one clique) the one-pass
 *                big-clique kernel (a 32-column item of every member held in registers, one HBM
 *                read per parameter); larger cliques a two-pass kernel (rows read twice)
 *   max_clique_res  largest number of residual terms of one clique (informational, >= 0)
 *   n_groups     1..4
 *   csr_ptr / csr_col / csr_val   the CSR of the same W^T (niidmix_mix_csr_f32's row_ptr / col /
 *                val, rows indexed like member_row): the non-finite guard.  The factored form
 *                combines every member into every output, the reference only a node's real edges
 *                (d_sgd.py:105-106) on top of self*0 (model/__init__.py:20-21); every output the
 *                kernel finds non-finite is recomputed from its CSR row (fast-mode arithmetic), so
 *                inf / NaN propagate exactly along real edges and a non-finite self gives NaN.
 * Range checks: x and y must not overlap over the member rows (NIIDMIX_EALIAS). */
#define NIIDMIX_MEMBER_GATEWAY 256

typedef struct niidmix_clique_plan {
    int32_t n_cliques;
    int32_t n_members;
    int32_t n_groups;
    int32_t max_clique;
    int32_t max_clique_res;
    const int32_t *clique_ptr;
    const int32_t *member_row;
    const int32_t *member_group;
    const float *coef;
    const int32_t *res_ptr;
    const int32_t *res_col;
    const float *res_val;
    const int32_t *res_member;
    const int64_t *csr_ptr;
    const int32_t *csr_col;
    const float *csr_val;
} niidmix_clique_plan;

int niidmix_mix_clique_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t p,
                           const niidmix_clique_plan *plan, void *stream);

/* The same clique-factored round on COLUMN-BLOCKED slabs: x and y are [K][rows][block_cols]
 * (K = ceil(p / block_cols) blocks of row-major [rows, block_cols] sub-slabs with row stride `ld`
 * floats and block strides block_stride_x / block_stride_y floats), element (r, c) at
 *   base + (c / block_cols) * block_stride + r * ld + c % block_cols.
 * block_cols: a power of two >= 256 (the register tile's 256-column chunks), >= 64 when
 * max_clique <= 112 (the multi-clique tile's 64-column items, which also serves every plan with
 * >= 4096 member rows: Q = 4 cliques per item keep a column chunk's rows in an XCD's L2), >= 32
 * when max_clique > 256 (the big-clique kernel's 32-column items).  This is the layout niidmix keeps
 * device-resident node state in (Mixer.device_layout: block_cols = 1024 for cliques of <= 256
 * members, 256 when a clique has > 64 gateway terms, 32 for big cliques; clique-contiguous rows),
 * which measured robust to the slab's physical placement.  Cliques of <= 256 members use
 * the register tile, 257..1024 members the one-pass big-clique kernel (32-column items). */
int niidmix_mix_clique_blocked_f32(const float *x, float *y, int64_t p, int64_t ld,
                                   int64_t block_cols, int64_t block_stride_x,
                                   int64_t block_stride_y, const niidmix_clique_plan *plan,
                                   void *stream);

/* Merged-order row tiles, exact or fast: the same result as niidmix_mix_csr_f32 (bit for bit in
 * NIIDMIX_MODE_EXACT: every row keeps its own operand order — self, then edges[rank] in list order,
 * d_sgd.py:105-106 — and its own roundings), computed so that rows sharing sources share the loads.
 * Output rows are cut into tiles of rt rows (e.g. parts of a clique).  Each tile has one merged list
 * of positions such that every row's entry list (self excluded) is a subsequence of it; a position
 * names a source row, the tile rows that take it (mask) and their weights.  Built on the host by
 * niidmix.tile.build_tile_plan.
 *   n_sub      tiles;  rt  rows per tile: 8, 16 or 32
 *   sub_ptr    [n_sub+1] int64 offsets into the position arrays
 *   sub_rows   [n_sub*rt] int32 output rows, -1 for an unused slot
 *   sub_wself  [n_sub*rt] fp32 W[r, r] of each tile row (its first CSR entry)
 *   pos_src    [L] int32 source row of every position, | NIIDMIX_TILE_POS_UNIFORM when every
 *              slot of the position's pos_w holds the same fp32 value (exact mode then forms the
 *              product fl(w*x) once per position and adds it to each taking row: same bits)
 *   pos_mask   [L] uint32: bit r set when tile row r takes the position (unused slots: set)
 *   pos_w      [L*rt] fp32 weight W[src, row] per tile row (0 where the row skips the position)
 *   (pos_* must be valid device pointers even when L == 0; they are read only inside sub_ptr ranges)
 * mode: NIIDMIX_MODE_EXACT / _FAST, optionally | NIIDMIX_FLAG_AVERAGE_ONLY. */
#define NIIDMIX_TILE_POS_UNIFORM (1 << 30)
typedef struct niidmix_tile_plan {
    int64_t n_sub;
    int32_t rt;
    int32_t reserved;
    const int64_t *sub_ptr;
    const int32_t *sub_rows;
    const float *sub_wself;
    const int32_t *pos_src;
    const uint32_t *pos_mask;
    const float *pos_w;
} niidmix_tile_plan;

int niidmix_mix_tile_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                         int64_t p, const niidmix_tile_plan *plan, int mode, void *stream);

/* LDS-staged merged-order row tiles (exact-mode default for clique topologies): the same tiles and
 * results as niidmix_mix_tile_f32 (bit for bit in NIIDMIX_MODE_EXACT), grouped: a group (a clique)
 * owns consecutive tiles and a list of the DISTINCT source rows its tiles read.  One workgroup per
 * (group, 128-column chunk) stages those rows' columns in LDS (one HBM read per row), then each
 * wave applies one tile's positions from LDS.  Built by niidmix.tile.build_tile_lds_plan.
 *   rt, n_sub, sub_ptr, sub_rows, sub_wself, pos_mask, pos_w   as niidmix_tile_plan
 *   pos_slot     [L] int32 index of the position's source in its group's grp_src_rows list
 *                (| NIIDMIX_TILE_POS_UNIFORM as for niidmix_tile_plan.pos_src)
 *   sub_slot     [n_sub*rt] int32 index of each tile row's own row in the group list (0 for unused)
 *   n_grp        groups;  grp_tile_ptr [n_grp+1] int32 tile ranges;  max_tiles = most tiles in a
 *                group: 1..16 for rt 8, 1..12 for rt 16, 1..4 for rt 32 (64*max_tiles threads)
 *   grp_src_ptr  [n_grp+1] int32;  grp_src_rows  int32 source rows;  max_src = largest list (<= 256:
 *                max_src * 512 B of LDS)
 * Needs even p and ld and 8-B aligned slabs (2 columns per lane).  mode as niidmix_mix_tile_f32. */
typedef struct niidmix_tile_lds_plan {
    int64_t n_sub;
    int32_t rt, n_grp, max_src, max_tiles;
    const int64_t *sub_ptr;
    const int32_t *sub_rows;
    const int32_t *sub_slot;
    const float *sub_wself;
    const int32_t *pos_slot;
    const uint32_t *pos_mask;
    const float *pos_w;
    const int32_t *grp_tile_ptr;
    const int32_t *grp_src_ptr;
    const int32_t *grp_src_rows;
    /* optional (rt 16; NULL = the per-position loop): the positions cut into segments, runs read
     * from consecutive LDS slots with immediate offsets (niidmix.tile.build_tile_segments):
     *   seg_ptr [n_sub+1] int32 segments of each tile;  seg [n_seg * 4] int32 per segment:
     *   a run: first slot | length << 12 | first skipped tile row << 20, weight-select bits, skip
     *   bits, 0;  a masked position: slot | 1 << 30, the tile rows that take it, its weight (fp32
     *   bits), 0;  seg_w [n_sub * 2] fp32 the tile's two weights */
    const int32_t *seg_ptr;
    const int32_t *seg;
    const float *seg_w;
    /* optional (rt 16 with segments, EXACT mode; NULL = the segment walker): the positions as
     * matrix-core lists (niidmix.tile.build_tile_mfma_positions), applied by v_mfma_f32_16x16x4_f32
     * 4 positions at a time, bit-identical; a block whose staged rows hold a non-finite value or
     * one below 1e-30 in magnitude takes the segment walker instead:
     *   mf_ptr [n_sub+1] int32 entries of each tile (multiples of 4);  mf [n_mf * 4] int32 per
     *   entry: slot, weight (fp32 bits), tile rows that take it, 0 */
    const int32_t *mf_ptr;
    const int32_t *mf;
    /* optional (rt 16 with segments, mf_ptr NULL; NULL = every source staged in LDS): REGISTER
     * rows, sources outside a group that only masked entries read (a gateway row's inter-clique
     * neighbour), kept per tile in registers instead of the LDS stage
     * (niidmix.tile.build_tile_lds_plan(remote_regs=True)):  rem_rows [n_sub * 16] int32 global
     * rows of each tile's register rows (-1 unused); a masked segment whose word 0 has bit 29 set
     * reads register row (word 0 & 0xfff).  Round 4 (ABI 4). */
    const int32_t *rem_rows;
    /* register rows the kernel loads per tile: 8 (every tile's rem_rows entries 8..15 are -1; 16
     * fewer VGPRs, so three 7-wave blocks fit a CU) or 16; 0 = 16; -16: all 16 in two phases of 8
     * in the 8-row kernel's registers, 8..15 loaded when the walk reaches the first segment that
     * reads one -- only for plans whose tiles read rows 0..7 before any of 8..15
     * (niidmix.tile.rem_two_phase) */
    int32_t rem_regs;
} niidmix_tile_lds_plan;

int niidmix_mix_tile_lds_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                             int64_t p, const niidmix_tile_lds_plan *plan, int mode, void *stream);

/* Dense mixing Y = W^T X on the fp32 matrix cores (v_mfma_f32_32x32x2_f32), for topologies dense
 * enough that W x Theta is a genuine GEMM (fully-connected, tools/setup/topology/fully-connected.py).
 *   w  [n, n] fp32 row-major, w[src*n + dst] = W[src, dst] — the reference's topology['weights']
 *      layout (topology/__init__.py:9) — device pointer
 *   x  [n, ld_x], y [n, ld_y]
 *   row_ptr / col / val   the CSR of the same W^T (as niidmix_mix_csr_f32): the non-finite guard
 *      (see niidmix_clique_plan.csr_ptr) — an output the GEMM finds non-finite (W = 0 off the edges
 *      gives 0*inf = NaN) is recomputed from its node's real edges. */
int niidmix_mix_dense_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n,
                          int64_t p, const float *w, const int64_t *row_ptr, const int32_t *col,
                          const float *val, void *stream);

/* The same GEMM on the BF16 matrix cores with fp32 accuracy (round 5, ABI 5): each fp32 operand is
 * split into three bf16 terms (a = a_h + a_m + a_l, residue < 2^-24 |a|) and the six partial
 * products reaching 2^-16 |a b| are accumulated in fp32 by v_mfma_f32_32x32x16_bf16 -- on gfx950 the
 * fp32-input MFMA runs at 1/16 of the bf16 rate, so six bf16 products cost 6/16 of one fp32 one.
 * The error is of the order of one fp32 rounding per product (fast mode's 1e-5 condition-aware
 * tolerance, like the fp32 kernel); non-finite outputs are recomputed from the CSR as above.
 *   wp  the split W^T from niidmix_dense_split_w (device, 16-B aligned,
 *       niidmix_dense_split_elems(n) uint16 elements); made once per topology.
 * Other arguments as niidmix_mix_dense_f32. */
int64_t niidmix_dense_split_elems(int64_t n);
int niidmix_dense_split_w(const float *w, int64_t n, uint16_t *wp, void *stream);
int niidmix_mix_dense_bf16x6_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n,
                                 int64_t p, const uint16_t *wp, const int64_t *row_ptr,
                                 const int32_t *col, const float *val, void *stream);

/* Column mean over rows (the uniform global average of setup.model.average(models) with
 * weights=None, model/__init__.py:17-18, used by d_sgd.init :137-141 and the logger :112,260),
 * with the per-row squared L2 distance to that mean (logger.model_distance, logger.py:42-48).
 *   mean  [p] fp32 output;  dist2 [n] fp64 output (may be NULL)
 *   mode EXACT reproduces the reference's left-to-right fl(acc + fl(w*x_k)) with w = fp32(1/n). */
int niidmix_mean_rows_f32(const float *x, int64_t ld_x, int64_t n, int64_t p, float *mean,
                          double *dist2, int mode, void *stream);

/* Segment gradient mean for --clique-gradient without removed clique edges (d_sgd.py:56-65):
 * segment s lists the member rows seg_row[seg_ptr[s] .. seg_ptr[s+1]) in clique order, and EVERY
 * member row of y receives the same mean of the members' rows of g:
 *   acc = +0; acc = fl(acc + g_m) in member order; y_m = fl(+0 + fl(acc / len))
 * = average_gradients (d_sgd.py:19-27) + update_gradients (d_sgd.py:37-45), bit for bit.  One read
 * of every member row and one write (HBM-bound), instead of len gathers per output row.
 *   g  [n_rows, ld_g] gradient slab (device), y [n_rows, ld_y] output (device, must not overlap g)
 *   seg_ptr [n_seg+1], seg_row [seg_ptr[n_seg]] int32 (device).  Rows in no segment are untouched. */
int niidmix_grad_segment_mean_f32(const float *g, int64_t ld_g, float *y, int64_t ld_y,
                                  int64_t n_rows, int64_t p, int64_t n_seg, const int32_t *seg_ptr,
                                  const int32_t *seg_row, void *stream);

/* niidmix_grad_segment_mean_f32 on column-blocked slabs [K][rows][block_cols] (see
 * niidmix_mix_clique_blocked_f32; block_cols a power of two >= 1024, p % 4 == 0). */
int niidmix_grad_segment_mean_blocked_f32(const float *g, float *y, int64_t n_rows, int64_t p,
                                          int64_t ld, int64_t block_cols, int64_t block_stride_g,
                                          int64_t block_stride_y, int64_t n_seg,
                                          const int32_t *seg_ptr, const int32_t *seg_row,
                                          void *stream);

/* SGD step on the listed rows: p[row] = fma(neg_lr, g[row], p[row]) — torch.optim.SGD with
 * momentum 0 and no weight decay (param.add_(grad, alpha=-lr); ATen's CPU kernel fuses it into one
 * fma with an fp32 alpha), the optimizer step the reference runs after gradient averaging
 * (d_sgd.py:63-64, :77-78, :88-90).  The fused drop-in round (niidmix.d_sgd) runs gradient mean ->
 * this step -> mixing on each device window, so the step never visits the host.
 *   p [*, ld_p] parameters (device, updated in place), g [*, ld_g] gradients (device)
 *   rows [n_rows] int32 rows to step (device) */
int niidmix_sgd_step_rows_f32(float *p, int64_t ld_p, const float *g, int64_t ld_g, int64_t ncols,
                              const int32_t *rows, int64_t n_rows, float neg_lr, void *stream);

/* update_models(all_models, avg) after the 'sample' topology's uniform average (d_sgd.py:240-250,
 * :29-35): every row y_i := fl(fl(x_i * 0) + avg) (p.mul_(0.); p.add_(new)) — avg everywhere
 * except NaN where x_i is non-finite and the sign rule of (+-0) + (+-0) where avg is 0.
 *   x [n_rows, ld_x], y [n_rows, ld_y] (device; y == x with ld_y == ld_x: in place, any other
 *   overlap is refused);  avg [p] (device, overlapping neither) */
int niidmix_update_rows_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                            int64_t p, const float *avg, void *stream);

/* Sharded round over several GPUs of ONE process (the simulator's own model: every node in one
 * process, run.py:136), nodes sharded by whole cliques (niidmix.shard.ShardPlan), the rows other
 * shards read exchanged every round, then each shard's rows mixed by niidmix_mix_csr_f32 over
 * [local rows | halo rows] (the local CSR keeps every row's operand order: exact mode is bitwise
 * the single-GPU round).  The handle holds one RCCL communicator per shard (ncclCommInitAll,
 * created once per topology and device set; librccl.so.1 is loaded on first use).  When several
 * shards share a device (tests, one-GPU boxes) the exchange is device-to-device copies instead.
 * Shard s, row-major slabs with ld = p:
 *   x [rows_in, p]: its n_local rows, then its halo rows;  y [n_local, p]
 *   row_ptr / col / val: CSR of its n_local rows over the rows_in input rows (device)
 *   peer[j], j < n_peers (host): the shards it exchanges with; it sends
 *     send_rows[send_ptr[j] .. send_ptr[j+1]) (device local row indices, in that peer's halo order;
 *     send_ptr host, send_ptr[0] may be > 0) through send_buf (device, [send_ptr[n_peers] -
 *     send_ptr[0], p]) and receives recv_count[j] rows into halo rows recv_row[j] .. (host)
 *   stream: the shard's HIP stream (on its device)
 * Every shard's receive count must equal what the peer sends it (checked); the call enqueues
 * pack -> exchange -> mix on every shard's stream and returns without waiting. */
typedef struct niidmix_sharded niidmix_sharded;
typedef struct niidmix_shard {
    int32_t device;
    int32_t n_peers;
    int64_t n_local, rows_in;
    float *x;
    float *y;
    const int64_t *row_ptr;
    const int32_t *col;
    const float *val;
    const int32_t *peer;
    const int64_t *send_ptr;
    const int32_t *send_rows;
    float *send_buf;
    const int64_t *recv_row;
    const int64_t *recv_count;
    void *stream;
} niidmix_shard;

int niidmix_sharded_create(int n_shards, const int *devices, niidmix_sharded **out);
int niidmix_sharded_destroy(niidmix_sharded *h);
/* 1 when the handle exchanges by device-to-device copies (shards sharing a device), 0 for RCCL. */
int niidmix_sharded_is_loopback(const niidmix_sharded *h);
int niidmix_mix_sharded_f32(niidmix_sharded *h, const niidmix_shard *shards, int64_t p, int mode);

/* Device memory for node-state slabs, with the signatures of a PyTorch pluggable allocator
 * (torch.cuda.memory.CUDAPluggableAllocator; niidmix.memory.slab_pool uses them for a MemPool).
 * The range is reserved with hipMemAddressReserve and mapped from 2 MiB physical chunks
 * (hipMemCreate / hipMemMap): the clique kernel's access pattern measured 1.32 ms per headline round
 * on every such slab, against 1.35-1.64 ms on hipMalloc'ed slabs depending on their physical
 * placement.  Returns NULL on failure (niidmix_last_error says why); free with
 * niidmix_hbm_free (size, device and stream are ignored). */
void *niidmix_hbm_alloc(ssize_t size, int device, void *stream);
void niidmix_hbm_free(void *ptr, ssize_t size, int device, void *stream);

/* Strided host <-> device copy (hipMemcpy2DAsync) of `rows` rows of `width_bytes` each, used by
 * the host-resident drop-in (niidmix.slab) to stream column windows of the pinned [N, P] host slab
 * through HBM while the previous window is being mixed.  kind: 0 = host->device, 1 = device->host,
 * 2 = device->device.  Stream-ordered; host memory must be pinned for the copy to be asynchronous. */
int niidmix_copy2d_async(void *dst, int64_t dpitch_bytes, const void *src, int64_t spitch_bytes,
                         int64_t width_bytes, int64_t rows, int kind, void *stream);

/* Streaming copy y[0:n] = x[0:n] (fp32, n % 4 == 0, 16-B aligned, no overlap) with non-temporal
 * loads and stores, one float4 per thread in linear order.  Not part of the reference's path: a
 * measurement primitive that gives bench.py this GPU's own HBM copy ceiling to report the mixing
 * kernel against (MI355X boxes differ by up to ~20 % in achievable HBM bandwidth). */
int niidmix_stream_copy_f32(const float *x, float *y, int64_t n, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* NIIDMIX_H */
