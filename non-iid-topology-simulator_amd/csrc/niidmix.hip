// niidmix.hip — gfx950 (MI355X, CDNA4) kernels for D-SGD neighbour parameter mixing and the C-ABI
// declared in include/niidmix.h.
//
// Reference hot path (what these kernels replace, one launch per round for ALL nodes):
//   d_sgd.average        /root/reference/tools/simulate/algorithm/d_sgd.py:96-116
//   setup.model.average  /root/reference/tools/setup/model/__init__.py:15-25
//   update_models        /root/reference/tools/simulate/algorithm/d_sgd.py:29-35
//
// Data layout: the N simulated nodes' flattened models are one row-major fp32 slab [N, ld] in HBM
// (row = node, flattened in model.parameters() order).  Mixing is out-of-place (x -> y ping-pong)
// because the reference computes every average from pre-round parameters before overwriting any
// model (Jacobi).
//
// This translation unit is compiled with -ffp-contract=off: every a*b+c below is two roundings
// unless written as __builtin_fmaf.  The exact kernel relies on that for bit-exactness with the
// reference's separate ATen mul and add_ (model/__init__.py:24: c1.add_(w*p1)).
//
// Kernels:
//   k_mix_csr<EXACT,VW>    generic CSR gather, one wave per (output row, 256-column chunk);
//                          XCD-aware work order so the rows one chunk needs stay in that XCD's L2.
//   k_mix_clique<RPW,G>    clique-factored: one 512-thread workgroup per (clique, 256-column chunk)
//                          reads each member row ONCE from HBM into registers, forms the per-group
//                          clique sums with a cross-wave LDS reduction, writes each output once.
//                          HBM-bound: 2*4 bytes per node-parameter.
//   k_mix_dense            Y = W^T X on v_mfma_f32_32x32x2_f32 (fp32 matrix cores), 128x128 tiles.
//   k_mean_cols / k_row_dist2   uniform average + squared distance to it (consensus distance).
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <dlfcn.h>
#include <stdarg.h>
#include <stdlib.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/types.h>

#include <mutex>
#include <unordered_map>
#include <type_traits>
#include <vector>

#include "../../include/niidmix.h"

typedef float floatx16 __attribute__((ext_vector_type(16)));

namespace {

thread_local char g_last_error[512] = "";

int set_error(int code, const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
    return code;
}

int check_launch(const char *what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(NIIDMIX_EHIP, "%s: %s", what, hipGetErrorString(e));
    g_last_error[0] = '\0';
    return NIIDMIX_OK;
}

constexpr int kWave = 64;
constexpr int64_t kChunk = 256;  // fp32 columns per (row, chunk) work item: 64 lanes x float4
constexpr int64_t kMaxGrid = 8 * 16384;  // grid-stride cap, multiple of 8 (keeps t % 8 fixed)

__device__ __forceinline__ int wave_id() {
    return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
}

__device__ __forceinline__ float4 ld4(const float *p) { return *reinterpret_cast<const float4 *>(p); }

__device__ __forceinline__ float4 ld4_nt(const float *p) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4 *>(p));
    return make_float4(v[0], v[1], v[2], v[3]);
}

// ----------------------------------------------------------------------------------------------
// Exact / fast per-element update rules.
//   exact: acc = fl(acc + fl(w*x))      (ATen CPU add_(w*p): separate roundings, no FMA)
//   fast : acc = fma(w, x, acc)
template <bool EXACT>
__device__ __forceinline__ float axpy(float w, float xv, float acc) {
    if constexpr (EXACT) {
        const float t = w * xv;  // rounded (fp-contract=off)
        return acc + t;
    } else {
        return __builtin_fmaf(w, xv, acc);
    }
}

template <bool EXACT>
__device__ __forceinline__ float4 axpy4(float w, float4 xv, float4 acc) {
    return make_float4(axpy<EXACT>(w, xv.x, acc.x), axpy<EXACT>(w, xv.y, acc.y),
                       axpy<EXACT>(w, xv.z, acc.z), axpy<EXACT>(w, xv.w, acc.w));
}

// ----------------------------------------------------------------------------------------------
// Non-finite guard of the factored and GEMM kernels (fast mode).  The reference sums only over a
// node's real edges ([self] + edges[rank], d_sgd.py:105-106) on top of self*0 (model/__init__.py:
// 20-21): a non-finite value reaches an output only along a real edge, and a non-finite SELF value
// makes the output NaN.  The factored form a*x_i + sum_g c_g*S_g + residuals (and a GEMM with W = 0
// off the edges) combines every clique member / every node into every output, so a non-finite x_j
// would leak into outputs that never read it (c*inf - c*inf = NaN for a removed clique edge, 0*inf
// = NaN in the GEMM).  Conversely a factored output is finite only if every value it combined is
// finite.  Hence every output the fast kernel finds non-finite is recomputed from the node's CSR
// row in the reference's operand order with fast-mode arithmetic (z = x_self*0, acc = fma(w, x_j,
// acc), y = z + acc: k_mix_csr's fast mode), which reproduces the reference's inf / NaN pattern.
// The check costs one v_cmp_class per output element.  What is recomputed: k_mix_clique recomputes
// every column of a row's chunk once any lane of it is non-finite (its finite neighbours then take
// the CSR form's bits, still within the tolerance); the multi-clique, big-clique and GEMM kernels
// recompute only the non-finite elements, each by an O(degree) CSR walk.  A round whose models
// have diverged to inf / NaN is therefore much slower than a finite one (every element recomputed
// serially); finite rounds never enter this path.
//   one row per call, V columns per lane: csr_refix;  one column: csr_refix1.
template <int V>
__device__ __forceinline__ void csr_refix(const float *__restrict__ xc, int64_t ld_x, unsigned lo, bool act,
                                       int64_t row, const int64_t *__restrict__ rp,
                                       const int32_t *__restrict__ col, const float *__restrict__ val,
                                       float *__restrict__ o) {
    const int64_t b = rp[row], e = rp[row + 1];
    float z[V], acc[V];
#pragma unroll
    for (int c = 0; c < V; ++c) { z[c] = 0.f; acc[c] = 0.f; }
    for (int64_t k = b; k < e; ++k) {
        const float *src = xc + (int64_t)col[k] * ld_x + lo;
        float xv[V];
#pragma unroll
        for (int c = 0; c < V; ++c) xv[c] = act ? src[c] : 0.f;
        if (k == b) {
#pragma unroll
            for (int c = 0; c < V; ++c) { z[c] = xv[c] * 0.f; acc[c] = z[c]; }
        }
        const float w = val[k];
#pragma unroll
        for (int c = 0; c < V; ++c) acc[c] = __builtin_fmaf(w, xv[c], acc[c]);
    }
#pragma unroll
    for (int c = 0; c < V; ++c) o[c] = z[c] + acc[c];
}

__device__ __forceinline__ float csr_refix1(const float *__restrict__ xc, int64_t ld_x, int64_t row,
                                         const int64_t *__restrict__ rp,
                                         const int32_t *__restrict__ col,
                                         const float *__restrict__ val) {
    const int64_t b = rp[row], e = rp[row + 1];
    if (b == e) return 0.f;
    const float z = xc[(int64_t)col[b] * ld_x] * 0.f;
    float acc = z;
    for (int64_t k = b; k < e; ++k) acc = __builtin_fmaf(val[k], xc[(int64_t)col[k] * ld_x], acc);
    return z + acc;
}

// ----------------------------------------------------------------------------------------------
// Generic CSR mixing.  Work item = (group of 4 output rows, chunk of 256 columns); each wave owns
// one output row.  Work order is XCD-aware: items t and t+8 share an XCD (round-robin dispatch),
// and consecutive items on one XCD sweep all rows of the SAME chunk, so the chunk's source rows
// (rows x 1 KiB) are reused from that XCD's L2 by every output row that gathers them.
// VW-wide loads/stores (VW = 4: float4, 2: float2, 1: float): a lane owns 4 columns of the chunk as
// 4/VW slots, slot q covering columns c0 + VW*lane + 64*VW*q + [0, VW) (each wave-instruction reads
// 64*VW contiguous floats).  VW is the widest width the slab's p, ld and alignment allow.
template <int VW> __device__ __forceinline__ void ldv(const float *p, float *o);
template <> __device__ __forceinline__ void ldv<4>(const float *p, float *o) {
    const float4 v = *reinterpret_cast<const float4 *>(p); o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <> __device__ __forceinline__ void ldv<2>(const float *p, float *o) {
    const float2 v = *reinterpret_cast<const float2 *>(p); o[0] = v.x; o[1] = v.y;
}
template <> __device__ __forceinline__ void ldv<1>(const float *p, float *o) { o[0] = *p; }
template <int VW> __device__ __forceinline__ void stv_nt(float *p, const float *o) {
#pragma unroll
    for (int e = 0; e < VW; ++e) __builtin_nontemporal_store(o[e], p + e);
}

template <bool EXACT, int VW, int SPL, int U>
__global__ __launch_bounds__(256) void k_mix_csr(const float *__restrict__ x, int64_t ld_x,
                                                 float *__restrict__ y, int64_t ld_y,
                                                 int64_t n_rows, int64_t p,
                                                 const int64_t *__restrict__ row_ptr,
                                                 const int32_t *__restrict__ col,
                                                 const float *__restrict__ val,
                                                 int64_t n_row_groups, int64_t n_items,
                                                 int flags) {
    // flags: NIIDMIX_FLAG_AVERAGE_ONLY (write acc), NIIDMIX_FLAG_MEAN (gradient mean: acc starts at
    // +0 instead of x_self*0, result fl(+0 + fl(acc / row length)))
    const bool avg_only = (flags & NIIDMIX_FLAG_AVERAGE_ONLY) != 0;
    const bool mean = (flags & NIIDMIX_FLAG_MEAN) != 0;
    constexpr int S = 4 * SPL / VW;           // slots per lane
    constexpr int NE = 4 * SPL;               // columns per lane
    constexpr int64_t CH = kChunk * SPL;      // columns per (row, chunk) work item
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int64_t chunk = (local / n_row_groups) * 8 + xcd;
        const int64_t row = (local % n_row_groups) * 4 + wave;
        const int64_t c0 = chunk * CH;
        if (row >= n_rows || c0 >= p) continue;  // wave-uniform
        const int64_t beg = row_ptr[row];
        const int64_t end = row_ptr[row + 1];
        // Column of each slot; slots past p read column c0 instead (loads stay unconditional — a
        // branch around a load makes hipcc drain vmcnt per load) and are never stored.
        int64_t cs[S];
        bool ok[S];
#pragma unroll
        for (int q = 0; q < S; ++q) {
            const int64_t cq = c0 + VW * lane + 64 * VW * q;
            ok[q] = cq < p;                   // p % VW == 0: a slot is all-in or all-out
            cs[q] = ok[q] ? cq : c0;
        }
        float z[NE], acc[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) { z[e] = 0.f; acc[e] = 0.f; }
        for (int64_t kb = beg; kb < end; kb += 64) {
            // 64 entries' (source row, weight) fetched lane-parallel, handed out by v_readlane:
            // no scalar-load round trip per gather
            const int cnt = (int)(end - kb < 64 ? end - kb : 64);
            const int li = lane < cnt ? lane : cnt - 1;          // clamped: loads unconditional
            const int d_col = col[kb + li];
            const float d_val = val[kb + li];
            for (int j = 0; j < cnt; j += U) {
                float xv[U][NE];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int jj = j + u < cnt ? j + u : cnt - 1;     // clamp: valid row
                    const float *src = x + (int64_t)__builtin_amdgcn_readlane(d_col, jj) * ld_x;
#pragma unroll
                    for (int q = 0; q < S; ++q) ldv<VW>(src + cs[q], xv[u] + q * VW);
                }
                if (kb == beg && j == 0 && !mean) {
                    // self * 0 (the first entry is the node itself): keeps -0.0, inf/NaN -> NaN
#pragma unroll
                    for (int e = 0; e < NE; ++e) { z[e] = xv[0][e] * 0.f; acc[e] = z[e]; }
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (j + u < cnt) {
                        const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d_val), j + u));
#pragma unroll
                        for (int e = 0; e < NE; ++e) acc[e] = axpy<EXACT>(w, xv[u][e], acc[e]);
                    }
            }
        }
        // update_models: p.mul_(0.); p.add_(new)  ->  z + acc   (AVERAGE_ONLY: acc)
        // MEAN: average_gradients' g.div_(len) then update_gradients' zero_(); add_(g) (d_sgd.py:19-45)
        float o[NE];
        if (mean) {
            const float len = (float)(end > beg ? end - beg : 1);   // empty row: +0 / 1
#pragma unroll
            for (int e = 0; e < NE; ++e) o[e] = 0.f + acc[e] / len;
        } else {
#pragma unroll
            for (int e = 0; e < NE; ++e) o[e] = avg_only ? acc[e] : z[e] + acc[e];
        }
        float *dst = y + row * ld_y;
#pragma unroll
        for (int q = 0; q < S; ++q)
            if (ok[q]) stv_nt<VW>(dst + cs[q], o + q * VW);
    }
}

// ----------------------------------------------------------------------------------------------
// Low-degree mixing over an ELL descriptor layout (ring, grid: every row lists <= K entries).  The
// CSR kernel's item is a chain row_ptr -> (col, val) -> gathers -> store per 256..512 columns; on a
// LeNet-size ring (100 rows x 62 006 columns, 3 entries) that chain, not the bytes, set the time.
// Here row r's entries sit at r*K + j (ell_col / ell_val, ell_len[r] of them, self first), so the
// gathers depend on ONE descriptor load, and a wave walks CH consecutive 256-column chunks of
// its row with all their gathers in flight together (descriptors amortised over CH chunks).
// Arithmetic as k_mix_csr (exact: fl(acc + fl(w*x)) in list order on top of x_self*0; fast: fma).
// Work order is XCD-aware: the rows of one column slice run on one XCD, so a source row gathered by
// its ~K readers is read from HBM once.
template <bool EXACT, int VW, int K, int CH>
__global__ __launch_bounds__(256) void k_mix_ell(const float *__restrict__ x, int64_t ld_x,
                                                 float *__restrict__ y, int64_t ld_y, int64_t n_rows,
                                                 int64_t p, const int32_t *__restrict__ ell_col,
                                                 const float *__restrict__ ell_val,
                                                 const int32_t *__restrict__ ell_len,
                                                 int64_t n_row_groups, int64_t n_items, int avg_only) {
    constexpr int S = 4 / VW;                 // slots per lane per chunk
    constexpr int NE = 4;                     // columns per lane per chunk
    constexpr int64_t CW = 64 * NE;           // columns per chunk (256)
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t t = blockIdx.x;
    if (t >= n_items) return;
    const int64_t xcd = t & 7, local = t >> 3;
    const int64_t slice = (local / n_row_groups) * 8 + xcd;
    const int64_t row = (local % n_row_groups) * 4 + wave;
    const int64_t c_beg = slice * CH * CW;
    if (row >= n_rows || c_beg >= p) return;  // wave-uniform
    float xv[CH][K][NE];
    int64_t cs[CH][S];
    bool ok[CH][S];
#pragma unroll
    for (int c = 0; c < CH; ++c)
#pragma unroll
        for (int q = 0; q < S; ++q) {
            const int64_t cq = c_beg + c * CW + VW * lane + 64 * VW * q;
            ok[c][q] = cq < p;                // p % VW == 0: a slot is all-in or all-out
            cs[c][q] = ok[c][q] ? cq : 0;
        }
    // the row's own data first (self is its list's first entry, d_sgd.py:105): its loads need no
    // descriptor, so they are in flight while the descriptors arrive
    {
        const float *src = x + row * ld_x;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int q = 0; q < S; ++q) ldv<VW>(src + cs[c][q], xv[c][0] + q * VW);
    }
    // descriptors by scalar loads (the row is wave-uniform): (col, val) of entry j
    const int64_t e0 = row * K;
    const int len = ell_len[row];
    int colj[K];
    float valj[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        colj[j] = ell_col[e0 + j];
        valj[j] = ell_val[e0 + j];
    }
    if (colj[0] != (int)row) {                // wave-uniform; not the plugin's layout: reload
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int q = 0; q < S; ++q) ldv<VW>(x + (int64_t)colj[0] * ld_x + cs[c][q], xv[c][0] + q * VW);
    }
    // gathers of every chunk of the slice, all in flight before the first use
#pragma unroll
    for (int j = 1; j < K; ++j) {
        const float *src = x + (int64_t)colj[j < len ? j : 0] * ld_x;
#pragma unroll
        for (int c = 0; c < CH; ++c)
#pragma unroll
            for (int q = 0; q < S; ++q) ldv<VW>(src + cs[c][q], xv[c][j] + q * VW);
    }
    float *dst = y + row * ld_y;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        float z[NE], acc[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) { z[e] = xv[c][0][e] * 0.f; acc[e] = z[e]; }   // self * 0
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (j < len) {                                                            // wave-uniform
                const float w = valj[j];
#pragma unroll
                for (int e = 0; e < NE; ++e) acc[e] = axpy<EXACT>(w, xv[c][j][e], acc[e]);
            }
        float o[NE];
#pragma unroll
        for (int e = 0; e < NE; ++e) o[e] = avg_only ? acc[e] : z[e] + acc[e];
#pragma unroll
        for (int q = 0; q < S; ++q)
            if (ok[c][q]) stv_nt<VW>(dst + cs[c][q], o + q * VW);
    }
}

// ----------------------------------------------------------------------------------------------
// Column strips for few nodes (n_rows <= 256; ring 100, BASELINE configs[1]): a block of SW waves
// owns 64 columns of EVERY row.  The strip lands in LDS (LDS-DMA, 4 B per lane per row; wave w
// stages rows w, w + SW, ...; every load in flight at once, no descriptor in front of any of them),
// then wave w combines the same rows' outputs from LDS in their ELL order and stores them.  Each
// element of x is read from memory exactly once (the ELL / band kernels read a row up to K times
// through L2).  The descriptors of a wave's rows are loaded lane-parallel with the strip (lane i:
// row w + SW i) and handed out by v_readlane: no scalar-load round trip per row.  Same arithmetic,
// in the same order, as k_mix_ell (z from the row's first entry, self).
#ifndef NIIDMIX_STRIP_AUX
#define NIIDMIX_STRIP_AUX 2   // cache policy of the strip's LDS-DMA loads: nt (each element is read
                              // once): ring 100 9.8-9.9 vs 10.7-10.8 us with 0 (tuning builds: -D)
#endif
template <bool EXACT, int K, int SW, int SV>
__global__ __launch_bounds__(64 * SW) void k_mix_strip(const float *__restrict__ x, int64_t ld_x,
                                                       float *__restrict__ y, int64_t ld_y,
                                                       int n_rows, int64_t p,
                                                       const int32_t *__restrict__ ell_col,
                                                       const float *__restrict__ ell_val,
                                                       const int32_t *__restrict__ ell_len,
                                                       int avg_only) {
    // SV columns per lane: 1 (any slab), or 4 (rows on a 16-B pitch with room for a lane's whole
    // float4 past p, niidmix_mix_strip_f32): 256-column strips, one 1 KiB LDS-DMA per row
    typedef float fv __attribute__((ext_vector_type(SV)));
    extern __shared__ float strip[];          // [n_rows][64 * SV]
    typedef __attribute__((address_space(3))) void lds_void;
    typedef __attribute__((address_space(1))) void glb_void;
    constexpr int RW = kWave * SV;            // floats per staged row
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = wave_id();
    const int64_t c0 = (int64_t)blockIdx.x * RW;
    const int64_t col = c0 + SV * lane;
    const bool any = col < p;                 // this lane stores some columns
    const float *xs = x + (any ? col : c0);   // lanes past p read valid columns, store nothing
    for (int r = wave; r < n_rows; r += SW) {
        if constexpr (SV == 4)
            __builtin_amdgcn_global_load_lds((glb_void *)(xs + (int64_t)r * ld_x),
                                             (lds_void *)(strip + r * RW), 16, 0, NIIDMIX_STRIP_AUX);
        else
            __builtin_amdgcn_global_load_lds((glb_void *)(xs + (int64_t)r * ld_x),
                                             (lds_void *)(strip + r * RW), 4, 0, NIIDMIX_STRIP_AUX);
    }
    const int mr = wave + SW * lane;          // the row this lane describes (n_rows <= 64 SW)
    const bool in = mr < n_rows;
    const int dlen = in ? ell_len[mr] : 0;
    int dcol[K];
    float dval[K];
#pragma unroll
    for (int j = 0; j < K; ++j) {
        dcol[j] = in ? ell_col[(int64_t)mr * K + j] : 0;
        dval[j] = in ? ell_val[(int64_t)mr * K + j] : 0.f;
    }
    __syncthreads();                          // the whole strip has landed (vmcnt(0) + barrier)
    float *dst = y + col;
    const int nw = (n_rows - wave + SW - 1) / SW;                  // rows of this wave
#pragma unroll 4
    for (int i = 0; i < nw; ++i) {
        const int r = wave + SW * i;
        const int len = __builtin_amdgcn_readlane(dlen, i);
        fv xv[K];
#pragma unroll
        for (int j = 0; j < K; ++j)
            xv[j] = *reinterpret_cast<const fv *>(
                strip + __builtin_amdgcn_readlane(dcol[j < len ? j : 0], i) * RW + SV * lane);
        fv z, acc;
#pragma unroll
        for (int e = 0; e < SV; ++e) { z[e] = xv[0][e] * 0.f; acc[e] = z[e]; }   // self * 0
#pragma unroll
        for (int j = 0; j < K; ++j)
            if (j < len) {                                                 // wave-uniform
                const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(dval[j]), i));
#pragma unroll
                for (int e = 0; e < SV; ++e) acc[e] = axpy<EXACT>(w, xv[j][e], acc[e]);
            }
        fv o;
#pragma unroll
        for (int e = 0; e < SV; ++e) o[e] = avg_only ? acc[e] : z[e] + acc[e];
        float *d = dst + (int64_t)r * ld_y;
        if (col + SV <= p) {
            __builtin_nontemporal_store(o, reinterpret_cast<fv *>(d));
        } else if (any) {
#pragma unroll
            for (int e = 0; e < SV; ++e)
                if (col + e < p) __builtin_nontemporal_store(o[e], d + e);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// Banded low-degree graphs (a ring in its cycle order: every entry of row r is a row r + d, |d| <=
// B, taken cyclically).  The ELL kernel above is a chain per wave — descriptor load, then the
// gathers it names, then the store — and reads every row K times.  Here a wave owns R consecutive
// output rows of CH column chunks and loads the R + 2B rows they can read straight away: the
// addresses need no descriptor, so the row loads and the scalar descriptor loads are in flight
// together (one memory round trip per wave), every row is loaded (R + 2B) / R times instead of K,
// and the operands come out of registers.  The descriptors are the ELL arrays of the same rows
// (absolute columns; the kernel takes d = (col - r) mod n folded into [-B, B], which the host
// checked for every entry).  Arithmetic and operand order as k_mix_ell (exact: bit-identical).
// Work order is XCD-aware: the row groups of one column slice run on one XCD, so the 2B rows a
// wave shares with its neighbours come from that XCD's L2.
template <bool EXACT, int VW, int K, int B, int R, int CH>
__global__ __launch_bounds__(256) void k_mix_band(const float *__restrict__ x, int64_t ld_x,
                                                  float *__restrict__ y, int64_t ld_y, int64_t n_rows,
                                                  int64_t p, const int32_t *__restrict__ ell_col,
                                                  const float *__restrict__ ell_val,
                                                  const int32_t *__restrict__ ell_len,
                                                  int64_t n_row_groups, int64_t n_items, int avg_only) {
    constexpr int NR = R + 2 * B;             // rows loaded per wave
    constexpr int64_t CW = 64 * VW;           // columns per chunk
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t t = blockIdx.x;
    if (t >= n_items) return;
    const int64_t xcd = t & 7, local = t >> 3;
    const int64_t slice = (local / n_row_groups) * 8 + xcd;
    const int64_t r0 = ((local % n_row_groups) * 4 + wave) * R;    // first output row of the wave
    const int64_t c_beg = slice * CH * CW;
    if (r0 >= n_rows || c_beg >= p) return;   // wave-uniform
    int64_t cs[CH];
    bool ok[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
        const int64_t cq = c_beg + c * CW + VW * lane;
        ok[c] = cq < p;                       // p % VW == 0: a slot is all-in or all-out
        cs[c] = ok[c] ? cq : 0;
    }
    // every row the wave can read, no descriptor needed: rows r0 - B .. r0 + R - 1 + B (cyclic)
    float xv[NR][CH][VW];
#pragma unroll
    for (int i = 0; i < NR; ++i) {
        int64_t ri = r0 - B + i;               // cyclic; n_rows may be < NR (no 64-bit modulo)
        while (ri < 0) ri += n_rows;
        while (ri >= n_rows) ri -= n_rows;
        const float *src = x + ri * ld_x;
#pragma unroll
        for (int c = 0; c < CH; ++c) ldv<VW>(src + cs[c], xv[i][c]);
    }
    // descriptors by scalar loads, in flight with the row loads
    int colj[R][K];
    float valj[R][K];
    int len[R];
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int64_t r = r0 + j < n_rows ? r0 + j : r0;
        len[j] = ell_len[r];
#pragma unroll
        for (int e = 0; e < K; ++e) {
            colj[j][e] = ell_col[r * K + e];
            valj[j][e] = ell_val[r * K + e];
        }
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const int64_t r = r0 + j;
        if (r >= n_rows) break;               // wave-uniform
        float *dst = y + r * ld_y;
        // d of every entry, folded into [-B, B] (the host checked the band)
        int dj[K];
#pragma unroll
        for (int e = 0; e < K; ++e) {
            int64_t d = (int64_t)colj[j][e] - r;
            d = d < 0 ? d + n_rows : d;        // [0, n)
            dj[e] = (int)(d > B ? d - n_rows : d);
        }
#pragma unroll
        for (int c = 0; c < CH; ++c) {
            float z[VW], acc[VW];
#pragma unroll
            for (int v = 0; v < VW; ++v) { z[v] = xv[j + B][c][v] * 0.f; acc[v] = z[v]; }   // self * 0
#pragma unroll
            for (int e = 0; e < K; ++e)
                if (e < len[j]) {                                                 // wave-uniform
                    float xe[VW];
#pragma unroll
                    for (int v = 0; v < VW; ++v) xe[v] = xv[j + B][c][v];
#pragma unroll
                    for (int d = -B; d <= B; ++d)
                        if (d != 0 && dj[e] == d) {                                // uniform select
#pragma unroll
                            for (int v = 0; v < VW; ++v) xe[v] = xv[j + B + d][c][v];
                        }
                    const float w = valj[j][e];
#pragma unroll
                    for (int v = 0; v < VW; ++v) acc[v] = axpy<EXACT>(w, xe[v], acc[v]);
                }
            float o[VW];
#pragma unroll
            for (int v = 0; v < VW; ++v) o[v] = avg_only ? acc[v] : z[v] + acc[v];
            if (ok[c]) stv_nt<VW>(dst + cs[c], o);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// Clique-factored mixing (fast mode).  Work item = (clique, 256-column chunk); WAVES waves; wave w
// holds members w, w+WAVES, w+2*WAVES, ... (RPW rows per wave, one float4 per lane per row) in
// registers.
//   0. lane r of each wave fetches the descriptor of the wave's r-th member (row, group,
//      coefficients, residual range) with ONE vector load per field; v_readlane hands them to the
//      scalar unit, so the RPW row loads issue back to back with no scalar-load round trips,
//   1. every member row is loaded once from HBM (all loads in flight before the first use),
//   2. per-wave partial group sums -> LDS; waves 0..G-1 each reduce one group -> LDS,
//   3. y_m = a_m x_m + sum_g c_{m,g} S_g + residual terms (gateway edges), stored once (nt).
// Work order is XCD-aware (the cliques of one chunk run back to back on one XCD) so the residual
// rows a gateway gathers from another clique are normally still in that XCD's L2.
// Work item t -> (chunk, clique).  XCD-aware: items t and t+8 share an XCD and consecutive items
// of one XCD sweep the cliques of one chunk.  skew (a multiple of 8 chunks, or 0) rotates each
// clique's chunk sequence by cq*skew, so the cliques in flight together read different column
// offsets (tuning: spreads the rows' concurrent addresses over more HBM channels).
__device__ __forceinline__ void clique_item(int64_t t, int32_t n_cliques, int64_t nc, int64_t skew,
                                            int64_t &chunk, int32_t &cq) {
    const int64_t local = t >> 3;
    const int64_t base = (local / n_cliques) * 8 + (t & 7);
    cq = (int32_t)(local % n_cliques);
    chunk = (skew && base < nc) ? (base + (int64_t)cq * skew) % nc : base;
}

constexpr int kMemberGroupMask = NIIDMIX_MEMBER_GATEWAY - 1;   // member_group: id | hint bits

template <int G, int RW>
struct CliqueDesc {        // one work item's descriptors, lane-parallel
    int32_t m0, M;         // wave-uniform: first member, members (0 past p)
    int32_t cr0, ncr;      // wave-uniform: the clique's residual entries [cr0, cr0 + ncr)
    int row, grp;          // lane r < RPW: the wave's r-th member (slot r)
    float cf[1 + G];
    int rsrc, rk;          // lane j < min(ncr, RW): the clique's j-th residual entry (source row,
    float rw;              //   member index within the clique, weight); rk = -1 past the list
};

// All descriptors of a work item in ONE dependent step after the clique offsets: the members'
// (row, group, coefficients) and the clique's residual entries (gateway edges), so the residual
// rows can be gathered right behind the member rows instead of one memory round trip later.
template <int WAVES, int RPW, int G, int RW, int64_t CW>
__device__ __forceinline__ void load_clique_desc(CliqueDesc<G, RW> &d, int64_t t, int32_t n_cliques,
                                                 int64_t p, int wave, int lane,
                                                 const int32_t *__restrict__ clique_ptr,
                                                 const int32_t *__restrict__ member_row,
                                                 const int32_t *__restrict__ member_group,
                                                 const float *__restrict__ coef,
                                                 const int32_t *__restrict__ res_ptr,
                                                 const int32_t *__restrict__ res_col,
                                                 const float *__restrict__ res_val,
                                                 const int32_t *__restrict__ res_member,
                                                 int64_t skew) {
    int64_t chunk;
    int32_t cq;
    clique_item(t, n_cliques, (p + CW - 1) / CW, skew, chunk, cq);
    const bool valid = chunk * CW < p;
    d.m0 = clique_ptr[cq];
    const int32_t m1 = clique_ptr[cq + 1];
    d.M = valid ? m1 - d.m0 : 0;
    d.cr0 = res_ptr[d.m0];
    d.ncr = valid ? res_ptr[m1] - d.cr0 : 0;
    const int kd = wave + WAVES * lane;
    d.row = 0; d.grp = 0;
#pragma unroll
    for (int g = 0; g <= G; ++g) d.cf[g] = 0.f;
    if (lane < RPW && kd < d.M) {
        const int32_t m = d.m0 + kd;
        d.row = member_row[m];
        d.grp = member_group[m];
#pragma unroll
        for (int g = 0; g <= G; ++g) d.cf[g] = coef[(int64_t)m * (1 + G) + g];
    }
    d.rsrc = 0; d.rk = -1; d.rw = 0.f;
    if (RW > 0 && lane < RW && lane < d.ncr) {
        d.rsrc = res_col[d.cr0 + lane];
        d.rk = res_member[d.cr0 + lane];
        d.rw = res_val[d.cr0 + lane];
    }
}

template <int V> __device__ __forceinline__ void ldv_nt(const float *p, float *o);
template <> __device__ __forceinline__ void ldv_nt<4>(const float *p, float *o) {
    const float4 v = ld4_nt(p); o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w;
}
template <> __device__ __forceinline__ void ldv_nt<2>(const float *p, float *o) {
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v v = __builtin_nontemporal_load(reinterpret_cast<const f2v *>(p)); o[0] = v[0]; o[1] = v[1];
}
template <> __device__ __forceinline__ void ldv_nt<1>(const float *p, float *o) {
    o[0] = __builtin_nontemporal_load(p);
}

template <int V> __device__ __forceinline__ bool finite_v(const float *v) {
    bool ok = true;
#pragma unroll
    for (int e = 0; e < V; ++e) ok &= __builtin_isfinite(v[e]);
    return ok;
}

// V = columns per lane per row: 4 (float4, 256-column chunks), 2 (float2, 128) or 1 (one float, 64
// columns).  Narrow chunks shrink a column chunk's working set (every clique's rows of that chunk)
// so that the gateway rows one clique gathers from the others stay in the XCD's 4 MB L2: the
// 10 000-node d-cliques round gathers ~1 gateway row per member.
template <int WAVES, int RPW, int G, int OCC, int RW, int FL, int V>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void k_mix_clique(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t p,
    int32_t n_cliques, const int32_t *__restrict__ clique_ptr,
    const int32_t *__restrict__ member_row, const int32_t *__restrict__ member_group,
    const float *__restrict__ coef, const int32_t *__restrict__ res_ptr,
    const int32_t *__restrict__ res_col, const float *__restrict__ res_val,
    const int32_t *__restrict__ res_member, int64_t n_items, int64_t skew, int cpb_shift,
    int64_t bs_x, int64_t bs_y, const int64_t *__restrict__ csr_ptr,
    const int32_t *__restrict__ csr_col, const float *__restrict__ csr_val) {
    // column-blocked slabs ([K][rows][B], B = CW << cpb_shift columns, block strides bs_x / bs_y
    // floats; a row-major slab is one block: cpb_shift = 62): chunk c lives in block c >> cpb_shift
    static_assert(RPW <= 64 && RW <= 64, "one descriptor lane per register row");
    static_assert(V == 1 || V == 2 || V == 4, "1, 2 or 4 columns per lane");
    static_assert(V == 4 || (FL & 16) == 0, "plain-store variant: float4 only");
    constexpr bool NTL = (FL & 2) != 0;       // non-temporal member-row loads (read-once stream)
    // timing-only ablations (WRONG results; instantiated only with -DNIIDMIX_ABLATIONS for
    // tools/tune_inproc.py): 4 = skip residual gathers, 8 = skip the cross-wave LDS reduction
    constexpr bool NO_RES = (FL & 4) != 0, NO_RED = (FL & 8) != 0;
    constexpr bool PLAIN_ST = (FL & 16) != 0;   // write-back (L2) stores instead of non-temporal
    constexpr int RQ = 2;                     // residual rows per wave held in registers
    // overflow residual gathers in flight per batch (N=8 stripes: 1.494 ms vs 1.506 ms one at a
    // time); G >= 3 tiles are at the register limit already
    constexpr int OVB = G <= 2 ? 3 : 1;
    constexpr int64_t CW = 64 * V;            // columns per work item
    __shared__ float red[G][WAVES][kWave * V];
    __shared__ float tot[G][kWave * V];
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    const int64_t t = blockIdx.x;             // one work item per block (grid = n_items)
    if (t >= n_items) return;
    CliqueDesc<G, RW> d;
    load_clique_desc<WAVES, RPW, G, RW, CW>(d, t, n_cliques, p, wave, lane, clique_ptr, member_row,
                                            member_group, coef, res_ptr, res_col, res_val,
                                            res_member, skew);
    int64_t chunk;
    int32_t cq_unused;
    clique_item(t, n_cliques, (p + CW - 1) / CW, skew, chunk, cq_unused);
    const bool act = chunk * CW + V * lane < p;
    const int32_t M = d.M;
    const int64_t kb = chunk >> cpb_shift, cin = chunk - (kb << cpb_shift);
    const float *xc = x + kb * bs_x + cin * CW;
    float *yc = y + kb * bs_y + cin * CW;
    const unsigned lo = (unsigned)(V * lane);

    // 1. member rows -> registers, all loads in flight before the first use
    float v[RPW][V];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
#pragma unroll
        for (int e = 0; e < V; ++e) v[r][e] = 0.f;
        if (wave + WAVES * r < M) {
            const int64_t row = __builtin_amdgcn_readlane(d.row, r);
            // a gateway row (NIIDMIX_MEMBER_GATEWAY) is gathered again as another clique's
            // residual term: a temporal load keeps it in L2 for that gather (wave-uniform branch)
            const bool gw = (__builtin_amdgcn_readlane(d.grp, r) & NIIDMIX_MEMBER_GATEWAY) != 0;
            if (act) {
                if (NTL && !gw) ldv_nt<V>(xc + row * ld_x + lo, v[r]);
                else ldv<V>(xc + row * ld_x + lo, v[r]);
            }
        }
    }
    // 1b. residual rows of this wave's members (clique entries whose member index k has
    //     k % WAVES == wave), issued right behind the member rows: up to RQ in registers, the
    //     rest (rare) gathered one by one in step 3.  Not non-temporal: a gateway row is another
    //     clique's member, read again by that clique's block (L2 hit).
    const int ncr = NO_RES ? 0 : d.ncr;
    const int nl = ncr < RW ? ncr : RW;
    uint64_t mine = __ballot(lane < nl && d.rk >= 0 && d.rk % WAVES == wave);
    float xr[RQ][V];
    int jq[RQ];
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
        jq[q] = mine ? __builtin_ctzll(mine) : -1;
        mine &= mine - 1;
        const int64_t row = __builtin_amdgcn_readlane(d.rsrc, jq[q] >= 0 ? jq[q] : 0);
#pragma unroll
        for (int e = 0; e < V; ++e) xr[q][e] = 0.f;
        if (act && jq[q] >= 0) ldv<V>(xc + row * ld_x + lo, xr[q]);
    }
    // 2. per-wave partial group sums -> LDS
    {
        float s[G][V];
#pragma unroll
        for (int g = 0; g < G; ++g)
#pragma unroll
            for (int e = 0; e < V; ++e) s[g][e] = 0.f;
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if (wave + WAVES * r < M) {
                const int gr = __builtin_amdgcn_readlane(d.grp, r) & kMemberGroupMask;
#pragma unroll
                for (int g = 0; g < G; ++g)
                    if (gr == g) {
#pragma unroll
                        for (int e = 0; e < V; ++e) s[g][e] += v[r][e];
                    }
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            if (V == 4) *reinterpret_cast<float4 *>(&red[g][wave][4 * lane]) = make_float4(s[g][0], s[g][V > 1 ? 1 : 0], s[g][V > 2 ? 2 : 0], s[g][V > 3 ? 3 : 0]);
            else if (V == 2) *reinterpret_cast<float2 *>(&red[g][wave][2 * lane]) = make_float2(s[g][0], s[g][V > 1 ? 1 : 0]);
            else red[g][wave][lane] = s[g][0];
        }
    }
    // 3. own term and residual terms (gateway edges) in place, BEFORE any store: v[r] := a_r x_r
    //    + sum_res w x_src.  On CDNA vmcnt counts stores too, so a gather issued after a store
    //    would make the gather's wait drain that store from HBM first.
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const float af = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d.cf[0]), r));
#pragma unroll
        for (int e = 0; e < V; ++e) v[r][e] *= af;
    }
#pragma unroll
    for (int q = 0; q < RQ; ++q) {
        if (jq[q] < 0) break;                                           // wave-uniform
        const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d.rw), jq[q]));
        const int slot = __builtin_amdgcn_readlane(d.rk, jq[q]) / WAVES;
#pragma unroll
        for (int r = 0; r < RPW; ++r)
            if (slot == r) {
#pragma unroll
                for (int e = 0; e < V; ++e) v[r][e] = __builtin_fmaf(w, xr[q][e], v[r][e]);
            }
    }
    // overflow: entries past the RQ held per wave (OVB gathers in flight per batch; the registers
    // of xr[] are free again here), then the clique's entries past the first RW, 64 descriptors at
    // a time fetched lane-parallel into the same descriptor registers and gathered in OVB batches
    // (a 10 000-node d-cliques clique has 99 gateway entries; N=8 column stripes 79)
    for (int32_t cb = d.cr0 + nl;;) {
        while (mine) {
            float xo[OVB][V];
            int jo[OVB];
#pragma unroll
            for (int b = 0; b < OVB; ++b) {
                jo[b] = mine ? __builtin_ctzll(mine) : -1;
                mine &= mine - 1;
                const int64_t row = __builtin_amdgcn_readlane(d.rsrc, jo[b] >= 0 ? jo[b] : 0);
#pragma unroll
                for (int e = 0; e < V; ++e) xo[b][e] = 0.f;
                if (act && jo[b] >= 0) ldv<V>(xc + row * ld_x + lo, xo[b]);
            }
#pragma unroll
            for (int b = 0; b < OVB; ++b) {
                if (jo[b] < 0) break;                                   // wave-uniform
                const float w = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d.rw), jo[b]));
                const int slot = __builtin_amdgcn_readlane(d.rk, jo[b]) / WAVES;
#pragma unroll
                for (int r = 0; r < RPW; ++r)
                    if (slot == r) {
#pragma unroll
                        for (int e = 0; e < V; ++e) v[r][e] = __builtin_fmaf(w, xo[b][e], v[r][e]);
                    }
            }
        }
        if (cb >= d.cr0 + ncr) break;                                   // wave-uniform
        const int32_t cnt = d.cr0 + ncr - cb < 64 ? d.cr0 + ncr - cb : 64;
        d.rsrc = 0; d.rk = -1; d.rw = 0.f;
        if (lane < cnt) {
            d.rsrc = res_col[cb + lane];
            d.rk = res_member[cb + lane];
            d.rw = res_val[cb + lane];
        }
        mine = __ballot(lane < cnt && d.rk % WAVES == wave);
        cb += 64;
    }
    // 4. group sums across waves through LDS (waves 0..G-1 each reduce one group)
    if (!NO_RED) __syncthreads();
    if (!NO_RED && wave < G) {
        float a[V];
#pragma unroll
        for (int e = 0; e < V; ++e) a[e] = red[wave][0][V * lane + e];
#pragma unroll 4
        for (int w = 1; w < WAVES; ++w)
#pragma unroll
            for (int e = 0; e < V; ++e) a[e] += red[wave][w][V * lane + e];
#pragma unroll
        for (int e = 0; e < V; ++e) tot[wave][V * lane + e] = a[e];
    }
    if (!NO_RED) __syncthreads();
    float sg[G][V];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
        for (int e = 0; e < V; ++e) sg[g][e] = NO_RED ? red[g][wave][V * lane + e] : tot[g][V * lane + e];
    // 5. y_r = v_r + sum_g c_{r,g} S_g, each stored as soon as it is formed (no loads from here);
    //    a row with a non-finite output (rare) is recomputed from its CSR row afterwards
    uint32_t bad = 0;                                                    // wave-uniform row bits
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        if (wave + WAVES * r < M) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const float cg = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d.cf[1 + g]), r));
#pragma unroll
                for (int e = 0; e < V; ++e) v[r][e] = __builtin_fmaf(cg, sg[g][e], v[r][e]);
            }
            const int64_t row = __builtin_amdgcn_readlane(d.row, r);
            if (__ballot(act && !finite_v<V>(v[r]))) {
                bad |= 1u << r;
            } else if (act) {
                if constexpr (PLAIN_ST) *reinterpret_cast<float4 *>(yc + row * ld_y + lo) = make_float4(v[r][0], v[r][V > 1 ? 1 : 0], v[r][V > 2 ? 2 : 0], v[r][V > 3 ? 3 : 0]);
                else stv_nt<V>(yc + row * ld_y + lo, v[r]);
            }
        }
    }
    while (bad) {                                                         // non-finite guard
        const int r = __builtin_ctz(bad);
        bad &= bad - 1;
        const int64_t row = __builtin_amdgcn_readlane(d.row, r);
        float o[V];
        csr_refix<V>(xc, ld_x, lo, act, row, csr_ptr, csr_col, csr_val, o);
        if (act) stv_nt<V>(yc + row * ld_y + lo, o);
    }
}

// ----------------------------------------------------------------------------------------------
// Multi-clique register tile for topologies with MANY cliques (10 000-node d-cliques: 100 cliques,
// each gathering one gateway row from every other clique, interclique.py:57-75).  k_mix_clique's
// item is one clique x 256 columns, so the rows one column chunk needs are N x 1 KB (10 MB at 10 000
// nodes): more than an XCD's 4 MB L2, and ~73 % of the gateway gathers (one per member) missed it.
// Here an item is Q cliques x 64 columns: lane quarter q = lane / (64 / Q) works on clique cg*Q + q,
// 4 columns per lane, so one wave-instruction loads a 256-B piece of Q rows of Q cliques.  Per item
// the bytes (and registers) are those of k_mix_clique's, but a column chunk's working set is N x 256
// B (2.5 MB at 10 000 nodes), and the chunk's items run together on one XCD (XCD-aware order), so a
// gateway row is in that XCD's L2 when its other reader comes for it.
//   descriptors: lane d < Q*RPW holds (clique d / RPW, slot d % RPW)'s member row, group, coefficients
//     and first residual entry; lanes fetch theirs with ds_bpermute (__shfl) when they use them;
//   1. member rows -> registers (RPW slots), then the first residual (gateway) row of slots [0, NA);
//   2. per-lane partial group sums -> LDS;  v := a*x;  gateway terms of slots [0, NA), then the
//      gathers of slots [NA, RPW) in the registers just freed; members with several residual
//      entries (rare) gather the rest one by one;
//   3. cross-wave group sums (LDS), y = v + sum_g c_g S_g, non-temporal stores; a non-finite output
//      is recomputed from its CSR row per lane (non-finite guard, see csr_refix).
template <bool OFF32>
__device__ __forceinline__ const float *qrow(const float *base, int row, int64_t ld, unsigned lo) {
    // OFF32: every row of a column block lies within 4 GiB of the block base, so the lane's address
    // is the block base (SGPRs) + a 32-bit offset (one VGPR, global_load ... saddr)
    if constexpr (OFF32)
        return reinterpret_cast<const float *>(reinterpret_cast<const char *>(base) +
                                               ((uint32_t)row * (uint32_t)(ld * 4) + lo * 4u));
    else
        return base + (int64_t)row * ld + lo;
}

// MS (member split, round 6; NIIDMIX_CLIQUE_QM): MS lane quarters share one clique, quarter q taking
// members q % MS, q % MS + MS, ... of each wave's slots; the group sums add those quarters' partials
// after the cross-wave reduction.  MS = Q: an item is one clique x 64 columns, so a chunk's 100
// items (10 000 nodes) rather than 25 are spread over the XCD's blocks in flight: fewer chunks in
// flight per XCD, whose rows the gateway gathers then find in its L2.  MS = 1: Q cliques per item.
template <int WAVES, int RPW, int G, int Q, int OCC, int GA, bool OFF32, int MS = 1>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(OCC, 8))) void k_mix_clique_q(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t p,
    int32_t n_cliques, const int32_t *__restrict__ clique_ptr,
    const int32_t *__restrict__ member_row, const int32_t *__restrict__ member_group,
    const float *__restrict__ coef, const int32_t *__restrict__ res_ptr,
    const int32_t *__restrict__ res_col, const float *__restrict__ res_val, int64_t n_cg,
    int64_t n_items, int cpb_shift, int64_t bs_x, int64_t bs_y,
    const int64_t *__restrict__ csr_ptr, const int32_t *__restrict__ csr_col,
    const float *__restrict__ csr_val) {
    static_assert(Q * RPW <= 64 && (Q == 1 || Q == 2 || Q == 4 || Q == 8), "descriptor lanes");
    constexpr int LQ = 64 / Q;                 // lanes per clique
    constexpr int64_t CW = 4 * LQ;             // columns per item
    constexpr int NA = GA;                     // gateway gathers in flight per batch (the first
                                               // batch loads behind the member rows)
    __shared__ float4 red[G][WAVES][kWave];
    __shared__ float4 tot[G][kWave];
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    const int q = lane / LQ, lc = lane - q * LQ;
    // one item per block, or (a grid of fewer blocks, a multiple of 8) items t, t + gridDim, ...:
    // then each XCD has only gridDim / 8 consecutive items of its sequence in flight, so the
    // column chunks they span (and the gateway rows they gather) stay within its L2
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
    const int64_t local = t >> 3;
    const int64_t chunk = (local / n_cg) * 8 + (t & 7);
    const int64_t cg = local % n_cg;
    if (chunk * CW >= p) continue;             // block-uniform, before any barrier
    const bool act = chunk * CW + 4 * lc < p;  // p % 4 == 0: a lane's 4 columns are all in or out
    const unsigned lo = act ? (unsigned)(4 * lc) : 0u;
    const int64_t kb = chunk >> cpb_shift, cin = chunk - (kb << cpb_shift);
    const float *xc = x + kb * bs_x + cin * CW;
    float *yc = y + kb * bs_y + cin * CW;

    // descriptors, lane-parallel: lane d < Q*RPW -> (clique cg*Q + d / RPW, slot d % RPW):
    // d_rg = member row | group << 28 (-1: no member), d_rc = first residual source row (-1: none)
    int d_rg = -1, d_rc = -1;
    float d_rv = 0.f, d_cf[1 + G];
#pragma unroll
    for (int g = 0; g <= G; ++g) d_cf[g] = 0.f;
    bool d_multi = false;
    if (lane < Q * RPW) {
        const int dq = lane / RPW, dr = lane - (lane / RPW) * RPW;
        const int64_t c = cg * (Q / MS) + dq / MS;
        if (c < n_cliques) {
            const int32_t m0 = clique_ptr[c], M = clique_ptr[c + 1] - m0;
            const int k = dq % MS + MS * (wave + WAVES * dr);
            if (k < M) {
                const int32_t m = m0 + k;
                d_rg = member_row[m] | ((member_group[m] & kMemberGroupMask) << 28);
#pragma unroll
                for (int g = 0; g <= G; ++g) d_cf[g] = coef[(int64_t)m * (1 + G) + g];
                const int32_t rb = res_ptr[m], rn = res_ptr[m + 1] - rb;
                d_multi = rn > 1;
                if (rn > 0) {
                    d_rc = res_col[rb];
                    d_rv = res_val[rb];
                }
            }
        }
    }
    const bool multi = __ballot(d_multi) != 0;
    const int sl0 = q * RPW;                   // this lane's descriptor lane of slot 0
    constexpr int kRowMask = (1 << 28) - 1;
    // 1. member rows, then the gateway rows of slots [0, NA) (in flight behind them)
    float v[RPW][4];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int rg = __shfl(d_rg, sl0 + r);
        ldv<4>(qrow<OFF32>(xc, rg < 0 ? 0 : rg & kRowMask, ld_x, lo), v[r]);
    }
    float ga[NA][4];
#pragma unroll
    for (int r = 0; r < NA; ++r) {
        const int rc = __shfl(d_rc, sl0 + r);
        ldv<4>(qrow<OFF32>(xc, rc < 0 ? 0 : rc, ld_x, lo), ga[r]);
    }
    // every load above is issued before any use below (the scheduler would otherwise fuse the
    // per-slot loops and serialise the loads slot by slot under the 64-VGPR budget)
    __builtin_amdgcn_sched_barrier(0);
    // 2. partial group sums, one group at a time (a slot without a member is masked by rg < 0)
#pragma unroll
    for (int g = 0; g < G; ++g) {
        float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int rg = __shfl(d_rg, sl0 + r);
            const bool in = rg >= 0 && (rg >> 28) == g;
#pragma unroll
            for (int e = 0; e < 4; ++e) s[e] += in ? v[r][e] : 0.f;
        }
        red[g][wave][lane] = make_float4(s[0], s[1], s[2], s[3]);
    }
    // own terms and the gateway terms of slots [0, NA)
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const float a = __shfl(d_cf[0], sl0 + r);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[r][e] *= a;
    }
#pragma unroll
    for (int r = 0; r < NA; ++r) {
        const bool has = __shfl(d_rc, sl0 + r) >= 0;
        const float w = __shfl(d_rv, sl0 + r);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[r][e] = has ? __builtin_fmaf(w, ga[r][e], v[r][e]) : v[r][e];
    }
    // gathers of slots [NA, RPW) in batches of NA, in ga's registers.  Issuing gateway gathers
    // later, so that the chunk's other items have their rows in L2 first, measured slower at 10 000
    // nodes every way tried: all after the group sums 18.1 vs 15.5 ms; the first batch after this
    // wave's member rows arrived 18.9 / 27.6 ms (13 gathers per batch, spills) and 15.2 ms (7)
    // against 14.3 ms (profiles/r03/clique_q_late_gathers_10k.txt)
#pragma unroll
    for (int b0 = NA; b0 < RPW; b0 += NA) {
#pragma unroll
        for (int r = b0; r < RPW && r < b0 + NA; ++r) {
            const int rc = __shfl(d_rc, sl0 + r);
            ldv<4>(qrow<OFF32>(xc, rc < 0 ? 0 : rc, ld_x, lo), ga[r - b0]);
        }
#pragma unroll
        for (int r = b0; r < RPW && r < b0 + NA; ++r) {
            const bool has = __shfl(d_rc, sl0 + r) >= 0;
            const float w = __shfl(d_rv, sl0 + r);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[r][e] = has ? __builtin_fmaf(w, ga[r - b0][e], v[r][e]) : v[r][e];
        }
    }
    // members with several residual entries (rare): the rest one by one, per lane
    if (multi) {
        const int64_t c = cg * (Q / MS) + q / MS;
        const int32_t m0 = c < n_cliques ? clique_ptr[c] : 0;
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            if (__shfl(d_rg, sl0 + r) < 0) continue;
            const int32_t m = m0 + q % MS + MS * (wave + WAVES * r);
            const int rb = res_ptr[m], re = res_ptr[m + 1];
            for (int j = rb + 1; j < re; ++j) {
                const float w = res_val[j];
                float xv[4];
                ldv<4>(xc + (int64_t)res_col[j] * ld_x + lo, xv);
#pragma unroll
                for (int e = 0; e < 4; ++e) v[r][e] = __builtin_fmaf(w, xv[e], v[r][e]);
            }
        }
    }
    // 3. group sums across waves
    __syncthreads();
    if (wave < G) {
        float4 a = red[wave][0][lane];
#pragma unroll 4
        for (int w = 1; w < WAVES; ++w) {
            const float4 b = red[wave][w][lane];
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        tot[wave][lane] = a;
    }
    __syncthreads();
    float sg[G][4];
#pragma unroll
    for (int g = 0; g < G; ++g) {
        const int q0 = q - q % MS;             // the clique's first quarter
        float4 a = tot[g][q0 * LQ + lc];
#pragma unroll
        for (int qq = 1; qq < MS; ++qq) {      // the clique's group sums: its quarters' partials
            const float4 b = tot[g][(q0 + qq) * LQ + lc];
            a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
        }
        sg[g][0] = a.x; sg[g][1] = a.y; sg[g][2] = a.z; sg[g][3] = a.w;
    }
    uint32_t bad = 0;                          // this lane's slots with a non-finite output
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
#pragma unroll
        for (int g = 0; g < G; ++g) {
            const float cg_ = __shfl(d_cf[1 + g], sl0 + r);
#pragma unroll
            for (int e = 0; e < 4; ++e) v[r][e] = __builtin_fmaf(cg_, sg[g][e], v[r][e]);
        }
        const int rg = __shfl(d_rg, sl0 + r);
        if (rg >= 0 && act) {
            if (finite_v<4>(v[r])) stv_nt<4>(const_cast<float *>(qrow<OFF32>(yc, rg & kRowMask, ld_y, lo)), v[r]);
            else bad |= 1u << r;
        }
    }
    // non-finite guard, per lane (see csr_refix).  The slot loop is wave-uniform: __shfl (ds_bpermute)
    // reads 0 from a lane that is not executing, so the row must be fetched with every lane active,
    // not inside a loop over this lane's own `bad` bits.
    if (__ballot(bad != 0u)) {
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int64_t row = __shfl(d_rg, sl0 + r) & kRowMask;
            if ((bad >> r) & 1u) {
                float o[4];
                csr_refix<4>(xc, ld_x, lo, true, row, csr_ptr, csr_col, csr_val, o);
                stv_nt<4>(yc + row * ld_y + lo, o);
            }
        }
    }
    if (t + (int64_t)gridDim.x < n_items) __syncthreads();   // red / tot are rewritten next item
    }
}

// ----------------------------------------------------------------------------------------------
// Dense Y = W^T X on fp32 MFMA.  Block tile 128 (output rows i) x 128 (columns j), K step 16,
// 4 waves in 2x2, each wave 64x64 = 2x2 tiles of v_mfma_f32_32x32x2_f32.
//   A[i][k] = W[k0+k][i0+i]  (LDS As[k][i]);  B[k][j] = X[k0+k][j0+j]  (LDS Bs[k][j])
//   operand maps (32x32x2 f32): lane l holds A[l&31][l>>5], B[l>>5][l&31];
//   C/D: col = l&31, row = (r&3) + 8*(r>>2) + 4*(l>>5), r = 0..15.
constexpr int kDBM = 128, kDBN = 128, kDBK = 32, kDPad = 4;

// Software pipeline: the next K-step's A/B tiles are fetched into registers while the MFMAs of
// the current step run; LDS is double-buffered so one barrier per K-step suffices.  SCHED: the
// operand reads of MFMA step u + 2 are issued between step u's MFMAs (sched_group_barrier), where
// the compiler's own schedule waited for four fresh LDS reads before every group of four MFMAs
// (MfmaUtil 74 %).  Tried and slower: k-contiguous LDS tiles read as ds_read_b128 with per-lane
// dword global loads (20.9 ms), and a branch-free clamped fetch (19.0 ms), vs 18.05 ms.
template <bool VEC, bool AVEC, bool SCHED = false, int BK = kDBK, int OCC = (BK == 32 ? 2 : 3)>
__global__ __launch_bounds__(256, OCC) void k_mix_dense(const float *__restrict__ x, int64_t ld_x,
                                                      float *__restrict__ y, int64_t ld_y, int64_t n,
                                                      int64_t p, const float *__restrict__ w,
                                                      int64_t n_it, int64_t n_items,
                                                      const int64_t *__restrict__ csr_ptr,
                                                      const int32_t *__restrict__ csr_col,
                                                      const float *__restrict__ csr_val) {
    __shared__ float As[2][BK][kDBM + kDPad];
    __shared__ float Bs[2][BK][kDBN + kDPad];
    const int tid = threadIdx.x;
    const int wave = wave_id();
    const int lane = tid & 63;
    const int wm = wave >> 1, wn = wave & 1;
    // loader mapping: 32 rows x 128 cols = 4096 floats per operand, 16 per thread (4 x float4)
    const int lk = tid >> 5;          // 0..7  (+8*h)
    const int lc = (tid & 31) * 4;    // 0..124
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int64_t jt = (local / n_it) * 8 + xcd;
        const int64_t it = local % n_it;
        const int64_t i0 = it * kDBM, j0 = jt * kDBN;
        if (j0 >= p) continue;  // block-uniform
        floatx16 acc[2][2];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

        constexpr int NH = BK / 8;           // float4 rows per thread per operand
        float ra[NH][4], rb[NH][4];
        // interior tiles and K-steps (block-uniform): no per-lane bounds, no zero-fill
        const bool inner = AVEC && VEC && i0 + kDBM <= n && j0 + kDBN <= p;
        auto fetch = [&](int64_t k0) {
            if (inner && k0 + BK <= n) {
#pragma unroll
                for (int h = 0; h < NH; ++h) {
                    const int64_t kr = k0 + lk + 8 * h;
                    const float4 a = ld4(w + kr * n + i0 + lc), b = ld4(x + kr * ld_x + j0 + lc);
                    ra[h][0] = a.x; ra[h][1] = a.y; ra[h][2] = a.z; ra[h][3] = a.w;
                    rb[h][0] = b.x; rb[h][1] = b.y; rb[h][2] = b.z; rb[h][3] = b.w;
                }
                return;
            }
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const int64_t kr = k0 + lk + 8 * h;
                if (AVEC) {
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (kr < n && i0 + lc < n) v = ld4(w + kr * n + i0 + lc);
                    ra[h][0] = v.x; ra[h][1] = v.y; ra[h][2] = v.z; ra[h][3] = v.w;
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int64_t i = i0 + lc + u;
                        ra[h][u] = (kr < n && i < n) ? w[kr * n + i] : 0.f;
                    }
                }
                if (VEC) {
                    const int64_t j = j0 + lc;
                    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                    if (kr < n && j < p) v = ld4(x + kr * ld_x + j);
                    rb[h][0] = v.x; rb[h][1] = v.y; rb[h][2] = v.z; rb[h][3] = v.w;
                } else {
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const int64_t j = j0 + lc + u;
                        rb[h][u] = (kr < n && j < p) ? x[kr * ld_x + j] : 0.f;
                    }
                }
            }
        };
        fetch(0);
        int buf = 0;
        for (int64_t k0 = 0; k0 < n; k0 += BK) {
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                *reinterpret_cast<float4 *>(&As[buf][lk + 8 * h][lc]) = make_float4(ra[h][0], ra[h][1], ra[h][2], ra[h][3]);
                *reinterpret_cast<float4 *>(&Bs[buf][lk + 8 * h][lc]) = make_float4(rb[h][0], rb[h][1], rb[h][2], rb[h][3]);
            }
            __syncthreads();
            if (k0 + BK < n) fetch(k0 + BK);          // in flight during the MFMAs below
            if (SCHED) {
                // every operand read written first, then the MFMAs; the scheduling groups below
                // interleave them so the reads of step u + 2 are in flight during step u's MFMAs
                float a0v[BK / 2], a1v[BK / 2], b0v[BK / 2], b1v[BK / 2];
#pragma unroll
                for (int u = 0; u < BK / 2; ++u) {
                    const int kq = 2 * u + (lane >> 5);
                    a0v[u] = As[buf][kq][wm * 64 + (lane & 31)];
                    a1v[u] = As[buf][kq][wm * 64 + 32 + (lane & 31)];
                    b0v[u] = Bs[buf][kq][wn * 64 + (lane & 31)];
                    b1v[u] = Bs[buf][kq][wn * 64 + 32 + (lane & 31)];
                }
#pragma unroll
                for (int u = 0; u < BK / 2; ++u) {
                    acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0v[u], b0v[u], acc[0][0], 0, 0, 0);
                    acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0v[u], b1v[u], acc[0][1], 0, 0, 0);
                    acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1v[u], b0v[u], acc[1][0], 0, 0, 0);
                    acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1v[u], b1v[u], acc[1][1], 0, 0, 0);
                }
                __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);          // DS reads, steps 0-1
#pragma unroll
                for (int u = 0; u < BK / 2 - 2; ++u) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);      // MFMAs of step u
                    __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);      // DS reads of step u + 2
                }
                __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
            } else {
#pragma unroll
            for (int kk = 0; kk < BK; kk += 2) {
                const int kq = kk + (lane >> 5);
                const float a0 = As[buf][kq][wm * 64 + (lane & 31)];
                const float a1 = As[buf][kq][wm * 64 + 32 + (lane & 31)];
                const float b0 = Bs[buf][kq][wn * 64 + (lane & 31)];
                const float b1 = Bs[buf][kq][wn * 64 + 32 + (lane & 31)];
                acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
                acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
                acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
                acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
            }
            }
            buf ^= 1;
        }
        uint64_t bad = 0;                         // this lane's non-finite outputs (a, b, r)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t i = i0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    const int64_t j = j0 + wn * 64 + b * 32 + (lane & 31);
                    if (i < n && j < p) {
                        if (__builtin_isfinite(acc[a][b][r])) __builtin_nontemporal_store(acc[a][b][r], y + i * ld_y + j);
                        else bad |= 1ull << (a * 32 + b * 16 + r);
                    }
                }
        while (bad) {                             // non-finite guard (see csr_refix): 0*inf from
            const int q = __builtin_ctzll(bad);   // W = 0 off the edges must not leak into outputs
            bad &= bad - 1;
            const int a = q >> 5, b = (q >> 4) & 1, r = q & 15;
            const int64_t i = i0 + wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
            const int64_t j = j0 + wn * 64 + b * 32 + (lane & 31);
            __builtin_nontemporal_store(csr_refix1(x + j, ld_x, i, csr_ptr, csr_col, csr_val), y + i * ld_y + j);
        }
        __syncthreads();   // LDS buffers are rewritten by the next tile
    }
}

// ----------------------------------------------------------------------------------------------
// Dense Y = W^T X on the BF16 matrix cores, fp32-accurate by three-term splitting (round 5).
// On gfx950 the fp32-input MFMA issues at 1/16 of the bf16 rate (64 vs 1024 FLOP/clk/SIMD,
// MI355X_MICROARCH.md § Matrix cores), so an fp32 product a*b is carried by bf16 splits
// a = a_h + a_m + a_l (a_h = RNE bf16 of a, a_m of a - a_h, a_l of a - a_h - a_m; the residue is below
// 2^-24 |a|) and the six partial products that reach 2^-16 |a b| are summed in fp32 by the MFMA:
//     a_h b_h + a_h b_m + a_m b_h + a_h b_l + a_l b_h + a_m b_m.
// The dropped terms (a_m b_l, a_l b_m, a_l b_l) and the residues stay below ~2^-23 |a b| -- the order
// of one fp32 rounding -- so the result keeps fast mode's 1e-5 condition-aware tolerance with an
// fp32 GEMM's margin, at 16/6 = 2.7x the fp32 MFMA's rate.  Non-finite inputs make the splits NaN
// (inf - inf) and the output non-finite, which the guard recomputes from the CSR (as k_mix_dense).
//   W^T is split ONCE per topology (k_dense_split_w): wp[3][mpad][kpad] bf16, row i = output node,
//   k contiguous, zero-padded (mpad = n rounded up to 256, kpad to 16).
//   X is split as it is staged: LDS [plane][column][16 k] bf16, so a B operand's run of 8 k is one
//   ds_read_b128; W tiles land in LDS [plane][row][16 k] the same way.
// Block tile 128 rows x 256 columns, 8 waves (2 x 4), each 64 x 64 = 2 x 2 accumulators of
// v_mfma_f32_32x32x16_bf16; K-step 16, LDS double-buffered (72 KB dynamic), the next K-step's W
// pieces and X values fetched into registers during the MFMAs, one barrier per K-step.  Operand
// maps (32x32x16 bf16): lane l holds A[l&31][8(l>>5) + 0..7] and B[8(l>>5) + 0..7][l&31]; C as
// k_mix_dense.  The two 16-B halves of every 32-B LDS row swap places on alternate groups of 8
// rows (half ^ (row >> 3 & 1)): the ds_read_b128 of 16 consecutive rows hit 16 distinct bank quads.
constexpr int kB6M = 256, kB6K = 16;   // W split padding: rows to 256, k to 16
// the six split products (plane of A, plane of B), smallest first: mm, lh, hl, mh, hm, hh
__device__ constexpr int kB6PA[6] = {1, 2, 0, 1, 0, 0}, kB6PB[6] = {1, 0, 2, 0, 1, 0};
typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

// two floats -> their three bf16 split planes, each as a packed pair (first value in the low half)
__device__ __forceinline__ void split3_pair(float a, float b, uint32_t &h, uint32_t &m, uint32_t &l) {
    const bf16x2v hv = {(__bf16)a, (__bf16)b};
    const uint32_t hb = __builtin_bit_cast(uint32_t, hv);
    const float ra = a - __builtin_bit_cast(float, hb << 16);
    const float rb = b - __builtin_bit_cast(float, hb & 0xffff0000u);
    const bf16x2v mv = {(__bf16)ra, (__bf16)rb};
    const uint32_t mb = __builtin_bit_cast(uint32_t, mv);
    const float sa = ra - __builtin_bit_cast(float, mb << 16);
    const float sb = rb - __builtin_bit_cast(float, mb & 0xffff0000u);
    const bf16x2v lv = {(__bf16)sa, (__bf16)sb};
    h = hb;
    m = mb;
    l = __builtin_bit_cast(uint32_t, lv);
}

// wp[p][i][k] = plane p of W[k][i] = w[k * n + i]; zero outside [n, n)
__global__ __launch_bounds__(256) void k_dense_split_w(const float *__restrict__ w, int64_t n,
                                                       int64_t mpad, int64_t kpad,
                                                       uint32_t *__restrict__ wp) {
    const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // k pair index
    const int64_t half = kpad / 2;
    if (q >= mpad * half) return;
    const int64_t i = q / half, k = 2 * (q - i * half);
    const float a = (i < n && k < n) ? w[k * n + i] : 0.f;
    const float b = (i < n && k + 1 < n) ? w[(k + 1) * n + i] : 0.f;
    uint32_t h, m, l;
    split3_pair(a, b, h, m, l);
    const int64_t plane = mpad * half;                  // uint32 words per plane
    wp[q] = h;
    wp[plane + q] = m;
    wp[2 * plane + q] = l;
}

// WN = waves along N: 4 -> 8-wave blocks of 128 x 256 (one block per CU: 176 VGPRs, 2 waves per
// SIMD, one barrier phase per CU), 2 -> 4-wave blocks of 128 x 128 (two blocks per CU, each with
// its own barrier phase, so one block's split and barrier overlap the other's MFMAs; W is re-read
// per 128 columns instead of 256)
// ABL (time-split builds only: -DNIIDMIX_ABLATIONS, NIIDMIX_DENSE_B6_ABL; results are wrong): 1 no
// global loads in the K loop, 2 no MFMAs, 3 no LDS operand reads, 4 X as if pre-split (three
// 16-B pieces loaded and stored per thread and K-step, no split)
template <int WN, int SCHED, int ABL = 0, int TM = 2>
__global__ __launch_bounds__(128 * WN, 4 / WN) void k_mix_dense_b6(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t n,
    int64_t p, const uint16_t *__restrict__ wp, int64_t mpad, int64_t kpad, int64_t n_it,
    int64_t n_items, const int64_t *__restrict__ csr_ptr, const int32_t *__restrict__ csr_col,
    const float *__restrict__ csr_val) {
    constexpr int NT = 128 * WN;                           // threads
    constexpr int BN = 64 * WN;                            // columns per block tile
    constexpr int BM = 64 * TM;                            // rows per block tile (2 waves along M)
    constexpr int NPIECE = 3 * BM * 2;                     // 16-B W pieces per K-step
    constexpr int NPT = (NPIECE + NT - 1) / NT;            // pieces per thread (2 or 3)
    static_assert(NPT <= 3, "W pieces per thread");
    extern __shared__ uint4 lds_b6[];
    // As[buf][plane][row][half] then Bs[buf][plane][col][half], 16 B each
    auto A_at = [&](int b, int pl, int row, int hf) -> uint4 & {
        return lds_b6[((b * 3 + pl) * BM + row) * 2 + hf];
    };
    auto B_at = [&](int b, int pl, int col, int hf) -> uint4 & {
        return lds_b6[2 * 3 * BM * 2 + ((b * 3 + pl) * BN + col) * 2 + hf];
    };
    const int tid = threadIdx.x;
    const int wave = wave_id();
    const int lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int bj = tid % BN, bh = tid / BN;                // X loader: column, k half
    // W loader: pieces q = tid + NT u (u = 0, 1, 2) of 768 (3 planes x 128 rows x 2 halves); a
    // thread past 768 loads a valid piece again and does not store it
    int qpl[3], qrow[3], qhf[3];
    bool qok[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        const int q0 = tid + NT * u;
        qok[u] = q0 < NPIECE;
        const int q = qok[u] ? q0 : tid;
        qpl[u] = q / (2 * BM);
        qrow[u] = (q >> 1) & (BM - 1);
        qhf[u] = q & 1;
    }
    const int hl = lane >> 5;
    const int64_t S = kpad / kB6K;
    const int64_t plane_el = mpad * kpad;                  // bf16 elements per W plane
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int64_t jt = (local / n_it) * 8 + xcd;
        const int64_t it = local % n_it;
        const int64_t i0 = it * BM, j0 = jt * BN;
        if (j0 >= p) continue;                             // block-uniform
        floatx16 acc[TM][2];
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
        // Two register sets of prefetched operands (K-steps s + 1 and s + 2): the loads of a K-step
        // are issued two steps before it is computed and split one step before, interleaved with
        // the MFMAs of the step in between.  Every load is unconditional (clamped addresses; the X
        // values past n or p are zeroed by a bit mask after the load, never by a branch): the
        // number of loads in flight is the same on every path, so each split waits only for its
        // own loads.  Written as macros over named registers (no arrays behind a lambda's
        // reference capture, which hipcc put in scratch memory).
        // Loads by buffer instructions: one SGPR resource + a per-lane 32-bit offset + a scalar
        // offset each (no 64-bit address arithmetic per load), and a load past the resource's
        // extent returns 0 -- X rows past n (the last K-step) and columns past p (their lanes'
        // offset is pushed out of range) arrive as zeros, with no clamp, select or branch.  The
        // launcher checks 16 rows x ld_x x 4 B < 2^31 and the split W < 2^31 B.
        const int64_t jx = j0 + bj;
        const bool jin = jx < p;
        const uint32_t xvoff = jin ? (uint32_t)jx * 4u : 0x80000000u;
        const uint32_t rowb = (uint32_t)ld_x * 4u;
        uint32_t wvoff[3];
#pragma unroll
        for (int u = 0; u < 3; ++u)
            wvoff[u] = (uint32_t)((((int64_t)qpl[u] * mpad + i0 + qrow[u]) * kpad + 8 * qhf[u]) * 2);
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint16_t *>(wp), (short)0, (int)(3 * plane_el * 2), 0x00020000);
        uint4 wa0, wb0, wc0, wa1, wb1, wc1;
        uint4 xq0[3], xq1[3];                              // ABL 4 only (pre-split X pieces)
        float xv0[8], xv1[8];
        const int bhu = __builtin_amdgcn_readfirstlane(bh);
#define B6_FETCH(SET, S_)                                                                          \
        do {                                                                                       \
            const int64_t k0_ = ((S_) < S ? (S_) : S - 1) * kB6K;                                 \
            const int64_t ext_ = (n - k0_) * (int64_t)rowb;                                        \
            const __amdgpu_buffer_rsrc_t xr_ = __builtin_amdgcn_make_buffer_rsrc(                  \
                const_cast<float *>(x + k0_ * ld_x), (short)0,                                     \
                (int)(ext_ < 0x7fffffffLL ? ext_ : 0x7fffffffLL), 0x00020000);                     \
            const int wso_ = (int)(k0_ * 2);                                                       \
            if (ABL != 1) {                                                                        \
            wa##SET = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoff[0], wso_, 0)); \
            wb##SET = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoff[1], wso_, 0)); \
            if (NPT == 3) wc##SET = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(wrs, wvoff[2], wso_, 0)); \
            if (ABL == 4) {                                                                        \
                _Pragma("unroll") for (int u = 0; u < 3; ++u)                                      \
                    xq##SET[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(  \
                        wrs, wvoff[u] ^ 0x400u, wso_, 0));                                         \
            } else                                                                                 \
            _Pragma("unroll") for (int u = 0; u < 8; ++u)                                          \
                xv##SET[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(       \
                                 xr_, xvoff, (int)((8 * bhu + u) * rowb), 0));                     \
            } else {                                                                               \
                wa##SET = make_uint4(k0_, 1, 2, 3); wb##SET = wa##SET; wc##SET = wa##SET;          \
                _Pragma("unroll") for (int u = 0; u < 8; ++u) xv##SET[u] = (float)(k0_ + u);       \
            }                                                                                      \
        } while (0)
#define B6_STASH(SET, BUF, S_)                                                                     \
        do {                                                                                       \
            A_at(BUF, qpl[0], qrow[0], qhf[0] ^ ((qrow[0] >> 3) & 1)) = wa##SET;                   \
            /* a thread without a second piece re-stores its first (q = tid): same data, same  \
               place -- no branch in the step */                                                   \
            A_at(BUF, qpl[1], qrow[1], qhf[1] ^ ((qrow[1] >> 3) & 1)) = wb##SET;                   \
            if (NPT == 3) A_at(BUF, qpl[2], qrow[2], qhf[2] ^ ((qrow[2] >> 3) & 1)) = wc##SET;      \
            const int sh_ = bh ^ ((bj >> 3) & 1);                                                  \
            if (ABL == 4) {                                                                        \
                _Pragma("unroll") for (int u = 0; u < 3; ++u) B_at(BUF, u, bj, sh_) = xq##SET[u];  \
            } else {                                                                               \
            uint32_t h_[4], m_[4], l_[4];                                                          \
            _Pragma("unroll") for (int u = 0; u < 4; ++u)                                          \
                split3_pair(xv##SET[2 * u], xv##SET[2 * u + 1], h_[u], m_[u], l_[u]);              \
            B_at(BUF, 0, bj, sh_) = make_uint4(h_[0], h_[1], h_[2], h_[3]);                        \
            B_at(BUF, 1, bj, sh_) = make_uint4(m_[0], m_[1], m_[2], m_[3]);                        \
            B_at(BUF, 2, bj, sh_) = make_uint4(l_[0], l_[1], l_[2], l_[3]);                        \
            }                                                                                      \
        } while (0)
        // K-step s on LDS buffer B = s & 1: issue the loads of s + 2 (register set B), read the
        // operands, run the MFMAs, split s + 1 (set B ^ 1) into buffer B ^ 1, barrier
#define B6_STEP(B, NB, S_)                                                                         \
        do {                                                                                       \
            B6_FETCH(B, (S_) + 2);                                                                 \
            /* SCHED 3: the loads stay at the top of the step (the compiler's schedule sinks them  \
               below the MFMAs, and the next step's split waits for them) */                       \
            if (SCHED == 3) __builtin_amdgcn_sched_barrier(0);                                     \
            bf16x8v af_[TM][3], bf_[2][3];                                                          \
            /* operand reads in the order the products use them: (A m, B m), (A l, B h), (A h, B l) */ \
            if (ABL == 3) {                                                                        \
                _Pragma("unroll") for (int q_ = 0; q_ < 3 * TM; ++q_)                              \
                    af_[q_ / 3][q_ % 3] = __builtin_bit_cast(bf16x8v, make_uint4(lane, q_, 1, 2)); \
                _Pragma("unroll") for (int q_ = 0; q_ < 6; ++q_)                                   \
                    bf_[q_ / 3][q_ % 3] = __builtin_bit_cast(bf16x8v, make_uint4(q_, lane, 3, 4)); \
            } else                                                                                 \
            _Pragma("unroll") for (int o = 0; o < 3; ++o) {                                        \
                const int pa_ = o == 0 ? 1 : o == 1 ? 2 : 0, pb_ = o == 0 ? 1 : o == 1 ? 0 : 2;    \
                _Pragma("unroll") for (int a = 0; a < TM; ++a) {                                   \
                    const int row_ = wm * 32 * TM + a * 32 + (lane & 31);                          \
                    af_[a][pa_] = __builtin_bit_cast(bf16x8v, A_at(B, pa_, row_, hl ^ ((row_ >> 3) & 1))); \
                }                                                                                  \
                _Pragma("unroll") for (int c = 0; c < 2; ++c) {                                    \
                    const int col_ = wn * 64 + c * 32 + (lane & 31);                               \
                    bf_[c][pb_] = __builtin_bit_cast(bf16x8v, B_at(B, pb_, col_, hl ^ ((col_ >> 3) & 1))); \
                }                                                                                  \
            }                                                                                      \
            if (ABL != 2)                                                                          \
            _Pragma("unroll") for (int e = 0; e < 6; ++e)                                          \
                _Pragma("unroll") for (int a = 0; a < TM; ++a)                                     \
                    _Pragma("unroll") for (int c = 0; c < 2; ++c)                                  \
                        acc[a][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(                       \
                            af_[a][kB6PA[e]], bf_[c][kB6PB[e]], acc[a][c], 0, 0, 0);               \
            else                                                                                   \
                _Pragma("unroll") for (int q_ = 0; q_ < 6; ++q_)                                   \
                    asm volatile("" :: "v"(af_[q_ % TM][q_ % 3]), "v"(bf_[q_ / 3][q_ % 3]));       \
            /* unconditional (no branch between the MFMAs and the split): past the last K-step  \
               it stores the clamped refetch into a buffer no step reads */                        \
            B6_STASH(NB, NB, (S_) + 1);                                                            \
            /* schedule: the loads; the operand reads in three slices of four (the products in  \
               plane order mm, lh, hl, then mh, hm, hh need no new operands), MFMAs starting as   \
               soon as the first slice lands; SCHED 0: the split beside the MFMAs, two VALU per    \
               MFMA; SCHED 1: the split after them; the LDS writes last */                         \
            if (SCHED < 2) {                                                                       \
            __builtin_amdgcn_sched_group_barrier(0x020, 12, 0);                                    \
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);                                     \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                                     \
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);                                     \
            __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);                                     \
            __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);                                     \
            }                                                                                      \
            if (SCHED == 0) {                                                                      \
                _Pragma("unroll") for (int i_ = 0; i_ < 20; ++i_) {                                \
                    __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                             \
                    __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);                             \
                }                                                                                  \
            } else if (SCHED == 1) {                                                               \
                __builtin_amdgcn_sched_group_barrier(0x008, 20, 0);                                \
                __builtin_amdgcn_sched_group_barrier(0x002, 80, 0);                                \
            }                                                                                      \
            if (SCHED < 2) __builtin_amdgcn_sched_group_barrier(0x200, 6, 0);                      \
            __syncthreads();                                                                       \
        } while (0)
        B6_FETCH(0, 0);
        B6_STASH(0, 0, 0);
        B6_FETCH(1, 1);
        __syncthreads();
        // the loop body is both steps with no branch between them and an odd last step peeled off:
        // with `if (s + 1 < S)` around the second step, the path that skips it reached the loop
        // header with the first step's loads in flight, and the compiler waited for every load
        // (vmcnt(0)) at the top of each iteration
        int64_t s = 0;
        for (; s + 1 < S; s += 2) {
            B6_STEP(0, 1, s);
            B6_STEP(1, 0, s + 1);
        }
        if (s < S) B6_STEP(0, 1, s);
#undef B6_STEP
#undef B6_STASH
#undef B6_FETCH
        uint64_t bad[2] = {0, 0};                          // this lane's non-finite outputs
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t i = i0 + wm * 32 * TM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    const int64_t j = j0 + wn * 64 + c * 32 + (lane & 31);
                    if (i < n && j < p) {
                        if (__builtin_isfinite(acc[a][c][r])) __builtin_nontemporal_store(acc[a][c][r], y + i * ld_y + j);
                        else bad[a >> 1] |= 1ull << ((a & 1) * 32 + c * 16 + r);
                    }
                }
#pragma unroll
        for (int h = 0; h < 2; ++h)
            while (bad[h]) {                               // non-finite guard (csr_refix1)
                const int q = __builtin_ctzll(bad[h]);
                bad[h] &= bad[h] - 1;
                const int a = 2 * h + (q >> 5), c = (q >> 4) & 1, r = q & 15;
                const int64_t i = i0 + wm * 32 * TM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int64_t j = j0 + wn * 64 + c * 32 + (lane & 31);
                __builtin_nontemporal_store(csr_refix1(x + j, ld_x, i, csr_ptr, csr_col, csr_val), y + i * ld_y + j);
            }
    }
}

// The same GEMM with ONE wave per SIMD (round 5, tuning A/B: NIIDMIX_DENSE_B6_W1=1): a 256 x 256
// block tile of 4 waves of 128 x 128 (4 x 4 accumulators = 256 registers, which the compiler puts
// in AGPRs: a wave of a one-wave-per-SIMD kernel has 256 VGPRs + 256 AGPRs), 96 MFMAs per wave per
// K-step -- twice the two-wave kernel's per barrier -- while the split, the LDS writes and the next
// loads issue between them.  Per thread and K-step: 6 W pieces and one column's 16 X values.
// Products, K order and MFMA per output element are those of k_mix_dense_b6: bit-identical results.
__global__ __launch_bounds__(256, 1) void k_mix_dense_b6w(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t n,
    int64_t p, const uint16_t *__restrict__ wp, int64_t mpad, int64_t kpad, int64_t n_it,
    int64_t n_items, const int64_t *__restrict__ csr_ptr, const int32_t *__restrict__ csr_col,
    const float *__restrict__ csr_val) {
    constexpr int NT = 256, BM = 256, BN = 256, TM = 4, TN = 4;
    constexpr int NPT = 3 * BM * 2 / NT;                   // W pieces per thread: 6
    extern __shared__ uint4 lds_b6[];
    auto A_at = [&](int b, int pl, int row, int hf) -> uint4 & {
        return lds_b6[((b * 3 + pl) * BM + row) * 2 + hf];
    };
    auto B_at = [&](int b, int pl, int col, int hf) -> uint4 & {
        return lds_b6[2 * 3 * BM * 2 + ((b * 3 + pl) * BN + col) * 2 + hf];
    };
    const int tid = threadIdx.x;
    const int wave = wave_id();
    const int lane = tid & 63;
    const int wm = wave >> 1, wn = wave & 1;
    const int bj = tid;                                    // X loader: one column, all 16 k
    int qpl[NPT], qrow[NPT], qhf[NPT];
#pragma unroll
    for (int u = 0; u < NPT; ++u) {
        const int q = tid + NT * u;
        qpl[u] = q / (2 * BM);
        qrow[u] = (q >> 1) & (BM - 1);
        qhf[u] = q & 1;
    }
    const int hl = lane >> 5;
    const int64_t S = kpad / kB6K;
    const int64_t plane_el = mpad * kpad;
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int64_t jt = (local / n_it) * 8 + xcd;
        const int64_t it = local % n_it;
        const int64_t i0 = it * BM, j0 = jt * BN;
        if (j0 >= p) continue;                             // block-uniform
        floatx16 acc[TM][TN];
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int c = 0; c < TN; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;
        const int64_t jx = j0 + bj;
        const uint32_t xvoff = jx < p ? (uint32_t)jx * 4u : 0x80000000u;
        const uint32_t rowb = (uint32_t)ld_x * 4u;
        uint32_t wvoff[NPT];
#pragma unroll
        for (int u = 0; u < NPT; ++u)
            wvoff[u] = (uint32_t)((((int64_t)qpl[u] * mpad + i0 + qrow[u]) * kpad + 8 * qhf[u]) * 2);
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint16_t *>(wp), (short)0, (int)(3 * plane_el * 2), 0x00020000);
        uint4 wq0[NPT], wq1[NPT];
        float xv0[16], xv1[16];
#define B6W_FETCH(SET, S_)                                                                         \
        do {                                                                                       \
            const int64_t k0_ = ((S_) < S ? (S_) : S - 1) * kB6K;                                 \
            const int64_t ext_ = (n - k0_) * (int64_t)rowb;                                        \
            const __amdgpu_buffer_rsrc_t xr_ = __builtin_amdgcn_make_buffer_rsrc(                  \
                const_cast<float *>(x + k0_ * ld_x), (short)0,                                     \
                (int)(ext_ < 0x7fffffffLL ? ext_ : 0x7fffffffLL), 0x00020000);                     \
            const int wso_ = (int)(k0_ * 2);                                                       \
            _Pragma("unroll") for (int u = 0; u < NPT; ++u)                                        \
                wq##SET[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(      \
                                 wrs, wvoff[u], wso_, 0));                                         \
            _Pragma("unroll") for (int u = 0; u < 16; ++u)                                         \
                xv##SET[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(       \
                                 xr_, xvoff, (int)(u * rowb), 0));                                 \
        } while (0)
#define B6W_STASH(SET, BUF)                                                                        \
        do {                                                                                       \
            _Pragma("unroll") for (int u = 0; u < NPT; ++u)                                        \
                A_at(BUF, qpl[u], qrow[u], qhf[u] ^ ((qrow[u] >> 3) & 1)) = wq##SET[u];            \
            _Pragma("unroll") for (int hf = 0; hf < 2; ++hf) {                                     \
                uint32_t h_[4], m_[4], l_[4];                                                      \
                _Pragma("unroll") for (int u = 0; u < 4; ++u)                                      \
                    split3_pair(xv##SET[8 * hf + 2 * u], xv##SET[8 * hf + 2 * u + 1], h_[u], m_[u], l_[u]); \
                const int sh_ = hf ^ ((bj >> 3) & 1);                                              \
                B_at(BUF, 0, bj, sh_) = make_uint4(h_[0], h_[1], h_[2], h_[3]);                    \
                B_at(BUF, 1, bj, sh_) = make_uint4(m_[0], m_[1], m_[2], m_[3]);                    \
                B_at(BUF, 2, bj, sh_) = make_uint4(l_[0], l_[1], l_[2], l_[3]);                    \
            }                                                                                      \
        } while (0)
#define B6W_STEP(B, NB, S_)                                                                        \
        do {                                                                                       \
            B6W_FETCH(B, (S_) + 2);                                                                \
            __builtin_amdgcn_sched_barrier(0);                                                     \
            bf16x8v af_[TM][3], bf_[TN][3];                                                         \
            _Pragma("unroll") for (int o = 0; o < 3; ++o) {                                        \
                const int pa_ = o == 0 ? 1 : o == 1 ? 2 : 0, pb_ = o == 0 ? 1 : o == 1 ? 0 : 2;    \
                _Pragma("unroll") for (int a = 0; a < TM; ++a) {                                   \
                    const int row_ = wm * 128 + a * 32 + (lane & 31);                              \
                    af_[a][pa_] = __builtin_bit_cast(bf16x8v, A_at(B, pa_, row_, hl ^ ((row_ >> 3) & 1))); \
                }                                                                                  \
                _Pragma("unroll") for (int c = 0; c < TN; ++c) {                                   \
                    const int col_ = wn * 128 + c * 32 + (lane & 31);                              \
                    bf_[c][pb_] = __builtin_bit_cast(bf16x8v, B_at(B, pb_, col_, hl ^ ((col_ >> 3) & 1))); \
                }                                                                                  \
            }                                                                                      \
            _Pragma("unroll") for (int e = 0; e < 6; ++e)                                          \
                _Pragma("unroll") for (int a = 0; a < TM; ++a)                                     \
                    _Pragma("unroll") for (int c = 0; c < TN; ++c)                                 \
                        acc[a][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(                       \
                            af_[a][kB6PA[e]], bf_[c][kB6PB[e]], acc[a][c], 0, 0, 0);               \
            B6W_STASH(NB, NB);                                                                     \
            __syncthreads();                                                                       \
        } while (0)
        B6W_FETCH(0, 0);
        B6W_STASH(0, 0);
        B6W_FETCH(1, 1);
        __syncthreads();
        int64_t s = 0;
        for (; s + 1 < S; s += 2) {
            B6W_STEP(0, 1, s);
            B6W_STEP(1, 0, s + 1);
        }
        if (s < S) B6W_STEP(0, 1, s);
#undef B6W_STEP
#undef B6W_STASH
#undef B6W_FETCH
        uint64_t bad[4] = {0, 0, 0, 0};                    // this lane's non-finite outputs
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int c = 0; c < TN; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t i = i0 + wm * 128 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    const int64_t j = j0 + wn * 128 + c * 32 + (lane & 31);
                    if (i < n && j < p) {
                        if (__builtin_isfinite(acc[a][c][r])) __builtin_nontemporal_store(acc[a][c][r], y + i * ld_y + j);
                        else bad[a] |= 1ull << (c * 16 + r);
                    }
                }
#pragma unroll
        for (int a = 0; a < TM; ++a)
            while (bad[a]) {                               // non-finite guard (csr_refix1)
                const int q = __builtin_ctzll(bad[a]);
                bad[a] &= bad[a] - 1;
                const int c = q >> 4, r = q & 15;
                const int64_t i = i0 + wm * 128 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int64_t j = j0 + wn * 128 + c * 32 + (lane & 31);
                __builtin_nontemporal_store(csr_refix1(x + j, ld_x, i, csr_ptr, csr_col, csr_val), y + i * ld_y + j);
            }
    }
}

// The same GEMM with the W tiles staged by LDS-DMA (round 6; NIIDMIX_DENSE_B6_DMA).
// The pre-split W pieces go straight from memory into LDS (buffer_load_dwordx4 ... lds: lane l of
// a wave-instruction writes 16 B at M0 + 16 l), so no W piece occupies VGPRs or costs a ds_write,
// and the W fetch of step s + NA - 1 goes out at the top of step s into an NA-deep ring of LDS
// buffers (NA 3: two K-steps ahead, as the X values; NA 2: one).  The A layout and its half swizzle
// are those of k_mix_dense_b6: the DMA's lane order fixes WHERE a piece lands, so each lane loads
// the piece that belongs at its slot.  X is fetched into registers two steps ahead and split into
// the double-buffered B planes as before.  The block barrier is an inline-asm s_barrier preceded by
// an explicit s_waitcnt that waits for this wave's W DMA of the next step only (the compiler's
// __syncthreads() drains vmcnt(0) once an LDS-DMA is in flight, which would also wait for the X
// fetch issued two steps ahead).  WN 2 (4 waves of 128 x 64 per 256 x 128 tile) with NA 2 fits two
// blocks per CU, whose barriers are independent: the two waves of a SIMD then belong to different
// blocks.  Products, K order and MFMA per output element are those of k_mix_dense_b6: bit-identical.
// one wave-instruction of the W ring's LDS-DMA: lane l's 16 B at voff + soff land at lds + 16 l
__device__ __forceinline__ void b6d_dma16(__amdgpu_buffer_rsrc_t rsrc, uint4 *lds, uint32_t voff,
                                          int soff) {
    typedef __attribute__((address_space(3))) void lds_void;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, (lds_void *)lds, 16, voff, soff, 0, 0);
}

template <int WN, int TM, int NA, int XD>
__global__ __launch_bounds__(128 * WN, (WN == 2 ? 2 : 1)) void k_mix_dense_b6d(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t n,
    int64_t p, const uint16_t *__restrict__ wp, int64_t mpad, int64_t kpad, int64_t n_it,
    int64_t n_items, const int64_t *__restrict__ csr_ptr, const int32_t *__restrict__ csr_col,
    const float *__restrict__ csr_val) {
    constexpr int NW = 2 * WN;                             // waves
    constexpr int BN = 64 * WN;                            // columns per block tile
    constexpr int BM = 64 * TM;                            // rows per block tile
    constexpr int ABUF = 3 * BM * 2;                       // 16-B W pieces per K-step (A buffer)
    constexpr int NDMA = ABUF / 64;                        // wave-level DMAs per K-step
    static_assert(NDMA % NW == 0, "DMAs per wave");
    constexpr int DPW = NDMA / NW;                         // DMAs per wave per K-step
    static_assert(NA == 2 || NA == 3, "A ring depth");
    static_assert(XD == 2 || (XD == 3 && NA == 2), "X prefetch distance (3: with a 2-deep W ring)");
    extern __shared__ uint4 lds_b6[];
    auto A_at = [&](int b, int pl, int row, int hf) -> uint4 & {
        return lds_b6[((b * 3 + pl) * BM + row) * 2 + hf];
    };
    auto B_at = [&](int b, int pl, int col, int hf) -> uint4 & {
        return lds_b6[NA * ABUF + ((b * 3 + pl) * BN + col) * 2 + hf];
    };
    const int tid = threadIdx.x;
    const int wave = wave_id();
    const int lane = tid & 63;
    const int wm = wave / WN, wn = wave % WN;
    const int bj = tid % BN, bh = tid / BN;                // X loader: column, k half
    const int hl = lane >> 5;
    const int64_t S = kpad / kB6K;
    const int64_t plane_el = mpad * kpad;
    // this lane's piece of each of its wave's DMAs: LDS slot q = 64 j + lane of the A buffer holds
    // plane pl, row, stored half hs; the piece there is W half hf = hs ^ (row >> 3 & 1)
    uint32_t wrel[DPW];
#pragma unroll
    for (int u = 0; u < DPW; ++u) {
        const int q = 64 * (wave + NW * u) + lane;
        const int pl = q / (2 * BM), rem = q % (2 * BM);
        const int row = rem >> 1, hf = (rem & 1) ^ ((row >> 3) & 1);
        wrel[u] = (uint32_t)((((int64_t)pl * mpad + row) * kpad + 8 * hf) * 2);
    }
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint16_t *>(wp), (short)0, (int)(3 * plane_el * 2), 0x00020000);
    const uint32_t rowb = (uint32_t)ld_x * 4u;
    const int bhu = __builtin_amdgcn_readfirstlane(bh);
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int64_t jt = (local / n_it) * 8 + xcd;
        const int64_t it = local % n_it;
        const int64_t i0 = it * BM, j0 = jt * BN;
        if (j0 >= p) continue;                             // block-uniform
        floatx16 acc[TM][2];
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int b = 0; b < 2; ++b)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
        const int64_t jx = j0 + bj;
        const uint32_t xvoff = jx < p ? (uint32_t)jx * 4u : 0x80000000u;
        uint32_t wvoff[DPW];
#pragma unroll
        for (int u = 0; u < DPW; ++u) wvoff[u] = wrel[u] + (uint32_t)(i0 * kpad * 2);
        float xv0[8], xv1[8], xv2[8];
        // W pieces of K-step S_ (clamped) into A buffer AB_ by this wave's DPW DMAs
#define B6D_WDMA(AB_, S_)                                                                          \
        do {                                                                                       \
            const int64_t k0_ = ((S_) < S ? (S_) : S - 1) * kB6K;                                 \
            _Pragma("unroll") for (int u = 0; u < DPW; ++u)                                        \
                b6d_dma16(wrs, lds_b6 + (AB_) * ABUF + 64 * (wave + NW * u), wvoff[u],             \
                          (int)(k0_ * 2));                                                         \
        } while (0)
#define B6D_XFETCH(SET, S_)                                                                        \
        do {                                                                                       \
            const int64_t k0_ = ((S_) < S ? (S_) : S - 1) * kB6K;                                 \
            const int64_t ext_ = (n - k0_) * (int64_t)rowb;                                        \
            const __amdgpu_buffer_rsrc_t xr_ = __builtin_amdgcn_make_buffer_rsrc(                  \
                const_cast<float *>(x + k0_ * ld_x), (short)0,                                     \
                (int)(ext_ < 0x7fffffffLL ? ext_ : 0x7fffffffLL), 0x00020000);                     \
            _Pragma("unroll") for (int u = 0; u < 8; ++u)                                          \
                xv##SET[u] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(       \
                                 xr_, xvoff, (int)((8 * bhu + u) * rowb), 0));                     \
        } while (0)
        // the planes go to LDS by inline-asm ds_write_b128: hipcc, which cannot tell them from
        // the W ring's LDS-DMA destinations, would otherwise wait for the DMA of step s + NA - 1
        // (vmcnt) before each write; the barrier's explicit lgkmcnt(0) covers them
        typedef unsigned b6d_u32x4 __attribute__((ext_vector_type(4)));
        const uint32_t bst = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint4 *)lds_b6) +
                             (uint32_t)(NA * ABUF + bj * 2 + (bh ^ ((bj >> 3) & 1))) * 16u;
#define B6D_XSTASH(SET, BUF)                                                                       \
        do {                                                                                       \
            uint32_t h_[4], m_[4], l_[4];                                                          \
            _Pragma("unroll") for (int u = 0; u < 4; ++u)                                          \
                split3_pair(xv##SET[2 * u], xv##SET[2 * u + 1], h_[u], m_[u], l_[u]);              \
            const b6d_u32x4 hv_ = {h_[0], h_[1], h_[2], h_[3]}, mv_ = {m_[0], m_[1], m_[2], m_[3]}, \
                            lv_ = {l_[0], l_[1], l_[2], l_[3]};                                    \
            asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(bst), "v"(hv_),                   \
                         "n"(((BUF) * 3 + 0) * BN * 32) : "memory");                               \
            asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(bst), "v"(mv_),                   \
                         "n"(((BUF) * 3 + 1) * BN * 32) : "memory");                               \
            asm volatile("ds_write_b128 %0, %1 offset:%2" ::"v"(bst), "v"(lv_),                   \
                         "n"(((BUF) * 3 + 2) * BN * 32) : "memory");                               \
        } while (0)
        // the barrier: this wave's DMA of the next K-step has landed (everything issued after it --
        // the X loads of step s + XD, and with NA 3 the DMA of step s + 2 -- may stay in flight),
        // and its LDS reads and writes are done
#define B6D_VMAFTER (NA == 3 ? DPW + 8 : 8)
#define B6D_BARRIER()                                                                              \
        asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(B6D_VMAFTER) : "memory")
        // K-step s: A buffer AB (runtime ring index), B buffer B; the W DMA of s + NA - 1 into
        // ring slot AN and the X fetch of s + XD into register set XL first, then the operand
        // reads, the MFMAs, the split of s + 1 (register set XS) into B buffer NB, the barrier
#define B6D_STEP(B, NB, XL, XS, S_, AB, AN)                                                        \
        do {                                                                                       \
            B6D_WDMA(AN, (S_) + NA - 1);                                                           \
            __builtin_amdgcn_sched_barrier(0);                                                     \
            B6D_XFETCH(XL, (S_) + XD);                                                             \
            __builtin_amdgcn_sched_barrier(0);                                                     \
            bf16x8v af_[TM][3], bf_[2][3];                                                          \
            _Pragma("unroll") for (int o = 0; o < 3; ++o) {                                        \
                const int pa_ = o == 0 ? 1 : o == 1 ? 2 : 0, pb_ = o == 0 ? 1 : o == 1 ? 0 : 2;    \
                _Pragma("unroll") for (int a = 0; a < TM; ++a) {                                   \
                    const int row_ = wm * 32 * TM + a * 32 + (lane & 31);                          \
                    af_[a][pa_] = __builtin_bit_cast(bf16x8v, A_at(AB, pa_, row_, hl ^ ((row_ >> 3) & 1))); \
                }                                                                                  \
                _Pragma("unroll") for (int c = 0; c < 2; ++c) {                                    \
                    const int col_ = wn * 64 + c * 32 + (lane & 31);                               \
                    bf_[c][pb_] = __builtin_bit_cast(bf16x8v, B_at(B, pb_, col_, hl ^ ((col_ >> 3) & 1))); \
                }                                                                                  \
            }                                                                                      \
            _Pragma("unroll") for (int e = 0; e < 6; ++e)                                          \
                _Pragma("unroll") for (int a = 0; a < TM; ++a)                                     \
                    _Pragma("unroll") for (int c = 0; c < 2; ++c)                                  \
                        acc[a][c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(                       \
                            af_[a][kB6PA[e]], bf_[c][kB6PB[e]], acc[a][c], 0, 0, 0);               \
            B6D_XSTASH(XS, NB);                                                                    \
            B6D_BARRIER();                                                                         \
        } while (0)
        // prologue: W of steps 0 .. NA - 2, X of steps 0 .. XD - 1, X 0 split into B buffer 0
#pragma unroll
        for (int a = 0; a < NA - 1; ++a) B6D_WDMA(a, a);
        __builtin_amdgcn_sched_barrier(0);
        B6D_XFETCH(0, 0);
        B6D_XFETCH(1, 1);
        if (XD == 3) B6D_XFETCH(2, 2);
        __builtin_amdgcn_sched_barrier(0);
        B6D_XSTASH(0, 0);
        if (XD == 3) asm volatile("s_waitcnt vmcnt(16) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        else asm volatile("s_waitcnt vmcnt(8) lgkmcnt(0)\n\ts_barrier" ::: "memory");
        int ab = 0;                                        // ring slot of step s
        int64_t s = 0;
        if constexpr (XD == 2) {
            for (; s + 1 < S; s += 2) {
                const int a1 = ab + 1 == NA ? 0 : ab + 1;
                const int an0 = ab + NA - 1 >= NA ? ab - 1 : ab + NA - 1;   // (s + NA - 1) % NA
                const int an1 = an0 + 1 == NA ? 0 : an0 + 1;
                B6D_STEP(0, 1, 0, 1, s, ab, an0);
                B6D_STEP(1, 0, 1, 0, s + 1, a1, an1);
                ab = a1 + 1 == NA ? 0 : a1 + 1;
            }
            if (s < S) {
                const int an0 = ab + NA - 1 >= NA ? ab - 1 : ab + NA - 1;
                B6D_STEP(0, 1, 0, 1, s, ab, an0);
            }
        } else {
            // three X register sets (set of step k: k % 3) and two B buffers: six steps per
            // iteration, the rest peeled one by one (NA 2: ring slot k % 2 = B buffer parity)
            for (; s + 5 < S; s += 6) {
                B6D_STEP(0, 1, 0, 1, s, 0, 1);
                B6D_STEP(1, 0, 1, 2, s + 1, 1, 0);
                B6D_STEP(0, 1, 2, 0, s + 2, 0, 1);
                B6D_STEP(1, 0, 0, 1, s + 3, 1, 0);
                B6D_STEP(0, 1, 1, 2, s + 4, 0, 1);
                B6D_STEP(1, 0, 2, 0, s + 5, 1, 0);
            }
            if (s < S) B6D_STEP(0, 1, 0, 1, s, 0, 1);
            if (s + 1 < S) B6D_STEP(1, 0, 1, 2, s + 1, 1, 0);
            if (s + 2 < S) B6D_STEP(0, 1, 2, 0, s + 2, 0, 1);
            if (s + 3 < S) B6D_STEP(1, 0, 0, 1, s + 3, 1, 0);
            if (s + 4 < S) B6D_STEP(0, 1, 1, 2, s + 4, 0, 1);
        }
#undef B6D_STEP
#undef B6D_BARRIER
#undef B6D_VMAFTER
#undef B6D_XSTASH
#undef B6D_XFETCH
#undef B6D_WDMA
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the clamped refetches past the end
        uint64_t bad[2] = {0, 0};                          // this lane's non-finite outputs
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int64_t i = i0 + wm * 32 * TM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                    const int64_t j = j0 + wn * 64 + c * 32 + (lane & 31);
                    if (i < n && j < p) {
                        if (__builtin_isfinite(acc[a][c][r])) __builtin_nontemporal_store(acc[a][c][r], y + i * ld_y + j);
                        else bad[a >> 1] |= 1ull << ((a & 1) * 32 + c * 16 + r);
                    }
                }
#pragma unroll
        for (int h = 0; h < 2; ++h)
            while (bad[h]) {                               // non-finite guard (csr_refix1)
                const int q = __builtin_ctzll(bad[h]);
                bad[h] &= bad[h] - 1;
                const int a = 2 * h + (q >> 5), c = (q >> 4) & 1, r = q & 15;
                const int64_t i = i0 + wm * 32 * TM + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
                const int64_t j = j0 + wn * 64 + c * 32 + (lane & 31);
                __builtin_nontemporal_store(csr_refix1(x + j, ld_x, i, csr_ptr, csr_col, csr_val), y + i * ld_y + j);
            }
        __syncthreads();   // LDS buffers are rewritten by the next item's prologue
    }
}

// ----------------------------------------------------------------------------------------------
// Clique-factored mixing for BIG cliques (> 256 members, e.g. a fully-connected topology with MH
// weights = one clique: W = a*I + c*11^T).  Work item = (clique, 64 columns), WAVES waves, lane =
// one column.  Pass 1 streams the members (wave w: a contiguous 1/WAVES of them) into per-group
// sums, an LDS reduction combines the waves; pass 2 streams the members again and writes
// y = a x + sum_g c_g S_g (+ residual terms).  The pass-2 re-read (M x 256 B per item) is served
// by L2 / the Infinity Cache for the most part.  Pass 2 is software-pipelined: the next U rows
// are loaded before this batch's U stores, because vmcnt counts stores too on CDNA (a load issued
// after a store would make its wait drain the store).
template <int G, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_mix_bigclique(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t p,
    int32_t n_cliques, const int32_t *__restrict__ clique_ptr,
    const int32_t *__restrict__ member_row, const int32_t *__restrict__ member_group,
    const float *__restrict__ coef, const int32_t *__restrict__ res_ptr,
    const int32_t *__restrict__ res_col, const float *__restrict__ res_val, int64_t n_items,
    const int64_t *__restrict__ csr_ptr, const int32_t *__restrict__ csr_col,
    const float *__restrict__ csr_val) {
    constexpr int U = 8;
    __shared__ float red[G][WAVES][kWave];
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int64_t chunk = (local / n_cliques) * 8 + xcd;
        const int32_t cq = (int32_t)(local % n_cliques);
        const int64_t c0 = chunk * kWave;
        if (c0 >= p) continue;                               // block-uniform
        const bool act = c0 + lane < p;
        const unsigned lo = act ? (unsigned)lane : 0u;
        const float *xc = x + c0;
        float *yc = y + c0;
        const int32_t m0 = clique_ptr[cq];
        const int32_t M = clique_ptr[cq + 1] - m0;
        const int32_t per = (M + WAVES - 1) / WAVES;
        const int32_t kb = m0 + (wave * per < M ? wave * per : M);
        const int32_t ke = m0 + ((wave + 1) * per < M ? (wave + 1) * per : M);
        float s[G];
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] = 0.f;
        for (int32_t k = kb; k < ke; k += U) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                v[u] = xc[(int64_t)member_row[k + u < ke ? k + u : kb] * ld_x + lo];
#pragma unroll
            for (int u = 0; u < U; ++u)
                if (k + u < ke) {
                    const int gr = member_group[k + u] & kMemberGroupMask;
#pragma unroll
                    for (int g = 0; g < G; ++g) s[g] += gr == g ? v[u] : 0.f;
                }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) red[g][wave][lane] = s[g];
        __syncthreads();
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float a = 0.f;
#pragma unroll
            for (int w = 0; w < WAVES; ++w) a += red[g][w][lane];
            s[g] = a;
        }
        __syncthreads();                                      // red[] is rewritten by the next item
        if (kb < ke) {
            float v[U];
#pragma unroll
            for (int u = 0; u < U; ++u)
                v[u] = xc[(int64_t)member_row[kb + u < ke ? kb + u : kb] * ld_x + lo];
            for (int32_t k = kb; k < ke; k += U) {
                // own terms and residual gathers of this batch (loads, before any store of it)
                float o[U];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int32_t m = k + u < ke ? k + u : kb;
                    const float *cf = coef + (int64_t)m * (1 + G);
                    o[u] = cf[0] * v[u];
#pragma unroll
                    for (int g = 0; g < G; ++g) o[u] = __builtin_fmaf(cf[1 + g], s[g], o[u]);
                    if (k + u < ke)
                        for (int32_t q = res_ptr[m]; q < res_ptr[m + 1]; ++q)
                            o[u] = __builtin_fmaf(res_val[q], xc[(int64_t)res_col[q] * ld_x + lo], o[u]);
                }
                // next batch's rows in flight before this batch's stores
                const int32_t kn = k + U;
#pragma unroll
                for (int u = 0; u < U; ++u)
                    v[u] = kn < ke ? xc[(int64_t)member_row[kn + u < ke ? kn + u : kn] * ld_x + lo] : 0.f;
                uint32_t bad = 0;
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (k + u < ke && act) {
                        if (__builtin_isfinite(o[u]))
                            __builtin_nontemporal_store(o[u], yc + (int64_t)member_row[k + u] * ld_y + lane);
                        else bad |= 1u << u;
                    }
                while (bad) {                                 // non-finite guard (see csr_refix)
                    const int u = __builtin_ctz(bad);
                    bad &= bad - 1;
                    const int64_t row = member_row[k + u];
                    __builtin_nontemporal_store(csr_refix1(xc + lo, ld_x, row, csr_ptr, csr_col, csr_val),
                                                yc + row * ld_y + lane);
                }
            }
        }
    }
}

// (the item geometry shared by k_mix_bigclique_v4 and k_mix_bigclique_reg below)
constexpr int kBigRegWaves = 16;
constexpr int kBigRegCols = 32;
// float4 lanes (round 6; launch_bigclique_reg picks it): the same item (clique, 32 columns) with
// lane = (row r8 = lane >> 3, column quad q = lane & 7), so one wave-instruction loads / stores 8
// member rows x 128 B = 1 KiB (k_mix_bigclique_reg: 2 rows x 128 B of 4-B lanes); wave w holds
// members 8 (8 w + i) + r8, i < 8 (<= 1024 members).  Group sums: three xor-shuffles over r8, then
// the 16 waves through LDS.  Same per-element arithmetic as k_mix_bigclique_reg (a x, then one fma
// per group, then the residual fmas); the column sums are added in another order (fast mode).
// Needs p % 4 == 0, ld % 4 == 0, 16-B aligned slabs, and column-blocked slabs whose blocks span
// < 4 GiB (32-bit row offsets, as k_mix_clique_q's OFF32).
template <int G, int OCC>
__global__ __launch_bounds__(kBigRegWaves * 64) __attribute__((amdgpu_waves_per_eu(OCC))) void k_mix_bigclique_v4(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t p,
    int32_t n_cliques, const int32_t *__restrict__ clique_ptr,
    const int32_t *__restrict__ member_row, const int32_t *__restrict__ member_group,
    const float *__restrict__ coef, const int32_t *__restrict__ res_ptr,
    const int32_t *__restrict__ res_col, const float *__restrict__ res_val, int64_t nch8,
    int bc_shift, int64_t bs_x, int64_t bs_y, int contig, const int64_t *__restrict__ csr_ptr,
    const int32_t *__restrict__ csr_col, const float *__restrict__ csr_val) {
    typedef float f4v __attribute__((ext_vector_type(4)));
    constexpr int RI = 8;                                     // rows per lane
    constexpr int MMAX = kBigRegWaves * 8 * RI;               // 1024
    __shared__ int32_t s_row[MMAX];
    __shared__ int32_t s_grp[MMAX];
    __shared__ int32_t s_res[MMAX + 1];
    __shared__ float s_cf[MMAX * (1 + G)];
    __shared__ f4v red[G][kBigRegWaves][8];
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    const int r8 = lane >> 3, q = lane & 7;
    const int64_t n_items = (int64_t)n_cliques * nch8 * 8;
    int32_t cur = -1, m0 = 0, M = 0;
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int32_t cq = (int32_t)(local / nch8);
        const int64_t chunk = contig ? xcd * nch8 + local % nch8 : (local % nch8) * 8 + xcd;
        const int64_t c0 = chunk * kBigRegCols;
        if (c0 >= p) continue;                               // block-uniform
        if (cq != cur) {                                     // block-uniform
            __syncthreads();                                 // previous item done with s_*
            cur = cq;
            m0 = clique_ptr[cq];
            M = clique_ptr[cq + 1] - m0;
            for (int k = threadIdx.x; k < M; k += blockDim.x) {
                s_row[k] = member_row[m0 + k];
                s_grp[k] = member_group[m0 + k] & kMemberGroupMask;
#pragma unroll
                for (int g = 0; g <= G; ++g) s_cf[k * (1 + G) + g] = coef[(int64_t)(m0 + k) * (1 + G) + g];
            }
            for (int k = threadIdx.x; k <= M; k += blockDim.x) s_res[k] = res_ptr[m0 + k];
            __syncthreads();
        }
        const bool act = c0 + 4 * q < p;                      // p % 4 == 0: a quad is all in or out
        const unsigned lo = act ? (unsigned)(4 * q) : 0u;
        const int64_t cin = c0 & (((int64_t)1 << bc_shift) - 1);
        // column-blocked slabs only: the item's block base (wave-uniform) + a 32-bit row offset
        const float *xb = x + (c0 >> bc_shift) * bs_x + cin;
        float *yb = y + (c0 >> bc_shift) * bs_y + cin;
        const float *xc = xb + lo;
        f4v v[RI];
#pragma unroll
        for (int i = 0; i < RI; ++i) {
            const int k = 8 * (wave * RI + i) + r8;
            v[i] = k < M ? __builtin_nontemporal_load(reinterpret_cast<const f4v *>(qrow<true>(xb, s_row[k], ld_x, lo)))
                         : f4v{0.f, 0.f, 0.f, 0.f};
        }
        f4v s[G];
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < RI; ++i) {
            if (G == 1) {
                s[0] += v[i];                                // rows past M hold 0
            } else {
                const int k = 8 * (wave * RI + i) + r8;
                const int gr = k < M ? s_grp[k] : -1;
#pragma unroll
                for (int g = 0; g < G; ++g) s[g] += gr == g ? v[i] : f4v{0.f, 0.f, 0.f, 0.f};
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
#pragma unroll
            for (int m = 8; m < kWave; m <<= 1)
#pragma unroll
                for (int e = 0; e < 4; ++e) s[g][e] += __shfl_xor(s[g][e], m);
            if (r8 == 0) red[g][wave][q] = s[g];
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < G; ++g) {
            f4v a = red[g][0][q];
#pragma unroll
            for (int w = 1; w < kBigRegWaves; ++w) a += red[g][w][q];
            s[g] = a;
        }
        __syncthreads();                                      // red[] is rewritten by the next item
#pragma unroll
        for (int i = 0; i < RI; ++i) {
            const int k = 8 * (wave * RI + i) + r8;
            const float *cf = s_cf + (k < M ? k : 0) * (1 + G);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                float o = cf[0] * v[i][e];
#pragma unroll
                for (int g = 0; g < G; ++g) o = __builtin_fmaf(cf[1 + g], s[g][e], o);
                v[i][e] = o;
            }
        }
        if (s_res[M] > s_res[0]) {                            // block-uniform: any gateway edges
#pragma unroll
            for (int i = 0; i < RI; ++i) {
                const int k = 8 * (wave * RI + i) + r8;
                if (k < M)
                    for (int32_t qq = s_res[k]; qq < s_res[k + 1]; ++qq) {
                        const f4v xr = *reinterpret_cast<const f4v *>(qrow<true>(xb, res_col[qq], ld_x, lo));
                        const float w = res_val[qq];
#pragma unroll
                        for (int e = 0; e < 4; ++e) v[i][e] = __builtin_fmaf(w, xr[e], v[i][e]);
                    }
            }
        }
        uint32_t bad = 0;                                     // this lane's rows with a non-finite output
#pragma unroll
        for (int i = 0; i < RI; ++i) {
            const int k = 8 * (wave * RI + i) + r8;
            if (k < M && act) {
                const int rowk = s_row[k];
                if (__builtin_isfinite(v[i][0]) && __builtin_isfinite(v[i][1]) &&
                    __builtin_isfinite(v[i][2]) && __builtin_isfinite(v[i][3]))
                    __builtin_nontemporal_store(v[i], reinterpret_cast<f4v *>(const_cast<float *>(qrow<true>(yb, rowk, ld_y, 4 * q))));
                else bad |= 1u << i;
            }
        }
        // non-finite guard (see csr_refix): the row's four outputs recomputed from its CSR row
        // (v[i] is not read: indexed by a runtime i it would put v in scratch memory)
        while (bad) {
            const int i = __builtin_ctz(bad);
            bad &= bad - 1;
            const int64_t row = s_row[8 * (wave * RI + i) + r8];
#pragma unroll 1
            for (int e = 0; e < 4; ++e)
                __builtin_nontemporal_store(csr_refix1(xc + e, ld_x, row, csr_ptr, csr_col, csr_val),
                                            yb + row * ld_y + 4 * q + e);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// One-pass big-clique mixing, register-resident (257..32*R members).  Work item = (clique, 32
// columns = 128 B of every member row); a block of 16 waves holds the whole item in VGPRs: lane =
// (half h, column lc), wave w holds members 2*(w*R + i) + h, i < R.  All R row loads of a lane
// issue back to back, the per-group column sums are reduced over the half-waves (swizzle) and the
// 16 waves (LDS), and the outputs y = a x + sum_g c_g S_g (+ residual terms) are computed from the
// registers -- each member row is read from HBM ONCE (the two-pass kernel reads it twice).  The
// clique's metadata (rows, coefficients, residual ranges) is staged in LDS and re-staged only when
// a block's clique changes: items are clique-major, so a grid-stride block stays on one clique.
template <int G, int R, int OCC>
__global__ __launch_bounds__(kBigRegWaves * 64) __attribute__((amdgpu_waves_per_eu(OCC))) void k_mix_bigclique_reg(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t p,
    int32_t n_cliques, const int32_t *__restrict__ clique_ptr,
    const int32_t *__restrict__ member_row, const int32_t *__restrict__ member_group,
    const float *__restrict__ coef, const int32_t *__restrict__ res_ptr,
    const int32_t *__restrict__ res_col, const float *__restrict__ res_val, int64_t nch8,
    int bc_shift, int64_t bs_x, int64_t bs_y, int contig, const int64_t *__restrict__ csr_ptr,
    const int32_t *__restrict__ csr_col, const float *__restrict__ csr_val) {
    // column c of row r: x[(c >> bc_shift) * bs_x + r * ld_x + (c & (2^bc_shift - 1))] -- the
    // column-blocked layout [P / B, N, B] (ld = B), or row-major with bc_shift = 62, bs = 0
    constexpr int MMAX = kBigRegWaves * 2 * R;
    __shared__ int32_t s_row[MMAX];
    __shared__ int32_t s_grp[MMAX];
    __shared__ int32_t s_res[MMAX + 1];
    __shared__ float s_cf[MMAX * (1 + G)];
    __shared__ float red[G][kBigRegWaves][kBigRegCols];
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    const int h = lane >> 5, lc = lane & (kBigRegCols - 1);
    const int64_t n_items = (int64_t)n_cliques * nch8 * 8;
    int32_t cur = -1, m0 = 0, M = 0;
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int32_t cq = (int32_t)(local / nch8);
        // contig: XCD x owns chunks [x*nch8, (x+1)*nch8), so the items one XCD runs together read
        // neighbouring 128-B pieces of the same rows; else chunks interleave over the XCDs
        const int64_t chunk = contig ? xcd * nch8 + local % nch8 : (local % nch8) * 8 + xcd;
        const int64_t c0 = chunk * kBigRegCols;
        if (c0 >= p) continue;                               // block-uniform
        if (cq != cur) {                                     // block-uniform
            __syncthreads();                                 // previous item done with s_*
            cur = cq;
            m0 = clique_ptr[cq];
            M = clique_ptr[cq + 1] - m0;
            for (int k = threadIdx.x; k < M; k += blockDim.x) {
                s_row[k] = member_row[m0 + k];
                s_grp[k] = member_group[m0 + k] & kMemberGroupMask;
#pragma unroll
                for (int g = 0; g <= G; ++g) s_cf[k * (1 + G) + g] = coef[(int64_t)(m0 + k) * (1 + G) + g];
            }
            for (int k = threadIdx.x; k <= M; k += blockDim.x) s_res[k] = res_ptr[m0 + k];
            __syncthreads();
        }
        const bool act = c0 + lc < p;
        const unsigned lo = act ? (unsigned)lc : 0u;
        const int64_t cin = c0 & (((int64_t)1 << bc_shift) - 1);
        const float *xc = x + (c0 >> bc_shift) * bs_x + cin + lo;
        float *yc = y + (c0 >> bc_shift) * bs_y + cin + lc;
        float v[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int k = 2 * (wave * R + i) + h;
            v[i] = k < M ? __builtin_nontemporal_load(xc + (int64_t)s_row[k] * ld_x) : 0.f;
        }
        float s[G];
#pragma unroll
        for (int g = 0; g < G; ++g) s[g] = 0.f;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            if (G == 1) {
                s[0] += v[i];                                // rows past M hold 0
            } else {
                const int k = 2 * (wave * R + i) + h;
                const int gr = k < M ? s_grp[k] : -1;
#pragma unroll
                for (int g = 0; g < G; ++g) s[g] += gr == g ? v[i] : 0.f;
            }
        }
#pragma unroll
        for (int g = 0; g < G; ++g) {
            s[g] += __shfl_xor(s[g], 32);
            if (h == 0) red[g][wave][lc] = s[g];
        }
        __syncthreads();
#pragma unroll
        for (int g = 0; g < G; ++g) {
            float a = 0.f;
#pragma unroll
            for (int w = 0; w < kBigRegWaves; ++w) a += red[g][w][lc];
            s[g] = a;
        }
        __syncthreads();                                      // red[] is rewritten by the next item
        // outputs in place, residual (gateway) gathers all before the first store: a load between
        // two stores would make its wait drain the earlier stores (vmcnt counts stores on CDNA)
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int k = 2 * (wave * R + i) + h;
            const float *cf = s_cf + (k < M ? k : 0) * (1 + G);
            float o = cf[0] * v[i];
#pragma unroll
            for (int g = 0; g < G; ++g) o = __builtin_fmaf(cf[1 + g], s[g], o);
            v[i] = o;
        }
        if (s_res[M] > s_res[0]) {                            // block-uniform: any gateway edges
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const int k = 2 * (wave * R + i) + h;
                if (k < M)
                    for (int32_t q = s_res[k]; q < s_res[k + 1]; ++q)
                        v[i] = __builtin_fmaf(res_val[q], xc[(int64_t)res_col[q] * ld_x], v[i]);
            }
        }
        uint32_t bad = 0;                                     // this lane's non-finite outputs
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int k = 2 * (wave * R + i) + h;
            if (k < M && act) {
                if (__builtin_isfinite(v[i])) __builtin_nontemporal_store(v[i], yc + (int64_t)s_row[k] * ld_y);
                else bad |= 1u << i;
            }
        }
        while (bad) {                                         // non-finite guard (see csr_refix)
            const int i = __builtin_ctz(bad);
            bad &= bad - 1;
            const int64_t row = s_row[2 * (wave * R + i) + h];
            __builtin_nontemporal_store(csr_refix1(xc, ld_x, row, csr_ptr, csr_col, csr_val),
                                        yc + row * ld_y);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// Merged-order row tiles (exact and fast).  The exact rule fixes every row's operand order (self,
// then edges[rank] in list order), so rows cannot share partial sums — but they can share LOADS.
// A tile is RT output rows (e.g. part of a clique) whose entry lists (self excluded) are all
// subsequences of one merged position list (host: niidmix.tile, majority merge; a source that the
// rows order differently appears more than once).  One wave owns (tile, column chunk) and holds
// the RT rows' accumulators in registers; per position it loads the source row's columns ONCE and
// applies them to every tile row that takes the position (mask bit), each row still in its own
// list order, so exact mode stays bit-identical to k_mix_csr.  Work per position is RT*NE
// mul+add per lane for one NE-column load: VALU-bound, not gather-bound.  Weights come in by
// scalar loads (uniform per position), the source row / mask lane-parallel by v_readlane.  A
// position every row takes (mask == FULL) skips the per-row select.
typedef float f2 __attribute__((ext_vector_type(2)));

// Packed (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32) forms of axpy on 2 columns.  Per component
// these are the same IEEE roundings as the scalar forms (exact: fl(acc + fl(w*x)), no contraction).
template <bool EXACT>
__device__ __forceinline__ f2 axpy2(float w, f2 xv, f2 acc) {
    if constexpr (EXACT) {
        const f2 t = xv * w;
        return acc + t;
    } else {
        return __builtin_elementwise_fma((f2){w, w}, xv, acc);
    }
}

// Position flag in pos_src (bit 30, NIIDMIX_TILE_POS_UNIFORM): every tile row's weight for this
// position is the same fp32 value (pos_w[pos*RT + r] == pos_w[pos*RT] for all r).  Exact mode then
// forms the product fl(w*x) ONCE and adds it to each taking row — the same bits as per-row products
// — so a position costs NE/2 packed muls + (rows taking it)*NE/2 packed adds per lane.
constexpr int kPosUniform = 1 << 30;
constexpr int kPosRowMask = kPosUniform - 1;

template <bool EXACT, int VW, int NE, int RT>
__global__ __launch_bounds__(256) void k_mix_tile(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t p,
    int64_t n_sub, const int64_t *__restrict__ sub_ptr, const int32_t *__restrict__ sub_rows,
    const float *__restrict__ sub_wself, const int32_t *__restrict__ pos_src,
    const uint32_t *__restrict__ pos_mask, const float *__restrict__ pos_w,
    int64_t n_sub_groups, int64_t n_items, int avg_only) {
    constexpr int S = NE / VW;                  // slots per lane
    constexpr int NH = NE / 2;                  // packed column pairs per lane
    constexpr int64_t CW = 64 * NE;             // columns per work item
    constexpr uint32_t FULL = (uint32_t)((1ull << RT) - 1ull);
    constexpr int D = 4;                        // positions whose loads are in flight together
    static_assert(NE % 2 == 0, "NE must be even (packed pairs)");
    const int wave = wave_id();
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t t = blockIdx.x; t < n_items; t += gridDim.x) {
        const int64_t xcd = t & 7;
        const int64_t local = t >> 3;
        const int64_t chunk = (local / n_sub_groups) * 8 + xcd;
        const int64_t sub = (local % n_sub_groups) * 4 + wave;
        const int64_t c0 = chunk * CW;
        if (sub >= n_sub || c0 >= p) continue;  // wave-uniform
        int64_t cs[S];
        bool ok[S];
#pragma unroll
        for (int q = 0; q < S; ++q) {
            const int64_t cq = c0 + VW * lane + 64 * VW * q;
            ok[q] = cq < p;
            cs[q] = ok[q] ? cq : c0;
        }
        const int li = lane < RT ? lane : RT - 1;
        const int d_row = sub_rows[sub * RT + li];
        const float d_ws = sub_wself[sub * RT + li];
        f2 acc[RT][NH];
        // first entry of every row: the node itself (acc = x*0; acc += w_self*x)
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            const int row = __builtin_amdgcn_readlane(d_row, r);
            const float *src = x + (int64_t)(row < 0 ? 0 : row) * ld_x;
            float xs[NE];
#pragma unroll
            for (int q = 0; q < S; ++q) ldv<VW>(src + cs[q], xs + q * VW);
            const float ws = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d_ws), r));
#pragma unroll
            for (int h = 0; h < NH; ++h) {
                const f2 xx = {xs[2 * h], xs[2 * h + 1]};
                acc[r][h] = axpy2<EXACT>(ws, xx, xx * 0.f);
            }
        }
        const int64_t beg = sub_ptr[sub], end = sub_ptr[sub + 1];
        for (int64_t kb = beg; kb < end; kb += 64) {
            const int cnt = (int)(end - kb < 64 ? end - kb : 64);
            const int lj = lane < cnt ? lane : cnt - 1;
            const int d_src = pos_src[kb + lj];
            const int d_mask = (int)pos_mask[kb + lj];
            for (int j = 0; j < cnt; j += D) {
                float xv[D][NE];
#pragma unroll
                for (int u = 0; u < D; ++u) {
                    const int jj = j + u < cnt ? j + u : cnt - 1;     // clamped: loads unconditional
                    const int srow = __builtin_amdgcn_readlane(d_src, jj) & kPosRowMask;
                    const float *src = x + (int64_t)srow * ld_x;
#pragma unroll
                    for (int q = 0; q < S; ++q) ldv<VW>(src + cs[q], xv[u] + q * VW);
                }
#pragma unroll
                for (int u = 0; u < D; ++u) {
                    if (j + u >= cnt) break;
                    const uint32_t m = (uint32_t)__builtin_amdgcn_readlane(d_mask, j + u);
                    const bool uni = (__builtin_amdgcn_readlane(d_src, j + u) & kPosUniform) != 0;
                    const float *wp = pos_w + (kb + j + u) * RT;
                    f2 xx[NH];
#pragma unroll
                    for (int h = 0; h < NH; ++h) xx[h] = (f2){xv[u][2 * h], xv[u][2 * h + 1]};
                    if (EXACT && uni) {
                        const float w = wp[0];
                        f2 tp[NH];
#pragma unroll
                        for (int h = 0; h < NH; ++h) tp[h] = xx[h] * w;
                        if (m == FULL) {
#pragma unroll
                            for (int r = 0; r < RT; ++r)
#pragma unroll
                                for (int h = 0; h < NH; ++h) acc[r][h] = acc[r][h] + tp[h];
                        } else {
#pragma unroll
                            for (int r = 0; r < RT; ++r)
                                if ((m >> r) & 1u) {                       // wave-uniform
#pragma unroll
                                    for (int h = 0; h < NH; ++h) acc[r][h] = acc[r][h] + tp[h];
                                }
                        }
                    } else if (m == FULL) {
#pragma unroll
                        for (int r = 0; r < RT; ++r) {
                            const float w = wp[r];
#pragma unroll
                            for (int h = 0; h < NH; ++h) acc[r][h] = axpy2<EXACT>(w, xx[h], acc[r][h]);
                        }
                    } else {
#pragma unroll
                        for (int r = 0; r < RT; ++r)
                            if ((m >> r) & 1u) {                           // wave-uniform
                                const float w = wp[r];
#pragma unroll
                                for (int h = 0; h < NH; ++h) acc[r][h] = axpy2<EXACT>(w, xx[h], acc[r][h]);
                            }
                    }
                }
            }
        }
        // update_models: z + acc with z = x_self*0 (the self rows are re-read: L2-resident, every
        // position load of the tile's clique touched them) — all RT re-reads are issued before the
        // first store, into the registers the position loads used, so the stores go out back to
        // back (vmcnt counts stores too on CDNA: a load between two stores would drain the first)
        if (!avg_only) {
#pragma unroll
            for (int r = 0; r < RT; ++r) {
                const int row = __builtin_amdgcn_readlane(d_row, r);
                float xs[NE];
#pragma unroll
                for (int q = 0; q < S; ++q) ldv<VW>(x + (int64_t)(row < 0 ? 0 : row) * ld_x + cs[q], xs + q * VW);
#pragma unroll
                for (int h = 0; h < NH; ++h) {
                    const f2 xx = {xs[2 * h], xs[2 * h + 1]};
                    acc[r][h] = xx * 0.f + acc[r][h];
                }
            }
        }
#pragma unroll
        for (int r = 0; r < RT; ++r) {
            const int row = __builtin_amdgcn_readlane(d_row, r);
            if (row < 0) continue;                                  // wave-uniform
            float *dst = y + (int64_t)row * ld_y;
            float o[NE];
#pragma unroll
            for (int h = 0; h < NH; ++h) { o[2 * h] = acc[r][h].x; o[2 * h + 1] = acc[r][h].y; }
#pragma unroll
            for (int q = 0; q < S; ++q)
                if (ok[q]) stv_nt<VW>(dst + cs[q], o + q * VW);
        }
    }
}

// ----------------------------------------------------------------------------------------------
// LDS-staged merged-order row tiles (exact and fast; the exact-mode default for clique graphs).
// Work item = (group, 128-column chunk); a group is a clique (its tiles, niidmix.tile).  The block
// first stages the chunk of every DISTINCT source row the group reads (its members + gateway rows of
// other cliques) in LDS — one HBM read per row — then each wave walks one tile's merged position
// list reading sources from LDS (ds_read_b64, no global-load latency in the loop) into RT packed
// accumulators per lane (2 columns per lane).  Exact: each row still applies its own entries in its
// own order with the reference's roundings; a POS_UNIFORM position forms fl(w*x) once.
// Work order is XCD-aware (the groups of one chunk run back to back on one XCD) so the gateway rows
// a group stages from other cliques are that XCD's L2 hits.
// A tile's RT accumulator pairs as register vectors of at most 16 pairs, so a row picked by a
// wave-uniform (SGPR) index is addressed through the GPR-index moves (s_set_gpr_idx_on + v_mov)
// instead of a select over every row (a 64-float vector would be indexed through scratch: RT 32
// keeps two halves and picks one by a uniform branch).
template <int RT>
struct TileAcc {
    static constexpr int H = RT < 16 ? RT : 16;
    typedef float V __attribute__((ext_vector_type(2 * H)));
    V v[RT / H];
    __device__ __forceinline__ f2 get(int r) const {
        if constexpr (RT <= 16) {
            return (f2){v[0][2 * r], v[0][2 * r + 1]};
        } else {
            if (r < H) return (f2){v[0][2 * r], v[0][2 * r + 1]};
            return (f2){v[1][2 * (r - H)], v[1][2 * (r - H) + 1]};
        }
    }
    // every row += t (one v_pk_add_f32 per row, in place)
    __device__ __forceinline__ void add_all(f2 t) {
        V tv;
#pragma unroll
        for (int i = 0; i < H; ++i) { tv[2 * i] = t.x; tv[2 * i + 1] = t.y; }
#pragma unroll
        for (int h = 0; h < RT / H; ++h) v[h] = v[h] + tv;
    }
    // every row = fma(w, x, row)
    __device__ __forceinline__ void fma_all(float w, f2 x) {
        V wv, xv;
#pragma unroll
        for (int i = 0; i < H; ++i) { wv[2 * i] = w; wv[2 * i + 1] = w; xv[2 * i] = x.x; xv[2 * i + 1] = x.y; }
#pragma unroll
        for (int h = 0; h < RT / H; ++h) v[h] = __builtin_elementwise_fma(wv, xv, v[h]);
    }
    __device__ __forceinline__ void set(int r, f2 a) {
        if constexpr (RT <= 16) {
            v[0][2 * r] = a.x;
            v[0][2 * r + 1] = a.y;
        } else if (r < H) {
            v[0][2 * r] = a.x;
            v[0][2 * r + 1] = a.y;
        } else {
            v[1][2 * (r - H)] = a.x;
            v[1][2 * (r - H) + 1] = a.y;
        }
    }
};
static_assert(sizeof(TileAcc<32>) == 64 * sizeof(float), "two halves of 16 pairs");

// The exact RT = 16 position loop over a run of "easy" positions (uniform weight, taken by every
// tile row or by all rows but one), hand-scheduled.  Written in C++, the dynamic row index of the
// skip-one form (s_set_gpr_idx + v_mov) made the compiler keep the 16 accumulator pairs in two
// register tuples and copy all of them at every merge of the loop's paths (16 v_mov_b64 per group
// of positions, more on the partial paths) — ~1/3 of the loop's VALU work.  Here the tuple is
// pinned to v[32:63] for the whole run and every update is in place.
//   positions j .. stop-1 of the current 64-position chunk (lanes of the descriptor registers):
//   v_addr  LDS byte address of the position's staged source row (lane j for position j)
//   v_w     the uniform weight (fp32 bits);  v_skip2  2 * (row that skips it), -1 = every row
//   lane8   this lane's byte offset in a staged row
// Per position: fl(w * x) once for the tile (v_pk_mul, the weight broadcast from an SGPR), then one
// v_pk_add per row in the reference's rounding; a skip-one position saves the skipped row, adds
// to all and restores it (bit-exact).  The next position's LDS read is in flight while the current
// one is applied (unrolled by 2: v[64:65] / v[66:67]).  Hazards: an SGPR written by v_readlane is
// read by a VALU at least 2 wait states later (s_nop 1 or other instructions in between).
#ifndef NIIDMIX_TLDS_ASM
#define NIIDMIX_TLDS_ASM 1
#endif
#define NIIDMIX_ADD16(T)                                                                            \
    "v_pk_add_f32 v[32:33], v[32:33], " T "\n\tv_pk_add_f32 v[34:35], v[34:35], " T "\n\t"          \
    "v_pk_add_f32 v[36:37], v[36:37], " T "\n\tv_pk_add_f32 v[38:39], v[38:39], " T "\n\t"          \
    "v_pk_add_f32 v[40:41], v[40:41], " T "\n\tv_pk_add_f32 v[42:43], v[42:43], " T "\n\t"          \
    "v_pk_add_f32 v[44:45], v[44:45], " T "\n\tv_pk_add_f32 v[46:47], v[46:47], " T "\n\t"          \
    "v_pk_add_f32 v[48:49], v[48:49], " T "\n\tv_pk_add_f32 v[50:51], v[50:51], " T "\n\t"          \
    "v_pk_add_f32 v[52:53], v[52:53], " T "\n\tv_pk_add_f32 v[54:55], v[54:55], " T "\n\t"          \
    "v_pk_add_f32 v[56:57], v[56:57], " T "\n\tv_pk_add_f32 v[58:59], v[58:59], " T "\n\t"          \
    "v_pk_add_f32 v[60:61], v[60:61], " T "\n\tv_pk_add_f32 v[62:63], v[62:63], " T "\n\t"
// exact: fl(w * x) once for the tile, then one add per row;  fast: one fma per row
#define NIIDMIX_UPD_EXACT(XD) "v_pk_mul_f32 v[72:73], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD16("v[72:73]")
#define NIIDMIX_FMA1(R, XD) "v_pk_fma_f32 " R ", " XD ", s[44:45], " R " op_sel_hi:[1,0,1]\n\t"
#define NIIDMIX_UPD_FAST(XD)                                                                        \
    NIIDMIX_FMA1("v[32:33]", XD) NIIDMIX_FMA1("v[34:35]", XD) NIIDMIX_FMA1("v[36:37]", XD)            \
    NIIDMIX_FMA1("v[38:39]", XD) NIIDMIX_FMA1("v[40:41]", XD) NIIDMIX_FMA1("v[42:43]", XD)            \
    NIIDMIX_FMA1("v[44:45]", XD) NIIDMIX_FMA1("v[46:47]", XD) NIIDMIX_FMA1("v[48:49]", XD)            \
    NIIDMIX_FMA1("v[50:51]", XD) NIIDMIX_FMA1("v[52:53]", XD) NIIDMIX_FMA1("v[54:55]", XD)            \
    NIIDMIX_FMA1("v[56:57]", XD) NIIDMIX_FMA1("v[58:59]", XD) NIIDMIX_FMA1("v[60:61]", XD)            \
    NIIDMIX_FMA1("v[62:63]", XD)
// one position k of the 4-way unrolled loop: data in XD (read two positions ago), its descriptor
// in SM; the read of position j+2 goes into XP with its descriptor into SP.  A skip-one position
// branches to an out-of-line block (SKIPBLK), so the common full position falls through.
#define NIIDMIX_TLDS_POS(XD, SM, XP, SP, K, UPD)                                                    \
    "s_add_u32 s47, %[j], 2\n\t"                                                                    \
    "s_min_u32 s47, s47, %[last]\n\t"                                                               \
    "v_readlane_b32 " SP ", %[vm], s47\n\t"                                                         \
    "v_readlane_b32 s44, %[vw], %[j]\n\t"                                                           \
    "s_and_b32 s46, " SP ", 0xffffff\n\t"                                                           \
    "v_add_u32 v76, s46, %[l8]\n\t"                                                                 \
    "ds_read_b64 " XP ", v76\n\t"                                                                   \
    "s_lshr_b32 s46, " SM ", 24\n\t"                                                                \
    "s_waitcnt lgkmcnt(2)\n\t"                                                                      \
    "s_cmp_lg_u32 s46, 0\n\t"                                                                       \
    "s_cbranch_scc1 .Ltlds_skip" K "_%=\n\t" UPD(XD)                                                \
    "\n.Ltlds_back" K "_%=:\n\t"                                                                    \
    "s_add_u32 %[j], %[j], 1\n\t"                                                                   \
    "s_cmp_ge_u32 %[j], %[stop]\n\t"                                                                \
    "s_cbranch_scc1 .Ltlds_done_%=\n\t"
#define NIIDMIX_TLDS_SKIPBLK(XD, K, UPD)                                                            \
    "\n.Ltlds_skip" K "_%=:\n\t"                                                                    \
    "s_sub_u32 s46, s46, 2\n\t"                                                                     \
    "s_set_gpr_idx_on s46, gpr_idx(SRC0)\n\t"                                                       \
    "v_mov_b32 v74, v32\n\t"                                                                        \
    "v_mov_b32 v75, v33\n\t"                                                                        \
    "s_set_gpr_idx_off\n\t" UPD(XD)                                                                 \
    "s_set_gpr_idx_on s46, gpr_idx(DST)\n\t"                                                        \
    "v_mov_b32 v32, v74\n\t"                                                                        \
    "v_mov_b32 v33, v75\n\t"                                                                        \
    "s_set_gpr_idx_off\n\t"                                                                         \
    "s_branch .Ltlds_back" K "_%=\n\t"
// descriptor of a position: LDS byte address of its staged row | (2 * skipped row + 2) << 24 (0:
// every row takes it)
#define NIIDMIX_TLDS_RUN(UPD)                                                                       \
    asm volatile("s_mov_b32 s47, %[j]\n\t"                                                          \
                 "v_readlane_b32 s40, %[vm], s47\n\t"                                               \
                 "s_add_u32 s47, %[j], 1\n\t"                                                       \
                 "s_min_u32 s47, s47, %[last]\n\t"                                                  \
                 "v_readlane_b32 s41, %[vm], s47\n\t"                                               \
                 "s_and_b32 s46, s40, 0xffffff\n\t"                                                 \
                 "v_add_u32 v76, s46, %[l8]\n\t"                                                    \
                 "ds_read_b64 v[64:65], v76\n\t"                                                    \
                 "s_and_b32 s46, s41, 0xffffff\n\t"                                                 \
                 "v_add_u32 v76, s46, %[l8]\n\t"                                                    \
                 "ds_read_b64 v[66:67], v76\n"                                                      \
                 ".Ltlds_loop_%=:\n\t"                                                              \
                 NIIDMIX_TLDS_POS("v[64:65]", "s40", "v[68:69]", "s42", "0", UPD)                  \
                 NIIDMIX_TLDS_POS("v[66:67]", "s41", "v[70:71]", "s43", "1", UPD)                  \
                 NIIDMIX_TLDS_POS("v[68:69]", "s42", "v[64:65]", "s40", "2", UPD)                  \
                 NIIDMIX_TLDS_POS("v[70:71]", "s43", "v[66:67]", "s41", "3", UPD)                  \
                 "s_branch .Ltlds_loop_%=\n\t"                                                      \
                 NIIDMIX_TLDS_SKIPBLK("v[64:65]", "0", UPD)                                         \
                 NIIDMIX_TLDS_SKIPBLK("v[66:67]", "1", UPD)                                         \
                 NIIDMIX_TLDS_SKIPBLK("v[68:69]", "2", UPD)                                         \
                 NIIDMIX_TLDS_SKIPBLK("v[70:71]", "3", UPD)                                         \
                 "\n.Ltlds_done_%=:\n\t"                                                            \
                 "s_waitcnt lgkmcnt(0)"                                                             \
                 : "+{v[32:63]}"(acc), [j] "+s"(j)                                                  \
                 : [stop] "s"(stop), [last] "s"(last), [vm] "v"(v_meta), [vw] "v"(v_w),             \
                   [l8] "v"(lane8)                                                                  \
                 : "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74",     \
                   "v75", "v76", "s40", "s41", "s42", "s43", "s44", "s45", "s46", "s47", "m0", "scc", \
                   "memory")
typedef TileAcc<16>::V Acc16;
template <bool EXACT>
__device__ __forceinline__ void tlds16_run(Acc16 &acc, int j, int stop, int v_meta, int v_w,
                                           int lane8) {
    const int last = stop - 1;
    if constexpr (EXACT) NIIDMIX_TLDS_RUN(NIIDMIX_UPD_EXACT);
    else NIIDMIX_TLDS_RUN(NIIDMIX_UPD_FAST);
}

// The RT = 16 segment walker (niidmix.tile.build_tile_segments): ONE asm block walks all of a
// tile's segments, so the accumulator tuple stays pinned in v[32:63] from the first segment to the
// last (one asm statement per segment let the compiler keep the tuple in other registers between
// them and copy all 16 pairs in and out around every segment: 32 v_mov per segment, ~30 % of the
// kernel's VALU instructions).  Segment j's descriptor words sit in lane j of dx / dy / dz.
//  * a RUN (bit 30 of dx clear): dx = first slot | length << 12 | first skipped row << 20,
//    dy = weight-select bits, dz = skip bits.  Positions i = 0 .. len-1 read consecutive LDS slots,
//    so position i's row sits at one base address + i * RB bytes -- an immediate offset, no
//    per-position descriptor; its weight is the tile's w0 or w1 (bit i of dy, picked by SALU) and it
//    is taken by every row, or (bit i of dz) by all rows but the next one of the run's skipped rows
//    r0, r0 + 1, ... (saved, updated with the others, restored: bit-exact).  The row two positions
//    ahead is read while one is applied; the LDS stage holds two spare rows for the reads past a
//    run's end (those reads land before the next run's own reads: LDS returns in order).
//  * a MASKED position (bit 30 set): dx = slot | 1 << 30, dy = the rows that take it, dz = its
//    weight (fp32 bits) -- a row taking a gateway's inter-clique edge alone, a source two rows order
//    differently, or one weight class of a position whose rows carry different weights (split by
//    weight, each row still takes it once, in its own order).  Each of its rows is reached by
//    GPR-index mode (s_set_gpr_idx).
// Fixed scratch SGPRs: s38 run length, s39 LDS address, s40 segment index, s41 dx, s42 dy (masked:
// the remaining rows), s43 dz, s44 weight, s46 skipped row * 2 / row index, s47 position.  VGPR
// scratch are compiler-allocated operands: x0..x3 rotating row pairs, pr the product, sv0 / sv1 the
// saved skipped row (one v_mov_b64 each way), q0 / q1 a masked position's product (exact) or row (fast), va the address.
#define NIIDMIX_SEG_UPD_EXACT(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD16("%[pr]")
// the same for tiles whose rows all sit in the first n slots: a 1000-node d-clique is cut into
// tiles of 16, 15 x 5 and its 9 gateway rows, a 10 000-node one into 15 x 2 and 14 x 5 rows; a tile
// adds only its own rows (row counts 9-15 exactly, 8 and 4 rounded up)
#define NIIDMIX_ADD4(T)                                                                             \
    "v_pk_add_f32 v[32:33], v[32:33], " T "\n\tv_pk_add_f32 v[34:35], v[34:35], " T "\n\t"          \
    "v_pk_add_f32 v[36:37], v[36:37], " T "\n\tv_pk_add_f32 v[38:39], v[38:39], " T "\n\t"
#define NIIDMIX_ADD8(T)                                                                             \
    NIIDMIX_ADD4(T)                                                                                 \
    "v_pk_add_f32 v[40:41], v[40:41], " T "\n\tv_pk_add_f32 v[42:43], v[42:43], " T "\n\t"          \
    "v_pk_add_f32 v[44:45], v[44:45], " T "\n\tv_pk_add_f32 v[46:47], v[46:47], " T "\n\t"
#define NIIDMIX_ADD12(T)                                                                            \
    NIIDMIX_ADD8(T)                                                                                 \
    "v_pk_add_f32 v[48:49], v[48:49], " T "\n\tv_pk_add_f32 v[50:51], v[50:51], " T "\n\t"          \
    "v_pk_add_f32 v[52:53], v[52:53], " T "\n\tv_pk_add_f32 v[54:55], v[54:55], " T "\n\t"
#define NIIDMIX_SEG_UPD_EXACT12(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD12("%[pr]")
#define NIIDMIX_SEG_UPD_EXACT8(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD8("%[pr]")
#define NIIDMIX_SEG_UPD_EXACT4(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD4("%[pr]")
#define NIIDMIX_UPD_FAST4(XD)                                                                       \
    NIIDMIX_FMA1("v[32:33]", XD) NIIDMIX_FMA1("v[34:35]", XD) NIIDMIX_FMA1("v[36:37]", XD)            \
    NIIDMIX_FMA1("v[38:39]", XD)
#define NIIDMIX_UPD_FAST8(XD)                                                                       \
    NIIDMIX_UPD_FAST4(XD) NIIDMIX_FMA1("v[40:41]", XD) NIIDMIX_FMA1("v[42:43]", XD)                 \
    NIIDMIX_FMA1("v[44:45]", XD) NIIDMIX_FMA1("v[46:47]", XD)
#define NIIDMIX_UPD_FAST12(XD)                                                                      \
    NIIDMIX_UPD_FAST8(XD) NIIDMIX_FMA1("v[48:49]", XD) NIIDMIX_FMA1("v[50:51]", XD)                 \
    NIIDMIX_FMA1("v[52:53]", XD) NIIDMIX_FMA1("v[54:55]", XD)
// one loop per row count 9..15 too (tiles of 14-15 rows: 10 000 nodes; 15: 1000 nodes)
#define NIIDMIX_ADD9(T) NIIDMIX_ADD8(T) "v_pk_add_f32 v[48:49], v[48:49], " T "\n\t"
#define NIIDMIX_ADD10(T) NIIDMIX_ADD9(T) "v_pk_add_f32 v[50:51], v[50:51], " T "\n\t"
#define NIIDMIX_ADD11(T) NIIDMIX_ADD10(T) "v_pk_add_f32 v[52:53], v[52:53], " T "\n\t"
#define NIIDMIX_ADD13(T) NIIDMIX_ADD12(T) "v_pk_add_f32 v[56:57], v[56:57], " T "\n\t"
#define NIIDMIX_ADD14(T) NIIDMIX_ADD13(T) "v_pk_add_f32 v[58:59], v[58:59], " T "\n\t"
#define NIIDMIX_ADD15(T) NIIDMIX_ADD14(T) "v_pk_add_f32 v[60:61], v[60:61], " T "\n\t"
#define NIIDMIX_SEG_UPD_EXACT9(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD9("%[pr]")
#define NIIDMIX_SEG_UPD_EXACT10(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD10("%[pr]")
#define NIIDMIX_SEG_UPD_EXACT11(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD11("%[pr]")
#define NIIDMIX_SEG_UPD_EXACT13(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD13("%[pr]")
#define NIIDMIX_SEG_UPD_EXACT14(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD14("%[pr]")
#define NIIDMIX_SEG_UPD_EXACT15(XD) "v_pk_mul_f32 %[pr], " XD ", s[44:45] op_sel_hi:[1,0]\n\t" NIIDMIX_ADD15("%[pr]")
#define NIIDMIX_UPD_FAST9(XD) NIIDMIX_UPD_FAST8(XD) NIIDMIX_FMA1("v[48:49]", XD)
#define NIIDMIX_UPD_FAST10(XD) NIIDMIX_UPD_FAST9(XD) NIIDMIX_FMA1("v[50:51]", XD)
#define NIIDMIX_UPD_FAST11(XD) NIIDMIX_UPD_FAST10(XD) NIIDMIX_FMA1("v[52:53]", XD)
#define NIIDMIX_UPD_FAST13(XD) NIIDMIX_UPD_FAST12(XD) NIIDMIX_FMA1("v[56:57]", XD)
#define NIIDMIX_UPD_FAST14(XD) NIIDMIX_UPD_FAST13(XD) NIIDMIX_FMA1("v[58:59]", XD)
#define NIIDMIX_UPD_FAST15(XD) NIIDMIX_UPD_FAST14(XD) NIIDMIX_FMA1("v[60:61]", XD)
#if NIIDMIX_TLDS_SPLIT == 6 || NIIDMIX_TLDS_SPLIT == 7
// time-split builds only (wrong results): 6 no per-position weight select and skip test, 7 no skip
// test (the cost of the per-position scalar bookkeeping a pre-split run table would remove)
#define NIIDMIX_SEG_POS(XD, XP, OFF, K, UPD)                                                         \
    "ds_read_b64 " XP ", %[va] offset:%[" OFF "]\n\t"                                                \
    NIIDMIX_SEG_WSEL                                                                                 \
    "s_waitcnt lgkmcnt(2)\n\t" UPD(XD)                                                               \
    "\n.Lseg_back" K "_%=:\n\t"                                                                     \
    "s_add_u32 s47, s47, 1\n\t"                                                                      \
    "s_cmp_ge_u32 s47, s38\n\t"                                                                      \
    "s_cbranch_scc1 .Lw_next_%=\n\t"
#if NIIDMIX_TLDS_SPLIT == 7
#define NIIDMIX_SEG_WSEL "s_bitcmp1_b32 s42, s47\n\t" "s_cselect_b32 s44, %[w1], %[w0]\n\t"
#else
#define NIIDMIX_SEG_WSEL
#endif
#else
#define NIIDMIX_SEG_POS(XD, XP, OFF, K, UPD)                                                         \
    "ds_read_b64 " XP ", %[va] offset:%[" OFF "]\n\t"                                                \
    "s_bitcmp1_b32 s42, s47\n\t"                                                                     \
    "s_cselect_b32 s44, %[w1], %[w0]\n\t"                                                            \
    "s_bitcmp1_b32 s43, s47\n\t"                                                                     \
    "s_waitcnt lgkmcnt(2)\n\t"                                                                       \
    "s_cbranch_scc1 .Lseg_skip" K "_%=\n\t" UPD(XD)                                                 \
    "\n.Lseg_back" K "_%=:\n\t"                                                                     \
    "s_add_u32 s47, s47, 1\n\t"                                                                      \
    "s_cmp_ge_u32 s47, s38\n\t"                                                                      \
    "s_cbranch_scc1 .Lw_next_%=\n\t"
#endif
#define NIIDMIX_SEG_SKIPBLK(XD, K, UPD)                                                              \
    "\n.Lseg_skip" K "_%=:\n\t"                                                                     \
    "s_set_gpr_idx_on s46, gpr_idx(SRC0)\n\t"                                                       \
    "v_mov_b64 %[sv], v[32:33]\n\t"                                                                 \
    "s_set_gpr_idx_off\n\t" UPD(XD)                                                                  \
    "s_set_gpr_idx_on s46, gpr_idx(DST)\n\t"                                                        \
    "v_mov_b64 v[32:33], %[sv]\n\t"                                                                 \
    "s_set_gpr_idx_off\n\t"                                                                          \
    "s_add_u32 s46, s46, 2\n\t"                                                                      \
    "s_branch .Lseg_back" K "_%=\n\t"
// a masked position's per-row update: exact adds the product formed once, fast fmas the row
#define NIIDMIX_MSK_EXACT                                                                            \
    "v_mul_f32 %[q0], s43, %[q0]\n\t"                                                                \
    "v_mul_f32 %[q1], s43, %[q1]\n"                                                                  \
    ".Lmsk_loop_%=:\n\t"                                                                             \
    "s_ff1_i32_b32 s46, s42\n\t"                                                                     \
    "s_cmp_lt_i32 s46, 0\n\t"                                                                        \
    "s_cbranch_scc1 .Lw_next_%=\n\t"                                                                 \
    "s_bitset0_b32 s42, s46\n\t"                                                                     \
    "s_lshl_b32 s46, s46, 1\n\t"                                                                     \
    "s_set_gpr_idx_on s46, gpr_idx(SRC0,DST)\n\t"                                                   \
    "v_add_f32 v32, v32, %[q0]\n\t"                                                                  \
    "v_add_f32 v33, v33, %[q1]\n\t"                                                                  \
    "s_set_gpr_idx_off\n\t"                                                                          \
    "s_branch .Lmsk_loop_%=\n\t"
#define NIIDMIX_MSK_FAST                                                                             \
    ".Lmsk_loop_%=:\n\t"                                                                             \
    "s_ff1_i32_b32 s46, s42\n\t"                                                                     \
    "s_cmp_lt_i32 s46, 0\n\t"                                                                        \
    "s_cbranch_scc1 .Lw_next_%=\n\t"                                                                 \
    "s_bitset0_b32 s42, s46\n\t"                                                                     \
    "s_lshl_b32 s46, s46, 1\n\t"                                                                     \
    "s_set_gpr_idx_on s46, gpr_idx(SRC2,DST)\n\t"                                                   \
    "v_fma_f32 v32, %[q0], s43, v32\n\t"                                                             \
    "v_fma_f32 v33, %[q1], s43, v33\n\t"                                                             \
    "s_set_gpr_idx_off\n\t"                                                                          \
    "s_branch .Lmsk_loop_%=\n\t"
// REGISTER rows (plans with rem_rows): a masked entry whose word 0 has bit 29 set takes its source
// from the tile's register rows, pinned in v[64:95] (register row i in v[64 + 2i : 65 + 2i]),
// picked by GPR-index mode, instead of from the LDS stage.
#define NIIDMIX_SEG_REMOTE NIIDMIX_SEG_REMOTE_M("0xfff")
// 8 register rows: index & 7 (the two-phase kernel walks rows 8..15 of a 16-row plan in v[64:79])
#define NIIDMIX_SEG_REMOTE8 NIIDMIX_SEG_REMOTE_M("7")
#define NIIDMIX_SEG_REMOTE_M(MASK)                                                                   \
    "s_bitcmp1_b32 s41, 29\n\t"                                                                     \
    "s_cbranch_scc0 .Lw_lds_%=\n\t"                                                                 \
    "s_and_b32 s46, s41, " MASK "\n\t"                                                              \
    "s_lshl_b32 s46, s46, 1\n\t"                                                                    \
    "s_set_gpr_idx_on s46, gpr_idx(SRC0)\n\t"                                                       \
    "v_mov_b32 %[q0], v64\n\t"                                                                      \
    "v_mov_b32 %[q1], v65\n\t"                                                                      \
    "s_set_gpr_idx_off\n\t"                                                                         \
    "s_branch .Lw_mskgo_%=\n"                                                                       \
    ".Lw_lds_%=:\n\t"
#define NIIDMIX_REM_IN , [rem] "{v[64:95]}"(rem)
#define NIIDMIX_REM_IN8 , [rem] "{v[64:79]}"(rem)
#define NIIDMIX_SEG_WALK(UPD, MSK) NIIDMIX_SEG_WALK_X(UPD, MSK, "", )
// a run's positions: %[nr] = 4, 8, 9, ..., 16 rows updated per position (the tile's rows sit in its
// first nr slots); the smaller loops are copies of the 16-row one with fewer adds
#define NIIDMIX_SEG_LOOP(S, UPD)                                                                     \
    ".Lseg_loop" S "_%=:\n\t"                                                                       \
    NIIDMIX_SEG_POS("%[x0]", "%[x2]", "o2", S "0", UPD)                                              \
    NIIDMIX_SEG_POS("%[x1]", "%[x3]", "o3", S "1", UPD)                                              \
    NIIDMIX_SEG_POS("%[x2]", "%[x0]", "o4", S "2", UPD)                                              \
    NIIDMIX_SEG_POS("%[x3]", "%[x1]", "o5", S "3", UPD)                                              \
    "v_add_u32 %[va], %[o4], %[va]\n\t"                                                             \
    "s_branch .Lseg_loop" S "_%=\n\t"                                                               \
    NIIDMIX_SEG_SKIPBLK("%[x0]", S "0", UPD)                                                         \
    NIIDMIX_SEG_SKIPBLK("%[x1]", S "1", UPD)                                                         \
    NIIDMIX_SEG_SKIPBLK("%[x2]", S "2", UPD)                                                         \
    NIIDMIX_SEG_SKIPBLK("%[x3]", S "3", UPD)
#define NIIDMIX_SEG_WALK_X(UPD, MSK, RMSK, RIN)                                                      \
    asm volatile("s_mov_b32 s36, %[sb0]\n"                                                           \
                 ".Lc_next_%=:\n\t"                                                                  \
                 "s_cmp_ge_u32 s36, %[sb1]\n\t"                                                      \
                 "s_cbranch_scc1 .Lw_end_%=\n\t"                                                     \
                 "s_sub_u32 s37, %[sb1], s36\n\t"                                                    \
                 "s_min_u32 s37, s37, 64\n\t"                                                        \
                 "s_sub_u32 s35, s37, 1\n\t"                                                         \
                 "v_min_u32 %[vo], %[ln], s35\n\t"                                                   \
                 "v_add_u32 %[vo], s36, %[vo]\n\t"                                                   \
                 "v_lshlrev_b32 %[vo], 4, %[vo]\n\t"                                                 \
                 "global_load_dword %[dx], %[vo], %[sp]\n\t"                                         \
                 "global_load_dword %[dy], %[vo], %[sp] offset:4\n\t"                                \
                 "global_load_dword %[dz], %[vo], %[sp] offset:8\n\t"                                \
                 "s_waitcnt vmcnt(0)\n\t"                                                            \
                 "s_mov_b32 s40, 0\n"                                                                \
                 ".Lw_next_%=:\n\t"                                                                  \
                 "s_cmp_ge_u32 s40, s37\n\t"                                                         \
                 "s_cbranch_scc1 .Lc_done_%=\n\t"                                                    \
                 "v_readlane_b32 s41, %[dx], s40\n\t"                                                \
                 "v_readlane_b32 s42, %[dy], s40\n\t"                                                \
                 "v_readlane_b32 s43, %[dz], s40\n\t"                                                \
                 "s_add_u32 s40, s40, 1\n\t"                                                         \
                 "s_and_b32 s39, s41, 0xfff\n\t"                                                     \
                 "s_mul_i32 s39, s39, %[o1]\n\t"                                                     \
                 "s_add_u32 s39, s39, %[base]\n\t"                                                   \
                 "v_add_u32 %[va], s39, %[l8]\n\t"                                                   \
                 "s_bitcmp1_b32 s41, 30\n\t"                                                         \
                 "s_cbranch_scc1 .Lw_masked_%=\n\t"                                                  \
                 "ds_read_b64 %[x0], %[va]\n\t"                                                      \
                 "ds_read_b64 %[x1], %[va] offset:%[o1]\n\t"                                         \
                 "s_bfe_u32 s38, s41, 0x8000c\n\t"                                                   \
                 "s_bfe_u32 s46, s41, 0x80014\n\t"                                                   \
                 "s_lshl_b32 s46, s46, 1\n\t"                                                        \
                 "s_mov_b32 s47, 0\n\t"                                                              \
                 "s_cmp_lt_u32 %[nr], 16\n\t"                                                        \
                 "s_cbranch_scc1 .Lseg_small_%=\n\t"                                                 \
                 NIIDMIX_SEG_LOOP("", UPD)                                                           \
                 "\n.Lseg_small_%=:\n\t"                                                             \
                 "s_cmp_le_u32 %[nr], 4\n\t"                                                         \
                 "s_cbranch_scc1 .Lseg_loopq_%=\n\t"                                                 \
                 "s_cmp_le_u32 %[nr], 8\n\t"                                                         \
                 "s_cbranch_scc1 .Lseg_looph_%=\n\t"                                                 \
                 "s_cmp_eq_u32 %[nr], 15\n\t"                                                        \
                 "s_cbranch_scc1 .Lseg_loopn15_%=\n\t"                                               \
                 "s_cmp_eq_u32 %[nr], 14\n\t"                                                        \
                 "s_cbranch_scc1 .Lseg_loopn14_%=\n\t"                                               \
                 "s_cmp_eq_u32 %[nr], 13\n\t"                                                        \
                 "s_cbranch_scc1 .Lseg_loopn13_%=\n\t"                                               \
                 "s_cmp_eq_u32 %[nr], 12\n\t"                                                        \
                 "s_cbranch_scc1 .Lseg_loopt_%=\n\t"                                                 \
                 "s_cmp_eq_u32 %[nr], 11\n\t"                                                        \
                 "s_cbranch_scc1 .Lseg_loopn11_%=\n\t"                                               \
                 "s_cmp_eq_u32 %[nr], 10\n\t"                                                        \
                 "s_cbranch_scc1 .Lseg_loopn10_%=\n\t"                                               \
                 NIIDMIX_SEG_LOOP("n9", UPD##9)                                                      \
                 NIIDMIX_SEG_LOOP("n10", UPD##10)                                                    \
                 NIIDMIX_SEG_LOOP("n11", UPD##11)                                                    \
                 NIIDMIX_SEG_LOOP("t", UPD##12)                                                      \
                 NIIDMIX_SEG_LOOP("n13", UPD##13)                                                    \
                 NIIDMIX_SEG_LOOP("n14", UPD##14)                                                    \
                 NIIDMIX_SEG_LOOP("n15", UPD##15)                                                    \
                 NIIDMIX_SEG_LOOP("h", UPD##8)                                                       \
                 NIIDMIX_SEG_LOOP("q", UPD##4)                                                       \
                 "\n.Lw_masked_%=:\n\t"                                                              \
                 RMSK                                                                                \
                 "ds_read_b32 %[q0], %[va]\n\t"                                                      \
                 "ds_read_b32 %[q1], %[va] offset:4\n\t"                                             \
                 "s_waitcnt lgkmcnt(0)\n"                                                             \
                 ".Lw_mskgo_%=:\n\t"                                                                 \
                 MSK                                                                                 \
                 "\n.Lc_done_%=:\n\t"                                                                \
                 "s_add_u32 s36, s36, 64\n\t"                                                        \
                 "s_branch .Lc_next_%=\n"                                                            \
                 ".Lw_end_%=:\n\t"                                                                   \
                 "s_waitcnt lgkmcnt(0)"                                                              \
                 : "+{v[32:63]}"(acc), [x0] "=&v"(x0), [x1] "=&v"(x1), [x2] "=&v"(x2),             \
                   [x3] "=&v"(x3), [pr] "=&v"(pr), [sv] "=&v"(sv),                                   \
                   [q0] "=&v"(q0), [q1] "=&v"(q1), [va] "=&v"(va), [dx] "=&v"(dx), [dy] "=&v"(dy),  \
                   [dz] "=&v"(dz), [vo] "=&v"(vo)                                                   \
                 : [sp] "s"(segp), [sb0] "s"(sb0), [sb1] "s"(sb1), [ln] "v"(lane), [base] "s"(base), \
                   [w0] "s"(w0), [w1] "s"(w1), [l8] "v"(lane8), [nr] "s"(nr), [o1] "i"(RB),            \
                   [o2] "i"(2 * RB), [o3] "i"(3 * RB), [o4] "i"(4 * RB), [o5] "i"(5 * RB) RIN         \
                 : "s35", "s36", "s37", "s38", "s39", "s40", "s41", "s42", "s43", "s44", "s45", "s46", \
                   "s47", "m0", "scc", "memory")
// segp: the segment words (int4 per segment); the tile's segments [sb0, sb1) are fetched 64 at a time
// INSIDE the asm (lane j: segment j's words), so no VALU address arithmetic sits between the tile's
// init and its walk -- hipcc otherwise moved the pinned tuple out of v[32:63] to make room for it
template <bool EXACT, int RB>
__device__ __forceinline__ void tlds16_walk(Acc16 &acc, const int32_t *segp, int sb0, int sb1, int base,
                                            int w0, int w1, int lane8, int lane, int nr) {
    static_assert(5 * RB < 65536, "ds_read immediate offset");
    uint64_t x0, x1, x2, x3, pr;
    uint64_t sv;
    uint32_t q0, q1, va, dx, dy, dz, vo;
    if constexpr (EXACT) NIIDMIX_SEG_WALK(NIIDMIX_SEG_UPD_EXACT, NIIDMIX_MSK_EXACT);
    else NIIDMIX_SEG_WALK(NIIDMIX_UPD_FAST, NIIDMIX_MSK_FAST);
    (void)pr;
}
typedef float Rem32 __attribute__((ext_vector_type(32)));
typedef float Rem16 __attribute__((ext_vector_type(16)));
template <int NREM> struct RemRegs { typedef Rem32 V; };        // NREM register rows, pairs
template <> struct RemRegs<8> { typedef Rem16 V; };
// the same walker with the tile's NREM register rows (rem) pinned in v[64:64 + 2 NREM)
template <bool EXACT, int RB, int NREM>
__device__ __forceinline__ void tlds16_walk_rem(Acc16 &acc, const int32_t *segp, int sb0, int sb1,
                                                int base, int w0, int w1, int lane8, int lane,
                                                int nr, const typename RemRegs<NREM>::V &rem) {
    static_assert(5 * RB < 65536, "ds_read immediate offset");
    static_assert(NREM == 8 || NREM == 16, "8 or 16 register rows");
    uint64_t x0, x1, x2, x3, pr;
    uint64_t sv;
    uint32_t q0, q1, va, dx, dy, dz, vo;
    if constexpr (EXACT && NREM == 16)
        NIIDMIX_SEG_WALK_X(NIIDMIX_SEG_UPD_EXACT, NIIDMIX_MSK_EXACT, NIIDMIX_SEG_REMOTE, NIIDMIX_REM_IN);
    else if constexpr (NREM == 16)
        NIIDMIX_SEG_WALK_X(NIIDMIX_UPD_FAST, NIIDMIX_MSK_FAST, NIIDMIX_SEG_REMOTE, NIIDMIX_REM_IN);
    else if constexpr (EXACT)
        NIIDMIX_SEG_WALK_X(NIIDMIX_SEG_UPD_EXACT, NIIDMIX_MSK_EXACT, NIIDMIX_SEG_REMOTE8, NIIDMIX_REM_IN8);
    else
        NIIDMIX_SEG_WALK_X(NIIDMIX_UPD_FAST, NIIDMIX_MSK_FAST, NIIDMIX_SEG_REMOTE8, NIIDMIX_REM_IN8);
    (void)pr;
}

// Tile init of the RT-16 segment kernels in asm: every row's accumulator acc_r = z_r + fl(ws_r x_r)
// (exact; fast: fma(ws_r, x_r, z_r)), z_r = x_r * 0 -- the self term (model/__init__.py:19-24) --
// written straight into the pinned tuple v[32:63].  Initialised in C++, the tuple lived in
// v[0:31] until the walker and was copied into v[32:63] there: 32 extra VGPRs at the peak (90, so
// only two 7-wave blocks per CU instead of the three the LDS allows).  Rows' LDS reads two ahead.
template <bool EXACT>
__device__ __forceinline__ void tlds16_init(Acc16 &acc, int d_slot, int d_ws, int rb, int base, int lane8) {
    uint64_t x0, x1, t, pr;
    uint32_t va;
    if constexpr (EXACT)
        asm volatile("s_mov_b64 s[46:47], 0\n\t"
                 "v_readlane_b32 s40, %[ds], 0\n\t""v_readlane_b32 s42, %[dw], 0\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "v_readlane_b32 s40, %[ds], 1\n\t""v_readlane_b32 s44, %[dw], 1\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x0], s[42:43] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[32:33], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 2\n\t""v_readlane_b32 s42, %[dw], 2\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x1], s[44:45] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[34:35], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 3\n\t""v_readlane_b32 s44, %[dw], 3\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x0], s[42:43] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[36:37], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 4\n\t""v_readlane_b32 s42, %[dw], 4\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x1], s[44:45] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[38:39], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 5\n\t""v_readlane_b32 s44, %[dw], 5\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x0], s[42:43] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[40:41], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 6\n\t""v_readlane_b32 s42, %[dw], 6\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x1], s[44:45] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[42:43], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 7\n\t""v_readlane_b32 s44, %[dw], 7\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x0], s[42:43] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[44:45], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 8\n\t""v_readlane_b32 s42, %[dw], 8\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x1], s[44:45] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[46:47], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 9\n\t""v_readlane_b32 s44, %[dw], 9\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x0], s[42:43] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[48:49], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 10\n\t""v_readlane_b32 s42, %[dw], 10\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x1], s[44:45] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[50:51], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 11\n\t""v_readlane_b32 s44, %[dw], 11\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x0], s[42:43] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[52:53], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 12\n\t""v_readlane_b32 s42, %[dw], 12\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x1], s[44:45] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[54:55], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 13\n\t""v_readlane_b32 s44, %[dw], 13\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x0], s[42:43] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[56:57], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 14\n\t""v_readlane_b32 s42, %[dw], 14\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x1], s[44:45] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[58:59], %[t], %[pr]\n\t"
                 "v_readlane_b32 s40, %[ds], 15\n\t""v_readlane_b32 s44, %[dw], 15\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x0], s[42:43] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[60:61], %[t], %[pr]\n\t"
                 "s_waitcnt lgkmcnt(0)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_mul_f32 %[pr], %[x1], s[44:45] op_sel_hi:[1,0]\n\t""v_pk_add_f32 v[62:63], %[t], %[pr]\n\t"
                 : "={v[32:63]}"(acc), [x0] "=&v"(x0), [x1] "=&v"(x1), [t] "=&v"(t), [pr] "=&v"(pr),
                   [va] "=&v"(va)
                 : [ds] "v"(d_slot), [dw] "v"(d_ws), [rb] "s"(rb), [base] "s"(base), [l8] "v"(lane8)
                 : "s40", "s42", "s43", "s44", "s45", "s46", "s47", "memory");
    else
        asm volatile("s_mov_b64 s[46:47], 0\n\t"
                 "v_readlane_b32 s40, %[ds], 0\n\t""v_readlane_b32 s42, %[dw], 0\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "v_readlane_b32 s40, %[ds], 1\n\t""v_readlane_b32 s44, %[dw], 1\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_fma_f32 v[32:33], %[x0], s[42:43] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 2\n\t""v_readlane_b32 s42, %[dw], 2\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_fma_f32 v[34:35], %[x1], s[44:45] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 3\n\t""v_readlane_b32 s44, %[dw], 3\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_fma_f32 v[36:37], %[x0], s[42:43] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 4\n\t""v_readlane_b32 s42, %[dw], 4\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_fma_f32 v[38:39], %[x1], s[44:45] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 5\n\t""v_readlane_b32 s44, %[dw], 5\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_fma_f32 v[40:41], %[x0], s[42:43] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 6\n\t""v_readlane_b32 s42, %[dw], 6\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_fma_f32 v[42:43], %[x1], s[44:45] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 7\n\t""v_readlane_b32 s44, %[dw], 7\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_fma_f32 v[44:45], %[x0], s[42:43] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 8\n\t""v_readlane_b32 s42, %[dw], 8\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_fma_f32 v[46:47], %[x1], s[44:45] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 9\n\t""v_readlane_b32 s44, %[dw], 9\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_fma_f32 v[48:49], %[x0], s[42:43] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 10\n\t""v_readlane_b32 s42, %[dw], 10\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_fma_f32 v[50:51], %[x1], s[44:45] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 11\n\t""v_readlane_b32 s44, %[dw], 11\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_fma_f32 v[52:53], %[x0], s[42:43] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 12\n\t""v_readlane_b32 s42, %[dw], 12\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_fma_f32 v[54:55], %[x1], s[44:45] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 13\n\t""v_readlane_b32 s44, %[dw], 13\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_fma_f32 v[56:57], %[x0], s[42:43] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 14\n\t""v_readlane_b32 s42, %[dw], 14\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x0], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_fma_f32 v[58:59], %[x1], s[44:45] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "v_readlane_b32 s40, %[ds], 15\n\t""v_readlane_b32 s44, %[dw], 15\n\t""s_mul_i32 s40, s40, %[rb]\n\t""s_add_u32 s40, s40, %[base]\n\t""v_add_u32 %[va], s40, %[l8]\n\t""ds_read_b64 %[x1], %[va]\n\t"
                 "s_waitcnt lgkmcnt(1)\n\t""v_pk_mul_f32 %[t], %[x0], s[46:47]\n\t""v_pk_fma_f32 v[60:61], %[x0], s[42:43] , %[t] op_sel_hi:[1,0,1]\n\t"
                 "s_waitcnt lgkmcnt(0)\n\t""v_pk_mul_f32 %[t], %[x1], s[46:47]\n\t""v_pk_fma_f32 v[62:63], %[x1], s[44:45] , %[t] op_sel_hi:[1,0,1]\n\t"
                 : "={v[32:63]}"(acc), [x0] "=&v"(x0), [x1] "=&v"(x1), [t] "=&v"(t), [pr] "=&v"(pr),
                   [va] "=&v"(va)
                 : [ds] "v"(d_slot), [dw] "v"(d_ws), [rb] "s"(rb), [base] "s"(base), [l8] "v"(lane8)
                 : "s40", "s42", "s43", "s44", "s45", "s46", "s47", "memory");
    (void)pr;
}

// Apply op(acc_row, r) to the rows of the wave-uniform mask m.  No per-row select: on gfx950 a lane
// mask or SGPR operand that a SALU op just wrote stalls the VALU ~30-40 cycles per row
// (tools/valu_probe.hip: the select form of a partial position cost ~10x a full one).  Instead,
// when one or two rows skip the position (a tile row is never its own source, so most partial
// masks miss exactly one row) those rows are saved, every row is updated and the saved registers
// are written back — bit-exact, the skipped rows keep their bits; sparser masks visit only their
// rows by dynamic register index.
template <int RT, class Op>
__device__ __forceinline__ void apply_mask(TileAcc<RT> &acc, uint32_t m, Op op) {
    constexpr uint32_t FULL = (uint32_t)((1ull << RT) - 1ull);
    if (m == FULL) {
#pragma unroll
        for (int r = 0; r < RT; ++r) acc.set(r, op(acc.get(r), r));
        return;
    }
    const uint32_t miss = ~m & FULL;                // != 0: the mask is not full
    const uint32_t rest = miss & (miss - 1u);
    if ((rest & (rest - 1u)) == 0u) {
        const int r0 = __builtin_ctz(miss), r1 = rest ? __builtin_ctz(rest) : r0;
        const f2 s0 = acc.get(r0), s1 = acc.get(r1);
#pragma unroll
        for (int r = 0; r < RT; ++r) acc.set(r, op(acc.get(r), r));
        acc.set(r1, s1);
        acc.set(r0, s0);
    } else {
        for (uint32_t b = m & FULL; b; b &= b - 1u) {
            const int r = __builtin_ctz(b);
            acc.set(r, op(acc.get(r), r));
        }
    }
}

// Time-split switch for tuning builds only (tools/tlds_split.sh builds variant libraries): 1 skips
// the position / segment loop, 2 skips the staging (the segment loop still runs); 3-5 strip the position loop down (3: every position full
// and uniform, 4: no product either, 5: no adds).  Product builds leave it 0.
#ifndef NIIDMIX_TLDS_SPLIT
#define NIIDMIX_TLDS_SPLIT 0
#endif
// The exact matrix-core path in the RT-16 segment kernels (1) or not (0).
#ifndef NIIDMIX_TLDS_MF
#define NIIDMIX_TLDS_MF 1
#endif
// Matrix-core path time split (tuning builds only): 3 no position loop.  Product builds leave it 0.
#ifndef NIIDMIX_MF_SPLIT
#define NIIDMIX_MF_SPLIT 0
#endif
// Stage by LDS-DMA (1) or through registers (0; tuning A/B builds only).
#ifndef NIIDMIX_TLDS_GLDS
#define NIIDMIX_TLDS_GLDS 1
#endif
// LDS bytes past the staged rows: the LDS-DMA staging writes whole 1 KiB wave-instructions, the last
// one up to 1008 B past the group's rows; the segment loop's two spare rows absorb part of that
// (an LDS allocation counts in 512-B granules: 1000-node d-cliques at 120 columns keep three
// blocks per CU only with <= 480 B more than the 111 rows)
inline size_t tlds_slack(bool seg, int cw) {
    const size_t spare = seg ? 2 * (size_t)cw * sizeof(float) : 0;
    return NIIDMIX_TLDS_GLDS && spare < 1024 ? 1024 - spare : 0;
}
// rt 16: up to 12 tiles per group, so a clique cut into shorter tiles (niidmix.tile: tile rows per
// plan) gets more waves per block where the VGPR budget leaves room for them
constexpr int tile_lds_max_waves(int rt) { return rt == 8 ? 16 : rt == 16 ? 12 : 4; }

template <bool B> struct BoolC { static constexpr bool value = B; };

// REM2 (NREM 8): the plan has up to 16 register rows per tile, walked in two phases of 8 (rows
// 0..7 loaded before the walk, 8..15 once the walk reaches the first segment that reads one)
template <bool EXACT, int RT, int SV, int RS, bool SEG, int NREM = 0, bool MF = false, bool REM2 = false>
__global__ __launch_bounds__(64 * tile_lds_max_waves(RT)) void k_mix_tile_lds(
    const float *__restrict__ x, int64_t ld_x, float *__restrict__ y, int64_t ld_y, int64_t p,
    int64_t n_grp, const int32_t *__restrict__ grp_tile_ptr, const int32_t *__restrict__ grp_src_ptr,
    const int32_t *__restrict__ grp_src_rows, const int64_t *__restrict__ sub_ptr,
    const int32_t *__restrict__ sub_rows, const int32_t *__restrict__ sub_slot,
    const float *__restrict__ sub_wself, const int32_t *__restrict__ pos_slot,
    const uint32_t *__restrict__ pos_mask, const float *__restrict__ pos_w, int tl_flags,
    const int32_t *__restrict__ seg_ptr, const int32_t *__restrict__ seg,
    const float *__restrict__ seg_w, const int32_t *__restrict__ mf_ptr,
    const int32_t *__restrict__ mf, int mf_waves, const int32_t *__restrict__ rem_rows) {
    // RS = column pairs per item and staged row: 64 (all lanes), or 60 / 48 so that another block
    // fits a CU's LDS (niidmix_mix_tile_lds_f32); lanes >= RS compute nothing that is stored
    constexpr int rs = RS;
    // tl_flags: bit 0 average only (no z term), bit 1 every tile walks all 16 rows (tuning A/B of
    // the walker's 8- / 4-row loops)
    const bool avg_only = (tl_flags & 1) != 0;
    const bool small_loops = (tl_flags & 2) == 0;
    constexpr int64_t CW = 2 * RS;               // columns per item
    constexpr uint32_t FULL = (uint32_t)((1ull << RT) - 1ull);
    constexpr int D = 4;                         // positions read together
    extern __shared__ float lds_tile[];          // [n_src][64] column pairs
    f2 *stage = reinterpret_cast<f2 *>(lds_tile);
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = wave_id();
    const int n_waves = (int)(blockDim.x >> 6);
    const int64_t t = blockIdx.x;
    const int64_t xcd = t & 7, local = t >> 3;
    const int64_t chunk = (local / n_grp) * 8 + xcd;
    const int64_t grp = local % n_grp;
    const int64_t c0 = chunk * CW;
    if (c0 >= p) return;                         // block-uniform; no barrier reached yet
    // 1. stage the group's source rows: SV floats per piece, pieces of one row are contiguous
    if (NIIDMIX_TLDS_SPLIT != 2) {
        constexpr int PPR = (int)(CW / SV);      // pieces per row
        const int s0 = grp_src_ptr[grp], ns = grp_src_ptr[grp + 1] - s0;
        const int total = ns * PPR;
        float *st = lds_tile;
        if constexpr (SV == 4 && NIIDMIX_TLDS_GLDS) {
            // LDS-DMA (global_load_lds_dwordx4): piece i of the stage lands at byte 16 i, so one
            // wave-instruction's 64 pieces are the lane-linear 1 KiB the instruction writes; the
            // per-lane source address gathers the rows.  The pieces of up to NB wave-instructions per
            // wave are in flight at once, with no VGPR round trip; __syncthreads() below waits for
            // them (vmcnt(0)).  Their row indices are loaded first, a batch at a time: hipcc waits
            // vmcnt(0) at the first use of a plain load's result while an LDS-DMA is in flight, so an
            // index load between two DMAs would drain the first.
            typedef __attribute__((address_space(3))) void lds_void;
            typedef __attribute__((address_space(1))) void glb_void;
            constexpr int NB = 8;
            const int step = n_waves * kWave;
            if constexpr (kWave % PPR == 0) {
                // a wave-instruction's 64 pieces are kWave / PPR whole rows (128-column items:
                // two), so a lane's piece -- its column offset -- is the same in every one: the
                // per-DMA address is one 32 x 32 -> 64-bit multiply-add on the row index (the
                // general form below spends ~23 VALU per DMA on divisions and 64-bit clamps)
                const int piece = lane % PPR;
                const int64_t cl = c0 + (int64_t)piece * 4;
                const uint64_t xl = reinterpret_cast<uint64_t>(x + (cl < p ? cl : c0));
                const uint32_t ldx4 = (uint32_t)ld_x * 4u;      // row pitch in bytes < 2^32
                                                                // (launcher: ld_x < 2^30)
                for (int b0 = wave * kWave; b0 < total; b0 += NB * step) {
                    int rowi[NB];
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        const int slot = (b0 + u * step) / PPR + lane / PPR;   // rows past the
                        rowi[u] = grp_src_rows[s0 + (slot < ns ? slot : ns - 1)]; // stage: any
                    }
                    uint64_t src[NB];
#pragma unroll
                    for (int u = 0; u < NB; ++u)
                        src[u] = xl + (uint64_t)(uint32_t)rowi[u] * ldx4;   // v_mad_u64_u32
                    asm volatile("" ::"v"(src[0]), "v"(src[1]), "v"(src[2]), "v"(src[3]), "v"(src[4]),
                                 "v"(src[5]), "v"(src[6]), "v"(src[7]));
#pragma unroll
                    for (int u = 0; u < NB; ++u) {
                        const int i0 = b0 + u * step;
                        if (i0 < total)
                            __builtin_amdgcn_global_load_lds(reinterpret_cast<glb_void *>(src[u]),
                                                             (lds_void *)(st + 4 * i0), 16, 0, 0);
                    }
                }
            } else
            for (int b0 = wave * kWave; b0 < total; b0 += NB * step) {
                int rowi[NB];
#pragma unroll
                for (int u = 0; u < NB; ++u) {
                    const int i = b0 + u * step + lane;
                    rowi[u] = grp_src_rows[s0 + (i < total ? i : total - 1) / PPR];
                }
                const float *src[NB];
#pragma unroll
                for (int u = 0; u < NB; ++u) {
                    const int i = b0 + u * step + lane;
                    const int ii = i < total ? i : total - 1;       // lanes past the stage: a valid
                    const int piece = ii - (ii / PPR) * PPR;        // source; they land in the slack
                    const int64_t c = c0 + (int64_t)piece * 4;
                    const int64_t cc = c < p ? c : c0;              // columns past p: any valid data
                    src[u] = x + (int64_t)rowi[u] * ld_x + cc;
                }
                // every index consumed before the first DMA: the empty asm uses all addresses
                // here, so no index load sinks between two DMAs (where it would cost a vmcnt(0))
                asm volatile("" ::"v"(src[0]), "v"(src[1]), "v"(src[2]), "v"(src[3]), "v"(src[4]),
                             "v"(src[5]), "v"(src[6]), "v"(src[7]));
                static_assert(NB == 8, "the asm above names NB addresses");
#pragma unroll
                for (int u = 0; u < NB; ++u) {
                    const int i0 = b0 + u * step;                   // wave-uniform: whole 1 KiB
                    if (i0 < total)                                 // pieces (tlds_slack covers the
                        __builtin_amdgcn_global_load_lds(           // last one's overhang)
                            (glb_void *)src[u], (lds_void *)(st + 4 * i0), 16, 0, 0);
                }
            }
        } else
        for (int i0 = 0; i0 < total; i0 += 4 * (int)blockDim.x) {
            float v[4][SV];
            int at[4];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int i = i0 + k * (int)blockDim.x + (int)threadIdx.x;
                const int ii = i < total ? i : total - 1;            // clamped: loads unconditional
                const int slot = ii / PPR, piece = ii - slot * PPR;
                const int64_t c = c0 + (int64_t)piece * SV;
                const int64_t cc = c < p ? c : c0;                  // columns past p: any valid data
                ldv<SV>(x + (int64_t)grp_src_rows[s0 + slot] * ld_x + cc, v[k]);
                at[k] = i < total ? slot * (int)CW + piece * SV : -1;
            }
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (at[k] >= 0) {
                    if constexpr (SV == 4)
                        *reinterpret_cast<float4 *>(st + at[k]) = make_float4(v[k][0], v[k][1], v[k][2], v[k][3]);
                    else
                        *reinterpret_cast<float2 *>(st + at[k]) = make_float2(v[k][0], v[k][1]);
                }
        }
    }
    // register rows of this wave's tile (plans with rem_rows): loaded while the stage lands, so
    // the barrier's wait covers them; lanes past the item re-read a valid column
    constexpr bool REM = NREM > 0;
    typename RemRegs<NREM ? NREM : 16>::V rem;
    if constexpr (REM) {
        const int sub = grp_tile_ptr[grp] + wave;
        const int subc = sub < grp_tile_ptr[grp + 1] ? sub : grp_tile_ptr[grp];
        const int sl_ = lane < rs ? lane : rs - 1;
        const int64_t cr = c0 + 2 * sl_ < p ? c0 + 2 * sl_ : c0;
#pragma unroll
        for (int r = 0; r < (NREM ? NREM : 1); ++r) {
            // -1 (unused, never read by the walker) loads row 0: skipping the load instead (a
            // branch per slot) cost 21 more VGPRs for 8 register rows and spilled the 16-row kernel
            // to scratch (2.95 -> 3.46 / 3.07 -> 12.7 ms)
            const int row = rem_rows[subc * 16 + r];
            const f2 v = *reinterpret_cast<const f2 *>(x + (int64_t)(row < 0 ? 0 : row) * ld_x + cr);
            rem[2 * r] = v.x;
            rem[2 * r + 1] = v.y;
        }
    }
    __syncthreads();
    if constexpr (NIIDMIX_TLDS_MF && EXACT && SEG && RT == 16 && NIIDMIX_TLDS_SPLIT == 0 && !REM) {
        // 2'. Matrix-core path (exact): v_mfma_f32_16x16x4_f32 applies 4 positions to the tile's 16
        // rows x 16 columns at a time as a k-ordered chain of single-rounding fmas: A[col][k] =
        // fl(w_k * x_k[col]), B[k][row] = 1 if the row takes position k else 0, so a row that
        // takes k gets fl(acc + fl(w x)) -- bit for bit the reference's add_(w*p) -- and the
        // others acc + (+-0), which is acc unless acc is -0 or the product is not finite.  Hence
        // the block-wide check: every staged value finite with |x| >= 1e-30 (each row's
        // accumulator is then non-zero from its self term on); otherwise the block falls back to
        // the segment walker below.  Position lists: niidmix.tile.build_tile_mfma_positions.
        // Lane l holds D[i = 4 (l >> 4) + r][j = l & 15]: tile row j, parameter columns
        // 8 i + cb (cb: the 8 accumulators), i.e. the 32 consecutive columns 32 (l >> 4) .. +31.
        // mf_waves >= 0: waves [0, mf_waves) of every block on the matrix cores; mf_waves = -k:
        // every k-th column chunk's blocks entirely on the matrix cores, the other blocks walk
        // segments (no matrix-core preamble), so the two pipes are fed by different blocks
        const bool mf_item = mf_waves >= 0 || chunk % (int64_t)(-mf_waves) == 0;
        // MF: a separate instance, so the walker-only kernel keeps the walker's register count
        // (the pipelined matrix-core path needs 91 VGPRs: two 7-wave blocks per CU instead of three)
        if (MF && mf_ptr != nullptr && mf_item) {
            bool bad = false;
            {
                const int nf = (grp_src_ptr[grp + 1] - grp_src_ptr[grp]) * (int)CW;
                for (int i = 4 * (int)threadIdx.x; i < nf; i += 4 * (int)blockDim.x) {
                    const float4 v = *reinterpret_cast<const float4 *>(lds_tile + i);
                    const float m0 = fminf(fminf(fabsf(v.x), fabsf(v.y)), fminf(fabsf(v.z), fabsf(v.w)));
                    const float m1 = fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
                    // NaN: fminf / fmaxf drop it, so test each value too
                    bad |= !(m0 >= 1e-30f) || !(m1 <= 3.4028235e38f) ||
                           (v.x != v.x) || (v.y != v.y) || (v.z != v.z) || (v.w != v.w);
                }
            }
            if (!__syncthreads_or(bad)) {
                typedef float f4v __attribute__((ext_vector_type(4)));
                const int jr = lane & 15, g4 = lane >> 4;
                const int tb = grp_tile_ptr[grp], te = grp_tile_ptr[grp + 1];
                // a block has at most one tile per wave (64 * max_tiles threads)
                const int sub = tb + wave;
                const bool have = sub < te;                                  // wave-uniform
                const int li = lane < RT ? lane : RT - 1;
                const int d_row = have ? sub_rows[sub * RT + li] : -1;
                const int d_slot = have ? sub_slot[sub * RT + li] : 0;
                const float d_ws = have ? sub_wself[sub * RT + li] : 0.f;
                const int row_j = __shfl(d_row, jr), slot_j = __shfl(d_slot, jr);
                const float ws_j = __shfl(d_ws, jr);
                float *srow = lds_tile + slot_j * (int)CW + 32 * g4;
                // waves [0, mf_waves) take the matrix cores, the others the segment walker: the two
                // pipes run side by side (a wave on either stores its rows itself)
                const bool mfw = wave < (mf_waves >= 0 ? mf_waves : n_waves);
                const int64_t colw = c0 + 2 * lane;
                const bool okw = lane < rs && colw < p;
                const int slw = lane < rs ? lane : rs - 1;
                if (have && !mfw) {
                    typedef __attribute__((address_space(3))) float lds_float_w;
                    const unsigned lds_base = (unsigned)(size_t)(lds_float_w *)lds_tile;
                    TileAcc<16> wacc;
                    const int l8w = slw * (int)sizeof(f2);
                    tlds16_init<EXACT>(wacc.v[0], d_slot, __float_as_int(d_ws), rs * (int)sizeof(f2),
                                       (int)lds_base, l8w);
                    const int sb0 = seg_ptr[sub], sb1 = seg_ptr[sub + 1];
                    tlds16_walk<EXACT, rs * (int)sizeof(f2)>(wacc.v[0], seg, sb0, sb1, (int)lds_base,
                                                             __float_as_int(seg_w[2 * sub]),
                                                             __float_as_int(seg_w[2 * sub + 1]), l8w, lane, 16);
#pragma unroll
                    for (int r = 0; r < RT; ++r) {
                        const int row = __builtin_amdgcn_readlane(d_row, r);
                        if (row < 0) continue;                               // wave-uniform
                        f2 o = wacc.get(r);
                        if (!avg_only) {
                            const f2 xs = stage[__builtin_amdgcn_readlane(d_slot, r) * rs + slw];
                            o = xs * 0.f + o;
                        }
                        if (okw) {
                            float *dst = y + (int64_t)row * ld_y + colw;
                            __builtin_nontemporal_store(o.x, dst);
                            __builtin_nontemporal_store(o.y, dst + 1);
                        }
                    }
                }
                f4v acc[8];
                if (have && mfw) {
#pragma unroll
                    for (int r = 0; r < 4; ++r) {                            // self: z + fl(ws * xs)
                        const float4 a = *reinterpret_cast<const float4 *>(srow + 8 * r);
                        const float4 b = *reinterpret_cast<const float4 *>(srow + 8 * r + 4);
                        const float xs[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                        for (int cb = 0; cb < 8; ++cb) acc[cb][r] = xs[cb] * 0.f + ws_j * xs[cb];
                    }
                    // Positions in groups of 4 (one 16x16x4 MFMA k-block per column block),
                    // software-pipelined: the descriptors (slot, weight, row mask) of group q + 1
                    // come by ds_bpermute and its rows by ds_read while group q's products and
                    // MFMAs issue, and the descriptor words of the next 64 positions are loaded
                    // one chunk ahead (round 3 waited for both at every group: ~45 % of a
                    // group's 256 MFMA cycles, profiles/r04/exact_mfma_pipelined.txt)
                    const int e0 = mf_ptr[sub], e1 = mf_ptr[sub + 1];
                    const int npos = e1 - e0;                                  // a multiple of 4
                    auto ldd = [&](int off) {                                  // 64 positions' words
                        const int cnt = npos - off < 64 ? npos - off : 64;
                        return reinterpret_cast<const int4 *>(mf)[e0 + off + (lane < cnt ? lane : cnt - 1)];
                    };
                    int4 dc = ldd(0);
                    int4 dn = npos > 64 ? ldd(64) : dc;
                    auto desc = [&](const int4 &d, int q, int &slot, float &w, float &bv) {
                        const int src = (q & 63) + g4;                         // position q + k, k = l >> 4
                        slot = __shfl(d.x, src);
                        w = __int_as_float(__shfl(d.y, src));
                        const uint32_t m = (uint32_t)__shfl(d.z, src);
                        bv = ((m >> jr) & 1u) ? 1.f : 0.f;
                    };
                    // two-deep: group q's rows are in registers and group q + 4's descriptors
                    // too; each iteration issues the rows of group q + 4 (address known a group
                    // ahead) and the descriptors of group q + 8 before group q's MFMAs
                    int slot, slot1;
                    float w, bv, w1, bv1;
                    desc(dc, 0, slot, w, bv);
                    {
                        const int q1 = 4 < npos ? 4 : 0;
                        desc(q1 < 64 ? dc : dn, q1, slot1, w1, bv1);
                    }
                    const float *xr = lds_tile + slot * (int)CW + 8 * jr;
                    float4 x0 = *reinterpret_cast<const float4 *>(xr);
                    float4 x1 = *reinterpret_cast<const float4 *>(xr + 4);
                    int base = 0;                  // dc holds positions [base, base + 64), dn the next 64
                    for (int q = 0; q < npos; q += 4) {
                        if (NIIDMIX_MF_SPLIT == 3) break;                     // tuning builds only
                        // rows of group q + 4 (a dummy re-read of group q's on the last group)
                        const float *xrn = lds_tile + slot1 * (int)CW + 8 * jr;
                        const float4 y0 = *reinterpret_cast<const float4 *>(xrn);
                        const float4 y1 = *reinterpret_cast<const float4 *>(xrn + 4);
                        // descriptors of group q + 8
                        const int q2 = q + 8 < npos ? q + 8 : q;
                        if (q2 >= base + 64) {                                 // wave-uniform
                            dc = dn;
                            base += 64;
                            if (base + 64 < npos) dn = ldd(base + 64);
                        }
                        int slot2;
                        float w2, bv2;
                        desc(q2 >= base ? dc : dn, q2, slot2, w2, bv2);
                        const float a[8] = {w * x0.x, w * x0.y, w * x0.z, w * x0.w,
                                            w * x1.x, w * x1.y, w * x1.z, w * x1.w};
#pragma unroll
                        for (int cb = 0; cb < 8; ++cb)
                            acc[cb] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[cb], bv, acc[cb], 0, 0, 0);
                        x0 = y0;
                        x1 = y1;
                        w = w1;
                        bv = bv1;
                        slot1 = slot2;
                        w1 = w2;
                        bv1 = bv2;
                    }
                    // update_models: o = z + acc (z from the row's own staged value), in place
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const float4 a = *reinterpret_cast<const float4 *>(srow + 8 * r);
                        const float4 b = *reinterpret_cast<const float4 *>(srow + 8 * r + 4);
                        const float xs[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
                        for (int cb = 0; cb < 8; ++cb)
                            if (!avg_only) acc[cb][r] = xs[cb] * 0.f + acc[cb][r];
                    }
                }
                // Stores: a lane holds 32 consecutive columns of ONE row, so storing from here would
                // write 64 rows' 8-16 B pieces per instruction (measured 25 ms per round).  Once every
                // wave is done reading the stage, each row's result goes to its own staged row
                // (distinct slots: a group's rows are distinct), then is stored row by row with the
                // walker's coalesced pattern (lane = column pair).
                __syncthreads();
                if (have && mfw && row_j >= 0) {
#pragma unroll
                    for (int r = 0; r < 4; ++r)
                        if (32 * g4 + 8 * r < (int)CW) {                     // CW: a multiple of 8
                            *reinterpret_cast<float4 *>(srow + 8 * r) =
                                make_float4(acc[0][r], acc[1][r], acc[2][r], acc[3][r]);
                            *reinterpret_cast<float4 *>(srow + 8 * r + 4) =
                                make_float4(acc[4][r], acc[5][r], acc[6][r], acc[7][r]);
                        }
                }
                if (have && mfw) {
                    const int64_t col = colw;
                    const bool okc = okw;
                    const int slc = slw;
#pragma unroll
                    for (int r = 0; r < RT; ++r) {
                        const int row = __builtin_amdgcn_readlane(d_row, r);
                        if (row < 0) continue;                               // wave-uniform
                        const f2 o = stage[__builtin_amdgcn_readlane(d_slot, r) * rs + slc];
                        if (okc) {
                            float *dst = y + (int64_t)row * ld_y + col;
                            __builtin_nontemporal_store(o.x, dst);
                            __builtin_nontemporal_store(o.y, dst + 1);
                        }
                    }
                }
                return;                                                      // block-uniform
            }
        }
    }
    const int64_t col = c0 + 2 * lane;
    const bool ok = lane < rs && col < p;        // p even: a lane's pair is all-in or all-out
    // LDS column index of this lane: lanes >= rs (120- / 96-column items) compute nothing that is
    // stored; they re-read column pair rs-1 so that no read leaves the staged row (the last slot
    // of a group would otherwise read past the dynamic LDS allocation)
    const int sl = lane < rs ? lane : rs - 1;
    const int tb = grp_tile_ptr[grp], te = grp_tile_ptr[grp + 1];
    typedef __attribute__((address_space(3))) float lds_float;
    const unsigned lds_base = (unsigned)(size_t)(lds_float *)lds_tile;   // LDS byte offset of stage
    const int lane8 = sl * (int)sizeof(f2);
    for (int sub = tb + wave; sub < te; sub += n_waves) {
        const int li = lane < RT ? lane : RT - 1;
        const int d_row = sub_rows[sub * RT + li];
        const int d_slot = sub_slot[sub * RT + li];
        const float d_ws = sub_wself[sub * RT + li];
        TileAcc<RT> acc;
        if constexpr (SEG && RT == 16 && NIIDMIX_TLDS_ASM && (NIIDMIX_TLDS_SPLIT == 0 || NIIDMIX_TLDS_SPLIT == 2)) {
            tlds16_init<EXACT>(acc.v[0], d_slot, __float_as_int(d_ws), rs * (int)sizeof(f2), (int)lds_base, lane8);
        } else {
#pragma unroll
            for (int r = 0; r < RT; ++r) {
                const f2 xs = stage[__builtin_amdgcn_readlane(d_slot, r) * rs + sl];
                const float ws = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d_ws), r));
                acc.set(r, axpy2<EXACT>(ws, xs, xs * 0.f));
            }
        }
        if constexpr (SEG && RT == 16 && NIIDMIX_TLDS_ASM && (NIIDMIX_TLDS_SPLIT == 0 || NIIDMIX_TLDS_SPLIT == 2)) {
            {                                                            // segment loop (tile.py)
                const int sb0 = seg_ptr[sub], sb1 = seg_ptr[sub + 1];
                const int w0 = __float_as_int(seg_w[2 * sub]), w1 = __float_as_int(seg_w[2 * sub + 1]);
                // rows updated per run position: the tile's used slots (9-16 exactly, else rounded up
                // to 4 / 8; wave-uniform; the slots above are unused and never stored)
                const uint64_t used = __ballot(lane < RT && d_row >= 0);
                const int hi = used ? 64 - __builtin_clzll(used) : 1;
                const int nr = __builtin_amdgcn_readfirstlane(
                    !small_loops ? 16 : hi <= 4 ? 4 : hi <= 8 ? 8 : hi);
                // segment words (int4 each): a run: first slot | length << 12 | first skipped row << 20,
                // weight-select bits, skip bits; a MASKED position: slot | 1 << 30, the rows that take
                // it, its weight (fp32 bits).  One walker for every tile: walkers specialised by the
                // tile's row count (4 / 8 / 12 / 16 pairs) measured no faster, and their four call
                // sites made hipcc keep a second copy of the tuple (90 VGPRs, two blocks per CU)
                if constexpr (REM && REM2) {
                    // two phases: the first segment reading register row 8..15 (a masked entry
                    // with SEG_REMOTE and index >= 8; the plan reads rows 0..7 only before it,
                    // niidmix.tile.rem_two_phase) splits the walk; rows 8..15 replace 0..7 there
                    int sm = sb1;
                    for (int b = sb0; b < sb1; b += kWave) {
                        const int i = b + lane;
                        const int dx = i < sb1 ? seg[4 * i] : 0;
                        const uint64_t hit = __ballot((dx & (3 << 29)) == (3 << 29) && (dx & 0xfff) >= 8);
                        if (hit) { sm = b + __builtin_ctzll(hit); break; }
                    }
                    tlds16_walk_rem<EXACT, rs * (int)sizeof(f2), 8>(acc.v[0], seg, sb0, sm, (int)lds_base,
                                                                     w0, w1, lane8, lane, nr, rem);
                    if (sm < sb1) {
                        const int sl_ = lane < rs ? lane : rs - 1;
                        const int64_t cr = c0 + 2 * sl_ < p ? c0 + 2 * sl_ : c0;
#pragma unroll
                        for (int r = 0; r < 8; ++r) {
                            const int row = rem_rows[sub * 16 + 8 + r];
                            const f2 v = *reinterpret_cast<const f2 *>(x + (int64_t)(row < 0 ? 0 : row) * ld_x + cr);
                            rem[2 * r] = v.x;
                            rem[2 * r + 1] = v.y;
                        }
                        tlds16_walk_rem<EXACT, rs * (int)sizeof(f2), 8>(acc.v[0], seg, sm, sb1, (int)lds_base,
                                                                         w0, w1, lane8, lane, nr, rem);
                    }
                } else if constexpr (REM)
                    tlds16_walk_rem<EXACT, rs * (int)sizeof(f2), (NREM ? NREM : 16)>(acc.v[0], seg, sb0, sb1, (int)lds_base, w0,
                                                                 w1, lane8, lane, nr, rem);
                else
                    tlds16_walk<EXACT, rs * (int)sizeof(f2)>(acc.v[0], seg, sb0, sb1, (int)lds_base, w0, w1,
                                                             lane8, lane, nr);
                goto tile_epilogue;
            }
        }
        {
        const bool pad_slot = __builtin_amdgcn_readlane(d_row, RT - 1) < 0;   // slot RT-1 unused
        const int64_t beg = sub_ptr[sub], end = sub_ptr[sub + 1];
        for (int64_t kb = beg; NIIDMIX_TLDS_SPLIT != 1 && kb < end; kb += 64) {
            // 64 positions' (slot, mask, uniform weight) fetched lane-parallel and handed out by
            // v_readlane: the position loop issues no scalar or global loads (only per-row weights
            // of a non-uniform position are read from pos_w)
            const int cnt = (int)(end - kb < 64 ? end - kb : 64);
            const int lj = lane < cnt ? lane : cnt - 1;
            const int d_src = pos_slot[kb + lj];
            const int d_mask = (int)pos_mask[kb + lj];
            const int d_wu = __float_as_int(pos_w[(kb + lj) * RT]);
            // per-chunk bit sets (one ballot each) instead of per-position v_readlane tests
            // A SIMPLE position — uniform weight, taken by every tile row but at most one (d_skip;
            // the pad slot RT-1 when every row takes it) — needs no per-position test: save the
            // skipped row, update every row, restore it (bit-exact).  A tile row is never its own
            // source, so a clique tile's partial positions are mostly its rows' own positions: with
            // a pad slot (tiles of <= RT-1 rows, niidmix.tile) most positions are simple.  32-row
            // tiles (two register halves make the dynamic row index a branch) test each position.
            const uint32_t miss = ~(uint32_t)d_mask & FULL;
            const bool simple = (d_src & kPosUniform) != 0 && (miss & (miss - 1u)) == 0u && (miss != 0u || pad_slot);
            if constexpr (RT == 16 && NIIDMIX_TLDS_ASM && NIIDMIX_TLDS_SPLIT == 0) {
                // Runs of positions with a uniform weight that every row or all rows but one take
                // go through tlds16_run (hand-scheduled, accumulators in place); any other
                // position (rare) through the per-row form.
                const bool easy = (d_src & kPosUniform) != 0 && (miss & (miss - 1u)) == 0u;
                const uint64_t hard_bits = __ballot(lane < cnt && !easy);
                const int v_meta = ((d_src & kPosRowMask) * (rs * (int)sizeof(f2)) + (int)lds_base) |
                                   (miss ? (2 * __builtin_ctz(miss) + 2) << 24 : 0);
                int j = 0;
                while (j < cnt) {
                    const uint64_t rest = hard_bits >> j;                // j < 64
                    const int stop = rest ? j + __builtin_ctzll(rest) : cnt;
                    if (stop > j) {
                        tlds16_run<EXACT>(acc.v[0], j, stop, v_meta, d_wu, lane8);
                        j = stop;
                    }
                    if (j < cnt) {                                       // one hard position
                        const int sj = __builtin_amdgcn_readlane(d_src, j);
                        const f2 xu = stage[(sj & kPosRowMask) * rs + sl];
                        const uint32_t m = (uint32_t)__builtin_amdgcn_readlane(d_mask, j) & FULL;
                        const float wu = __int_as_float(__builtin_amdgcn_readlane(d_wu, j));
                        const float *wp = pos_w + (kb + j) * RT;
                        for (uint32_t b = m; b; b &= b - 1u) {
                            const int r = __builtin_ctz(b);
                            acc.set(r, axpy2<EXACT>((sj & kPosUniform) ? wu : wp[r], xu, acc.get(r)));
                        }
                        ++j;
                    }
                }
                continue;
            }
            if (RT <= 16 && NIIDMIX_TLDS_SPLIT == 0) {
                const int d_skip = miss ? __builtin_ctz(miss) : RT - 1;
                // SIMPLE position: save the skipped row, update all rows in place, restore it
                auto update = [&](float w, f2 xu) {
                    if (EXACT) {
                        f2 tp = xu * w;                           // one product for the tile
                        asm("" : "+v"(tp));                       // kept as one pair, not re-formed per row
                        acc.add_all(tp);
                    } else {
                        acc.fma_all(w, xu);
                    }
                };
                auto step = [&](int jj, f2 xu) {
                    const int r0 = __builtin_amdgcn_readlane(d_skip, jj);
                    const float w = __int_as_float(__builtin_amdgcn_readlane(d_wu, jj));
                    const f2 keep = acc.get(r0);
                    update(w, xu);
                    acc.set(r0, keep);
                };
                // every row takes it: no save/restore
                auto step_full = [&](int jj, f2 xu) {
                    update(__int_as_float(__builtin_amdgcn_readlane(d_wu, jj)), xu);
                };
                // any other position (a row taking it alone, a source two rows order differently,
                // a per-row weight; rare): visit only the mask's rows, by dynamic register index
                const uint64_t uni_bits = __ballot(lane < cnt && (d_src & kPosUniform) != 0);
                auto general = [&](int jj, f2 xu) {
                    const uint32_t m = (uint32_t)__builtin_amdgcn_readlane(d_mask, jj) & FULL;
                    const bool uni = ((uni_bits >> jj) & 1ull) != 0;
                    const float wu = __int_as_float(__builtin_amdgcn_readlane(d_wu, jj));
                    const float *wp = pos_w + (kb + jj) * RT;
                    for (uint32_t b = m; b; b &= b - 1u) {
                        const int r = __builtin_ctz(b);
                        acc.set(r, axpy2<EXACT>(uni ? wu : wp[r], xu, acc.get(r)));
                    }
                };
                // groups of D positions with the LDS reads of the next group in flight; no exit
                // inside a group (an early exit would give every exit its own register copy); SGPR
                // bit test per group: all D taken by every row -> no save/restore at all (most
                // groups); otherwise per position: simple -> save/restore, else the slow form.
                // (A third form for all-simple groups measured the same: 4.80 vs 4.79 ms.)
                const uint64_t slow_bits = __ballot(lane < cnt && !simple);
                const uint64_t part_bits = slow_bits | __ballot(lane < cnt && miss != 0u);
                const int d_addr = (d_src & kPosRowMask) * rs;   // LDS f2 index of each position
                const int nd = cnt & ~(D - 1);
                f2 xa[D], xb[D];
#pragma unroll
                for (int u = 0; u < D; ++u)
                    xa[u] = stage[__builtin_amdgcn_readlane(d_addr, u) + sl];
                for (int j = 0; j < nd; j += D) {
#pragma unroll
                    for (int u = 0; u < D; ++u)
                        xb[u] = stage[__builtin_amdgcn_readlane(d_addr, j + D + u) + sl];
                    constexpr uint64_t GM = (1ull << D) - 1ull;
                    if (((part_bits >> j) & GM) == 0ull) {        // all D taken by every row
#pragma unroll
                        for (int u = 0; u < D; ++u) step_full(j + u, xa[u]);
                    } else {
#pragma unroll
                        for (int u = 0; u < D; ++u) {
                            if ((slow_bits >> (j + u)) & 1ull) general(j + u, xa[u]);
                            else step(j + u, xa[u]);
                        }
                    }
#pragma unroll
                    for (int u = 0; u < D; ++u) xa[u] = xb[u];
                }
                for (int j = nd; j < cnt; ++j) {                  // the chunk's last cnt % D
                    const f2 xu = stage[__builtin_amdgcn_readlane(d_addr, j) + sl];
                    if ((slow_bits >> j) & 1ull) general(j, xu);
                    else step(j, xu);
                }
                continue;
            }
            // the uniform flag as one ballot per chunk; the mask comes by v_readlane and is tested
            // by SALU compares only (a bool kept as a lane mask would cost a SALU->VALU mask
            // round trip per position)
            const uint64_t uni_bits = __ballot(lane < cnt && (d_src & kPosUniform) != 0);
            // LDS reads double-buffered: batch j+D is read while batch j is applied
            f2 xa[D], xb[D];
#pragma unroll
            for (int u = 0; u < D; ++u)
                xa[u] = stage[(__builtin_amdgcn_readlane(d_src, u < cnt ? u : cnt - 1) & kPosRowMask) * rs + sl];
            for (int j = 0; j < cnt; j += D) {
#pragma unroll
                for (int u = 0; u < D; ++u) {
                    const int jn = j + D + u < cnt ? j + D + u : cnt - 1;
                    xb[u] = stage[(__builtin_amdgcn_readlane(d_src, jn) & kPosRowMask) * rs + sl];
                }
#pragma unroll
                for (int u = 0; u < D; ++u) {
                    if (j + u >= cnt) break;
                    const f2 xu = xa[u];
                    if constexpr (NIIDMIX_TLDS_SPLIT >= 3) {   // tuning builds: loop-cost decomposition
                        f2 tp = xu;
                        if (NIIDMIX_TLDS_SPLIT == 3) tp = xu * __int_as_float(__builtin_amdgcn_readlane(d_wu, j + u));
                        asm("" : "+v"(tp));
                        if (NIIDMIX_TLDS_SPLIT == 5) acc.set(0, acc.get(0) + tp);
                        else
#pragma unroll
                            for (int r = 0; r < RT; ++r) acc.set(r, acc.get(r) + tp);
                        continue;
                    }
                    const uint32_t m = (uint32_t)__builtin_amdgcn_readlane(d_mask, j + u);
                    if ((uni_bits >> (j + u)) & 1ull) {
                        const float w = __int_as_float(__builtin_amdgcn_readlane(d_wu, j + u));
                        if (EXACT) {
                            f2 tp = xu * w;                       // one product for the tile
                            asm("" : "+v"(tp));                   // kept as one pair, not re-formed per row
                            apply_mask<RT>(acc, m, [&](f2 a, int) { return a + tp; });
                        } else {
                            apply_mask<RT>(acc, m, [&](f2 a, int) { return axpy2<false>(w, xu, a); });
                        }
                    } else {
                        const float *wp = pos_w + (kb + j + u) * RT;
                        apply_mask<RT>(acc, m, [&](f2 a, int r) { return axpy2<EXACT>(wp[r], xu, a); });
                    }
                }
#pragma unroll
                for (int u = 0; u < D; ++u) xa[u] = xb[u];
            }
        }
        }
    tile_epilogue:
        // update_models: z + acc, z = x_self*0 (AVERAGE_ONLY: acc).  Four rows at a time: their
        // own staged values are read together (an unused slot reads slot 0), then combined and
        // stored, so the LDS latency is paid once per four rows instead of once per row
        // (avg_only is tested once, not per row: per row it became two v_cndmask per row)
        auto epilogue = [&](auto with_z) {
#pragma unroll
            for (int r0 = 0; r0 < RT; r0 += 4) {
                f2 xs[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) xs[u] = stage[sub_slot[sub * RT + r0 + u] * rs + sl];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int row = sub_rows[sub * RT + r0 + u];    // scalar loads, not v_readlane
                    if (row < 0) continue;                          // wave-uniform
                    f2 o = acc.get(r0 + u);
                    if constexpr (decltype(with_z)::value) o = xs[u] * 0.f + o;
                    if (ok) {
                        float *dst = y + (int64_t)row * ld_y + col;
                        __builtin_nontemporal_store(o.x, dst);
                        __builtin_nontemporal_store(o.y, dst + 1);
                    }
                }
            }
        };
        if (avg_only)
            epilogue(BoolC<false>{});
        else
            epilogue(BoolC<true>{});
    }
}

// ----------------------------------------------------------------------------------------------
// Streaming copy ceiling (measurement primitive, not part of the mixing path): one float4 per
// thread, non-temporal loads and stores, linear order — the access shape that measured fastest on
// MI355X (tools/hbm_probe2.hip: ~6.6 TB/s), so bench.py can report the mixing kernel against this
// box's own copy rate next to the 8 TB/s spec.
__global__ __launch_bounds__(256) void k_stream_copy(const float *__restrict__ x, float *__restrict__ y,
                                                     int64_t n4) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n4)
        __builtin_nontemporal_store(__builtin_nontemporal_load(reinterpret_cast<const f4 *>(x) + i),
                                    reinterpret_cast<f4 *>(y) + i);
}

// ----------------------------------------------------------------------------------------------
// Uniform average over rows (model/__init__.py:17-24 with weights=None): one lane per column,
// left-to-right over rows.  EXACT: mean = fl(...fl(fl(x0*0) + fl(w x0)) + ...), w = fp32(1/n).
template <bool EXACT>
__global__ __launch_bounds__(256) void k_mean_cols(const float *__restrict__ x, int64_t ld_x,
                                                   int64_t n, int64_t p, float w,
                                                   float *__restrict__ mean) {
    for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < p;
         c += (int64_t)gridDim.x * blockDim.x) {
        float acc = n > 0 ? x[c] * 0.f : 0.f;
        int64_t k = 0;
        for (; k + 8 <= n; k += 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = x[(k + u) * ld_x + c];
#pragma unroll
            for (int u = 0; u < 8; ++u) acc = axpy<EXACT>(w, v[u], acc);
        }
        for (; k < n; ++k) acc = axpy<EXACT>(w, x[k * ld_x + c], acc);
        mean[c] = acc;
    }
}

// Squared L2 distance of every row to the mean (logger.model_distance, logger.py:42-48), fp64
// accumulation, one workgroup per row, deterministic order.
__global__ __launch_bounds__(256) void k_row_dist2(const float *__restrict__ x, int64_t ld_x,
                                                   int64_t p, const float *__restrict__ mean,
                                                   double *__restrict__ dist2) {
    __shared__ double part[256];
    const int64_t row = blockIdx.x;
    double acc = 0.0;
    for (int64_t c = threadIdx.x; c < p; c += blockDim.x) {
        const double d = (double)x[row * ld_x + c] - (double)mean[c];
        acc += d * d;
    }
    part[threadIdx.x] = acc;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) part[threadIdx.x] += part[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) dist2[row] = part[0];
}

// ----------------------------------------------------------------------------------------------
// Segment gradient mean (--clique-gradient without removed edges, d_sgd.py:56-65): every member of
// a segment (clique) receives the SAME mean of the members' gradients, so each gradient row is read
// once and each output row written once — HBM-bound, 8 B per node-parameter, like k_mix_clique.
// Exact: acc = +0 (zeros_like), acc = fl(acc + g_m) in the segment's member order (add_),
// mean = fl(acc / len) (div_, true division), out = fl(+0 + mean) (update_gradients: zero_(); add_).
// Work item = (segment, chunk of 256*V columns); 256 threads, V columns per thread; member rows are
// fetched 64 at a time lane-parallel and handed out by v_readlane; U loads in flight per batch
// (NTL: non-temporal, the rows are read once).
template <int V, int U, bool NTL = false>
__global__ __launch_bounds__(256) void k_grad_segment_mean(const float *__restrict__ g, int64_t ld_g,
                                                           float *__restrict__ y, int64_t ld_y,
                                                           int64_t p, int64_t n_seg,
                                                           const int32_t *__restrict__ seg_ptr,
                                                           const int32_t *__restrict__ seg_row,
                                                           int64_t n_chunks, int cpb_shift,
                                                           int64_t bs_g, int64_t bs_y) {
    // column-blocked slabs: chunk k (256*V columns) lives in block k >> cpb_shift, block strides
    // bs_g / bs_y floats (row-major: cpb_shift = 62, one block)
    const int lane = threadIdx.x & (kWave - 1);
    for (int64_t t = blockIdx.x; t < n_seg * n_chunks; t += gridDim.x) {
        const int64_t seg = t / n_chunks;
        const int64_t chunk = t % n_chunks;
        const int64_t kb = chunk >> cpb_shift;
        const int64_t cin = (chunk - (kb << cpb_shift)) * (256 * V) + (int64_t)threadIdx.x * V;
        const int64_t c = chunk * (256 * V) + (int64_t)threadIdx.x * V;   // global column
        const bool ok = c < p;                   // p % V == 0: a thread is all-in or all-out
        const int64_t cc = ok ? cin : 0;         // loads stay unconditional
        const float *gb = g + kb * bs_g;
        float *yb = y + kb * bs_y;
        const int beg = seg_ptr[seg], end = seg_ptr[seg + 1];
        float acc[V];
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = 0.f;
        for (int kb = beg; kb < end; kb += 64) {
            const int cnt = end - kb < 64 ? end - kb : 64;
            const int d_row = seg_row[kb + (lane < cnt ? lane : cnt - 1)];
            for (int j = 0; j < cnt; j += U) {
                float v[U][V];
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    const int jj = j + u < cnt ? j + u : cnt - 1;
                    if (NTL) ldv_nt<V>(gb + (int64_t)__builtin_amdgcn_readlane(d_row, jj) * ld_g + cc, v[u]);
                    else ldv<V>(gb + (int64_t)__builtin_amdgcn_readlane(d_row, jj) * ld_g + cc, v[u]);
                }
#pragma unroll
                for (int u = 0; u < U; ++u)
                    if (j + u < cnt) {
#pragma unroll
                        for (int e = 0; e < V; ++e) acc[e] = acc[e] + v[u][e];
                    }
            }
        }
        const float len = (float)(end > beg ? end - beg : 1);
        float o[V];
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = 0.f + acc[e] / len;
        // every lane fetches the descriptors (v_readlane reads lanes that must be active): only
        // the stores are masked by `ok`
        for (int kb = beg; kb < end; kb += 64) {
            const int cnt = end - kb < 64 ? end - kb : 64;
            const int d_row = seg_row[kb + (lane < cnt ? lane : cnt - 1)];
            for (int j = 0; j < cnt; ++j) {
                float *dst = yb + (int64_t)__builtin_amdgcn_readlane(d_row, j) * ld_y + cin;
                if (ok) stv_nt<V>(dst, o);
            }
        }
    }
}

// ----------------------------------------------------------------------------------------------
// update_models(all_models, avg) of the 'sample' topology's round (d_sgd.py:246-250 via :29-35):
// every row y_i := fl(fl(x_i * 0) + avg) (p.mul_(0.); p.add_(new); y == x: in place): avg
// everywhere, except that a non-finite x_i gives NaN and a zero avg keeps the sign rule of
// (+-0) + (+-0).
template <int V>
__global__ __launch_bounds__(256) void k_update_rows(const float *x, int64_t ld_x, float *y,
                                                     int64_t ld_y, int64_t n_rows, int64_t p,
                                                     const float *__restrict__ avg, int64_t n_chunks) {
    for (int64_t t = blockIdx.x; t < n_rows * n_chunks; t += gridDim.x) {
        const int64_t r = t / n_chunks;
        const int64_t c = (t % n_chunks) * (256 * V) + (int64_t)threadIdx.x * V;
        if (c >= p) continue;
        float xv[V], av[V];
        ldv<V>(x + r * ld_x + c, xv);
        ldv<V>(avg + c, av);
#pragma unroll
        for (int e = 0; e < V; ++e) xv[e] = xv[e] * 0.f + av[e];    // two roundings (fp-contract off)
        stv_nt<V>(y + r * ld_y + c, xv);
    }
}

// ----------------------------------------------------------------------------------------------
// SGD step on listed rows (torch.optim.SGD, momentum 0, no weight decay: param.add_(grad,
// alpha=-lr), whose ATen CPU kernel computes fma(-lr, g, p) with fp32 alpha — one rounding):
//   p[row] = fma(neg_lr, g[row], p[row])    for row in rows
// The fused drop-in round runs it between the gradient mean and the mixing, on device windows.
template <int V>
__global__ __launch_bounds__(256) void k_sgd_step_rows(float *__restrict__ p, int64_t ld_p,
                                                       const float *__restrict__ g, int64_t ld_g,
                                                       int64_t ncols, const int32_t *__restrict__ rows,
                                                       int64_t n_rows, float neg_lr, int64_t n_chunks) {
    for (int64_t t = blockIdx.x; t < n_rows * n_chunks; t += gridDim.x) {
        const int64_t r = rows[t / n_chunks];
        const int64_t c = (t % n_chunks) * (256 * V) + (int64_t)threadIdx.x * V;
        if (c >= ncols) continue;
        float pv[V], gv[V];
        ldv<V>(p + r * ld_p + c, pv);
        ldv<V>(g + r * ld_g + c, gv);
#pragma unroll
        for (int e = 0; e < V; ++e) pv[e] = __builtin_fmaf(neg_lr, gv[e], pv[e]);
        if constexpr (V == 4) *reinterpret_cast<float4 *>(p + r * ld_p + c) = make_float4(pv[0], pv[1], pv[2], pv[3]);
        else p[r * ld_p + c] = pv[0];
    }
}

// ----------------------------------------------------------------------------------------------
// Halo pack of the sharded round: out[i, :] = x[rows[i], :] (the rows a peer shard reads), so that
// one contiguous send per peer carries them.
template <int V>
__global__ __launch_bounds__(256) void k_gather_rows(const float *__restrict__ x, int64_t ld_x,
                                                     const int32_t *__restrict__ rows, int64_t n_rows,
                                                     int64_t p, float *__restrict__ out, int64_t ld_o,
                                                     int64_t n_chunks) {
    for (int64_t t = blockIdx.x; t < n_rows * n_chunks; t += gridDim.x) {
        const int64_t i = t / n_chunks;
        const int64_t c = (t % n_chunks) * (256 * V) + (int64_t)threadIdx.x * V;
        if (c >= p) continue;
        float v[V];
        ldv<V>(x + (int64_t)rows[i] * ld_x + c, v);
        if constexpr (V == 4) *reinterpret_cast<float4 *>(out + i * ld_o + c) = make_float4(v[0], v[1], v[2], v[3]);
        else out[i * ld_o + c] = v[0];
    }
}

// RCCL, loaded on first use by niidmix_sharded_create (torch has usually loaded the same
// librccl.so.1 already; dlopen then returns it): the library itself never depends on it.
struct RcclApi {
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGetErrorString) error = nullptr;
};

const RcclApi *rccl_api() {
    static RcclApi api;
    static bool tried = false, ok = false;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (!tried) {
        tried = true;
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
        if (h) {
            api.init_all = reinterpret_cast<decltype(api.init_all)>(dlsym(h, "ncclCommInitAll"));
            api.destroy = reinterpret_cast<decltype(api.destroy)>(dlsym(h, "ncclCommDestroy"));
            api.group_start = reinterpret_cast<decltype(api.group_start)>(dlsym(h, "ncclGroupStart"));
            api.group_end = reinterpret_cast<decltype(api.group_end)>(dlsym(h, "ncclGroupEnd"));
            api.send = reinterpret_cast<decltype(api.send)>(dlsym(h, "ncclSend"));
            api.recv = reinterpret_cast<decltype(api.recv)>(dlsym(h, "ncclRecv"));
            api.error = reinterpret_cast<decltype(api.error)>(dlsym(h, "ncclGetErrorString"));
            ok = api.init_all && api.destroy && api.group_start && api.group_end && api.send &&
                 api.recv && api.error;
        }
    }
    return ok ? &api : nullptr;
}

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int64_t grid_for(int64_t items) { return items < kMaxGrid ? ((items + 7) / 8) * 8 : kMaxGrid; }

bool overlaps(const float *a, int64_t a_elems, const float *b, int64_t b_elems) {
    return a < b + b_elems && b < a + a_elems;
}

// NIIDMIX_CLIQUE_SKEW=<chunks> (multiple of 8; tuning): per-clique chunk rotation, 0 = off
int64_t clique_skew() {
    const char *e = getenv("NIIDMIX_CLIQUE_SKEW");
    const int64_t v = e ? atoll(e) : 0;
    return v > 0 ? (v + 7) / 8 * 8 : 0;
}

struct BlockGeom {            // column blocking of the slabs (row-major: one block)
    int bc_shift = 70;         // block_cols = 1 << bc_shift (row-major: "infinite")
    int64_t bs_x = 0, bs_y = 0;
    // (64*V)-column chunks per block = 1 << cpb_shift(V)
    int cpb_shift(int v) const { return bc_shift >= 62 ? 62 : bc_shift - (v == 4 ? 8 : v == 2 ? 7 : 6); }
};

template <int WAVES, int RPW, int G, int OCC, int RW, int FL, int V>
void launch_clique(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t p,
                   const niidmix_clique_plan *pl, int64_t n_items, hipStream_t s, const BlockGeom &bg) {
    const int64_t grid = n_items;   // one block per (clique, chunk) item; < 2^31 checked by the caller
    hipLaunchKernelGGL((k_mix_clique<WAVES, RPW, G, OCC, RW, FL, V>), dim3((unsigned)grid),
                       dim3(WAVES * 64), 0, s, x, ld_x, y, ld_y, p, pl->n_cliques, pl->clique_ptr,
                       pl->member_row, pl->member_group, pl->coef, pl->res_ptr, pl->res_col,
                       pl->res_val, pl->res_member, n_items, clique_skew(), bg.cpb_shift(V), bg.bs_x,
                       bg.bs_y, pl->csr_ptr, pl->csr_col, pl->csr_val);
}

template <int WAVES, int RPW, int OCC, int RW, int FL, int V>
int launch_clique_g(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t p,
                    const niidmix_clique_plan *pl, hipStream_t s, const BlockGeom &bg) {
    const int64_t n_chunks = (p + 64 * V - 1) / (64 * V);
    const int64_t n_items = (int64_t)pl->n_cliques * ((n_chunks + 7) / 8) * 8;
    if (n_items > 0x7fffffffLL) return set_error(NIIDMIX_EUNSUPPORTED, "too many (clique, chunk) items for one grid");
    switch (pl->n_groups) {
        case 1: launch_clique<WAVES, RPW, 1, OCC, RW, FL, V>(x, ld_x, y, ld_y, p, pl, n_items, s, bg); break;
        case 2: launch_clique<WAVES, RPW, 2, OCC, RW, FL, V>(x, ld_x, y, ld_y, p, pl, n_items, s, bg); break;
        case 3: launch_clique<WAVES, RPW, 3, OCC, RW, FL, V>(x, ld_x, y, ld_y, p, pl, n_items, s, bg); break;
        case 4: launch_clique<WAVES, RPW, 4, OCC, RW, FL, V>(x, ld_x, y, ld_y, p, pl, n_items, s, bg); break;
        default: return set_error(NIIDMIX_EUNSUPPORTED, "n_groups %d not in 1..4", pl->n_groups);
    }
    return check_launch("k_mix_clique");
}

// Multi-clique tile (k_mix_clique_q): Q cliques x 64 columns per item, 16 waves x 7 slots (cliques
// of <= 112 members).  Chosen when a 256-column chunk of all member rows (n_members KB) would not
// fit an XCD's L2; NIIDMIX_CLIQUE_Q=1 disables it, =4 forces it (A/B).
constexpr int64_t kQRowsMin = 4096;
template <int G, int W, int R, int OCC, int GA, int Q, int MS = 1>
int launch_clique_q(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t p,
                    const niidmix_clique_plan *pl, hipStream_t s, const BlockGeom &bg) {
    constexpr int64_t CW = 4 * (64 / Q);
    constexpr int CW_SHIFT = Q == 8 ? 5 : 6;
    if (bg.bc_shift < CW_SHIFT) return set_error(NIIDMIX_EINVAL, "%d-column items do not fit %d-column blocks", (int)CW, 1 << bg.bc_shift);
    const int64_t n_cg = (pl->n_cliques + Q / MS - 1) / (Q / MS);
    const int64_t n_chunks = (p + CW - 1) / CW;
    const int64_t n_items = n_cg * ((n_chunks + 7) / 8) * 8;
    if (n_items > 0x7fffffffLL) return set_error(NIIDMIX_EUNSUPPORTED, "too many (clique group, chunk) items for one grid");
    const int cpb = bg.bc_shift >= 62 ? 62 : bg.bc_shift - CW_SHIFT;
    // 32-bit row offsets when every block (column-blocked slabs) spans < 4 GiB
    const bool off32 = bg.bc_shift < 62 && bg.bs_x * 4 <= (int64_t)0xffffffffLL &&
                       bg.bs_y * 4 <= (int64_t)0xffffffffLL;
    // NIIDMIX_Q_PERSIST=k (tuning): k blocks per CU loop over the items instead of one block each
    int64_t grid = n_items;
    if (const char *e = getenv("NIIDMIX_Q_PERSIST")) {
        const int k = atoi(e);
        int dev = 0, n_cu = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1) n_cu = 256;
        if (k > 0 && (int64_t)k * n_cu < n_items) grid = (int64_t)k * n_cu / 8 * 8;
    }
#define NIIDMIX_CQ(O) hipLaunchKernelGGL((k_mix_clique_q<W, R, G, Q, OCC, GA, O, MS>), dim3((unsigned)grid), dim3(W * 64), 0, s, x, ld_x, y, ld_y, p, pl->n_cliques, pl->clique_ptr, pl->member_row, pl->member_group, pl->coef, pl->res_ptr, pl->res_col, pl->res_val, n_cg, n_items, cpb, bg.bs_x, bg.bs_y, pl->csr_ptr, pl->csr_col, pl->csr_val)
    if (off32) NIIDMIX_CQ(true); else NIIDMIX_CQ(false);
#undef NIIDMIX_CQ
    return check_launch("k_mix_clique_q");
}

template <int W, int R, int OCC, int GA, int Q = 4, int MS = 1>
int launch_clique_q_g(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t p,
                      const niidmix_clique_plan *pl, hipStream_t s, const BlockGeom &bg) {
    switch (pl->n_groups) {
        case 1: return launch_clique_q<1, W, R, OCC, GA, Q, MS>(x, ld_x, y, ld_y, p, pl, s, bg);
        case 2: return launch_clique_q<2, W, R, OCC, GA, Q, MS>(x, ld_x, y, ld_y, p, pl, s, bg);
        case 3: return launch_clique_q<3, W, R, OCC, GA, Q, MS>(x, ld_x, y, ld_y, p, pl, s, bg);
        case 4: return launch_clique_q<4, W, R, OCC, GA, Q, MS>(x, ld_x, y, ld_y, p, pl, s, bg);
        default: return set_error(NIIDMIX_EUNSUPPORTED, "n_groups %d not in 1..4", pl->n_groups);
    }
}

bool use_clique_q(const niidmix_clique_plan *pl, const BlockGeom &bg) {
    if (pl->max_clique > 112 || bg.bc_shift < 6) return false;
    if (bg.bc_shift < 8) return true;          // 64- / 128-column blocks: only this tile reads them
    if (const char *e = getenv("NIIDMIX_CLIQUE_Q")) return atoi(e) == 4;
    return pl->n_members >= kQRowsMin;
}

// Register tile per clique size: WAVES x RPW >= max_clique, OCC = waves/SIMD the register budget
// targets, RW = residual entries per wave held lane-parallel (gathered in batches, then further
// chunks of 64), FL = flags (2: non-temporal member loads), V = columns per lane (4: 256-column
// chunks).  Narrower chunks (V = 2 / 1, which would keep a 10 000-node chunk's rows in L2 for the
// gateway gathers) measured far slower: too few bytes in flight per wave (10 000 nodes: 20.5 /
// 37.9 ms vs 15.5 ms; 1000 nodes 1.57 / 2.85 vs 1.37 ms), so only V = 4 is instantiated.
// NIIDMIX_CLIQUE_TILE=<waves>x<rpw>x<occ>x<rw>x<flags>x<v> overrides the choice (tuning only).
int launch_clique_tiled(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t p,
                        const niidmix_clique_plan *pl, bool vec4, hipStream_t s,
                        const BlockGeom &bg = BlockGeom()) {
    int waves = 0, rpw = 0, occ = 0, rw = 0, ob = 0, v = 0;
    if (const char *e = getenv("NIIDMIX_CLIQUE_TILE")) sscanf(e, "%dx%dx%dx%dx%dx%d", &waves, &rpw, &occ, &rw, &ob, &v);
    const int vmax = bg.bc_shift >= 8 ? 4 : bg.bc_shift == 7 ? 2 : 1;    // chunks never straddle blocks
    if (v == 0) v = vmax;
    if (v > vmax) return set_error(NIIDMIX_EINVAL, "%d columns per lane do not fit %d-column blocks", v, 1 << bg.bc_shift);
    const int mc = pl->max_clique;
    if (!vec4) return set_error(NIIDMIX_EUNSUPPORTED, "clique kernel needs p, ld multiples of 4 and 16-B aligned slabs");
    if (waves == 0 && use_clique_q(pl, bg)) {
        // tile: <waves>x<slots>x<occupancy>x<gateway gathers per batch>; NIIDMIX_CLIQUE_QT overrides
        int qw = 0, qr = 0, qo = 0, qg = 0, qq = 4;
        if (const char *e = getenv("NIIDMIX_CLIQUE_QT")) sscanf(e, "%dx%dx%dx%dx%d", &qw, &qr, &qo, &qg, &qq);
        if (qw == 0) {
            if (mc <= 104) { qw = 8; qr = 13; qo = 4; qg = 13; }
            else { qw = 16; qr = 7; qo = 8; qg = 2; }
        }
        // NIIDMIX_CLIQUE_QM=W,R,OCC[,MS]: the member-split tile (MS lane quarters per clique,
        // default 4: one clique per item; W waves x MS quarters x R slots >= the clique)
        if (const char *e = getenv("NIIDMIX_CLIQUE_QM")) {
            int mw = 0, mr = 0, mo = 0, ms = 4;
            if (sscanf(e, "%d,%d,%d,%d", &mw, &mr, &mo, &ms) >= 3 && mw > 0) {
                if (mw * mr * ms < mc) return set_error(NIIDMIX_EINVAL, "member-split tile %dx%dx%d < %d members", mw, ms, mr, mc);
#define NIIDMIX_QM(W, R, O, M) if (mw == W && mr == R && mo == O && ms == M) return launch_clique_q_g<W, R, O, R, 4, M>(x, ld_x, y, ld_y, p, pl, s, bg)
                NIIDMIX_QM(8, 4, 4, 4); NIIDMIX_QM(16, 2, 8, 4); NIIDMIX_QM(8, 7, 4, 2); NIIDMIX_QM(16, 4, 4, 2);
#undef NIIDMIX_QM
                return set_error(NIIDMIX_EUNSUPPORTED, "no member-split tile %s", e);
            }
        }
        if (qw * qr < mc) return set_error(NIIDMIX_EINVAL, "clique tile %dx%d < %d members", qw, qr, mc);
#define NIIDMIX_QT(W, R, O, GA, QQ) if (qw == W && qr == R && qo == O && qg == GA && qq == QQ) return launch_clique_q_g<W, R, O, GA, QQ>(x, ld_x, y, ld_y, p, pl, s, bg)
        NIIDMIX_QT(8, 13, 4, 13, 4); NIIDMIX_QT(16, 7, 8, 2, 4); NIIDMIX_QT(16, 7, 8, 3, 4); NIIDMIX_QT(16, 7, 4, 7, 4);
        // 8 cliques x 32 columns per item (a chunk's rows are N x 128 B)
        NIIDMIX_QT(16, 7, 4, 7, 8); NIIDMIX_QT(16, 7, 8, 2, 8);
#undef NIIDMIX_QT
        return set_error(NIIDMIX_EUNSUPPORTED, "no multi-clique tile %dx%dx%dx%dx%d", qw, qr, qo, qg, qq);
    }
    if (waves * rpw < mc) {
        rw = 64; ob = 2; v = vmax;  // non-temporal member loads: 1.39 vs 1.47 ms (headline, same box)
        if (mc <= 16) { waves = 8; rpw = 2; occ = 8; }
        else if (mc <= 32) { waves = 8; rpw = 4; occ = 8; }
        else if (mc <= 64) { waves = 16; rpw = 4; occ = 8; }
        else if (mc <= 112) { waves = 16; rpw = 7; occ = 8; }
        else if (mc <= 128) { waves = 16; rpw = 8; occ = 4; }
        else if (mc <= 256) { waves = 16; rpw = 16; occ = 4; }
        else return set_error(NIIDMIX_EUNSUPPORTED, "clique of %d members > 256", mc);
        if (v < 4) {                // narrow-chunk tiles: instantiated for the two largest shapes
            if (mc <= 112) { waves = 16; rpw = 7; occ = 8; }
            else if (v == 2) { waves = 16; rpw = 16; occ = 4; }
            else return set_error(NIIDMIX_EUNSUPPORTED, "64-column blocks: cliques of <= 112 members "
                                  "(a 16 x 16 one-float tile spills)");
        }
    }
#define NIIDMIX_TILE(W, R, O, RWV, OB, VV) if (waves == W && rpw == R && occ == O && rw == RWV && ob == OB && v == VV) return launch_clique_g<W, R, O, RWV, OB, VV>(x, ld_x, y, ld_y, p, pl, s, bg)
    NIIDMIX_TILE(8, 2, 8, 64, 2, 4); NIIDMIX_TILE(8, 4, 8, 64, 2, 4); NIIDMIX_TILE(16, 4, 8, 64, 2, 4);
    NIIDMIX_TILE(16, 7, 8, 64, 2, 4); NIIDMIX_TILE(16, 8, 4, 64, 2, 4); NIIDMIX_TILE(16, 16, 4, 64, 2, 4);
    // tuning alternatives (all exact-result variants; the timing-only ablations FL & 4 / FL & 8 are
    // built only with -DNIIDMIX_ABLATIONS, never into the shipped library)
    NIIDMIX_TILE(16, 7, 8, 64, 0, 4); NIIDMIX_TILE(16, 7, 8, 0, 2, 4); NIIDMIX_TILE(8, 13, 4, 64, 2, 4);
    NIIDMIX_TILE(16, 7, 8, 64, 16, 4);
#ifdef NIIDMIX_ABLATIONS
    NIIDMIX_TILE(16, 7, 8, 64, 6, 4); NIIDMIX_TILE(16, 7, 8, 64, 10, 4);
#endif
#undef NIIDMIX_TILE
    return set_error(NIIDMIX_EUNSUPPORTED, "no clique tile %dx%dx%dx%dx%dx%d", waves, rpw, occ, rw, ob, v);
}

// ----------------------------------------------------------------------------------------------
// Node-state slab memory.  Measured (tools/hbm_probe7.hip): the clique access pattern (100 rows of
// a clique x 1 KiB column chunk, all cliques of a chunk in flight together) runs at 1.32 ms on
// slabs mapped from 2 MiB physical chunks through the HIP virtual-memory API on every allocation
// tried, but at 1.35-1.64 ms on hipMalloc'ed slabs depending on where the driver places them (a
// physically contiguous hipExtMallocWithFlags slab: 1.49-1.57 ms every time; a linear copy is
// unaffected).  niidmix_hbm_alloc therefore reserves a VA range and maps it chunk by chunk.
struct HbmBlock {
    size_t bytes;
    std::vector<hipMemGenericAllocationHandle_t> chunks;
    std::vector<size_t> slot;        // VA chunk slot of chunks[i]
};
// never destroyed: frees may arrive from other libraries' teardown after static destruction began
std::mutex &g_hbm_mu = *new std::mutex;
std::unordered_map<void *, HbmBlock> &g_hbm = *new std::unordered_map<void *, HbmBlock>;
constexpr size_t kHbmChunk = 2u << 20;

void hbm_release(void *va, HbmBlock &b, size_t mapped) {
    for (size_t i = 0; i < mapped; ++i) (void)hipMemUnmap((char *)va + b.slot[i] * kHbmChunk, kHbmChunk);
    for (auto h : b.chunks) (void)hipMemRelease(h);
    (void)hipMemAddressFree(va, b.bytes);
}

}  // namespace

struct niidmix_sharded {
    int n = 0;
    std::vector<int> dev;
    std::vector<ncclComm_t> comm;      // RCCL: one communicator per shard (rank = shard index)
    bool loopback = false;             // several shards share a device: device-to-device copies
    std::vector<hipEvent_t> ev_pack, ev_copy;
};

extern "C" {

void *niidmix_hbm_alloc(ssize_t size, int device, void *stream) {
    (void)stream;
    if (size <= 0) return nullptr;
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = device;
    size_t gran = 0;
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) != hipSuccess ||
        gran == 0 || kHbmChunk % gran != 0) {
        set_error(NIIDMIX_EHIP, "hbm_alloc: no usable VMM granularity");
        return nullptr;
    }
    HbmBlock b;
    const size_t n = ((size_t)size + kHbmChunk - 1) / kHbmChunk;
    b.bytes = n * kHbmChunk;
    void *va = nullptr;
    if (hipMemAddressReserve(&va, b.bytes, kHbmChunk, nullptr, 0) != hipSuccess) {
        set_error(NIIDMIX_EHIP, "hbm_alloc: VA reservation of %zu B failed", b.bytes);
        return nullptr;
    }
    b.chunks.reserve(n);
    bool ok = true;
    for (size_t i = 0; i < n && ok; ++i) {
        hipMemGenericAllocationHandle_t h;
        if (hipMemCreate(&h, kHbmChunk, &prop, 0) != hipSuccess) { ok = false; break; }
        b.chunks.push_back(h);
    }
    // chunk i goes to VA slot slot[i], a fixed pseudo-random permutation (Fisher-Yates over
    // xorshift64), so consecutive VA chunks do not sit on consecutive physical chunks even when
    // the driver hands them out in order
    std::vector<size_t> slot(b.chunks.size());
    for (size_t i = 0; i < slot.size(); ++i) slot[i] = i;
    uint64_t st = 0x9E3779B97F4A7C15ull ^ (uint64_t)n;
    for (size_t i = slot.size(); i > 1; --i) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;                 // xorshift64
        const size_t j = (size_t)(st % i);
        const size_t t = slot[i - 1]; slot[i - 1] = slot[j]; slot[j] = t;
    }
    b.slot = slot;
    size_t mapped = 0;
    for (size_t i = 0; i < b.chunks.size() && ok; ++i) {
        if (hipMemMap((char *)va + b.slot[i] * kHbmChunk, kHbmChunk, 0, b.chunks[i], 0) != hipSuccess) { ok = false; break; }
        ++mapped;
    }
    if (ok) {
        hipMemAccessDesc d = {};
        d.location.type = hipMemLocationTypeDevice;
        d.location.id = device;
        d.flags = hipMemAccessFlagsProtReadWrite;
        ok = hipMemSetAccess(va, b.bytes, &d, 1) == hipSuccess;
    }
    if (!ok) {
        hbm_release(va, b, mapped);
        set_error(NIIDMIX_EHIP, "hbm_alloc: mapping %zu B failed (out of device memory?)", b.bytes);
        return nullptr;
    }
    std::lock_guard<std::mutex> lk(g_hbm_mu);
    g_hbm.emplace(va, std::move(b));
    return va;
}

void niidmix_hbm_free(void *ptr, ssize_t size, int device, void *stream) {
    (void)size; (void)device; (void)stream;
    if (!ptr) return;
    HbmBlock b;
    {
        std::lock_guard<std::mutex> lk(g_hbm_mu);
        auto it = g_hbm.find(ptr);
        if (it == g_hbm.end()) return;
        b = std::move(it->second);
        g_hbm.erase(it);
    }
    (void)hipDeviceSynchronize();          // the caching allocator frees only idle blocks; be safe
    hbm_release(ptr, b, b.chunks.size());
}


int niidmix_abi_version(void) { return NIIDMIX_ABI_VERSION; }

const char *niidmix_last_error(void) { return g_last_error; }

int niidmix_mix_csr_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                        int64_t p, const int64_t *row_ptr, const int32_t *col, const float *val,
                        int mode, void *stream) {
    if (n_rows < 0 || p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    const int kflags = mode & (NIIDMIX_FLAG_AVERAGE_ONLY | NIIDMIX_FLAG_MEAN);
    const int low_degree = (mode & NIIDMIX_FLAG_LOW_DEGREE) ? 1 : 0;
    if ((kflags & NIIDMIX_FLAG_AVERAGE_ONLY) && (kflags & NIIDMIX_FLAG_MEAN))
        return set_error(NIIDMIX_EINVAL, "AVERAGE_ONLY and MEAN are exclusive");
    mode &= ~(NIIDMIX_FLAG_AVERAGE_ONLY | NIIDMIX_FLAG_LOW_DEGREE | NIIDMIX_FLAG_MEAN);
    if (mode != NIIDMIX_MODE_EXACT && mode != NIIDMIX_MODE_FAST)
        return set_error(NIIDMIX_EINVAL, "unknown mode %d", mode);
    if (n_rows == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !row_ptr || !col || !val) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (overlaps(x, (n_rows - 1) * ld_x + p, y, (n_rows - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uintptr_t align = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y);
    const int vw = (p % 4 == 0 && ld_x % 4 == 0 && ld_y % 4 == 0 && (align & 15) == 0) ? 4
                 : (p % 2 == 0 && ld_x % 2 == 0 && ld_y % 2 == 0 && (align & 7) == 0) ? 2 : 1;
    // work-item width: 2 chunks per wave for a low-degree graph (ring-100, P = 62006: 15.7 us vs
    // 16.6 us for 1 chunk and 16.6 us for 4 chunks, whose 142 VGPRs cap occupancy at 3 waves/SIMD;
    // profiles/r01/ring100_spl.txt), else 1.  NIIDMIX_CSR_SPL=1|2|4 overrides (tuning).
    const char *spl_env = getenv("NIIDMIX_CSR_SPL");
    const int spl = spl_env ? (atoi(spl_env) == 4 ? 4 : atoi(spl_env) == 2 ? 2 : 1) : (low_degree ? 2 : 1);
    const int64_t n_chunks = (p + kChunk * spl - 1) / (kChunk * spl);
    const int64_t n_row_groups = (n_rows + 3) / 4;
    const int64_t n_items = n_row_groups * ((n_chunks + 7) / 8) * 8;
    const dim3 grid((unsigned)grid_for(n_items)), block(256);
    // gathers in flight per batch: 4 when the caller flags a low-degree graph (ring, grid), else 8
    const bool lowdeg = low_degree != 0;
#define NIIDMIX_CSR(E, V, S, UU) hipLaunchKernelGGL((k_mix_csr<E, V, S, UU>), grid, block, 0, s, x, ld_x, y, ld_y, n_rows, p, row_ptr, col, val, n_row_groups, n_items, kflags)
#define NIIDMIX_CSR_U(E, V, S) do { if (lowdeg) NIIDMIX_CSR(E, V, S, 4); else NIIDMIX_CSR(E, V, S, 8); } while (0)
#define NIIDMIX_CSR_S(E, V) do { if (spl == 4) NIIDMIX_CSR_U(E, V, 4); else if (spl == 2) NIIDMIX_CSR_U(E, V, 2); else NIIDMIX_CSR_U(E, V, 1); } while (0)
    if (mode == NIIDMIX_MODE_EXACT) {
        if (vw == 4) NIIDMIX_CSR_S(true, 4); else if (vw == 2) NIIDMIX_CSR_S(true, 2); else NIIDMIX_CSR_S(true, 1);
    } else {
        if (vw == 4) NIIDMIX_CSR_S(false, 4); else if (vw == 2) NIIDMIX_CSR_S(false, 2); else NIIDMIX_CSR_S(false, 1);
    }
#undef NIIDMIX_CSR_U
#undef NIIDMIX_CSR_S
#undef NIIDMIX_CSR
    return check_launch("k_mix_csr");
}

static int cu_count() {
    static int n_cu = 0;
    if (!n_cu) {
        int dev = 0;
        (void)hipGetDevice(&dev);
        if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1) n_cu = 256;
    }
    return n_cu;
}

// One-pass big-clique launch (k_mix_bigclique_reg) for cliques of 257..1024 members: 2 blocks of
// 16 waves per CU (<= 64 VGPRs), or 1 block where a 64-VGPR budget would spill (R = 32 with
// groups).  Row-major slabs: bc_shift 62, block strides 0; column-blocked slabs: B = 2^bc_shift.
static int launch_bigclique_reg(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t p,
                                const niidmix_clique_plan *plan, int bc_shift, int64_t bs_x,
                                int64_t bs_y, hipStream_t s) {
    const int64_t nch8 = ((p + kBigRegCols - 1) / kBigRegCols + 7) / 8;
    const int64_t items = (int64_t)plan->n_cliques * nch8 * 8;
    const bool r16 = plan->max_clique <= 2 * kBigRegWaves * 16;
    const int bpc = (r16 || plan->n_groups == 1) ? 2 : 1;
    // item map, measured on FC-1000 (tools/s74.sh, one box): row-major slabs contiguous chunk
    // ranges per XCD 1.85 ms vs 2.02 ms interleaved; column-blocked slabs interleaved 1.70 ms vs
    // 1.73 ms.  NIIDMIX_BIGREG_MAP=interleave|contig overrides (A/B).
    const char *map_env = getenv("NIIDMIX_BIGREG_MAP");
    const int contig = map_env ? (!strcmp(map_env, "contig") ? 1 : 0) : (bc_shift >= 62 ? 1 : 0);
    int64_t gsz = (int64_t)bpc * cu_count();
    if (gsz > items) gsz = items;
    const dim3 grid((unsigned)gsz), block(kBigRegWaves * 64);
    // float4 lanes (k_mix_bigclique_v4) on column-blocked slabs whose p, ld and block strides are
    // multiples of 4 floats, 16-B aligned: the default for one-group cliques (FC-1000, P = 2^20,
    // same box: 1.355 vs 1.407 ms, profiles/r06/bigclique_v4/); NIIDMIX_BIGREG_V4=0 / 1 turns it
    // off / on for every group count
    const char *v4_env = getenv("NIIDMIX_BIGREG_V4");
    const bool v4 = v4_env ? atoi(v4_env) == 1 : plan->n_groups == 1;
    if (v4 && p % 4 == 0 && ld_x % 4 == 0 && ld_y % 4 == 0 && bs_x % 4 == 0 &&
        bs_y % 4 == 0 && aligned16(x) && aligned16(y) && bc_shift < 62 &&
        bs_x * 4 <= (int64_t)0xffffffffLL && bs_y * 4 <= (int64_t)0xffffffffLL) {
#define NIIDMIX_BIGV4(G, OCC) hipLaunchKernelGGL((k_mix_bigclique_v4<G, OCC>), grid, block, 0, s, x, ld_x, y, ld_y, p, plan->n_cliques, plan->clique_ptr, plan->member_row, plan->member_group, plan->coef, plan->res_ptr, plan->res_col, plan->res_val, nch8, bc_shift, bs_x, bs_y, contig, plan->csr_ptr, plan->csr_col, plan->csr_val)
        switch (plan->n_groups) {
        case 1: NIIDMIX_BIGV4(1, 8); break; case 2: NIIDMIX_BIGV4(2, 4); break;
        case 3: NIIDMIX_BIGV4(3, 4); break; case 4: NIIDMIX_BIGV4(4, 4); break;
        default: return set_error(NIIDMIX_EUNSUPPORTED, "n_groups %d not in 1..4", plan->n_groups);
        }
#undef NIIDMIX_BIGV4
        return check_launch("k_mix_bigclique_v4");
    }
#define NIIDMIX_BIGREG(G, R, OCC) hipLaunchKernelGGL((k_mix_bigclique_reg<G, R, OCC>), grid, block, 0, s, x, ld_x, y, ld_y, p, plan->n_cliques, plan->clique_ptr, plan->member_row, plan->member_group, plan->coef, plan->res_ptr, plan->res_col, plan->res_val, nch8, bc_shift, bs_x, bs_y, contig, plan->csr_ptr, plan->csr_col, plan->csr_val)
    if (r16) {
        switch (plan->n_groups) {
        case 1: NIIDMIX_BIGREG(1, 16, 8); break; case 2: NIIDMIX_BIGREG(2, 16, 8); break;
        case 3: NIIDMIX_BIGREG(3, 16, 8); break; case 4: NIIDMIX_BIGREG(4, 16, 8); break;
        default: return set_error(NIIDMIX_EUNSUPPORTED, "n_groups %d not in 1..4", plan->n_groups);
        }
    } else {
        switch (plan->n_groups) {
        case 1: NIIDMIX_BIGREG(1, 32, 8); break; case 2: NIIDMIX_BIGREG(2, 32, 4); break;
        case 3: NIIDMIX_BIGREG(3, 32, 4); break; case 4: NIIDMIX_BIGREG(4, 32, 4); break;
        default: return set_error(NIIDMIX_EUNSUPPORTED, "n_groups %d not in 1..4", plan->n_groups);
        }
    }
#undef NIIDMIX_BIGREG
    return check_launch("k_mix_bigclique_reg");
}

int niidmix_mix_clique_blocked_f32(const float *x, float *y, int64_t p, int64_t ld,
                                   int64_t block_cols, int64_t block_stride_x,
                                   int64_t block_stride_y, const niidmix_clique_plan *plan,
                                   void *stream) {
    if (!plan) return set_error(NIIDMIX_EINVAL, "null plan");
    if (p < 0 || plan->n_cliques < 0 || plan->n_members < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (plan->n_cliques == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !plan->clique_ptr || !plan->member_row || !plan->member_group || !plan->coef ||
        !plan->res_ptr || (!plan->res_col && plan->n_members > 0) || (!plan->res_val && plan->n_members > 0) ||
        (!plan->res_member && plan->n_members > 0) || !plan->csr_ptr || !plan->csr_col || !plan->csr_val)
        return set_error(NIIDMIX_EINVAL, "null pointer");
    // the register tile's items are 256 columns wide, the big-clique kernel's 32: an item never
    // straddles a block
    // (64 for cliques of <= 112 members: the multi-clique tile's 64-column items)
    const int64_t min_bc = plan->max_clique > 256 ? kBigRegCols : plan->max_clique <= 112 ? 64 : 256;
    if (block_cols < min_bc || (block_cols & (block_cols - 1)))
        return set_error(NIIDMIX_EINVAL, "block_cols %lld: a power of two >= %lld", (long long)block_cols,
                         (long long)min_bc);
    if (ld < block_cols) return set_error(NIIDMIX_EINVAL, "row stride < block_cols");
    if (block_stride_x < ld || block_stride_y < ld)
        return set_error(NIIDMIX_EINVAL, "block stride < row stride");
    {   // extents of the member rows in both slabs (x may hold more rows: halo rows of a shard)
        const int64_t k_blocks = (p + block_cols - 1) / block_cols;
        const int64_t rows = plan->n_members > 0 ? plan->n_members : 1;
        if (overlaps(x, (k_blocks - 1) * block_stride_x + (rows - 1) * ld + block_cols,
                     y, (k_blocks - 1) * block_stride_y + (rows - 1) * ld + block_cols))
            return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    }
    if (plan->max_clique > 2 * kBigRegWaves * 32)
        return set_error(NIIDMIX_EUNSUPPORTED, "blocked slabs: cliques of <= 1024 members");
    if (plan->max_clique_res < 0) return set_error(NIIDMIX_EINVAL, "negative max_clique_res");
    const bool vec4 = (ld % 4 == 0) && (block_stride_x % 4 == 0) && (block_stride_y % 4 == 0) &&
                      aligned16(x) && aligned16(y);
    if (plan->max_clique > 256)                               // one pass, 32-column items
        return launch_bigclique_reg(x, ld, y, ld, p, plan, __builtin_ctzll((unsigned long long)block_cols),
                                    block_stride_x, block_stride_y, reinterpret_cast<hipStream_t>(stream));
    BlockGeom bg;
    bg.bc_shift = __builtin_ctzll((unsigned long long)block_cols);
    bg.bs_x = block_stride_x;
    bg.bs_y = block_stride_y;
    return launch_clique_tiled(x, ld, y, ld, p, plan, vec4, reinterpret_cast<hipStream_t>(stream), bg);
}

// One-pass big-clique launch (k_mix_bigclique_reg), row-major (bc_shift 62, block strides 0) or
// column-blocked slabs.
int niidmix_mix_clique_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t p,
                           const niidmix_clique_plan *plan, void *stream) {
    if (!plan) return set_error(NIIDMIX_EINVAL, "null plan");
    if (p < 0 || plan->n_cliques < 0 || plan->n_members < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (plan->n_cliques == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !plan->clique_ptr || !plan->member_row || !plan->member_group || !plan->coef ||
        !plan->res_ptr || (!plan->res_col && plan->n_members > 0) || (!plan->res_val && plan->n_members > 0) ||
        (!plan->res_member && plan->n_members > 0) || !plan->csr_ptr || !plan->csr_col || !plan->csr_val)
        return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    {   // extents of the member rows in both slabs (x may hold more rows: halo rows of a shard)
        const int64_t rows = plan->n_members > 0 ? plan->n_members : 1;
        if (overlaps(x, (rows - 1) * ld_x + p, y, (rows - 1) * ld_y + p))
            return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    }
    if (plan->max_clique_res < 0) return set_error(NIIDMIX_EINVAL, "negative max_clique_res");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool vec4 = (p % 4 == 0) && (ld_x % 4 == 0) && (ld_y % 4 == 0) && aligned16(x) && aligned16(y);
    if (plan->max_clique > 256) {
        // big cliques (e.g. fully-connected = one clique): two-pass, one lane per column, a grid of
        // bpc blocks per CU walking the items.  Measured on FC-1000, P = 2^20 (tools/ab_clique.py):
        // 8 waves x 16 blocks/CU 2.36 ms; capping residency (to keep the pass-2 re-read in the
        // Infinity Cache) was slower: 8x4 2.57, 16x1 2.95 ms.  NIIDMIX_BIG=<waves>x<blocks per CU>
        // overrides (tuning).
        static int n_cu = 0;
        if (!n_cu) {
            int dev = 0;
            (void)hipGetDevice(&dev);
            if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cu < 1) n_cu = 256;
        }
        const char *big_env = getenv("NIIDMIX_BIG");         // "WxB": the two-pass kernel (tuning)
        if (big_env && !strcmp(big_env, "reg")) big_env = nullptr;
        if (!big_env && plan->max_clique <= 2 * kBigRegWaves * 32)
            return launch_bigclique_reg(x, ld_x, y, ld_y, p, plan, 62, 0, 0, s);
        int waves = 8, bpc = 16;
        if (big_env) sscanf(big_env, "%dx%d", &waves, &bpc);
        if (bpc < 1) bpc = 1;
        const int64_t n_ch = (p + kWave - 1) / kWave;
        const int64_t items = (int64_t)plan->n_cliques * ((n_ch + 7) / 8) * 8;
        int64_t gsz = ((int64_t)bpc * n_cu + 7) / 8 * 8;
        if (gsz > items) gsz = items;
        const dim3 grid((unsigned)gsz), block(waves * 64);
        const size_t lds = 0;
#define NIIDMIX_BIG(G, W) hipLaunchKernelGGL((k_mix_bigclique<G, W>), grid, block, lds, s, x, ld_x, y, ld_y, p, plan->n_cliques, plan->clique_ptr, plan->member_row, plan->member_group, plan->coef, plan->res_ptr, plan->res_col, plan->res_val, items, plan->csr_ptr, plan->csr_col, plan->csr_val)
#define NIIDMIX_BIGW(W) switch (plan->n_groups) { case 1: NIIDMIX_BIG(1, W); break; case 2: NIIDMIX_BIG(2, W); break; case 3: NIIDMIX_BIG(3, W); break; case 4: NIIDMIX_BIG(4, W); break; default: return set_error(NIIDMIX_EUNSUPPORTED, "n_groups %d not in 1..4", plan->n_groups); }
        if (waves == 4) { NIIDMIX_BIGW(4); }
        else if (waves == 8) { NIIDMIX_BIGW(8); }
        else { NIIDMIX_BIGW(16); }
#undef NIIDMIX_BIGW
#undef NIIDMIX_BIG
        return check_launch("k_mix_bigclique");
    }
    return launch_clique_tiled(x, ld_x, y, ld_y, p, plan, vec4, s);
}

int niidmix_mix_ell_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                        int64_t p, int k, const int32_t *ell_col, const float *ell_val,
                        const int32_t *ell_len, int mode, void *stream) {
    if (n_rows < 0 || p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    const int avg_only = (mode & NIIDMIX_FLAG_AVERAGE_ONLY) ? 1 : 0;
    mode &= ~(NIIDMIX_FLAG_AVERAGE_ONLY | NIIDMIX_FLAG_LOW_DEGREE);
    if (mode != NIIDMIX_MODE_EXACT && mode != NIIDMIX_MODE_FAST)
        return set_error(NIIDMIX_EINVAL, "unknown mode %d", mode);
    if (k < 1 || k > 8) return set_error(NIIDMIX_EUNSUPPORTED, "ELL width %d (1..8 supported)", k);
    if (n_rows == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !ell_col || !ell_val || !ell_len) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (overlaps(x, (n_rows - 1) * ld_x + p, y, (n_rows - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uintptr_t align = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y);
    const int vw = (p % 4 == 0 && ld_x % 4 == 0 && ld_y % 4 == 0 && (align & 15) == 0) ? 4
                 : (p % 2 == 0 && ld_x % 2 == 0 && ld_y % 2 == 0 && (align & 7) == 0) ? 2 : 1;
    // ELL width rounded up to an instantiated one; chunks in flight per wave by width (48 / 40 / 32
    // gather VGPRs).  NIIDMIX_ELL_CH overrides the chunks (tuning).
    const int kk = k <= 3 ? 3 : k <= 5 ? 5 : 8;
    int ch = kk == 3 ? 4 : kk == 5 ? 2 : 1;
    if (const char *e = getenv("NIIDMIX_ELL_CH")) { const int v = atoi(e); if (v == 1 || v == 2 || v == 4) ch = v; }
    if (kk != k) return set_error(NIIDMIX_EINVAL, "ELL width %d: pad the rows to %d entries (ell_len keeps the lengths)", k, kk);
    const int64_t n_slices = (p + 256 * ch - 1) / (256 * ch);
    const int64_t n_row_groups = (n_rows + 3) / 4;
    const int64_t n_items = n_row_groups * ((n_slices + 7) / 8) * 8;
    if (n_items > 0x7fffffffLL) return set_error(NIIDMIX_EUNSUPPORTED, "too many (rows, slice) items");
    const dim3 grid((unsigned)n_items), block(256);
#define NIIDMIX_ELL(E, V, KK, C) hipLaunchKernelGGL((k_mix_ell<E, V, KK, C>), grid, block, 0, s, x, ld_x, y, ld_y, n_rows, p, ell_col, ell_val, ell_len, n_row_groups, n_items, avg_only)
#define NIIDMIX_ELL_C(E, V, KK) do { if (ch == 4) NIIDMIX_ELL(E, V, KK, 4); else if (ch == 2) NIIDMIX_ELL(E, V, KK, 2); else NIIDMIX_ELL(E, V, KK, 1); } while (0)
#define NIIDMIX_ELL_K(E, V) do { if (kk == 3) NIIDMIX_ELL_C(E, V, 3); else if (kk == 5) NIIDMIX_ELL_C(E, V, 5); else NIIDMIX_ELL_C(E, V, 8); } while (0)
#define NIIDMIX_ELL_V(E) do { if (vw == 4) NIIDMIX_ELL_K(E, 4); else if (vw == 2) NIIDMIX_ELL_K(E, 2); else NIIDMIX_ELL_K(E, 1); } while (0)
    if (mode == NIIDMIX_MODE_EXACT) NIIDMIX_ELL_V(true); else NIIDMIX_ELL_V(false);
#undef NIIDMIX_ELL_V
#undef NIIDMIX_ELL_K
#undef NIIDMIX_ELL_C
#undef NIIDMIX_ELL
    return check_launch("k_mix_ell");
}

int niidmix_mix_band_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                         int64_t p, int k, int band, const int32_t *ell_col, const float *ell_val,
                         const int32_t *ell_len, int mode, void *stream) {
    if (n_rows < 0 || p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    const int avg_only = (mode & NIIDMIX_FLAG_AVERAGE_ONLY) ? 1 : 0;
    mode &= ~(NIIDMIX_FLAG_AVERAGE_ONLY | NIIDMIX_FLAG_LOW_DEGREE);
    if (mode != NIIDMIX_MODE_EXACT && mode != NIIDMIX_MODE_FAST)
        return set_error(NIIDMIX_EINVAL, "unknown mode %d", mode);
    if (!((k == 3 && band == 1) || (k == 5 && band == 2)))
        return set_error(NIIDMIX_EUNSUPPORTED, "band kernel: (k, band) = (%d, %d), (3, 1) or (5, 2) supported", k, band);
    if (n_rows == 0 || p == 0) return NIIDMIX_OK;
    if (n_rows < 2 * band + 1) return set_error(NIIDMIX_EUNSUPPORTED, "band %d needs >= %d rows", band, 2 * band + 1);
    if (!x || !y || !ell_col || !ell_val || !ell_len) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (overlaps(x, (n_rows - 1) * ld_x + p, y, (n_rows - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uintptr_t align = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y);
    const int vw = (p % 4 == 0 && ld_x % 4 == 0 && ld_y % 4 == 0 && (align & 15) == 0) ? 4
                 : (p % 2 == 0 && ld_x % 2 == 0 && ld_y % 2 == 0 && (align & 7) == 0) ? 2 : 1;
    if (vw == 1) return set_error(NIIDMIX_EUNSUPPORTED, "band kernel needs even p and ld, 8-B aligned slabs");
    // rows per wave x column chunks per wave (R x CH): NIIDMIX_BAND_RC = "R,CH" among the built
    // shapes (tuning); default 4 x 1 (ring 100, P = 62 006 in a hipGraph: 15.6 us per round; 4 x 4
    // 18.3, 2 x 2 15.8, 1 x 4 16.5, 8 x 2 17.3; tools/band_probe.py, profiles/r04/band_probe.txt)
    int rr = 4, ch = 1;
    if (const char *e = getenv("NIIDMIX_BAND_RC")) {
        int a = 0, b = 0;
        if (sscanf(e, "%d,%d", &a, &b) == 2 &&
            ((a == 1 && (b == 1 || b == 2 || b == 4)) || (a == 2 && (b == 1 || b == 2)) ||
             (a == 4 && (b == 1 || b == 4)) || (a == 8 && b == 2))) { rr = a; ch = b; }
    }
    const int64_t n_slices = (p + 64 * vw * ch - 1) / (64 * vw * ch);
    const int64_t n_row_groups = (n_rows + 4 * rr - 1) / (4 * rr);
    const int64_t n_items = n_row_groups * ((n_slices + 7) / 8) * 8;
    if (n_items > 0x7fffffffLL) return set_error(NIIDMIX_EUNSUPPORTED, "too many (rows, slice) items");
    const dim3 grid((unsigned)n_items), block(256);
#define NIIDMIX_BAND(E, V, KK, BB, RR, C) hipLaunchKernelGGL((k_mix_band<E, V, KK, BB, RR, C>), grid, block, 0, s, x, ld_x, y, ld_y, n_rows, p, ell_col, ell_val, ell_len, n_row_groups, n_items, avg_only)
#define NIIDMIX_BAND_R(E, V, KK, BB) do { \
        if (rr == 1) { if (ch == 1) NIIDMIX_BAND(E, V, KK, BB, 1, 1); else if (ch == 2) NIIDMIX_BAND(E, V, KK, BB, 1, 2); else NIIDMIX_BAND(E, V, KK, BB, 1, 4); } \
        else if (rr == 2) { if (ch == 1) NIIDMIX_BAND(E, V, KK, BB, 2, 1); else NIIDMIX_BAND(E, V, KK, BB, 2, 2); } \
        else if (rr == 4) { if (ch == 1) NIIDMIX_BAND(E, V, KK, BB, 4, 1); else NIIDMIX_BAND(E, V, KK, BB, 4, 4); } \
        else NIIDMIX_BAND(E, V, KK, BB, 8, 2); } while (0)
#define NIIDMIX_BAND_K(E, V) do { if (k == 3) NIIDMIX_BAND_R(E, V, 3, 1); else NIIDMIX_BAND_R(E, V, 5, 2); } while (0)
#define NIIDMIX_BAND_V(E) do { if (vw == 4) NIIDMIX_BAND_K(E, 4); else NIIDMIX_BAND_K(E, 2); } while (0)
    if (mode == NIIDMIX_MODE_EXACT) NIIDMIX_BAND_V(true); else NIIDMIX_BAND_V(false);
#undef NIIDMIX_BAND_V
#undef NIIDMIX_BAND_K
#undef NIIDMIX_BAND_R
#undef NIIDMIX_BAND
    return check_launch("k_mix_band");
}

int niidmix_mix_strip_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                          int64_t p, int k, const int32_t *ell_col, const float *ell_val,
                          const int32_t *ell_len, int mode, void *stream) {
    if (n_rows < 0 || p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    const int avg_only = (mode & NIIDMIX_FLAG_AVERAGE_ONLY) ? 1 : 0;
    mode &= ~(NIIDMIX_FLAG_AVERAGE_ONLY | NIIDMIX_FLAG_LOW_DEGREE);
    if (mode != NIIDMIX_MODE_EXACT && mode != NIIDMIX_MODE_FAST)
        return set_error(NIIDMIX_EINVAL, "unknown mode %d", mode);
    if (k != 3 && k != 5 && k != 8) return set_error(NIIDMIX_EUNSUPPORTED, "ELL width %d (3, 5 or 8)", k);
    if (n_rows == 0 || p == 0) return NIIDMIX_OK;
    if (n_rows > 256) return set_error(NIIDMIX_EUNSUPPORTED, "strip kernel: %lld rows (<= 256)", (long long)n_rows);
    if (!x || !y || !ell_col || !ell_val || !ell_len) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (overlaps(x, (n_rows - 1) * ld_x + p, y, (n_rows - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    if (reinterpret_cast<uintptr_t>(x) & 3) return set_error(NIIDMIX_EUNSUPPORTED, "x not 4-B aligned");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // float4 lanes (256-column strips, 1 KiB per staged row) when every lane's float4 stays inside
    // its row (ld >= p rounded up to 4) and the rows sit on 16-B boundaries, and the strip fits the
    // device's per-block LDS (gfx950: 160 KB, so up to 156 rows); else one float per lane (64-column
    // strips, 256 B per row).  NIIDMIX_STRIP_SV=1 forces the latter (tuning)
    int dev = 0, lds_max = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeSharedMemPerBlockOptin, dev) != hipSuccess || lds_max <= 0)
        if (hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || lds_max <= 0)
            lds_max = 65536;
    const uintptr_t al = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y);
    int sv = (ld_x % 4 == 0 && ld_y % 4 == 0 && (al & 15) == 0 && ld_x >= (p + 3) / 4 * 4 &&
              n_rows * kWave * 4 * (int64_t)sizeof(float) <= (int64_t)lds_max - 4096) ? 4 : 1;
    if (const char *e = getenv("NIIDMIX_STRIP_SV")) if (atoi(e) == 1) sv = 1;
    if (n_rows * kWave * sv * (int64_t)sizeof(float) > (int64_t)lds_max)
        return set_error(NIIDMIX_EUNSUPPORTED, "strip kernel: %lld rows do not fit %d B of LDS",
                         (long long)n_rows, lds_max);
    const int64_t n_strips = (p + kWave * sv - 1) / (kWave * sv);
    if (n_strips > 0x7fffffffLL) return set_error(NIIDMIX_EUNSUPPORTED, "too many strips");
    const size_t lds = (size_t)n_rows * kWave * sv * sizeof(float);   // <= lds_max
    // waves per strip: 8 (NIIDMIX_STRIP_SW = 4 / 8 / 16 overrides, tuning)
    int sw = 8;
    if (const char *e = getenv("NIIDMIX_STRIP_SW")) { const int v = atoi(e); if (v == 4 || v == 8 || v == 16) sw = v; }
    const dim3 grid((unsigned)n_strips), block(sw * kWave);
#define NIIDMIX_STRIP_W(E, KK, V, W) do { \
        auto kfn = k_mix_strip<E, KK, W, V>; \
        if (lds > 65536 && hipFuncSetAttribute(reinterpret_cast<const void *>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) \
            return set_error(NIIDMIX_EHIP, "k_mix_strip: %zu B of LDS refused", lds); \
        hipLaunchKernelGGL(kfn, grid, block, lds, s, x, ld_x, y, ld_y, (int)n_rows, p, ell_col, ell_val, ell_len, avg_only); \
    } while (0)
#define NIIDMIX_STRIP(E, KK, V) do { if (sw == 4) NIIDMIX_STRIP_W(E, KK, V, 4); else if (sw == 8) NIIDMIX_STRIP_W(E, KK, V, 8); else NIIDMIX_STRIP_W(E, KK, V, 16); } while (0)
#define NIIDMIX_STRIP_V(E, KK) do { if (sv == 4) NIIDMIX_STRIP(E, KK, 4); else NIIDMIX_STRIP(E, KK, 1); } while (0)
#define NIIDMIX_STRIP_K(E) do { if (k == 3) NIIDMIX_STRIP_V(E, 3); else if (k == 5) NIIDMIX_STRIP_V(E, 5); else NIIDMIX_STRIP_V(E, 8); } while (0)
    if (mode == NIIDMIX_MODE_EXACT) NIIDMIX_STRIP_K(true); else NIIDMIX_STRIP_K(false);
#undef NIIDMIX_STRIP_K
#undef NIIDMIX_STRIP_V
#undef NIIDMIX_STRIP
#undef NIIDMIX_STRIP_W
    return check_launch("k_mix_strip");
}

int niidmix_mix_tile_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                         int64_t p, const niidmix_tile_plan *plan, int mode, void *stream) {
    if (!plan) return set_error(NIIDMIX_EINVAL, "null plan");
    const int avg_only = (mode & NIIDMIX_FLAG_AVERAGE_ONLY) ? 1 : 0;
    mode &= ~NIIDMIX_FLAG_AVERAGE_ONLY;
    if (mode != NIIDMIX_MODE_EXACT && mode != NIIDMIX_MODE_FAST)
        return set_error(NIIDMIX_EINVAL, "unknown mode %d", mode);
    if (p < 0 || plan->n_sub < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (plan->rt != 8 && plan->rt != 16 && plan->rt != 32)
        return set_error(NIIDMIX_EUNSUPPORTED, "tile of %d rows (8, 16 or 32 supported)", plan->rt);
    if (plan->n_sub == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !plan->sub_ptr || !plan->sub_rows || !plan->sub_wself || !plan->pos_src ||
        !plan->pos_mask || !plan->pos_w)
        return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (n_rows < 1) return set_error(NIIDMIX_EINVAL, "n_rows < 1");
    if (overlaps(x, (n_rows - 1) * ld_x + p, y, (n_rows - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const uintptr_t align = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y);
    // columns per lane: 4 for 8- and 16-row tiles, 2 for 32-row tiles (register budget);
    // NIIDMIX_TILE_NE=2|4 overrides (tuning)
    int ne = plan->rt == 32 ? 2 : 4;
    if (const char *e = getenv("NIIDMIX_TILE_NE")) { const int v = atoi(e); if (v == 2 || v == 4) ne = v; }
    int vw = (p % 2 == 0 && ld_x % 2 == 0 && ld_y % 2 == 0 && (align & 7) == 0) ? 2 : 1;
    if (ne == 4 && vw == 2 && p % 4 == 0 && ld_x % 4 == 0 && ld_y % 4 == 0 && (align & 15) == 0) vw = 4;
    const int64_t cw = 64 * ne;
    const int64_t n_chunks = (p + cw - 1) / cw;
    const int64_t n_sub_groups = (plan->n_sub + 3) / 4;
    const int64_t n_items = n_sub_groups * ((n_chunks + 7) / 8) * 8;
    const dim3 grid((unsigned)grid_for(n_items)), block(256);
#define NIIDMIX_TILEK(E, V, N, R) hipLaunchKernelGGL((k_mix_tile<E, V, N, R>), grid, block, 0, s, x, ld_x, y, ld_y, p, plan->n_sub, plan->sub_ptr, plan->sub_rows, plan->sub_wself, plan->pos_src, plan->pos_mask, plan->pos_w, n_sub_groups, n_items, avg_only)
#define NIIDMIX_TILE_V(E, N, R) do { if (vw == 4) NIIDMIX_TILEK(E, 4, 4, R); else if (vw == 2) NIIDMIX_TILEK(E, 2, N, R); else NIIDMIX_TILEK(E, 1, N, R); } while (0)
#define NIIDMIX_TILE_N(E, R) do { if (ne == 4) NIIDMIX_TILE_V(E, 4, R); else NIIDMIX_TILE_V(E, 2, R); } while (0)
#define NIIDMIX_TILE_R(E) do { if (plan->rt == 8) NIIDMIX_TILE_N(E, 8); else if (plan->rt == 16) NIIDMIX_TILE_N(E, 16); else NIIDMIX_TILE_N(E, 32); } while (0)
    if (mode == NIIDMIX_MODE_EXACT) NIIDMIX_TILE_R(true); else NIIDMIX_TILE_R(false);
#undef NIIDMIX_TILE_R
#undef NIIDMIX_TILE_N
#undef NIIDMIX_TILE_V
#undef NIIDMIX_TILEK
    return check_launch("k_mix_tile");
}

int niidmix_mix_tile_lds_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                             int64_t p, const niidmix_tile_lds_plan *plan, int mode, void *stream) {
    if (!plan) return set_error(NIIDMIX_EINVAL, "null plan");
    int avg_only = (mode & NIIDMIX_FLAG_AVERAGE_ONLY) ? 1 : 0;
    mode &= ~NIIDMIX_FLAG_AVERAGE_ONLY;
    if (mode != NIIDMIX_MODE_EXACT && mode != NIIDMIX_MODE_FAST)
        return set_error(NIIDMIX_EINVAL, "unknown mode %d", mode);
    if (const char *e = getenv("NIIDMIX_TLDS_SMALL"))           // tuning: 0 = 16-row loop only
        if (atoi(e) == 0) avg_only |= 2;
    if (p < 0 || plan->n_grp < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (plan->rt != 8 && plan->rt != 16 && plan->rt != 32)
        return set_error(NIIDMIX_EUNSUPPORTED, "tile of %d rows (8, 16 or 32 supported)", plan->rt);
    if (plan->n_grp == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !plan->grp_tile_ptr || !plan->grp_src_ptr || !plan->grp_src_rows ||
        !plan->sub_ptr || !plan->sub_rows || !plan->sub_slot || !plan->sub_wself ||
        !plan->pos_slot || !plan->pos_mask || !plan->pos_w)
        return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (ld_x >= (1LL << 30)) return set_error(NIIDMIX_EUNSUPPORTED, "ld_x >= 2^30");
    if (n_rows < 1) return set_error(NIIDMIX_EINVAL, "n_rows < 1");
    if (overlaps(x, (n_rows - 1) * ld_x + p, y, (n_rows - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    if (plan->max_src < 1 || plan->max_src > 256)
        return set_error(NIIDMIX_EUNSUPPORTED, "group with %d source rows (1..256 supported)", plan->max_src);
    const int max_waves = tile_lds_max_waves(plan->rt);
    if (plan->max_tiles < 1 || plan->max_tiles > max_waves)
        return set_error(NIIDMIX_EUNSUPPORTED, "group with %d tiles of %d rows (1..%d supported)",
                         plan->max_tiles, plan->rt, max_waves);
    const uintptr_t align = reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y);
    if (p % 2 || ld_x % 2 || ld_y % 2 || (align & 7))
        return set_error(NIIDMIX_EUNSUPPORTED, "LDS tile kernel needs even p, ld and 8-B aligned slabs");
    const int sv = (p % 4 == 0 && ld_x % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0) ? 4 : 2;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    // Item width (rt 16): the widest of 128, 120 and 96 columns that fits the most blocks per CU in
    // its 160 KB of LDS, up to three (three 7-wave blocks fill the 6 waves per SIMD the kernel's 80
    // VGPRs allow).  The position loop is latency-bound, so another block's waves are worth idle
    // lanes.  1000-node d-cliques: 109 staged rows -> 120 columns, three blocks (same box 3.85 vs
    // 4.07 ms at 128; one block per CU 7.3 ms); 10 000 nodes: 199 rows -> 96 columns, two blocks
    // instead of one.  124 and 112 columns measured slower than 120.
    int cw = 128;
    const size_t lds_cu = 160 * 1024;
    // segment loop (RT 16, plan->seg_ptr set): two spare staged rows for its reads past a segment
    const bool seg = plan->rt == 16 && plan->seg_ptr != nullptr;
    if (seg && (!plan->seg || !plan->seg_w)) return set_error(NIIDMIX_EINVAL, "null segment arrays");
    // matrix-core path (exact mode, segment plans only: the walker is its per-block fallback)
    const bool mf = seg && mode == NIIDMIX_MODE_EXACT && plan->mf_ptr != nullptr;
    // register rows (rem_rows): the segment walker only (the other loops read every source from LDS)
    const bool rem = plan->rem_rows != nullptr;
    if (rem && (!seg || plan->mf_ptr != nullptr))
        return set_error(NIIDMIX_EINVAL, "rem_rows needs the segment walker (seg_ptr set, mf_ptr NULL)");
    if (rem && plan->rem_regs != 0 && plan->rem_regs != 8 && plan->rem_regs != 16 && plan->rem_regs != -16)
        return set_error(NIIDMIX_EINVAL, "rem_regs %d (0, 8, 16 or -16)", plan->rem_regs);
    const bool rem8 = rem && plan->rem_regs == 8;
    // -16: up to 16 register rows walked in two phases of 8 (80 VGPRs instead of 96); the host
    // sets it only for plans whose tiles read rows 0..7 before any of 8..15 (tile.rem_two_phase)
    const bool rem2 = rem && plan->rem_regs == -16;
    if (mf && !plan->mf) return set_error(NIIDMIX_EINVAL, "null MFMA position list");
    // waves of a block on the matrix cores (the rest walk segments on the VALU side by side);
    // NIIDMIX_TLDS_MF_WAVES overrides (tuning), default every wave
    int mf_waves = plan->max_tiles;
    if (const char *e = getenv("NIIDMIX_TLDS_MF_WAVES")) mf_waves = atoi(e);
    const int stage_rows = plan->max_src + (seg ? 2 : 0);
    if (plan->rt == 16) {
        auto blocks = [&](int c) {
            const size_t per = (size_t)stage_rows * c * sizeof(float) + tlds_slack(seg, c);
            const size_t b = per ? lds_cu / per : 3;
            return (int)(b < 3 ? b : 3);
        };
        const int target = blocks(96);
        for (int c : {128, 120, 96})
            if (blocks(c) >= target) { cw = c; break; }
    }
    if (const char *e = getenv("NIIDMIX_TLDS_COLS")) {          // tuning override: 128, 120 or 96
        const int v = atoi(e);
        if (v == 128 || v == 120 || v == 96) cw = v;
    }
    const int64_t n_chunks = (p + cw - 1) / cw;
    const int64_t n_items = (int64_t)plan->n_grp * ((n_chunks + 7) / 8) * 8;
    if (n_items > 0x7fffffffLL) return set_error(NIIDMIX_EUNSUPPORTED, "too many (group, chunk) items");
    const size_t lds = (size_t)stage_rows * cw * sizeof(float) + tlds_slack(seg, cw);
    const dim3 grid((unsigned)n_items), block((unsigned)(64 * plan->max_tiles));
#define NIIDMIX_TLDS_CW2(E, R, V, SG, RM, M, R2) (cw == 120 ? k_mix_tile_lds<E, R, V, 60, SG, RM, M, R2> : cw == 96 ? k_mix_tile_lds<E, R, V, 48, SG, RM, M, R2> : k_mix_tile_lds<E, R, V, 64, SG, RM, M, R2>)
#define NIIDMIX_TLDS_CW(E, R, V, SG, RM, M) NIIDMIX_TLDS_CW2(E, R, V, SG, RM, M, false)
#define NIIDMIX_TLDS(E, R, V) do { \
        auto kfn = seg ? (rem ? (rem8 ? NIIDMIX_TLDS_CW(E, R, V, (R == 16), (R == 16 ? 8 : 0), false) \
                                : rem2 ? NIIDMIX_TLDS_CW2(E, R, V, (R == 16), (R == 16 ? 8 : 0), false, (R == 16)) \
                                     : NIIDMIX_TLDS_CW(E, R, V, (R == 16), (R == 16 ? 16 : 0), false)) \
                              : mf ? NIIDMIX_TLDS_CW(E, R, V, (R == 16), 0, (E && R == 16)) \
                                   : NIIDMIX_TLDS_CW(E, R, V, (R == 16), 0, false)) \
                       : NIIDMIX_TLDS_CW(E, R, V, false, 0, false); \
        if (lds > 65536 && hipFuncSetAttribute(reinterpret_cast<const void *>(kfn), hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) \
            return set_error(NIIDMIX_EHIP, "k_mix_tile_lds: %zu B of LDS refused", lds); \
        hipLaunchKernelGGL(kfn, grid, block, lds, s, x, ld_x, y, ld_y, p, (int64_t)plan->n_grp, plan->grp_tile_ptr, plan->grp_src_ptr, plan->grp_src_rows, plan->sub_ptr, plan->sub_rows, plan->sub_slot, plan->sub_wself, plan->pos_slot, plan->pos_mask, plan->pos_w, avg_only, seg ? plan->seg_ptr : nullptr, plan->seg, plan->seg_w, mf ? plan->mf_ptr : nullptr, plan->mf, mf_waves, plan->rem_rows); \
    } while (0)
#define NIIDMIX_TLDS_V(E, R) do { if (sv == 4) NIIDMIX_TLDS(E, R, 4); else NIIDMIX_TLDS(E, R, 2); } while (0)
#define NIIDMIX_TLDS_R(E) do { if (plan->rt == 8) NIIDMIX_TLDS_V(E, 8); else if (plan->rt == 16) NIIDMIX_TLDS_V(E, 16); else NIIDMIX_TLDS_V(E, 32); } while (0)
    if (mode == NIIDMIX_MODE_EXACT) NIIDMIX_TLDS_R(true); else NIIDMIX_TLDS_R(false);
#undef NIIDMIX_TLDS_R
#undef NIIDMIX_TLDS_V
#undef NIIDMIX_TLDS
#undef NIIDMIX_TLDS_CW
#undef NIIDMIX_TLDS_CW2
    return check_launch("k_mix_tile_lds");
}

int niidmix_mix_dense_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n,
                          int64_t p, const float *w, const int64_t *row_ptr, const int32_t *col,
                          const float *val, void *stream) {
    if (n < 0 || p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (n == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !w || !row_ptr || !col || !val) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (overlaps(x, (n - 1) * ld_x + p, y, (n - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool vec = (p % 4 == 0) && (ld_x % 4 == 0) && aligned16(x);
    const int64_t n_it = (n + kDBM - 1) / kDBM;
    const int64_t n_jt = (p + kDBN - 1) / kDBN;
    const int64_t n_items = n_it * ((n_jt + 7) / 8) * 8;
    const dim3 grid((unsigned)grid_for(n_items)), block(256);
    const bool avec = (n % 4 == 0) && aligned16(w);
#define NIIDMIX_DENSE(V, A) hipLaunchKernelGGL((k_mix_dense<V, A>), grid, block, 0, s, x, ld_x, y, ld_y, n, p, w, n_it, n_items, row_ptr, col, val)
    // vectorised operands: the interleaved DS-read / MFMA schedule (18.05 vs 18.87 ms on FC-1000);
    // NIIDMIX_DENSE_SCHED=0 restores the compiler's schedule (tuning)
    const char *sc = getenv("NIIDMIX_DENSE_SCHED");
    // K-steps of 16 (168 VGPRs, half the LDS: three blocks per CU) 17.2 vs 18.0 ms with 32 (256
    // VGPRs, two blocks; NIIDMIX_DENSE_BK=32 restores it, =8 and NIIDMIX_DENSE_OCC=4: tuning)
    const char *bk = getenv("NIIDMIX_DENSE_BK");
    const char *oc = getenv("NIIDMIX_DENSE_OCC");
    const int bkv = bk ? atoi(bk) : 16, occ = oc ? atoi(oc) : 0;
    if (vec && avec && !(sc && sc[0] == '0') && (bkv == 16 || bkv == 8)) {
#define NIIDMIX_DENSE_T(B, O) hipLaunchKernelGGL((k_mix_dense<true, true, true, B, O>), grid, block, 0, s, x, ld_x, y, ld_y, n, p, w, n_it, n_items, row_ptr, col, val)
        if (bkv == 16) { if (occ == 4) NIIDMIX_DENSE_T(16, 4); else NIIDMIX_DENSE_T(16, 3); }
        else { if (occ == 4) NIIDMIX_DENSE_T(8, 4); else NIIDMIX_DENSE_T(8, 3); }
#undef NIIDMIX_DENSE_T
        return check_launch("k_mix_dense");
    }
    if (vec && avec && !(sc && sc[0] == '0')) {
        hipLaunchKernelGGL((k_mix_dense<true, true, true>), grid, block, 0, s, x, ld_x, y, ld_y, n, p, w, n_it, n_items, row_ptr, col, val);
        return check_launch("k_mix_dense");
    }
    if (vec) { if (avec) NIIDMIX_DENSE(true, true); else NIIDMIX_DENSE(true, false); }
    else     { if (avec) NIIDMIX_DENSE(false, true); else NIIDMIX_DENSE(false, false); }
#undef NIIDMIX_DENSE
    return check_launch("k_mix_dense");
}

int64_t niidmix_dense_split_elems(int64_t n) {
    if (n <= 0) return 0;
    const int64_t mpad = (n + kB6M - 1) / kB6M * kB6M, kpad = (n + kB6K - 1) / kB6K * kB6K;
    return 3 * mpad * kpad;
}

int niidmix_dense_split_w(const float *w, int64_t n, uint16_t *wp, void *stream) {
    if (n < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (n == 0) return NIIDMIX_OK;
    if (!w || !wp) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (reinterpret_cast<uintptr_t>(wp) & 15) return set_error(NIIDMIX_EUNSUPPORTED, "wp not 16-B aligned");
    const int64_t mpad = (n + kB6M - 1) / kB6M * kB6M, kpad = (n + kB6K - 1) / kB6K * kB6K;
    if (overlaps(w, n * n, reinterpret_cast<const float *>(wp), 3 * mpad * kpad / 2))
        return set_error(NIIDMIX_EALIAS, "w and wp overlap");
    const int64_t pairs = mpad * kpad / 2;
    hipLaunchKernelGGL(k_dense_split_w, dim3((unsigned)((pairs + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), w, n, mpad, kpad,
                       reinterpret_cast<uint32_t *>(wp));
    return check_launch("k_dense_split_w");
}

int niidmix_mix_dense_bf16x6_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n,
                                 int64_t p, const uint16_t *wp, const int64_t *row_ptr,
                                 const int32_t *col, const float *val, void *stream) {
    if (n < 0 || p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (n == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !wp || !row_ptr || !col || !val) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (reinterpret_cast<uintptr_t>(wp) & 15) return set_error(NIIDMIX_EUNSUPPORTED, "wp not 16-B aligned");
    if (overlaps(x, (n - 1) * ld_x + p, y, (n - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "x and y overlap (mixing is out-of-place / Jacobi)");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t mpad = (n + kB6M - 1) / kB6M * kB6M, kpad = (n + kB6K - 1) / kB6K * kB6K;
    if (16 * ld_x * 4 >= (int64_t)0x7fffffffLL || 3 * mpad * kpad * 2 >= (int64_t)0x7fffffffLL)
        return set_error(NIIDMIX_EUNSUPPORTED, "bf16x6 dense GEMM: 16 rows of ld_x %lld or the split W "
                         "of n %lld exceed 2^31 B (use niidmix_mix_dense_f32)", (long long)ld_x, (long long)n);
    // block tile 256 x 256 (8 waves of 128 x 64: X re-read by 4 row tiles instead of 8, 48 MFMAs
    // per wave between barriers): 9.81-9.86 vs 11.20-11.30 ms for 128 x 256 on the same box
    // (profiles/r05/dense_b6/); NIIDMIX_DENSE_B6_TM=2 selects the latter (with _WN / _SCHED: A/B)
    const int tm = (getenv("NIIDMIX_DENSE_B6_TM") && atoi(getenv("NIIDMIX_DENSE_B6_TM")) == 2) ? 2 : 4;
    // tuning A/B of the 128 x 256 tile (TM 2): NIIDMIX_DENSE_B6_WN=2 128 x 128 (4 waves, two blocks
    // per CU); NIIDMIX_DENSE_B6_SCHED 2 the compiler's schedule (11.2 ms on FC-1000 at P = 2^20),
    // 0 / 1 operand reads in three slices with the split beside / after the MFMAs (11.6-12.4 ms,
    // profiles/r05/dense_b6/)
    // SCHED 3 (loads pinned at the top of each K-step) by default on the 256 x 256 tile: 9.70-9.75
    // vs 9.80-9.84 ms for the compiler's schedule (2), same box, interleaved (profiles/r05/dense_b6/)
    int wn = 4, sched = tm == 4 ? 3 : 2;
    if (const char *e = getenv("NIIDMIX_DENSE_B6_WN")) if (atoi(e) == 2) wn = 2;
    if (const char *e = getenv("NIIDMIX_DENSE_B6_SCHED")) { const int v = atoi(e); if (v >= 0 && v <= 3) sched = v; }
#define NIIDMIX_B6T(WN, SC, AB, TM) do { \
        const int64_t n_it = mpad / (64 * TM); \
        const int64_t n_jt = (p + 64 * WN - 1) / (64 * WN); \
        const int64_t n_items = n_it * ((n_jt + 7) / 8) * 8; \
        const size_t lds = (size_t)2 * 3 * (64 * TM + 64 * WN) * 2 * sizeof(uint4); \
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_mix_dense_b6<WN, SC, AB, TM>), \
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) \
            return set_error(NIIDMIX_EHIP, "k_mix_dense_b6: %zu B of LDS refused", lds); \
        hipLaunchKernelGGL((k_mix_dense_b6<WN, SC, AB, TM>), dim3((unsigned)grid_for(n_items)), dim3(128 * WN), lds, s, \
                           x, ld_x, y, ld_y, n, p, wp, mpad, kpad, n_it, n_items, row_ptr, col, val); \
    } while (0)
    // W tiles by LDS-DMA (k_mix_dense_b6d): NIIDMIX_DENSE_B6_DMA = "WN,NA[,XD]" -- 4,3 (256 x 256,
    // one block per CU, W two K-steps ahead), 4,2, or 2,2 (256 x 128, two blocks per CU); XD 3:
    // X fetched three K-steps ahead (a third register set, with the 2-deep W ring)
    if (const char *e = getenv("NIIDMIX_DENSE_B6_DMA")) {
        int dwn = 0, dna = 0, dxd = 2;
        if (sscanf(e, "%d,%d,%d", &dwn, &dna, &dxd) >= 2 && dwn != 0) {
#define NIIDMIX_B6D(WN, NA, XD) do { \
            const int64_t n_it = mpad / 256, n_jt = (p + 64 * WN - 1) / (64 * WN); \
            const int64_t n_items = n_it * ((n_jt + 7) / 8) * 8; \
            const size_t lds = ((size_t)NA * 3 * 256 * 2 + (size_t)2 * 3 * 64 * WN * 2) * sizeof(uint4); \
            if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_mix_dense_b6d<WN, 4, NA, XD>), \
                                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) \
                return set_error(NIIDMIX_EHIP, "k_mix_dense_b6d: %zu B of LDS refused", lds); \
            hipLaunchKernelGGL((k_mix_dense_b6d<WN, 4, NA, XD>), dim3((unsigned)grid_for(n_items)), dim3(128 * WN), lds, s, \
                               x, ld_x, y, ld_y, n, p, wp, mpad, kpad, n_it, n_items, row_ptr, col, val); \
        } while (0)
            if (dwn == 4 && dna == 3 && dxd == 2) NIIDMIX_B6D(4, 3, 2);
            else if (dwn == 4 && dna == 2 && dxd == 2) NIIDMIX_B6D(4, 2, 2);
            else if (dwn == 4 && dna == 2 && dxd == 3) NIIDMIX_B6D(4, 2, 3);
            else if (dwn == 2 && dna == 2 && dxd == 2) NIIDMIX_B6D(2, 2, 2);
            else if (dwn == 2 && dna == 2 && dxd == 3) NIIDMIX_B6D(2, 2, 3);
            else return set_error(NIIDMIX_EINVAL, "NIIDMIX_DENSE_B6_DMA=%s: 4,3 / 4,2[,3] / 2,2[,3]", e);
#undef NIIDMIX_B6D
            return check_launch("k_mix_dense_b6d");
        }
    }
    // one wave per SIMD (k_mix_dense_b6w, 256 x 256 tile of 4 waves of 128 x 128): tuning A/B
    if (const char *e = getenv("NIIDMIX_DENSE_B6_W1")) if (atoi(e) == 1) {
        const int64_t n_it = mpad / 256, n_jt = (p + 255) / 256;
        const int64_t n_items = n_it * ((n_jt + 7) / 8) * 8;
        const size_t lds = (size_t)2 * 3 * (256 + 256) * 2 * sizeof(uint4);
        if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_mix_dense_b6w),
                                hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
            return set_error(NIIDMIX_EHIP, "k_mix_dense_b6w: %zu B of LDS refused", lds);
        hipLaunchKernelGGL(k_mix_dense_b6w, dim3((unsigned)grid_for(n_items)), dim3(256), lds, s,
                           x, ld_x, y, ld_y, n, p, wp, mpad, kpad, n_it, n_items, row_ptr, col, val);
        return check_launch("k_mix_dense_b6w");
    }
    int abl = 0;
#ifdef NIIDMIX_ABLATIONS
    // time-split builds only (wrong results by construction; never in the shipped library)
    if (const char *e = getenv("NIIDMIX_DENSE_B6_ABL")) abl = atoi(e);
#endif
#define NIIDMIX_B6(WN, SC, AB) NIIDMIX_B6T(WN, SC, AB, 2)
    if (tm == 4 && abl == 0 && wn == 4 && sched == 2) NIIDMIX_B6T(4, 2, 0, 4);
    else if (tm == 4 && abl == 0 && wn == 4 && sched == 3) NIIDMIX_B6T(4, 3, 0, 4);
#ifdef NIIDMIX_ABLATIONS
    else if (abl == 1) NIIDMIX_B6T(4, 2, 1, 4);
    else if (abl == 2) NIIDMIX_B6T(4, 2, 2, 4);
    else if (abl == 3) NIIDMIX_B6T(4, 2, 3, 4);
    else if (abl == 4) NIIDMIX_B6T(4, 3, 4, 4);
    else if (abl == 5) NIIDMIX_B6T(4, 3, 0, 4);
#endif
    else if (wn == 2) { if (sched >= 2) NIIDMIX_B6(2, 2, 0); else if (sched == 1) NIIDMIX_B6(2, 1, 0); else NIIDMIX_B6(2, 0, 0); }
    else { if (sched >= 2) NIIDMIX_B6(4, 2, 0); else if (sched == 1) NIIDMIX_B6(4, 1, 0); else NIIDMIX_B6(4, 0, 0); }
#undef NIIDMIX_B6
#undef NIIDMIX_B6T
    return check_launch("k_mix_dense_b6");
}

int niidmix_mean_rows_f32(const float *x, int64_t ld_x, int64_t n, int64_t p, float *mean,
                          double *dist2, int mode, void *stream) {
    if (n < 0 || p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (mode != NIIDMIX_MODE_EXACT && mode != NIIDMIX_MODE_FAST)
        return set_error(NIIDMIX_EINVAL, "unknown mode %d", mode);
    if (n == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !mean) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (overlaps(x, (n - 1) * ld_x + p, mean, p)) return set_error(NIIDMIX_EALIAS, "mean overlaps x");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const float w = (float)(1.0 / (double)n);
    const int64_t blocks = (p + 255) / 256 < 16384 ? (p + 255) / 256 : 16384;
    if (mode == NIIDMIX_MODE_EXACT)
        hipLaunchKernelGGL((k_mean_cols<true>), dim3((unsigned)blocks), dim3(256), 0, s, x, ld_x, n, p, w, mean);
    else
        hipLaunchKernelGGL((k_mean_cols<false>), dim3((unsigned)blocks), dim3(256), 0, s, x, ld_x, n, p, w, mean);
    int rc = check_launch("k_mean_cols");
    if (rc != NIIDMIX_OK || !dist2) return rc;
    hipLaunchKernelGGL(k_row_dist2, dim3((unsigned)n), dim3(256), 0, s, x, ld_x, p, mean, dist2);
    return check_launch("k_row_dist2");
}

static bool grad_nt() {
    const char *e = getenv("NIIDMIX_GRAD_NT");
    return !(e && atoi(e) == 0);
}

int niidmix_grad_segment_mean_f32(const float *g, int64_t ld_g, float *y, int64_t ld_y,
                                  int64_t n_rows, int64_t p, int64_t n_seg, const int32_t *seg_ptr,
                                  const int32_t *seg_row, void *stream) {
    if (p < 0 || n_seg < 0 || n_rows < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (n_seg == 0 || p == 0 || n_rows == 0) return NIIDMIX_OK;
    if (!g || !y || !seg_ptr || !seg_row) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_g < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    if (overlaps(g, (n_rows - 1) * ld_g + p, y, (n_rows - 1) * ld_y + p))
        return set_error(NIIDMIX_EALIAS, "g and y overlap: the mean is out-of-place");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool vec4 = p % 4 == 0 && ld_g % 4 == 0 && ld_y % 4 == 0 && aligned16(g) && aligned16(y);
    const int64_t cols = vec4 ? 1024 : 256;
    const int64_t n_chunks = (p + cols - 1) / cols;
    const int64_t n_items = n_seg * n_chunks;
    const dim3 grid((unsigned)(n_items < kMaxGrid ? n_items : kMaxGrid)), block(256);
    if (vec4 && grad_nt())
        hipLaunchKernelGGL((k_grad_segment_mean<4, 8, true>), grid, block, 0, s, g, ld_g, y, ld_y, p, n_seg,
                           seg_ptr, seg_row, n_chunks, 62, (int64_t)0, (int64_t)0);
    else if (vec4)
        hipLaunchKernelGGL((k_grad_segment_mean<4, 8, false>), grid, block, 0, s, g, ld_g, y, ld_y, p, n_seg,
                           seg_ptr, seg_row, n_chunks, 62, (int64_t)0, (int64_t)0);
    else
        hipLaunchKernelGGL((k_grad_segment_mean<1, 16>), grid, block, 0, s, g, ld_g, y, ld_y, p, n_seg,
                           seg_ptr, seg_row, n_chunks, 62, (int64_t)0, (int64_t)0);
    return check_launch("k_grad_segment_mean");
}

int niidmix_grad_segment_mean_blocked_f32(const float *g, float *y, int64_t n_rows, int64_t p,
                                          int64_t ld, int64_t block_cols, int64_t block_stride_g,
                                          int64_t block_stride_y, int64_t n_seg,
                                          const int32_t *seg_ptr, const int32_t *seg_row,
                                          void *stream) {
    if (p < 0 || n_seg < 0 || n_rows < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (n_seg == 0 || p == 0 || n_rows == 0) return NIIDMIX_OK;
    if (!g || !y || !seg_ptr || !seg_row) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (block_cols < 1024 || (block_cols & (block_cols - 1)))
        return set_error(NIIDMIX_EINVAL, "block_cols %lld: a power of two >= 1024", (long long)block_cols);
    if (ld < block_cols || block_stride_g < ld || block_stride_y < ld)
        return set_error(NIIDMIX_EINVAL, "row stride < block_cols or block stride < row stride");
    {   // extents of both blocked slabs, each with its own block stride
        const int64_t k_blocks = (p + block_cols - 1) / block_cols;
        if (overlaps(g, (k_blocks - 1) * block_stride_g + (n_rows - 1) * ld + block_cols,
                     y, (k_blocks - 1) * block_stride_y + (n_rows - 1) * ld + block_cols))
            return set_error(NIIDMIX_EALIAS, "g and y overlap: the mean is out-of-place");
    }
    if (p % 4 || ld % 4 || block_stride_g % 4 || block_stride_y % 4 || !aligned16(g) || !aligned16(y))
        return set_error(NIIDMIX_EUNSUPPORTED, "blocked gradient mean needs p, strides % 4 == 0 and 16-B aligned slabs");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int64_t n_chunks = (p + 1023) / 1024;
    const int64_t n_items = n_seg * n_chunks;
    const dim3 grid((unsigned)(n_items < kMaxGrid ? n_items : kMaxGrid)), block(256);
    const int shift = __builtin_ctzll((unsigned long long)(block_cols / 1024));
    // non-temporal gradient-row loads (each row is read once): 1.375 vs 1.401 ms on the headline
    // shape, same box (profiles/r05/grad_nt/); NIIDMIX_GRAD_NT=0 restores the default cache policy
    if (grad_nt())
        hipLaunchKernelGGL((k_grad_segment_mean<4, 8, true>), grid, block, 0, s, g, ld, y, ld, p, n_seg, seg_ptr,
                           seg_row, n_chunks, shift, block_stride_g, block_stride_y);
    else
        hipLaunchKernelGGL((k_grad_segment_mean<4, 8, false>), grid, block, 0, s, g, ld, y, ld, p, n_seg, seg_ptr,
                           seg_row, n_chunks, shift, block_stride_g, block_stride_y);
    return check_launch("k_grad_segment_mean");
}

int niidmix_sgd_step_rows_f32(float *p, int64_t ld_p, const float *g, int64_t ld_g, int64_t ncols,
                              const int32_t *rows, int64_t n_rows, float neg_lr, void *stream) {
    if (ncols < 0 || n_rows < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (ncols == 0 || n_rows == 0) return NIIDMIX_OK;
    if (!p || !g || !rows) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_p < ncols || ld_g < ncols) return set_error(NIIDMIX_EINVAL, "leading dimension < ncols");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool vec4 = ncols % 4 == 0 && ld_p % 4 == 0 && ld_g % 4 == 0 && aligned16(p) && aligned16(g);
    const int64_t cols = vec4 ? 1024 : 256;
    const int64_t n_chunks = (ncols + cols - 1) / cols;
    const int64_t items = n_rows * n_chunks;
    const dim3 grid((unsigned)(items < kMaxGrid ? items : kMaxGrid)), block(256);
    if (vec4)
        hipLaunchKernelGGL(k_sgd_step_rows<4>, grid, block, 0, s, p, ld_p, g, ld_g, ncols, rows, n_rows, neg_lr, n_chunks);
    else
        hipLaunchKernelGGL(k_sgd_step_rows<1>, grid, block, 0, s, p, ld_p, g, ld_g, ncols, rows, n_rows, neg_lr, n_chunks);
    return check_launch("k_sgd_step_rows");
}

int niidmix_update_rows_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t n_rows,
                            int64_t p, const float *avg, void *stream) {
    if (n_rows < 0 || p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (n_rows == 0 || p == 0) return NIIDMIX_OK;
    if (!x || !y || !avg) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (ld_x < p || ld_y < p) return set_error(NIIDMIX_EINVAL, "leading dimension < p");
    const int64_t ext_x = (n_rows - 1) * ld_x + p, ext_y = (n_rows - 1) * ld_y + p;
    if (!(x == y && ld_x == ld_y) && overlaps(x, ext_x, y, ext_y))
        return set_error(NIIDMIX_EALIAS, "x and y overlap without being the same slab");
    if (overlaps(x, ext_x, avg, p) || overlaps(y, ext_y, avg, p))
        return set_error(NIIDMIX_EALIAS, "avg overlaps a slab");
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const bool vec4 = p % 4 == 0 && ld_x % 4 == 0 && ld_y % 4 == 0 && aligned16(x) && aligned16(y) &&
                      aligned16(avg);
    const int64_t cols = vec4 ? 1024 : 256;
    const int64_t n_chunks = (p + cols - 1) / cols;
    const int64_t items = n_rows * n_chunks;
    const dim3 grid((unsigned)(items < kMaxGrid ? items : kMaxGrid)), block(256);
    if (vec4) hipLaunchKernelGGL(k_update_rows<4>, grid, block, 0, s, x, ld_x, y, ld_y, n_rows, p, avg, n_chunks);
    else hipLaunchKernelGGL(k_update_rows<1>, grid, block, 0, s, x, ld_x, y, ld_y, n_rows, p, avg, n_chunks);
    return check_launch("k_update_rows");
}

int niidmix_sharded_create(int n_shards, const int *devices, niidmix_sharded **out) {
    if (!out) return set_error(NIIDMIX_EINVAL, "null handle pointer");
    *out = nullptr;
    if (n_shards < 1 || !devices) return set_error(NIIDMIX_EINVAL, "n_shards < 1 or null device list");
    int n_dev = 0;
    if (hipGetDeviceCount(&n_dev) != hipSuccess) return set_error(NIIDMIX_EHIP, "hipGetDeviceCount failed");
    for (int i = 0; i < n_shards; ++i)
        if (devices[i] < 0 || devices[i] >= n_dev)
            return set_error(NIIDMIX_EINVAL, "device %d of shard %d not visible (%d devices)", devices[i], i, n_dev);
    niidmix_sharded *h = new niidmix_sharded;
    h->n = n_shards;
    h->dev.assign(devices, devices + n_shards);
    for (int i = 0; i < n_shards && !h->loopback; ++i)
        for (int j = 0; j < i; ++j)
            if (devices[i] == devices[j]) h->loopback = true;
    int cur = 0;
    (void)hipGetDevice(&cur);
    int rc = NIIDMIX_OK;
    h->ev_pack.assign(n_shards, nullptr);
    h->ev_copy.assign(n_shards, nullptr);
    for (int i = 0; i < n_shards && rc == NIIDMIX_OK; ++i) {
        (void)hipSetDevice(devices[i]);
        if (hipEventCreateWithFlags(&h->ev_pack[i], hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&h->ev_copy[i], hipEventDisableTiming) != hipSuccess)
            rc = set_error(NIIDMIX_EHIP, "hipEventCreate failed");
    }
    (void)hipSetDevice(cur);
    if (rc == NIIDMIX_OK && !h->loopback) {
        const RcclApi *api = rccl_api();
        if (!api) {
            rc = set_error(NIIDMIX_EHIP, "librccl.so.1 could not be loaded");
        } else {
            h->comm.assign(n_shards, nullptr);
            const ncclResult_t r = api->init_all(h->comm.data(), n_shards, devices);
            if (r != ncclSuccess) {
                h->comm.clear();
                rc = set_error(NIIDMIX_EHIP, "ncclCommInitAll: %s", api->error(r));
            }
        }
    }
    if (rc != NIIDMIX_OK) {
        niidmix_sharded_destroy(h);
        return rc;
    }
    *out = h;
    g_last_error[0] = '\0';
    return NIIDMIX_OK;
}

int niidmix_sharded_destroy(niidmix_sharded *h) {
    if (!h) return NIIDMIX_OK;
    if (!h->comm.empty()) {
        if (const RcclApi *api = rccl_api())
            for (ncclComm_t c : h->comm)
                if (c) (void)api->destroy(c);
    }
    for (hipEvent_t e : h->ev_pack) if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : h->ev_copy) if (e) (void)hipEventDestroy(e);
    delete h;
    return NIIDMIX_OK;
}

int niidmix_sharded_is_loopback(const niidmix_sharded *h) { return h && h->loopback ? 1 : 0; }

int niidmix_mix_sharded_f32(niidmix_sharded *h, const niidmix_shard *sh, int64_t p, int mode) {
    if (!h || !sh) return set_error(NIIDMIX_EINVAL, "null handle or shards");
    if (p < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    const int n = h->n;
    for (int s = 0; s < n; ++s) {                 // host-side validation of every shard first
        const niidmix_shard &a = sh[s];
        if (a.device != h->dev[s]) return set_error(NIIDMIX_EINVAL, "shard %d: device %d, handle has %d", s, a.device, h->dev[s]);
        if (a.n_local < 0 || a.rows_in < a.n_local || a.n_peers < 0 || a.n_peers > n - 1)
            return set_error(NIIDMIX_EINVAL, "shard %d: bad sizes", s);
        if (a.n_local > 0 && (!a.x || !a.y || !a.row_ptr || !a.col || !a.val))
            return set_error(NIIDMIX_EINVAL, "shard %d: null slab or CSR", s);
        if (a.n_peers > 0 && (!a.peer || !a.send_ptr || !a.recv_row || !a.recv_count))
            return set_error(NIIDMIX_EINVAL, "shard %d: null exchange lists", s);
        if (a.x && a.y && overlaps(a.x, a.rows_in * p, a.y, a.n_local * p))
            return set_error(NIIDMIX_EALIAS, "shard %d: x and y overlap", s);
        for (int j = 0; j < a.n_peers; ++j) {
            const int q = a.peer[j];
            if (q < 0 || q >= n || q == s) return set_error(NIIDMIX_EINVAL, "shard %d: bad peer %d", s, q);
            if (a.send_ptr[j + 1] < a.send_ptr[j] || a.recv_count[j] < 0 || a.recv_row[j] < a.n_local ||
                a.recv_row[j] + a.recv_count[j] > a.rows_in)
                return set_error(NIIDMIX_EINVAL, "shard %d: bad exchange ranges for peer %d", s, q);
            if (a.send_ptr[j + 1] > a.send_ptr[0] && (!a.send_rows || !a.send_buf))
                return set_error(NIIDMIX_EINVAL, "shard %d: null send rows / buffer", s);
            // the peer sends exactly what this shard receives from it
            const niidmix_shard &b = sh[q];
            int64_t cnt = -1;
            for (int k = 0; k < b.n_peers; ++k)
                if (b.peer[k] == s) cnt = b.send_ptr[k + 1] - b.send_ptr[k];
            if (cnt != a.recv_count[j] && !(cnt < 0 && a.recv_count[j] == 0))
                return set_error(NIIDMIX_EINVAL, "shard %d receives %lld rows from %d, which sends %lld",
                                 s, (long long)a.recv_count[j], q, (long long)cnt);
        }
    }
    if (p == 0) return NIIDMIX_OK;
    int cur = 0;
    (void)hipGetDevice(&cur);
    int rc = NIIDMIX_OK;
    // 1. pack the rows every peer reads (each shard's stream)
    for (int s = 0; s < n && rc == NIIDMIX_OK; ++s) {
        const niidmix_shard &a = sh[s];
        (void)hipSetDevice(a.device);
        hipStream_t st = reinterpret_cast<hipStream_t>(a.stream);
        const int64_t rows = a.n_peers ? a.send_ptr[a.n_peers] - a.send_ptr[0] : 0;
        if (rows > 0) {
            const bool v4 = p % 4 == 0 && aligned16(a.x) && aligned16(a.send_buf);
            const int64_t cols = v4 ? 1024 : 256, nch = (p + cols - 1) / cols;
            const int64_t items = rows * nch;
            const dim3 grid((unsigned)(items < kMaxGrid ? items : kMaxGrid)), block(256);
            const int32_t *r0 = a.send_rows + a.send_ptr[0];
            float *b0 = a.send_buf;
            if (v4) hipLaunchKernelGGL(k_gather_rows<4>, grid, block, 0, st, a.x, p, r0, rows, p, b0, p, nch);
            else hipLaunchKernelGGL(k_gather_rows<1>, grid, block, 0, st, a.x, p, r0, rows, p, b0, p, nch);
            rc = check_launch("k_gather_rows");
        }
        if (rc == NIIDMIX_OK && h->loopback && hipEventRecord(h->ev_pack[s], st) != hipSuccess)
            rc = set_error(NIIDMIX_EHIP, "hipEventRecord failed");
    }
    // 2. exchange: RCCL point-to-point (one group over every shard), or device-to-device copies
    //    when shards share a device
    if (rc == NIIDMIX_OK && !h->loopback && n > 1) {
        const RcclApi *api = rccl_api();
        ncclResult_t r = api->group_start();
        for (int s = 0; s < n && r == ncclSuccess; ++s) {
            const niidmix_shard &a = sh[s];
            hipStream_t st = reinterpret_cast<hipStream_t>(a.stream);
            for (int j = 0; j < a.n_peers && r == ncclSuccess; ++j) {
                const int64_t ns = a.send_ptr[j + 1] - a.send_ptr[j];
                if (ns > 0) r = api->send(a.send_buf + (a.send_ptr[j] - a.send_ptr[0]) * p, (size_t)(ns * p),
                                          ncclFloat32, a.peer[j], h->comm[s], st);
                if (r == ncclSuccess && a.recv_count[j] > 0)
                    r = api->recv(a.x + a.recv_row[j] * p, (size_t)(a.recv_count[j] * p), ncclFloat32,
                                  a.peer[j], h->comm[s], st);
            }
        }
        const ncclResult_t r2 = api->group_end();
        if (r != ncclSuccess || r2 != ncclSuccess)
            rc = set_error(NIIDMIX_EHIP, "RCCL halo exchange: %s", api->error(r != ncclSuccess ? r : r2));
    } else if (rc == NIIDMIX_OK && h->loopback) {
        for (int s = 0; s < n && rc == NIIDMIX_OK; ++s) {
            const niidmix_shard &a = sh[s];
            (void)hipSetDevice(a.device);
            hipStream_t st = reinterpret_cast<hipStream_t>(a.stream);
            for (int j = 0; j < a.n_peers && rc == NIIDMIX_OK; ++j) {
                if (a.recv_count[j] == 0) continue;
                const niidmix_shard &b = sh[a.peer[j]];
                int k = 0;
                while (b.peer[k] != s) ++k;                   // validated above
                if (hipStreamWaitEvent(st, h->ev_pack[a.peer[j]], 0) != hipSuccess ||
                    hipMemcpyAsync(a.x + a.recv_row[j] * p, b.send_buf + (b.send_ptr[k] - b.send_ptr[0]) * p,
                                   (size_t)(a.recv_count[j] * p) * sizeof(float), hipMemcpyDeviceToDevice,
                                   st) != hipSuccess)
                    rc = set_error(NIIDMIX_EHIP, "loopback halo copy failed");
            }
            if (rc == NIIDMIX_OK && hipEventRecord(h->ev_copy[s], st) != hipSuccess)
                rc = set_error(NIIDMIX_EHIP, "hipEventRecord failed");
        }
        // no shard packs again (next round) before every copy out of its buffer is done
        for (int s = 0; s < n && rc == NIIDMIX_OK; ++s) {
            (void)hipSetDevice(sh[s].device);
            for (int q = 0; q < n; ++q)
                if (q != s && hipStreamWaitEvent(reinterpret_cast<hipStream_t>(sh[s].stream), h->ev_copy[q], 0) != hipSuccess)
                    rc = set_error(NIIDMIX_EHIP, "hipStreamWaitEvent failed");
        }
    }
    // 3. mix every shard's rows over [local | halo] (stream-ordered after its receives)
    for (int s = 0; s < n && rc == NIIDMIX_OK; ++s) {
        const niidmix_shard &a = sh[s];
        if (a.n_local == 0) continue;
        (void)hipSetDevice(a.device);
        rc = niidmix_mix_csr_f32(a.x, p, a.y, p, a.n_local, p, a.row_ptr, a.col, a.val, mode, a.stream);
    }
    (void)hipSetDevice(cur);
    return rc;
}

int niidmix_copy2d_async(void *dst, int64_t dpitch_bytes, const void *src, int64_t spitch_bytes,
                         int64_t width_bytes, int64_t rows, int kind, void *stream) {
    if (rows < 0 || width_bytes < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (rows == 0 || width_bytes == 0) return NIIDMIX_OK;
    if (!dst || !src) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (dpitch_bytes < width_bytes || spitch_bytes < width_bytes)
        return set_error(NIIDMIX_EINVAL, "pitch < width");
    hipMemcpyKind k;
    switch (kind) {
        case 0: k = hipMemcpyHostToDevice; break;
        case 1: k = hipMemcpyDeviceToHost; break;
        case 2: k = hipMemcpyDeviceToDevice; break;
        default: return set_error(NIIDMIX_EINVAL, "unknown copy kind %d", kind);
    }
    hipError_t e = hipMemcpy2DAsync(dst, (size_t)dpitch_bytes, src, (size_t)spitch_bytes,
                                    (size_t)width_bytes, (size_t)rows, k,
                                    reinterpret_cast<hipStream_t>(stream));
    if (e != hipSuccess) return set_error(NIIDMIX_EHIP, "hipMemcpy2DAsync: %s", hipGetErrorString(e));
    g_last_error[0] = '\0';
    return NIIDMIX_OK;
}

int niidmix_stream_copy_f32(const float *x, float *y, int64_t n, void *stream) {
    if (n < 0) return set_error(NIIDMIX_EINVAL, "negative size");
    if (n == 0) return NIIDMIX_OK;
    if (!x || !y) return set_error(NIIDMIX_EINVAL, "null pointer");
    if (n % 4 != 0 || !aligned16(x) || !aligned16(y))
        return set_error(NIIDMIX_EUNSUPPORTED, "stream copy needs n %% 4 == 0 and 16-B aligned buffers");
    if ((x < y && x + n > y) || (y < x && y + n > x) || x == y)
        return set_error(NIIDMIX_EALIAS, "x and y overlap");
    const int64_t n4 = n / 4, blocks = (n4 + 255) / 256;
    if (blocks > 0x7fffffffLL) return set_error(NIIDMIX_EUNSUPPORTED, "copy too large for one grid");
    hipLaunchKernelGGL(k_stream_copy, dim3((unsigned)blocks), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), x, y, n4);
    return check_launch("k_stream_copy");
}

}  // extern "C"
