/*
 * mix_oracle.c — TEST INFRASTRUCTURE ONLY (the checker, never the product path).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library.
 *
 * Plain-C restatement of the reference's per-round mixing, order- and rounding-preserving:
 *   d_sgd.average         /root/reference/tools/simulate/algorithm/d_sgd.py:96-116
 *     models   = [self] + [nodes[src] for src in edges[rank]]             (:105)
 *     _weights = [W[rank,rank]] + [W[src,rank] for src in edges[rank]]    (:106)
 *   setup.model.average   /root/reference/tools/setup/model/__init__.py:15-25
 *     center = deepcopy(models[0]); p.mul_(0)       -> z = x_self * 0      (:19-21)
 *     for m, w: c1.add_(w*p1)                        -> acc = fl(acc + fl(w*x_j))  (:22-24)
 *   update_models         /root/reference/tools/simulate/algorithm/d_sgd.py:29-35
 *     p.mul_(0.); p.add_(new_p)                      -> y = fl(x_self*0 + acc)     (:33-34)
 * ATen's CPU mul/add_ round each operation separately (no contraction); so does this file, compiled
 * with -ffp-contract=off and without -ffast-math (see oracle/Makefile).  Parity of this restatement
 * with the reference itself is pinned by the tests/golden npz fixtures, produced by running the reference
 * (tests/golden/make_golden.py); tests/test_oracle_golden.py checks it bit for bit.
 *
 * CSR convention (same as include/niidmix.h): row r's entries [row_ptr[r], row_ptr[r+1]) list
 * (input row, weight) in the reference's order, the node itself first.
 */
#include <stdint.h>
#include <string.h>

#if defined(__FP_FAST_FMAF) || defined(__FAST_MATH__)
#error "mix_oracle.c must be compiled without fast-math / FMA contraction"
#endif

/* y[r, 0:p) for r in [r0, r1).  Columns are independent, so any column slice [c0, c1) of the full
 * problem can be checked in isolation (used for full-size parity on sampled column windows). */
void oracle_mix_csr_f32(const float *x, int64_t ld_x, float *y, int64_t ld_y, int64_t r0,
                        int64_t r1, int64_t c0, int64_t c1, const int64_t *row_ptr,
                        const int32_t *col, const float *val, int average_only) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t r = r0; r < r1; ++r) {
        const int64_t beg = row_ptr[r], end = row_ptr[r + 1];
        float *out = y + r * ld_y;
        if (beg == end) {
            for (int64_t c = c0; c < c1; ++c) out[c] = 0.0f;
            continue;
        }
        const float *self = x + (int64_t)col[beg] * ld_x;
        for (int64_t c = c0; c < c1; ++c) {
            const float z = self[c] * 0.0f;
            float acc = z;
            for (int64_t k = beg; k < end; ++k) {
                const float t = val[k] * x[(int64_t)col[k] * ld_x + c];
                acc = acc + t;
            }
            out[c] = average_only ? acc : z + acc;
        }
    }
}

/* Uniform average of n rows (setup.model.average with weights=None: w = float(1./len(models)),
 * applied as an fp32 multiply, model/__init__.py:17-18). */
void oracle_mean_rows_f32(const float *x, int64_t ld_x, int64_t n, int64_t p, float *mean) {
    const float w = (float)(1.0 / (double)n);
#pragma omp parallel for schedule(static)
    for (int64_t c = 0; c < p; ++c) {
        float acc = n > 0 ? x[c] * 0.0f : 0.0f;
        for (int64_t k = 0; k < n; ++k) {
            const float t = w * x[k * ld_x + c];
            acc = acc + t;
        }
        mean[c] = acc;
    }
}

/* Gradient mean (the --clique-gradient / --unbiased-gradient path): row r of g_out is the mean of
 * the gradients its CSR row lists, in the reference's order:
 *   average_gradients (d_sgd.py:19-27): acc = zeros_like (+0); acc.add_(g_j) per model; div_(len)
 *   update_gradients  (d_sgd.py:37-45): grad.zero_(); grad.add_(mean)   ->  +0 + mean
 * Rows with no entries are written as +0. */
void oracle_grad_mean_f32(const float *g, int64_t ld_g, float *y, int64_t ld_y, int64_t r0,
                          int64_t r1, int64_t c0, int64_t c1, const int64_t *row_ptr,
                          const int32_t *col) {
#pragma omp parallel for schedule(dynamic, 4)
    for (int64_t r = r0; r < r1; ++r) {
        const int64_t beg = row_ptr[r], end = row_ptr[r + 1];
        float *out = y + r * ld_y;
        const float len = (float)(end > beg ? end - beg : 1);
        for (int64_t c = c0; c < c1; ++c) {
            float acc = 0.0f;
            for (int64_t k = beg; k < end; ++k) acc = acc + g[(int64_t)col[k] * ld_g + c];
            const float mean = acc / len;
            out[c] = 0.0f + mean;
        }
    }
}
