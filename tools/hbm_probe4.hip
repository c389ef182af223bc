// hbm_probe4.hip — measurement tool (not product code): the clique kernel's access pattern on two
// slab layouts.
//   rowmajor  [N, P]            element (r, c) at r*P + c
//   panel     [P/256, N, 256]   element (r, c) at (c/256)*N*256 + r*256 + c%256: a 256-column panel
//                               of all N rows is one contiguous 1 KB-per-row block
// Items are (clique of 100 rows, 256-column chunk), every row of the clique in registers; rows of a
// clique are either consecutive or a random permutation (the reference's random cliques).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe4 tools/hbm_probe4.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

// ORD 0: XCD-interleaved chunk-major (k_mix_clique); 1: plain chunk-major (t -> chunk t / C)
template <int WAVES, int RPW, bool NTL, int OCC, int ORD>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(OCC, 8)))
void rows(const float *__restrict__ x, float *__restrict__ y, long rs, long cs, const int *__restrict__ members, int rpc, int n_cliques, long n_chunks) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long t = blockIdx.x;
    long chunk; int cq;
    if (ORD == 0) {
        const long xcd = t & 7, local = t >> 3;
        chunk = (local / n_cliques) * 8 + xcd;
        cq = (int)(local % n_cliques);
    } else {
        chunk = t / n_cliques;
        cq = (int)(t % n_cliques);
    }
    if (chunk >= n_chunks) return;
    const float *xc = x + chunk * cs + 4 * lane;
    float *yc = y + chunk * cs + 4 * lane;
    int myrow = 0;
    if (lane < RPW && wave + WAVES * lane < rpc) myrow = members[cq * rpc + wave + WAVES * lane];
    f4 v[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int k = wave + WAVES * r;
        if (k < rpc) {
            const long row = __builtin_amdgcn_readlane(myrow, r);
            const f4 *src = (const f4 *)(xc + row * rs);
            v[r] = NTL ? __builtin_nontemporal_load(src) : *src;
        }
    }
    f4 s = v[0];
#pragma unroll
    for (int r = 1; r < RPW; ++r) s += v[r];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int k = wave + WAVES * r;
        if (k < rpc) {
            const long row = __builtin_amdgcn_readlane(myrow, r);
            __builtin_nontemporal_store(v[r] + 1e-30f * s, (f4 *)(yc + row * rs));
        }
    }
}

int main() {
    const long N = 1000, P = 1 << 20, R = 100, C = N / R, NCH = P / 256;
    const size_t bytes = (size_t)N * P * 4;
    float *x, *y;
    CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes));
    CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
    std::vector<int> seq(N), rnd(N);
    for (int i = 0; i < N; ++i) seq[i] = rnd[i] = i;
    std::mt19937 g(1337);
    std::shuffle(rnd.begin(), rnd.end(), g);
    int *dseq, *drnd;
    CK(hipMalloc(&dseq, N * 4)); CK(hipMalloc(&drnd, N * 4));
    CK(hipMemcpy(dseq, seq.data(), N * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(drnd, rnd.data(), N * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](const char *name, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(a));
        for (int i = 0; i < it; ++i) launch();
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        printf("%-40s %8.3f ms  %8.1f GB/s\n", name, ms / it, 2.0 * bytes / (ms / it / 1e3) / 1e9);
        fflush(stdout);
    };
    const long items = C * ((NCH + 7) / 8) * 8;
    for (int layout = 0; layout < 2; ++layout) {
        const long rs = layout ? 256 : P, cs = layout ? N * 256 : 256;
        const char *ln = layout ? "panel" : "rowmajor";
        for (int perm = 0; perm < 2; ++perm) {
            const int *m = perm ? drnd : dseq;
            const char *pn = perm ? "rand" : "seq";
            char nm[80];
            snprintf(nm, 80, "%s %s 16x7 xcd", ln, pn);
            timeit(nm, [&] { rows<16, 7, false, 8, 0><<<items, 1024>>>(x, y, rs, cs, m, R, C, NCH); });
            snprintf(nm, 80, "%s %s 16x7 xcd ntl", ln, pn);
            timeit(nm, [&] { rows<16, 7, true, 8, 0><<<items, 1024>>>(x, y, rs, cs, m, R, C, NCH); });
            snprintf(nm, 80, "%s %s 16x7 lin", ln, pn);
            timeit(nm, [&] { rows<16, 7, false, 8, 1><<<items, 1024>>>(x, y, rs, cs, m, R, C, NCH); });
            snprintf(nm, 80, "%s %s 16x7 lin ntl", ln, pn);
            timeit(nm, [&] { rows<16, 7, true, 8, 1><<<items, 1024>>>(x, y, rs, cs, m, R, C, NCH); });
            snprintf(nm, 80, "%s %s 8x13 lin ntl", ln, pn);
            timeit(nm, [&] { rows<8, 13, true, 4, 1><<<items, 512>>>(x, y, rs, cs, m, R, C, NCH); });
        }
    }
    return 0;
}
