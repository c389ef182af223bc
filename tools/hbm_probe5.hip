// hbm_probe5.hip — measurement tool (not product code): narrow column panels.
// Layout [P/PW][N][PW]: a PW-column panel of all N rows is contiguous (PW*4 bytes per row).  An
// item is (clique of 100 rows, panel); a wave instruction covers 64/(PW/4) rows x PW columns
// (float4 per lane).  Rows of a clique are consecutive (seq) or a random permutation (rand).
// Every row of the item is held in registers, copied x -> y with a tiny column-sum term.
// Compared with the row-major [N, P] pattern of k_mix_clique on the same box.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe5 tools/hbm_probe5.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

// PW columns per panel; LPR = PW/4 lanes per row; RPI = 64/LPR rows per wave instruction;
// each wave holds K instructions (K*RPI rows); WAVES waves -> WAVES*K*RPI >= rows per clique.
template <int PW, int WAVES, int K, bool NTL, int ORD>
__global__ __launch_bounds__(WAVES * 64) void panel(const float *__restrict__ x, float *__restrict__ y, long n, const int *__restrict__ members, int rpc, int n_cliques, long n_panels) {
    constexpr int LPR = PW / 4, RPI = 64 / LPR;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long t = blockIdx.x;
    long pn; int cq;
    if (ORD == 0) { const long xcd = t & 7, local = t >> 3; pn = (local / n_cliques) * 8 + xcd; cq = (int)(local % n_cliques); }
    else { pn = t / n_cliques; cq = (int)(t % n_cliques); }
    if (pn >= n_panels) return;
    const float *xp = x + pn * n * PW + 4 * (lane % LPR);
    float *yp = y + pn * n * PW + 4 * (lane % LPR);
    const int sub = lane / LPR;
    f4 v[K];
    long rowoff[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        const int m = (wave * K + k) * RPI + sub;      // member index
        rowoff[k] = -1;
        v[k] = (f4){0.f, 0.f, 0.f, 0.f};
        if (m < rpc) {
            rowoff[k] = (long)members[cq * rpc + m] * PW;
            v[k] = NTL ? __builtin_nontemporal_load((const f4 *)(xp + rowoff[k])) : *(const f4 *)(xp + rowoff[k]);
        }
    }
    f4 s = v[0];
#pragma unroll
    for (int k = 1; k < K; ++k) s += v[k];
#pragma unroll
    for (int k = 0; k < K; ++k)
        if (rowoff[k] >= 0) __builtin_nontemporal_store(v[k] + 1e-30f * s, (f4 *)(yp + rowoff[k]));
}

template <int WAVES, int RPW, bool NTL>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(8, 8)))
void rows(const float *__restrict__ x, float *__restrict__ y, long p, const int *__restrict__ members, int rpc, int n_cliques, long n_chunks) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long t = blockIdx.x;
    const long xcd = t & 7, local = t >> 3;
    const long chunk = (local / n_cliques) * 8 + xcd;
    const int cq = (int)(local % n_cliques);
    if (chunk >= n_chunks) return;
    const float *xc = x + chunk * 256 + 4 * lane;
    float *yc = y + chunk * 256 + 4 * lane;
    int myrow = 0;
    if (lane < RPW && wave + WAVES * lane < rpc) myrow = members[cq * rpc + wave + WAVES * lane];
    f4 v[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
        if (wave + WAVES * r < rpc) {
            const long row = __builtin_amdgcn_readlane(myrow, r);
            v[r] = NTL ? __builtin_nontemporal_load((const f4 *)(xc + row * p)) : *(const f4 *)(xc + row * p);
        }
    f4 s = v[0];
#pragma unroll
    for (int r = 1; r < RPW; ++r) s += v[r];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
        if (wave + WAVES * r < rpc) {
            const long row = __builtin_amdgcn_readlane(myrow, r);
            __builtin_nontemporal_store(v[r] + 1e-30f * s, (f4 *)(yc + row * p));
        }
}

template <bool NTL>
__global__ __launch_bounds__(256) void once(const f4 *__restrict__ x, f4 *__restrict__ y, size_t n) {
    const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(NTL ? __builtin_nontemporal_load(x + i) : x[i], y + i);
}

int main() {
    const long N = 1000, P = 1 << 20, R = 100, C = N / R;
    const size_t bytes = (size_t)N * P * 4, n4 = bytes / 16;
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
    for (int rep = 0; rep < 2; ++rep) {
        timeit("once ntl", [&] { once<true><<<(n4 + 255) / 256, 256>>>((const f4 *)x, (f4 *)y, n4); });
        const long it1 = C * (((P / 256) + 7) / 8) * 8;
        timeit("rowmajor rand 16x7", [&] { rows<16, 7, false><<<it1, 1024>>>(x, y, P, drnd, R, C, P / 256); });
        timeit("rowmajor rand 16x7 ntl", [&] { rows<16, 7, true><<<it1, 1024>>>(x, y, P, drnd, R, C, P / 256); });
        for (int perm = 0; perm < 2; ++perm) {
            const int *m = perm ? drnd : dseq;
            const char *pn = perm ? "rand" : "seq";
            char nm[80];
            {   // PW 64: 16 lanes per row, 4 rows per instruction; 4 waves x 7 instr = 112 rows
                const long np = P / 64, it = C * ((np + 7) / 8) * 8;
                snprintf(nm, 80, "panel64 %s 4x7 xcd", pn);
                timeit(nm, [&] { panel<64, 4, 7, false, 0><<<it, 256>>>(x, y, N, m, R, C, np); });
                snprintf(nm, 80, "panel64 %s 4x7 xcd ntl", pn);
                timeit(nm, [&] { panel<64, 4, 7, true, 0><<<it, 256>>>(x, y, N, m, R, C, np); });
                snprintf(nm, 80, "panel64 %s 4x7 lin ntl", pn);
                timeit(nm, [&] { panel<64, 4, 7, true, 1><<<it, 256>>>(x, y, N, m, R, C, np); });
                snprintf(nm, 80, "panel64 %s 2x13 xcd ntl", pn);
                timeit(nm, [&] { panel<64, 2, 13, true, 0><<<it, 128>>>(x, y, N, m, R, C, np); });
            }
            {   // PW 128: 32 lanes per row, 2 rows per instruction; 8 waves x 7 = 112 rows
                const long np = P / 128, it = C * ((np + 7) / 8) * 8;
                snprintf(nm, 80, "panel128 %s 8x7 xcd ntl", pn);
                timeit(nm, [&] { panel<128, 8, 7, true, 0><<<it, 512>>>(x, y, N, m, R, C, np); });
                snprintf(nm, 80, "panel128 %s 4x13 xcd ntl", pn);
                timeit(nm, [&] { panel<128, 4, 13, true, 0><<<it, 256>>>(x, y, N, m, R, C, np); });
            }
            {   // PW 256: 64 lanes per row; 16 waves x 7 = 112 rows
                const long np = P / 256, it = C * ((np + 7) / 8) * 8;
                snprintf(nm, 80, "panel256 %s 16x7 xcd ntl", pn);
                timeit(nm, [&] { panel<256, 16, 7, true, 0><<<it, 1024>>>(x, y, N, m, R, C, np); });
            }
        }
    }
    return 0;
}
