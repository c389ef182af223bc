// hbm_probe3.hip — measurement tool (not product code): the clique kernel's access pattern
// (item = clique of R rows x column chunk, every row of the clique in registers) under different
// item orders, chunk widths, row paddings and load policies.  Copies x -> y (+ a tiny reduction so
// the loads are all live), reports GB/s of 2*N*P*4 bytes.
//   order sc = 0: XCD-interleaved chunk-major (k_mix_clique's order)
//   order sc > 0: super-chunks of sc chunks, inside one super-chunk clique-major
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe3 tools/hbm_probe3.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

template <int WAVES, int RPW, int VPL, bool NTL, int OCC>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(OCC, 8)))
void rows(const float *__restrict__ x, float *__restrict__ y, long ld, long p, int rpc, int n_cliques, long n_items, long sc) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long t = blockIdx.x;
    long chunk; int cq;
    if (sc == 0) {
        const long xcd = t & 7, local = t >> 3;
        chunk = (local / n_cliques) * 8 + xcd;
        cq = (int)(local % n_cliques);
    } else {
        const long per = sc * n_cliques, s0 = t / per, rem = t % per;
        cq = (int)(rem / sc);
        chunk = s0 * sc + rem % sc;
    }
    constexpr long CW = 256 * VPL;
    if (chunk * CW >= p) return;
    const float *xc = x + chunk * CW + 4 * lane;
    float *yc = y + chunk * CW + 4 * lane;
    f4 v[RPW][VPL];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int k = wave + WAVES * r;
        if (k < rpc) {
#pragma unroll
            for (int u = 0; u < VPL; ++u) {
                const f4 *src = (const f4 *)(xc + ((long)cq * rpc + k) * ld + 256 * u);
                v[r][u] = NTL ? __builtin_nontemporal_load(src) : *src;
            }
        }
    }
    f4 s = v[0][0];
#pragma unroll
    for (int r = 1; r < RPW; ++r) s += v[r][0];
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
        const int k = wave + WAVES * r;
        if (k < rpc) {
#pragma unroll
            for (int u = 0; u < VPL; ++u)
                __builtin_nontemporal_store(v[r][u] + 1e-30f * s, (f4 *)(yc + ((long)cq * rpc + k) * ld + 256 * u));
        }
    }
}

int main(int argc, char **argv) {
    const long N = 1000, P = 1 << 20, R = 100, C = N / R;
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    const size_t bytes = (size_t)N * P * 4;
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
    for (long pad : {0L, 256L, 1024L}) {
        const long ld = P + pad;
        float *x, *y;
        CK(hipMalloc(&x, N * ld * 4)); CK(hipMalloc(&y, N * ld * 4));
        CK(hipMemset(x, 0, N * ld * 4)); CK(hipMemset(y, 0, N * ld * 4));
        for (long sc : {0L, 64L, 512L, 4096L}) {
            char nm[80];
            const long it1 = C * (((P + 255) / 256 + 7) / 8) * 8;
            snprintf(nm, 80, "8x13 v1 pad%ld sc%ld", pad, sc);
            timeit(nm, [&] { rows<8, 13, 1, false, 4><<<it1, 512>>>(x, y, ld, P, R, C, it1, sc); });
            snprintf(nm, 80, "8x13 v1 ntl pad%ld sc%ld", pad, sc);
            timeit(nm, [&] { rows<8, 13, 1, true, 4><<<it1, 512>>>(x, y, ld, P, R, C, it1, sc); });
            const long sc4 = sc / 4;
            if (sc == 0 || sc4 > 0) {
                const long it4 = C * (((P + 1023) / 1024 + 7) / 8) * 8;
                snprintf(nm, 80, "16x7 v4 pad%ld sc%ld", pad, sc4);
                timeit(nm, [&] { rows<16, 7, 4, false, 1><<<it4, 1024>>>(x, y, ld, P, R, C, it4, sc4); });
                snprintf(nm, 80, "16x7 v4 ntl pad%ld sc%ld", pad, sc4);
                timeit(nm, [&] { rows<16, 7, 4, true, 1><<<it4, 1024>>>(x, y, ld, P, R, C, it4, sc4); });
                const long it2 = C * (((P + 511) / 512 + 7) / 8) * 8;
                snprintf(nm, 80, "16x7 v2 ntl pad%ld sc%ld", pad, sc / 2);
                timeit(nm, [&] { rows<16, 7, 2, true, 2><<<it2, 1024>>>(x, y, ld, P, R, C, it2, sc / 2); });
            }
        }
        CK(hipFree(x)); CK(hipFree(y));
    }
    return 0;
}
