// hbm_probe.hip — measurement tool (not product code): what HBM rate can a kernel with the clique
// kernel's access pattern reach on this MI355X?  Prints GB/s (algorithmic bytes / time) for:
//   copy_lin      linear float4 copy, grid-stride (the guide's "float4 copy" ceiling)
//   copy_lin_nt   same with non-temporal stores
//   read_lin      linear float4 read (sum), write_lin: linear float4 fill
//   copy_rows     clique pattern: item = (clique of R rows, 256-float chunk), XCD-aware order,
//                 every row copied (no reduction) — the access-pattern ceiling of k_mix_clique
//   copy_rows_w   same with 512-float chunks (2 float4 per lane per row)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe tools/hbm_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void copy_lin(const float4 *__restrict__ x, float4 *__restrict__ y, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) y[i] = x[i];
}
__global__ void copy_lin_nt(const float4 *__restrict__ x, float4 *__restrict__ y, size_t n) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = x[i];
        f4 w = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(w, (f4 *)(y + i));
    }
}
__global__ void copy_lin_ntnt(const float4 *__restrict__ x, float4 *__restrict__ y, size_t n) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        f4 w = __builtin_nontemporal_load((const f4 *)(x + i));
        __builtin_nontemporal_store(w, (f4 *)(y + i));
    }
}
// 2 float4 per thread per iteration, loads first
__global__ void copy_lin2_nt(const float4 *__restrict__ x, float4 *__restrict__ y, size_t n) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
        f4 w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) if (i + u * stride < n) w[u] = *(const f4 *)(x + i + u * stride);
#pragma unroll
        for (int u = 0; u < 4; ++u) if (i + u * stride < n) __builtin_nontemporal_store(w[u], (f4 *)(y + i + u * stride));
    }
}
template <int U>
__global__ __launch_bounds__(256) void copy_once(const float4 *__restrict__ x, float4 *__restrict__ y, size_t n) {
    typedef float f4 __attribute__((ext_vector_type(4)));
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    f4 w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) if (base + 256 * u < n) w[u] = *(const f4 *)(x + base + 256 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) if (base + 256 * u < n) __builtin_nontemporal_store(w[u], (f4 *)(y + base + 256 * u));
}
__global__ void read_lin(const float4 *__restrict__ x, float *__restrict__ out, size_t n) {
    float s = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        float4 v = x[i]; s += v.x + v.y + v.z + v.w;
    }
    if (s == 12345.678f) out[0] = s;
}
__global__ void write_lin(float4 *__restrict__ y, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) y[i] = make_float4(1.f, 2.f, 3.f, 4.f);
}

template <int WAVES, int RPW, int VPL, int NBAR = 0>
__global__ __launch_bounds__(WAVES * 64) void copy_rows(const float *__restrict__ x, float *__restrict__ y, long ld, long p, int rows_per_clique, int n_cliques, long n_items, long sc = 0) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long chunkw = 256 * VPL;
    for (long t = blockIdx.x; t < n_items; t += gridDim.x) {
        long chunk; int cq;
        if (sc == 0) {
            const long xcd = t & 7, local = t >> 3;
            chunk = (local / n_cliques) * 8 + xcd;
            cq = (int)(local % n_cliques);
        } else {   // super-chunks of sc chunks; inside one, clique-major
            const long per = sc * n_cliques, s0 = t / per, rem = t % per;
            cq = (int)(rem / sc);
            chunk = s0 * sc + rem % sc;
        }
        if (chunk * chunkw >= p) continue;
        const float *xc = x + chunk * chunkw;
        float *yc = y + chunk * chunkw;
        float4 v[RPW][VPL];
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int k = wave + WAVES * r;
            if (k < rows_per_clique) {
                const long row = (long)cq * rows_per_clique + k;
#pragma unroll
                for (int u = 0; u < VPL; ++u) v[r][u] = *(const float4 *)(xc + row * ld + 4 * lane + 256 * u);
            }
        }
        if (NBAR > 0) {
            __shared__ float4 red[WAVES][64];
            float4 a = v[0][0];
#pragma unroll
            for (int r = 1; r < RPW; ++r) { a.x += v[r][0].x; a.y += v[r][0].y; }
            red[wave][lane] = a;
            __syncthreads();
            float4 b = red[(wave + 1) % WAVES][lane];
            if (NBAR > 1) __syncthreads();
            v[0][0].x += b.x * 1e-30f;
            if (NBAR > 1) __syncthreads();
        }
#pragma unroll
        for (int r = 0; r < RPW; ++r) {
            const int k = wave + WAVES * r;
            if (k < rows_per_clique) {
                const long row = (long)cq * rows_per_clique + k;
#pragma unroll
                for (int u = 0; u < VPL; ++u) {
                    typedef float f4 __attribute__((ext_vector_type(4)));
                    f4 w = {v[r][u].x, v[r][u].y, v[r][u].z, v[r][u].w};
                    __builtin_nontemporal_store(w, (f4 *)(yc + row * ld + 4 * lane + 256 * u));
                }
            }
        }
    }
}

// wave per (clique, 64-float chunk): lane = one column, all rows of the clique in registers
template <int ROWS>
__global__ __launch_bounds__(256) void copy_rows_dw(const float *__restrict__ x, float *__restrict__ y, long ld, long p, int n_cliques, long n_items) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    for (long t = blockIdx.x; t < n_items; t += gridDim.x) {
        const long xcd = t & 7, local = t >> 3;
        const long chunk = (local / n_cliques) * 8 + xcd;   // 256-float block chunk
        const int cq = (int)(local % n_cliques);
        if (chunk * 256 >= p) continue;
        const float *xc = x + chunk * 256 + wave * 64;
        float *yc = y + chunk * 256 + wave * 64;
        float v[ROWS];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) v[r] = xc[((long)cq * ROWS + r) * ld + lane];
        float s = 0.f;
#pragma unroll
        for (int r = 0; r < ROWS; ++r) s += v[r];
#pragma unroll
        for (int r = 0; r < ROWS; ++r) __builtin_nontemporal_store(0.01f * s + 0.5f * v[r], yc + ((long)cq * ROWS + r) * ld + lane);
    }
}

int main(int argc, char **argv) {
    const long N = argc > 1 ? atol(argv[1]) : 1000, P = argc > 2 ? atol(argv[2]) : (1 << 20);
    const long PAD = argc > 3 ? atol(argv[3]) : 0;      // row padding in floats (ld = P + PAD)
    const long LD = P + PAD;
    const size_t n4 = (size_t)N * P / 4, bytes = (size_t)N * P * 4, alloc = (size_t)N * LD * 4;
    float *x, *y, *o;
    CK(hipMalloc(&x, alloc)); CK(hipMalloc(&y, alloc)); CK(hipMalloc(&o, 64));
    CK(hipMemset(x, 0, alloc)); CK(hipMemset(y, 0, alloc));
    printf("N=%ld P=%ld ld=%ld\n", N, P, LD);
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](const char *name, double moved, auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(a));
        for (int i = 0; i < it; ++i) launch();
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        printf("%-28s %8.3f ms  %8.1f GB/s\n", name, ms / it, moved / (ms / it / 1e3) / 1e9);
    };
    for (int grid : {2048, 8192, 65536}) {
        char nm[64];
        snprintf(nm, 64, "copy_lin g%d", grid);
        timeit(nm, 2.0 * bytes, [&] { copy_lin<<<grid, 256>>>((const float4 *)x, (float4 *)y, n4); });
        snprintf(nm, 64, "copy_lin_nt g%d", grid);
        timeit(nm, 2.0 * bytes, [&] { copy_lin_nt<<<grid, 256>>>((const float4 *)x, (float4 *)y, n4); });
    }
    timeit("copy_lin_ntnt g65536", 2.0 * bytes, [&] { copy_lin_ntnt<<<65536, 256>>>((const float4 *)x, (float4 *)y, n4); });
    timeit("copy_lin2_nt g16384", 2.0 * bytes, [&] { copy_lin2_nt<<<16384, 256>>>((const float4 *)x, (float4 *)y, n4); });
    timeit("copy_lin2_nt g4096", 2.0 * bytes, [&] { copy_lin2_nt<<<4096, 256>>>((const float4 *)x, (float4 *)y, n4); });
    timeit("copy_once U1", 2.0 * bytes, [&] { copy_once<1><<<(n4 + 255) / 256, 256>>>((const float4 *)x, (float4 *)y, n4); });
    timeit("copy_once U2", 2.0 * bytes, [&] { copy_once<2><<<(n4 + 511) / 512, 256>>>((const float4 *)x, (float4 *)y, n4); });
    timeit("copy_once U4", 2.0 * bytes, [&] { copy_once<4><<<(n4 + 1023) / 1024, 256>>>((const float4 *)x, (float4 *)y, n4); });
    timeit("read_lin g8192", 1.0 * bytes, [&] { read_lin<<<8192, 256>>>((const float4 *)x, o, n4); });
    timeit("write_lin g8192", 1.0 * bytes, [&] { write_lin<<<8192, 256>>>((float4 *)y, n4); });
    const int R = 100, C = (int)(N / R);
    {
        const long items = (long)C * (((P + 255) / 256 + 7) / 8) * 8;
        timeit("copy_rows 16x7 c256", 2.0 * bytes, [&] { copy_rows<16, 7, 1><<<items, 1024>>>(x, y, LD, P, R, C, items); });
        for (long sc : {64L, 256L, 1024L, 4096L}) {
            char nm[64];
            snprintf(nm, 64, "copy_rows 16x7 c256 sc%ld", sc);
            timeit(nm, 2.0 * bytes, [&] { copy_rows<16, 7, 1><<<items, 1024>>>(x, y, LD, P, R, C, items, sc); });
            snprintf(nm, 64, "copy_rows 8x13 c256 sc%ld", sc);
            timeit(nm, 2.0 * bytes, [&] { copy_rows<8, 13, 1><<<items, 512>>>(x, y, LD, P, R, C, items, sc); });
        }
        timeit("copy_rows 8x13 c256", 2.0 * bytes, [&] { copy_rows<8, 13, 1><<<items, 512>>>(x, y, LD, P, R, C, items); });
        timeit("copy_rows 16x7 c256 bar1", 2.0 * bytes, [&] { copy_rows<16, 7, 1, 1><<<items, 1024>>>(x, y, LD, P, R, C, items); });
        timeit("copy_rows 16x7 c256 bar2", 2.0 * bytes, [&] { copy_rows<16, 7, 1, 2><<<items, 1024>>>(x, y, LD, P, R, C, items); });
        timeit("copy_rows 8x13 c256 bar1", 2.0 * bytes, [&] { copy_rows<8, 13, 1, 1><<<items, 512>>>(x, y, LD, P, R, C, items); });
        timeit("copy_rows 8x13 c256 bar2", 2.0 * bytes, [&] { copy_rows<8, 13, 1, 2><<<items, 512>>>(x, y, LD, P, R, C, items); });
        timeit("copy_rows 4x25 c256 bar2", 2.0 * bytes, [&] { copy_rows<4, 25, 1, 2><<<items, 256>>>(x, y, LD, P, R, C, items); });
        timeit("copy_rows 4x25 c256", 2.0 * bytes, [&] { copy_rows<4, 25, 1><<<items, 256>>>(x, y, LD, P, R, C, items); });
        timeit("copy_rows_dw 100 c256", 2.0 * bytes, [&] { copy_rows_dw<100><<<items, 256>>>(x, y, LD, P, C, items); });
    }
    {
        const long items = (long)C * (((P + 511) / 512 + 7) / 8) * 8;
        timeit("copy_rows 16x7 c512", 2.0 * bytes, [&] { copy_rows<16, 7, 2><<<items, 1024>>>(x, y, LD, P, R, C, items); });
        timeit("copy_rows 8x13 c512", 2.0 * bytes, [&] { copy_rows<8, 13, 2><<<items, 512>>>(x, y, LD, P, R, C, items); });
    }
    return 0;
}
