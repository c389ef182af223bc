// Rate probe (measurement tool): can the fp32 matrix-core path and the packed-fp32 VALU run side by
// side in one wave?  The exact walker (k_mix_tile_lds) is VALU-issue bound at one v_pk_add_f32 per
// (row, position, column pair); the exact matrix-core path (v_mfma_f32_16x16x4_f32 as a k-ordered
// fma chain) runs at the same 32 fp32 adds / cycle / SIMD.  A hybrid pays only if the two overlap.
//   mode 0: 8 independent v_mfma_f32_16x16x4_f32 per iteration (MFMA only)
//   mode 1: NV independent v_pk_add_f32 per iteration (VALU only)
//   mode 2: both, NV / 8 pk_adds after each MFMA (one instruction stream)
//   mode 3: NV independent v_add_f32 per iteration (unpacked VALU only)
//   mode 4: 8 MFMAs with NV / 8 v_add_f32 after each
// Cycles per iteration (s_memtime, per wave) for 1 and 2 waves per SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE, int NV>
__global__ void k_coexec(int iters, float *out, long long *cyc) {
    f4 acc[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) acc[c] = (f4){0.f, 0.f, 0.f, 0.f};
    f2 v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) v[r] = (f2){1e-3f * r, 2e-3f * r};
    const float a = 1.0f + 1e-3f * threadIdx.x, b = (threadIdx.x & 1) ? 1.f : 0.f;
    const f2 pr = (f2){1e-7f * threadIdx.x, 2e-7f};
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0 || MODE == 2 || MODE == 4) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[c], 0, 0, 0);
                if constexpr (MODE == 2) {
#pragma unroll
                    for (int j = 0; j < NV / 8; ++j)
                        asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v[(c * (NV / 8) + j) & 15]) : "v"(pr));
                } else if constexpr (MODE == 4) {
#pragma unroll
                    for (int j = 0; j < NV / 8; ++j)
                        asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[(c * (NV / 8) + j) & 15][0]) : "v"(pr[0]));
                }
            }
        } else if constexpr (MODE == 3) {
#pragma unroll
            for (int j = 0; j < NV; ++j)
                asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[j & 15][0]) : "v"(pr[0]));
        } else {
#pragma unroll
            for (int j = 0; j < NV; ++j)
                asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(v[j & 15]) : "v"(pr));
        }
    }
    const long long t1 = clock64();
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
#pragma unroll
    for (int r = 0; r < 16; ++r) s += v[r][0] + v[r][1];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE, int NV>
static double run(int waves_per_simd, int iters) {
    const int threads = 256 * waves_per_simd, blocks = 256;
    float *out;
    long long *cyc;
    hipMalloc(&out, sizeof(float) * threads * blocks);
    hipMalloc(&cyc, sizeof(long long) * blocks * (threads / 64));
    hipLaunchKernelGGL((k_coexec<MODE, NV>), dim3(blocks), dim3(threads), 0, 0, iters, out, cyc);
    hipLaunchKernelGGL((k_coexec<MODE, NV>), dim3(blocks), dim3(threads), 0, 0, iters, out, cyc);
    hipDeviceSynchronize();
    const int n = blocks * (threads / 64);
    long long *h = (long long *)malloc(sizeof(long long) * n);
    hipMemcpy(h, cyc, sizeof(long long) * n, hipMemcpyDeviceToHost);
    double m = 0;
    for (int i = 0; i < n; ++i) m += (double)h[i];
    free(h);
    hipFree(out);
    hipFree(cyc);
    return m / n / iters;
}

int main() {
    const int iters = 20000;
    for (int w = 1; w <= 2; ++w) {
        printf("waves/SIMD %d: mfma8 %.1f | pk_add x32 %.1f | mfma8+pk32 %.1f | pk_add x64 %.1f | "
               "mfma8+pk64 %.1f | pk_add x16 %.1f | mfma8+pk16 %.1f cycles/iteration/wave\n", w,
               run<0, 8>(w, iters), run<1, 32>(w, iters), run<2, 32>(w, iters), run<1, 64>(w, iters),
               run<2, 64>(w, iters), run<1, 16>(w, iters), run<2, 16>(w, iters));
        printf("waves/SIMD %d: v_add x32 %.1f | mfma8+add32 %.1f | v_add x64 %.1f | mfma8+add64 %.1f | "
               "v_add x16 %.1f | mfma8+add16 %.1f cycles/iteration/wave\n", w,
               run<3, 32>(w, iters), run<4, 32>(w, iters), run<3, 64>(w, iters), run<4, 64>(w, iters),
               run<3, 16>(w, iters), run<4, 16>(w, iters));
    }
    return 0;
}
