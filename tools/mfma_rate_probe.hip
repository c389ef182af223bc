// Rate probe (measurement tool): cycles per iteration of 8 independent v_mfma_f32_16x16x4_f32 fed
// by VALU products, as the exact LDS tile kernel's matrix-core path issues them.
//   mode 0: each product computed right before its MFMA (one SrcA register reused, as hipcc emits)
//   mode 1: the 8 products computed first into 8 registers, then the 8 MFMAs
//   mode 2: MFMAs only (operands loop-invariant)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void k_rate(int iters, float *out, long long *cyc) {
    f4 acc[8];
    for (int c = 0; c < 8; ++c) acc[c] = (f4){0.f, 0.f, 0.f, 0.f};
    float x[8];
    for (int c = 0; c < 8; ++c) x[c] = 1.0f + 0.001f * (threadIdx.x + c);
    float w = 0.5f + 1e-7f * threadIdx.x, b = (threadIdx.x & 1) ? 1.f : 0.f;
    const long long t0 = clock64();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0) {
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(w * x[c], b, acc[c], 0, 0, 0);
        } else if constexpr (MODE == 1) {
            float a[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) a[c] = w * x[c];
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[c], b, acc[c], 0, 0, 0);
        } else {
#pragma unroll
            for (int c = 0; c < 8; ++c) acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[c], b, acc[c], 0, 0, 0);
        }
        w = w * 1.0000001f;
    }
    const long long t1 = clock64();
    float s = 0.f;
    for (int c = 0; c < 8; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main(int argc, char **argv) {
    const int iters = 4096;
    float *out; long long *cyc;
    (void)hipMalloc(&out, 1024 * 512 * 4); (void)hipMalloc(&cyc, 1024 * 8);
    for (int waves = 1; waves <= 8; waves *= 2)
        for (int mode = 0; mode < 3; ++mode) {
            // one block per CU-ish: 256 blocks of `waves` waves (waves per SIMD ~ waves / 4)
            hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
            (void)hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(k_rate<0>, dim3(256), dim3(64 * waves), 0, 0, iters, out, cyc);
            if (mode == 1) hipLaunchKernelGGL(k_rate<1>, dim3(256), dim3(64 * waves), 0, 0, iters, out, cyc);
            if (mode == 2) hipLaunchKernelGGL(k_rate<2>, dim3(256), dim3(64 * waves), 0, 0, iters, out, cyc);
            (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
            float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
            long long c = 0; (void)hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
            printf("waves/block %d mode %d: %.1f clock64 cycles per iteration (8 MFMA) in block 0, kernel %.3f ms\n",
                   waves, mode, (double)c / iters, ms);
        }
    return 0;
}
