// Feasibility probe (measurement tool, not product code): is v_mfma_f32_16x16x4_f32 with one operand
// in {0, 1} bit-for-bit the k-ordered sequence of IEEE fp32 adds the exact mixing rule needs
// (acc = fl(acc + p_k) for the positions k a row takes, in order)?  D[i][j] = C[i][j] +
// sum_k A[i][k] * B[k][j] with A = products p_k[col i] and B = 0/1 row masks, compared element by
// element with the VALU chain.  Inputs: random magnitudes over 2^-20 .. 2^20 with mixed signs
// (cancellations, rounding ties), several steps chained through the accumulator.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>

typedef float f4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16; return x;
}
__device__ __forceinline__ float rnd(uint32_t s) {
    const uint32_t h = hash32(s), e = hash32(s ^ 0x9e3779b9U);
    const float m = 1.0f + (float)(h & 0xffffff) * (1.0f / 16777216.0f);
    return ((h >> 31) ? -m : m) * __builtin_ldexpf(1.0f, (int)(e % 41) - 20);
}

// each wave: one 16x16 tile (rows i = tile rows, cols j = parameter columns), STEPS x 4 positions
__global__ void k_probe(int steps, uint32_t seed, unsigned long long *bad, float *dump) {
    const int lane = threadIdx.x & 63;
    const uint32_t w = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int i_a = lane & 15, k_a = lane >> 4;        // A[i][k]: here A = product for column i
    const int j_b = lane & 15, k_b = lane >> 4;        // B[k][j]: mask of row j
    f4 acc;
    float ref[4];
    for (int r = 0; r < 4; ++r) {                      // D: col = lane & 15 (row of the tile), row = 4*(lane>>4)+r (column)
        const int col = 4 * (lane >> 4) + r, row = lane & 15;
        const float c0 = rnd(seed + w * 977u + (uint32_t)(col * 16 + row));
        acc[r] = c0;
        ref[r] = c0;
    }
    for (int s = 0; s < steps; ++s) {
        const uint32_t base = seed * 7919u + w * 100003u + (uint32_t)s * 131u;
        const float a = rnd(base + (uint32_t)(k_a * 16 + i_a) + 12345u);             // p_k[col i]
        const uint32_t mk = hash32(base + 777u + (uint32_t)k_b);                        // mask of position k
        const float b = ((mk >> j_b) & 1u) ? 1.0f : 0.0f;                              // row j takes k?
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc, 0, 0, 0);
        // reference chain for this lane's 4 outputs: (row = lane & 15, col = 4*(lane>>4)+r)
        for (int r = 0; r < 4; ++r) {
            const int col = 4 * (lane >> 4) + r, row = lane & 15;
            for (int k = 0; k < 4; ++k) {
                const float p = rnd(base + (uint32_t)(k * 16 + col) + 12345u);
                const uint32_t m = hash32(base + 777u + (uint32_t)k);
                if ((m >> row) & 1u) ref[r] = ref[r] + p;
            }
        }
    }
    for (int r = 0; r < 4; ++r) {
        if (__float_as_uint(acc[r]) != __float_as_uint(ref[r])) {
            atomicAdd(bad, 1ull);
            if (w == 0) { dump[2 * (lane * 4 + r)] = acc[r]; dump[2 * (lane * 4 + r) + 1] = ref[r]; }
        }
    }
}

int main(int argc, char **argv) {
    const int waves = argc > 1 ? atoi(argv[1]) : 65536, steps = argc > 2 ? atoi(argv[2]) : 64;
    unsigned long long *bad; float *dump;
    hipMalloc(&bad, 8); hipMemset(bad, 0, 8);
    hipMalloc(&dump, 64 * 4 * 2 * 4); hipMemset(dump, 0, 64 * 4 * 2 * 4);
    hipLaunchKernelGGL(k_probe, dim3(waves / 4), dim3(256), 0, 0, steps, 12345u, bad, dump);
    unsigned long long h = 0; float d[512];
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(d, dump, sizeof(d), hipMemcpyDeviceToHost);
    printf("mfma 16x16x4 f32 vs sequential adds: %d waves x 1024 outputs x %d steps (4 positions each): %llu mismatching outputs\n",
           waves, steps, h);
    for (int q = 0; q < 8 && h; ++q) printf("  mfma %.9g ref %.9g\n", d[2 * q], d[2 * q + 1]);
    return h ? 1 : 0;
}
