// VALU issue-cost probe (tuning tool): cycles per wave-instruction per SIMD for the instruction
// shapes the exact tile kernel's position loop is made of — v_pk_add_f32, v_add_f32, v_cndmask_b32,
// v_mov_b32 and the s_set_gpr_idx save/restore of one accumulator pair — at several waves/SIMD.
//   hipcc --offload-arch=gfx950 -O3 -o valu_probe tools/valu_probe.hip && ./valu_probe
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
typedef float f32v __attribute__((ext_vector_type(32)));
constexpr int ITERS = 4096;

template <int KIND>
__global__ __launch_bounds__(256) void k(float *out, float w, int sel, long long *tick) {
    f32v acc;
#pragma unroll
    for (int i = 0; i < 32; ++i) acc[i] = (float)(threadIdx.x + i);
    f2 tp = {w, w * 2.f};
    float nz = -0.0f * w;
    const int idxv = (int)(threadIdx.x * 7 + sel) & 1023;
    const long long c0 = clock64(), r0w = wall_clock64();
#pragma unroll 2
    for (int it = 0; it < ITERS; ++it) {
        asm volatile("" : "+v"(tp));
        if (KIND == 0) {            // 16 v_pk_add_f32
            f32v T = __builtin_shufflevector(tp, tp, 0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1);
            acc = acc + T;
        } else if (KIND == 1) {     // 32 v_add_f32
#pragma unroll
            for (int i = 0; i < 32; ++i) { float t = tp.x; asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(t)); }
        } else if (KIND == 2) {     // 16 v_pk_add_f32 via asm
#pragma unroll
            for (int i = 0; i < 16; ++i) { f2 a = {acc[2*i], acc[2*i+1]}; asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(tp)); acc[2*i] = a.x; acc[2*i+1] = a.y; }
        } else if (KIND == 3) {     // 32 v_cndmask + 16 pk_add (select path)
            const int m = __builtin_amdgcn_readfirstlane(sel + it);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                f2 t = ((m >> i) & 1) ? tp : (f2){nz, nz};
                f2 a = {acc[2*i], acc[2*i+1]}; a = a + t; acc[2*i] = a.x; acc[2*i+1] = a.y;
            }
        } else if (KIND == 4) {     // 16 pk_add + gpr-idx save/restore of one pair
            const int r0 = __builtin_amdgcn_readfirstlane((sel + it) & 15);
            float s0 = acc[2 * r0], s1 = acc[2 * r0 + 1];
            f32v T = __builtin_shufflevector(tp, tp, 0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1);
            acc = acc + T;
            acc[2 * r0] = s0; acc[2 * r0 + 1] = s1;
        } else if (KIND == 5) {     // 32 v_mov
#pragma unroll
            for (int i = 0; i < 32; ++i) { float t = tp.x; asm volatile("v_mov_b32 %0, %1" : "=v"(acc[i]) : "v"(t)); }
        } else if (KIND == 6) {     // 16 v_pk_mul_f32 via asm
#pragma unroll
            for (int i = 0; i < 16; ++i) { f2 a = {acc[2*i], acc[2*i+1]}; asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "v"(tp)); acc[2*i] = a.x; acc[2*i+1] = a.y; }
        } else if (KIND == 7) {     // 16 v_pk_fma_f32 via asm
#pragma unroll
            for (int i = 0; i < 16; ++i) { f2 a = {acc[2*i], acc[2*i+1]}; asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(a) : "v"(tp)); acc[2*i] = a.x; acc[2*i+1] = a.y; }
        } else if (KIND == 10) {    // as 4, the index from a v_readlane (VALU -> SALU dependency)
            const int r0 = __builtin_amdgcn_readlane(idxv, it & 63) & 15;
            float s0 = acc[2 * r0], s1 = acc[2 * r0 + 1];
            f32v T = __builtin_shufflevector(tp, tp, 0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1);
            acc = acc + T;
            acc[2 * r0] = s0; acc[2 * r0 + 1] = s1;
        } else if (KIND == 11) {    // 16 pk_add + a v_readlane feeding a SALU compare + branch
            const int m = __builtin_amdgcn_readlane(idxv, it & 63);
            f32v T = __builtin_shufflevector(tp, tp, 0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1);
            if (m == 12345) acc[0] += 1.f;
            acc = acc + T;
        } else if (KIND == 12 || KIND == 13) {   // 16 pk_add, and a uniform SGPR-bit branch around a 2-move save/restore
            const uint64_t bits = KIND == 12 ? 0x8040201008040201ull : 0ull;
            f32v T = __builtin_shufflevector(tp, tp, 0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1,0,1);
            const uint64_t bb = (uint64_t)__builtin_amdgcn_readfirstlane(sel) | bits;
            if ((bb >> (it & 63)) & 1ull) {
                const int r0 = (it * 5) & 15;
                float s0 = acc[2 * r0], s1 = acc[2 * r0 + 1];
                acc = acc + T;
                acc[2 * r0] = s0; acc[2 * r0 + 1] = s1;
            } else {
                acc = acc + T;
            }
        } else if (KIND == 14) {  // 16 pk_add, accumulator pairs in banks 0-1, shared operand in 2-3
            asm volatile("v_mov_b64 v[66:67], %0\nv_pk_add_f32 v[0:1], v[0:1], v[66:67]\nv_pk_add_f32 v[4:5], v[4:5], v[66:67]\nv_pk_add_f32 v[8:9], v[8:9], v[66:67]\nv_pk_add_f32 v[12:13], v[12:13], v[66:67]\nv_pk_add_f32 v[16:17], v[16:17], v[66:67]\nv_pk_add_f32 v[20:21], v[20:21], v[66:67]\nv_pk_add_f32 v[24:25], v[24:25], v[66:67]\nv_pk_add_f32 v[28:29], v[28:29], v[66:67]\nv_pk_add_f32 v[32:33], v[32:33], v[66:67]\nv_pk_add_f32 v[36:37], v[36:37], v[66:67]\nv_pk_add_f32 v[40:41], v[40:41], v[66:67]\nv_pk_add_f32 v[44:45], v[44:45], v[66:67]\nv_pk_add_f32 v[48:49], v[48:49], v[66:67]\nv_pk_add_f32 v[52:53], v[52:53], v[66:67]\nv_pk_add_f32 v[56:57], v[56:57], v[66:67]\nv_pk_add_f32 v[60:61], v[60:61], v[66:67]" :: "v"(tp) : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67");
        } else if (KIND == 15) {  // 16 pk_add, accumulator pairs and shared operand all in banks 2-3
            asm volatile("v_mov_b64 v[66:67], %0\nv_pk_add_f32 v[2:3], v[2:3], v[66:67]\nv_pk_add_f32 v[6:7], v[6:7], v[66:67]\nv_pk_add_f32 v[10:11], v[10:11], v[66:67]\nv_pk_add_f32 v[14:15], v[14:15], v[66:67]\nv_pk_add_f32 v[18:19], v[18:19], v[66:67]\nv_pk_add_f32 v[22:23], v[22:23], v[66:67]\nv_pk_add_f32 v[26:27], v[26:27], v[66:67]\nv_pk_add_f32 v[30:31], v[30:31], v[66:67]\nv_pk_add_f32 v[34:35], v[34:35], v[66:67]\nv_pk_add_f32 v[38:39], v[38:39], v[66:67]\nv_pk_add_f32 v[42:43], v[42:43], v[66:67]\nv_pk_add_f32 v[46:47], v[46:47], v[66:67]\nv_pk_add_f32 v[50:51], v[50:51], v[66:67]\nv_pk_add_f32 v[54:55], v[54:55], v[66:67]\nv_pk_add_f32 v[58:59], v[58:59], v[66:67]\nv_pk_add_f32 v[62:63], v[62:63], v[66:67]" :: "v"(tp) : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67");
        } else if (KIND == 16) {  // 16 pk_add, accumulator pairs consecutive (v[0:1], v[2:3], ...)
            asm volatile("v_mov_b64 v[66:67], %0\nv_pk_add_f32 v[0:1], v[0:1], v[66:67]\nv_pk_add_f32 v[2:3], v[2:3], v[66:67]\nv_pk_add_f32 v[4:5], v[4:5], v[66:67]\nv_pk_add_f32 v[6:7], v[6:7], v[66:67]\nv_pk_add_f32 v[8:9], v[8:9], v[66:67]\nv_pk_add_f32 v[10:11], v[10:11], v[66:67]\nv_pk_add_f32 v[12:13], v[12:13], v[66:67]\nv_pk_add_f32 v[14:15], v[14:15], v[66:67]\nv_pk_add_f32 v[16:17], v[16:17], v[66:67]\nv_pk_add_f32 v[18:19], v[18:19], v[66:67]\nv_pk_add_f32 v[20:21], v[20:21], v[66:67]\nv_pk_add_f32 v[22:23], v[22:23], v[66:67]\nv_pk_add_f32 v[24:25], v[24:25], v[66:67]\nv_pk_add_f32 v[26:27], v[26:27], v[66:67]\nv_pk_add_f32 v[28:29], v[28:29], v[66:67]\nv_pk_add_f32 v[30:31], v[30:31], v[66:67]" :: "v"(tp) : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67");
        } else if (KIND == 17) {  // kind 14 without the compiler's unroll (a branch per 17 instructions)
            asm volatile("v_mov_b64 v[66:67], %0\nv_pk_add_f32 v[0:1], v[0:1], v[66:67]\nv_pk_add_f32 v[2:3], v[2:3], v[66:67]\nv_pk_add_f32 v[4:5], v[4:5], v[66:67]\nv_pk_add_f32 v[6:7], v[6:7], v[66:67]\nv_pk_add_f32 v[8:9], v[8:9], v[66:67]\nv_pk_add_f32 v[10:11], v[10:11], v[66:67]\nv_pk_add_f32 v[12:13], v[12:13], v[66:67]\nv_pk_add_f32 v[14:15], v[14:15], v[66:67]\nv_pk_add_f32 v[16:17], v[16:17], v[66:67]\nv_pk_add_f32 v[18:19], v[18:19], v[66:67]\nv_pk_add_f32 v[20:21], v[20:21], v[66:67]\nv_pk_add_f32 v[22:23], v[22:23], v[66:67]\nv_pk_add_f32 v[24:25], v[24:25], v[66:67]\nv_pk_add_f32 v[26:27], v[26:27], v[66:67]\nv_pk_add_f32 v[28:29], v[28:29], v[66:67]\nv_pk_add_f32 v[30:31], v[30:31], v[66:67]" :: "v"(tp) : "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9", "v10", "v11", "v12", "v13", "v14", "v15", "v16", "v17", "v18", "v19", "v20", "v21", "v22", "v23", "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", "v63", "v64", "v65", "v66", "v67");
        } else if (KIND == 8) {     // select by bit-field insert, SALU row mask: 16 s_bfe + 32 v_bfi + 16 pk_add
            const int m = __builtin_amdgcn_readfirstlane(sel + it);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                int mr;
                asm volatile("s_bfe_i32 %0, %1, %2" : "=s"(mr) : "s"(m), "i"((1 << 16) | i));
                f2 t;
                asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(t.x) : "s"(mr), "v"(tp.x), "v"(nz));
                asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(t.y) : "s"(mr), "v"(tp.y), "v"(nz));
                f2 a = {acc[2*i], acc[2*i+1]}; a = a + t; acc[2*i] = a.x; acc[2*i+1] = a.y;
            }
        } else if (KIND == 9) {     // same, row mask by VALU: 16 v_bfe + 32 v_bfi + 16 pk_add
            const int m = __builtin_amdgcn_readfirstlane(sel + it);
            int vm = m;
            asm volatile("" : "+v"(vm));
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                int mr;
                asm volatile("v_bfe_i32 %0, %1, %2, 1" : "=v"(mr) : "v"(vm), "i"(i));
                f2 t;
                asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(t.x) : "v"(mr), "v"(tp.x), "v"(nz));
                asm volatile("v_bfi_b32 %0, %1, %2, %3" : "=v"(t.y) : "v"(mr), "v"(tp.y), "v"(nz));
                f2 a = {acc[2*i], acc[2*i+1]}; a = a + t; acc[2*i] = a.x; acc[2*i+1] = a.y;
            }
        }
    }
    asm volatile("" :: "v"(acc));
    const long long c1 = clock64(), r1w = wall_clock64();
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) s += acc[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if ((threadIdx.x & 63) == 0) {
        const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
        tick[2 * wv] = c1 - c0;
        tick[2 * wv + 1] = r1w - r0w;
    }
}

static const char *names[] = {"16 pk_add (compiler)", "32 v_add_f32", "16 pk_add (asm)", "select path: 32 cndmask + 16 pk_add",
                              "16 pk_add + gpr_idx save/restore", "32 v_mov", "16 pk_mul (asm)", "16 pk_fma (asm)",
                              "bfi select, SALU mask: 32 v_bfi + 16 pk_add", "bfi select, VALU mask: 16 v_bfe + 32 v_bfi + 16 pk_add",
                              "16 pk_add + gpr_idx, index by v_readlane", "16 pk_add + v_readlane->s_cmp->branch",
                              "16 pk_add, SGPR-bit branch, 1/8 save/restore", "16 pk_add, SGPR-bit branch never taken",
                              "16 pk_add, no VGPR bank conflict (+1 v_mov_b64)", "16 pk_add, every one bank-conflicted (+1 mov)",
                              "16 pk_add, consecutive pairs (+1 mov)", "16 pk_add, consecutive pairs, loop not unrolled"};
static const int instrs[] = {16, 32, 16, 48, 16, 32, 16, 16, 48, 64, 16, 16, 16, 16, 17, 17, 17, 17};

template <int KIND>
void run(float *out, long long *tick, int blocks_per_cu) {
    int cus = 256;
    int blocks = cus * blocks_per_cu;                 // 4 waves per block -> blocks_per_cu waves/SIMD
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    k<KIND><<<blocks, 256>>>(out, 1.0001f, 0x5a5a, tick);
    hipEventRecord(a);
    for (int r = 0; r < 5; ++r) k<KIND><<<blocks, 256>>>(out, 1.0001f, 0x5a5a, tick);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    ms /= 5;
    // in-kernel: shader-clock cycles (clock64) and 100 MHz wall ticks (wall_clock64) per wave over
    // the loop; with W waves sharing a SIMD, cycles per wave-instruction of SIMD issue =
    // loop cycles / (W * ITERS * instrs)
    const int waves = blocks * 4;
    static long long h[2 * 256 * 16 * 4];
    hipMemcpy(h, tick, sizeof(long long) * 2 * waves, hipMemcpyDeviceToHost);
    double cyc = 0, wall = 0;
    for (int i = 0; i < waves; ++i) { cyc += h[2 * i]; wall += h[2 * i + 1]; }
    cyc /= waves; wall /= waves;
    const double ghz = cyc / (wall * 10.0);           // wall ticks are 10 ns
    const double per_instr = cyc / ((double)blocks_per_cu * ITERS * instrs[KIND]);
    printf("%-44s waves/SIMD %2d: %.3f ms/launch, loop %.0f cyc @ %.2f GHz -> %.2f cyc per wave-instr"
           " (%.2f by wall time @2.4GHz)\n", names[KIND], blocks_per_cu, ms, cyc, ghz, per_instr,
           ms * 1e-3 * 2.4e9 / ((double)blocks_per_cu * ITERS * instrs[KIND]));
}

int main() {
    float *out;
    long long *tick;
    hipMalloc(&out, 256 * 16 * 256 * sizeof(float));
    hipMalloc(&tick, 2 * 256 * 16 * 4 * sizeof(long long));
    // back-to-back packed and scalar fp32 adds at one and two waves per SIMD
    for (int occ : {1, 2, 4}) {
        run<2>(out, tick, occ); run<1>(out, tick, occ); run<0>(out, tick, occ); run<7>(out, tick, occ);
        run<14>(out, tick, occ); run<15>(out, tick, occ); run<16>(out, tick, occ);
    }
    for (int occ : {2, 4}) { run<4>(out, tick, occ); run<3>(out, tick, occ); }
    hipFree(out);
    hipFree(tick);
    return 0;
}
