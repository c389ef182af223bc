// hbm_probe7.hip — measurement tool (not product code): does the PHYSICAL placement of the slabs
// decide the clique access pattern's speed?  Runs the clique pattern (item = 100 random rows x 1 KiB
// chunk in registers, nt loads + nt stores, XCD-aware order) on several fresh hipMalloc pairs and on
// hipExtMallocWithFlags(hipDeviceMallocContiguous) pairs, with a linear nt copy as reference.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/hbm_probe7 tools/hbm_probe7.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>
#include <algorithm>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)
typedef float f4 __attribute__((ext_vector_type(4)));

template <int WAVES, int RPW>
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
            v[r] = __builtin_nontemporal_load((const f4 *)(xc + row * p));
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

// blocked layout [P/B][N][B]: item = (column block kb, clique, 1 KiB chunk inside the block)
template <int WAVES, int RPW>
__global__ __launch_bounds__(WAVES * 64) __attribute__((amdgpu_waves_per_eu(8, 8)))
void rows_blocked(const float *__restrict__ x, float *__restrict__ y, long n, long bw, const int *__restrict__ members, int rpc, int n_cliques, long n_chunks) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    const long t = blockIdx.x;
    const long xcd = t & 7, local = t >> 3;
    const long chunk = (local / n_cliques) * 8 + xcd;       // global 256-column chunk
    const int cq = (int)(local % n_cliques);
    if (chunk >= n_chunks) return;
    const long cpb = bw / 256, kb = chunk / cpb, cin = chunk % cpb;
    const float *xc = x + kb * n * bw + cin * 256 + 4 * lane;
    float *yc = y + kb * n * bw + cin * 256 + 4 * lane;
    int myrow = 0;
    if (lane < RPW && wave + WAVES * lane < rpc) myrow = members[cq * rpc + wave + WAVES * lane];
    f4 v[RPW];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
        if (wave + WAVES * r < rpc) {
            const long row = __builtin_amdgcn_readlane(myrow, r);
            v[r] = __builtin_nontemporal_load((const f4 *)(xc + row * bw));
        }
    f4 s = v[0];
#pragma unroll
    for (int r = 1; r < RPW; ++r) s += v[r];
#pragma unroll
    for (int r = 0; r < RPW; ++r)
        if (wave + WAVES * r < rpc) {
            const long row = __builtin_amdgcn_readlane(myrow, r);
            __builtin_nontemporal_store(v[r] + 1e-30f * s, (f4 *)(yc + row * bw));
        }
}

__global__ void once(const f4 *__restrict__ x, f4 *__restrict__ y, long n4) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i < n4) __builtin_nontemporal_store(__builtin_nontemporal_load(x + i), y + i);
}

// VMM slab: `bytes` of device memory built from chunks of the allocation granularity, mapped into
// one VA range in the given chunk order (scramble = shuffled physical placement of VA chunks).
struct VmmSlab { void *va = nullptr; size_t bytes = 0, gran = 0; std::vector<hipMemGenericAllocationHandle_t> h; };
static bool vmm_alloc(VmmSlab &s, size_t bytes, bool scramble, unsigned seed, size_t chunk_mult) {
    hipMemAllocationProp prop = {};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    size_t gran = 0;
    if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum) != hipSuccess) return false;
    const size_t two_mb = 2u << 20;
    gran = (gran < two_mb ? two_mb : gran) * chunk_mult;
    const size_t n = (bytes + gran - 1) / gran;
    s.bytes = n * gran; s.gran = gran; s.h.resize(n);
    for (size_t i = 0; i < n; ++i) if (hipMemCreate(&s.h[i], gran, &prop, 0) != hipSuccess) return false;
    if (hipMemAddressReserve(&s.va, s.bytes, 0, nullptr, 0) != hipSuccess) return false;
    std::vector<size_t> order(n);
    for (size_t i = 0; i < n; ++i) order[i] = i;
    if (scramble) { std::mt19937 g(seed); std::shuffle(order.begin(), order.end(), g); }
    for (size_t i = 0; i < n; ++i)
        if (hipMemMap((char *)s.va + i * gran, gran, 0, s.h[order[i]], 0) != hipSuccess) return false;
    hipMemAccessDesc d = {};
    d.location.type = hipMemLocationTypeDevice; d.location.id = 0; d.flags = hipMemAccessFlagsProtReadWrite;
    return hipMemSetAccess(s.va, s.bytes, &d, 1) == hipSuccess;
}
static void vmm_free(VmmSlab &s) {
    CK(hipMemUnmap(s.va, s.bytes));
    for (auto h : s.h) CK(hipMemRelease(h));
    CK(hipMemAddressFree(s.va, s.bytes));
    s = VmmSlab();
}

int main() {
    const long N = 1000, P = 1 << 20, R = 100, C = N / R;
    const size_t bytes = (size_t)N * P * 4;
    std::vector<int> perm(N);
    for (int i = 0; i < N; ++i) perm[i] = i;
    std::mt19937 g(1337);
    std::shuffle(perm.begin(), perm.end(), g);
    int *dm; CK(hipMalloc(&dm, N * 4)); CK(hipMemcpy(dm, perm.data(), N * 4, hipMemcpyHostToDevice));
    hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    auto timeit = [&](auto launch) {
        for (int i = 0; i < 3; ++i) launch();
        CK(hipDeviceSynchronize());
        const int it = 20;
        CK(hipEventRecord(a));
        for (int i = 0; i < it; ++i) launch();
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        return ms / it;
    };
    const long it1 = C * (((P / 256) + 7) / 8) * 8;
    const long n4 = N * P / 4;
    std::vector<void *> hold;
    // fresh VMM pairs held alive (no chunk reuse), row-major vs blocked B=4096 on each
    {
        std::vector<VmmSlab> keep;
        for (int k = 0; k < 8; ++k) {
            VmmSlab sx, sy;
            if (!vmm_alloc(sx, bytes, false, 0, 1) || !vmm_alloc(sy, bytes, false, 0, 1)) { printf("VMM allocation failed\n"); break; }
            float *x = (float *)sx.va, *y = (float *)sy.va;
            CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
            const float t0 = timeit([&] { rows<16, 7><<<it1, 1024>>>(x, y, P, dm, R, C, P / 256); });
            const float t1 = timeit([&] { rows_blocked<16, 7><<<it1, 1024>>>(x, y, N, 4096, dm, R, C, P / 256); });
            const float t2 = timeit([&] { rows_blocked<16, 7><<<it1, 1024>>>(x, y, N, 16384, dm, R, C, P / 256); });
            printf("fresh VMM pair %d: row-major %.3f ms  blocked B=4096 %.3f ms  B=16384 %.3f ms\n", k, t0, t1, t2);
            fflush(stdout);
            keep.push_back(sx); keep.push_back(sy);
        }
        for (auto &v : keep) vmm_free(v);
    }
    // fresh hipMalloc pairs held alive
    {
        std::vector<float *> keep;
        for (int k = 0; k < 6; ++k) {
            float *x = nullptr, *y = nullptr;
            CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes));
            CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
            const float t0 = timeit([&] { rows<16, 7><<<it1, 1024>>>(x, y, P, dm, R, C, P / 256); });
            const float t1 = timeit([&] { rows_blocked<16, 7><<<it1, 1024>>>(x, y, N, 4096, dm, R, C, P / 256); });
            printf("fresh hipMalloc pair %d: row-major %.3f ms  blocked B=4096 %.3f ms\n", k, t0, t1);
            fflush(stdout);
            keep.push_back(x); keep.push_back(y);
        }
        for (auto v : keep) CK(hipFree(v));
    }
    return 0;
    // blocked layouts on physically contiguous slabs
    {
        float *x = nullptr, *y = nullptr;
        if (hipExtMallocWithFlags((void **)&x, bytes, hipDeviceMallocContiguous) == hipSuccess &&
            hipExtMallocWithFlags((void **)&y, bytes, hipDeviceMallocContiguous) == hipSuccess) {
            CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
            for (long bw : {1L << 20, 1L << 18, 1L << 16, 1L << 14, 1L << 12, 1L << 10}) {
                const float tc = timeit([&] { rows_blocked<16, 7><<<it1, 1024>>>(x, y, N, bw, dm, R, C, P / 256); });
                printf("contiguous, blocked layout B=%8ld: clique pattern %.3f ms\n", bw, tc);
                fflush(stdout);
            }
            CK(hipFree(x)); CK(hipFree(y));
        }
    }
    // x and y inside ONE physically contiguous allocation, y = x + bytes + delta
    {
        const size_t extra = 64u << 20;
        char *buf = nullptr;
        if (hipExtMallocWithFlags((void **)&buf, 2 * bytes + extra, hipDeviceMallocContiguous) == hipSuccess) {
            CK(hipMemset(buf, 0, 2 * bytes + extra));
            for (size_t delta : {0UL, 1024UL, 4096UL, 65536UL, 1UL << 20, 2UL << 20, 3UL << 20, 6UL << 20, 8UL << 20, 17UL << 20, 32UL << 20}) {
                float *x = (float *)buf, *y = (float *)(buf + bytes + delta);
                const float tc = timeit([&] { rows<16, 7><<<it1, 1024>>>(x, y, P, dm, R, C, P / 256); });
                printf("one contiguous buffer, y = x + 4 GiB + %8zu: clique pattern %.3f ms\n", delta, tc);
                fflush(stdout);
            }
            // read-only and write-only halves of the pattern
            CK(hipFree(buf));
        } else {
            printf("contiguous 8 GiB refused\n");
        }
    }
    {
        hipMemAllocationProp prop = {};
        prop.type = hipMemAllocationTypePinned; prop.location.type = hipMemLocationTypeDevice; prop.location.id = 0;
        size_t gran = 0; CK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
        printf("VMM granularity %zu B (chunks used: max(gran, 2 MiB) x mult)\n", gran);
        fflush(stdout);
    }
    for (size_t mult : {1UL, 8UL}) {
        for (int scr = 0; scr < 2; ++scr) {
            for (int k = 0; k < 3; ++k) {
                VmmSlab sx, sy;
                if (!vmm_alloc(sx, bytes, scr, 11 + k, mult) || !vmm_alloc(sy, bytes, scr, 97 + k, mult)) { printf("VMM allocation failed\n"); return 1; }
                float *x = (float *)sx.va, *y = (float *)sy.va;
                CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
                const float tc = timeit([&] { rows<16, 7><<<it1, 1024>>>(x, y, P, dm, R, C, P / 256); });
                const float tl = timeit([&] { once<<<(n4 + 255) / 256, 256>>>((const f4 *)x, (f4 *)y, n4); });
                printf("VMM chunk %zux %s %d: clique pattern %.3f ms (%.0f GB/s)  linear copy %.3f ms\n", mult,
                       scr ? "scrambled " : "in order  ", k, tc, 2.0 * bytes / (tc / 1e3) / 1e9, tl);
                fflush(stdout);
                vmm_free(sx); vmm_free(sy);
            }
        }
    }
    // padded leading dimension on contiguous allocations
    for (long pad : {0L, 64L, 256L, 512L, 768L, 1024L, 4096L, 16384L, 65536L}) {
        const long ld = P + pad;
        const size_t pb = (size_t)N * ld * 4;
        float *x = nullptr, *y = nullptr;
        if (hipExtMallocWithFlags((void **)&x, pb, hipDeviceMallocContiguous) != hipSuccess ||
            hipExtMallocWithFlags((void **)&y, pb, hipDeviceMallocContiguous) != hipSuccess) {
            printf("contiguous allocation refused\n"); break;
        }
        CK(hipMemset(x, 0, pb)); CK(hipMemset(y, 0, pb));
        const float tc = timeit([&] { rows<16, 7><<<it1, 1024>>>(x, y, ld, dm, R, C, P / 256); });
        printf("contiguous pad %6ld: clique pattern %.3f ms (%.0f GB/s)\n", pad, tc, 2.0 * bytes / (tc / 1e3) / 1e9);
        fflush(stdout);
        CK(hipFree(x)); CK(hipFree(y));
    }
    for (int mode = 0; mode < 2; ++mode) {
        for (int k = 0; k < 4; ++k) {
            float *x = nullptr, *y = nullptr;
            if (mode == 0) { CK(hipMalloc(&x, bytes)); CK(hipMalloc(&y, bytes)); }
            else {
                if (hipExtMallocWithFlags((void **)&x, bytes, hipDeviceMallocContiguous) != hipSuccess ||
                    hipExtMallocWithFlags((void **)&y, bytes, hipDeviceMallocContiguous) != hipSuccess) {
                    printf("contiguous allocation refused\n"); break;
                }
            }
            CK(hipMemset(x, 0, bytes)); CK(hipMemset(y, 0, bytes));
            const float tc = timeit([&] { rows<16, 7><<<it1, 1024>>>(x, y, P, dm, R, C, P / 256); });
            const float tl = timeit([&] { once<<<(n4 + 255) / 256, 256>>>((const f4 *)x, (f4 *)y, n4); });
            printf("%s alloc %d: clique pattern %.3f ms (%.0f GB/s)  linear copy %.3f ms\n",
                   mode ? "contiguous" : "hipMalloc ", k, tc, 2.0 * bytes / (tc / 1e3) / 1e9, tl);
            fflush(stdout);
            hold.push_back(x); hold.push_back(y);
            if (hold.size() > 4) { CK(hipFree(hold[0])); CK(hipFree(hold[1])); hold.erase(hold.begin(), hold.begin() + 2); }
        }
        for (void *h : hold) CK(hipFree(h));
        hold.clear();
    }
    return 0;
}
