// How fast can a kernel read a replicated 1M-target batch (20 MB) at all? The floor under rt_shard_kernel's
// "nothing in reach" case (not product code).
// Build: hipcc --offload-arch=gfx950 -O3 tools/mb_stream.hip -o tools/mb_stream.bin
//   empty      : the shard kernel's grid (q / 1,024 workgroups of 256), no memory work: dispatch + drain
//   lds<NR,PAD>: the shard kernel's load: 256 * NR targets per workgroup as 16-byte non-temporal loads into LDS, one
//                compare per target (the reach test), NR = 2, 4 (1,024 per workgroup) or 8; PAD more LDS words held
//   reg<U>     : grid-stride 16-byte loads into registers, U per thread in flight, folded; grid = G workgroups
// Each case: `bufs` distinct batches rotated (so the Infinity Cache holds some, as in the shard runs), 200 launches
// timed between two events, plus each launch alone between events (median), µs per launch.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                         \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_empty(uint32_t* flag, uint32_t v) {
    if (v == 0x5EEDF00Du && threadIdx.x == 0) flag[blockIdx.x] = v;
}

template <uint32_t NR, uint32_t PAD = 0>
__global__ __launch_bounds__(256) void k_lds(const uint8_t* __restrict__ tg, uint32_t q, uint64_t lo, uint64_t hi,
                                             uint32_t* flag) {
    __shared__ __attribute__((aligned(16))) uint32_t st[256 * NR * 5 + PAD];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * 256 * NR;
    const uint32_t nq = (uint32_t)std::min<uint64_t>(256 * NR, q - base);
    const u32x4_t* s4 = reinterpret_cast<const u32x4_t*>(tg + 20 * base);
    u32x4_t* d4 = reinterpret_cast<u32x4_t*>(st);
    const uint32_t n4 = 5 * nq / 4;
#pragma unroll
    for (uint32_t k = 0; k < (5 * NR + 3) / 4; k++) {
        const uint32_t x = tid + k * 256;
        if (x < n4) d4[x] = __builtin_nontemporal_load(s4 + x);
    }
    __syncthreads();
    uint32_t hit = 0;
#pragma unroll
    for (uint32_t r = 0; r < NR; r++) {
        const uint32_t j = r * 256 + tid;
        if (j < nq) {
            const uint64_t h = ((uint64_t)__builtin_bswap32(st[5 * j]) << 32) | __builtin_bswap32(st[5 * j + 1]);
            hit += h >= lo && h < hi;
        }
    }
    if (PAD && hit == 0x5EEDF00Du) hit += st[256 * NR * 5 + PAD - 1 - tid];  // (keeps the pad)
    if (hit) flag[blockIdx.x] = hit;
}

// k_lds<4> with at most 4 waves per SIMD (the occupancy of the shard kernel's 105 VGPRs)
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 4))) void k_lds4_occ4(
    const uint8_t* __restrict__ tg, uint32_t q, uint64_t lo, uint64_t hi, uint32_t* flag) {
    __shared__ __attribute__((aligned(16))) uint32_t st[256 * 4 * 5];
    const uint32_t tid = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * 1024;
    const uint32_t nq = (uint32_t)std::min<uint64_t>(1024, q - base);
    const u32x4_t* s4 = reinterpret_cast<const u32x4_t*>(tg + 20 * base);
    u32x4_t* d4 = reinterpret_cast<u32x4_t*>(st);
    const uint32_t n4 = 5 * nq / 4;
#pragma unroll
    for (uint32_t k = 0; k < 5; k++) {
        const uint32_t x = tid + k * 256;
        if (x < n4) d4[x] = __builtin_nontemporal_load(s4 + x);
    }
    __syncthreads();
    uint32_t hit = 0;
#pragma unroll
    for (uint32_t r = 0; r < 4; r++) {
        const uint32_t j = r * 256 + tid;
        if (j < nq) {
            const uint64_t h = ((uint64_t)__builtin_bswap32(st[5 * j]) << 32) | __builtin_bswap32(st[5 * j + 1]);
            hit += h >= lo && h < hi;
        }
    }
    if (hit) flag[blockIdx.x] = hit;
}

template <uint32_t U>
__global__ __launch_bounds__(256) void k_reg(const u32x4_t* __restrict__ src, uint64_t n4, uint32_t* flag) {
    const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
    uint32_t acc = 0;
    for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < n4; b += stride) {
        u32x4_t v[U];
#pragma unroll
        for (uint32_t u = 0; u < U; u++) {
            const uint64_t x = b + (uint64_t)u * 256;
            v[u] = x < n4 ? __builtin_nontemporal_load(src + x) : u32x4_t{0, 0, 0, 0};
        }
#pragma unroll
        for (uint32_t u = 0; u < U; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x5EEDF00Du) flag[blockIdx.x] = acc;
}

template <class F>
static void timeit(const char* name, int bufs, F&& launch) {
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int i = 0; i < 20; i++) launch(i % bufs);
    CK(hipDeviceSynchronize());
    const int R = 200;
    CK(hipEventRecord(a));
    for (int i = 0; i < R; i++) launch(i % bufs);
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::vector<float> one;
    for (int i = 0; i < 41; i++) {
        CK(hipEventRecord(a));
        launch(i % bufs);
        CK(hipEventRecord(b));
        CK(hipEventSynchronize(b));
        float m = 0;
        CK(hipEventElapsedTime(&m, a, b));
        one.push_back(m);
    }
    std::sort(one.begin(), one.end());
    printf("{\"case\": \"%s\", \"us_back_to_back\": %.2f, \"us_alone_median\": %.2f}\n", name, 1e3 * ms / R,
           1e3 * one[one.size() / 2]);
    fflush(stdout);
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
}

int main(int argc, char** argv) {
    const uint32_t q = argc > 1 ? (uint32_t)atol(argv[1]) : (1u << 20);
    const int bufs = argc > 2 ? atoi(argv[2]) : 8;
    const size_t nb = 20ull * q;
    std::vector<uint8_t*> tg(bufs);
    for (auto& p : tg) {
        CK(hipMalloc(&p, nb));
        CK(hipMemset(p, 0x5A, nb));
    }
    uint32_t* flag;
    CK(hipMalloc(&flag, 1 << 20));
    CK(hipDeviceSynchronize());
    printf("{\"targets\": %u, \"bytes\": %zu, \"bufs\": %d}\n", q, nb, bufs);
    const uint64_t lo = 1ull << 60, hi = 1ull << 61;  // (0x5A5A... is outside: nothing in reach)
    timeit("empty, q/1024 workgroups", bufs, [&](int) { k_empty<<<(q + 1023) / 1024, 256>>>(flag, 0); });
    timeit("lds NR=4 (the shard kernel's load)", bufs,
           [&](int i) { k_lds<4><<<(q + 1023) / 1024, 256>>>(tg[i], q, lo, hi, flag); });
    timeit("lds NR=4 + 9 KB LDS (the shard kernel's 29 KB)", bufs,
           [&](int i) { k_lds<4, 2304><<<(q + 1023) / 1024, 256>>>(tg[i], q, lo, hi, flag); });
    timeit("lds NR=4 + 20 KB LDS", bufs,
           [&](int i) { k_lds<4, 5120><<<(q + 1023) / 1024, 256>>>(tg[i], q, lo, hi, flag); });
    timeit("lds NR=4, at most 4 waves per SIMD", bufs,
           [&](int i) { k_lds4_occ4<<<(q + 1023) / 1024, 256>>>(tg[i], q, lo, hi, flag); });
    timeit("lds NR=8", bufs, [&](int i) { k_lds<8><<<(q + 2047) / 2048, 256>>>(tg[i], q, lo, hi, flag); });
    timeit("lds NR=2", bufs, [&](int i) { k_lds<2><<<(q + 511) / 512, 256>>>(tg[i], q, lo, hi, flag); });
    const uint64_t n4 = nb / 16;
    for (uint32_t G : {256u, 512u, 1024u, 2048u}) {
        char nm[64];
        snprintf(nm, sizeof nm, "reg U=4 grid %u", G);
        timeit(nm, bufs, [&](int i) {
            k_reg<4><<<G, 256>>>(reinterpret_cast<const u32x4_t*>(tg[i]), n4, flag);
        });
        snprintf(nm, sizeof nm, "reg U=8 grid %u", G);
        timeit(nm, bufs, [&](int i) {
            k_reg<8><<<G, 256>>>(reinterpret_cast<const u32x4_t*>(tg[i]), n4, flag);
        });
    }
    for (auto p : tg) CK(hipFree(p));
    CK(hipFree(flag));
    return 0;
}
