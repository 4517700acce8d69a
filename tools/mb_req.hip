// Where the random-line request ceiling sits (tools/mb_req.py; not product code).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/mb_req.hip -o tools/libmbreq.so
//   k_vec<ST>  : grid-stride, one random 64-byte line per query by vector loads (4 x 16 B, lane-private);
//                ST: the query's 20-byte target read and 32-byte row write (non-temporal), else the line index
//                comes from a hash of the query number and nothing is written
//   k_mix<ST>  : the first S lanes of each wave fetch their line through the scalar unit (the wave walks them one
//                by one: uniform address, scalar loads into SGPRs, the folded value kept by the owner lane), the
//                other lanes by vector loads as k_vec; S = 0 is k_vec, S = 64 is all-scalar
// The grid size is a parameter, so the rate can be read against the number of workgroups in flight.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

__device__ __forceinline__ uint32_t piece_of(uint64_t h, uint32_t np) {
    return (uint32_t)(((uint64_t)(uint32_t)h * np) >> 32);
}

template <bool ST>
__device__ __forceinline__ uint64_t query_hash(const uint8_t* __restrict__ tg, uint32_t i) {
    if (!ST) return mix(0x9E3779B97F4A7C15ull ^ i);
    const uint32_t* tp = reinterpret_cast<const uint32_t*>(tg + 20ull * i);
    const uint64_t a = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(tp));
    const uint64_t b = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(tp + 2));
    const uint32_t c = __builtin_nontemporal_load(tp + 4);
    return mix(a ^ (b >> 32) ^ (uint32_t)b ^ c);
}

template <bool ST>
__device__ __forceinline__ void emit(uint32_t* __restrict__ out, uint32_t i, uint32_t acc) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    if (ST) {
        v4* o = reinterpret_cast<v4*>(out + 8ull * i);
        __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o);
        __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o + 1);
    } else if (acc == 0x9E3779B9u) {
        out[i & 1023] = acc;  // practically never: keeps the loads alive
    }
}

template <bool ST>
__global__ __launch_bounds__(256) void k_vec(const uint4* __restrict__ tab, uint32_t np, const uint8_t* __restrict__ tg,
                                             uint32_t n, uint32_t* __restrict__ out) {
    for (uint32_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        const uint32_t pc = piece_of(query_hash<ST>(tg, i), np);
        uint4 v[4];
#pragma unroll
        for (int x = 0; x < 4; x++) v[x] = tab[4ull * pc + x];
        uint32_t acc = 0;
#pragma unroll
        for (int x = 0; x < 4; x++) acc += v[x].x ^ v[x].w ^ v[x].y ^ v[x].z;
        emit<ST>(out, i, acc);
    }
}

template <bool ST>
__global__ __launch_bounds__(256) void k_mix(const uint4* __restrict__ tab, uint32_t np, const uint8_t* __restrict__ tg,
                                             uint32_t n, uint32_t S, uint32_t* __restrict__ out) {
    const uint32_t lane = threadIdx.x & 63;
    for (uint32_t i0 = blockIdx.x * 256 + (threadIdx.x & ~63u); i0 < n; i0 += gridDim.x * 256) {
        const uint32_t i = i0 + lane;
        const bool act = i < n;
        const uint32_t pc = act ? piece_of(query_hash<ST>(tg, i), np) : 0;
        uint4 v[4] = {};
        const bool vec = lane >= S && act;
        if (vec) {
#pragma unroll
            for (int x = 0; x < 4; x++) v[x] = tab[4ull * pc + x];
        }
        uint32_t acc = 0;
        for (uint32_t j = 0; j < S; j += 4) {  // four lines in flight per wave (S is a multiple of 4)
            uint32_t a[4];
            uint4 u[4][4];
#pragma unroll
            for (int y = 0; y < 4; y++) {
                const uint4* p = tab + 4ull * __builtin_amdgcn_readlane(pc, j + y);
#pragma unroll
                for (int x = 0; x < 4; x++) u[y][x] = p[x];
            }
#pragma unroll
            for (int y = 0; y < 4; y++) {
                a[y] = 0;
#pragma unroll
                for (int x = 0; x < 4; x++) a[y] += u[y][x].x ^ u[y][x].w ^ u[y][x].y ^ u[y][x].z;
                acc = lane == j + y ? a[y] : acc;
            }
        }
        if (vec) {
#pragma unroll
            for (int x = 0; x < 4; x++) acc += v[x].x ^ v[x].w ^ v[x].y ^ v[x].z;
        }
        if (act) emit<ST>(out, i, acc);
    }
}


// The streams alone and in other forms. F bits: 1 targets (per-lane 8+8+4-byte loads), 2 targets coalesced (the
// wave's 1280 contiguous bytes as 16-byte pieces through LDS), 4 rows (two 16-byte stores per lane), 8 rows coalesced
// (the wave's 2 KB of rows through LDS, 16-byte pieces at consecutive addresses), 16 one random line per query,
// 32 plain (not non-temporal) streams.
template <int F>
__global__ __launch_bounds__(256) void k_parts(const uint4* __restrict__ tab, uint32_t np, const uint8_t* __restrict__ tg,
                                               uint32_t n, uint32_t* __restrict__ out) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    __shared__ uint4 lds[4][128];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    for (uint32_t i0 = blockIdx.x * 256 + (threadIdx.x & ~63u); i0 < n; i0 += gridDim.x * 256) {
        const uint32_t i = i0 + lane;
        uint64_t h = mix(0x9E3779B97F4A7C15ull ^ i);
        if (F & 1) {
            const uint32_t* tp = reinterpret_cast<const uint32_t*>(tg + 20ull * i);
            uint64_t a, b;
            uint32_t c;
            if (F & 32) {
                a = *reinterpret_cast<const uint64_t*>(tp); b = *reinterpret_cast<const uint64_t*>(tp + 2); c = tp[4];
            } else {
                a = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(tp));
                b = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(tp + 2));
                c = __builtin_nontemporal_load(tp + 4);
            }
            h = mix(a ^ (b >> 32) ^ (uint32_t)b ^ c);
        }
        if (F & 2) {  // 80 pieces of 16 bytes per wave (n is a multiple of 64)
            const v4* src = reinterpret_cast<const v4*>(tg + 20ull * i0);
            const v4 p0 = (F & 32) ? src[lane] : __builtin_nontemporal_load(src + lane);
            v4 p1 = {};
            if (lane < 16) p1 = (F & 32) ? src[64 + lane] : __builtin_nontemporal_load(src + 64 + lane);
            uint4* L = lds[w];
            L[lane] = make_uint4(p0.x, p0.y, p0.z, p0.w);
            if (lane < 16) L[64 + lane] = make_uint4(p1.x, p1.y, p1.z, p1.w);
            __builtin_amdgcn_wave_barrier();
            const uint32_t* d = reinterpret_cast<const uint32_t*>(L) + 5 * lane;
            h = mix(((uint64_t)d[0] << 32 | d[1]) ^ d[2] ^ d[3] ^ d[4]);
            __builtin_amdgcn_wave_barrier();
        }
        uint32_t acc = (uint32_t)h;
        if (F & 16) {
            const uint32_t pc = piece_of(h, np);
            uint4 v[4];
#pragma unroll
            for (int x = 0; x < 4; x++) v[x] = tab[4ull * pc + x];
#pragma unroll
            for (int x = 0; x < 4; x++) acc += v[x].x ^ v[x].w ^ v[x].y ^ v[x].z;
        }
        if (F & 4) {
            v4* o = reinterpret_cast<v4*>(out + 8ull * i);
            if (F & 32) { o[0] = v4{acc, acc + 1, acc + 2, acc + 3}; o[1] = v4{acc, acc + 1, acc + 2, acc + 3}; }
            else {
                __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o);
                __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o + 1);
            }
        } else if (F & 8) {
            uint4* L = lds[w];
            L[2 * lane] = make_uint4(acc, acc + 1, acc + 2, acc + 3);
            L[2 * lane + 1] = make_uint4(acc, acc + 1, acc + 2, acc + 3);
            __builtin_amdgcn_wave_barrier();
            v4* o = reinterpret_cast<v4*>(out + 8ull * i0);
            const uint4 r0 = L[lane], r1 = L[64 + lane];
            if (F & 32) { o[lane] = v4{r0.x, r0.y, r0.z, r0.w}; o[64 + lane] = v4{r1.x, r1.y, r1.z, r1.w}; }
            else {
                __builtin_nontemporal_store(v4{r0.x, r0.y, r0.z, r0.w}, o + lane);
                __builtin_nontemporal_store(v4{r1.x, r1.y, r1.z, r1.w}, o + 64 + lane);
            }
            __builtin_amdgcn_wave_barrier();
        } else if (acc == 0x9E3779B9u) {
            out[i & 1023] = acc;
        }
    }
}

// The count-32 shape: 256-byte lines read by four lanes per query (lane p: bytes 64x + 16p, x = 0..3, as
// rt_wl32q_kernel), 128-byte rows stored as the wave's 2 KB run, the 20-byte target. F bits: 1 target, 2 line, 4 rows.
template <int F>
__global__ __launch_bounds__(256) void k_parts32(const uint4* __restrict__ tab, uint32_t np, const uint8_t* __restrict__ tg,
                                                 uint32_t n, uint32_t* __restrict__ out) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const uint32_t lane = threadIdx.x & 63u, p = lane & 3u;
    for (uint32_t g0 = blockIdx.x * 256 + (threadIdx.x & ~63u); (g0 >> 2) < n; g0 += gridDim.x * 256) {
        const uint32_t i = (g0 + lane) >> 2, i0 = g0 >> 2;  // 16 queries per wave
        uint64_t h = mix(0x9E3779B97F4A7C15ull ^ i);
        if (F & 1) {
            const uint32_t* tp = reinterpret_cast<const uint32_t*>(tg + 20ull * i);
            const uint64_t a = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(tp));
            const uint32_t c = __builtin_nontemporal_load(tp + 2 + (p < 2 ? p : 2u));  // the quad reads the rest (dwords 2..4)
            h = mix(a ^ (uint32_t)__shfl((int)c, (int)(lane & ~3u), 64));  // one line per quad
        }
        uint32_t acc = (uint32_t)h;
        if (F & 2) {
            const uint32_t pc = piece_of(h, np / 4);
            uint4 v[4];
#pragma unroll
            for (int x = 0; x < 4; x++) v[x] = tab[16ull * pc + 4 * x + p];
#pragma unroll
            for (int x = 0; x < 4; x++) acc += v[x].x ^ v[x].w ^ v[x].y ^ v[x].z;
        }
        if (F & 4) {  // piece 64h + lane of the wave's 128 pieces
            v4* o = reinterpret_cast<v4*>(out + 32ull * i0);
            __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o + lane);
            __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o + 64 + lane);
        } else if (F & 8) {  // the kernel's per-quad form: 64 contiguous bytes per quad and instruction
            v4* o = reinterpret_cast<v4*>(out + 32ull * i);
            __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o + p);
            __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o + 4 + p);
        } else if (acc == 0x9E3779B9u) {
            out[i & 1023] = acc;
        }
    }
}

}  // namespace

extern "C" int mb_req(const void* table, uint64_t bytes, const uint8_t* targets, uint32_t n, uint32_t mode,
                      uint32_t streams, uint32_t S, uint32_t blocks, uint32_t* out, void* s) {
    const uint4* t = (const uint4*)table;
    const uint32_t np = (uint32_t)(bytes / 64);
    hipStream_t st = (hipStream_t)s;
    dim3 g(blocks ? blocks : (n + 255) / 256), b(256);
    if (mode == 0) {
        if (streams) hipLaunchKernelGGL(k_vec<true>, g, b, 0, st, t, np, targets, n, out);
        else hipLaunchKernelGGL(k_vec<false>, g, b, 0, st, t, np, targets, n, out);
    } else if (mode >= 2) {
        switch (mode - 2) {
#define P(f) case f: hipLaunchKernelGGL(k_parts<f>, g, b, 0, st, t, np, targets, n, out); break;
            P(1) P(4) P(5) P(2) P(8) P(10) P(33) P(36) P(17) P(20) P(21) P(24) P(26) P(18) P(53) P(16)
#undef P
#define P32(f) case 100 + f: hipLaunchKernelGGL(k_parts32<f>, dim3(blocks ? blocks : (4 * n + 255) / 256), b, 0, st, t, np, targets, n, out); break;
            P32(2) P32(4) P32(6) P32(7) P32(3) P32(8) P32(10) P32(11)
#undef P32
            default: return -1;
        }
    } else {
        if (streams) hipLaunchKernelGGL(k_mix<true>, g, b, 0, st, t, np, targets, n, S, out);
        else hipLaunchKernelGGL(k_mix<false>, g, b, 0, st, t, np, targets, n, S, out);
    }
    return hipGetLastError();
}
