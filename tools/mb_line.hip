// Calibration microbenchmarks for the bucket-record layout (not product code).
// Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/mb_line.hip -o tools/libmbline.so
//   k_lane<NX>  : per lane one random NX*16-byte piece (NX x 16-byte loads, lane-private), then with
//                 probability p2/256 a second random piece (dependent round), plus a 20-byte target
//                 read and a 32-byte row write per lane (the query's streaming part)
//   k_lane_nt<NX>: k_lane<NX> with non-temporal target reads and row writes (coop = 2), the engine's stream policy
//   k_coop      : the same 128-byte pieces, but 8 lanes x 16 B load one piece per instruction and
//                 the piece is redistributed through LDS to its owner lane
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

template <int NX>
__global__ __launch_bounds__(256) void k_lane(const uint4* table, uint64_t npieces, const uint8_t* targets,
                                              uint32_t n, uint32_t p2, uint32_t* out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t* tp = reinterpret_cast<const uint32_t*>(targets + 20ull * i);
    uint64_t h = mix(((uint64_t)tp[0] << 32 | tp[1]) ^ tp[2] ^ tp[3] ^ tp[4]);
    uint4 v[NX];
    const uint64_t piece = h % npieces;
#pragma unroll
    for (int x = 0; x < NX; x++) v[x] = table[piece * NX + x];
    uint32_t acc = 0;
#pragma unroll
    for (int x = 0; x < NX; x++) acc += v[x].x ^ v[x].w ^ v[x].y;
    if (((h >> 40) & 255) < p2) {
        const uint64_t p2i = mix(h ^ acc) % npieces;
#pragma unroll
        for (int x = 0; x < NX; x++) v[x] = table[p2i * NX + x];
#pragma unroll
        for (int x = 0; x < NX; x++) acc += v[x].x ^ v[x].w ^ v[x].z;
    }
    uint4 r = make_uint4(acc, acc + 1, acc + 2, acc + 3);
    reinterpret_cast<uint4*>(out + 8ull * i)[0] = r;
    reinterpret_cast<uint4*>(out + 8ull * i)[1] = r;
}

// k_lane<NX> with the streams non-temporal (the target read and the row write), as the engine's kernels do
template <int NX>
__global__ __launch_bounds__(256) void k_lane_nt(const uint4* table, uint64_t npieces, const uint8_t* targets,
                                                 uint32_t n, uint32_t p2, uint32_t* out) {
    typedef uint32_t v4 __attribute__((ext_vector_type(4)));
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t* tp = reinterpret_cast<const uint32_t*>(targets + 20ull * i);
    const uint64_t a = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(tp));
    const uint64_t b = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(tp + 2));
    const uint32_t c = __builtin_nontemporal_load(tp + 4);
    uint64_t h = mix(a ^ (b >> 32) ^ (uint32_t)b ^ c);
    uint4 v[NX];
    const uint64_t piece = h % npieces;
#pragma unroll
    for (int x = 0; x < NX; x++) v[x] = table[piece * NX + x];
    uint32_t acc = 0;
#pragma unroll
    for (int x = 0; x < NX; x++) acc += v[x].x ^ v[x].w ^ v[x].y;
    v4* o = reinterpret_cast<v4*>(out + 8ull * i);
    __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o);
    __builtin_nontemporal_store(v4{acc, acc + 1, acc + 2, acc + 3}, o + 1);
}

// 128-byte pieces; lane l of each 8-lane group loads 16-byte part (l & 7) of the piece of query
// (g*8 + j) for j = 0..7 over 8 instructions; the parts land in LDS and each lane reads its own piece.
__global__ __launch_bounds__(256) void k_coop(const uint4* table, uint64_t npieces, const uint8_t* targets,
                                              uint32_t n, uint32_t p2, uint32_t* out) {
    __shared__ uint4 lds[256 * 8];
    const uint32_t tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const uint32_t i = blockIdx.x * 256 + tid;
    const uint32_t* tp = reinterpret_cast<const uint32_t*>(targets + 20ull * min(i, n - 1));
    uint64_t h = mix(((uint64_t)tp[0] << 32 | tp[1]) ^ tp[2] ^ tp[3] ^ tp[4]);
    const uint64_t piece = h % npieces;
    uint4* my = lds + w * 512;
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t src = (lane & 56) + j;  // query lane whose piece this lane loads part of
        const uint64_t pc = __shfl(piece, src, 64);
        my[src * 8 + (lane & 7)] = table[pc * 8 + (lane & 7)];
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    uint32_t acc = 0;
#pragma unroll
    for (int x = 0; x < 8; x++) { const uint4 v = my[lane * 8 + x]; acc += v.x ^ v.w ^ v.y; }
    if (((h >> 40) & 255) < p2) {
        const uint64_t p2i = mix(h ^ acc) % npieces;
#pragma unroll
        for (int x = 0; x < 8; x++) { const uint4 v = table[p2i * 8 + x]; acc += v.x ^ v.w ^ v.z; }
    }
    if (i >= n) return;
    uint4 r = make_uint4(acc, acc + 1, acc + 2, acc + 3);
    reinterpret_cast<uint4*>(out + 8ull * i)[0] = r;
    reinterpret_cast<uint4*>(out + 8ull * i)[1] = r;
}

extern "C" int mb_line(const void* table, uint64_t bytes, const uint8_t* targets, uint32_t n, uint32_t nx,
                       uint32_t p2, uint32_t coop, uint32_t* out, void* s) {
    dim3 g((n + 255) / 256), b(256);
    const uint4* t = (const uint4*)table;
    hipStream_t st = (hipStream_t)s;
    const uint64_t np = bytes / (16ull * nx);
    if (coop == 2 && nx == 4) hipLaunchKernelGGL(k_lane_nt<4>, g, b, 0, st, t, np, targets, n, p2, out);
    else if (coop == 2 && nx == 8) hipLaunchKernelGGL(k_lane_nt<8>, g, b, 0, st, t, np, targets, n, p2, out);
    else if (coop) hipLaunchKernelGGL(k_coop, g, b, 0, st, t, bytes / 128, targets, n, p2, out);
    else if (nx == 1) hipLaunchKernelGGL(k_lane<1>, g, b, 0, st, t, np, targets, n, p2, out);
    else if (nx == 2) hipLaunchKernelGGL(k_lane<2>, g, b, 0, st, t, np, targets, n, p2, out);
    else if (nx == 4) hipLaunchKernelGGL(k_lane<4>, g, b, 0, st, t, np, targets, n, p2, out);
    else if (nx == 8) hipLaunchKernelGGL(k_lane<8>, g, b, 0, st, t, np, targets, n, p2, out);
    else if (nx == 16) hipLaunchKernelGGL(k_lane<16>, g, b, 0, st, t, np, targets, n, p2, out);
    return hipGetLastError();
}

// dependent-load latency: each lane chases `hops` random pointers in a table of `n` uint32
// (table[i] = next index < n, a permutation), one wave per block; every start index is < n
__global__ void k_chase(const uint32_t* table, uint32_t n, uint32_t hops, uint32_t* out) {
    uint32_t x = (uint32_t)(((uint64_t)threadIdx.x * 7919u + (uint64_t)blockIdx.x * 104729u) % n);
    for (uint32_t h = 0; h < hops; h++) x = table[x];
    out[blockIdx.x * 64 + threadIdx.x] = x;
}

extern "C" int mb_chase(const uint32_t* table, uint32_t n, uint32_t hops, uint32_t blocks, uint32_t* out, void* s) {
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_chase, dim3(blocks), dim3(64), 0, (hipStream_t)s, table, n, hops, out);
    return hipGetLastError();
}
