// Microbenchmarks that calibrate the access patterns of the closest-node kernels on MI355X
// (not product code). Build: hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/microbench.hip -o tools/libmb.so
//   mb_stream   : per lane 20-byte record read (5 dwords) + 32-byte row write (2 x 16 B)  [abl1 pattern]
//   mb_gather   : per lane R random 64-byte pieces (4 x 16 B loads each), dependent rounds D
//   mb_gather_coop: same bytes, but 4 lanes x 16 B per piece (one line per 4 lanes)
#include <hip/hip_runtime.h>
#include <cstdint>

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    return x;
}

__global__ void k_stream(const uint8_t* in, uint32_t* out, uint32_t n) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t* p = (const uint32_t*)(in + 20ull * i);
    uint32_t a = p[0] ^ p[1] ^ p[2] ^ p[3] ^ p[4];
    uint4 v = make_uint4(a, a + 1, a + 2, a + 3);
    ((uint4*)(out + 8ull * i))[0] = v;
    ((uint4*)(out + 8ull * i))[1] = v;
}

// rounds: D dependent steps, each R independent 64-byte pieces per lane
template <int R>
__global__ void k_gather(const uint4* table, uint64_t npieces, uint32_t n, uint32_t D, uint32_t* out) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t h = mix(i + 12345);
    uint32_t acc = 0;
    for (uint32_t d = 0; d < D; d++) {
        uint4 v[R][4];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint64_t piece = mix(h + r) % npieces;
#pragma unroll
            for (int x = 0; x < 4; x++) v[r][x] = table[piece * 4 + x];
        }
#pragma unroll
        for (int r = 0; r < R; r++)
#pragma unroll
            for (int x = 0; x < 4; x++) acc += v[r][x].x ^ v[r][x].w;
        h = mix(h ^ acc);
    }
    out[i] = acc;
}

// cooperative: a lane quad shares one query; each lane loads one 16-byte part of the piece
template <int R>
__global__ void k_gather_coop(const uint4* table, uint64_t npieces, uint32_t n, uint32_t D, uint32_t* out) {
    uint32_t t = blockIdx.x * 256 + threadIdx.x;
    uint32_t i = t >> 2, part = t & 3;
    if (i >= n) return;
    uint64_t h = mix(i + 12345);
    uint32_t acc = 0;
    for (uint32_t d = 0; d < D; d++) {
        uint4 v[R];
#pragma unroll
        for (int r = 0; r < R; r++) {
            const uint64_t piece = mix(h + r) % npieces;
            v[r] = table[piece * 4 + part];
        }
#pragma unroll
        for (int r = 0; r < R; r++) acc += v[r].x ^ v[r].w;
        acc += __shfl_xor(acc, 1, 64);
        acc += __shfl_xor(acc, 2, 64);
        h = mix(h ^ acc);
    }
    if (part == 0) out[i] = acc;
}

// rounds of R independent pieces of NX x 16 bytes per lane (piece-size calibration)
template <int R, int NX>
__global__ void k_gather_sz(const uint4* table, uint64_t npieces, uint32_t n, uint32_t* out) {
    uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    uint64_t h = mix(i + 777);
    uint32_t acc = 0;
    uint4 v[R][NX];
#pragma unroll
    for (int r = 0; r < R; r++) {
        const uint64_t piece = mix(h + r) % npieces;
#pragma unroll
        for (int x = 0; x < NX; x++) v[r][x] = table[piece * NX + x];
    }
#pragma unroll
    for (int r = 0; r < R; r++)
#pragma unroll
        for (int x = 0; x < NX; x++) acc += v[r][x].x ^ v[r][x].w;
    out[i] = acc;
}

extern "C" {
int mb_gather_sz(const void* table, uint64_t bytes, uint32_t n, uint32_t R, uint32_t NX, uint32_t* out, void* s) {
    dim3 g((n + 255) / 256), b(256);
    const uint4* t = (const uint4*)table;
    hipStream_t st = (hipStream_t)s;
    const uint64_t np = bytes / (16ull * NX);
    if (R == 1 && NX == 2) hipLaunchKernelGGL((k_gather_sz<1, 2>), g, b, 0, st, t, np, n, out);
    if (R == 1 && NX == 4) hipLaunchKernelGGL((k_gather_sz<1, 4>), g, b, 0, st, t, np, n, out);
    if (R == 1 && NX == 8) hipLaunchKernelGGL((k_gather_sz<1, 8>), g, b, 0, st, t, np, n, out);
    if (R == 1 && NX == 16) hipLaunchKernelGGL((k_gather_sz<1, 16>), g, b, 0, st, t, np, n, out);
    if (R == 2 && NX == 8) hipLaunchKernelGGL((k_gather_sz<2, 8>), g, b, 0, st, t, np, n, out);
    if (R == 4 && NX == 2) hipLaunchKernelGGL((k_gather_sz<4, 2>), g, b, 0, st, t, np, n, out);
    return hipGetLastError();
}

int mb_stream(const uint8_t* in, uint32_t* out, uint32_t n, void* s) {
    hipLaunchKernelGGL(k_stream, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)s, in, out, n);
    return hipGetLastError();
}
int mb_gather(const void* table, uint64_t npieces, uint32_t n, uint32_t R, uint32_t D, uint32_t* out, void* s) {
    dim3 g((n + 255) / 256), b(256);
    const uint4* t = (const uint4*)table;
    hipStream_t st = (hipStream_t)s;
    if (R == 1) hipLaunchKernelGGL(k_gather<1>, g, b, 0, st, t, npieces, n, D, out);
    if (R == 2) hipLaunchKernelGGL(k_gather<2>, g, b, 0, st, t, npieces, n, D, out);
    if (R == 4) hipLaunchKernelGGL(k_gather<4>, g, b, 0, st, t, npieces, n, D, out);
    return hipGetLastError();
}
int mb_gather_coop(const void* table, uint64_t npieces, uint32_t n, uint32_t R, uint32_t D, uint32_t* out, void* s) {
    dim3 g((4ull * n + 255) / 256), b(256);
    const uint4* t = (const uint4*)table;
    hipStream_t st = (hipStream_t)s;
    if (R == 1) hipLaunchKernelGGL(k_gather_coop<1>, g, b, 0, st, t, npieces, n, D, out);
    if (R == 2) hipLaunchKernelGGL(k_gather_coop<2>, g, b, 0, st, t, npieces, n, D, out);
    if (R == 4) hipLaunchKernelGGL(k_gather_coop<4>, g, b, 0, st, t, npieces, n, D, out);
    return hipGetLastError();
}
}
