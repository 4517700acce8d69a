// kad_hash.hip — batched InfoHash::get: the 20-byte ID of a key is its SHA-1
// (src/infohash.cpp:46-61: gnutls_fingerprint with GNUTLS_DIG_SHA1 since HASH_LEN = 20). FIPS 180-4
// SHA-1, one lane per key, pinned by the standard's test vectors (tests/test_sha1.py).
// Keys are byte strings packed back to back: key i = data[off[i] .. off[i+1]). Message words are
// read as aligned dwords and funnel-shifted (a dword holding a valid byte never crosses a page),
// the padding words byte by byte.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/kadgpu.h"

namespace kadgpu_internal {
int set_error(int code, const char* msg);
}  // namespace kadgpu_internal

namespace {

constexpr int BLOCK = 256;

__device__ __forceinline__ uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// big-endian message word at byte j of the padded message of a `len`-byte key at p
__device__ __forceinline__ uint32_t msg_word(const uint8_t* p, uint64_t len, uint64_t j, uint64_t nbits, bool last_blk,
                                             int k) {
    if (last_blk && k >= 14) return k == 14 ? (uint32_t)(nbits >> 32) : (uint32_t)nbits;
    if (j + 4 <= len) {
        const uintptr_t a = (uintptr_t)(p + j);
        const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3);
        const uint32_t lo = q[0], hi = sh ? q[1] : 0u;
        return __builtin_bswap32(__builtin_amdgcn_alignbyte(hi, lo, sh));  // byte shift
    }
    uint32_t w = 0;
    for (int b = 0; b < 4; b++) {
        const uint64_t x = j + b;
        const uint32_t v = x < len ? p[x] : (x == len ? 0x80u : 0u);
        w |= v << (24 - 8 * b);
    }
    return w;
}

__global__ void sha1_kernel(const uint8_t* __restrict__ data, const uint64_t* __restrict__ off, uint32_t n,
                            uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = data + off[i];
    const uint64_t len = off[i + 1] - off[i];
    uint32_t h0 = 0x67452301u, h1 = 0xEFCDAB89u, h2 = 0x98BADCFEu, h3 = 0x10325476u, h4 = 0xC3D2E1F0u;
    const uint64_t nblk = (len + 8) / 64 + 1;
    for (uint64_t bk = 0; bk < nblk; bk++) {
        uint32_t w[16];
        const bool last = bk == nblk - 1;
#pragma unroll
        for (int k = 0; k < 16; k++) w[k] = msg_word(p, len, 64 * bk + 4 * k, len * 8, last, k);
        uint32_t a = h0, b = h1, c = h2, d = h3, e = h4;
#pragma unroll
        for (int r = 0; r < 80; r++) {
            uint32_t wr;
            if (r < 16) {
                wr = w[r];
            } else {
                wr = rol(w[(r - 3) & 15] ^ w[(r - 8) & 15] ^ w[(r - 14) & 15] ^ w[r & 15], 1);
                w[r & 15] = wr;
            }
            uint32_t f, kc;
            if (r < 20) { f = (b & c) | (~b & d); kc = 0x5A827999u; }
            else if (r < 40) { f = b ^ c ^ d; kc = 0x6ED9EBA1u; }
            else if (r < 60) { f = (b & c) | (b & d) | (c & d); kc = 0x8F1BBCDCu; }
            else { f = b ^ c ^ d; kc = 0xCA62C1D6u; }
            const uint32_t t = rol(a, 5) + f + e + kc + wr;
            e = d; d = c; c = rol(b, 30); b = a; a = t;
        }
        h0 += a; h1 += b; h2 += c; h3 += d; h4 += e;
    }
    // 20-byte digest, big-endian words (InfoHash byte 0 = most significant)
    uint8_t* o = out + 20ull * i;
    const uint32_t hs[5] = {h0, h1, h2, h3, h4};
#pragma unroll
    for (int x = 0; x < 5; x++)
#pragma unroll
        for (int y = 0; y < 4; y++) o[4 * x + y] = (uint8_t)(hs[x] >> (24 - 8 * y));
}

}  // namespace

extern "C" int kad_infohash_get_batch(const uint8_t* data, const uint64_t* offsets, uint32_t n, uint8_t* out_ids,
                                      int device, void* stream) {
    if (n == 0) return KAD_OK;
    if (!data || !offsets || !out_ids) return kadgpu_internal::set_error(KAD_ERR_INVALID, "NULL buffer");
    int prev = -1;
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != device) (void)hipSetDevice(device);
    hipLaunchKernelGGL(sha1_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, (hipStream_t)stream, data, offsets, n,
                       out_ids);
    const hipError_t e = hipGetLastError();
    if (prev >= 0 && prev != device) (void)hipSetDevice(prev);
    if (e != hipSuccess) return kadgpu_internal::set_error(KAD_ERR_HIP, hipGetErrorString(e));
    return KAD_OK;
}
