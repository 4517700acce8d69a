// kad_hash.hip — batched InfoHash::get: the 20-byte ID of a key is its SHA-1
// (src/infohash.cpp:46-61: gnutls_fingerprint with GNUTLS_DIG_SHA1 since HASH_LEN = 20). FIPS 180-4
// SHA-1, one lane per key, pinned by the standard's test vectors (tests/test_sha1.py).
// Keys are byte strings packed back to back: key i = data[off[i] .. off[i+1]). For each 64-byte
// message block a lane loads the 17 dwords from the 4-aligned address at or below the block start
// in one burst (16-byte loads where the whole chunk holds key bytes, single dwords at the key's end;
// a dword is read only if it holds a key byte, so no read leaves the key's pages), then funnel-shifts
// them into the 16 big-endian message words and applies the padding arithmetically.
// One burst per block matters: reading word by word with the lanes strided by the key length
// re-fetched each line many times (100-byte keys ran 3x slower per block than 20-byte keys).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "../../include/kadgpu.h"

namespace kadgpu_internal {
int set_error(int code, const char* msg);
}  // namespace kadgpu_internal

namespace {

constexpr int BLOCK = 256;

__device__ __forceinline__ uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

// The 16 message words of block bk of the padded message of the `len`-byte key at p.
__device__ __forceinline__ void load_block(const uint8_t* p, uint64_t len, uint64_t bk, bool last, uint32_t (&w)[16]) {
    const uint64_t j0 = 64 * bk;  // first byte of the block
    uint32_t d[17];
#pragma unroll
    for (int x = 0; x < 17; x++) d[x] = 0;
    uint32_t sh = 0;
    if (j0 < len) {
        const uint8_t* pb = p + j0;
        sh = (uint32_t)((uintptr_t)pb & 3);
        const uint32_t* q = reinterpret_cast<const uint32_t*>(pb - sh);
        const uint64_t rem = len - j0 + sh;  // key bytes from q on
#pragma unroll
        for (int c = 0; c < 4; c++) {
            if (16 * c + 16 <= rem) {
                uint4 v;
                __builtin_memcpy(&v, q + 4 * c, 16);
                d[4 * c] = v.x, d[4 * c + 1] = v.y, d[4 * c + 2] = v.z, d[4 * c + 3] = v.w;
            } else {
#pragma unroll
                for (int e = 0; e < 4; e++)
                    if ((uint64_t)(16 * c + 4 * e) < rem) d[4 * c + e] = q[4 * c + e];
            }
        }
        if (64 < rem) d[16] = q[16];
    }
#pragma unroll
    for (int k = 0; k < 16; k++) {
        const uint64_t j = j0 + 4 * k;
        uint32_t v = __builtin_bswap32(__builtin_amdgcn_alignbyte(d[k + 1], d[k], sh));  // byte shift
        if (j + 4 > len) {  // key end inside or before this word: 0x80 after the last key byte, then zeros
            const uint32_t nv = j < len ? (uint32_t)(len - j) : 0u;
            const uint32_t keep = nv ? ~0u << (32 - 8 * nv) : 0u;
            v = (v & keep) | (j <= len ? 0x80u << (24 - 8 * nv) : 0u);
        }
        w[k] = v;
    }
    if (last) {
        const uint64_t nbits = len * 8;
        w[14] = (uint32_t)(nbits >> 32);
        w[15] = (uint32_t)nbits;
    }
}

__global__ __launch_bounds__(BLOCK) void sha1_kernel(const uint8_t* __restrict__ data,
                                                     const uint64_t* __restrict__ off, uint32_t n,
                                                     uint8_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint8_t* p = data + off[i];
    const uint64_t len = off[i + 1] - off[i];
    uint32_t h0 = 0x67452301u, h1 = 0xEFCDAB89u, h2 = 0x98BADCFEu, h3 = 0x10325476u, h4 = 0xC3D2E1F0u;
    const uint64_t nblk = (len + 8) / 64 + 1;
    for (uint64_t bk = 0; bk < nblk; bk++) {
        uint32_t w[16];
        load_block(p, len, bk, bk == nblk - 1, w);
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
