// kad_route.hip — owner routing of a serving front end: the headline form shards
// the table by ID range, one GPU per range, and every query is answered by the GPU that owns its target. The
// reference answers each request on the node it arrives at (Dht::onFindNode / onGetValues, dht.cpp:3189-3217); a
// front end that spreads lookups over N shard GPUs must send each target to its owner and the rows back. Device-only
// pieces of that exchange, so that it needs no host read per batch:
//   route_pack_kernel   targets -> `world` fixed-size send blocks (the owner's block), each query's place recorded;
//                       per-workgroup counts in LDS (one LDS atomic per wave and owner), one global atomic per
//                       (workgroup, owner) on the counter of the workgroup's sub-block (8 per block); a full
//                       sub-block sets a sticky overflow word (the caller grows the blocks and runs the batch again)
//   route_unpack_kernel rows that came back in the send layout -> each query's original position
//   route_compress_kernel / route_unpack_packed_kernel: the rows travel back packed (the smallest index + one byte
//                       per entry: 12 bytes for count 8 instead of 33); a row spanning more than 254 indices sets a
//                       sticky word and the caller sends that batch's rows unpacked
// The blocks travel with all_to_all_single (RCCL over xGMI), equal splits: opendht_amd/sharded.py OwnerRoute.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>

#include "../../include/kadgpu.h"

namespace kadgpu_internal {
int set_error(int code, const char* msg);
}  // namespace kadgpu_internal

namespace {

constexpr uint32_t BLOCK = 256, QPT = KAD_ROUTE_QPW / BLOCK;  // queries per thread: a workgroup packs 1,024 targets
constexpr uint32_t NONE = 0xFFFFFFFFu;
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// KEYS (kad_route_pack_keys): each record is the target's top 64 bits as one native 8-byte key instead of its 20 bytes
// (owner routing's key-only exchange: the owner's line paths read nothing else).
template <bool KEYS>
__global__ __launch_bounds__(BLOCK) void route_pack_kernel(const uint8_t* __restrict__ targets, uint32_t q,
                                                            uint32_t world, uint32_t shard_bits, uint32_t cap,
                                                            uint8_t* __restrict__ send, uint32_t* __restrict__ slot,
                                                            uint32_t* __restrict__ ctr) {
    __shared__ uint32_t hcnt[KAD_ROUTE_MAX_WORLD], hbase[KAD_ROUTE_MAX_WORLD];
    const uint32_t tid = threadIdx.x;
    if (tid < KAD_ROUTE_MAX_WORLD) hcnt[tid] = 0;
    __syncthreads();
    uint32_t w[QPT][5], dst[QPT], pos[QPT];
    const uint64_t base = (uint64_t)blockIdx.x * BLOCK * QPT;
    // every target's loads first (QPT x 5 in flight per lane): the LDS atomics below would otherwise order each
    // round's loads after the previous round's placement, QPT dependent memory round trips per workgroup
    // (only the words the record carries: the top 8 bytes for a key). The loads are unconditional — lanes past q
    // re-read record q - 1 (the kernel runs only for q > 0) and are dropped below — so that no use of a record is
    // sunk into a per-round branch with its own wait (the key form then waited for each round's load in turn)
#pragma unroll
    for (uint32_t r = 0; r < QPT; r++) {
        const uint64_t i = min(base + r * BLOCK + tid, (uint64_t)q - 1u);  // consecutive lanes, consecutive records
        const uint32_t* p = reinterpret_cast<const uint32_t*>(targets + 20 * i);
#pragma unroll
        for (int x = 0; x < (KEYS ? 2 : 5); x++) w[r][x] = __builtin_nontemporal_load(p + x);
    }
    // places in the workgroup's count of each owner, the wave's lanes of one owner at consecutive places (their
    // records then leave as contiguous runs): each lane's mask of the lanes sharing its owner from one ballot per
    // owner bit (at most 4 for world <= 16), then one LDS atomic instruction per round for all the wave's owners
    // (the lowest lane of each owner adds its lane count) and one bpermute of the bases — instead of a ballot, an
    // atomic and a read-back per owner, `world` dependent LDS round trips per round
    const uint32_t nbits = world > 1u ? 32u - (uint32_t)__builtin_clz(world - 1u) : 0u;  // (wave-uniform)
    uint32_t lead[QPT], rank[QPT], bse[QPT];
#pragma unroll
    for (uint32_t r = 0; r < QPT; r++) {
        const uint64_t i = base + r * BLOCK + tid;
        dst[r] = NONE;
        if (i < q) {
            const uint32_t b0 = w[r][0] & 0xFFu;  // InfoHash byte 0: the most significant
            dst[r] = shard_bits ? (b0 >> (8 - shard_bits)) % world : 0u;
        }
        uint64_t m = __ballot(dst[r] != NONE);
        for (uint32_t bit = 0; bit < nbits; bit++) {
            const bool set = (dst[r] >> bit) & 1u;
            const uint64_t bb = __ballot(set);
            m &= set ? bb : ~bb;
        }
        rank[r] = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
        lead[r] = m ? (uint32_t)__builtin_ctzll(m) : 0u;
        bse[r] = 0;
        if (dst[r] != NONE && rank[r] == 0u) bse[r] = atomicAdd(&hcnt[dst[r]], (uint32_t)__builtin_popcountll(m));
    }
#pragma unroll
    for (uint32_t r = 0; r < QPT; r++) pos[r] = __shfl(bse[r], (int)lead[r], 64) + rank[r];
    __syncthreads();
    // the workgroup's sub-block of each block: KAD_ROUTE_SUBS counters per block instead of one for every workgroup
    const uint32_t sub = cap / KAD_ROUTE_SUBS, rg = blockIdx.x % KAD_ROUTE_SUBS;
    if (tid < world)
        hbase[tid] = hcnt[tid] ? atomicAdd(ctr + (tid * KAD_ROUTE_SUBS + rg) * KAD_ROUTE_CSTRIDE, hcnt[tid]) : 0u;
    __syncthreads();
#pragma unroll
    for (uint32_t r = 0; r < QPT; r++) {
        const uint64_t i = base + r * BLOCK + tid;
        if (dst[r] == NONE) continue;
        const uint32_t s = hbase[dst[r]] + pos[r];
        uint32_t out = NONE;
        if (s < sub) {
            out = dst[r] * cap + rg * sub + s;
            if (KEYS) {
                uint32_t* o = reinterpret_cast<uint32_t*>(send + 8ull * out);
                o[0] = __builtin_bswap32(w[r][1]);  // (InfoHash bytes 4..7: the key's low word)
                o[1] = __builtin_bswap32(w[r][0]);
            } else {
                uint32_t* o = reinterpret_cast<uint32_t*>(send + 20ull * out);
#pragma unroll
                for (int x = 0; x < 5; x++) o[x] = w[r][x];
            }
        } else {
            atomicOr(ctr + KAD_ROUTE_OVERFLOW_WORD(world), 1u);
        }
        __builtin_nontemporal_store(out, slot + i);
    }
}

// One thread per 16-byte piece of a row when count is a multiple of 4 (the common counts 8, 16, 32), else per
// word; the row of query i comes from place slot[i] of the returned blocks.
template <bool VEC>
__global__ __launch_bounds__(BLOCK) void route_unpack_kernel(const uint32_t* __restrict__ slot, uint32_t q,
                                                             uint32_t count, const uint32_t* __restrict__ back_idx,
                                                             const uint8_t* __restrict__ back_cnt,
                                                             uint32_t* __restrict__ out_idx,
                                                             uint8_t* __restrict__ out_cnt) {
    const uint32_t per = VEC ? count / 4 : count;  // pieces per row
    const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t i = per ? t / per : t;
    if (i >= q) return;
    const uint32_t c = per ? (uint32_t)(t - i * per) : 0u;
    const uint32_t p = slot[i];
    if (per) {
        if (VEC) {
            uint4 v = make_uint4(NONE, NONE, NONE, NONE);
            if (p != NONE) v = *reinterpret_cast<const uint4*>(back_idx + (uint64_t)p * count + 4 * c);
            __builtin_nontemporal_store(v.x, out_idx + i * count + 4 * c);
            __builtin_nontemporal_store(v.y, out_idx + i * count + 4 * c + 1);
            __builtin_nontemporal_store(v.z, out_idx + i * count + 4 * c + 2);
            __builtin_nontemporal_store(v.w, out_idx + i * count + 4 * c + 3);
        } else {
            out_idx[i * count + c] = p != NONE ? back_idx[(uint64_t)p * count + c] : NONE;
        }
    }
    if (c == 0) out_cnt[i] = p != NONE ? back_cnt[p] : (uint8_t)0;
}

// One thread per row: the row's smallest index, then each entry's offset from it in a byte (0xFF past the count).
// W = KAD_ROUTE_PACKED_WORDS(count) words per packed row.
__global__ __launch_bounds__(BLOCK) void route_compress_kernel(const uint32_t* __restrict__ idx,
                                                               const uint8_t* __restrict__ cnt, uint32_t n,
                                                               uint32_t count, uint32_t* __restrict__ packed,
                                                               uint32_t* __restrict__ escape) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t c = min((uint32_t)cnt[i], count), W = KAD_ROUTE_PACKED_WORDS(count);
    const uint32_t* r = idx + (uint64_t)i * count;
    uint32_t lo = NONE, hi = 0;
    for (uint32_t j = 0; j < c; j++) {
        const uint32_t v = r[j];
        lo = min(lo, v);
        hi = max(hi, v);
    }
    uint32_t* o = packed + (uint64_t)i * W;
    o[0] = lo;
    if (c && hi - lo > 254u) atomicOr(escape, 1u);
    for (uint32_t w = 1; w < W; w++) {
        uint32_t b = 0;
#pragma unroll
        for (uint32_t x = 0; x < 4; x++) {
            const uint32_t j = 4 * (w - 1) + x;
            const uint32_t off = j < c ? min(r[j] - lo, 254u) : 255u;
            b |= off << (8 * x);
        }
        o[w] = b;
    }
}

// kad_route_unpack_packed_fold: the batch's counters folded into the caller's flags and zeroed for the next
// kad_route_pack_ex(KAD_ROUTE_ZEROED), by workgroup 0 of the unpack (which runs after the pack, the answer and the
// compress that write them): flags[0..2] |= the overflow / escape / tail words, flags[3] = max(flags[3], KAD_ROUTE_SUBS
// x the fullest sub-block count). No memset before the next pack, no fold launch after this one.
struct RouteFold {
    uint32_t* ctr;  // NULL: no fold
    uint32_t world;
    uint32_t* flags;
};

__device__ void fold_reset(const RouteFold& F) {
    __shared__ uint32_t mx;
    const uint32_t tid = threadIdx.x, nsub = F.world * KAD_ROUTE_SUBS, ov = KAD_ROUTE_OVERFLOW_WORD(F.world);
    if (tid == 0) mx = 0;
    __syncthreads();
    uint32_t m = 0;
    for (uint32_t j = tid; j < nsub; j += BLOCK) m = max(m, F.ctr[j * KAD_ROUTE_CSTRIDE]);
    if (m) atomicMax(&mx, m);
    const uint32_t w = tid < 3 ? F.ctr[ov + tid] : 0u;
    __syncthreads();
    if (tid < 3 && w) F.flags[tid] |= w;
    if (tid == 0) F.flags[3] = max(F.flags[3], KAD_ROUTE_SUBS * mx);
    for (uint32_t j = tid; j < KAD_ROUTE_CTR_WORDS(F.world); j += BLOCK) F.ctr[j] = 0;  // (every read is done)
}

// One thread per query: its packed row (slot[i]) expanded into out_idx row i and out_cnt[i].
__global__ __launch_bounds__(BLOCK) void route_unpack_packed_kernel(const uint32_t* __restrict__ slot, uint32_t q,
                                                                    uint32_t count,
                                                                    const uint32_t* __restrict__ back_packed,
                                                                    uint32_t* __restrict__ out_idx,
                                                                    uint8_t* __restrict__ out_cnt, RouteFold F) {
    if (F.ctr && blockIdx.x == 0) fold_reset(F);
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    const uint32_t p = slot[i], W = KAD_ROUTE_PACKED_WORDS(count);
    const uint32_t* pr = p != NONE ? back_packed + (uint64_t)p * W : nullptr;
    const uint32_t lo = pr ? pr[0] : NONE;
    uint32_t* row = out_idx + (uint64_t)i * count;
    uint32_t c = 0;
    for (uint32_t w = 1; w < W; w++) {
        const uint32_t b = pr ? pr[w] : 0xFFFFFFFFu;
        uint32_t v[4];
#pragma unroll
        for (uint32_t x = 0; x < 4; x++) {
            const uint32_t off = (b >> (8 * x)) & 255u;
            v[x] = off == 255u ? NONE : lo + off;
            c += off != 255u ? 1u : 0u;
        }
        const uint32_t j = 4 * (w - 1);
        if (j + 4 <= count && (count & 3u) == 0 && ((uintptr_t)row & 15u) == 0) {
            __builtin_nontemporal_store(v[0], row + j);
            __builtin_nontemporal_store(v[1], row + j + 1);
            __builtin_nontemporal_store(v[2], row + j + 2);
            __builtin_nontemporal_store(v[3], row + j + 3);
        } else {
#pragma unroll
            for (uint32_t x = 0; x < 4; x++)
                if (j + x < count) row[j + x] = v[x];
        }
    }
    out_cnt[i] = (uint8_t)c;
}

// Counts that are multiples of 4 (the common 8, 16, 32): L = count / 4 lanes per row (a power-of-two group G >= L),
// lane j moving entries 4j..4j+3 as one 16-byte load and one packed dword; the group's min / max by shuffles.
template <uint32_t G>
__global__ __launch_bounds__(BLOCK) void route_compress4_kernel(const uint32_t* __restrict__ idx,
                                                                const uint8_t* __restrict__ cnt, uint32_t n,
                                                                uint32_t count, uint32_t* __restrict__ packed,
                                                                uint32_t* __restrict__ escape) {
    const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t i = t / G;
    const uint32_t j = (uint32_t)(t % G), L = count / 4;
    const bool row = i < n, mine = row && j < L;
    const uint32_t c = row ? min((uint32_t)cnt[i], count) : 0u;
    u32x4_t v = {NONE, NONE, NONE, NONE};
    if (mine) v = __builtin_nontemporal_load(reinterpret_cast<const u32x4_t*>(idx + i * count) + j);
    const uint32_t e[4] = {v.x, v.y, v.z, v.w};
    uint32_t lo = NONE, hi = 0;
#pragma unroll
    for (uint32_t x = 0; x < 4; x++)
        if (4 * j + x < c) {
            lo = min(lo, e[x]);
            hi = max(hi, e[x]);
        }
#pragma unroll
    for (uint32_t o = 1; o < G; o <<= 1) {
        lo = min(lo, (uint32_t)__shfl_xor((int)lo, (int)o, 64));
        hi = max(hi, (uint32_t)__shfl_xor((int)hi, (int)o, 64));
    }
    if (!mine) return;
    uint32_t b = 0;
#pragma unroll
    for (uint32_t x = 0; x < 4; x++) b |= (4 * j + x < c ? min(e[x] - lo, 254u) : 255u) << (8 * x);
    uint32_t* o = packed + i * (1 + L);
    o[1 + j] = b;
    if (j == 0) {
        o[0] = lo;
        if (c && hi - lo > 254u) atomicOr(escape, 1u);
    }
}

template <uint32_t G>
__global__ __launch_bounds__(BLOCK) void route_unpack_packed4_kernel(const uint32_t* __restrict__ slot, uint32_t q,
                                                                     uint32_t count,
                                                                     const uint32_t* __restrict__ back_packed,
                                                                     uint32_t* __restrict__ out_idx,
                                                                     uint8_t* __restrict__ out_cnt, RouteFold F) {
    if (F.ctr && blockIdx.x == 0) fold_reset(F);
    const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
    const uint64_t i = t / G;
    const uint32_t j = (uint32_t)(t % G), L = count / 4;
    const bool mine = i < q && j < L;
    uint32_t lo = NONE, b = 0xFFFFFFFFu;
    if (mine) {
        const uint32_t p = slot[i];
        if (p != NONE) {
            const uint32_t* pr = back_packed + (uint64_t)p * (1 + L);
            lo = pr[0];
            b = pr[1 + j];
        }
    }
    uint32_t v[4], c = 0;
#pragma unroll
    for (uint32_t x = 0; x < 4; x++) {
        const uint32_t off = (b >> (8 * x)) & 255u;
        v[x] = off == 255u ? NONE : lo + off;
        c += off != 255u ? 1u : 0u;
    }
#pragma unroll
    for (uint32_t o = 1; o < G; o <<= 1) c += (uint32_t)__shfl_xor((int)c, (int)o, 64);
    if (!mine) return;
    const u32x4_t w = {v[0], v[1], v[2], v[3]};
    __builtin_nontemporal_store(w, reinterpret_cast<u32x4_t*>(out_idx + i * count) + j);
    if (j == 0) out_cnt[i] = (uint8_t)c;
}

struct DevSwitch {
    int prev = -1;
    explicit DevSwitch(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) (void)hipSetDevice(device);
    }
    ~DevSwitch() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

}  // namespace

static int route_pack(bool keys, bool zeroed, const uint8_t* targets, uint32_t q, uint32_t world, uint32_t shard_bits,
                      uint32_t cap, uint8_t* send, uint32_t* slot, uint32_t* ctr, int device, void* stream) {
    using kadgpu_internal::set_error;
    if (world == 0 || world > KAD_ROUTE_MAX_WORLD) return set_error(KAD_ERR_INVALID, "world must be 1..16");
    if (shard_bits > 8) return set_error(KAD_ERR_INVALID, "shard_bits must be 0..8");
    if (cap == 0 || cap % KAD_ROUTE_SUBS || (uint64_t)world * cap >= NONE)
        return set_error(KAD_ERR_INVALID, "cap must be a positive multiple of KAD_ROUTE_SUBS and world * cap < 2^32 - 1");
    if (!ctr || (q && (!targets || !send || !slot))) return set_error(KAD_ERR_INVALID, "NULL buffer");
    // the kernel moves the 20-byte records as five dwords, the slots and counters as dwords
    if (((uintptr_t)targets | (uintptr_t)send | (uintptr_t)slot | (uintptr_t)ctr) & 3u)
        return set_error(KAD_ERR_INVALID, "targets, send, slot and ctr must be 4-byte aligned");
    DevSwitch g(device);
    hipStream_t s = (hipStream_t)stream;
    hipError_t e = zeroed ? hipSuccess : hipMemsetAsync(ctr, 0, 4ull * KAD_ROUTE_CTR_WORDS(world), s);
    if (e == hipSuccess && q) {
        const uint32_t nb = (uint32_t)(((uint64_t)q + BLOCK * QPT - 1) / (BLOCK * QPT));
        if (keys)
            hipLaunchKernelGGL(route_pack_kernel<true>, dim3(nb), dim3(BLOCK), 0, s, targets, q, world, shard_bits, cap,
                               send, slot, ctr);
        else
            hipLaunchKernelGGL(route_pack_kernel<false>, dim3(nb), dim3(BLOCK), 0, s, targets, q, world, shard_bits, cap,
                               send, slot, ctr);
        e = hipGetLastError();
    }
    if (e != hipSuccess) return set_error(KAD_ERR_HIP, hipGetErrorString(e));
    return KAD_OK;
}

extern "C" int kad_route_pack(const uint8_t* targets, uint32_t q, uint32_t world, uint32_t shard_bits, uint32_t cap,
                              uint8_t* send, uint32_t* slot, uint32_t* ctr, int device, void* stream) {
    return route_pack(false, false, targets, q, world, shard_bits, cap, send, slot, ctr, device, stream);
}

extern "C" int kad_route_pack_ex(const uint8_t* targets, uint32_t q, uint32_t world, uint32_t shard_bits, uint32_t cap,
                                 void* send, uint32_t* slot, uint32_t* ctr, uint32_t mode, int device, void* stream) {
    if (mode & ~(KAD_ROUTE_KEYS | KAD_ROUTE_ZEROED)) return kadgpu_internal::set_error(KAD_ERR_INVALID, "unknown mode bits");
    if ((mode & KAD_ROUTE_KEYS) && ((uintptr_t)send & 7u))
        return kadgpu_internal::set_error(KAD_ERR_INVALID, "send keys must be 8-byte aligned");
    return route_pack(mode & KAD_ROUTE_KEYS, mode & KAD_ROUTE_ZEROED, targets, q, world, shard_bits, cap,
                      reinterpret_cast<uint8_t*>(send), slot, ctr, device, stream);
}

extern "C" int kad_route_pack_keys(const uint8_t* targets, uint32_t q, uint32_t world, uint32_t shard_bits,
                                   uint32_t cap, uint64_t* send_keys, uint32_t* slot, uint32_t* ctr, int device,
                                   void* stream) {
    if ((uintptr_t)send_keys & 7u) return kadgpu_internal::set_error(KAD_ERR_INVALID, "send_keys must be 8-byte aligned");
    return route_pack(true, false, targets, q, world, shard_bits, cap, reinterpret_cast<uint8_t*>(send_keys), slot, ctr,
                      device, stream);
}

extern "C" int kad_route_unpack(const uint32_t* slot, uint32_t q, uint32_t count, const uint32_t* back_idx,
                                const uint8_t* back_cnt, uint32_t* out_idx, uint8_t* out_cnt, int device,
                                void* stream) {
    using kadgpu_internal::set_error;
    if (q == 0) return KAD_OK;
    if (!slot || !back_cnt || !out_cnt || (count && (!back_idx || !out_idx))) return set_error(KAD_ERR_INVALID, "NULL buffer");
    DevSwitch g(device);
    const bool vec = count && count % 4 == 0 && ((uintptr_t)back_idx % 16 == 0) && ((uintptr_t)out_idx % 16 == 0);
    const uint64_t per = count == 0 ? 1 : vec ? count / 4 : count;
    const uint64_t threads = (uint64_t)q * per;
    const dim3 grid((uint32_t)((threads + BLOCK - 1) / BLOCK));
    if (vec)
        hipLaunchKernelGGL(route_unpack_kernel<true>, grid, dim3(BLOCK), 0, (hipStream_t)stream, slot, q, count,
                           back_idx, back_cnt, out_idx, out_cnt);
    else
        hipLaunchKernelGGL(route_unpack_kernel<false>, grid, dim3(BLOCK), 0, (hipStream_t)stream, slot, q, count,
                           back_idx, back_cnt, out_idx, out_cnt);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(KAD_ERR_HIP, hipGetErrorString(e));
    return KAD_OK;
}

extern "C" int kad_route_compress(const uint32_t* idx, const uint8_t* cnt, uint32_t n, uint32_t count,
                                  uint32_t* packed, uint32_t* escape, int device, void* stream) {
    using kadgpu_internal::set_error;
    if (count == 0 || count > KAD_ROUTE_PACKED_MAX_COUNT) return set_error(KAD_ERR_INVALID, "count must be 1..32");
    if (n == 0) return KAD_OK;
    if (!idx || !cnt || !packed || !escape) return set_error(KAD_ERR_INVALID, "NULL buffer");
    DevSwitch g(device);
    hipStream_t s = (hipStream_t)stream;
    if (count % 4 == 0 && (uintptr_t)idx % 16 == 0) {
        const uint32_t L = count / 4, G = L <= 1 ? 1u : L <= 2 ? 2u : L <= 4 ? 4u : 8u;
        const dim3 grid((uint32_t)(((uint64_t)n * G + BLOCK - 1) / BLOCK));
        if (G == 1) hipLaunchKernelGGL(route_compress4_kernel<1>, grid, dim3(BLOCK), 0, s, idx, cnt, n, count, packed, escape);
        else if (G == 2) hipLaunchKernelGGL(route_compress4_kernel<2>, grid, dim3(BLOCK), 0, s, idx, cnt, n, count, packed, escape);
        else if (G == 4) hipLaunchKernelGGL(route_compress4_kernel<4>, grid, dim3(BLOCK), 0, s, idx, cnt, n, count, packed, escape);
        else hipLaunchKernelGGL(route_compress4_kernel<8>, grid, dim3(BLOCK), 0, s, idx, cnt, n, count, packed, escape);
    } else {
        hipLaunchKernelGGL(route_compress_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, idx, cnt, n, count,
                           packed, escape);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(KAD_ERR_HIP, hipGetErrorString(e));
    return KAD_OK;
}

static int unpack_packed(const uint32_t* slot, uint32_t q, uint32_t count, const uint32_t* back_packed,
                         uint32_t* out_idx, uint8_t* out_cnt, RouteFold F, int device, void* stream) {
    using kadgpu_internal::set_error;
    if (count == 0 || count > KAD_ROUTE_PACKED_MAX_COUNT) return set_error(KAD_ERR_INVALID, "count must be 1..32");
    if (q == 0 && !F.ctr) return KAD_OK;
    if (q && (!slot || !back_packed || !out_idx || !out_cnt)) return set_error(KAD_ERR_INVALID, "NULL buffer");
    DevSwitch g(device);
    hipStream_t s = (hipStream_t)stream;
    if (count % 4 == 0 && (uintptr_t)out_idx % 16 == 0) {
        const uint32_t L = count / 4, G = L <= 1 ? 1u : L <= 2 ? 2u : L <= 4 ? 4u : 8u;
        const dim3 grid((uint32_t)std::max<uint64_t>(1, ((uint64_t)q * G + BLOCK - 1) / BLOCK));
        if (G == 1) hipLaunchKernelGGL(route_unpack_packed4_kernel<1>, grid, dim3(BLOCK), 0, s, slot, q, count, back_packed, out_idx, out_cnt, F);
        else if (G == 2) hipLaunchKernelGGL(route_unpack_packed4_kernel<2>, grid, dim3(BLOCK), 0, s, slot, q, count, back_packed, out_idx, out_cnt, F);
        else if (G == 4) hipLaunchKernelGGL(route_unpack_packed4_kernel<4>, grid, dim3(BLOCK), 0, s, slot, q, count, back_packed, out_idx, out_cnt, F);
        else hipLaunchKernelGGL(route_unpack_packed4_kernel<8>, grid, dim3(BLOCK), 0, s, slot, q, count, back_packed, out_idx, out_cnt, F);
    } else {
        hipLaunchKernelGGL(route_unpack_packed_kernel, dim3(std::max<uint32_t>(1, (q + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                           s, slot, q, count, back_packed, out_idx, out_cnt, F);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(KAD_ERR_HIP, hipGetErrorString(e));
    return KAD_OK;
}

extern "C" int kad_route_unpack_packed(const uint32_t* slot, uint32_t q, uint32_t count, const uint32_t* back_packed,
                                       uint32_t* out_idx, uint8_t* out_cnt, int device, void* stream) {
    return unpack_packed(slot, q, count, back_packed, out_idx, out_cnt, RouteFold{nullptr, 0, nullptr}, device, stream);
}

extern "C" int kad_route_unpack_packed_fold(const uint32_t* slot, uint32_t q, uint32_t count,
                                            const uint32_t* back_packed, uint32_t* out_idx, uint8_t* out_cnt,
                                            uint32_t* ctr, uint32_t world, uint32_t* flags, int device, void* stream) {
    if (!ctr || !flags) return kadgpu_internal::set_error(KAD_ERR_INVALID, "NULL ctr or flags");
    if (world == 0 || world > KAD_ROUTE_MAX_WORLD) return kadgpu_internal::set_error(KAD_ERR_INVALID, "world must be 1..16");
    return unpack_packed(slot, q, count, back_packed, out_idx, out_cnt, RouteFold{ctr, world, flags}, device, stream);
}
