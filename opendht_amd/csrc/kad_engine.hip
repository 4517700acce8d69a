// kad_engine.hip — MI355X (gfx950) batched Kademlia closest-node engine.
//
// Device kernels for OpenDHT's XOR-distance lookup path and the extern "C" ABI declared in
// include/kadgpu.h. Reference semantics reproduced bit-exactly (paths relative to the
// OpenDHT 1.2.1 tree):
//   InfoHash::xorCmp / cmp / commonBits / lowbit   include/opendht/infohash.h:84-146
//   RoutingTable::findBucket                        src/routing_table.cpp:113-135
//   RoutingTable::findClosestNodes                  src/routing_table.cpp:67-111
//   Node::isGood / isExpired (status snapshot)      src/node.cpp:34-40, include/opendht/node.h:67
//   NodeCache::getCachedNodes                       src/node_cache.cpp:36-66
//
// HBM layout of one table (one address family, one shard), all arrays node- or bucket-major:
//   key[n]      u64  ID bits 0..63 (InfoHash bytes 0..7, big-endian -> native integer)  HOT
//   tail[n][3]  u32  ID bits 64..159 (bytes 8..19)                                      COLD: read only
//                    when two candidates' top-64 XOR distances tie
//   status[n]   u8   bit0 isGood(now), bit1 isExpired()   (NodeCache walk, wide-bucket fallback)
//   dir[B+1]    u32x2 {first node of bucket b (bit31: bucket wider than 32 nodes), good bitmask of
//                      b's nodes}: 8 bytes per bucket, good counts are popcounts
//   gpre[B+1]   u32  good nodes in buckets < b (slow path / deferred queries)
//   dmask[B]    u32  "top 64 ID bits shared with another node" bitmask (only if any node has one)
//   fkey[B], ftail[B][3]   bucket `first` IDs (read only when the radix slot is ambiguous)
//   rrdx[S+1]   u32  #bucket firsts below radix slot s (bit31: bucket starts exactly at slot)
//   nrdx[S'+1]  u32  #node IDs below radix slot s (NodeCache lower_bound; sorted tables only)
//
// A RoutingTable query, one lane per query:
//   1. target -> radix slot -> bucket b = upper_bound(first, t) - 1 (clamped to 0); tables whose
//      buckets are exactly the radix slots (U(d)) map the slot to the bucket with no load
//   2. ONE burst of 2P+3 independent 16-byte directory loads around b; the good prefix sums give
//      the least round R whose window W(R) = [max(0,b-1-R), min(B-1,b+R)] holds >= count good
//      nodes or is the whole table (routing_table.cpp:89-104 closed form)
//   3. W(R)'s keys stream in 16-node chunks of eight 16-byte loads issued back to back (each
//      lane's window lines are fetched once, not once per node); good bits come from the bucket
//      masks; the `count` smallest (XOR distance, index) live in a register-resident sorted list
//      (branch-free insertion chain). The exact 160-bit compare runs only for nodes whose top 64
//      bits are shared with another node of the table (dup mask), so a top-64 tie is impossible
//      on the fast path. Windows beyond the prefetch or with >32-node buckets take a per-node
//      slow path with the same results.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kadgpu.h"

#define KAD_VERSION 100  // 0.1.0

namespace {

thread_local std::string g_err;

int set_err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_TRY(expr)                                                                      \
    do {                                                                                   \
        hipError_t e_ = (expr);                                                            \
        if (e_ != hipSuccess)                                                              \
            return set_err(KAD_ERR_HIP, "%s failed: %s", #expr, hipGetErrorString(e_));    \
    } while (0)

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t RDX_EXACT = 0x80000000u;
constexpr uint32_t RDX_MASK = 0x7FFFFFFFu;
constexpr int BLOCK = 256;

// ---------------------------------------------------------------------------------------
// Device view of a table (passed by value as a kernel argument)
// ---------------------------------------------------------------------------------------
struct DevTable {
    const uint64_t* key;
    const uint32_t* tail;
    const uint8_t* status;
    const uint2* dir;
    const uint32_t* gpre;
    const uint32_t* dmask;
    const uint64_t* fkey;
    const uint32_t* ftail;
    const uint32_t* rrdx;
    const uint32_t* nrdx;
    const uint4* rec;    // bucket records (TF_REC): 4 copies x rec_lines 128-byte lines, see rt_rec_kernel
    uint32_t rec_lines;  // lines per copy
    uint64_t rbase, nbase;
    uint32_t rshift, rslots, nshift, nslots;
    uint32_t n, B, index_base, flags;
};

constexpr uint32_t TF_DIRECT = 1u;   // radix slot s holds exactly bucket s (no locate load)
constexpr uint32_t TF_HAS_DUP = 2u;  // some nodes share their top 64 ID bits
constexpr uint32_t TF_REC = 8u;      // bucket-record layout present (direct-mapped, depth <= 48)
constexpr uint32_t WIDE = 0x80000000u;  // dir[].x flag: bucket holds > 32 nodes (masks invalid)
constexpr uint32_t KEY_PAD = 32;        // key[] is padded so 16-node chunk loads never leave it

struct Target {
    uint64_t hi;       // bits 0..63
    uint32_t t2, t3, t4;
};

__device__ __forceinline__ Target load_target(const uint8_t* targets, uint32_t i) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(targets + 20ull * i);
    Target t;
    uint32_t w0 = __builtin_bswap32(p[0]), w1 = __builtin_bswap32(p[1]);
    t.hi = ((uint64_t)w0 << 32) | w1;
    t.t2 = __builtin_bswap32(p[2]);
    t.t3 = __builtin_bswap32(p[3]);
    t.t4 = __builtin_bswap32(p[4]);
    return t;
}

// 160-bit compare of (hi, a2, a3, a4) vs (hi', b2, b3, b4): returns <0, 0, >0
__device__ __forceinline__ int cmp160(uint64_t ah, uint32_t a2, uint32_t a3, uint32_t a4,
                                      uint64_t bh, uint32_t b2, uint32_t b3, uint32_t b4) {
    if (ah != bh) return ah < bh ? -1 : 1;
    if (a2 != b2) return a2 < b2 ? -1 : 1;
    if (a3 != b3) return a3 < b3 ? -1 : 1;
    if (a4 != b4) return a4 < b4 ? -1 : 1;
    return 0;
}

// RoutingTable::findBucket (routing_table.cpp:113-127) = upper_bound(first, t) - 1, clamped to 0.
__device__ __forceinline__ uint32_t locate_bucket(const DevTable& T, const Target& t) {
    if (T.flags & TF_DIRECT) {
        if (t.hi < T.rbase) return 0;
        const uint64_t s = (t.hi - T.rbase) >> T.rshift;
        return s >= T.B ? T.B - 1 : (uint32_t)s;
    }
    uint32_t ub;
    if (t.hi < T.rbase) {
        ub = 0;
    } else {
        uint64_t s = (t.hi - T.rbase) >> T.rshift;
        if (s >= T.rslots) {
            ub = T.B;
        } else {
            uint32_t r0 = T.rrdx[s], r1 = T.rrdx[s + 1];
            uint32_t lo = r0 & RDX_MASK, hi = r1 & RDX_MASK;
            if (hi - lo == 1 && (r0 & RDX_EXACT)) {
                ub = hi;  // a bucket starts exactly at the slot start <= t
            } else {
                // count firsts <= t among [lo, hi)
                while (lo < hi) {
                    uint32_t mid = (lo + hi) >> 1;
                    const uint32_t* ft = T.ftail + 3ull * mid;
                    int c = cmp160(T.fkey[mid], ft[0], ft[1], ft[2], t.hi, t.t2, t.t3, t.t4);
                    if (c <= 0) lo = mid + 1; else hi = mid;
                }
                ub = lo;
            }
        }
    }
    return ub == 0 ? 0u : ub - 1;
}

// NodeCache lower_bound (node_cache.cpp:39) on a sorted table: #ids < t.
__device__ __forceinline__ uint32_t node_lower_bound(const DevTable& T, const Target& t) {
    if (t.hi < T.nbase) return 0;
    uint64_t s = (t.hi - T.nbase) >> T.nshift;
    if (s >= T.nslots) return T.n;
    uint32_t lo = T.nrdx[s], hi = T.nrdx[s + 1];
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        const uint32_t* tt = T.tail + 3ull * mid;
        int c = cmp160(T.key[mid], tt[0], tt[1], tt[2], t.hi, t.t2, t.t3, t.t4);
        if (c < 0) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// ---------------------------------------------------------------------------------------
// RoutingTable::findClosestNodes, one query per lane (routing_table.cpp:67-111)
// ---------------------------------------------------------------------------------------

// Register-resident sorted list of the K best (XOR distance, index) pairs. Insertion: once the
// candidate lands at slot s every later entry shifts down one slot (`sh`), so displaced entries
// keep their relative order; an empty slot (NONE) sorts after every real node.
template <int K>
struct TopK {
    uint64_t dk[K];
    uint32_t di[K];
    __device__ __forceinline__ void init() {
#pragma unroll
        for (int s = 0; s < K; s++) { dk[s] = ~0ull; di[s] = NONE; }
    }
    // Fast insertion: valid while every list entry has a distinct top-64 distance and the candidate is
    // not the all-ones distance (which an empty slot also holds). The list is sorted, so the
    // compares lt[s] = cd < dk[s] are monotone in s and all K of them are independent: slot s
    // keeps its entry (!lt[s]), takes the candidate (lt[s] && !lt[s-1]) or its predecessor's entry.
    // Dependency depth 3 instead of a serial compare/select chain through K slots.
    __device__ __forceinline__ void insert_fast(uint64_t cd, uint32_t ci) {
        bool lt[K];
#pragma unroll
        for (int s = 0; s < K; s++) lt[s] = cd < dk[s];
#pragma unroll
        for (int s = K - 1; s > 0; s--) {
            const uint64_t nk = lt[s - 1] ? dk[s - 1] : cd;
            const uint32_t ni = lt[s - 1] ? di[s - 1] : ci;
            dk[s] = lt[s] ? nk : dk[s];
            di[s] = lt[s] ? ni : di[s];
        }
        dk[0] = lt[0] ? cd : dk[0];
        di[0] = lt[0] ? ci : di[0];
    }
};

template <int K>
__device__ __forceinline__ void write_row(const TopK<K>& L, const DevTable& T, uint32_t count, uint32_t m,
                                          uint32_t* __restrict__ out_row, uint8_t* out_cnt_p) {
    if (count == (uint32_t)K && (K % 4) == 0) {
#pragma unroll
        for (int s = 0; s < K; s += 4) {
            uint4 v;
            v.x = (uint32_t)s < m ? L.di[s] + T.index_base : NONE;
            v.y = (uint32_t)s + 1 < m ? L.di[s + 1] + T.index_base : NONE;
            v.z = (uint32_t)s + 2 < m ? L.di[s + 2] + T.index_base : NONE;
            v.w = (uint32_t)s + 3 < m ? L.di[s + 3] + T.index_base : NONE;
            *reinterpret_cast<uint4*>(out_row + s) = v;
        }
    } else {
#pragma unroll
        for (int s = 0; s < K; s++)
            if ((uint32_t)s < count) out_row[s] = (uint32_t)s < m ? L.di[s] + T.index_base : NONE;
    }
    if (out_cnt_p) *out_cnt_p = (uint8_t)m;
}

// ---- fast path, phase 1: the window ------------------------------------------------------
// P = directory prefetch radius (2P+3 records around b). The fast path handles windows with
// R <= P, no bucket wider than 32 nodes, at most 64*MW nodes from the 64-byte aligned base, no good
// node whose top 64 bits are shared with another node (a possible top-64 tie) and no good node at
// the all-ones top-64 distance (which empty list slots also hold). Anything else is deferred to
// the exact per-node kernel (rt_query_slow).
template <int K>
struct Window {
    static constexpr int MW = K > 16 ? 2 : 1;
    uint32_t base, ne, good;  // 64-byte aligned first node, one past the last node, good nodes in W(R)
    uint64_t gm[MW];          // good bitmap of nodes base .. base + 64*MW
    __device__ __forceinline__ uint32_t chunks() const { return (ne - base + 7) >> 3; }
};

enum { WIN_READY = 1, WIN_DEFER = 2 };

// rec[i] = dir[clamp(b - P - 1 + i, 0, B)]: rec[P - r] = dir[lo_r] and rec[P + r + 2] = dir[hi_r + 1]
// for round r (the clamp IS the window's edge clamp).
template <int P>
__device__ __forceinline__ void load_recs(const DevTable& T, uint32_t b, uint2 (&rec)[2 * P + 3]) {
#pragma unroll
    for (int i = 0; i < 2 * P + 3; i++) {
        const int64_t w = (int64_t)b - (P + 1) + i;
        rec[i] = T.dir[w < 0 ? 0 : (w > (int64_t)T.B ? T.B : (uint32_t)w)];
    }
}

template <int K, int P>
__device__ __forceinline__ int rt_window(const DevTable& T, uint32_t b, const uint2 (&rec)[2 * P + 3],
                                         uint32_t count, Window<K>& W) {
    constexpr int NR = 2 * P + 3;
    constexpr int MW = Window<K>::MW;
    const uint32_t B = T.B;
    uint32_t g[NR];
#pragma unroll
    for (int i = 0; i < NR; i++) {  // good count of bucket b-P-1+i (0 outside the table)
        const int64_t w = (int64_t)b - (P + 1) + i;
        g[i] = (w >= 0 && w < (int64_t)B) ? (uint32_t)__builtin_popcount(rec[i].y) : 0u;
    }
    // rounds: W(r) = buckets b-1-r .. b+r = rec indices P-r .. P+r+1
    int R = -1;
    uint32_t good = g[P] + g[P + 1];
#pragma unroll
    for (int r = 0; r <= P; r++) {
        if (r > 0) good += (R < 0) ? g[P - r] + g[P + r + 1] : 0u;
        const bool whole = (b <= (uint32_t)r + 1) & (b + r >= B - 1);
        if (R < 0 && (good >= count || whole)) R = r;
    }
    if (R < 0) return WIN_DEFER;
    uint32_t nb = 0, ne = 0, wide = 0;
#pragma unroll
    for (int r = 0; r <= P; r++)
        if (r == R) { nb = rec[P - r].x; ne = rec[P + r + 2].x; }
#pragma unroll
    for (int i = 0; i < NR - 1; i++) wide |= (i >= P - R && i <= P + R + 1) ? rec[i].x : 0u;
    nb &= ~WIDE;
    ne &= ~WIDE;
    const uint32_t base = nb & ~7u;
    if ((wide & WIDE) || ne - base > 64u * MW) return WIN_DEFER;
#pragma unroll
    for (int w = 0; w < MW; w++) W.gm[w] = 0;
#pragma unroll
    for (int i = 0; i < NR - 1; i++) {
        const bool in = (i >= P - R) & (i <= P + R + 1);
        const uint32_t rel = (rec[i].x & ~WIDE) - base;  // window buckets start at or after base
#pragma unroll
        for (int w = 0; w < MW; w++) {
            const uint64_t z = rec[i].y;
            const uint64_t c = rel >= 64u * w ? (rel - 64u * w < 64u ? z << (rel - 64u * w) : 0ull)
                                              : (64u * w - rel < 32u ? z >> (64u * w - rel) : 0ull);
            W.gm[w] |= in ? c : 0ull;
        }
    }
    if (T.flags & TF_HAS_DUP) {
        uint32_t dup = 0;
#pragma unroll
        for (int i = 0; i < NR - 1; i++) {
            const int64_t w = (int64_t)b - (P + 1) + i;
            const bool in = (i >= P - R) & (i <= P + R + 1) & (w >= 0) & (w < (int64_t)B);
            dup |= in ? (T.dmask[in ? (uint32_t)w : 0u] & rec[i].y) : 0u;
        }
        if (dup) return WIN_DEFER;
    }
    W.base = base;
    W.ne = ne;
    W.good = good;
    return WIN_READY;
}

// ---- fast path, phase 2: rank one 8-node (64-byte) chunk of keys --------------------------
template <int K>
__device__ __forceinline__ void rank_chunk(TopK<K>& L, const uint4 (&kv)[4], uint64_t th, uint32_t g8,
                                           uint32_t j0, bool& ones) {
#pragma unroll
    for (int x = 0; x < 4; x++) {
        const uint64_t d0 = (((uint64_t)kv[x].y << 32) | kv[x].x) ^ th;
        const uint64_t d1 = (((uint64_t)kv[x].w << 32) | kv[x].z) ^ th;
        if ((g8 >> (2 * x)) & 1u) { ones |= d0 == ~0ull; L.insert_fast(d0, j0 + 2 * x); }
        if ((g8 >> (2 * x + 1)) & 1u) { ones |= d1 == ~0ull; L.insert_fast(d1, j0 + 2 * x + 1); }
    }
}

template <int K>
__device__ __forceinline__ uint32_t chunk_bits(const Window<K>& W, uint32_t c /* node offset, multiple of 8 */) {
    constexpr int MW = Window<K>::MW;
    return (uint32_t)((MW == 1 || c < 64 ? W.gm[0] : W.gm[MW - 1]) >> (c & 63)) & 0xFFu;
}

// Lane-per-query fast path with per-lane loads (the K=32 kernel, and the dual-family kernel).
// Returns false (nothing written) when the query must be deferred.
template <int K, int P>
__device__ __forceinline__ bool rt_query_fast(const DevTable& T, const Target& t, uint32_t count,
                                              uint32_t* __restrict__ out_row, uint8_t* out_cnt_p) {
    if (T.B == 0 || count == 0) {
        for (uint32_t s = 0; s < count; s++) out_row[s] = NONE;
        if (out_cnt_p) *out_cnt_p = 0;
        return true;
    }
    const uint32_t b = locate_bucket(T, t);
    uint2 rec[2 * P + 3];
    load_recs<P>(T, b, rec);
    Window<K> W;
    if (rt_window<K, P>(T, b, rec, count, W) != WIN_READY) return false;
    TopK<K> L;
    L.init();
    bool ones = false;
    // key chunks double-buffered two deep: chunks c and c+1 are in flight together, chunk c+2 is
    // issued as soon as chunk c has been ranked
    const uint4* kp = reinterpret_cast<const uint4*>(T.key + W.base);
    const uint32_t M = W.chunks();
    uint4 ba[4], bb[4];
#pragma unroll
    for (int x = 0; x < 4; x++) ba[x] = kp[x];
    if (M > 1) {
#pragma unroll
        for (int x = 0; x < 4; x++) bb[x] = kp[4 + x];
    }
    for (uint32_t c = 0; c < M; c += 2) {
        rank_chunk<K>(L, ba, t.hi, chunk_bits<K>(W, 8 * c), W.base + 8 * c, ones);
        if (c + 2 < M) {
#pragma unroll
            for (int x = 0; x < 4; x++) ba[x] = kp[4 * (c + 2) + x];
        }
        if (c + 1 < M) {
            rank_chunk<K>(L, bb, t.hi, chunk_bits<K>(W, 8 * (c + 1)), W.base + 8 * (c + 1), ones);
            if (c + 3 < M) {
#pragma unroll
                for (int x = 0; x < 4; x++) bb[x] = kp[4 * (c + 3) + x];
            }
        }
    }
    if (ones) return false;
    write_row<K>(L, T, count, min(W.good, count), out_row, out_cnt_p);
    return true;
}

// ---------------------------------------------------------------------------------------
// Wave-cooperative exact query: the fallback of every RoutingTable kernel for the few queries
// its fast path cannot rank (windows beyond its prefetch, wide buckets, records with equal short
// keys, top-64 ties). The whole wave answers ONE query with the reference's exact order:
//   1. W(R): lane l tests round r0 + l from the good prefix sums; a ballot gives the least R
//      (routing_table.cpp:89-104 closed form), 64 rounds per probe
//   2. W(R)'s nodes in tiles of 64 (lane l <- node beg + 64u + l): good bit, full 160-bit XOR
//      distance to the target, node index
//   3. in a window of <= 64 nodes (nearly every case) each lane ranks its node against the good
//      nodes of the window, read back from LDS by wave-uniform (broadcast) reads;
//      a larger one is ranked tile by tile: each lane ranks its tile node and its list entry
//      against (list U tile) by broadcasting the candidates (readlane), and entries of rank
//      < count form the new sorted list in lanes 0..count-1.
//      Order = (160-bit distance, node index): equal IDs only meet inside one bucket, where index
//      order is the reference's insertion order (routing_table.cpp:75-87).
// Must be called from wave-uniform control flow with all 64 lanes active; `t` is wave-uniform.
// Latency ~ three dependent memory phases + ~1k VALU: the calling wave's other lanes have
// already written their rows, and other waves hide it.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) { return __builtin_amdgcn_readlane(v, l); }
__device__ __forceinline__ uint64_t rdl64(uint64_t v, uint32_t l) {
    return ((uint64_t)rdl((uint32_t)(v >> 32), l) << 32) | rdl((uint32_t)v, l);
}
__device__ __forceinline__ uint64_t shfl_xor64(uint64_t v, uint32_t h) {
    return ((uint64_t)(uint32_t)__shfl_xor((int)(v >> 32), (int)h, 64) << 32) | (uint32_t)__shfl_xor((int)(uint32_t)v, (int)h, 64);
}
// (a0, a1, a2) < (b0, b1, b2) lexicographically
__device__ __forceinline__ bool lt3(uint64_t a0, uint64_t a1, uint64_t a2, uint64_t b0, uint64_t b1, uint64_t b2) {
    return a0 < b0 || (a0 == b0 && (a1 < b1 || (a1 == b1 && a2 < b2)));
}

// stamp point (diagnostics): lane 0 records s_memrealtime after waiting for its memory ops
#define XSTAMP(k)                                                               \
    do {                                                                        \
        if (sp && lane == 0) {                                                  \
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");         \
            sp[k] = __builtin_amdgcn_s_memrealtime();                           \
        }                                                                       \
    } while (0)

__device__ void wave_exact(const DevTable& T, const Target& t, uint32_t count, uint32_t* row, uint8_t* cp,
                           uint64_t* xs /* this wave's 64 x 3 LDS words */, uint64_t* sp = nullptr) {
    const uint32_t lane = threadIdx.x & 63u, B = T.B;
    XSTAMP(0);
    if (B == 0 || count == 0) {
        if (lane < count) row[lane] = NONE;
        if (lane == 0 && cp) *cp = 0;
        return;
    }
    const uint32_t b = locate_bucket(T, t);
    uint32_t beg = 0, end = 0, good = 0;
    for (uint32_t r0 = 0;; r0 += 64) {  // the window's good count and node range for rounds r0..r0+63
        const uint32_t r = r0 + lane;
        const uint32_t l_ = b > r ? b - 1 - r : 0u;
        const uint32_t h_ = (uint64_t)b + r >= (uint64_t)B - 1 ? B - 1 : b + r;
        const uint32_t g_ = T.gpre[h_ + 1] - T.gpre[l_];
        const uint32_t b_ = T.dir[l_].x & ~WIDE, e_ = T.dir[h_ + 1].x & ~WIDE;
        const uint64_t ok = __ballot(g_ >= count || (l_ == 0 && h_ == B - 1));
        if (ok) {
            const uint32_t R = (uint32_t)__builtin_ctzll(ok);
            beg = rdl(b_, R);
            end = rdl(e_, R);
            good = rdl(g_, R);
            break;
        }
    }
    XSTAMP(1);
    const uint32_t m = min(count, good);
    XSTAMP(2);
    if (end - beg <= 64) {  // one tile (nearly every case): rank by broadcast LDS reads
        const uint32_t j = beg + lane;
        uint64_t V0 = ~0ull, V1 = ~0ull, V2 = ~0ull;
        bool v = false;
        if (j < end) {  // independent loads, one phase
            const uint8_t st = T.status[j];
            const uint64_t k = T.key[j];
            const uint32_t* tl = T.tail + 3ull * j;
            const uint32_t a2 = tl[0], a3 = tl[1], a4 = tl[2];
            v = st & KAD_STATUS_GOOD;
            if (v) {
                V0 = k ^ t.hi;
                V1 = ((uint64_t)(a2 ^ t.t2) << 32) | (a3 ^ t.t3);
                V2 = ((uint64_t)(a4 ^ t.t4) << 32) | j;
            }
        }
        xs[3 * lane] = V0;
        xs[3 * lane + 1] = V1;
        xs[3 * lane + 2] = V2;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        XSTAMP(3);
        // rank on the top 64 distance bits (unique unless two nodes share them); ties -> full order
        uint32_t lt = 0, le = 0;
#pragma unroll 16
        for (uint32_t sl = 0; sl < 64; sl++) {
            const uint64_t S0 = xs[3 * sl];  // wave-uniform address: broadcast read
            lt += S0 < V0;
            le += S0 <= V0;
        }
        uint32_t rank = lt;
        if (__ballot(v && le - lt > 1)) {
            rank = 0;
            for (uint64_t mm = __ballot(v); mm; mm &= mm - 1) {
                const uint32_t sl = (uint32_t)__builtin_ctzll(mm);
                rank += lt3(xs[3 * sl], xs[3 * sl + 1], xs[3 * sl + 2], V0, V1, V2);
            }
        }
        XSTAMP(4);
        __builtin_amdgcn_wave_barrier();  // xs is reused by the wave's next query
        if (v && rank < count) row[rank] = j + T.index_base;
        if (lane >= m && lane < count) row[lane] = NONE;
        if (lane == 0 && cp) *cp = (uint8_t)m;
        return;
    }
    uint64_t L0 = ~0ull, L1 = ~0ull, L2 = ~0ull;  // list entry of this lane (lanes < nl)
    uint32_t nl = 0;
    for (uint32_t base = beg; base < end; base += 64) {
        const uint32_t j = base + lane;
        bool cv = false;
        uint64_t C0 = 0, C1 = 0, C2 = 0;  // (dist bits 0..63, dist bits 64..127, dist bits 128..159 : index)
        if (j < end) {
            cv = T.status[j] & KAD_STATUS_GOOD;
            const uint32_t* tl = T.tail + 3ull * j;
            C0 = T.key[j] ^ t.hi;
            C1 = ((uint64_t)(tl[0] ^ t.t2) << 32) | (tl[1] ^ t.t3);
            C2 = ((uint64_t)(tl[2] ^ t.t4) << 32) | j;
        }
        const bool lv = lane < nl;
        const uint64_t cm = __ballot(cv);
        uint32_t rL = 0, rC = 0;
        for (uint64_t mm = cm; mm; mm &= mm - 1) {
            const uint32_t sl = (uint32_t)__builtin_ctzll(mm);
            const uint64_t S0 = rdl64(C0, sl), S1 = rdl64(C1, sl), S2 = rdl64(C2, sl);
            rL += lt3(S0, S1, S2, L0, L1, L2);
            rC += lt3(S0, S1, S2, C0, C1, C2);
        }
        for (uint32_t e = 0; e < nl; e++) {
            const uint64_t S0 = rdl64(L0, e), S1 = rdl64(L1, e), S2 = rdl64(L2, e);
            rL += lt3(S0, S1, S2, L0, L1, L2);
            rC += lt3(S0, S1, S2, C0, C1, C2);
        }
        const uint32_t nn = min(nl + (uint32_t)__builtin_popcountll(cm), count);
        uint64_t N0 = ~0ull, N1 = ~0ull, N2 = ~0ull;
        for (uint32_t r = 0; r < nn; r++) {
            const uint64_t mL = __ballot(lv && rL == r), mC = __ballot(cv && rC == r);
            uint64_t S0, S1, S2;
            if (mL) {
                const uint32_t sl = (uint32_t)__builtin_ctzll(mL);
                S0 = rdl64(L0, sl); S1 = rdl64(L1, sl); S2 = rdl64(L2, sl);
            } else {
                const uint32_t sl = (uint32_t)__builtin_ctzll(mC);
                S0 = rdl64(C0, sl); S1 = rdl64(C1, sl); S2 = rdl64(C2, sl);
            }
            if (lane == r) { N0 = S0; N1 = S1; N2 = S2; }
        }
        L0 = N0; L1 = N1; L2 = N2;
        nl = nn;
    }
    if (lane < count) row[lane] = lane < m ? (uint32_t)L2 + T.index_base : NONE;
    if (lane == 0 && cp) *cp = (uint8_t)m;
}

// The exact path for every lane of the wave whose fast path gave up (`ex`), one query at a time.
// `pick` maps a lane's flag to the table it queries (dual-family kernel) - here a single table.
__device__ __forceinline__ void exact_tail(const DevTable& T, const Target& t, bool ex, uint32_t i, uint32_t count,
                                           uint32_t* out_idx, uint8_t* out_cnt, uint64_t* xs) {
    for (uint64_t m = __ballot(ex); m; m &= m - 1) {
        const uint32_t l = (uint32_t)__builtin_ctzll(m);
        Target u;
        u.hi = rdl64(t.hi, l);
        u.t2 = rdl(t.t2, l);
        u.t3 = rdl(t.t3, l);
        u.t4 = rdl(t.t4, l);
        const uint32_t il = rdl(i, l);
        wave_exact(T, u, count, out_idx + (size_t)il * count, out_cnt ? out_cnt + il : nullptr, xs);
    }
}

// Exact-path queue of the record kernel: the kernel appends the queries its fast path cannot rank
// (wave-aggregated atomic add), and rt_exact_list_kernel, launched right after on the same stream,
// answers each with one wave (wave_exact) and resets the counter. Inline wave_exact cost the
// record kernel ~18 us per 1M queries (0.3% of lanes stall 19% of the waves); the queue turns it
// into one short launch. Scratch is per (table, stream): see kad_table::exact_scratch.
struct ExactQ {
    uint32_t* ctr;   // [0] entries appended, [1] blocks of the list kernel done
    uint32_t* list;  // 32-byte entries: query index, target (hi64, t2, t3, t4)
    uint32_t cap;
};

__device__ __forceinline__ void exact_enqueue(const ExactQ& Q, const DevTable& T, const Target& t, bool ex, uint32_t i,
                                              uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, uint64_t* xs) {
    const uint64_t m = __ballot(ex);
    if (!m) return;
    if (Q.cap == 0) {  // no queue: answer inline
        exact_tail(T, t, ex, i, count, out_idx, out_cnt, xs);
        return;
    }
    const uint32_t lane = threadIdx.x & 63u, first = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == first) base = atomicAdd(Q.ctr, (uint32_t)__builtin_popcountll(m));
    base = rdl(base, first);
    const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    const bool over = ex && pos >= Q.cap;
    if (ex && !over) {  // entry = query index + its target (the list kernel needs no second load)
        uint4* e = reinterpret_cast<uint4*>(Q.list) + 2ull * pos;
        e[0] = make_uint4(i, (uint32_t)t.hi, (uint32_t)(t.hi >> 32), t.t2);
        e[1] = make_uint4(t.t3, t.t4, 0u, 0u);
    }
    exact_tail(T, t, over, i, count, out_idx, out_cnt, xs);  // queue full: answer inline
}

// Diagnostics (KAD_EXACT_STAMPS=1, tools/exact_stamps.py): per wave s_memrealtime at entry, after the
// counter read, after its first item and at exit (100 MHz ticks), for waves < STAMP_WAVES.
constexpr uint32_t STAMP_WAVES = 4096;
__device__ uint64_t g_stamps[STAMP_WAVES * 12];

template <bool ST>
__global__ __launch_bounds__(BLOCK) void rt_exact_list_kernel(DevTable T, ExactQ Q, const uint8_t* __restrict__ targets,
                                                              uint32_t count, uint32_t* __restrict__ out_idx,
                                                              uint8_t* __restrict__ out_cnt) {
    const uint32_t w = (blockIdx.x * BLOCK + threadIdx.x) >> 6, nw = gridDim.x * (BLOCK / 64);
    const bool st = ST && w < STAMP_WAVES && (threadIdx.x & 63) == 0;
    if (st) g_stamps[4 * w] = __builtin_amdgcn_s_memrealtime();
    const uint32_t n = min(__hip_atomic_load(Q.ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), Q.cap);
    if (st) g_stamps[4 * w + 1] = __builtin_amdgcn_s_memrealtime() | ((uint64_t)(w < n) << 63);
    __shared__ uint64_t xs[BLOCK / 64][192];
    uint4 e0 = make_uint4(0, 0, 0, 0), e1 = e0;
    if (w < Q.cap) {  // the wave's first entry, loaded together with the counter
        const uint4* e = reinterpret_cast<const uint4*>(Q.list) + 2ull * w;
        e0 = e[0];
        e1 = e[1];
    }
    for (uint32_t k = w; k < n; k += nw) {
        if (k != w) {
            const uint4* e = reinterpret_cast<const uint4*>(Q.list) + 2ull * k;
            e0 = e[0];
            e1 = e[1];
        }
        Target t;
        t.hi = ((uint64_t)e0.z << 32) | e0.y;
        t.t2 = e0.w;
        t.t3 = e1.x;
        t.t4 = e1.y;
        const uint32_t i = e0.x;
        wave_exact(T, t, count, out_idx + (size_t)i * count, out_cnt ? out_cnt + i : nullptr, xs[threadIdx.x >> 6],
                   (ST && k == w && w < STAMP_WAVES) ? g_stamps + STAMP_WAVES * 4 + 8 * w : nullptr);
        if (st && k == w) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            g_stamps[4 * w + 2] = __builtin_amdgcn_s_memrealtime();
        }
    }
    if (st) g_stamps[4 * w + 3] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();
    if (threadIdx.x == 0 && atomicAdd(Q.ctr + 1, 1u) == gridDim.x - 1) {  // every block has read ctr[0]
        atomicExch(Q.ctr, 0u);
        atomicExch(Q.ctr + 1, 0u);
    }
}
constexpr uint32_t EXACT_LIST_BLOCKS = 1024;  // 4096 waves: one wave_exact latency for <= 4096 entries

// Lane-per-query RoutingTable kernel (any table shape, count <= 32).
template <int K>
__global__ __launch_bounds__(BLOCK) void rt_closest_kernel(DevTable T, const uint8_t* __restrict__ targets,
                                                           uint32_t q, uint32_t count,
                                                           uint32_t* __restrict__ out_idx,
                                                           uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool ex = false;
    Target t{};
    if (i < q) {
        t = load_target(targets, i);
        ex = !rt_query_fast<K, (K > 16 ? 6 : 3)>(T, t, count, out_idx + (size_t)i * count, out_cnt ? out_cnt + i : nullptr);
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, ex, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}

// ---------------------------------------------------------------------------------------
// Bucket-record RoutingTable kernel (count <= 8; direct-mapped tables of uniform depth d <= 48,
// the U(d) shape of the bench shards). The default kernel where the table supports it.
//
// A random gather on MI355X costs one 128-byte line whether 32 or 128 bytes of it are used, and
// wherever the table sits (tools/mb_line.py: ~34 G lines/s with the target read and row write,
// the same for 128 MB and 1 GB tables), so a query should touch exactly ONE line. Each bucket is
// a 32-byte record:
//   dword 0    first node index (27 bits) | good count G (4 bits) << 27 | defer flag << 31
//   halfword 2 good bitmask of the bucket's nodes (slot s = node first + s; at most 16 nodes)
//   halfwords 3..15  key16 of the bucket's good nodes in slot order (at most 13): ID bits [d, d+16)
// The defer flag marks a record the kernel cannot rank exactly (more than 16 nodes, more than 13
// good nodes, or two good nodes with equal key16); a query whose window holds one takes the
// wave-cooperative exact path (wave_exact).
//
// Layout: record r = bucket + 2 (two empty records precede bucket 0, empty records pad the end).
// The records are stored in FOUR copies, copy c cut into aligned 128-byte lines that start at
// records r = c (mod 4): line k of copy c holds records 4k+c .. 4k+c+3. Bucket b's rounds 0 and 1,
// buckets b-2 .. b+1 = records b .. b+3, are then line b/4 of copy b%4: one aligned line, always.
// (4 x 32 B per bucket: 268 MB for a 2^21-bucket shard; table size does not change the gather
// rate.) Windows needing round 2 (~0.14% at k = 8 on an 80%-good uniform shard) take wave_exact.
//
// Ranking. Buckets of equal depth are dyadic: the XOR images of two of them are disjoint
// intervals ordered by D = prefix(bucket) XOR prefix(b), and inside one bucket the order is that
// of key16 XOR the target's bits [d, d+16) (exact: two good nodes of a record never share key16).
// So a node's rank value is the 32-bit word (ord(D) << 23 | record << 20 | key16^t16 << 4 | g),
// g = its index among the record's good nodes. Each record's up-to-13 values go through a
// 45-comparator min/max network that leaves its 8 smallest sorted; the per-record lists are merged
// by bitonic 8+8 merges (min/max only: 2 VALU ops per compare-exchange). The output slot of
// value (record, g) is the g-th set bit of the record's good mask.
// Reference semantics: routing_table.cpp:67-111 (window rounds, sorted insertion, truncation).
// ---------------------------------------------------------------------------------------
constexpr uint32_t REC_FIRST_MASK = (1u << 27) - 1;
constexpr uint32_t REC_MAXG = 13;
constexpr uint32_t REC_PAD = 2;
constexpr uint32_t REC_NONE = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t rec_half(const uint4& lo, const uint4& hi, int h) {
    const int w = h >> 1;  // static after unrolling
    const uint32_t d = w == 0 ? lo.x : w == 1 ? lo.y : w == 2 ? lo.z : w == 3 ? lo.w
                     : w == 4 ? hi.x : w == 5 ? hi.y : w == 6 ? hi.z : hi.w;
    return (h & 1) ? d >> 16 : d & 0xFFFFu;
}

__device__ __forceinline__ void cx(uint32_t& a, uint32_t& b) {
    const uint32_t lo = min(a, b);
    b = max(a, b);
    a = lo;
}

// Batcher's 16-input odd-even merge sort restricted to 13 inputs and pruned to the 8 smallest
// outputs (tools/netgen.py; checked exhaustively by the 0-1 principle in tests/test_networks.py).
constexpr int NET13_TOP8_LEN = 45;
__device__ constexpr uint8_t NET13_TOP8[NET13_TOP8_LEN][2] = {
    {0, 1}, {2, 3}, {4, 5}, {6, 7}, {8, 9}, {10, 11}, {0, 2}, {1, 3}, {4, 6}, {5, 7}, {8, 10}, {9, 11},
    {1, 2}, {5, 6}, {9, 10}, {0, 4}, {1, 5}, {2, 6}, {3, 7}, {8, 12}, {2, 4}, {3, 5}, {10, 12}, {1, 2},
    {3, 4}, {5, 6}, {9, 10}, {11, 12}, {0, 8}, {1, 9}, {2, 10}, {3, 11}, {4, 12}, {4, 8}, {5, 9}, {6, 10},
    {7, 11}, {2, 4}, {3, 5}, {6, 8}, {7, 9}, {1, 2}, {3, 4}, {5, 6}, {7, 8}};

// a = the 8 smallest of (a, s), sorted; a and s sorted ascending on entry.
__device__ __forceinline__ void merge8(uint32_t (&a)[8], const uint32_t (&s)[8]) {
#pragma unroll
    for (int i = 0; i < 8; i++) a[i] = min(a[i], s[7 - i]);  // bitonic
#pragma unroll
    for (int i = 0; i < 4; i++) cx(a[i], a[i + 4]);
#pragma unroll
    for (int i = 0; i < 8; i++)
        if ((i & 2) == 0) cx(a[i], a[i + 2]);
#pragma unroll
    for (int i = 0; i < 8; i += 2) cx(a[i], a[i + 1]);
}

// The 8 smallest rank values of one record (NONE-padded), sorted.
__device__ __forceinline__ void rec_rank(const uint4& lo, const uint4& hi, bool inw, uint32_t tag, uint32_t t16,
                                         uint32_t (&s)[8]) {
    const uint32_t G = inw ? (lo.x >> 27) & 15u : 0u;
    uint32_t v[REC_MAXG];
#pragma unroll
    for (int e = 0; e < (int)REC_MAXG; e++)
        v[e] = (uint32_t)e < G ? (tag | ((rec_half(lo, hi, 3 + e) ^ t16) << 4) | (uint32_t)e) : REC_NONE;
#pragma unroll
    for (int c = 0; c < NET13_TOP8_LEN; c++) cx(v[NET13_TOP8[c][0]], v[NET13_TOP8[c][1]]);
#pragma unroll
    for (int j = 0; j < 8; j++) s[j] = v[j];
}

// Index of the g-th set bit of a 16-bit mask (g < popcount(mask)).
__device__ __forceinline__ uint32_t select_bit16(uint32_t m, uint32_t g) {
    uint32_t s = 0, c;
    c = __builtin_popcount(m & 0xFFu);
    if (g >= c) { g -= c; m >>= 8; s = 8; }
    c = __builtin_popcount(m & 0xFu);
    if (g >= c) { g -= c; m >>= 4; s += 4; }
    c = __builtin_popcount(m & 0x3u);
    if (g >= c) { g -= c; m >>= 2; s += 2; }
    return s + (g >= (m & 1u) ? 1u : 0u);
}

// ABL (timing ablations only, KAD_RT_KERNEL=rec_abl1|rec_abl2, results wrong): 1 = no exact
// path, 2 = also no ranking networks.
template <int K, int ABL>
__global__ __launch_bounds__(BLOCK) void rt_rec_kernel(DevTable T, ExactQ Q, const uint8_t* __restrict__ targets,
                                                       uint32_t q, uint32_t count, uint32_t* __restrict__ out_idx,
                                                       uint8_t* __restrict__ out_cnt) {
    static_assert(K == 8, "record kernel: count <= 8");
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool ex = false;
    Target t{};
    if (i < q && count == 0) {
        if (out_cnt) out_cnt[i] = 0;
    } else if (i < q) {
        uint32_t* row = out_idx + (size_t)i * count;
        t = load_target(targets, i);
        const uint32_t B = T.B, d = 64 - T.rshift;
        const uint32_t b = locate_bucket(T, t);
        const uint32_t t16 = (uint32_t)((t.hi << d) >> 48);
        const uint4* L = T.rec + 8ull * ((size_t)(b & 3u) * T.rec_lines + (b >> 2));  // records b-2 .. b+1
        uint4 v[8];
#pragma unroll
        for (int x = 0; x < 8; x++) v[x] = L[x];
        const uint32_t G0 = (v[0].x >> 27) & 15u, G1 = (v[2].x >> 27) & 15u, G2 = (v[4].x >> 27) & 15u,
                       G3 = (v[6].x >> 27) & 15u;
        const uint32_t good0 = G1 + G2;  // {b-1, b}
        const bool r0 = good0 >= count || ((b <= 1) & (b + 1 >= B));
        const uint32_t good1 = good0 + G0 + G3;  // + {b-2, b+1}
        const bool r1 = !r0 && (good1 >= count || ((b <= 2) & (b + 2 >= B)));
        ex = !(r0 | r1) | (v[2].x >> 31) | (v[4].x >> 31) | (r1 & ((v[0].x | v[6].x) >> 31));
        if (!ex) {
            // bucket order by D = prefix XOR the target's top d bits (b is first unless the target
            // lies outside the table's range and was clamped to bucket 0 or B-1)
            const uint64_t pb = (T.rbase >> T.rshift) + b, tp = t.hi >> T.rshift;
            const uint64_t dm2 = (pb - 2) ^ tp, dm1 = (pb - 1) ^ tp, d00 = pb ^ tp, dp1 = (pb + 1) ^ tp;
            const uint32_t om2 = (dm1 < dm2) + (d00 < dm2) + (dp1 < dm2), om1 = (dm2 < dm1) + (d00 < dm1) + (dp1 < dm1),
                           o00 = (dm2 < d00) + (dm1 < d00) + (dp1 < d00), op1 = (dm2 < dp1) + (dm1 < dp1) + (d00 < dp1);
            uint32_t acc[8], s[8];
            if (ABL >= 2) {
#pragma unroll
                for (int j = 0; j < 8; j++) acc[j] = (v[j].z ^ om1 ^ t16) & 0x7FFFFFu;
            } else {
                rec_rank(v[2], v[3], true, (om1 << 23) | (1u << 20), t16, acc);  // b-1
                rec_rank(v[4], v[5], true, (o00 << 23) | (2u << 20), t16, s);    // b
                merge8(acc, s);
                if (__any(r1)) {
                    rec_rank(v[0], v[1], r1, (om2 << 23) | (0u << 20), t16, s);  // b-2
                    merge8(acc, s);
                    rec_rank(v[6], v[7], r1, (op1 << 23) | (3u << 20), t16, s);  // b+1
                    merge8(acc, s);
                }
            }
            const uint32_t m = min(r0 ? good0 : good1, count);
            uint32_t o[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const uint32_t pv = acc[j], p = (pv >> 20) & 3u;
                const uint32_t h = p == 0 ? v[0].x : p == 1 ? v[2].x : p == 2 ? v[4].x : v[6].x;
                const uint32_t mk = (p == 0 ? v[0].y : p == 1 ? v[2].y : p == 2 ? v[4].y : v[6].y) & 0xFFFFu;
                o[j] = (uint32_t)j < m ? (h & REC_FIRST_MASK) + select_bit16(mk, pv & 15u) + T.index_base : NONE;
            }
            if (count == 8) {
                reinterpret_cast<uint4*>(row)[0] = make_uint4(o[0], o[1], o[2], o[3]);
                reinterpret_cast<uint4*>(row)[1] = make_uint4(o[4], o[5], o[6], o[7]);
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if ((uint32_t)j < count) row[j] = o[j];
            }
            if (out_cnt) out_cnt[i] = (uint8_t)m;
        }
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    if (ABL == 0) exact_enqueue(Q, T, t, ex, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}

// Bucket records after a status change (or at table creation): one thread per bucket.
__global__ void rec_build_kernel(const uint64_t* key, const uint8_t* status, const uint2* dir, uint32_t B, uint32_t d,
                                 uint4* rec, uint32_t rec_lines) {
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    if (b >= B) return;
    const uint32_t j0 = dir[b].x & ~WIDE, j1 = dir[b + 1].x & ~WIDE, n = j1 - j0;
    uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint32_t G = 0, mask = 0;
    bool flag = n > 16;
    for (uint32_t j = j0; j < j1; j++) {
        if (!(status[j] & KAD_STATUS_GOOD)) continue;
        if (j - j0 < 16) mask |= 1u << (j - j0);
        const uint32_t k16 = (uint32_t)((key[j] << d) >> 48);
        if (G < REC_MAXG) {
            const uint32_t h = 3 + G;
            w[h >> 1] |= k16 << (16 * (h & 1));
            for (uint32_t a = 0; a < G; a++) {  // equal key16 among good nodes: not rankable here
                const uint32_t ha = 3 + a;
                flag |= ((w[ha >> 1] >> (16 * (ha & 1))) & 0xFFFFu) == k16;
            }
        }
        G++;
    }
    flag |= G > REC_MAXG;
    w[0] = (j0 & REC_FIRST_MASK) | (min(G, 15u) << 27) | ((flag ? 1u : 0u) << 31);
    w[1] |= flag ? 0u : mask;
    const uint4 lo = make_uint4(w[0], w[1], w[2], w[3]), hi = make_uint4(w[4], w[5], w[6], w[7]);
    const uint32_t r = b + REC_PAD;
#pragma unroll
    for (uint32_t c = 0; c < 4; c++) {  // copy c: line (r - c) / 4, slot (r - c) % 4
        if (r < c) continue;
        uint4* dst = rec + 8ull * ((size_t)c * rec_lines + ((r - c) >> 2)) + 2u * ((r - c) & 3u);
        dst[0] = lo;
        dst[1] = hi;
    }
}

template <int K>
__global__ __launch_bounds__(BLOCK) void rt_closest_dual_kernel(DevTable T4, DevTable T6,
                                                                const uint8_t* __restrict__ targets,
                                                                const uint8_t* __restrict__ af, uint32_t q,
                                                                uint32_t count, uint32_t* __restrict__ out_idx,
                                                                uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    bool ex = false, six = false;
    Target t{};
    if (i < q) {
        t = load_target(targets, i);
        six = af[i] != 0;
        ex = !rt_query_fast<K, (K > 16 ? 6 : 3)>(six ? T6 : T4, t, count, out_idx + (size_t)i * count,
                                                  out_cnt ? out_cnt + i : nullptr);
    }
    // exact path per family (each call is wave-uniform in its table)
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T4, t, ex && !six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    exact_tail(T6, t, ex && six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}

__global__ __launch_bounds__(BLOCK) void find_bucket_kernel(DevTable T, const uint8_t* __restrict__ targets,
                                                            uint32_t q, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    out[i] = T.B == 0 ? NONE : locate_bucket(T, load_target(targets, i));
}

// ---------------------------------------------------------------------------------------
// NodeCache::getCachedNodes, one query per lane (node_cache.cpp:36-66): two-pointer walk
// outward from lower_bound(t); p-side taken when xorCmp(p, n) < 0; taking node 0 exhausts
// the p side; expired nodes are walked over but not emitted.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(BLOCK) void nc_closest_kernel(DevTable T, const uint8_t* __restrict__ targets,
                                                           uint32_t q, uint32_t count,
                                                           uint32_t* __restrict__ out_idx,
                                                           uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    const Target t = load_target(targets, i);
    uint32_t* row = out_idx + (size_t)i * count;
    const uint32_t N = T.n;
    const uint32_t lb = N ? node_lower_bound(T, t) : 0;
    uint32_t n = lb < N ? lb : NONE;
    uint32_t p = N == 0 ? NONE : (lb > 0 ? lb - 1 : (lb < N ? lb : NONE));
    uint64_t kp = p != NONE ? T.key[p] : 0, kn = n != NONE ? T.key[n] : 0;
    uint32_t m = 0;
    while (m < count && (n != NONE || p != NONE)) {
        uint32_t it;
        bool take_p;
        if (p == NONE) take_p = false;
        else if (n == NONE) take_p = true;
        else if (p == n) take_p = false;  // xorCmp(x, x) == 0
        else {
            const uint64_t dp = kp ^ t.hi, dn = kn ^ t.hi;
            if (dp != dn) take_p = dp < dn;
            else {
                const uint32_t* tp = T.tail + 3ull * p;
                const uint32_t* tn = T.tail + 3ull * n;
                take_p = cmp160(0, tp[0] ^ t.t2, tp[1] ^ t.t3, tp[2] ^ t.t4,
                                0, tn[0] ^ t.t2, tn[1] ^ t.t3, tn[2] ^ t.t4) < 0;
            }
        }
        if (take_p) {
            it = p;
            p = p > 0 ? p - 1 : NONE;
            if (p != NONE) kp = T.key[p];
        } else {
            it = n;
            n = n + 1 < N ? n + 1 : NONE;
            if (n != NONE) kn = T.key[n];
        }
        if (it == 0) p = NONE;
        if (!(T.status[it] & KAD_STATUS_EXPIRED)) row[m++] = it + T.index_base;
    }
    for (uint32_t s = m; s < count; s++) row[s] = NONE;
    if (out_cnt) out_cnt[i] = (uint8_t)m;
}

// ---------------------------------------------------------------------------------------
// InfoHash primitives (infohash.h:84-146)
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void load_words(const uint8_t* p, uint32_t w[5]) {
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
#pragma unroll
    for (int k = 0; k < 5; k++) w[k] = __builtin_bswap32(q[k]);
}

__global__ void xor_cmp_kernel(const uint8_t* t, const uint8_t* a, const uint8_t* b, uint32_t n, int8_t* out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t tw[5], aw[5], bw[5];
    load_words(t + 20ull * i, tw);
    load_words(a + 20ull * i, aw);
    load_words(b + 20ull * i, bw);
    int r = 0;
#pragma unroll
    for (int k = 4; k >= 0; k--) {
        const uint32_t x = aw[k] ^ tw[k], y = bw[k] ^ tw[k];
        r = x != y ? (x < y ? -1 : 1) : r;
    }
    out[i] = (int8_t)r;
}

__global__ void common_bits_kernel(const uint8_t* a, const uint8_t* b, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t aw[5], bw[5];
    load_words(a + 20ull * i, aw);
    load_words(b + 20ull * i, bw);
    uint32_t r = 160;
#pragma unroll
    for (int k = 4; k >= 0; k--) {
        const uint32_t x = aw[k] ^ bw[k];
        r = x ? 32u * k + __builtin_clz(x) : r;
    }
    out[i] = r;
}

__global__ void lowbit_kernel(const uint8_t* a, uint32_t n, uint32_t* out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    uint32_t aw[5];
    load_words(a + 20ull * i, aw);
    uint32_t r = NONE;
#pragma unroll
    for (int k = 0; k < 5; k++) r = aw[k] ? 32u * k + 31u - __builtin_ctz(aw[k]) : r;
    out[i] = r;
}

// ---------------------------------------------------------------------------------------
// Table maintenance: status from times, per-bucket good counts, exclusive scan -> dir.y
// ---------------------------------------------------------------------------------------
__global__ void status_from_times_kernel(const int64_t* time_ns, const int64_t* reply_ns, const uint8_t* expired,
                                         uint32_t n, int64_t now, uint8_t* status) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    // node.cpp:34-40 with NODE_GOOD_TIME = 120 min, NODE_EXPIRE_TIME = 10 min (node.h:91-94)
    const int64_t GOOD = 120LL * 60 * 1000000000LL, EXP = 10LL * 60 * 1000000000LL;
    const bool ex = expired[i] != 0;
    const bool good = !ex && reply_ns[i] >= now - GOOD && time_ns[i] >= now - EXP;
    status[i] = (uint8_t)((good ? KAD_STATUS_GOOD : 0u) | (ex ? KAD_STATUS_EXPIRED : 0u));
}

// Per bucket: good count (for the prefix sums) and the good bitmask of its nodes (dir[b].y).
__global__ void bucket_good_kernel(const uint8_t* status, uint2* dir, uint32_t B, uint32_t* cnt) {
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    if (b > B) return;
    if (b == B) { cnt[b] = 0; return; }
    const uint32_t j0 = dir[b].x & ~WIDE, j1 = dir[b + 1].x & ~WIDE;
    uint32_t g = 0, mask = 0;
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t gb = status[j] & KAD_STATUS_GOOD;
        g += gb;
        if (j - j0 < 32) mask |= gb << (j - j0);
    }
    cnt[b] = g;
    dir[b].y = (j1 - j0 <= 32) ? mask : 0u;
}

constexpr int SCAN_ITEMS = 4;
constexpr int SCAN_TILE = BLOCK * SCAN_ITEMS;

__device__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t& total) {
    // wave-level inclusive scan via shuffles, then across the 4 waves of the block
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds[wid] = x;
    __syncthreads();
    uint32_t base = 0;
    for (int w = 0; w < wid; w++) base += lds[w];
    total = lds[0] + lds[1] + lds[2] + lds[3];
    __syncthreads();
    return base + x - v;
}

// Tile-local exclusive scan of cnt[0..m) written to out; tile sums to sums[tile].
__global__ __launch_bounds__(BLOCK) void scan_tiles_kernel(const uint32_t* cnt, uint32_t m, uint32_t* out, uint32_t* sums) {
    __shared__ uint32_t lds[4];
    const uint32_t base = blockIdx.x * SCAN_TILE + threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) { v[k] = base + k < m ? cnt[base + k] : 0; s += v[k]; }
    uint32_t total;
    uint32_t ex = block_exclusive_scan(s, lds, total);
#pragma unroll
    for (int k = 0; k < SCAN_ITEMS; k++) {
        if (base + k < m) out[base + k] = ex;
        ex += v[k];
    }
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// Single-block exclusive scan of the tile sums (in place), looping over chunks.
__global__ __launch_bounds__(BLOCK) void scan_sums_kernel(uint32_t* sums, uint32_t m) {
    __shared__ uint32_t lds[4];
    uint32_t carry = 0;
    for (uint32_t c = 0; c < m; c += BLOCK) {
        const uint32_t i = c + threadIdx.x;
        const uint32_t v = i < m ? sums[i] : 0;
        uint32_t total;
        const uint32_t ex = block_exclusive_scan(v, lds, total);
        if (i < m) sums[i] = carry + ex;
        carry += total;
    }
}

__global__ void scan_apply_kernel(const uint32_t* part, const uint32_t* sums, uint32_t m, uint32_t* gpre) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= m) return;
    gpre[i] = part[i] + sums[i / SCAN_TILE];
}

inline uint32_t grid_for(uint64_t n) { return (uint32_t)((n + BLOCK - 1) / BLOCK); }

// ---------------------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------------------
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

struct Radix {
    uint64_t base = 0;
    uint32_t shift = 63, slots = 1, bits = 0;
};

// Choose (base, shift, slots) so that slot(x) = (x - base) >> shift covers [min_hi, max_hi]
// with at most 2^target_bits slots and the finest shift that fits.
Radix choose_radix(uint64_t min_hi, uint64_t max_hi, uint32_t target_bits) {
    Radix r;
    const unsigned __int128 S = (unsigned __int128)1 << target_bits;
    int best = -1;
    for (int sh = 63; sh >= 0; sh--) {
        const uint64_t base = sh >= 64 ? 0 : (min_hi >> sh) << sh;
        const unsigned __int128 slots = (((unsigned __int128)(max_hi - base)) >> sh) + 1;
        if (slots <= S) best = sh; else break;
    }
    if (best < 0) best = 63;
    r.shift = (uint32_t)best;
    r.base = (min_hi >> best) << best;
    r.slots = (uint32_t)((((unsigned __int128)(max_hi - r.base)) >> best) + 1);
    uint32_t bits = 0;
    while ((1ull << bits) < r.slots) bits++;
    r.bits = bits;
    return r;
}

inline uint64_t id_hi(const uint8_t* p) {
    uint64_t x = 0;
    for (int k = 0; k < 8; k++) x = (x << 8) | p[k];
    return x;
}
inline uint32_t id_word(const uint8_t* p, int w) {
    return ((uint32_t)p[4 * w] << 24) | ((uint32_t)p[4 * w + 1] << 16) | ((uint32_t)p[4 * w + 2] << 8) | p[4 * w + 3];
}
inline bool id_low_zero(const uint8_t* p) {
    for (int k = 8; k < 20; k++)
        if (p[k]) return false;
    return true;
}

// rdx[s] = #items with hi64 < slot_start(s) for s in [0, slots]; items ascending by hi64.
// exact_flag: mark slots whose first item starts exactly at the slot start (low bits zero).
std::vector<uint32_t> build_radix(const Radix& r, uint32_t m, const uint8_t* items, bool exact_flag) {
    std::vector<uint32_t> rdx(r.slots + 1);
    uint32_t j = 0;
    for (uint32_t s = 0; s <= r.slots; s++) {
        const unsigned __int128 start = (unsigned __int128)r.base + ((unsigned __int128)s << r.shift);
        while (j < m && (unsigned __int128)id_hi(items + 20ull * j) < start) j++;
        uint32_t v = j;
        if (exact_flag && j < m && s < r.slots) {
            const uint8_t* it = items + 20ull * j;
            if ((unsigned __int128)id_hi(it) == start && id_low_zero(it)) v |= RDX_EXACT;
        }
        rdx[s] = v;
    }
    return rdx;
}

template <class T>
int dev_upload(T** dptr, const void* src, size_t count, std::vector<void*>& owned, uint64_t& bytes) {
    *dptr = nullptr;
    size_t nb = std::max<size_t>(count * sizeof(T), 16);
    void* p = nullptr;
    hipError_t e = hipMalloc(&p, nb);
    if (e != hipSuccess) return set_err(KAD_ERR_NOMEM, "hipMalloc(%zu) failed: %s", nb, hipGetErrorString(e));
    owned.push_back(p);
    bytes += nb;
    if (src && count) HIP_TRY(hipMemcpy(p, src, count * sizeof(T), hipMemcpyHostToDevice));
    *dptr = static_cast<T*>(p);
    return KAD_OK;
}

}  // namespace

struct kad_table {
    int device = 0;
    uint32_t flags = 0;
    DevTable d{};
    std::vector<void*> owned;
    uint64_t bytes = 0;
    uint32_t rbits = 0, nbits = 0;
    uint8_t* status_mut = nullptr;
    uint2* dir_mut = nullptr;
    uint32_t* gpre_mut = nullptr;
    uint4* rec_mut = nullptr;
    uint32_t rec_depth = 0;
    int64_t* time_ns = nullptr;
    int64_t* reply_ns = nullptr;
    uint8_t* expired = nullptr;
    uint32_t* scan_cnt = nullptr;   // B+1
    uint32_t* scan_part = nullptr;  // B+1
    uint32_t* scan_sums = nullptr;  // tiles
    // exact-path queues of the record kernel, one per stream that queried this table (so that
    // concurrent const queries on distinct streams stay independent)
    std::mutex xq_mu;
    std::vector<std::pair<void*, uint32_t*>> xq;  // (stream, device buffer: 2 counters + list)
    ~kad_table() {
        for (auto& e : xq) (void)hipFree(e.second);
        for (void* p : owned) (void)hipFree(p);
    }
};

namespace {

bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// Rebuild dir[].y (good prefix sums) from the device status array. Async on stream.
int rebuild_good_prefix(kad_table* t, hipStream_t s) {
    const uint32_t B = t->d.B;
    if (B == 0) return KAD_OK;
    const uint32_t m = B + 1;
    const uint32_t tiles = (m + SCAN_TILE - 1) / SCAN_TILE;
    hipLaunchKernelGGL(bucket_good_kernel, dim3(grid_for(m)), dim3(BLOCK), 0, s, t->d.status, t->dir_mut, B, t->scan_cnt);
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(tiles), dim3(BLOCK), 0, s, t->scan_cnt, m, t->scan_part, t->scan_sums);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(BLOCK), 0, s, t->scan_sums, tiles);
    hipLaunchKernelGGL(scan_apply_kernel, dim3(grid_for(m)), dim3(BLOCK), 0, s, t->scan_part, t->scan_sums, m, t->gpre_mut);
    if (t->rec_mut)
        hipLaunchKernelGGL(rec_build_kernel, dim3(grid_for(B)), dim3(BLOCK), 0, s, t->d.key, t->d.status, t->d.dir, B,
                           t->rec_depth, t->rec_mut, t->d.rec_lines);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int check_count(uint32_t count) {
    if (count > KAD_MAX_COUNT) return set_err(KAD_ERR_UNSUPPORTED, "count %u > KAD_MAX_COUNT (%u)", count, KAD_MAX_COUNT);
    return KAD_OK;
}

// KAD_RT_KERNEL=lane forces the lane-per-query kernel where the record kernel would run (A/B
// timing, tools/ab_bench.py); read per call so one process can time both.
constexpr uint32_t EXACT_CAP = 1u << 16;

// The (table, stream) exact-path queue, created zeroed on first use.
int exact_queue(const kad_table* tc, hipStream_t s, ExactQ& Q) {
    kad_table* t = const_cast<kad_table*>(tc);
    std::lock_guard<std::mutex> lk(t->xq_mu);
    uint32_t* buf = nullptr;
    for (auto& e : t->xq)
        if (e.first == (void*)s) buf = e.second;
    if (!buf) {
        HIP_TRY(hipMalloc(&buf, 64 + 32ull * EXACT_CAP));
        HIP_TRY(hipMemset(buf, 0, 8));
        t->xq.emplace_back((void*)s, buf);
    }
    Q.ctr = buf;
    Q.list = buf + 16;  // 64-byte aligned entries
    Q.cap = EXACT_CAP;
    return KAD_OK;
}

template <int K>
int launch_rt(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out, uint8_t* cnt,
              hipStream_t s) {
    const DevTable& d = t->d;
    const char* ev = std::getenv("KAD_RT_KERNEL");
    if (K == 8 && (d.flags & TF_REC) && !(ev && std::strcmp(ev, "lane") == 0)) {
        ExactQ Q;
        int rc = exact_queue(t, s, Q);
        if (rc) return rc;
        if (ev && std::strcmp(ev, "rec_inline") == 0) Q.cap = 0;  // A/B: exact path inline, no list kernel
        if (ev && std::strcmp(ev, "rec_abl1") == 0) {
            hipLaunchKernelGGL((rt_rec_kernel<8, 1>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d, Q, targets, q, count, out, cnt);
            return KAD_OK;
        }
        if (ev && std::strcmp(ev, "rec_abl2") == 0) {
            hipLaunchKernelGGL((rt_rec_kernel<8, 2>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d, Q, targets, q, count, out, cnt);
            return KAD_OK;
        }
        hipLaunchKernelGGL((rt_rec_kernel<8, 0>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d, Q, targets, q, count, out, cnt);
        if (Q.cap == 0) return KAD_OK;
        if (std::getenv("KAD_EXACT_STAMPS"))
            hipLaunchKernelGGL(rt_exact_list_kernel<true>, dim3(EXACT_LIST_BLOCKS), dim3(BLOCK), 0, s, d, Q, targets, count,
                               out, cnt);
        else
            hipLaunchKernelGGL(rt_exact_list_kernel<false>, dim3(EXACT_LIST_BLOCKS), dim3(BLOCK), 0, s, d, Q, targets, count,
                               out, cnt);
    } else {
        hipLaunchKernelGGL(rt_closest_kernel<K>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    }
    return KAD_OK;
}
template <int K>
void launch_rt_dual(const DevTable& d4, const DevTable& d6, const uint8_t* targets, const uint8_t* af, uint32_t q,
                    uint32_t count, uint32_t* out, uint8_t* cnt, hipStream_t s) {
    hipLaunchKernelGGL(rt_closest_dual_kernel<K>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                       out, cnt);
}

int rt_dispatch(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out, uint8_t* cnt,
                hipStream_t s) {
    int rc;
    if (count <= 8) rc = launch_rt<8>(t, targets, q, count, out, cnt, s);
    else if (count <= 16) rc = launch_rt<16>(t, targets, q, count, out, cnt, s);
    else rc = launch_rt<32>(t, targets, q, count, out, cnt, s);
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

}  // namespace

extern "C" {

const char* kad_last_error(void) { return g_err.c_str(); }
int kad_version(void) { return KAD_VERSION; }

int kad_device_count(int* out_n) {
    if (!out_n) return set_err(KAD_ERR_INVALID, "out_n is NULL");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    int k = 0;
    for (int i = 0; i < n; i++) k += is_gfx950(i);
    *out_n = k;
    return KAD_OK;
}

int kad_table_create(kad_table** out, int device, uint32_t n_nodes, const uint8_t* ids, const uint8_t* status,
                     uint32_t n_buckets, const uint8_t* bucket_first, const uint32_t* bucket_offset,
                     uint32_t index_base, uint32_t flags) {
    if (!out) return set_err(KAD_ERR_INVALID, "out is NULL");
    *out = nullptr;
    if (n_nodes && (!ids || !status)) return set_err(KAD_ERR_INVALID, "ids/status NULL with n_nodes=%u", n_nodes);
    if (n_buckets && (!bucket_first || !bucket_offset)) return set_err(KAD_ERR_INVALID, "bucket arrays NULL");
    if (n_nodes >= 0x7FFFFFFFu || n_buckets >= 0x7FFFFFFFu) return set_err(KAD_ERR_INVALID, "table too large");
    if ((uint64_t)index_base + n_nodes >= 0xFFFFFFFEull)
        return set_err(KAD_ERR_INVALID, "index_base + n_nodes must stay below 0xFFFFFFFE");
    // validate directory
    if (n_buckets) {
        if (bucket_offset[0] != 0 || bucket_offset[n_buckets] != n_nodes)
            return set_err(KAD_ERR_INVALID, "bucket_offset must start at 0 and end at n_nodes");
        for (uint32_t b = 0; b < n_buckets; b++) {
            if (bucket_offset[b + 1] < bucket_offset[b]) return set_err(KAD_ERR_INVALID, "bucket_offset not monotone at %u", b);
            if (b && std::memcmp(bucket_first + 20ull * (b - 1), bucket_first + 20ull * b, 20) >= 0)
                return set_err(KAD_ERR_INVALID, "bucket firsts not strictly ascending at %u", b);
        }
    } else if (!(flags & KAD_TABLE_SORTED) && n_nodes) {
        return set_err(KAD_ERR_INVALID, "a table without buckets must be KAD_TABLE_SORTED");
    }
    if (flags & KAD_TABLE_SORTED) {
        for (uint32_t i = 1; i < n_nodes; i++)
            if (std::memcmp(ids + 20ull * (i - 1), ids + 20ull * i, 20) >= 0)
                return set_err(KAD_ERR_NOT_SORTED, "ids not strictly ascending at %u", i);
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev)
        return set_err(KAD_ERR_NO_DEVICE, "device %d not available (%d devices)", device, ndev);
    if (!is_gfx950(device)) return set_err(KAD_ERR_NO_DEVICE, "device %d is not gfx950", device);
    DeviceGuard g(device);

    auto* t = new kad_table();
    t->device = device;
    t->flags = flags;
    DevTable& d = t->d;
    d.n = n_nodes;
    d.B = n_buckets;
    d.index_base = index_base;
    int rc;
    // node arrays: key[] padded by KEY_PAD so chunked 16-byte loads stay inside the allocation
    std::vector<uint64_t> key(n_nodes + KEY_PAD, ~0ull);
    std::vector<uint32_t> tail(3ull * n_nodes);
    for (uint32_t i = 0; i < n_nodes; i++) {
        const uint8_t* p = ids + 20ull * i;
        key[i] = id_hi(p);
        tail[3ull * i] = id_word(p, 2);
        tail[3ull * i + 1] = id_word(p, 3);
        tail[3ull * i + 2] = id_word(p, 4);
    }
    // nodes whose top 64 ID bits are shared with another node: only they can tie on the
    // top-64 XOR distance, so only they take the exact 160-bit compare
    std::vector<uint8_t> dup(n_nodes, 0);
    bool any_dup = false;
    {
        bool asc = true;
        for (uint32_t i = 1; i < n_nodes && asc; i++) asc = key[i - 1] <= key[i];
        if (asc) {
            for (uint32_t i = 1; i < n_nodes; i++)
                if (key[i - 1] == key[i]) { dup[i - 1] = dup[i] = 1; any_dup = true; }
        } else {
            std::vector<uint64_t> sk(key.begin(), key.begin() + n_nodes);
            std::sort(sk.begin(), sk.end());
            for (uint32_t i = 1; i < n_nodes && !any_dup; i++) any_dup = sk[i - 1] == sk[i];
            if (any_dup)
                for (uint32_t i = 0; i < n_nodes; i++) {
                    auto r = std::equal_range(sk.begin(), sk.end(), key[i]);
                    dup[i] = (r.second - r.first) > 1;
                }
        }
    }
    if (any_dup) d.flags |= TF_HAS_DUP;
    uint64_t* dkey; uint32_t* dtail; uint8_t* dst;
    if ((rc = dev_upload(&dkey, key.data(), key.size(), t->owned, t->bytes)) ||
        (rc = dev_upload(&dtail, tail.data(), 3ull * n_nodes, t->owned, t->bytes)) ||
        (rc = dev_upload(&dst, status, n_nodes, t->owned, t->bytes))) { delete t; return rc; }
    d.key = dkey; d.tail = dtail; d.status = dst; t->status_mut = dst;
    std::vector<uint64_t>().swap(key);
    std::vector<uint32_t>().swap(tail);

    // bucket directory
    if (n_buckets) {
        std::vector<uint2> dir(n_buckets + 1);
        std::vector<uint32_t> gpre(n_buckets + 1), dmask(any_dup ? n_buckets : 0);
        uint32_t g = 0;
        for (uint32_t b = 0; b <= n_buckets; b++) {
            dir[b].x = bucket_offset[b];
            dir[b].y = 0;
            gpre[b] = g;
            if (b < n_buckets) {
                const uint32_t j0 = bucket_offset[b], j1 = bucket_offset[b + 1];
                if (j1 - j0 > 32) dir[b].x |= WIDE;
                for (uint32_t j = j0; j < j1; j++) {
                    const uint32_t gb = status[j] & KAD_STATUS_GOOD;
                    g += gb;
                    if (j1 - j0 <= 32) {
                        dir[b].y |= gb << (j - j0);
                        if (any_dup) dmask[b] |= (uint32_t)dup[j] << (j - j0);
                    }
                }
                // a wide bucket's dup nodes are handled by the slow path (wide -> deferred)
            }
        }
        std::vector<uint64_t> fkey(n_buckets);
        std::vector<uint32_t> ftail(3ull * n_buckets);
        for (uint32_t b = 0; b < n_buckets; b++) {
            const uint8_t* p = bucket_first + 20ull * b;
            fkey[b] = id_hi(p);
            ftail[3ull * b] = id_word(p, 2);
            ftail[3ull * b + 1] = id_word(p, 3);
            ftail[3ull * b + 2] = id_word(p, 4);
        }
        uint32_t tb = 1;
        while ((1u << tb) < n_buckets && tb < 24) tb++;
        Radix r = choose_radix(fkey[0], fkey[n_buckets - 1], std::min<uint32_t>(tb + 1, 24));
        // Uniform depth (U(d) tables, shards of them): firsts equally spaced by a power of two
        // 2^k and aligned to it, low 96 bits zero -> the radix IS the bucket index (shift k).
        if (n_buckets >= 2) {
            const uint64_t step = fkey[1] - fkey[0];
            bool uni = step && (step & (step - 1)) == 0 && (fkey[0] & (step - 1)) == 0;
            for (uint32_t b = 0; b < n_buckets && uni; b++) {
                uni = (b == 0 || fkey[b] - fkey[b - 1] == step) && !ftail[3ull * b] && !ftail[3ull * b + 1] &&
                      !ftail[3ull * b + 2];
            }
            if (uni) {
                r.shift = (uint32_t)__builtin_ctzll(step);
                r.base = fkey[0];
                r.slots = n_buckets;
                r.bits = tb;
            }
        }
        std::vector<uint32_t> rdx = build_radix(r, n_buckets, bucket_first, true);
        // direct-mapped locate: slot s holds exactly bucket s, starting at the slot start
        bool direct = r.slots == n_buckets;
        for (uint32_t sl = 0; sl < r.slots && direct; sl++) direct = rdx[sl] == (sl | RDX_EXACT);
        if (direct) d.flags |= TF_DIRECT;
        const uint32_t depth = 64 - r.shift;
        uint2* ddir; uint64_t* dfk; uint32_t *dft, *drdx, *dgp, *ddm = nullptr;
        if ((rc = dev_upload(&ddir, dir.data(), n_buckets + 1, t->owned, t->bytes)) ||
            (rc = dev_upload(&dgp, gpre.data(), n_buckets + 1, t->owned, t->bytes)) ||
            (any_dup && (rc = dev_upload(&ddm, dmask.data(), n_buckets, t->owned, t->bytes))) ||
            (rc = dev_upload(&dfk, fkey.data(), n_buckets, t->owned, t->bytes)) ||
            (rc = dev_upload(&dft, ftail.data(), 3ull * n_buckets, t->owned, t->bytes)) ||
            (rc = dev_upload(&drdx, rdx.data(), rdx.size(), t->owned, t->bytes)) ||
            (rc = dev_upload(&t->scan_cnt, nullptr, n_buckets + 1, t->owned, t->bytes)) ||
            (rc = dev_upload(&t->scan_part, nullptr, n_buckets + 1, t->owned, t->bytes)) ||
            (rc = dev_upload(&t->scan_sums, nullptr, (n_buckets + 1 + SCAN_TILE - 1) / SCAN_TILE, t->owned, t->bytes))) {
            delete t;
            return rc;
        }
        d.dir = ddir; t->dir_mut = ddir; d.gpre = dgp; t->gpre_mut = dgp; d.dmask = ddm; d.fkey = dfk; d.ftail = dft; d.rrdx = drdx;
        d.rbase = r.base; d.rshift = r.shift; d.rslots = r.slots; t->rbits = r.bits;
        // bucket records (rt_rec_kernel): direct-mapped, uniform depth 1..48, every node inside its
        // bucket's dyadic range, first node index below 2^27
        if (direct && depth >= 1 && depth <= 48 && n_nodes <= REC_FIRST_MASK) {
            bool inside = true;
            const uint64_t pre0 = r.base >> r.shift;
            for (uint32_t b = 0; b < n_buckets && inside; b++)
                for (uint32_t j = bucket_offset[b]; j < bucket_offset[b + 1] && inside; j++)
                    inside = (id_hi(ids + 20ull * j) >> r.shift) == pre0 + b;
            if (inside) {
                const uint32_t lines = (n_buckets + 1) / 4 + 2;  // per copy: covers records 0 .. B+1 (+ pad)
                uint4* rp;
                if ((rc = dev_upload(&rp, nullptr, 4ull * 8 * lines, t->owned, t->bytes))) {
                    delete t;
                    return rc;
                }
                if (hipMemset(rp, 0, 4ull * 128 * lines) != hipSuccess) {
                    delete t;
                    return set_err(KAD_ERR_HIP, "hipMemset failed");
                }
                hipLaunchKernelGGL(rec_build_kernel, dim3(grid_for(n_buckets)), dim3(BLOCK), 0, 0, d.key, d.status, d.dir,
                                   n_buckets, depth, rp, lines);
                if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
                    delete t;
                    return set_err(KAD_ERR_HIP, "record build failed");
                }
                d.rec = rp; d.rec_lines = lines; t->rec_mut = rp; t->rec_depth = depth;
                d.flags |= TF_REC;
            }
        }
    }
    // NodeCache radix
    if ((flags & KAD_TABLE_SORTED) && n_nodes) {
        uint32_t tb = 1;
        while ((1u << tb) < n_nodes && tb < 23) tb++;
        const Radix r = choose_radix(id_hi(ids), id_hi(ids + 20ull * (n_nodes - 1)), tb);
        std::vector<uint32_t> rdx = build_radix(r, n_nodes, ids, false);
        uint32_t* dn;
        if ((rc = dev_upload(&dn, rdx.data(), rdx.size(), t->owned, t->bytes))) { delete t; return rc; }
        d.nrdx = dn; d.nbase = r.base; d.nshift = r.shift; d.nslots = r.slots; t->nbits = r.bits;
    }
    *out = t;
    return KAD_OK;
}

int kad_table_destroy(kad_table* t) {
    if (!t) return KAD_OK;
    DeviceGuard g(t->device);
    (void)hipDeviceSynchronize();
    delete t;
    return KAD_OK;
}

int kad_table_get_info(const kad_table* t, kad_table_info* out) {
    if (!t || !out) return set_err(KAD_ERR_INVALID, "NULL argument");
    out->n_nodes = t->d.n;
    out->n_buckets = t->d.B;
    out->index_base = t->d.index_base;
    out->flags = t->flags;
    out->device = t->device;
    out->rt_radix_bits = t->rbits;
    out->nc_radix_bits = t->nbits;
    out->device_bytes = t->bytes;
    out->n_good = 0;
    if (t->d.B) {
        DeviceGuard g(t->device);
        uint32_t last;
        HIP_TRY(hipMemcpy(&last, t->d.gpre + t->d.B, sizeof last, hipMemcpyDeviceToHost));
        out->n_good = last;
    }
    return KAD_OK;
}

int kad_table_update_status(kad_table* t, const uint8_t* status) {
    if (!t || (!status && t->d.n)) return set_err(KAD_ERR_INVALID, "NULL argument");
    DeviceGuard g(t->device);
    if (t->d.n) HIP_TRY(hipMemcpy(t->status_mut, status, t->d.n, hipMemcpyHostToDevice));
    int rc = rebuild_good_prefix(t, nullptr);
    if (rc) return rc;
    HIP_TRY(hipDeviceSynchronize());
    return KAD_OK;
}

int kad_table_set_times(kad_table* t, const int64_t* time_ns, const int64_t* reply_ns, const uint8_t* expired) {
    if (!t || (t->d.n && (!time_ns || !reply_ns || !expired))) return set_err(KAD_ERR_INVALID, "NULL argument");
    DeviceGuard g(t->device);
    int rc;
    if (!t->time_ns) {
        if ((rc = dev_upload(&t->time_ns, nullptr, t->d.n, t->owned, t->bytes)) ||
            (rc = dev_upload(&t->reply_ns, nullptr, t->d.n, t->owned, t->bytes)) ||
            (rc = dev_upload(&t->expired, nullptr, t->d.n, t->owned, t->bytes)))
            return rc;
    }
    if (t->d.n) {
        HIP_TRY(hipMemcpy(t->time_ns, time_ns, 8ull * t->d.n, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(t->reply_ns, reply_ns, 8ull * t->d.n, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(t->expired, expired, t->d.n, hipMemcpyHostToDevice));
    }
    return KAD_OK;
}

int kad_table_refresh_status(kad_table* t, int64_t now_ns, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (!t->time_ns) return set_err(KAD_ERR_INVALID, "kad_table_set_times was not called");
    DeviceGuard g(t->device);
    hipStream_t s = (hipStream_t)stream;
    if (t->d.n)
        hipLaunchKernelGGL(status_from_times_kernel, dim3(grid_for(t->d.n)), dim3(BLOCK), 0, s, t->time_ns, t->reply_ns,
                           t->expired, t->d.n, now_ns, t->status_mut);
    HIP_TRY(hipGetLastError());
    return rebuild_good_prefix(t, s);
}

int kad_rt_closest_batch(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                         uint8_t* out_cnt, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    int rc = check_count(count);
    if (rc) return rc;
    if (q == 0) return KAD_OK;
    if (!targets || (!out_idx && count)) return set_err(KAD_ERR_INVALID, "NULL buffer");
    if (count == 0 && !out_cnt) return KAD_OK;
    if (((uintptr_t)targets & 3) || ((uintptr_t)out_idx & 3)) return set_err(KAD_ERR_INVALID, "device buffers must be 4-byte aligned");
    DeviceGuard g(t->device);
    return rt_dispatch(t, targets, q, count, out_idx, out_cnt, (hipStream_t)stream);
}

int kad_rt_closest_batch_dual(const kad_table* t4, const kad_table* t6, const uint8_t* targets, const uint8_t* af,
                              uint32_t q, uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, void* stream) {
    if (!t4 && !t6) return set_err(KAD_ERR_INVALID, "both tables NULL");
    if (t4 && t6 && t4->device != t6->device) return set_err(KAD_ERR_INVALID, "tables on different devices");
    int rc = check_count(count);
    if (rc) return rc;
    if (q == 0) return KAD_OK;
    if (!targets || !af || !out_idx) return set_err(KAD_ERR_INVALID, "NULL buffer");
    // A missing family behaves as an empty table (zero results), as an empty RoutingTable does.
    DevTable empty{};
    const DevTable& d4 = t4 ? t4->d : empty;
    const DevTable& d6 = t6 ? t6->d : empty;
    DeviceGuard g(t4 ? t4->device : t6->device);
    hipStream_t s = (hipStream_t)stream;
    if (count <= 8) launch_rt_dual<8>(d4, d6, targets, af, q, count, out_idx, out_cnt, s);
    else if (count <= 16) launch_rt_dual<16>(d4, d6, targets, af, q, count, out_idx, out_cnt, s);
    else launch_rt_dual<32>(d4, d6, targets, af, q, count, out_idx, out_cnt, s);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_rt_find_bucket_batch(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t* out_bucket, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (q == 0) return KAD_OK;
    if (!targets || !out_bucket) return set_err(KAD_ERR_INVALID, "NULL buffer");
    DeviceGuard g(t->device);
    hipLaunchKernelGGL(find_bucket_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d, targets, q,
                       out_bucket);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_nc_closest_batch(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                         uint8_t* out_cnt, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (!(t->flags & KAD_TABLE_SORTED)) return set_err(KAD_ERR_NOT_SORTED, "NodeCache query needs a KAD_TABLE_SORTED table");
    if (count > 255) return set_err(KAD_ERR_UNSUPPORTED, "count %u > 255", count);
    if (q == 0) return KAD_OK;
    if (!targets || (!out_idx && count)) return set_err(KAD_ERR_INVALID, "NULL buffer");
    DeviceGuard g(t->device);
    hipLaunchKernelGGL(nc_closest_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d, targets, q, count,
                       out_idx, out_cnt);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

static int host_query(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                      uint8_t* out_cnt, bool nc) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (q == 0) return KAD_OK;
    if (!targets || !out_idx) return set_err(KAD_ERR_INVALID, "NULL buffer");
    DeviceGuard g(t->device);
    uint8_t* dt = nullptr; uint32_t* di = nullptr; uint8_t* dc = nullptr;
    const size_t nidx = std::max<size_t>((size_t)q * count, 1);
    HIP_TRY(hipMalloc(&dt, 20ull * q));
    if (hipMalloc(&di, 4ull * nidx) != hipSuccess || hipMalloc(&dc, q) != hipSuccess) {
        (void)hipFree(dt); (void)hipFree(di);
        return set_err(KAD_ERR_NOMEM, "hipMalloc failed");
    }
    int rc = KAD_OK;
    if (hipMemcpy(dt, targets, 20ull * q, hipMemcpyHostToDevice) != hipSuccess) rc = set_err(KAD_ERR_HIP, "H2D failed");
    if (!rc) rc = nc ? kad_nc_closest_batch(t, dt, q, count, di, dc, nullptr) : kad_rt_closest_batch(t, dt, q, count, di, dc, nullptr);
    if (!rc && hipDeviceSynchronize() != hipSuccess) rc = set_err(KAD_ERR_HIP, "kernel failed");
    if (!rc && count && hipMemcpy(out_idx, di, 4ull * q * count, hipMemcpyDeviceToHost) != hipSuccess) rc = set_err(KAD_ERR_HIP, "D2H failed");
    if (!rc && out_cnt && hipMemcpy(out_cnt, dc, q, hipMemcpyDeviceToHost) != hipSuccess) rc = set_err(KAD_ERR_HIP, "D2H failed");
    (void)hipFree(dt); (void)hipFree(di); (void)hipFree(dc);
    return rc;
}

int kad_rt_closest_batch_host(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                              uint8_t* out_cnt) {
    return host_query(t, targets, q, count, out_idx, out_cnt, false);
}
int kad_nc_closest_batch_host(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                              uint8_t* out_cnt) {
    return host_query(t, targets, q, count, out_idx, out_cnt, true);
}

/* Diagnostics (not in kadgpu.h): copy the exact-list kernel's per-wave stamps (KAD_EXACT_STAMPS=1). */
int kad_debug_exact_stamps(uint64_t* host, uint32_t n) {
    if (!host) return set_err(KAD_ERR_INVALID, "NULL buffer");
    HIP_TRY(hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), 8ull * std::min<uint32_t>(n, STAMP_WAVES * 12)));
    return KAD_OK;
}

int kad_xor_cmp_batch(const uint8_t* targets, const uint8_t* a, const uint8_t* b, uint32_t n, int8_t* out, void* stream) {
    if (n == 0) return KAD_OK;
    if (!targets || !a || !b || !out) return set_err(KAD_ERR_INVALID, "NULL buffer");
    hipLaunchKernelGGL(xor_cmp_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, targets, a, b, n, out);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}
int kad_common_bits_batch(const uint8_t* a, const uint8_t* b, uint32_t n, uint32_t* out, void* stream) {
    if (n == 0) return KAD_OK;
    if (!a || !b || !out) return set_err(KAD_ERR_INVALID, "NULL buffer");
    hipLaunchKernelGGL(common_bits_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, a, b, n, out);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}
int kad_lowbit_batch(const uint8_t* a, uint32_t n, uint32_t* out, void* stream) {
    if (n == 0) return KAD_OK;
    if (!a || !out) return set_err(KAD_ERR_INVALID, "NULL buffer");
    hipLaunchKernelGGL(lowbit_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, a, n, out);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

}  // extern "C"
