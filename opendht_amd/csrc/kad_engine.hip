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
//   gcnt[B+1]   u32  good nodes of bucket b (gcnt[B] = 0): window sizes for the slow path and the line builders
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
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <array>
#include <chrono>
#include <map>
#include <unordered_map>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/kadgpu.h"
#include "kad_mirror_plan.h"

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
    const uint32_t* gcnt;  // good nodes per bucket, B + 1 entries (the last 0)
    const uint32_t* dmask;
    const uint64_t* fkey;
    const uint32_t* ftail;
    const uint32_t* rrdx;
    const uint32_t* nrdx;
    const uint4* wl;    // window lines (TF_WL): 128 bytes per bucket, see rt_wl_kernel
    const uint4* wl16;  // window lines for counts 9..16 (TF_WL16): 128 bytes per bucket
    const uint4* wl32;  // window lines for counts 17..32 (TF_WL32): 256 bytes per bucket
    const uint4* ncl;   // NodeCache lines (TF_NCL): 256 bytes per node radix slot
    const uint4* gl;    // general window lines, count <= 8 (TF_GL, any table shape): 128 bytes per bucket
    const uint4* gl32;  // general window lines, counts 9..32 (TF_GL32): 256 bytes per bucket
    const uint4* ws;    // short window lines, count <= 8 (TF_WS, with TF_WL): 64 bytes per bucket
    const uint4* ncl32; // NodeCache lines for counts 17..32 (TF_NCL32): 512 bytes per node radix slot
    const uint4* sl;    // slot lines, count <= 8 (TF_SL, with TF_GL): 64 bytes per coarse radix slot
    const uint4* gl16;  // general window lines, counts 9..16 (TF_GL16): 128 bytes per bucket
    const uint4* sl16;  // slot lines, counts 9..16 (TF_SL16, with TF_SL): 128 bytes per coarse radix slot
    const uint32_t* slb;  // (TF_SL) the bucket of every coarse radix slot, NONE where a bucket starts inside it
    uint32_t slshift, slslots;
    uint64_t rbase, nbase;
    uint32_t rshift, rslots, nshift, nslots;
    uint32_t n, B, index_base, flags;
};

constexpr uint32_t TF_DIRECT = 1u;   // radix slot s holds exactly bucket s (no locate load)
constexpr uint32_t TF_HAS_DUP = 2u;  // some nodes share their top 64 ID bits
constexpr uint32_t TF_WL = 8u;       // window lines present (direct-mapped, uniform depth 1..43)
constexpr uint32_t TF_WL16 = 16u;    // window lines for counts 9..16 present
constexpr uint32_t TF_WL32 = 32u;    // window lines for counts 17..32 present
constexpr uint32_t TF_NCL = 64u;     // NodeCache lines present (sorted tables)
constexpr uint32_t TF_GL = 128u;     // general window lines (tables without TF_WL: split-policy, per-peer shapes)
constexpr uint32_t TF_GL32 = 256u;   // general window lines for counts 9..32
constexpr uint32_t TF_NCL32 = 1024u; // 512-byte NodeCache lines (counts 17..32) present
constexpr uint32_t TF_SL = 2048u;    // slot lines (count <= 8, general tables: no locate load)
constexpr uint32_t TF_GL16 = 4096u;  // general window lines for counts 9..16 (one 128-byte line)
constexpr uint32_t TF_SL16 = 8192u;  // slot lines for counts 9..16 (copies of the gl16 lines by coarse radix slot)
constexpr uint32_t TF_WS = 512u;     // short (64-byte) window lines for count <= 8 (uniform tables, with TF_WL)
constexpr uint32_t WIDE = 0x80000000u;  // dir[].x flag: bucket holds > 32 nodes (masks invalid)
constexpr uint32_t KEY_PAD = 32;        // key[] is padded so 16-node chunk loads never leave it

struct Target {
    uint64_t hi;       // bits 0..63
    uint32_t t2, t3, t4;
};

// Which lines a line builder (re)builds: every one (idx == NULL) or the *n listed ones (the compacted
// dirty flags of an incremental status refresh). Thread j picks line b.
struct LineSel {
    const uint32_t* idx;
    const uint32_t* n;
    __device__ __forceinline__ bool pick(uint32_t j, uint32_t total, uint32_t& b) const {
        if (!idx) { b = j; return j < total; }
        if (j >= *n) return false;
        b = idx[j];
        return true;
    }
};

// Target batches are read once: non-temporal loads (as the rows, st_row4 below), two 8-byte and one 4-byte load (two
// 4-byte non-temporal loads may be merged into one plain 8-byte load). KAD_PLAIN_STREAMS: the plain policy.
__device__ __forceinline__ Target load_target(const uint8_t* targets, uint32_t i) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(targets + 20ull * i);
    Target t;
#ifdef KAD_PLAIN_STREAMS
    const uint32_t w0 = p[0], w1 = p[1], w2 = p[2], w3 = p[3], w4 = p[4];
#else
    const uint64_t a = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p));
    const uint64_t b = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(p + 2));
    const uint32_t w0 = (uint32_t)a, w1 = (uint32_t)(a >> 32), w2 = (uint32_t)b, w3 = (uint32_t)(b >> 32);
    const uint32_t w4 = __builtin_nontemporal_load(p + 4);
#endif
    t.hi = ((uint64_t)__builtin_bswap32(w0) << 32) | __builtin_bswap32(w1);
    t.t2 = __builtin_bswap32(w2);
    t.t3 = __builtin_bswap32(w3);
    t.t4 = __builtin_bswap32(w4);
    return t;
}

// The top 64 bits of target i (direct-mapped tables locate with these alone).
__device__ __forceinline__ uint64_t load_target_hi(const uint8_t* targets, uint32_t i) {
#ifdef KAD_PLAIN_STREAMS
    const uint32_t* p = reinterpret_cast<const uint32_t*>(targets + 20ull * i);
    return ((uint64_t)__builtin_bswap32(p[0]) << 32) | __builtin_bswap32(p[1]);
#else
    const uint64_t w = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(targets + 20ull * i));
    return ((uint64_t)__builtin_bswap32((uint32_t)w) << 32) | __builtin_bswap32((uint32_t)(w >> 32));
#endif
}

// Result rows leave with the non-temporal policy: written once, they would otherwise displace the line tables from
// the Infinity Cache (the headline kernel: 32.7 -> 31.8 us per 1M, profiles/r03/ab_ws_nts/). KAD_PLAIN_STREAMS (an
// A/B build of the tools, like KAD_ABLATIONS) keeps the plain policy.
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_row4(uint32_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
#ifdef KAD_PLAIN_STREAMS
    *reinterpret_cast<uint4*>(p) = make_uint4(a, b, c, d);
#else
    __builtin_nontemporal_store(u32x4_t{a, b, c, d}, reinterpret_cast<u32x4_t*>(p));
#endif
}
__device__ __forceinline__ void st_row1(uint32_t* p, uint32_t v) {
#ifdef KAD_PLAIN_STREAMS
    *p = v;
#else
    __builtin_nontemporal_store(v, p);
#endif
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
    // tables with slot lines: the coarse slot's bucket, one load, unless a bucket starts inside the slot (~1 %); the
    // radix below otherwise (one or two loads, and a search of the bucket firsts where a radix slot holds several)
    if ((T.flags & TF_SL) && t.hi >= T.rbase) {
        const uint64_t j = (t.hi - T.rbase) >> T.slshift;
        if (j < T.slslots) {
            const uint32_t b = T.slb[j];
            if (b != NONE) return b;
        }
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
                // count firsts <= t among [lo, hi); the first's low 96 bits are read only on a top-64 tie
                while (lo < hi) {
                    uint32_t mid = (lo + hi) >> 1;
                    const uint64_t fk = T.fkey[mid];
                    int c;
                    if (fk != t.hi) {
                        c = fk < t.hi ? -1 : 1;
                    } else {
                        const uint32_t* ft = T.ftail + 3ull * mid;
                        c = cmp160(fk, ft[0], ft[1], ft[2], t.hi, t.t2, t.t3, t.t4);
                    }
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

// Ranks nodes [beg, end) of T (`good` of them good) for the wave-uniform target t: row[0..count) =
// the first min(count, good) good nodes by (160-bit XOR distance, index), + index_base, padded with
// NONE. If `dist` is given, dist[5*r .. 5*r+4] = the XOR distance of row entry r as five native
// words (most significant first): the merge key of kad_rt_merge_parts.
// tie (key-only queries, kad_rt_closest_keys_packed: the target's low 96 bits unknown, taken as zero): the order is
// that of the full target unless two nodes of [beg, end) share their top 64 bits (equal keys are adjacent in a sorted
// table), which sets *tie: the caller answers the batch again from full targets.
__device__ void wave_rank(const DevTable& T, const Target& t, uint32_t beg, uint32_t end, uint32_t good,
                          uint32_t count, uint32_t* row, uint32_t* dist, uint64_t* xs, uint32_t* tie = nullptr) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m = min(count, good);
    if (tie) {
        bool eq = false;
        for (uint32_t j = beg + lane; j + 1 < end; j += 64) eq |= T.key[j] == T.key[j + 1];
        if (__any(eq) && lane == 0) atomicOr(tie, 1u);
    }
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
        __builtin_amdgcn_wave_barrier();  // xs is reused by the wave's next query
        if (v && rank < count) {
            row[rank] = j + T.index_base;
            if (dist) {
                uint32_t* dd = dist + 5 * rank;
                dd[0] = (uint32_t)(V0 >> 32); dd[1] = (uint32_t)V0;
                dd[2] = (uint32_t)(V1 >> 32); dd[3] = (uint32_t)V1;
                dd[4] = (uint32_t)(V2 >> 32);
            }
        }
        if (lane >= m && lane < count) row[lane] = NONE;
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
    if (dist && lane < m) {
        uint32_t* dd = dist + 5 * lane;
        dd[0] = (uint32_t)(L0 >> 32); dd[1] = (uint32_t)L0;
        dd[2] = (uint32_t)(L1 >> 32); dd[3] = (uint32_t)L1;
        dd[4] = (uint32_t)(L2 >> 32);
    }
}

// Good nodes that round r adds to the window of bucket b: W(0) = [b-1, b], round r >= 1 adds b-1-r and b+r
// (each only if it exists; routing_table.cpp:89-104 closed form).
__device__ __forceinline__ uint32_t ring_good(const uint32_t* gcnt, uint32_t B, uint32_t b, uint32_t r) {
    if (r == 0) return gcnt[b] + (b ? gcnt[b - 1] : 0u);
    return (b > r ? gcnt[b - 1 - r] : 0u) + ((uint64_t)b + r < (uint64_t)B ? gcnt[b + r] : 0u);
}

// W(R) of a wave-uniform target on one table (routing_table.cpp:89-104 closed form): lane l takes round
// r0 + l, a wave scan of the per-round good counts gives each round's window size and a ballot the least R;
// 64 rounds per probe. Returns the window's buckets [lo, hi] and good count.
__device__ __forceinline__ void wave_window(const uint32_t* gcnt, uint32_t B, uint32_t b, uint32_t count,
                                            uint32_t& lo, uint32_t& hi, uint32_t& good) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t carry = 0;
    for (uint32_t r0 = 0;; r0 += 64) {
        const uint32_t r = r0 + lane;
        const uint32_t l_ = b > r ? b - 1 - r : 0u;
        const uint32_t h_ = (uint64_t)b + r >= (uint64_t)B - 1 ? B - 1 : b + r;
        uint32_t g_ = ring_good(gcnt, B, b, r);
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(g_, o, 64);
            if (lane >= (uint32_t)o) g_ += y;
        }
        g_ += carry;
        const uint64_t ok = __ballot(g_ >= count || (l_ == 0 && h_ == B - 1));
        if (ok) {
            const uint32_t R = (uint32_t)__builtin_ctzll(ok);
            lo = rdl(l_, R);
            hi = rdl(h_, R);
            good = rdl(g_, R);
            return;
        }
        carry = rdl(g_, 63);
    }
}

// wave_window over good prefix sums (the north-star shard's replicated global directory, GB + 1 entries).
__device__ __forceinline__ void wave_window_pre(const uint32_t* gpre, uint32_t B, uint32_t b, uint32_t count,
                                                uint32_t& lo, uint32_t& hi, uint32_t& good) {
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t r0 = 0;; r0 += 64) {
        const uint32_t r = r0 + lane;
        const uint32_t l_ = b > r ? b - 1 - r : 0u;
        const uint32_t h_ = (uint64_t)b + r >= (uint64_t)B - 1 ? B - 1 : b + r;
        const uint32_t g_ = gpre[h_ + 1] - gpre[l_];
        const uint64_t ok = __ballot(g_ >= count || (l_ == 0 && h_ == B - 1));
        if (ok) {
            const uint32_t R = (uint32_t)__builtin_ctzll(ok);
            lo = rdl(l_, R);
            hi = rdl(h_, R);
            good = rdl(g_, R);
            return;
        }
    }
}

// Sum of gcnt[a, e) by the whole wave (wave-uniform arguments).
__device__ __forceinline__ uint32_t wave_good_sum(const uint32_t* gcnt, uint32_t a, uint32_t e) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t s = 0;
    for (uint32_t x = a + lane; x < e; x += 64) s += gcnt[x];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    return s;
}

__device__ void wave_exact(const DevTable& T, const Target& t, uint32_t count, uint32_t* row, uint8_t* cp,
                           uint64_t* xs /* this wave's 64 x 3 LDS words */, uint32_t* tie = nullptr) {
    const uint32_t lane = threadIdx.x & 63u, B = T.B;
    if (B == 0 || count == 0) {
        if (lane < count) row[lane] = NONE;
        if (lane == 0 && cp) *cp = 0;
        return;
    }
    uint32_t lo, hi, good;
    wave_window(T.gcnt, B, locate_bucket(T, t), count, lo, hi, good);
    wave_rank(T, t, T.dir[lo].x & ~WIDE, T.dir[hi + 1].x & ~WIDE, good, count, row, nullptr, xs, tie);
    if (lane == 0 && cp) *cp = (uint8_t)min(count, good);
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

// Lane-per-query RoutingTable kernel (any table shape, count <= 32).
template <int K>
__device__ __forceinline__ void rt_closest_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets,
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
template <int K>
__global__ __launch_bounds__(BLOCK) void rt_closest_kernel(DevTable T, const uint8_t* __restrict__ targets,
                                                           uint32_t q, uint32_t count,
                                                           uint32_t* __restrict__ out_idx,
                                                           uint8_t* __restrict__ out_cnt) {
    rt_closest_kernel_body<K>(T, targets, q, count, out_idx, out_cnt);
}

// ---------------------------------------------------------------------------------------
// Any count (the reference takes any size_t, routing_table.h:48): counts above the line kernels' 32 take one
// wave per query. The window W(R) comes from the good prefix sums (wave_window), and every good node of it
// is ranked by counting, tile against tile: a lane holds one node of its 64-node tile and counts the good
// nodes of every tile that precede it in (160-bit XOR distance, index) order, so windows of any size need
// only the wave's 1.5 KB of LDS. Rows beyond the result are padded with NONE; the count byte saturates at
// 255 (a caller asking for more reads the count off the padding).
// ---------------------------------------------------------------------------------------
__device__ void wave_rank_any(const DevTable& T, const Target& t, uint32_t beg, uint32_t end, uint32_t good,
                              uint32_t count, uint32_t* row, uint8_t* cp, uint64_t* xs) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t m = min(count, good);
    for (uint32_t a = beg; a < end; a += 64) {
        const uint32_t j = a + lane;
        uint64_t V0 = ~0ull, V1 = ~0ull, V2 = ~0ull;
        const bool v = j < end && (T.status[j] & KAD_STATUS_GOOD);
        if (v) {
            const uint32_t* tl = T.tail + 3ull * j;
            V0 = T.key[j] ^ t.hi;
            V1 = ((uint64_t)(tl[0] ^ t.t2) << 32) | (tl[1] ^ t.t3);
            V2 = ((uint64_t)(tl[2] ^ t.t4) << 32) | j;
        }
        uint32_t rank = 0;
        for (uint32_t c = beg; c < end; c += 64) {
            const uint32_t jc = c + lane;
            uint64_t C0 = ~0ull, C1 = ~0ull, C2 = ~0ull;  // not good: after every node
            if (jc < end && (T.status[jc] & KAD_STATUS_GOOD)) {
                const uint32_t* tl = T.tail + 3ull * jc;
                C0 = T.key[jc] ^ t.hi;
                C1 = ((uint64_t)(tl[0] ^ t.t2) << 32) | (tl[1] ^ t.t3);
                C2 = ((uint64_t)(tl[2] ^ t.t4) << 32) | jc;
            }
            __builtin_amdgcn_wave_barrier();
            xs[3 * lane] = C0;
            xs[3 * lane + 1] = C1;
            xs[3 * lane + 2] = C2;
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
#pragma unroll 8
            for (uint32_t sl = 0; sl < 64; sl++) rank += lt3(xs[3 * sl], xs[3 * sl + 1], xs[3 * sl + 2], V0, V1, V2);
            __builtin_amdgcn_wave_barrier();
        }
        if (v && rank < count) row[rank] = j + T.index_base;
    }
    for (uint32_t p = m + lane; p < count; p += 64) row[p] = NONE;
    if (lane == 0 && cp) *cp = (uint8_t)min(m, 255u);
}

// One wave per query; af (may be NULL): the query's family, 0 -> T4, 1 -> T6 (kad_rt_closest_batch_dual).
__global__ __launch_bounds__(BLOCK) void rt_wave_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ af,
                                                        const uint8_t* __restrict__ targets, uint32_t q, uint32_t count,
                                                        uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    __shared__ uint64_t xs[BLOCK / 64][192];
    const uint32_t w = threadIdx.x >> 6, i = blockIdx.x * (BLOCK / 64) + w;
    if (i >= q) return;  // wave-uniform
    const DevTable& T = (af && af[i]) ? T6 : T4;
    const Target t = load_target(targets, i);
    uint32_t* row = out_idx + (size_t)i * count;
    uint8_t* cp = out_cnt ? out_cnt + i : nullptr;
    const uint32_t lane = threadIdx.x & 63u;
    if (T.B == 0) {  // an empty table: an empty result (routing_table.cpp:73)
        for (uint32_t p = lane; p < count; p += 64) row[p] = NONE;
        if (lane == 0 && cp) *cp = 0;
        return;
    }
    uint32_t lo, hi, good;
    wave_window(T.gcnt, T.B, locate_bucket(T, t), count, lo, hi, good);
    wave_rank_any(T, t, T.dir[lo].x & ~WIDE, T.dir[hi + 1].x & ~WIDE, good, count, row, cp, xs[w]);
}

// ---------------------------------------------------------------------------------------
// Window-line RoutingTable kernel (count <= 8; direct-mapped tables of uniform depth d,
// 1 <= d <= 43: the U(d) shape of the bench shards). The default kernel where the table has lines.
//
// A random gather on MI355X costs one 128-byte line whether 32 or 128 bytes of it are used, and
// wherever the table sits (tools/mb_line.py: ~34 G lines/s with the target read and row write,
// the same for 128 MB and 1 GB tables), so a query should touch exactly ONE line. Line b holds
// everything a query whose target lies in bucket b needs, for any count <= 8:
//
// * For count c <= 8 the window W(R_c) depends on b alone, and W(R_c) is inside W(R_8);
//   R_8 <= 2 unless the six buckets b-3 .. b+2 hold fewer than 8 good nodes.
// * Buckets of equal depth are dyadic: the XOR images of two of them are disjoint intervals
//   ordered by D(x) = prefix(x) XOR prefix(b) (the target has b's prefix), so the reference's
//   result is W(R_c)'s buckets in D order, each bucket's good nodes by XOR distance to the target.
// * Inside one bucket that order is the order of ID bits [d, d+21) XOR the target's bits [d, d+21),
//   unless two good nodes of the bucket share those 21 bits (the line is then marked defer).
//
// Line b, 32 dwords:
//   dw0      node index of the first node of W(R_8)'s lowest bucket (`base`)
//   dw1      G(r) for r = 0..2, the good nodes of W(r) (6 bits each, capped at 63) | whole(r) << (18+r)
//            | R_8 << 21 | S << 23 | defer << 31.  whole(r): W(r) is the whole table
//   dw2      round of the bucket of D rank j, 2 bits each (j < 6)
//   dw3      tie: 0, or one pair of stored nodes of one bucket sharing key21, valid << 31 | bn << 30 | p << 16 |
//            off_a << 8 | off_b (off_a < off_b; p = the first of the top 64 ID bits where they differ, bn = node
//            b's bit p). Their rank values differ only in off, so off_a ranks first; a target whose bit p is bn
//            is closer to node b, and the answer exchanges the two offsets.
//   dw4..27  slot s (s < S <= 24): jd << 29 | key21 << 8 | off. The good nodes of W(R_8) in
//            (D rank jd, node index) order, whole buckets only; off = node index - base (< 256)
//   others   0xFFFFFFFF
// A query's rank value of slot s is slot XOR (t21 << 8): (D rank, in-bucket distance, offset),
// distinct within a line. The 8 smallest values (three sorted groups of 8, two bitonic merges,
// min/max only) are the answer, provided the stored slots hold the first m = min(c, G(R_c)) of
// W(R_c)'s nodes; otherwise, and for marked lines or targets outside b's range (clamped to the
// first/last bucket), the query takes the wave-cooperative exact path (wave_exact).
// Reference semantics: routing_table.cpp:67-111 (window rounds, sorted insertion, truncation).
// ---------------------------------------------------------------------------------------
constexpr uint32_t WL_SLOTS = 24;
constexpr uint32_t WL_SLOT0 = 4;   // first slot dword
constexpr uint32_t WL_KBITS = 21;  // in-bucket key bits
constexpr uint32_t WL_DEFER = 0x80000000u;

__device__ __forceinline__ void cx(uint32_t& a, uint32_t& b) {
    const uint32_t lo = min(a, b);
    b = max(a, b);
    a = lo;
}

// Batcher's odd-even merge sort for 8 inputs (19 comparators; checked by the 0-1 principle in
// tests/test_networks.py, which parses this table).
constexpr int SORT8_LEN = 19;
__device__ constexpr uint8_t SORT8[SORT8_LEN][2] = {
    {0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}, {1, 2}, {5, 6},
    {0, 4}, {1, 5}, {2, 6}, {3, 7}, {2, 4}, {3, 5}, {1, 2}, {3, 4}, {5, 6}};

__device__ __forceinline__ void sort8(uint32_t* v) {
#pragma unroll
    for (int c = 0; c < SORT8_LEN; c++) cx(v[SORT8[c][0]], v[SORT8[c][1]]);
}

// a = the 8 smallest of (a, s), sorted; a and s sorted ascending on entry.
__device__ __forceinline__ void merge8(uint32_t* a, const uint32_t* s) {
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

__device__ __forceinline__ uint32_t dw(const uint4 (&L)[8], int k) {  // static k after unrolling
    const uint4& q = L[k >> 2];
    return (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
}

// The window-line answer of lane's query: target t in bucket b of T (lines present, 1 <= count <= 8).
// Returns true with o[0..8) (node indices + index_base, NONE from m on) and m = min(count, good
// nodes of W(R_c)), or false when the query needs the exact path (marked line, target outside b's
// range, too few stored slots). Contains a wave vote: call from uniform control flow, inactive lanes
// with act = false (they return false). The line's key21 tie (dw3), if any, is applied to the answer.
// ABL (timing ablations only, KAD_RT_KERNEL=wl_abl1|wl_abl2 in the KAD_ABLATIONS tools build; results
// wrong): 2 = no ranking.
template <int ABL>
__device__ __forceinline__ bool wl_answer(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                          uint32_t (&o)[8], uint32_t& m) {
    uint4 L[8];
    if (act) {
        const uint4* lp = T.wl + 8ull * b;
#pragma unroll
        for (int x = 0; x < 8; x++) L[x] = lp[x];
    } else {
#pragma unroll
        for (int x = 0; x < 8; x++) L[x] = make_uint4(NONE, NONE, NONE, NONE);
    }
    const uint32_t d = 64 - T.rshift;
    const uint32_t h = L[0].y, rounds = L[0].z;
    // R_c = the least r <= R_8 with G(r) >= c or W(r) = the whole table
    const uint32_t G0 = h & 63u, G1 = (h >> 6) & 63u, G2 = (h >> 12) & 63u, R8 = (h >> 21) & 3u, S = (h >> 23) & 31u;
    const uint32_t Rc = (G0 >= count || (h >> 18) & 1u) ? 0u : (G1 >= count || (h >> 19) & 1u) ? 1u : 2u;
    m = min(count, Rc == 0 ? G0 : Rc == 1 ? G1 : G2);
    const bool own = (t.hi >> T.rshift) == (T.rbase >> T.rshift) + b;  // target inside bucket b's range
    bool ex = !act || (h & WL_DEFER) || !own || (Rc == R8 && S < m);
    const uint32_t tx = (uint32_t)((t.hi << d) >> (64 - WL_KBITS)) << 8;
    uint32_t v[WL_SLOTS];
#pragma unroll
    for (int s = 0; s < (int)WL_SLOTS; s++) v[s] = dw(L, WL_SLOT0 + s) ^ tx;
    if (__any(!ex && Rc < R8)) {  // count < 8 with a smaller window: drop the later rounds' buckets
        uint32_t inc = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) inc |= (((rounds >> (2 * j)) & 3u) <= Rc ? 1u : 0u) << j;
        uint32_t have = 0;
#pragma unroll
        for (int s = 0; s < (int)WL_SLOTS; s++) {
            const bool in = (uint32_t)s < S && ((inc >> (v[s] >> 29)) & 1u);
            v[s] = in ? v[s] : NONE;
            have += in;
        }
        ex |= have < m;
    }
    if (ABL < 2) {
        sort8(v);
        sort8(v + 8);
        sort8(v + 16);
        merge8(v, v + 8);
        merge8(v, v + 16);
    }
    const uint32_t base = L[0].x + T.index_base, tie = L[0].w;
    uint32_t oa = NONE, ob = NONE;
    if ((tie >> 31) && ((t.hi >> (63 - ((tie >> 16) & 63u))) & 1u) == ((tie >> 30) & 1u)) {
        oa = (tie >> 8) & 255u;
        ob = tie & 255u;
    }
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint32_t x = v[j] & 255u, y = x == oa ? ob : x == ob ? oa : x;
        o[j] = (uint32_t)j < m ? base + y : NONE;
    }
    return !ex;
}

__device__ __forceinline__ void store_row8(uint32_t* row, const uint32_t (&o)[8], uint32_t count) {
    if (count == 8 && ((uintptr_t)row & 15u) == 0) {
        reinterpret_cast<uint4*>(row)[0] = make_uint4(o[0], o[1], o[2], o[3]);
        reinterpret_cast<uint4*>(row)[1] = make_uint4(o[4], o[5], o[6], o[7]);
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++)
            if ((uint32_t)j < count) row[j] = o[j];
    }
}

// The wave's count-8 rows through LDS, stored as two 1 KB runs of 16-byte non-temporal pieces at consecutive addresses
// (piece 64h + lane = half lane & 1 of the row of query 32h + lane / 2); only the rows of lanes with `st` are written
// (the others are left to their fallbacks). Needs i = blockIdx.x * BLOCK + threadIdx.x, count 8 and a 16-byte aligned
// out_idx; call from wave-uniform control flow. The headline's rows: 31.85 -> 31.0 us per 1M (profiles/r03/ab_ws_cr/).
__device__ __forceinline__ void store_rows8_wave(uint32_t* __restrict__ out_idx, uint32_t i, const uint32_t (&o)[8],
                                                 bool st) {
    __shared__ uint4 wrow[BLOCK / 64][128];
    const uint32_t lane = threadIdx.x & 63u, i0 = i - lane;
    uint4* R = wrow[threadIdx.x >> 6];
    R[2 * lane] = make_uint4(o[0], o[1], o[2], o[3]);
    R[2 * lane + 1] = make_uint4(o[4], o[5], o[6], o[7]);
    const uint64_t okm = __ballot(st);
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    u32x4_t* r = reinterpret_cast<u32x4_t*>(out_idx + (size_t)i0 * 8u);
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const uint4 u = R[64 * h + lane];
        if ((okm >> (32 * h + (lane >> 1))) & 1u) __builtin_nontemporal_store(u32x4_t{u.x, u.y, u.z, u.w}, r + 64 * h + lane);
    }
}

// ABL 1 = no exact path, 2 = also no ranking (timing ablations only). CR: count-8 rows as wave runs (store_rows8_wave;
// the launch path; the resident service keeps per-lane rows).
template <int ABL, bool CR = false>
__device__ __forceinline__ void rt_wl_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q,
                                                      uint32_t count, uint32_t* __restrict__ out_idx,
                                                      uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q && count > 0;
    if (i < q && count == 0 && out_cnt) out_cnt[i] = 0;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t = load_target(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t o[8], m;
    const bool ok = wl_answer<ABL>(T, t, b, count, act, o, m);
    if (CR && count == 8 && ((uintptr_t)out_idx & 15u) == 0) {  // kernel-uniform
        store_rows8_wave(out_idx, i, o, act && ok);
        if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    } else if (act && ok) {
        store_row8(out_idx + (size_t)i * count, o, count);
        if (out_cnt) out_cnt[i] = (uint8_t)m;
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    if (ABL == 0) exact_tail(T, t, act && !ok, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
template <int ABL>
__global__ __launch_bounds__(BLOCK) void rt_wl_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                      uint32_t count, uint32_t* __restrict__ out_idx,
                                                      uint8_t* __restrict__ out_cnt) {
    rt_wl_kernel_body<ABL, true>(T, targets, q, count, out_idx, out_cnt);
}

// The good nodes of bucket x in index order: fn(node index, key). Buckets of <= 32 nodes take their good
// mask from dir[x].y (current whenever a line builder runs) and load the keys 8 at a time, independently,
// so a builder thread waits for one round trip per 8 good nodes instead of two per node.
template <class F>
__device__ __forceinline__ void for_good(const uint64_t* key, const uint8_t* status, const uint2* dir, uint32_t x, F fn) {
    const uint2 a = dir[x];
    const uint32_t j0 = a.x & ~WIDE;
    if (!(a.x & WIDE)) {
        uint32_t m = a.y;
        while (m) {
            uint32_t pos[8];
            uint64_t kk[8];
            int c = 0;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                pos[u] = m ? (uint32_t)__builtin_ctz(m) : 0u;
                if (m) { m &= m - 1; c = u + 1; }
            }
#pragma unroll
            for (int u = 0; u < 8; u++) kk[u] = u < c ? key[j0 + pos[u]] : 0ull;
            for (int u = 0; u < c; u++) fn(j0 + pos[u], kk[u]);
        }
    } else {
        const uint32_t j1 = dir[x + 1].x & ~WIDE;
        for (uint32_t n = j0; n < j1; n++)
            if (status[n] & KAD_STATUS_GOOD) fn(n, key[n]);
    }
}

// The good-node count of bucket x (popcount of its mask; gcnt for wide buckets).
__device__ __forceinline__ uint32_t good_of(const uint2* dir, const uint32_t* gcnt, uint32_t x) {
    const uint2 a = dir[x];
    return (a.x & WIDE) ? gcnt[x] : (uint32_t)__popc(a.y);
}

// A line assembled in the thread's LDS row (odd stride: conflict-free), then stored as 16-byte pieces.
template <int W>
__device__ __forceinline__ void store_line(const uint32_t* L, uint32_t* dst) {
#pragma unroll
    for (int k = 0; k < W; k += 4)
        *reinterpret_cast<uint4*>(dst + k) = make_uint4(L[k], L[k + 1], L[k + 2], L[k + 3]);
}

// Window line b after a status change (or at table creation), assembled in L (an LDS row of 33 dwords) and
// stored (d = depth).
__device__ void wl_build_line(const uint64_t* key, const uint8_t* status, const uint2* dir, const uint32_t* gcnt,
                              uint32_t B, uint32_t d, uint64_t pre0, uint32_t* lines, uint32_t b, uint32_t* L) {
    for (int k = 0; k < 32; k++) L[k] = NONE;
    // R_8 and the per-round good counts (routing_table.cpp:89-104 closed form)
    uint32_t h = 0, R8 = 3, g = 0;
    for (uint32_t r = 0; r < 3; r++) {
        const uint32_t lo = b > r ? b - 1 - r : 0u, hi = min(B - 1, b + r);
        g += ring_good(gcnt, B, b, r);
        const bool whole = lo == 0 && hi == B - 1;
        h |= (min(g, 63u) << (6 * r)) | ((whole ? 1u : 0u) << (18 + r));
        if (R8 == 3 && (g >= 8 || whole)) R8 = r;
    }
    if (R8 == 3) {
        L[1] = WL_DEFER;
        L[3] = 0;
        store_line<32>(L, lines + 32ull * b);
        return;
    }
    const uint32_t lo = b > R8 ? b - 1 - R8 : 0u, hi = min(B - 1, b + R8), nb = hi - lo + 1;
    const uint32_t base = dir[lo].x & ~WIDE;
    uint32_t rounds = 0, S = 0, tie = 0;
    bool defer = false, full = false;
    for (uint32_t j = 0; j < nb; j++) {  // buckets in D order: the one whose D rank is j
        uint32_t x = lo;
        for (uint32_t y = lo; y <= hi; y++) {
            uint32_t rk = 0;
            for (uint32_t z = lo; z <= hi; z++) rk += ((pre0 + z) ^ (pre0 + b)) < ((pre0 + y) ^ (pre0 + b));
            if (rk == j) x = y;
        }
        rounds |= (x >= b ? x - b : b - 1 - x) << (2 * j);
        const uint32_t g = good_of(dir, gcnt, x);
        if (full || S + g > WL_SLOTS) { full = true; continue; }  // whole buckets only
        const uint32_t s0 = S;
        for_good(key, status, dir, x, [&](uint32_t n, uint64_t kn) {
            const uint32_t k21 = (uint32_t)((kn << d) >> (64 - WL_KBITS)), off = n - base;
            defer |= off > 255u;
            for (uint32_t s = s0; s < S; s++) {
                if (((L[WL_SLOT0 + s] >> 8) & ((1u << WL_KBITS) - 1)) != k21) continue;
                // one pair sharing key21 is resolved by the first bit p where the two keys differ (dw3);
                // a second pair, or keys equal in all 64 bits, defers the line
                const uint32_t oa = L[WL_SLOT0 + s] & 255u;
                const uint64_t x = kn ^ key[base + oa];
                if (tie || x == 0 || off > 255u) {
                    defer = true;
                } else {
                    const uint32_t p = (uint32_t)__builtin_clzll(x), bn = (uint32_t)(kn >> (63 - p)) & 1u;
                    tie = WL_DEFER | (bn << 30) | (p << 16) | (oa << 8) | (off & 255u);
                }
            }
            L[WL_SLOT0 + S] = (j << 29) | (k21 << 8) | (off & 255u);
            S++;
        });
    }
    L[0] = base;
    L[1] = h | (R8 << 21) | (S << 23) | (defer ? WL_DEFER : 0u);
    L[2] = rounds;
    L[3] = tie;
    store_line<32>(L, lines + 32ull * b);
}

// ---------------------------------------------------------------------------------------
// Short window lines (TF_WS): the count <= 8 line in 64 bytes, so a uniform table's lines take half the
// bytes (a 2^21-bucket shard: 134 MB, inside the 256 MiB Infinity Cache, instead of 268 MB) and a query's
// random gather is one 64-byte line. A short line is transcoded from the 128-byte line of the same bucket,
// as a 512-bit little-endian bit string:
//   [0, 32)    base (as the 128-byte line)
//   [32, 55)   G0 | G1 << 4 | G2 << 8 (G(r) capped at 15: only compared with counts <= 8) | whole(r) << 12
//              | R_8 << 15 | S << 17 (short slots stored: whole buckets, <= 19) | fallback << 22
//   [55, 67)   round of the k-th stored bucket, 2 bits each (k < 6)
//   [67, 504)  19 slots of 23 bits: start << 22 | key16 << 6 | off. start marks a slot that opens the next
//              stored bucket (D-rank order), key16 = the top 16 of the 21 key bits; unused slots are all
//              ones. fallback: the 128-byte line is deferred, a stored node has off >= 64, or two stored
//              nodes of one bucket share their 16 key bits.
// A query's rank value of slot s is (k << 22) | (slot's low 22 bits XOR t16 << 6), k = the number of start
// bits up to s: (stored-bucket rank, in-bucket distance, offset), distinct within a line unless marked. A
// query the short line cannot answer (fallback, or fewer stored slots than its m) reads the 128-byte line
// (wl_answer), and from there the exact path: results are those of the 128-byte line. The stored slots
// are a D-rank prefix of whole buckets of the 128-byte line's (buckets without good nodes store nothing
// and are skipped by k), so the 128-byte line's argument carries over: the m smallest stored values are
// W(R_c)'s first m nodes.
// ---------------------------------------------------------------------------------------
constexpr uint32_t WS_SLOTS = 19;
constexpr uint32_t WS_KBITS = 16;
constexpr uint32_t WS_SBITS = 23;  // slot bits
constexpr uint32_t WS_HDR = 32, WS_ROUNDS = 55, WS_SLOT0 = 67;

__device__ __forceinline__ uint32_t dw(const uint4 (&L)[4], int k) {  // static k after unrolling
    const uint4& q = L[k >> 2];
    return (k & 3) == 0 ? q.x : (k & 3) == 1 ? q.y : (k & 3) == 2 ? q.z : q.w;
}

// w (<= 32) bits at bit p of a short line held as 4 x uint4 (static p, w after unrolling)
__device__ __forceinline__ uint32_t ws_bits(const uint4 (&L)[4], int p, int w) {
    const int k = p >> 5, sh = p & 31;
    const uint32_t mask = w == 32 ? NONE : (1u << w) - 1u;
    if (sh + w <= 32) return (dw(L, k) >> sh) & mask;
    return (uint32_t)((((uint64_t)dw(L, k + 1) << 32) | dw(L, k)) >> sh) & mask;
}

__device__ __forceinline__ void put_bits(uint32_t* L, uint32_t p, uint32_t w, uint32_t v) {
    const uint32_t k = p >> 5, sh = p & 31;
    const uint64_t mask = ((1ull << w) - 1ull) << sh;
    uint64_t x = (uint64_t)L[k] | ((uint64_t)L[k + 1] << 32);
    x = (x & ~mask) | (((uint64_t)v << sh) & mask);
    L[k] = (uint32_t)x;
    L[k + 1] = (uint32_t)(x >> 32);
}

// Short line b transcoded from its 128-byte line W (an LDS row), assembled in L (an LDS row of 17 dwords).
__device__ void ws_build_line(const uint32_t* W, uint32_t* __restrict__ ws, uint32_t b, uint32_t* L) {
    const uint32_t h = W[1], rounds = W[2], S = (h >> 23) & 31u;
    bool fb = (h & WL_DEFER) != 0;
    // the longest whole-bucket prefix of the 128-byte line's slots that fits
    uint32_t keep = 0;
    for (uint32_t s = 0; s < S && s < WS_SLOTS; s++)
        if (s + 1 == S || (W[WL_SLOT0 + s + 1] >> 29) != (W[WL_SLOT0 + s] >> 29)) keep = s + 1;
    for (int k = 0; k < 17; k++) L[k] = NONE;
    constexpr uint32_t KSH = 8 + WL_KBITS - WS_KBITS;
    uint32_t nb = 0, rk = 0;
    for (uint32_t s = 0; s < keep; s++) {
        const uint32_t v = W[WL_SLOT0 + s], j = v >> 29, k16 = (v >> KSH) & 0xFFFFu, off = v & 255u;
        fb |= off >= 64u;
        for (uint32_t r = 0; r < s; r++) {
            const uint32_t u = W[WL_SLOT0 + r];
            fb |= (u >> 29) == j && ((u >> KSH) & 0xFFFFu) == k16;
        }
        const bool start = s == 0 || (W[WL_SLOT0 + s - 1] >> 29) != j;
        if (start) rk |= ((rounds >> (2 * j)) & 3u) << (2 * nb++);
        put_bits(L, WS_SLOT0 + WS_SBITS * s, WS_SBITS, (start ? 1u << 22 : 0u) | (k16 << 6) | off);
    }
    const uint32_t G0 = min(h & 63u, 15u), G1 = min((h >> 6) & 63u, 15u), G2 = min((h >> 12) & 63u, 15u);
    const uint32_t hw = G0 | (G1 << 4) | (G2 << 8) | (((h >> 18) & 7u) << 12) | (((h >> 21) & 3u) << 15) |
                        (keep << 17) | ((fb ? 1u : 0u) << 22);
    L[0] = W[0];
    put_bits(L, WS_HDR, 23, hw);
    put_bits(L, WS_ROUNDS, 12, rk);
    store_line<16>(L, ws + 16ull * b);
}

// Window lines, one thread per bucket: every bucket's line, or only the listed ones (sel: incremental status
// refresh), grid-stride (an incremental rebuild launches a capped grid). WS: the short line of each bucket is
// transcoded from the 128-byte line while it is still in the thread's LDS row.
template <bool WS>
__global__ __launch_bounds__(BLOCK) void wl_build_kernel(const uint64_t* key, const uint8_t* status, const uint2* dir,
                                                          const uint32_t* gcnt, uint32_t B, uint32_t d, uint64_t pre0,
                                                          uint32_t* lines, uint32_t* ws, LineSel sel) {
    __shared__ uint32_t lds[BLOCK][33];
    __shared__ uint32_t lds_s[WS ? BLOCK : 1][17];
    for (uint32_t j_ = blockIdx.x * BLOCK + threadIdx.x;; j_ += gridDim.x * BLOCK) {
        uint32_t b;
        if (!sel.pick(j_, B, b)) return;
        wl_build_line(key, status, dir, gcnt, B, d, pre0, lines, b, lds[threadIdx.x]);
        if (WS) ws_build_line(lds[threadIdx.x], ws, b, lds_s[WS ? threadIdx.x : 0]);
    }
}

// The short-line answer (same contract as wl_answer; the caller falls back to wl_answer when it fails).
// ABL 2 (timing ablation, tools build only; results wrong): no ranking.
template <int ABL>
__device__ __forceinline__ bool ws_answer(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                          uint32_t (&o)[8], uint32_t& m) {
    uint4 L[4];
    if (act) {
        const uint4* lp = T.ws + 4ull * b;
#pragma unroll
        for (int x = 0; x < 4; x++) L[x] = lp[x];
    } else {
#pragma unroll
        for (int x = 0; x < 4; x++) L[x] = make_uint4(NONE, NONE, NONE, NONE);
    }
    const uint32_t d = 64 - T.rshift;
    const uint32_t h = ws_bits(L, WS_HDR, 23), rounds = ws_bits(L, WS_ROUNDS, 12);
    const uint32_t G0 = h & 15u, G1 = (h >> 4) & 15u, G2 = (h >> 8) & 15u, R8 = (h >> 15) & 3u, S = (h >> 17) & 31u;
    const uint32_t Rc = (G0 >= count || (h >> 12) & 1u) ? 0u : (G1 >= count || (h >> 13) & 1u) ? 1u : 2u;
    m = min(count, Rc == 0 ? G0 : Rc == 1 ? G1 : G2);
    const bool own = (t.hi >> T.rshift) == (T.rbase >> T.rshift) + b;  // target inside bucket b's range
    bool ex = !act || ((h >> 22) & 1u) || !own || (Rc == R8 && S < m);
    const uint32_t tx = (uint32_t)((t.hi << d) >> (64 - WS_KBITS)) << 6;
    uint32_t v[WS_SLOTS], k = 0;
#pragma unroll
    for (int s = 0; s < (int)WS_SLOTS; s++) {
        const uint32_t x = ws_bits(L, WS_SLOT0 + WS_SBITS * s, WS_SBITS);
        k += x >> 22;
        v[s] = (k << 22) | ((x & 0x3FFFFFu) ^ tx);
    }
    if (__any(!ex && Rc < R8)) {  // count < 8 with a smaller window: drop the later rounds' buckets
        uint32_t inc = 0;
#pragma unroll
        for (int j = 0; j < 6; j++) inc |= (((rounds >> (2 * j)) & 3u) <= Rc ? 1u : 0u) << (j + 1);
        uint32_t have = 0;
#pragma unroll
        for (int s = 0; s < (int)WS_SLOTS; s++) {
            const bool in = (uint32_t)s < S && ((inc >> (v[s] >> 22)) & 1u);
            v[s] = in ? v[s] : NONE;
            have += in;
        }
        ex |= have < m;
    }
    if (ABL < 2) {
        sort8(v);
        sort8(v + 8);
        merge8(v, v + 8);
#pragma unroll
        for (int s = 16; s < (int)WS_SLOTS; s++) {  // insert the rest: one bubble pass each
            v[7] = min(v[7], v[s]);
#pragma unroll
            for (int j = 7; j > 0; j--) cx(v[j - 1], v[j]);
        }
    }
    const uint32_t base = L[0].x + T.index_base;
#pragma unroll
    for (int j = 0; j < 8; j++) o[j] = (uint32_t)j < m ? base + (v[j] & 63u) : NONE;
    return !ex;
}

// 8 waves per SIMD (<= 64 VGPRs): the gather is latency-bound, occupancy is what hides it.
// ABL 1 = no fallback and no exact path, 2 = also no ranking, 3 = fallback but no exact path (timing ablations
// only); 4 = path statistics: out_cnt = 100 + m for queries answered by the 128-byte line, 250 for the exact path;
// 5 = the exact path compiled in but never taken.
// NTS: the streams (targets in, rows out) with the non-temporal policy, so that they do not displace the line table
// from the Infinity Cache: 32.7 -> 31.8 us per 1M on the bench shard, 3 interleaved bench runs each
// (profiles/r03/ab_ws_nts/). The launch path's default; the service (rows into host memory) keeps the plain policy.
// CR (with NTS, count 8, 16-byte aligned rows): the wave's 64 rows leave through LDS as two 1 KB runs of 16-byte
// pieces at consecutive addresses (tools/mb_req.py: line + coalesced rows 27.8 against 29.4 us per 1M).
template <int ABL, bool NTS = false, bool CR = false>
__device__ __forceinline__ void rt_ws_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q,
                                                      uint32_t count, uint32_t* __restrict__ out_idx,
                                                      uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q && count > 0;
    if (i < q && count == 0 && out_cnt) out_cnt[i] = 0;
    // short lines exist only on direct-mapped tables, whose locate and line paths use the target's top 64
    // bits alone: the other 96 are loaded by the (rare) exact path
    Target t{};
    uint32_t b = 0;
    if (act) {
        t.hi = load_target_hi(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t o[8], m;
    const bool ok = ws_answer<ABL>(T, t, b, count, act, o, m);
    if (CR && count == 8 && ((uintptr_t)out_idx & 15u) == 0) {  // count: kernel-uniform, so the branch is too
        store_rows8_wave(out_idx, i, o, act && ok);
        if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    } else if (act && ok) {
        if (NTS && count == 8 && ((uintptr_t)out_idx & 15u) == 0) {
            u32x4_t* r = reinterpret_cast<u32x4_t*>(out_idx + (size_t)i * 8u);
            __builtin_nontemporal_store(u32x4_t{o[0], o[1], o[2], o[3]}, r);
            __builtin_nontemporal_store(u32x4_t{o[4], o[5], o[6], o[7]}, r + 1);
        } else {
            store_row8(out_idx + (size_t)i * count, o, count);
        }
        if (out_cnt) out_cnt[i] = (uint8_t)m;
    }
    bool need = (ABL == 0 || ABL >= 3) && act && !ok;
    if (__any(need)) {  // the 128-byte line of the (few) queries the short line cannot answer
        const bool ok2 = wl_answer<0>(T, t, b, count, need, o, m);
        if (need && ok2) {
            store_row8(out_idx + (size_t)i * count, o, count);
            if (out_cnt) out_cnt[i] = (uint8_t)(ABL == 4 ? 100 + m : m);
        }
        need = need && !ok2;
    }
    if (ABL == 0 || ABL == 4 || ABL == 5) {
        __shared__ uint64_t xs[BLOCK / 64][192];
        if (ABL == 5) need = need && T.n == 0xFFFFFFFFu;  // opaque to the compiler, false in practice
        if (__any(need)) {
            if (need) t = load_target(targets, i);
            exact_tail(T, t, need, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
        }
        if (ABL == 4 && need && out_cnt) out_cnt[i] = 250;
    }
}
template <int ABL, bool NTS = false, bool CR = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void rt_ws_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                      uint32_t count, uint32_t* __restrict__ out_idx,
                                                      uint8_t* __restrict__ out_cnt) {
    rt_ws_kernel_body<ABL, NTS, CR>(T, targets, q, count, out_idx, out_cnt);
}

// Count 8 with the row written packed for owner routing's way back (kad_rt_closest_batch_packed; KAD_ROUTE_PACKED_WORDS
// (8) = 3 words: a base index, then one byte per entry, index - base, 0xFF past the count): the short line's answer,
// else the 128-byte line's, else the exact path's (by the wave, into LDS), packed in the kernel, so that no row of 33
// bytes is written and read again. A row wider than 254 indices sets *escape and writes nothing: the caller answers
// that batch again unpacked.
// KEYS (kad_rt_closest_keys_packed, owner routing's key-only exchange): the batch is the targets' top 64 bits alone
// (8-byte keys, native order), which is all the short and 128-byte lines read; the exact path runs with the low 96
// bits taken as zero, exact unless two nodes of its window share their top 64 bits — then *tail is set and the caller
// answers the batch again from full targets (wave_rank).
template <bool KEYS = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void rt_ws_packed_kernel(
    DevTable T, const uint8_t* __restrict__ targets, uint32_t q, uint32_t* __restrict__ packed,
    uint32_t* __restrict__ escape, uint32_t* __restrict__ tail = nullptr) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t.hi = KEYS ? __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(targets) + i)
                    : load_target_hi(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t o[8], m;
    bool ok = ws_answer<0>(T, t, b, 8u, act, o, m);
    bool need = act && !ok;
    if (__any(need)) {  // the 128-byte line of the (few) queries the short line cannot answer
        uint32_t o2[8], m2;
        const bool ok2 = wl_answer<0>(T, t, b, 8u, need, o2, m2);
        if (need && ok2) {
#pragma unroll
            for (int j = 0; j < 8; j++) o[j] = o2[j];
            m = m2;
            ok = true;
        }
        need = need && !ok2;
    }
    if (__any(need)) {  // the exact path, one query at a time by the wave, its row in LDS
        __shared__ uint64_t xs[BLOCK / 64][192];
        __shared__ uint32_t xrow[BLOCK / 64][8];
        __shared__ uint8_t xcnt[BLOCK / 64];
        const uint32_t w = threadIdx.x >> 6, lane = threadIdx.x & 63u;
        if (need && !KEYS) t = load_target(targets, i);
        for (uint64_t mm = __ballot(need); mm; mm &= mm - 1) {
            const uint32_t l = (uint32_t)__builtin_ctzll(mm);
            Target u;
            u.hi = rdl64(t.hi, l);
            u.t2 = KEYS ? 0u : rdl(t.t2, l);
            u.t3 = KEYS ? 0u : rdl(t.t3, l);
            u.t4 = KEYS ? 0u : rdl(t.t4, l);
            wave_exact(T, u, 8u, xrow[w], &xcnt[w], xs[w], KEYS ? tail : nullptr);
            __builtin_amdgcn_wave_barrier();
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
            if (lane == l) {
#pragma unroll
                for (int j = 0; j < 8; j++) o[j] = xrow[w][j];
                m = xcnt[w];
                ok = true;
            }
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (!act) return;
    uint32_t lo = NONE, hi = 0;
#pragma unroll
    for (int j = 0; j < 8; j++)
        if ((uint32_t)j < m) {
            lo = min(lo, o[j]);
            hi = max(hi, o[j]);
        }
    if (!ok || (m && hi - lo > 254u)) {
        atomicOr(escape, 1u);
        return;
    }
    uint32_t w1 = 0, w2 = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        w1 |= ((uint32_t)j < m ? o[j] - lo : 255u) << (8 * j);
        w2 |= ((uint32_t)j + 4 < m ? o[j + 4] - lo : 255u) << (8 * j);
    }
    uint32_t* pr = packed + 3ull * i;
    __builtin_nontemporal_store(lo, pr);
    __builtin_nontemporal_store(w1, pr + 1);
    __builtin_nontemporal_store(w2, pr + 2);
}

// The count <= 8 line answer for kernels that serve other paths too (dual-family, shard): lanes with `ws`
// (their table has short lines) try the 64-byte line, lanes with `act` it did not answer read the 128-byte
// line. Same contract as wl_answer; call from uniform control flow.
__device__ __forceinline__ bool line8_answer(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                             bool ws, uint32_t (&o)[8], uint32_t& m) {
    bool ok = false;
    m = 0;
    if (__any(ws)) ok = ws_answer<0>(T, t, b, count, ws, o, m) && ws;
    const bool need = act && !ok;
    if (__any(need)) {
        uint32_t o2[8], m2;
        const bool ok2 = wl_answer<0>(T, t, b, count, need, o2, m2);
        if (need) {
#pragma unroll
            for (int j = 0; j < 8; j++) o[j] = o2[j];
            m = m2;
            ok = ok2;
        }
    }
    return ok;
}

// ---------------------------------------------------------------------------------------
// Window lines for 9 <= count <= 16 (TF_WL16): the same construction as the count <= 8 lines with
// R_16 <= 3 (windows of up to 8 buckets) and 29 slots, so a line is 32 dwords: one aligned 128-byte
// line per bucket, one random line gather per query (the 32-slot, 144-byte form took two):
//   dw0      base (first node of W(R_16)'s lowest bucket)
//   dw1      G(r) for r = 0..3 (5 bits each, capped at 31) | whole(r) << (20+r) | R_16 << 24 | S << 26 | defer << 31
//            (S = stored slots, whole buckets only, <= 29)
//   dw2      round of the bucket of D rank j, 2 bits each (j < 8) | stored D-rank mask << 16 | buckets in W(R_16) << 24
//   dw3..31  slots: jd << 29 | key21 << 8 | off
// Buckets are stored whole: first the D-rank prefix of W(R_16) holding its 16 closest good nodes, then the
// rest of W(R_16 - 1) (< 16 good nodes), then whatever fits.
// The 16 smallest of the 29 rank values (padded to 32 with NONE: two sorted groups of 16 by Batcher's
// network, one bitonic merge), restricted to the longest fully stored D-rank prefix of W(R_c), are the
// answer when that prefix holds at least m good nodes (checked; otherwise the query takes the exact path).
// ---------------------------------------------------------------------------------------
constexpr uint32_t WL16_SLOTS = 29, WL16_HDR = 3, WL16_STRIDE = 32;  // dwords
#ifndef WL16_P1
#define WL16_P1 16u
#endif

// A 16-input sorting network of 60 comparators in 10 layers (the best known size; one of those listed by B. Dobbelaere,
// "SorterHunter"), 3 fewer than Batcher's odd-even merge sort; checked by the 0-1 principle in tests/test_networks.py.
constexpr int SORT16_LEN = 60;
__device__ constexpr uint8_t SORT16[SORT16_LEN][2] = {
    {0, 13}, {1, 12}, {2, 15}, {3, 14}, {4, 8}, {5, 6}, {7, 11}, {9, 10},
    {0, 5}, {1, 7}, {2, 9}, {3, 4}, {6, 13}, {8, 14}, {10, 15}, {11, 12},
    {0, 1}, {2, 3}, {4, 5}, {6, 8}, {7, 9}, {10, 11}, {12, 13}, {14, 15},
    {0, 2}, {1, 3}, {4, 10}, {5, 11}, {6, 7}, {8, 9}, {12, 14}, {13, 15},
    {1, 2}, {3, 12}, {4, 6}, {5, 7}, {8, 10}, {9, 11}, {13, 14},
    {1, 4}, {2, 6}, {5, 8}, {7, 10}, {9, 13}, {11, 14},
    {2, 4}, {3, 6}, {9, 12}, {11, 13},
    {3, 5}, {6, 8}, {7, 9}, {10, 12},
    {3, 4}, {5, 6}, {7, 8}, {9, 10}, {11, 12},
    {6, 7}, {8, 9}};

__device__ __forceinline__ void sort16(uint32_t* v) {
#pragma unroll
    for (int c = 0; c < SORT16_LEN; c++) cx(v[SORT16[c][0]], v[SORT16[c][1]]);
}

// a = the 16 smallest of (a, s), sorted; a and s sorted ascending on entry.
__device__ __forceinline__ void merge16(uint32_t* a, const uint32_t* s) {
#pragma unroll
    for (int i = 0; i < 16; i++) a[i] = min(a[i], s[15 - i]);
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < 16; i++)
            if ((i & w) == 0) cx(a[i], a[i + w]);
}

__device__ __forceinline__ bool wl16_answer(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                            uint32_t (&o)[16], uint32_t& m) {
    uint32_t L[WL16_HDR + WL16_SLOTS];
    if (act) {
        const uint4* lp = T.wl16 + (WL16_STRIDE / 4) * (size_t)b;
#pragma unroll
        for (int x = 0; x < (int)(WL16_HDR + WL16_SLOTS) / 4; x++) {
            const uint4 q = lp[x];
            L[4 * x] = q.x; L[4 * x + 1] = q.y; L[4 * x + 2] = q.z; L[4 * x + 3] = q.w;
        }
    } else {
#pragma unroll
        for (int x = 0; x < (int)(WL16_HDR + WL16_SLOTS); x++) L[x] = NONE;
    }
    const uint32_t d = 64 - T.rshift;
    const uint32_t h = L[1], rounds = L[2] & 0xFFFFu, S = (h >> 26) & 31u, R16 = (h >> 24) & 3u;
    const uint32_t st = (L[2] >> 16) & 255u, nb = (L[2] >> 24) & 15u;
    uint32_t G[4];
#pragma unroll
    for (int r = 0; r < 4; r++) G[r] = (h >> (5 * r)) & 31u;
    uint32_t Rc = 3;
#pragma unroll
    for (int r = 3; r >= 0; r--)
        if (G[r] >= count || ((h >> (20 + r)) & 1u)) Rc = (uint32_t)r;
    m = min(count, Rc == 0 ? G[0] : Rc == 1 ? G[1] : Rc == 2 ? G[2] : G[3]);
    const bool own = (t.hi >> T.rshift) == (T.rbase >> T.rshift) + b;
    bool ex = !act || (h & WL_DEFER) || !own || Rc > R16 || (Rc == R16 && S < m);
    const uint32_t tx = (uint32_t)((t.hi << d) >> (64 - WL_KBITS)) << 8;
    uint32_t v[32];
#pragma unroll  // empty slots must stay last: with D rank 7 a real value can exceed NONE ^ tx
    for (int s = 0; s < 32; s++) v[s] = s < (int)WL16_SLOTS && (uint32_t)s < S ? L[WL16_HDR + s] ^ tx : NONE;
    // W(R_c)'s buckets (D ranks with round <= R_c); the answer is the first m good nodes of the longest D-rank
    // prefix of them that the line stores whole (a bucket of round R_16 may not have fit).
    uint32_t inc = 0;
#pragma unroll
    for (int j = 0; j < 8; j++) inc |= ((uint32_t)j < nb && ((rounds >> (2 * j)) & 3u) <= Rc ? 1u : 0u) << j;
    const uint32_t miss = inc & ~st;
    if (__any(!ex && (Rc < R16 || miss))) {  // drop the buckets outside that prefix
        const uint32_t lim = miss ? (uint32_t)__builtin_ctz(miss) : 8u;
        uint32_t have = 0;
#pragma unroll
        for (int s = 0; s < (int)WL16_SLOTS; s++) {
            const uint32_t j = v[s] >> 29;
            const bool in = (uint32_t)s < S && ((inc >> j) & 1u) && j < lim;
            v[s] = in ? v[s] : NONE;
            have += in;
        }
        ex |= have < m;
    }
    sort16(v);
    sort16(v + 16);
    merge16(v, v + 16);
    const uint32_t base = L[0] + T.index_base;
#pragma unroll
    for (int j = 0; j < 16; j++) o[j] = (uint32_t)j < m ? base + (v[j] & 255u) : NONE;
    return !ex;
}

// Row of up to 16 indices: 16-byte stores for count 16, 8-byte stores for even counts (SEARCH_NODES = 14).
__device__ __forceinline__ void store_row16(uint32_t* row, const uint32_t (&o)[16], uint32_t count) {
    if (count == 16 && ((uintptr_t)row & 15u) == 0) {
#pragma unroll
        for (int x = 0; x < 4; x++)
            reinterpret_cast<uint4*>(row)[x] = make_uint4(o[4 * x], o[4 * x + 1], o[4 * x + 2], o[4 * x + 3]);
    } else if ((count & 1u) == 0 && ((uintptr_t)row & 7u) == 0) {
#pragma unroll
        for (int x = 0; x < 8; x++)
            if ((uint32_t)(2 * x) < count) reinterpret_cast<uint2*>(row)[x] = make_uint2(o[2 * x], o[2 * x + 1]);
    } else {
#pragma unroll
        for (int j = 0; j < 16; j++)
            if ((uint32_t)j < count) row[j] = o[j];
    }
}

// The block's rows (count 9..16 or 17..32) leave through LDS as one contiguous run of 16-byte stores: per-lane
// rows of 36..128 bytes (a 56-byte stride for count 14) left every store instruction part-filling its lines. Rows
// whose lane takes the exact path (ok false) are skipped dword by dword; exact_tail writes them afterwards.
template <int MAXK>  // count in 4..MAXK: a 16-byte chunk spans at most two rows
__device__ __forceinline__ void store_rows_block(uint32_t* __restrict__ out_idx, uint32_t q, uint32_t count,
                                                 const uint32_t (&o)[MAXK], bool ok) {
    __shared__ uint32_t rows[BLOCK * MAXK];
    __shared__ uint32_t okm[BLOCK / 32];
    const uint32_t tid = threadIdx.x, q0 = blockIdx.x * BLOCK;
    if (tid < BLOCK / 32) okm[tid] = 0;
    __syncthreads();
    if (ok) atomicOr(&okm[tid >> 5], 1u << (tid & 31));
#pragma unroll
    for (int j = 0; j < MAXK; j++)
        if ((uint32_t)j < count) rows[tid * count + j] = o[j];
    __syncthreads();
    const uint32_t nq = min((uint32_t)BLOCK, q - q0), nw = nq * count;
    uint32_t* dst = out_idx + (size_t)q0 * count;  // 16-byte aligned: BLOCK * count * 4 is a multiple of 16
    for (uint32_t c = tid; 4 * c < nw; c += BLOCK) {
        const uint32_t w0 = 4 * c;
        const uint32_t r0 = w0 / count, r1 = min(w0 + 3, nw - 1) / count;
        const bool ok0 = (okm[r0 >> 5] >> (r0 & 31)) & 1u, ok1 = (okm[r1 >> 5] >> (r1 & 31)) & 1u;
        if (ok0 && ok1 && w0 + 4 <= nw && (((uintptr_t)out_idx & 15u) == 0)) {
            st_row4(dst + w0, rows[w0], rows[w0 + 1], rows[w0 + 2], rows[w0 + 3]);
        } else {
            for (uint32_t w = w0; w < min(w0 + 4, nw); w++) {
                const uint32_t r = w / count;
                if ((okm[r >> 5] >> (r & 31)) & 1u) st_row1(dst + w, rows[w]);
            }
        }
    }
}

__device__ bool wave_wl32(const DevTable& T, const Target& t, uint32_t b, uint32_t count, uint32_t lane, uint32_t* row,
                          uint8_t* cp);  // below, with the 32-count lines

// ABL 1 = no exact path (timing ablation only, KAD_RT_KERNEL=wl16_abl1; deferred rows are left unwritten); 3 = path
// statistics (wl16_stats: out_cnt 250 where the line could not answer).
template <int ABL>
__device__ __forceinline__ void rt_wl16_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t = load_target(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t o[16], m;
    bool ok = wl16_answer(T, t, b, count, act, o, m);
    if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    store_rows_block<16>(out_idx, q, count, o, act && ok);
    if (ABL == 1) return;
    if (ABL == 3) {  // path statistics (tools build): 250 = the 16-count line could not answer
        if (act && !ok && out_cnt) out_cnt[i] = 250;
        return;
    }
    // the queries the 16-count line cannot answer (its 29 slots could not hold both the count 14 and the count 16
    // D-rank prefixes, a deferred line): the 32-count line of the same bucket (58 slots) by the wave, one query at a
    // time, then the exact path
    bool need = act && !ok;
    if (T.flags & TF_WL32) {
        const uint32_t lane = threadIdx.x & 63u;
        for (uint64_t pm = __ballot(need); pm; pm &= pm - 1) {
            const uint32_t l = (uint32_t)__builtin_ctzll(pm);
            Target u;
            u.hi = rdl64(t.hi, l);
            u.t2 = rdl(t.t2, l);
            u.t3 = rdl(t.t3, l);
            u.t4 = rdl(t.t4, l);
            const uint32_t il = rdl(i, l);
            if (wave_wl32(T, u, rdl(b, l), count, lane, out_idx + (size_t)il * count, out_cnt ? out_cnt + il : nullptr) &&
                lane == l)
                need = false;
        }
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, need, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
template <int ABL>
__global__ __launch_bounds__(BLOCK) void rt_wl16_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    rt_wl16_kernel_body<ABL>(T, targets, q, count, out_idx, out_cnt);
}

// Window lines for counts 9..16 after a status change (or at creation): one thread per bucket.
__global__ __launch_bounds__(BLOCK) void wl16_build_kernel(const uint64_t* key, const uint8_t* status, const uint2* dir,
                                                            const uint32_t* gcnt, uint32_t B, uint32_t d, uint64_t pre0,
                                                            uint32_t* lines, LineSel sel) {
    __shared__ uint32_t lds[BLOCK][33];
    // one item per thread, grid-stride (an incremental rebuild launches a capped grid)
    for (uint32_t j_ = blockIdx.x * BLOCK + threadIdx.x;; j_ += gridDim.x * BLOCK) {
        uint32_t b;
        if (!sel.pick(j_, B, b)) return;
        [&] {
    uint32_t* L = lds[threadIdx.x];
    for (uint32_t k = 0; k < WL16_STRIDE; k++) L[k] = NONE;
    uint32_t h = 0, R = 4, g = 0, Gr[4];
    for (uint32_t r = 0; r < 4; r++) {
        const uint32_t lo = b > r ? b - 1 - r : 0u, hi = min(B - 1, b + r);
        g += ring_good(gcnt, B, b, r);
        Gr[r] = g;
        const bool whole = lo == 0 && hi == B - 1;
        h |= (min(g, 31u) << (5 * r)) | ((whole ? 1u : 0u) << (20 + r));
        if (R == 4 && (g >= 16 || whole)) R = r;
    }
    if (R == 4) {
        L[1] = WL_DEFER;
        store_line<32>(L, lines + (size_t)WL16_STRIDE * b);
        return;
    }
    const uint32_t lo = b > R ? b - 1 - R : 0u, hi = min(B - 1, b + R), nb = hi - lo + 1;
    const uint32_t base = dir[lo].x & ~WIDE;
    uint32_t rounds = 0, S = 0, st = 0, xj[8], gj[8];
    bool defer = false;
    for (uint32_t j = 0; j < nb; j++) {  // the bucket of D rank j and its round
        uint32_t x = lo;
        for (uint32_t y = lo; y <= hi; y++) {
            uint32_t rk = 0;
            for (uint32_t z = lo; z <= hi; z++) rk += ((pre0 + z) ^ (pre0 + b)) < ((pre0 + y) ^ (pre0 + b));
            if (rk == j) x = y;
        }
        xj[j] = x;
        gj[j] = good_of(dir, gcnt, x);
        rounds |= (x >= b ? x - b : b - 1 - x) << (2 * j);
    }
    // Whole buckets, in four passes: (0) the D-rank prefix of W(R_14) up to its 14th good node (count 14 =
    // SEARCH_NODES, dht.cpp:3354, the count the reference asks for); (1) the D-rank prefix of W(R_16) up to its
    // 16th good node (every count with R_c = R_16); (2) the rest of W(R_16 - 1), which holds < 16 good nodes (every
    // count with R_c < R_16); (3) whatever else fits, in D order.
    auto put = [&](uint32_t j) {
        if (((st >> j) & 1u) || S + gj[j] > WL16_SLOTS) return;
        st |= 1u << j;
        const uint32_t s0 = S;
        for_good(key, status, dir, xj[j], [&](uint32_t n, uint64_t kn) {
            const uint32_t k21 = (uint32_t)((kn << d) >> (64 - WL_KBITS)), off = n - base;
            defer |= off > 255u;
            for (uint32_t s = s0; s < S; s++) defer |= ((L[WL16_HDR + s] >> 8) & ((1u << WL_KBITS) - 1)) == k21;
            L[WL16_HDR + S] = (j << 29) | (k21 << 8) | (off & 255u);
            S++;
        });
    };
    uint32_t R14 = R;
    for (int r = (int)R; r >= 0; r--) {
        const uint32_t lo_r = b > (uint32_t)r ? b - 1 - r : 0u, hi_r = min(B - 1, b + r);
        if (Gr[r] >= 14u || (lo_r == 0 && hi_r == B - 1)) R14 = (uint32_t)r;
    }
    for (uint32_t j = 0, cum = 0; j < nb && cum < 14u; j++)
        if (((rounds >> (2 * j)) & 3u) <= R14) {
            put(j);
            cum += gj[j];
        }
    for (uint32_t j = 0, cum = 0; j < nb && cum < WL16_P1; j++) {
        put(j);
        cum += gj[j];
    }
    for (uint32_t j = 0; j < nb; j++)
        if (((rounds >> (2 * j)) & 3u) < R) put(j);
    for (uint32_t j = 0; j < nb; j++) put(j);
    L[0] = base;
    L[1] = h | (R << 24) | (S << 26) | (defer ? WL_DEFER : 0u);
    L[2] = rounds | (st << 16) | (nb << 24);
    store_line<32>(L, lines + (size_t)WL16_STRIDE * b);
        }();
    }
}

// ---------------------------------------------------------------------------------------
// Window lines for 17 <= count <= 32 (TF_WL32): the count <= 16 construction with R_32 <= 7
// (windows of up to 16 buckets, a 4-bit D rank) and 58 slots with 20-bit in-bucket keys. A line is
// 64 dwords (two 128-byte lines per bucket):
//   dw0      base (first node of W(R_32)'s lowest bucket)
//   dw1, 2   G(r) for r = 0..3 and 4..7, 8 bits each (clamped to 255)
//   dw3      whole(r) bits 0..7 | R_32 << 8 | S << 12 (stored slots, whole buckets only, <= 58) | defer << 31
//   dw4, 5   round of the bucket of D rank j, 3 bits each (j < 10 in dw4, 10..15 in dw5)
//   dw6..63  slots: jd << 28 | key20 << 8 | off
// A query ranks the 58 slot values (padded to 64): four sorted groups of 16 (Batcher), two bitonic joins into sorted
// 32s and one top-32 bitonic merge, min/max only. (Ranking only slots 0..47 when no lane masks rounds, valid with at
// most 16 good nodes per bucket, measured slower: 120 against 111 us per 1M queries.) As for the 16-slot lines the answer is exact when the slots kept (those of W(R_c)'s buckets)
// number at least m = min(c, G(R_c)): the slots hold whole buckets in D order, so those of W(R_c) are its
// first buckets in D order.
// ---------------------------------------------------------------------------------------
constexpr uint32_t WL32_SLOTS = 58, WL32_HDR = 6, WL32_STRIDE = 64, WL32_KBITS = 20;  // dwords / bits

// a[0..2H) sorted from its two sorted halves: one compare-exchange rank against the reversed upper
// half splits it into two bitonic halves (lows, highs), then a half-cleaner cascade on each.
template <int H>
__device__ __forceinline__ void join_sorted(uint32_t* a) {
#pragma unroll
    for (int i = 0; i < H; i++) cx(a[i], a[2 * H - 1 - i]);
#pragma unroll
    for (int w = H / 2; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < 2 * H; i++)
            if ((i & w) == 0) cx(a[i], a[i + w]);
}

// a = the 32 smallest of (a, s), sorted; a and s sorted ascending on entry.
__device__ __forceinline__ void merge32(uint32_t* a, const uint32_t* s) {
#pragma unroll
    for (int i = 0; i < 32; i++) a[i] = min(a[i], s[31 - i]);
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < 32; i++)
            if ((i & w) == 0) cx(a[i], a[i + w]);
}

__device__ __forceinline__ bool wl32_answer(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                            uint32_t (&o)[32], uint32_t& m) {
    uint32_t L[WL32_STRIDE], v[64];
    if (act) {
        const uint4* lp = T.wl32 + (WL32_STRIDE / 4) * (size_t)b;
#pragma unroll
        for (int x = 0; x < (int)WL32_STRIDE / 4; x++) {
            const uint4 u = lp[x];
            L[4 * x] = u.x; L[4 * x + 1] = u.y; L[4 * x + 2] = u.z; L[4 * x + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int x = 0; x < (int)WL32_STRIDE; x++) L[x] = NONE;
    }
    const uint32_t* H = L;
    const uint32_t d = 64 - T.rshift;
    const uint32_t h = H[3], S = (h >> 12) & 127u, R = (h >> 8) & 15u;
    uint32_t Rc = 8, Gc = 0;
#pragma unroll
    for (int r = 7; r >= 0; r--) {
        const uint32_t g = (H[1 + (r >> 2)] >> (8 * (r & 3))) & 255u;
        if (g >= count || ((h >> r) & 1u)) { Rc = (uint32_t)r; Gc = g; }
    }
    m = min(count, Gc);
    const bool own = (t.hi >> T.rshift) == (T.rbase >> T.rshift) + b;
    bool ex = !act || (h & WL_DEFER) || !own || Rc > R;
    const uint32_t tx = (uint32_t)((t.hi << d) >> (64 - WL32_KBITS)) << 8;
#pragma unroll  // empty slots stay NONE (a real value of D rank 15 can exceed NONE ^ tx)
    for (int s = 0; s < 64; s++) {
        const int li = s < (int)WL32_SLOTS ? (int)WL32_HDR + s : 0;
        v[s] = s < (int)WL32_SLOTS && (uint32_t)s < S ? L[li] ^ tx : NONE;
    }
    uint32_t have = S;
    if (__any(!ex && Rc < R)) {  // a smaller window: drop the later rounds' buckets
        uint32_t inc = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t rj = j < 10 ? (H[4] >> (3 * j)) & 7u : (H[5] >> (3 * (j - 10))) & 7u;
            inc |= (rj <= Rc ? 1u : 0u) << j;
        }
        have = 0;
#pragma unroll
        for (int s = 0; s < (int)WL32_SLOTS; s++) {
            const bool in = (uint32_t)s < S && ((inc >> (v[s] >> 28)) & 1u);
            v[s] = in ? v[s] : NONE;
            have += in;
        }
    }
    sort16(v);
    sort16(v + 16);
    sort16(v + 32);
    sort16(v + 48);
    join_sorted<16>(v);
    join_sorted<16>(v + 32);
    merge32(v, v + 32);
    ex |= have < m;
    const uint32_t base = H[0] + T.index_base;
#pragma unroll
    for (int j = 0; j < 32; j++) o[j] = (uint32_t)j < m ? base + (v[j] & 255u) : NONE;
    return !ex;
}

// Row of up to 32 indices: 16-byte stores for counts divisible by 4, 8-byte stores for even counts.
// One query of count <= 32 by the whole wave from its bucket's 32-count line (wave-uniform b and t): lane s holds slot
// s (the rounds beyond R_c masked), one 64-lane bitonic sort, lanes < count write the row. False when the line cannot
// answer (deferred, clamped target, R_c > R_32, fewer stored nodes than m): the caller takes the exact path.
__device__ bool wave_wl32(const DevTable& T, const Target& t, uint32_t b, uint32_t count, uint32_t lane, uint32_t* row,
                          uint8_t* cp) {
    const uint32_t* L = reinterpret_cast<const uint32_t*>(T.wl32) + (size_t)WL32_STRIDE * b;
    const uint32_t h = L[3], S = (h >> 12) & 127u, R = (h >> 8) & 15u;
    uint32_t Rc = 8, Gc = 0;
    for (int r = 7; r >= 0; r--) {
        const uint32_t g = (L[1 + (r >> 2)] >> (8 * (r & 3))) & 255u;
        if (g >= count || ((h >> r) & 1u)) { Rc = (uint32_t)r; Gc = g; }
    }
    const uint32_t m = min(count, Gc);
    const bool own = (t.hi >> T.rshift) == (T.rbase >> T.rshift) + b;
    if ((h & WL_DEFER) || !own || Rc > R) return false;
    const uint32_t tx = (uint32_t)((t.hi << (64 - T.rshift)) >> (64 - WL32_KBITS)) << 8;
    uint32_t v = NONE;
    bool in = false;
    if (lane < WL32_SLOTS && lane < S) {
        const uint32_t w = L[WL32_HDR + lane], j = w >> 28;
        const uint32_t rj = j < 10 ? (L[4] >> (3 * j)) & 7u : (L[5] >> (3 * (j - 10))) & 7u;
        in = rj <= Rc;
        v = in ? w ^ tx : NONE;
    }
    if ((uint32_t)__popcll(__ballot(in)) < m) return false;
#pragma unroll
    for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            const uint32_t o = (uint32_t)__shfl_xor((int)v, (int)j, 64);
            v = (((lane & j) == 0) == ((lane & k) == 0)) ? min(v, o) : max(v, o);
        }
    if (lane < count) row[lane] = lane < m ? L[0] + T.index_base + (v & 255u) : NONE;
    if (lane == 0 && cp) *cp = (uint8_t)m;
    return true;
}

__device__ __forceinline__ void store_row32(uint32_t* row, const uint32_t (&o)[32], uint32_t count) {
    if ((count & 3u) == 0 && ((uintptr_t)row & 15u) == 0) {
#pragma unroll
        for (int x = 0; x < 8; x++)
            if ((uint32_t)(4 * x) < count)
                reinterpret_cast<uint4*>(row)[x] = make_uint4(o[4 * x], o[4 * x + 1], o[4 * x + 2], o[4 * x + 3]);
    } else if ((count & 1u) == 0 && ((uintptr_t)row & 7u) == 0) {
#pragma unroll
        for (int x = 0; x < 16; x++)
            if ((uint32_t)(2 * x) < count) reinterpret_cast<uint2*>(row)[x] = make_uint2(o[2 * x], o[2 * x + 1]);
    } else {
#pragma unroll
        for (int j = 0; j < 32; j++)
            if ((uint32_t)j < count) row[j] = o[j];
    }
}

__device__ __forceinline__ void rt_wl32_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t = load_target(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t o[32], m;
    const bool ok = wl32_answer(T, t, b, count, act, o, m);
    if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    store_rows_block<32>(out_idx, q, count, o, act && ok);
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, act && !ok, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
__global__ __launch_bounds__(BLOCK) void rt_wl32_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    rt_wl32_kernel_body(T, targets, q, count, out_idx, out_cnt);
}

// ---------------------------------------------------------------------------------------
// Counts 17..32 with FOUR lanes per query (rt_wl32q_kernel, the default for TF_WL32). The one-lane form
// ranks 58 slots in 151 VGPRs (three waves per SIMD) and stalls on its two line loads; here the quad loads
// the 256-byte line as four 64-byte pieces (lane p: dwords 16x + 4p .. +3, x = 0..3: each instruction one
// contiguous 64-byte segment per quad), each lane sorts its 16 slot values, and three cross-lane bitonic
// steps over DPP quad permutes give the top 32 (lanes 0 and 1: ranks 0..15 and 16..31):
//   B  lanes (0,1) and (2,3): half-cleaner of A ++ reverse(B) (element i against the partner's 15 - i; the
//      high lane keeps the max at its index j = position 31 - j, still bitonic), then 8, 4, 2, 1 in-lane:
//      P0 = lanes 0,1 ascending, P1 = lanes 2,3 ascending
//   C  Q[i] = min(P0[i], P1[31 - i]): lane 0 against lane 3, lane 1 against lane 2 (xor 3, element 15 - i):
//      the 32 smallest, bitonic
//   D  half-cleaner 16 across lanes 0 and 1, then 8, 4, 2, 1 in-lane.
// The values, masks and fallbacks are wl32_answer's, so the rows are identical.
// ---------------------------------------------------------------------------------------
// qdpp0: the same permute with old = 0, which the compiler folds into a following v_min (v_min_u32_dpp)
template <int CTRL>
__device__ __forceinline__ uint32_t qdpp0(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ uint32_t qdpp(uint32_t v) {
    // every row and bank enabled and quad_perm always names a lane of the quad, so the old value is never read:
    // mov_dpp leaves it undefined (no v_mov to initialise it before every permute)
    return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, false);
}
constexpr int QP_X1 = 0xB1, QP_X2 = 0x4E, QP_X3 = 0x1B, QP_B0 = 0x00, QP_B1 = 0x55;  // quad_perm encodings

// element i against the quad partner's element (REV ? 15 - i : i); the low lane keeps the min, the other the max:
// med3(v, w, 0) = min, med3(v, w, ~0) = max, one v_med3_u32 instead of min, max and a select
template <int CTRL, bool REV>
__device__ __forceinline__ void quad_exchange(uint32_t (&v)[16], bool low) {
    uint32_t w[16];
    const uint32_t c = low ? 0u : 0xFFFFFFFFu;
#pragma unroll
    for (int i = 0; i < 16; i++) w[i] = (CTRL == QP_X3 ? qdpp0<CTRL>(v[REV ? 15 - i : i]) : qdpp<CTRL>(v[REV ? 15 - i : i]));
#pragma unroll
    for (int i = 0; i < 16; i++) v[i] = max(min(v[i], w[i]), min(max(v[i], w[i]), c));
}

// a bitonic 16 in one lane, sorted ascending by half-cleaners 8, 4, 2, 1
__device__ __forceinline__ void clean16(uint32_t (&v)[16]) {
#pragma unroll
    for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
        for (int i = 0; i < 16; i++)
            if ((i & w) == 0) cx(v[i], v[i + w]);
}

// A quad lane's part of its query's row (entries r0 .. r0 + 15): node index base + offset, NONE from m on. When every
// row of the wave that is stored is full (m == count), the entries from count on are never stored: no selects.
__device__ __forceinline__ void quad_row(const uint32_t (&v)[16], uint32_t r0, uint32_t bi, uint32_t m, uint32_t count,
                                         bool stored, uint32_t (&o)[16]) {
    if (__all(m == count || !stored)) {
#pragma unroll
        for (int k = 0; k < 16; k++) o[k] = bi + (v[k] & 255u);
    } else {
#pragma unroll
        for (int k = 0; k < 16; k++) o[k] = r0 + k < m ? bi + (v[k] & 255u) : NONE;
    }
}

// RANK false: timing ablation only (the values unranked; results wrong). LOAD_ALL: the table has the line set, so
// lanes without a query load bucket b's line too (b = 0 for them; their answer is never stored) instead of filling
// the registers with NONE under a branch.
template <bool RANK = true, bool LOAD_ALL = false>
__device__ __forceinline__ bool wl32_answer4(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                             uint32_t p, uint32_t (&v)[16], uint32_t& m, uint32_t& base) {
    uint32_t L[16];
    if (LOAD_ALL || act) {
        const uint4* lp = T.wl32 + (WL32_STRIDE / 4) * (size_t)b;
#pragma unroll
        for (int x = 0; x < 4; x++) {
            const uint4 u = lp[4 * x + p];
            L[4 * x] = u.x; L[4 * x + 1] = u.y; L[4 * x + 2] = u.z; L[4 * x + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int x = 0; x < 16; x++) L[x] = NONE;
    }
    // the header: dwords 0..3 are lane 0's L[0..3], dwords 4, 5 lane 1's L[0], L[1]
    const uint32_t h = qdpp<QP_B0>(L[3]), g03 = qdpp<QP_B0>(L[1]), g47 = qdpp<QP_B0>(L[2]);
    const uint32_t r04 = qdpp<QP_B1>(L[0]), r15 = qdpp<QP_B1>(L[1]);
    base = qdpp<QP_B0>(L[0]);
    const uint32_t S = (h >> 12) & 127u, R = (h >> 8) & 15u;
    uint32_t Rc = 8, Gc = 0;
#pragma unroll
    for (int r = 7; r >= 0; r--) {
        const uint32_t g = ((r < 4 ? g03 : g47) >> (8 * (r & 3))) & 255u;
        if (g >= count || ((h >> r) & 1u)) { Rc = (uint32_t)r; Gc = g; }
    }
    m = min(count, Gc);
    const bool own = (t.hi >> T.rshift) == (T.rbase >> T.rshift) + b;
    bool ex = !act || (h & WL_DEFER) || !own || Rc > R;
    const uint32_t tx = (uint32_t)((t.hi << (64 - T.rshift)) >> (64 - WL32_KBITS)) << 8;
    const bool mask = __any(!ex && Rc < R);  // a smaller window: drop the later rounds' buckets
    uint32_t inc = ~0u;
    if (mask) {
        inc = 0;
#pragma unroll
        for (int j = 0; j < 16; j++) {
            const uint32_t rj = j < 10 ? (r04 >> (3 * j)) & 7u : (r15 >> (3 * (j - 10))) & 7u;
            inc |= (rj <= Rc ? 1u : 0u) << j;
        }
    }
    uint32_t have = S;  // every stored slot is in unless a smaller window masks the later rounds' buckets
    if (mask) {
        have = 0;
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const uint32_t s = 16u * (e >> 2) + 4u * p + (e & 3) - WL32_HDR;  // header dwords wrap to > S
            const bool in = s < S && ((inc >> (L[e] >> 28)) & 1u);
            v[e] = in ? L[e] ^ tx : NONE;  // empty slots stay NONE
            have += in;
        }
        have += qdpp<QP_X1>(have);
        have += qdpp<QP_X2>(have);
    } else {
#pragma unroll
        for (int e = 0; e < 16; e++) {
            const uint32_t s = 16u * (e >> 2) + 4u * p + (e & 3) - WL32_HDR;
            v[e] = s < S ? L[e] ^ tx : NONE;
        }
    }
    const bool low = (p & 1u) == 0;
    if (RANK) {
        sort16(v);
        quad_exchange<QP_X1, true>(v, low);
        clean16(v);
        quad_exchange<QP_X3, true>(v, true);
        quad_exchange<QP_X1, false>(v, low);
        clean16(v);
    }
    ex |= have < m;
    return !ex;
}

// The rows of a block's BLOCK / 4 quad-form queries (lanes 0 and 1 of a quad hold entries [0, 16) and
// [16, 32)), staged in LDS and stored as coalesced 16-byte pieces, as store_rows_block.
__device__ __forceinline__ void store_rows_quad(uint32_t* __restrict__ out_idx, uint32_t q, uint32_t count,
                                                const uint32_t (&o)[16], bool ok, uint32_t p) {
    constexpr uint32_t NQ = BLOCK / 4;
    __shared__ uint32_t rows[NQ * 32];
    __shared__ uint32_t okm[NQ / 32];
    const uint32_t tid = threadIdx.x, ql = tid >> 2, q0 = blockIdx.x * NQ;
    if (tid < NQ / 32) okm[tid] = 0;
    __syncthreads();
    if (ok && p == 0) atomicOr(&okm[ql >> 5], 1u << (ql & 31));
    if (p < 2)
#pragma unroll
        for (int k = 0; k < 16; k++)
            if (16u * p + k < count) rows[ql * count + 16u * p + k] = o[k];
    __syncthreads();
    const uint32_t nq = min(NQ, q - q0), nw = nq * count;
    uint32_t* dst = out_idx + (size_t)q0 * count;  // 16-byte aligned: NQ * count * 4 is a multiple of 16
    for (uint32_t c = tid; 4 * c < nw; c += BLOCK) {
        const uint32_t w0 = 4 * c;
        const uint32_t ra = w0 / count, rb = min(w0 + 3, nw - 1) / count;
        const bool oka = (okm[ra >> 5] >> (ra & 31)) & 1u, okb = (okm[rb >> 5] >> (rb & 31)) & 1u;
        if (oka && okb && w0 + 4 <= nw && (((uintptr_t)out_idx & 15u) == 0)) {
            st_row4(dst + w0, rows[w0], rows[w0 + 1], rows[w0 + 2], rows[w0 + 3]);
        } else {
            for (uint32_t w = w0; w < min(w0 + 4, nw); w++) {
                const uint32_t r = w / count;
                if ((okm[r >> 5] >> (r & 31)) & 1u) st_row1(dst + w, rows[w]);
            }
        }
    }
}

// QS: the row leaves through a per-quad LDS row, lane p storing entries [4p, 4p+4) and [16+4p, 20+4p) (16-byte pieces,
// 64 contiguous bytes per quad and instruction) or, for rows that are not 16-byte aligned, entry 4j+p in instruction j
// (16 contiguous bytes per quad and instruction); no block barrier. !QS: lanes 0 and 1 store their 16 entries from
// registers (aligned rows) or the block's rows go through store_rows_quad.
template <int ABL, bool QS>
__global__ __launch_bounds__(BLOCK) void rt_wl32q_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                         uint32_t count, uint32_t* __restrict__ out_idx,
                                                         uint8_t* __restrict__ out_cnt) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x, i = g >> 2, p = g & 3u;
    const bool act = i < q;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t = load_target(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t v[16], m, base;
    const bool ok = wl32_answer4<ABL == 0, true>(T, t, b, count, act, p, v, m, base);  // launched on TF_WL32 tables
    const uint32_t r0 = 16u * (p & 1u), bi = base + T.index_base;
    uint32_t o[16];
    quad_row(v, r0, bi, m, count, act && ok, o);
    if (act && ok && p == 0 && out_cnt) out_cnt[i] = (uint8_t)m;
    if (QS) {
        __shared__ uint4 qrow[BLOCK / 4][9];  // per quad: 32 entries + a 16-byte pad
        uint32_t* R = reinterpret_cast<uint32_t*>(qrow[threadIdx.x >> 2]);
        if (p < 2u) {
#pragma unroll
            for (int x = 0; x < 4; x++)
                reinterpret_cast<uint4*>(R + 16u * p)[x] = make_uint4(o[4 * x], o[4 * x + 1], o[4 * x + 2], o[4 * x + 3]);
        }
        __builtin_amdgcn_wave_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_wave_barrier();
        if (act && ok) {
            uint32_t* row = out_idx + (size_t)i * count;
            if ((count & 3u) == 0 && ((uintptr_t)out_idx & 15u) == 0) {
#pragma unroll
                for (int h = 0; h < 2; h++)
                    if (16u * h + 4u * p < count)
                        st_row4(row + 16 * h + 4 * p, R[16 * h + 4 * p], R[16 * h + 4 * p + 1], R[16 * h + 4 * p + 2],
                                R[16 * h + 4 * p + 3]);
            } else {
#pragma unroll
                for (int j = 0; j < 8; j++)
                    if (4u * j + p < count) st_row1(row + 4 * j + p, R[4 * j + p]);
            }
        }
    } else if ((count & 3u) == 0 && ((uintptr_t)out_idx & 15u) == 0) {  // lanes 0 and 1 store 16-byte pieces
        if (act && ok && p < 2u) {
            uint4* row = reinterpret_cast<uint4*>(out_idx + (size_t)i * count + r0);
#pragma unroll
            for (int x = 0; x < 4; x++)
                if (r0 + 4 * x < count) row[x] = make_uint4(o[4 * x], o[4 * x + 1], o[4 * x + 2], o[4 * x + 3]);
        }
    } else {  // staged through LDS (block-uniform branch)
        store_rows_quad(out_idx, q, count, o, act && ok, p);
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, act && !ok && p == 0u, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}

// Window lines for counts 17..32 after a status change (or at creation): one thread per bucket.
// The window's buckets are put in D order by rank (O(buckets^2), at most 16 buckets).
__global__ __launch_bounds__(BLOCK) void wl32_build_kernel(const uint64_t* key, const uint8_t* status, const uint2* dir,
                                                            const uint32_t* gcnt, uint32_t B, uint32_t d, uint64_t pre0,
                                                            uint32_t* lines, LineSel sel) {
    __shared__ uint32_t lds[BLOCK][WL32_STRIDE + 1];
    // one item per thread, grid-stride (an incremental rebuild launches a capped grid)
    for (uint32_t j_ = blockIdx.x * BLOCK + threadIdx.x;; j_ += gridDim.x * BLOCK) {
        uint32_t b;
        if (!sel.pick(j_, B, b)) return;
        [&] {
    uint32_t* L = lds[threadIdx.x];
    for (uint32_t k = 0; k < WL32_STRIDE; k++) L[k] = NONE;
    uint32_t g01 = 0, g23 = 0, whole = 0, R = 8, gs = 0;
    for (uint32_t r = 0; r < 8; r++) {
        const uint32_t lo = b > r ? b - 1 - r : 0u, hi = min(B - 1, b + r);
        gs += ring_good(gcnt, B, b, r);
        const uint32_t g = min(gs, 255u);
        const bool w = lo == 0 && hi == B - 1;
        if (r < 4) g01 |= g << (8 * r); else g23 |= g << (8 * (r - 4));
        whole |= (w ? 1u : 0u) << r;
        if (R == 8 && (g >= 32 || w)) R = r;
    }
    if (R == 8) {
        L[3] = WL_DEFER;
        store_line<WL32_STRIDE>(L, lines + (size_t)WL32_STRIDE * b);
        return;
    }
    const uint32_t lo = b > R ? b - 1 - R : 0u, hi = min(B - 1, b + R), nb = hi - lo + 1;
    uint32_t ord[16];
    for (uint32_t y = lo; y <= hi; y++) {
        uint32_t rk = 0;
        for (uint32_t z = lo; z <= hi; z++) rk += ((pre0 + z) ^ (pre0 + b)) < ((pre0 + y) ^ (pre0 + b));
        ord[rk] = y;
    }
    const uint32_t base = dir[lo].x & ~WIDE;
    uint32_t r04 = 0, r15 = 0, S = 0;
    bool defer = false, full = false;
    for (uint32_t j = 0; j < nb; j++) {
        const uint32_t x = ord[j];
        const uint32_t rd = x >= b ? x - b : b - 1 - x;
        if (j < 10) r04 |= rd << (3 * j); else r15 |= rd << (3 * (j - 10));
        const uint32_t g = good_of(dir, gcnt, x);
        if (full || S + g > WL32_SLOTS) { full = true; continue; }  // whole buckets only
        const uint32_t s0 = S;
        for_good(key, status, dir, x, [&](uint32_t n, uint64_t kn) {
            const uint32_t k20 = (uint32_t)((kn << d) >> (64 - WL32_KBITS)), off = n - base;
            defer |= off > 255u;
            for (uint32_t s = s0; s < S; s++)
                defer |= ((L[WL32_HDR + s] >> 8) & ((1u << WL32_KBITS) - 1)) == k20;
            L[WL32_HDR + S] = (j << 28) | (k20 << 8) | (off & 255u);
            S++;
        });
    }
    L[0] = base;
    L[1] = g01;
    L[2] = g23;
    L[3] = whole | (R << 8) | (S << 12) | (defer ? WL_DEFER : 0u);
    L[4] = r04;
    L[5] = r15;
    store_line<WL32_STRIDE>(L, lines + (size_t)WL32_STRIDE * b);
        }();
    }
}

// ---------------------------------------------------------------------------------------
// General window lines (TF_GL / TF_GL32): one line per bucket for tables of ANY bucket shape -- the
// reference split policy (dht.cpp:903-934), per-peer K tables, shards -- where the uniform-depth lines
// above do not apply. The bucket of the target comes from the locate radix (locate_bucket).
//
// Every ID of the window W(R) = [lo, hi] lies in [first_lo, end) (end = first_{hi+1}, or 2^160 after the
// last bucket), and so does every target of bucket b (except a target below the first bucket, which
// findBucket clamps to bucket 0: exact path). All of them share that range's common prefix of cp bits,
// so the XOR distance of two window nodes to the target compares like their ID bits [cp, cp+24) XOR the
// target's, unless two stored nodes agree on those 24 bits (the line is then marked defer). A slot is
// key24 << 8 | off (off = node index - base < 256); a query XORs every slot with t24 << 8 and keeps the
// smallest: (distance, offset) order, no bucket ranks needed.
//
// Which nodes a line stores: all good nodes of W(R) when they fit; otherwise whole buckets in D order
// (the order of their XOR images, first_c ^ first_b), as the uniform lines do. That order holds for every
// target of b unless two window buckets first differ at a bit >= b's depth (or b is not dyadic): such a
// line is marked defer when it had to truncate. Slots are placed ring by ring (W(0), then the buckets
// added by round 1, ...), so the stored nodes of W(r) are exactly the first S_r slots: a count with a
// smaller window R_c masks the slots from S_{R_c} on, and the answer is exact when S_{R_c} >= m.
//
// GL (count <= 8, 32 dwords):                      GL32 (counts 9..32, 64 dwords):
//   dw0  base                                        dw0  base
//   dw1  G(0..2) 6 bits | whole(r) << 18 |           dw1, 2  G(0..7), 8 bits each
//        R_8 << 21 | S << 23 | defer << 31           dw3  whole(r) | R_32 << 8 | S << 12 | defer << 31
//   dw2  S_0 | S_1 << 5 | cp << 10                   dw4  S_0..S_4, 6 bits each; dw5 S_5 | S_6 << 6 | cp << 12
//   dw4..27  24 slots                                dw6..63  58 slots
// Reference semantics: routing_table.cpp:67-111 (window rounds, sorted insertion, truncation).
// ---------------------------------------------------------------------------------------
constexpr uint32_t GL_SLOTS = 24, GL_HDR = 4, GL_STRIDE = 32;
constexpr uint32_t GL32_SLOTS = 58, GL32_HDR = 6, GL32_STRIDE = 64;
constexpr uint32_t GL_MAXCP = 40;  // key24 = ID bits [cp, cp + 24) from the top 64 bits

// A target below the first bucket (findBucket clamps it to bucket 0; it shares no window prefix).
__device__ __forceinline__ bool below_first(const DevTable& T, const Target& t) {
    const uint32_t* ft = T.ftail;
    return cmp160(t.hi, t.t2, t.t3, t.t4, T.fkey[0], ft[0], ft[1], ft[2]) < 0;
}

__device__ __forceinline__ bool gl_answer(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                          uint32_t (&o)[8], uint32_t& m) {
    uint4 L[8];
    if (act) {
        const uint4* lp = T.gl + (GL_STRIDE / 4) * (size_t)b;
#pragma unroll
        for (int x = 0; x < 8; x++) L[x] = lp[x];
    } else {
#pragma unroll
        for (int x = 0; x < 8; x++) L[x] = make_uint4(NONE, NONE, NONE, NONE);
    }
    const uint32_t h = L[0].y, h2 = L[0].z;
    const uint32_t G0 = h & 63u, G1 = (h >> 6) & 63u, G2 = (h >> 12) & 63u, R = (h >> 21) & 3u, S = (h >> 23) & 31u;
    const uint32_t Rc = (G0 >= count || (h >> 18) & 1u) ? 0u : (G1 >= count || (h >> 19) & 1u) ? 1u : 2u;
    m = min(count, Rc == 0 ? G0 : Rc == 1 ? G1 : G2);
    const uint32_t lim = Rc >= R ? S : Rc == 0 ? (h2 & 31u) : ((h2 >> 5) & 31u);
    bool ex = !act || (h & WL_DEFER) || lim < m || Rc > R;
    if (act && b == 0) ex |= below_first(T, t);
    const uint32_t cp = (h2 >> 10) & 63u;
    const uint32_t tx = (uint32_t)((t.hi << (cp & 63u)) >> 40) << 8;
    uint32_t v[GL_SLOTS];
#pragma unroll
    for (int s = 0; s < (int)GL_SLOTS; s++) v[s] = (uint32_t)s < lim ? dw(L, GL_HDR + s) ^ tx : NONE;
    sort8(v);
    sort8(v + 8);
    sort8(v + 16);
    merge8(v, v + 8);
    merge8(v, v + 16);
    const uint32_t base = L[0].x + T.index_base;
#pragma unroll
    for (int j = 0; j < 8; j++) o[j] = (uint32_t)j < m ? base + (v[j] & 255u) : NONE;
    return !ex;
}

__device__ __forceinline__ void rt_gl_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q,
                                                      uint32_t count, uint32_t* __restrict__ out_idx,
                                                      uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q && count > 0;
    if (i < q && count == 0 && out_cnt) out_cnt[i] = 0;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t = load_target(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t o[8], m;
    const bool ok = gl_answer(T, t, b, count, act, o, m);
    if (act && ok) {
        store_row8(out_idx + (size_t)i * count, o, count);
        if (out_cnt) out_cnt[i] = (uint8_t)m;
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, act && !ok, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
__global__ __launch_bounds__(BLOCK) void rt_gl_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                      uint32_t count, uint32_t* __restrict__ out_idx,
                                                      uint8_t* __restrict__ out_cnt) {
    rt_gl_kernel_body(T, targets, q, count, out_idx, out_cnt);
}

// ---------------------------------------------------------------------------------------
// Slot lines (TF_SL): general tables locate the target's bucket through the radix (one dependent load, plus a
// search over bucket firsts when the slot holds several bucket starts) before reading the bucket's line. A
// slot line is indexed by the target's top bits alone: coarse radix slot j = (t - rbase) >> slshift covers
// 2^(slshift - rshift) locate slots; when no bucket starts strictly inside it, every target in it lies in
// one bucket b, and slot line j is b's count <= 8 general line in 64 bytes (a 512-bit string):
//   [0, 32) base   [32, 44) G(0..2) capped at 15   [44, 47) whole(r)   [47, 49) R   [49, 54) S (the 128-byte
//   line's stored slots)   [54, 59) S_0   [59, 64) S_1   [64, 70) cp   [70] fallback
//   [71, 511) 20 slots of 22 bits: key16 << 6 | off (key16 = the top 16 of the 128-byte line's key24)
// A slot whose line cannot answer count 8 (the 128-byte line is deferred or stores more than 20 slots, a
// stored node has off >= 64, two stored nodes share key16) or in which a bucket starts holds a FALLBACK line
// instead: dw0 = the bucket at the slot start (NONE below the first bucket, or with several inner starts /
// an inner first with nonzero low bits), dw1 = NONE (the marker: a line's dw1 never is), dw2:dw3 = the top
// 64 bits of the one bucket first inside the slot, dw4 bit 0 = there is one. Its query reads the 128-byte
// line of the bucket that gives (no locate load); dw0 = NONE takes the locate path. The results are always
// the 128-byte line's (and from there the exact path's).
// ---------------------------------------------------------------------------------------
constexpr uint32_t SL_SLOTS = 20, SL_SBITS = 22, SL_SLOT0 = 71;

// The bucket of every coarse slot (NONE: a bucket starts inside it, or it lies below the first bucket).
__global__ void sl_index_kernel(const uint32_t* __restrict__ rrdx, uint32_t rslots, uint32_t k, uint32_t slslots,
                                uint32_t* __restrict__ slb) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= slslots) return;
    const uint32_t a = j << k, e = min((j + 1) << k, rslots);
    const uint32_t r0 = rrdx[a], r1 = rrdx[e];
    const uint32_t lo = r0 & RDX_MASK, hi = r1 & RDX_MASK;
    const bool exact = (r0 & RDX_EXACT) != 0;
    const uint32_t inner = hi - lo - (exact ? 1u : 0u);
    slb[j] = inner || (lo == 0 && !exact) ? NONE : (exact ? lo : lo - 1);
}

// Slot line j from 128-byte general line slb[j] (or its fallback line): every slot (gdirty == NULL) or those whose
// bucket is flagged (a fallback line of a slot with a bucket start depends on the bucket firsts only).
__global__ __launch_bounds__(BLOCK) void sl_build_kernel(const uint32_t* __restrict__ gl, const uint32_t* __restrict__ slb,
                                                          uint32_t slslots, const uint8_t* __restrict__ gdirty,
                                                          const uint32_t* __restrict__ rrdx, uint32_t rslots, uint32_t k,
                                                          const uint64_t* __restrict__ fkey,
                                                          const uint32_t* __restrict__ ftail, uint32_t* __restrict__ sl) {
    __shared__ uint32_t lds[BLOCK][17];
    for (uint32_t j = blockIdx.x * BLOCK + threadIdx.x; j < slslots; j += gridDim.x * BLOCK) {
        const uint32_t b = slb[j];
        if (gdirty && (b == NONE || !gdirty[b])) continue;
        uint32_t* L = lds[threadIdx.x];
        for (int x = 0; x < 17; x++) L[x] = NONE;
        bool fb = b == NONE;
        uint32_t fb_b = b, split_hi = 0, split_lo = 0, has_split = 0;
        if (b == NONE) {  // a bucket starts inside the slot: the bucket at its start and the one inner first
            const uint32_t r0 = rrdx[j << k], r1 = rrdx[min((j + 1) << k, rslots)];
            const uint32_t lo = r0 & RDX_MASK, hi = r1 & RDX_MASK;
            const bool exact = (r0 & RDX_EXACT) != 0;
            const uint32_t inner = hi - lo - (exact ? 1u : 0u);
            fb_b = (lo == 0 && !exact) ? NONE : (exact ? lo : lo - 1);
            if (fb_b != NONE && inner == 1) {
                const uint32_t ii = exact ? lo + 1 : lo;
                const uint32_t* ft = ftail + 3ull * ii;
                if ((ft[0] | ft[1] | ft[2]) == 0) {
                    split_hi = (uint32_t)(fkey[ii] >> 32);
                    split_lo = (uint32_t)fkey[ii];
                    has_split = 1;
                } else {
                    fb_b = NONE;
                }
            } else {
                fb_b = NONE;
            }
        } else {
            const uint32_t* W = gl + (size_t)GL_STRIDE * b;
            const uint32_t h = W[1], h2 = W[2], S = (h >> 23) & 31u;
            fb = (h & WL_DEFER) != 0 || S > SL_SLOTS || ((h >> 21) & 3u) > 2u;
            for (uint32_t u = 0; u < S && !fb; u++) {
                const uint32_t v = W[GL_HDR + u], k16 = v >> 16, off = v & 255u;
                fb |= off >= 64u;
                for (uint32_t r = 0; r < u; r++) fb |= (W[GL_HDR + r] >> 16) == k16;
                put_bits(L, SL_SLOT0 + SL_SBITS * u, SL_SBITS, (k16 << 6) | off);
            }
            if (!fb) {
                L[0] = W[0];
                L[1] = min(h & 63u, 15u) | (min((h >> 6) & 63u, 15u) << 4) | (min((h >> 12) & 63u, 15u) << 8) |
                       (((h >> 18) & 7u) << 12) | (((h >> 21) & 3u) << 15) | (S << 17) | ((h2 & 31u) << 22) |
                       (((h2 >> 5) & 31u) << 27);
                put_bits(L, 64, 7, (h2 >> 10) & 63u);
            }
        }
        if (fb) {
            for (int x = 0; x < 17; x++) L[x] = 0;
            L[0] = fb_b;
            L[1] = NONE;
            L[2] = split_hi;
            L[3] = split_lo;
            L[4] = has_split;
        }
        store_line<16>(L, sl + 16ull * j);
    }
}

// The slot-line answer of a query in coarse slot j (same contract as gl_answer). bh: the bucket whose 128-byte line
// a failed query reads next (a fallback line names it), NONE: locate it.
__device__ __forceinline__ bool sl_answer(const DevTable& T, uint64_t thi, uint32_t j, uint32_t count, bool act,
                                          uint32_t (&o)[8], uint32_t& m, uint32_t& bh) {
    uint4 L[4];
    if (act) {
        const uint4* lp = T.sl + 4ull * j;
#pragma unroll
        for (int x = 0; x < 4; x++) L[x] = lp[x];
    } else {
#pragma unroll
        for (int x = 0; x < 4; x++) L[x] = make_uint4(NONE, NONE, NONE, NONE);
    }
    const uint32_t h = L[0].y, x6 = ws_bits(L, 64, 7);
    const bool fbl = h == NONE;
    bh = NONE;
    if (act && fbl && L[0].x != NONE)
        bh = L[0].x + ((L[1].x & 1u) && thi >= (((uint64_t)L[0].z << 32) | L[0].w) ? 1u : 0u);
    const uint32_t G0 = h & 15u, G1 = (h >> 4) & 15u, G2 = (h >> 8) & 15u, R = (h >> 15) & 3u, S = (h >> 17) & 31u;
    const uint32_t Rc = (G0 >= count || (h >> 12) & 1u) ? 0u : (G1 >= count || (h >> 13) & 1u) ? 1u : 2u;
    m = min(count, Rc == 0 ? G0 : Rc == 1 ? G1 : G2);
    const uint32_t lim = Rc >= R ? S : Rc == 0 ? ((h >> 22) & 31u) : ((h >> 27) & 31u);
    const bool ex = !act || fbl || lim < m || Rc > R || lim > SL_SLOTS;
    const uint32_t cp = x6 & 63u;
    const uint32_t tx = (uint32_t)((thi << cp) >> 48) << 6;
    uint32_t v[24];
#pragma unroll
    for (int u = 0; u < 24; u++)
        v[u] = u < (int)SL_SLOTS && (uint32_t)u < lim ? ws_bits(L, SL_SLOT0 + SL_SBITS * (u < (int)SL_SLOTS ? u : 0), SL_SBITS) ^ tx
                                                      : NONE;
    sort8(v);
    sort8(v + 8);
    merge8(v, v + 8);
#pragma unroll
    for (int u = 16; u < (int)SL_SLOTS; u++) {  // insert the rest: one bubble pass each
        v[7] = min(v[7], v[u]);
#pragma unroll
        for (int r = 7; r > 0; r--) cx(v[r - 1], v[r]);
    }
    const uint32_t base = L[0].x + T.index_base;
#pragma unroll
    for (int r = 0; r < 8; r++) o[r] = (uint32_t)r < m ? base + (v[r] & 63u) : NONE;
    return !ex;
}

// count <= 8 on a general table with slot lines: the slot line, else locate + the 128-byte line, else exact.
// ABL 1 (timing ablation only, results wrong): slot lines only.
template <int ABL, bool CR = false>  // CR: as rt_wl_kernel_body
__device__ __forceinline__ void rt_sl_kernel_body(
    const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q, uint32_t count, uint32_t* __restrict__ out_idx,
    uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q && count > 0;
    if (i < q && count == 0 && out_cnt) out_cnt[i] = 0;
    const uint64_t thi = act ? load_target_hi(targets, i) : 0ull;
    const bool in = act && thi >= T.rbase && ((thi - T.rbase) >> T.slshift) < T.slslots;
    uint32_t o[8], m, bh;
    const bool ok = sl_answer(T, thi, in ? (uint32_t)((thi - T.rbase) >> T.slshift) : 0u, count, in, o, m, bh);
    if (CR && count == 8 && ((uintptr_t)out_idx & 15u) == 0) {  // kernel-uniform
        store_rows8_wave(out_idx, i, o, act && ok);
        if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    } else if (act && ok) {
        store_row8(out_idx + (size_t)i * count, o, count);
        if (out_cnt) out_cnt[i] = (uint8_t)m;
    }
    if (ABL) return;
    bool need = act && !ok;
    if (__any(need)) {  // locate and the 128-byte line (the full target: the locate may compare the low bits)
        Target t{};
        uint32_t b = 0;
        if (need) {
            t = load_target(targets, i);
            b = bh != NONE ? bh : locate_bucket(T, t);
        }
        const bool ok2 = gl_answer(T, t, b, count, need, o, m);
        if (need && ok2) {
            store_row8(out_idx + (size_t)i * count, o, count);
            if (out_cnt) out_cnt[i] = (uint8_t)m;
        }
        need = need && !ok2;
        __shared__ uint64_t xs[BLOCK / 64][192];
        exact_tail(T, t, need, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    }
}
template <int ABL>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void rt_sl_kernel(
    DevTable T, const uint8_t* __restrict__ targets, uint32_t q, uint32_t count, uint32_t* __restrict__ out_idx,
    uint8_t* __restrict__ out_cnt) {
    rt_sl_kernel_body<ABL, true>(T, targets, q, count, out_idx, out_cnt);
}

// Fallback slot lines (dw1 == NONE) and those without a bucket (dw0 == NONE): cnt[0], cnt[1] (KAD_DEBUG).
__global__ void sl_count_kernel(const uint32_t* sl, uint32_t slslots, uint32_t* cnt) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= slslots || sl[16ull * j + 1] != NONE) return;
    atomicAdd(cnt, 1u);
    if (sl[16ull * j] == NONE) atomicAdd(cnt + 1, 1u);
}

// flags[b] = v for the buckets of a line selection (a compacted dirty list)
__global__ void mark_sel_kernel(LineSel sel, uint32_t B, uint8_t* flags, uint8_t v) {
    for (uint32_t j = blockIdx.x * BLOCK + threadIdx.x;; j += gridDim.x * BLOCK) {
        uint32_t b;
        if (!sel.pick(j, B, b)) return;
        flags[b] = v;
    }
}

__device__ __forceinline__ bool gl32_answer(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                            uint32_t (&o)[32], uint32_t& m) {
    uint32_t L[GL32_STRIDE], v[64];
    if (act) {
        const uint4* lp = T.gl32 + (GL32_STRIDE / 4) * (size_t)b;
#pragma unroll
        for (int x = 0; x < (int)GL32_STRIDE / 4; x++) {
            const uint4 u = lp[x];
            L[4 * x] = u.x; L[4 * x + 1] = u.y; L[4 * x + 2] = u.z; L[4 * x + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int x = 0; x < (int)GL32_STRIDE; x++) L[x] = NONE;
    }
    const uint32_t h = L[3], S = (h >> 12) & 127u, R = (h >> 8) & 15u;
    uint32_t Rc = 8, Gc = 0;
#pragma unroll
    for (int r = 7; r >= 0; r--) {
        const uint32_t g = (L[1 + (r >> 2)] >> (8 * (r & 3))) & 255u;
        if (g >= count || ((h >> r) & 1u)) { Rc = (uint32_t)r; Gc = g; }
    }
    m = min(count, Gc);
    uint32_t lim = S;
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const uint32_t sr = r < 5 ? (L[4] >> (6 * r)) & 63u : (L[5] >> (6 * (r - 5))) & 63u;
        if ((uint32_t)r == Rc && Rc < R) lim = sr;
    }
    bool ex = !act || (h & WL_DEFER) || Rc > R || lim < m;
    if (act && b == 0) ex |= below_first(T, t);
    const uint32_t cp = (L[5] >> 12) & 63u;
    const uint32_t tx = (uint32_t)((t.hi << (cp & 63u)) >> 40) << 8;
#pragma unroll
    for (int s = 0; s < 64; s++) {
        const int li = s < (int)GL32_SLOTS ? (int)GL32_HDR + s : 0;
        v[s] = s < (int)GL32_SLOTS && (uint32_t)s < lim ? L[li] ^ tx : NONE;
    }
    sort16(v);
    sort16(v + 16);
    sort16(v + 32);
    sort16(v + 48);
    join_sorted<16>(v);
    join_sorted<16>(v + 32);
    merge32(v, v + 32);
    const uint32_t base = L[0] + T.index_base;
#pragma unroll
    for (int j = 0; j < 32; j++) o[j] = (uint32_t)j < m ? base + (v[j] & 255u) : NONE;
    return !ex;
}

// gl32_answer with FOUR lanes per query (rt_gl32q_kernel, counts 24 / 28 / 32 on tables with general lines: the
// reference's split-policy shape): lane p of the quad loads 64 of the line's 256 bytes (dwords 16x + 4p .. +3), sorts
// its 16 slot values and the quad merges them to the top 32 (as wl32_answer4). The header is lane 0's dwords 0..3
// and lane 1's 4, 5; the values, masks and fallbacks are gl32_answer's, so the rows are identical.
template <bool LOAD_ALL = false>  // as wl32_answer4's
__device__ __forceinline__ bool gl32_answer4(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                             uint32_t p, uint32_t (&v)[16], uint32_t& m, uint32_t& base) {
    uint32_t L[16];
    if (LOAD_ALL || act) {
        const uint4* lp = T.gl32 + (GL32_STRIDE / 4) * (size_t)b;
#pragma unroll
        for (int x = 0; x < 4; x++) {
            const uint4 u = lp[4 * x + p];
            L[4 * x] = u.x; L[4 * x + 1] = u.y; L[4 * x + 2] = u.z; L[4 * x + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int x = 0; x < 16; x++) L[x] = NONE;
    }
    const uint32_t h = qdpp<QP_B0>(L[3]), g03 = qdpp<QP_B0>(L[1]), g47 = qdpp<QP_B0>(L[2]);
    const uint32_t s04 = qdpp<QP_B1>(L[0]), s56 = qdpp<QP_B1>(L[1]);  // dwords 4, 5
    base = qdpp<QP_B0>(L[0]);
    const uint32_t S = (h >> 12) & 127u, R = (h >> 8) & 15u;
    uint32_t Rc = 8, Gc = 0;
#pragma unroll
    for (int r = 7; r >= 0; r--) {
        const uint32_t g = ((r < 4 ? g03 : g47) >> (8 * (r & 3))) & 255u;
        if (g >= count || ((h >> r) & 1u)) { Rc = (uint32_t)r; Gc = g; }
    }
    m = min(count, Gc);
    uint32_t lim = S;
#pragma unroll
    for (int r = 0; r < 7; r++) {
        const uint32_t sr = r < 5 ? (s04 >> (6 * r)) & 63u : (s56 >> (6 * (r - 5))) & 63u;
        if ((uint32_t)r == Rc && Rc < R) lim = sr;
    }
    bool ex = !act || (h & WL_DEFER) || Rc > R || lim < m;
    if (act && b == 0) ex |= below_first(T, t);
    const uint32_t cp = (s56 >> 12) & 63u;
    const uint32_t tx = (uint32_t)((t.hi << (cp & 63u)) >> 40) << 8;
#pragma unroll
    for (int e = 0; e < 16; e++) {
        const uint32_t dwi = 16u * (e >> 2) + 4u * p + (e & 3), sl = dwi - GL32_HDR;
        v[e] = dwi >= GL32_HDR && sl < lim ? L[e] ^ tx : NONE;  // empty slots stay NONE
    }
    const bool low = (p & 1u) == 0;
    sort16(v);
    quad_exchange<QP_X1, true>(v, low);
    clean16(v);
    quad_exchange<QP_X3, true>(v, true);
    quad_exchange<QP_X1, false>(v, low);
    clean16(v);
    return !ex;
}

// Counts 24, 28, 32 on general lines: four lanes per query, the row through a per-quad LDS row (rt_wl32q_kernel's).
// Held to 64 VGPRs (eight waves per SIMD instead of seven; no spill): 79.2-81.0 -> 78.1-78.5 us per 1M on the 4M-node
// split-policy table (profiles/r05/q32_occ8/; rt_wl32q_kernel measured the same either way).
// ABL (tools build only, KAD_RT_KERNEL=gl32q_abl1 / gl32q_stats): 1 = no exact path (those rows left unwritten);
// 3 = path statistics (out_cnt = 250 for the queries the exact path answers).
template <int ABL>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void rt_gl32q_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                         uint32_t count, uint32_t* __restrict__ out_idx,
                                                         uint8_t* __restrict__ out_cnt) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x, i = g >> 2, p = g & 3u;
    const bool act = i < q;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t = load_target(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t v[16], m, base;
    const bool ok = gl32_answer4<true>(T, t, b, count, act, p, v, m, base);  // launched on TF_GL32 tables
    const uint32_t r0 = 16u * (p & 1u), bi = base + T.index_base;
    uint32_t o[16];
    quad_row(v, r0, bi, m, count, act && ok, o);
    if (act && ok && p == 0 && out_cnt) out_cnt[i] = (uint8_t)m;
    __shared__ uint4 qrow[BLOCK / 4][9];  // per quad: 32 entries + a 16-byte pad
    uint32_t* R = reinterpret_cast<uint32_t*>(qrow[threadIdx.x >> 2]);
    if (p < 2u) {
#pragma unroll
        for (int x = 0; x < 4; x++)
            reinterpret_cast<uint4*>(R + 16u * p)[x] = make_uint4(o[4 * x], o[4 * x + 1], o[4 * x + 2], o[4 * x + 3]);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    if (act && ok) {
        uint32_t* row = out_idx + (size_t)i * count;
        if ((count & 3u) == 0 && ((uintptr_t)out_idx & 15u) == 0) {
#pragma unroll
            for (int hh = 0; hh < 2; hh++)
                if (16u * hh + 4u * p < count)
                    st_row4(row + 16 * hh + 4 * p, R[16 * hh + 4 * p], R[16 * hh + 4 * p + 1], R[16 * hh + 4 * p + 2],
                            R[16 * hh + 4 * p + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (4u * j + p < count) st_row1(row + 4 * j + p, R[4 * j + p]);
        }
    }
    if (ABL == 1) return;
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, act && !ok && p == 0u, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    if (ABL == 3 && act && !ok && p == 0u && out_cnt) out_cnt[i] = 250;
}

__device__ __forceinline__ void rt_gl32_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t = load_target(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t o[32], m;
    const bool ok = gl32_answer(T, t, b, count, act, o, m);
    if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    store_rows_block<32>(out_idx, q, count, o, act && ok);
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, act && !ok, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
__global__ __launch_bounds__(BLOCK) void rt_gl32_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    rt_gl32_kernel_body(T, targets, q, count, out_idx, out_cnt);
}

// ---------------------------------------------------------------------------------------
// General window lines for counts 9..16 (TF_GL16): the count <= 8 construction sized for 16 (R_16 <= 3, windows of up
// to 8 buckets) in ONE 128-byte line, so SEARCH_NODES = 14 (dht.cpp:1650, the refill of a search) reads 128 bytes
// instead of the 256-byte line of counts 17..32. Line b (32 dwords):
//   dw0  base    dw1  G(0..3), 6 bits each | whole(r) << 24 | R_16 << 28 | defer << 31
//   dw2  S | S_0 << 5 | S_1 << 10 | S_2 << 15 | cp << 20     dw3  0     dw4..31  28 slots: key24 << 8 | off
// The ranking is wl16's: 28 slot values padded to 32, two Batcher-16 sorts and one top-16 bitonic merge.
// ---------------------------------------------------------------------------------------
constexpr uint32_t GL16_SLOTS = 28, GL16_HDR = 4, GL16_STRIDE = 32;

// The count 9..16 answer from a loaded gl16 line (also the slot-indexed copies, TF_SL16): false when the query
// must take the exact path (deferred line, the window's slots do not hold m nodes).
__device__ __forceinline__ bool gl16_rank(const uint32_t (&L)[GL16_STRIDE], uint64_t thi, uint32_t count,
                                          uint32_t index_base, uint32_t (&o)[16], uint32_t& m) {
    const uint32_t h = L[1], h2 = L[2], R = (h >> 28) & 3u, S = h2 & 31u;
    uint32_t Rc = 4, Gc = 0;
#pragma unroll
    for (int r = 3; r >= 0; r--) {
        const uint32_t g = (h >> (6 * r)) & 63u;
        if (g >= count || ((h >> (24 + r)) & 1u)) { Rc = (uint32_t)r; Gc = g; }
    }
    m = min(count, Gc);
    const uint32_t lim = Rc >= R ? S : (h2 >> (5 + 5 * min(Rc, 2u))) & 31u;
    const bool ex = (h & WL_DEFER) || Rc > R || lim < m;
    const uint32_t cp = (h2 >> 20) & 63u;
    const uint32_t tx = (uint32_t)((thi << (cp & 63u)) >> 40) << 8;
    uint32_t v[32];
#pragma unroll
    for (int s = 0; s < 32; s++) {
        const int li = s < (int)GL16_SLOTS ? (int)GL16_HDR + s : 0;
        v[s] = s < (int)GL16_SLOTS && (uint32_t)s < lim ? L[li] ^ tx : NONE;
    }
    sort16(v);
    sort16(v + 16);
    merge16(v, v + 16);
    const uint32_t base = L[0] + index_base;
#pragma unroll
    for (int j = 0; j < 16; j++) o[j] = (uint32_t)j < m ? base + (v[j] & 255u) : NONE;
    return !ex;
}

__device__ __forceinline__ void load_line32(const uint4* lp, bool act, uint32_t (&L)[32]) {
    if (act) {
#pragma unroll
        for (int x = 0; x < 8; x++) {
            const uint4 u = lp[x];
            L[4 * x] = u.x; L[4 * x + 1] = u.y; L[4 * x + 2] = u.z; L[4 * x + 3] = u.w;
        }
    } else {
#pragma unroll
        for (int x = 0; x < 32; x++) L[x] = NONE;
    }
}

__device__ __forceinline__ bool gl16_answer(const DevTable& T, const Target& t, uint32_t b, uint32_t count, bool act,
                                            uint32_t (&o)[16], uint32_t& m) {
    uint32_t L[GL16_STRIDE];
    load_line32(T.gl16 + (GL16_STRIDE / 4) * (size_t)b, act, L);
    bool ok = gl16_rank(L, t.hi, count, T.index_base, o, m) && act;
    if (act && b == 0) ok &= !below_first(T, t);
    return ok;
}

__device__ __forceinline__ void rt_gl16_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    Target t{};
    uint32_t b = 0;
    if (act) {
        t = load_target(targets, i);
        b = locate_bucket(T, t);
    }
    uint32_t o[16], m;
    const bool ok = gl16_answer(T, t, b, count, act, o, m);
    if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    store_rows_block<16>(out_idx, q, count, o, act && ok);
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, act && !ok, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
__global__ __launch_bounds__(BLOCK) void rt_gl16_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    rt_gl16_kernel_body(T, targets, q, count, out_idx, out_cnt);
}

// ---------------------------------------------------------------------------------------
// Slot lines for counts 9..16 (TF_SL16): the count <= 8 slot lines' indexing (coarse radix slot j of the target's
// top bits, no locate load) for the gl16 lines. Line j (128 bytes) is a copy of gl16[b] when slot j lies inside one
// bucket b (slb[j]), else a fallback line in the count <= 8 slot lines' form: dw0 = the bucket at the slot start
// (NONE: locate), dw1 = NONE, dw2:dw3 = the top 64 bits of the one bucket first inside the slot, dw4 bit 0 = there
// is one. A query whose copied line cannot answer takes the exact path (the copy IS the bucket's line); a
// fallback query reads the named (or located) bucket's gl16 line. Results are the gl16 lines' in every case.
// ---------------------------------------------------------------------------------------
// Eight lanes per slot line: lane g copies 16-byte piece g (every slot, or those whose bucket is flagged).
__global__ __launch_bounds__(BLOCK) void sl16_build_kernel(const uint32_t* __restrict__ gl16,
                                                            const uint32_t* __restrict__ slb, uint32_t slslots,
                                                            const uint8_t* __restrict__ gdirty,
                                                            const uint32_t* __restrict__ rrdx, uint32_t rslots,
                                                            uint32_t k, const uint64_t* __restrict__ fkey,
                                                            const uint32_t* __restrict__ ftail, uint32_t* __restrict__ sl16) {
    const uint32_t g = threadIdx.x & 7u;
    for (uint32_t j = (blockIdx.x * BLOCK + threadIdx.x) >> 3; j < slslots; j += (gridDim.x * BLOCK) >> 3) {
        const uint32_t b = slb[j];
        if (gdirty && (b == NONE || !gdirty[b])) continue;
        uint4* dst = reinterpret_cast<uint4*>(sl16 + (size_t)GL16_STRIDE * j);
        if (b != NONE) {
            dst[g] = reinterpret_cast<const uint4*>(gl16 + (size_t)GL16_STRIDE * b)[g];
            continue;
        }
        if (g > 1) {  // the unused rest of a fallback line: zero, so a line's bytes are a function of the table
            dst[g] = make_uint4(0u, 0u, 0u, 0u);
            continue;
        }
        const uint32_t r0 = rrdx[j << k], r1 = rrdx[min((j + 1) << k, rslots)];
        const uint32_t lo = r0 & RDX_MASK, hi = r1 & RDX_MASK;
        const bool exact = (r0 & RDX_EXACT) != 0;
        const uint32_t inner = hi - lo - (exact ? 1u : 0u);
        uint32_t fb_b = (lo == 0 && !exact) ? NONE : (exact ? lo : lo - 1), split_hi = 0, split_lo = 0, has_split = 0;
        if (fb_b != NONE && inner == 1) {
            const uint32_t ii = exact ? lo + 1 : lo;
            const uint32_t* ft = ftail + 3ull * ii;
            if ((ft[0] | ft[1] | ft[2]) == 0) {
                split_hi = (uint32_t)(fkey[ii] >> 32);
                split_lo = (uint32_t)fkey[ii];
                has_split = 1;
            } else {
                fb_b = NONE;
            }
        } else {
            fb_b = NONE;
        }
        dst[g] = g == 0 ? make_uint4(fb_b, NONE, split_hi, split_lo) : make_uint4(has_split, 0u, 0u, 0u);
    }
}

__device__ __forceinline__ void rt_sl16_kernel_body(const DevTable& T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    const uint64_t thi = act ? load_target_hi(targets, i) : 0ull;
    const bool in = act && thi >= T.rbase && ((thi - T.rbase) >> T.slshift) < T.slslots;
    uint32_t L[GL16_STRIDE];
    load_line32(T.sl16 + (GL16_STRIDE / 4) * (size_t)(in ? (thi - T.rbase) >> T.slshift : 0ull), in, L);
    const bool fbl = L[1] == NONE;
    uint32_t o[16], m;
    bool ok = gl16_rank(L, thi, count, T.index_base, o, m) && in && !fbl;
    // fallback lines and targets outside the slot range: the named (or located) bucket's gl16 line; the rest of
    // the misses (a copied line that cannot answer) go straight to the exact path
    const bool miss = act && !ok;
    Target t{};
    if (miss) t = load_target(targets, i);
    const bool need = miss && (!in || fbl);
    if (__any(need)) {
        uint32_t b = 0;
        if (need) {
            const uint32_t bh = L[0] == NONE ? NONE
                                             : L[0] + ((L[4] & 1u) && thi >= (((uint64_t)L[2] << 32) | L[3]) ? 1u : 0u);
            b = in && bh != NONE ? bh : locate_bucket(T, t);
        }
        uint32_t o2[16], m2;
        const bool ok2 = gl16_answer(T, t, b, count, need, o2, m2) && need;
        if (ok2) {
#pragma unroll
            for (int j = 0; j < 16; j++) o[j] = o2[j];
            m = m2;
            ok = true;
        }
    }
    if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    store_rows_block<16>(out_idx, q, count, o, act && ok);
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T, t, act && !ok, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
__global__ __launch_bounds__(BLOCK) void rt_sl16_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    rt_sl16_kernel_body(T, targets, q, count, out_idx, out_cnt);
}

// One general window line of bucket b into L (LDS, W dwords, slots from HDR): see the layout above.
// NEED = 8, 16 or 32 (the count the window radius is sized for), RMAX = 2, 3 or 7.
struct GlInfo {
    uint32_t R, S, cp, base, whole, G[8], Sr[8];
    bool defer;
};

template <int RMAX, uint32_t NEED, uint32_t SLOTS, uint32_t HDR>
__device__ void gl_build_line(const uint64_t* key, const uint8_t* status, const uint2* dir, const uint32_t* gcnt,
                              const uint64_t* fkey, const uint32_t* ftail, uint32_t B, uint32_t b, uint32_t* L,
                              GlInfo& I) {
    I.R = RMAX + 1; I.S = 0; I.cp = 0; I.base = 0; I.whole = 0; I.defer = false;
    for (int r = 0; r < 8; r++) { I.G[r] = 0; I.Sr[r] = 0; }
    for (uint32_t r = 0, g = 0; r <= (uint32_t)RMAX; r++) {
        const uint32_t lo = b > r ? b - 1 - r : 0u, hi = min(B - 1, b + r);
        g += ring_good(gcnt, B, b, r);
        I.G[r] = g;
        const bool w = lo == 0 && hi == B - 1;
        I.whole |= (w ? 1u : 0u) << r;
        if (I.R > (uint32_t)RMAX && (I.G[r] >= NEED || w)) I.R = r;
    }
    if (I.R > (uint32_t)RMAX) { I.defer = true; return; }
    const uint32_t R = I.R, lo = b > R ? b - 1 - R : 0u, hi = min(B - 1, b + R), nb = hi - lo + 1;
    I.base = dir[lo].x & ~WIDE;
    // common prefix of the window's ID range [first_lo, end)
    const uint64_t klo = fkey[lo];
    uint64_t kend = ~0ull;
    if (hi + 1 < B) {
        const uint32_t* te = ftail + 3ull * (hi + 1);
        kend = fkey[hi + 1] - ((te[0] | te[1] | te[2]) == 0 ? 1ull : 0ull);
    }
    const uint32_t cp = klo == kend ? 64u : (uint32_t)__builtin_clzll(klo ^ kend);
    if (cp > GL_MAXCP) { I.defer = true; return; }
    I.cp = cp;
    // D order of the window's buckets (XOR images first_c ^ first_b) and whether it can depend on the target
    const uint64_t kb = fkey[b];
    uint32_t ord[16];
    bool amb = false;
    for (uint32_t y = lo; y <= hi; y++) {
        uint32_t rk = 0;
        for (uint32_t z = lo; z <= hi; z++) {
            const uint64_t iz = fkey[z] ^ kb, iy = fkey[y] ^ kb;
            rk += iz < iy || (iz == iy && z < y);
            amb |= z != y && iz == iy;  // buckets that differ only below bit 64
        }
        ord[rk] = y;
    }
    {   // b's depth: its size must be a power of two, aligned, with the low 96 bits of both ends zero
        const uint32_t* tb = ftail + 3ull * b;
        uint64_t size = (b + 1 < B ? fkey[b + 1] : 0ull) - kb;  // 2^64 wrap for the last bucket
        bool dy = (tb[0] | tb[1] | tb[2]) == 0 && size && (size & (size - 1)) == 0 && (kb & (size - 1)) == 0;
        if (b + 1 < B) {
            const uint32_t* tn = ftail + 3ull * (b + 1);
            dy &= (tn[0] | tn[1] | tn[2]) == 0;
        } else if (kb == 0) {
            dy = true;  // one bucket covers everything: depth 0
            size = 0;
        }
        const uint32_t db = size ? 64u - (uint32_t)__builtin_ctzll(size) : 0u;
        amb |= !dy;
        for (uint32_t y = lo; y <= hi && !amb; y++)
            for (uint32_t z = y + 1; z <= hi; z++)
                if ((uint32_t)__builtin_clzll((fkey[y] ^ fkey[z]) | 1ull) >= db) { amb = true; break; }
    }
    // whole buckets in D order while they fit
    uint32_t stored = 0, used = 0;  // bit (c - lo)
    bool full = false;
    for (uint32_t j = 0; j < nb; j++) {
        const uint32_t x = ord[j], g = good_of(dir, gcnt, x);
        if (full || used + g > SLOTS) { full = true; continue; }
        used += g;
        stored |= 1u << (x - lo);
    }
    if (full && amb) { I.defer = true; return; }
    // slots ring by ring: W(0) = {b-1, b}, round r >= 1 adds b+r and b-1-r
    uint32_t S = 0;
    for (uint32_t r = 0; r <= R; r++) {
        const uint32_t cand[2] = {r == 0 ? b : b + r, b >= r + 1 ? b - 1 - r : NONE};
        for (int k = 0; k < 2; k++) {
            const uint32_t x = cand[k];
            if (x == NONE || x < lo || x > hi || !((stored >> (x - lo)) & 1u)) continue;
            for_good(key, status, dir, x, [&](uint32_t n, uint64_t kn) {
                const uint32_t off = n - I.base;
                I.defer |= off > 255u || (cp && ((kn ^ klo) >> (64 - cp)) != 0);  // outside the window's range
                const uint32_t k24 = (uint32_t)((kn << cp) >> 40);
                for (uint32_t u = 0; u < S; u++) I.defer |= (L[HDR + u] >> 8) == k24;
                L[HDR + S] = (k24 << 8) | (off & 255u);
                S++;
            });
        }
        I.Sr[r] = S;
    }
    I.S = S;
}

// General line b (count <= 8) assembled in L (an LDS row of GL_STRIDE + 1 dwords) and stored.
__device__ void gl8_build_line(const uint64_t* key, const uint8_t* status, const uint2* dir, const uint32_t* gcnt,
                               const uint64_t* fkey, const uint32_t* ftail, uint32_t B, uint32_t* lines, uint32_t b,
                               uint32_t* L) {
    for (uint32_t k = 0; k < GL_STRIDE; k++) L[k] = NONE;
    GlInfo I;
    gl_build_line<2, 8, GL_SLOTS, GL_HDR>(key, status, dir, gcnt, fkey, ftail, B, b, L, I);
    uint32_t h = 0;
    for (int r = 0; r < 3; r++) h |= min(I.G[r], 63u) << (6 * r);
    h |= (I.whole & 7u) << 18;
    L[0] = I.base;
    L[1] = h | (min(I.R, 3u) << 21) | (I.S << 23) | (I.defer ? WL_DEFER : 0u);
    L[2] = I.Sr[0] | (I.Sr[1] << 5) | (I.cp << 10);
    L[3] = 0;
    store_line<GL_STRIDE>(L, lines + (size_t)GL_STRIDE * b);
}

__global__ __launch_bounds__(BLOCK) void gl_build_kernel(const uint64_t* key, const uint8_t* status, const uint2* dir,
                                                         const uint32_t* gcnt, const uint64_t* fkey, const uint32_t* ftail,
                                                         uint32_t B, uint32_t* lines, LineSel sel) {
    __shared__ uint32_t lds[BLOCK][GL_STRIDE + 1];
    // one item per thread, grid-stride (an incremental rebuild launches a capped grid)
    for (uint32_t j_ = blockIdx.x * BLOCK + threadIdx.x;; j_ += gridDim.x * BLOCK) {
        uint32_t b;
        if (!sel.pick(j_, B, b)) return;
        gl8_build_line(key, status, dir, gcnt, fkey, ftail, B, lines, b, lds[threadIdx.x]);
    }
}

__global__ __launch_bounds__(BLOCK) void gl16_build_kernel(const uint64_t* key, const uint8_t* status, const uint2* dir,
                                                           const uint32_t* gcnt, const uint64_t* fkey,
                                                           const uint32_t* ftail, uint32_t B, uint32_t* lines,
                                                           LineSel sel) {
    __shared__ uint32_t lds[BLOCK][GL16_STRIDE + 1];
    for (uint32_t j_ = blockIdx.x * BLOCK + threadIdx.x;; j_ += gridDim.x * BLOCK) {
        uint32_t b;
        if (!sel.pick(j_, B, b)) return;
        uint32_t* L = lds[threadIdx.x];
        for (uint32_t k = 0; k < GL16_STRIDE; k++) L[k] = NONE;
        GlInfo I;
        gl_build_line<3, 16, GL16_SLOTS, GL16_HDR>(key, status, dir, gcnt, fkey, ftail, B, b, L, I);
        uint32_t h = 0;
        for (int r = 0; r < 4; r++) h |= min(I.G[r], 63u) << (6 * r);
        L[0] = I.base;
        L[1] = h | ((I.whole & 15u) << 24) | (min(I.R, 3u) << 28) | (I.defer ? WL_DEFER : 0u);
        L[2] = I.S | (I.Sr[0] << 5) | (I.Sr[1] << 10) | (I.Sr[2] << 15) | (I.cp << 20);
        L[3] = 0;
        store_line<GL16_STRIDE>(L, lines + (size_t)GL16_STRIDE * b);
    }
}

__global__ __launch_bounds__(BLOCK) void gl32_build_kernel(const uint64_t* key, const uint8_t* status, const uint2* dir,
                                                           const uint32_t* gcnt, const uint64_t* fkey,
                                                           const uint32_t* ftail, uint32_t B, uint32_t* lines,
                                                           LineSel sel) {
    __shared__ uint32_t lds[BLOCK][GL32_STRIDE + 1];
    // one item per thread, grid-stride (an incremental rebuild launches a capped grid)
    for (uint32_t j_ = blockIdx.x * BLOCK + threadIdx.x;; j_ += gridDim.x * BLOCK) {
        uint32_t b;
        if (!sel.pick(j_, B, b)) return;
        [&] {
    uint32_t* L = lds[threadIdx.x];
    for (uint32_t k = 0; k < GL32_STRIDE; k++) L[k] = NONE;
    GlInfo I;
    gl_build_line<7, 32, GL32_SLOTS, GL32_HDR>(key, status, dir, gcnt, fkey, ftail, B, b, L, I);
    uint32_t g01 = 0, g23 = 0;
    for (int r = 0; r < 8; r++) {
        const uint32_t g = min(I.G[r], 255u);
        if (r < 4) g01 |= g << (8 * r); else g23 |= g << (8 * (r - 4));
    }
    L[0] = I.base;
    L[1] = g01;
    L[2] = g23;
    L[3] = (I.whole & 255u) | (min(I.R, 15u) << 8) | (I.S << 12) | (I.defer ? WL_DEFER : 0u);
    L[4] = I.Sr[0] | (I.Sr[1] << 6) | (I.Sr[2] << 12) | (I.Sr[3] << 18) | (I.Sr[4] << 24);
    L[5] = I.Sr[5] | (I.Sr[6] << 6) | (I.cp << 12);
    store_line<GL32_STRIDE>(L, lines + (size_t)GL32_STRIDE * b);
        }();
    }
}

// Deferred lines of a line set (decides at table creation whether the general lines pay off).
__global__ void count_deferred_kernel(const uint32_t* lines, uint32_t stride, uint32_t hdr_word, uint32_t B,
                                      uint32_t* n) {
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    const bool d = b < B && (lines[(size_t)stride * b + hdr_word] & WL_DEFER);
    const uint64_t bal = __ballot(d);
    if ((threadIdx.x & 63) == 0 && bal) atomicAdd(n, (uint32_t)__popcll(bal));
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

// Dual-family batch for count <= 8 where a family has window lines: per lane the family's table,
// its window line when it has lines, the lane fast path otherwise, then the exact path per family.
// LEAN (both families have the lines or are empty, as in config 4): no lane fast path compiled in (its registers
// cost occupancy), an empty family's queries get empty rows.
template <bool LEAN>
__device__ __forceinline__ void rt_dual_wl_body(const DevTable& T4, const DevTable& T6, const uint8_t* __restrict__ targets,
                                                const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q && count > 0;
    if (i < q && count == 0 && out_cnt) out_cnt[i] = 0;
    Target t{};
    bool six = false;
    if (act) {
        t = load_target(targets, i);
        six = af[i] != 0;
    }
    const DevTable& T = six ? T6 : T4;
    const bool wl = act && (T.flags & TF_WL);
    const uint32_t b = wl ? locate_bucket(T, t) : 0u;
    uint32_t o[8], m;
    const bool ok = line8_answer(T, t, b, count, wl, wl && (T.flags & TF_WS), o, m);
    uint32_t* row = out_idx + (size_t)i * count;
    bool ex = wl && !ok;
    if (wl && ok) {
        store_row8(row, o, count);
        if (out_cnt) out_cnt[i] = (uint8_t)m;
    } else if (act && !wl) {
        if (LEAN) {  // an empty family (routing_table.cpp:73)
            for (uint32_t s = 0; s < count; s++) row[s] = NONE;
            if (out_cnt) out_cnt[i] = 0;
        } else {
            ex = !rt_query_fast<8, 3>(T, t, count, row, out_cnt ? out_cnt + i : nullptr);
        }
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T4, t, ex && !six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    exact_tail(T6, t, ex && six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
__global__ __launch_bounds__(BLOCK) void rt_dual_wl_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ targets,
                                                           const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                           uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    rt_dual_wl_body<false>(T4, T6, targets, af, q, count, out_idx, out_cnt);
}
__global__ __launch_bounds__(BLOCK) void rt_dual_wl_lean_kernel(
    DevTable T4, DevTable T6, const uint8_t* __restrict__ targets, const uint8_t* __restrict__ af, uint32_t q,
    uint32_t count, uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    rt_dual_wl_body<true>(T4, T6, targets, af, q, count, out_idx, out_cnt);
}

// Dual-family batch (af per query) for families with general window lines (split-policy tables, the shape the
// reference builds): count range K = 8 / 16 / 32 -> the gl / gl16 / gl32 line of the lane's family (locate first);
// a family without that line set takes the lane path, an unanswered query the exact path of its family.
template <int K>
__global__ __launch_bounds__(BLOCK) void rt_dual_gl_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ targets,
                                                           const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                           uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q && count > 0;
    if (i < q && count == 0 && out_cnt) out_cnt[i] = 0;
    Target t{};
    bool six = false;
    if (act) {
        t = load_target(targets, i);
        six = af[i] != 0;
    }
    const DevTable& T = six ? T6 : T4;
    const bool gl = act && (T.flags & (K == 8 ? TF_GL : K == 16 ? TF_GL16 : TF_GL32));
    const uint32_t b = gl ? locate_bucket(T, t) : 0u;
    uint32_t o[K], m = 0;
    bool ok;
    if constexpr (K == 8) ok = gl_answer(T, t, b, count, gl, o, m);
    else if constexpr (K == 16) ok = gl16_answer(T, t, b, count, gl, o, m);
    else ok = gl32_answer(T, t, b, count, gl, o, m);
    ok = ok && gl;
    if (ok && out_cnt) out_cnt[i] = (uint8_t)m;
    if constexpr (K == 8) {
        if (ok) store_row8(out_idx + (size_t)i * count, o, count);
    } else {
        store_rows_block<K>(out_idx, q, count, o, ok);
    }
    bool ex = gl && !ok;
    if (act && !gl) ex = !rt_query_fast<K, 3>(T, t, count, out_idx + (size_t)i * count, out_cnt ? out_cnt + i : nullptr);
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T4, t, ex && !six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    exact_tail(T6, t, ex && six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}

// Dual-family batch for counts 9..16 where a family has 16-slot window lines (same structure). LEAN: rows through
// LDS as coalesced 16-byte stores (store_rows_block, as rt_wl16_kernel) and no lane fast path.
template <bool LEAN>
__device__ __forceinline__ void rt_dual_wl16_body(const DevTable& T4, const DevTable& T6,
                                                  const uint8_t* __restrict__ targets,
                                                  const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                  uint32_t* __restrict__ out_idx,
                                                  uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    Target t{};
    bool six = false;
    if (act) {
        t = load_target(targets, i);
        six = af[i] != 0;
    }
    const DevTable& T = six ? T6 : T4;
    const bool wl = act && (T.flags & TF_WL16);
    const uint32_t b = wl ? locate_bucket(T, t) : 0u;
    uint32_t o[16], m;
    const bool ok = wl16_answer(T, t, b, count, wl, o, m);
    uint32_t* row = out_idx + (size_t)i * count;
    bool ex = wl && !ok;
    if (LEAN) {
        if (wl && ok && out_cnt) out_cnt[i] = (uint8_t)m;
        store_rows_block<16>(out_idx, q, count, o, wl && ok);
        if (act && !wl) {  // an empty family (routing_table.cpp:73)
            for (uint32_t s = 0; s < count; s++) row[s] = NONE;
            if (out_cnt) out_cnt[i] = 0;
        }
    } else if (wl && ok) {
        store_row16(row, o, count);
        if (out_cnt) out_cnt[i] = (uint8_t)m;
    } else if (act && !wl) {
        ex = !rt_query_fast<16, 3>(T, t, count, row, out_cnt ? out_cnt + i : nullptr);
    }
    // the line's misses: the family's 32-count line by the wave (as rt_wl16_kernel), then the exact path
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t sixm = __ballot(six);
    for (uint64_t pm = __ballot(wl && !ok); pm; pm &= pm - 1) {
        const uint32_t l = (uint32_t)__builtin_ctzll(pm);
        const DevTable& Tl = ((sixm >> l) & 1ull) ? T6 : T4;  // wave-uniform
        if (!(Tl.flags & TF_WL32)) continue;
        Target u;
        u.hi = rdl64(t.hi, l);
        u.t2 = rdl(t.t2, l);
        u.t3 = rdl(t.t3, l);
        u.t4 = rdl(t.t4, l);
        const uint32_t il = rdl(i, l);
        if (wave_wl32(Tl, u, rdl(b, l), count, lane, out_idx + (size_t)il * count, out_cnt ? out_cnt + il : nullptr) &&
            lane == l)
            ex = false;
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T4, t, ex && !six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    exact_tail(T6, t, ex && six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}
template <bool LEAN>
__global__ __launch_bounds__(BLOCK) void rt_dual_wl16_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ targets,
                                                             const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                             uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    rt_dual_wl16_body<LEAN>(T4, T6, targets, af, q, count, out_idx, out_cnt);
}

// Dual-family batch for counts 17..32 where a family has 64-slot window lines (same structure). LEAN: no lane fast
// path compiled in.
template <bool LEAN>
__global__ __launch_bounds__(BLOCK) void rt_dual_wl32_kernel(DevTable T4, DevTable T6,
                                                             const uint8_t* __restrict__ targets,
                                                             const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                             uint32_t* __restrict__ out_idx,
                                                             uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    Target t{};
    bool six = false;
    if (act) {
        t = load_target(targets, i);
        six = af[i] != 0;
    }
    const DevTable& T = six ? T6 : T4;
    const bool wl = act && (T.flags & TF_WL32);
    const uint32_t b = wl ? locate_bucket(T, t) : 0u;
    uint32_t o[32], m;
    const bool ok = wl32_answer(T, t, b, count, wl, o, m);
    uint32_t* row = out_idx + (size_t)i * count;
    bool ex = wl && !ok;
    if (wl && ok) {
        store_row32(row, o, count);
        if (out_cnt) out_cnt[i] = (uint8_t)m;
    } else if (act && !wl) {
        if (LEAN) {  // an empty family (routing_table.cpp:73)
            for (uint32_t s = 0; s < count; s++) row[s] = NONE;
            if (out_cnt) out_cnt[i] = 0;
        } else {
            ex = !rt_query_fast<32, 6>(T, t, count, row, out_cnt ? out_cnt + i : nullptr);
        }
    }
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T4, t, ex && !six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    exact_tail(T6, t, ex && six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}

// Dual-family batch on slot lines (both families with them or empty; the reference's split-policy shape, as
// Dht::onGetValues asks both tables): rt_sl_kernel (count <= 8) and rt_sl16_kernel (9..16) with the table per lane,
// the fallback line of the lane's family, the exact path per family.
__global__ __launch_bounds__(BLOCK) void rt_dual_sl_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ targets,
                                                           const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                           uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q && count > 0;
    if (i < q && count == 0 && out_cnt) out_cnt[i] = 0;
    const bool six = act && af[i] != 0;
    const DevTable& T = six ? T6 : T4;
    const bool empty = act && T.B == 0;  // an empty family (routing_table.cpp:73)
    const uint64_t thi = act ? load_target_hi(targets, i) : 0ull;
    const bool in = act && !empty && thi >= T.rbase && ((thi - T.rbase) >> T.slshift) < T.slslots;
    uint32_t o[8], m, bh;
    const bool ok = sl_answer(T, thi, in ? (uint32_t)((thi - T.rbase) >> T.slshift) : 0u, count, in, o, m, bh);
    uint32_t* row = out_idx + (size_t)i * count;
    if (act && ok) {
        store_row8(row, o, count);
        if (out_cnt) out_cnt[i] = (uint8_t)m;
    } else if (empty) {
        for (uint32_t c = 0; c < count; c++) row[c] = NONE;
        if (out_cnt) out_cnt[i] = 0;
    }
    bool need = act && !ok && !empty;
    if (__any(need)) {  // locate and the family's 128-byte line, then the exact path of the family
        Target t{};
        uint32_t b = 0;
        if (need) {
            t = load_target(targets, i);
            b = bh != NONE ? bh : locate_bucket(T, t);
        }
        const bool ok2 = gl_answer(T, t, b, count, need, o, m);
        if (need && ok2) {
            store_row8(row, o, count);
            if (out_cnt) out_cnt[i] = (uint8_t)m;
        }
        need = need && !ok2;
        __shared__ uint64_t xs[BLOCK / 64][192];
        exact_tail(T4, t, need && !six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
        exact_tail(T6, t, need && six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    }
}

__global__ __launch_bounds__(BLOCK) void rt_dual_sl16_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ targets,
                                                             const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                             uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    const bool act = i < q;
    const bool six = act && af[i] != 0;
    const DevTable& T = six ? T6 : T4;
    const bool empty = act && T.B == 0;  // an empty family (routing_table.cpp:73)
    const uint64_t thi = act ? load_target_hi(targets, i) : 0ull;
    const bool in = act && !empty && thi >= T.rbase && ((thi - T.rbase) >> T.slshift) < T.slslots;
    uint32_t L[GL16_STRIDE];
    load_line32(T.sl16 + (GL16_STRIDE / 4) * (size_t)(in ? (thi - T.rbase) >> T.slshift : 0ull), in, L);
    const bool fbl = L[1] == NONE;
    uint32_t o[16], m;
    bool ok = gl16_rank(L, thi, count, T.index_base, o, m) && in && !fbl;
    const bool miss = act && !ok && !empty;
    Target t{};
    if (miss) t = load_target(targets, i);
    const bool need = miss && (!in || fbl);
    if (__any(need)) {
        uint32_t b = 0;
        if (need) {
            const uint32_t bh = L[0] == NONE ? NONE
                                             : L[0] + ((L[4] & 1u) && thi >= (((uint64_t)L[2] << 32) | L[3]) ? 1u : 0u);
            b = in && bh != NONE ? bh : locate_bucket(T, t);
        }
        uint32_t o2[16], m2;
        const bool ok2 = gl16_answer(T, t, b, count, need, o2, m2) && need;
        if (ok2) {
#pragma unroll
            for (int j = 0; j < 16; j++) o[j] = o2[j];
            m = m2;
            ok = true;
        }
    }
    if (empty) {
#pragma unroll
        for (int j = 0; j < 16; j++) o[j] = NONE;
        m = 0;
        ok = true;
    }
    if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    store_rows_block<16>(out_idx, q, count, o, act && ok);
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T4, t, act && !ok && !six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    exact_tail(T6, t, act && !ok && six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}

// Dual-family counts 24, 28, 32 (both families with 64-slot lines or empty): rt_wl32q_kernel's four lanes per
// query and per-quad LDS row store, the family per quad. GL: the general lines (gl32_answer4, split-policy tables).
template <bool GL>
__global__ __launch_bounds__(BLOCK) void rt_dual_wl32q_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ targets,
                                                              const uint8_t* __restrict__ af, uint32_t q, uint32_t count,
                                                              uint32_t* __restrict__ out_idx,
                                                              uint8_t* __restrict__ out_cnt) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x, i = g >> 2, p = g & 3u;
    const bool act = i < q;
    Target t{};
    bool six = false;
    if (act) {
        t = load_target(targets, i);
        six = af[i] != 0;
    }
    const DevTable& T = six ? T6 : T4;  // quad-uniform
    const bool wl = act && (T.flags & (GL ? TF_GL32 : TF_WL32));
    const uint32_t b = wl ? locate_bucket(T, t) : 0u;
    uint32_t v[16], m, base;
    const bool ok = GL ? gl32_answer4<false>(T, t, b, count, wl, p, v, m, base) : wl32_answer4<true>(T, t, b, count, wl, p, v, m, base);
    const uint32_t r0 = 16u * (p & 1u), bi = base + T.index_base;
    uint32_t o[16];
    quad_row(v, r0, bi, m, count, wl && ok, o);
    if (wl && ok && p == 0 && out_cnt) out_cnt[i] = (uint8_t)m;
    __shared__ uint4 qrow[BLOCK / 4][9];  // per quad: 32 entries + a 16-byte pad
    uint32_t* R = reinterpret_cast<uint32_t*>(qrow[threadIdx.x >> 2]);
    if (p < 2u) {
#pragma unroll
        for (int x = 0; x < 4; x++)
            reinterpret_cast<uint4*>(R + 16u * p)[x] = make_uint4(o[4 * x], o[4 * x + 1], o[4 * x + 2], o[4 * x + 3]);
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    uint32_t* row = out_idx + (size_t)i * count;
    if (wl && ok) {
        if ((count & 3u) == 0 && ((uintptr_t)out_idx & 15u) == 0) {
#pragma unroll
            for (int h = 0; h < 2; h++)
                if (16u * h + 4u * p < count)
                    st_row4(row + 16 * h + 4 * p, R[16 * h + 4 * p], R[16 * h + 4 * p + 1], R[16 * h + 4 * p + 2],
                            R[16 * h + 4 * p + 3]);
        } else {
#pragma unroll
            for (int j = 0; j < 8; j++)
                if (4u * j + p < count) st_row1(row + 4 * j + p, R[4 * j + p]);
        }
    } else if (act && !wl) {  // an empty family (routing_table.cpp:73)
        for (uint32_t j = p; j < count; j += 4) row[j] = NONE;
        if (p == 0 && out_cnt) out_cnt[i] = 0;
    }
    const bool ex = wl && !ok && p == 0u;
    __shared__ uint64_t xs[BLOCK / 64][192];
    exact_tail(T4, t, ex && !six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
    exact_tail(T6, t, ex && six, i, count, out_idx, out_cnt, xs[threadIdx.x >> 6]);
}

// ---------------------------------------------------------------------------------------
// Sharded table without halo: the north-star multi-GPU variant.
// The global uniform-depth table is cut into contiguous bucket ranges, one per GPU. Every rank
// holds the GLOBAL good prefix sums (all-gathered once at setup), so it can compute any query's
// global window W(R), and answers W(R) ∩ its shard for every query of a replicated batch:
//   * W(R) misses the shard       -> nothing; a lane whose bucket lies outside [reach_lo, reach_hi)
//                                    exits after one compare, without a load
//   * W(R) inside the shard       -> its final row, appended to `rows` (compact)
//   * W(R) crosses a shard edge   -> this shard's top-count of W(R) ∩ shard with the entries' XOR
//                                    distances, appended to `parts`; kad_rt_merge_parts merges them
// Queries whose bucket is >= 4 buckets inside the shard use the window line (its local window is the
// global one); the others take the wave-cooperative path on the global window.
// Row layout (uint32): qid, m, 0, 0, idx[count] (padded to 4): KAD_ROW_WORDS(count).
// Part layout: the row, then dist[count][5]: KAD_PART_WORDS(count).
// Complete rows of workgroup w (QB = 256, 1,024 or 2,048 queries, shard_qb) go to region w % 8 of KAD_SHARD_REGIONS
// regions of row_cap rows: one atomic per workgroup and home rank for the window-line rows, eight counters per home
// (a single counter hit by every wave cost ~10 ns per wave, 160 us per 1M queries). A query takes at most two rows (a
// tombstone and its wave-path row), so row_cap >= 2 * ceil(W / 8) * QB never overflows, W = the workgroups holding
// a home range's queries (ceil(q / QB) for one home; ceil(ceil(q / 256) / world / (QB / 256)) + 1 per home).
// ---------------------------------------------------------------------------------------
struct ShardCtx {
    const uint32_t* gpre;  // global good prefix sums, GB + 1
    uint64_t gbase;        // top 64 bits of global bucket 0's first ID
    uint32_t gshift, GB;   // global direct locate: b = (t.hi - gbase) >> gshift, clamped to [0, GB)
    uint32_t s_lo, s_hi;   // global buckets held by this shard (local bucket = global - s_lo)
    uint32_t reach_lo, reach_hi;
    uint32_t* rows;
    uint32_t* parts;
    uint32_t* ctr;  // counter k at word KAD_SHARD_COUNTER_STRIDE*k (own 128-byte line): [0..7] rows appended
                    // per region, [8] parts appended, [9] overflow flag
    uint32_t row_cap, part_cap, rs, ps;
    // home-rank exchange (kad_rt_shard_batch_home): rows and parts of query block k go to the send block of rank
    // home(k) = k * dests / nblk (dest_words apart); dests = 1: one block for every query (the all-gather layout)
    uint32_t dests, nblk;
    uint64_t dest_words;
};

// The rank a query's rows and parts go to: query blocks of BLOCK queries split evenly over the ranks, in order.
__host__ __device__ __forceinline__ uint32_t home_of_block(uint32_t k, uint32_t dests, uint32_t nblk) {
    return (uint32_t)(((uint64_t)k * dests) / nblk);
}
__device__ __forceinline__ uint64_t dest_off(const ShardCtx& S, uint32_t qid) {
    return S.dests > 1 ? (uint64_t)home_of_block(qid / BLOCK, S.dests, S.nblk) * S.dest_words : 0ull;
}

__device__ __forceinline__ uint32_t shard_bucket(const ShardCtx& S, const Target& t) {
    if (t.hi < S.gbase) return 0;
    const uint64_t s = (t.hi - S.gbase) >> S.gshift;
    return s >= S.GB ? S.GB - 1 : (uint32_t)s;
}

__device__ __forceinline__ uint32_t lanes_below(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// Queries and threads per workgroup of rt_shard_kernel<LK>: 1,024 and 256 for LK 0 / 8 / 16; 256 and 64 for LK 32,
// whose 193 VGPRs hold two waves per SIMD: one-wave workgroups wait at no barrier for the other waves' line work
// (rank 0 of 8, k = 32: 33.6 -> 30.7 us; held to 128 VGPRs for four waves per SIMD it spills 36 and takes 33.0;
// k = 8 and 16 measured slower with 64- or 128-thread workgroups:
// tools/shard_ab.py, profiles/r05/shard_shape/). (2,048 per workgroup measured no faster at N = 8 and costs k = 8 /
// 16 5 / 4 us: KAD_SHARD_ABL=16, tools build.) The tools-build A/B libraries set the KAD_SHARD_* macros.
#ifndef KAD_SHARD_QB8
#define KAD_SHARD_QB8 1024u
#endif
#ifndef KAD_SHARD_WG8
#define KAD_SHARD_WG8 256u
#endif
#ifndef KAD_SHARD_QB32
#define KAD_SHARD_QB32 256u
#endif
#ifndef KAD_SHARD_WG32
#define KAD_SHARD_WG32 64u
#endif
__host__ __device__ constexpr uint32_t shard_qb(int lk) { return lk == 32 ? KAD_SHARD_QB32 : KAD_SHARD_QB8; }
__host__ __device__ constexpr uint32_t shard_wg(int lk) { return lk == 32 ? KAD_SHARD_WG32 : KAD_SHARD_WG8; }

// One query, wave-uniform: global window, intersection with the shard, wave_rank, append (complete rows to `region`,
// the region of the query's workgroup, as its line rows').
__device__ void wave_shard(const DevTable& T, const ShardCtx& S, const Target& t, uint32_t qid, uint32_t count,
                           uint32_t region, uint64_t* xs) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t lo, hi, good;
    wave_window_pre(S.gpre, S.GB, shard_bucket(S, t), count, lo, hi, good);
    const uint32_t a = max(lo, S.s_lo), e = min(hi + 1, S.s_hi);
    if (a >= e) return;
    const bool complete = lo >= S.s_lo && hi < S.s_hi;
    const uint32_t al = a - S.s_lo, el = e - S.s_lo;
    // the window's node range, the row slot and (parts only) the local good count: independent round trips, issued
    // together (a complete window's good count is the global one)
    const uint32_t beg = T.dir[al].x & ~WIDE, end = T.dir[el].x & ~WIDE;
    uint32_t slot = 0;
    const uint64_t dof = dest_off(S, qid);
    uint32_t* ctr = S.ctr + dof;
    if (lane == 0) slot = atomicAdd(ctr + KAD_SHARD_COUNTER_STRIDE * (complete ? region : 8u), 1u);
    const uint32_t lgood = complete ? good : wave_good_sum(T.gcnt, al, el);
    slot = rdl(slot, 0);
    if (slot >= (complete ? S.row_cap : S.part_cap)) {
        if (lane == 0) atomicOr(ctr + KAD_SHARD_COUNTER_STRIDE * 9u, 1u);
        return;
    }
    uint32_t* row = complete ? S.rows + dof + ((size_t)region * S.row_cap + slot) * S.rs
                             : S.parts + dof + (size_t)slot * S.ps;
    if (lane == 0) {
        row[0] = qid;
        row[1] = min(count, lgood);
        row[2] = 0;
        row[3] = 0;
    }
    wave_rank(T, t, beg, end, lgood, count, row + 4, complete ? nullptr : row + (S.rs), xs);
}

// LK: the window-line set the shard's uniform table answers from (8: counts <= 8, 16: 9..16, 32: 17..32; 0: none).
// A window of that set spans at most LK / 2 buckets on either side, so a query whose bucket lies that far inside the
// shard has the same window locally as globally.
// A workgroup of WG threads takes QB queries of the replicated batch (shard_qb / shard_wg: 1,024 over 256 threads, or 256
// over one wave for LK 32): their 20 * QB bytes of targets come in as coalesced 16-byte non-temporal loads into LDS
// (5 * QB / (4 * WG) per thread, all in flight at once: a lane-per-query form had only three
// small loads in flight per lane and read the batch at ~2 TB/s, 10.6 us per 1M with nothing in reach), the in-reach
// ones are compacted (at N ranks a shard reaches ~1/N of the batch), then answered WG at a time: the window line of
// the count's set for queries far enough inside the shard, the wave path on the global window for the rest.
// Complete rows of the workgroup's queries go to region (workgroup index) % 8 of their home rank home_of_block(k):
// one atomic per workgroup and home rank (usually one per workgroup).
template <int LK, uint32_t QB, uint32_t WG>
__global__ __launch_bounds__(WG) void rt_shard_kernel(DevTable T, ShardCtx S, const uint8_t* __restrict__ targets,
                                                      uint32_t q, uint32_t count, uint32_t aligned16, uint32_t abl) {
    // abl (tools build only, KAD_SHARD_ABL; results wrong on purpose): 1 = no wave path (edge queries dropped),
    // 2 = no line work either (the load and the reach compaction alone), 4 = plain (not non-temporal) target loads,
    // 8 = the target load alone
    constexpr uint32_t MARGIN = LK == 8 ? 4u : LK == 16 ? 8u : 16u;
    constexpr uint32_t NR = QB / WG;     // WG-query chunks per workgroup (the reach test)
    constexpr uint32_t NH = QB / BLOCK;  // 256-query home blocks per workgroup (the row slots)
    constexpr uint32_t NW = WG / 64;     // waves
    static_assert(QB % BLOCK == 0 && QB % WG == 0 && (5 * QB) % (4 * WG) == 0, "shard workgroup shape");
    __shared__ __attribute__((aligned(16))) uint32_t st[QB * 5];  // the block's targets, as stored
    __shared__ uint16_t cq[QB];                                   // in-reach queries (block-local index)
    __shared__ uint32_t c_w[NW + 1];
    __shared__ uint64_t xs[NW][192];
    __shared__ uint32_t wcnt[NH][NW], qbase_slot[NH];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint64_t base = (uint64_t)blockIdx.x * QB;
    const uint32_t nq = (uint32_t)min<uint64_t>(QB, q - base);
    {  // the block's 20 * nq bytes
        const uint32_t nw = 5 * nq;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(targets) + 5 * base;
        uint32_t o = 0;
        if (aligned16) {  // (targets 16-byte aligned; 5 * base dwords is a multiple of 4)
            const uint32_t n4 = nw / 4;
            const u32x4_t* s4 = reinterpret_cast<const u32x4_t*>(src);
            u32x4_t* d4 = reinterpret_cast<u32x4_t*>(st);
            if (abl & 4) {
#pragma unroll
                for (uint32_t k = 0; k < 5 * QB / (4 * WG); k++) {
                    const uint32_t x = tid + k * WG;
                    if (x < n4) d4[x] = s4[x];
                }
            } else {
                // every piece's load issued before the first LDS write: unconditional loads (a lane past the block's
                // pieces re-reads its last one, n4 >= 1), guarded writes — with the guard around each load the
                // compiler waited for each round's load before issuing the next
                constexpr uint32_t K = 5 * QB / (4 * WG);
                u32x4_t v[K];
#pragma unroll
                for (uint32_t k = 0; k < K; k++) v[k] = __builtin_nontemporal_load(s4 + min(tid + k * WG, n4 - 1u));
#pragma unroll
                for (uint32_t k = 0; k < K; k++)
                    if (tid + k * WG < n4) d4[tid + k * WG] = v[k];
            }
            o = 4 * n4;
        }
        for (uint32_t x = o + tid; x < nw; x += WG) st[x] = __builtin_nontemporal_load(src + x);
    }
    __syncthreads();
    if (abl & 8) {
        if (st[tid] == 0x5EEDF00Du && st[tid + 1] == 0x5EEDF00Du) S.ctr[KAD_SHARD_COUNTER_STRIDE * 9u] = 1u;  // (keeps the load)
        return;
    }
    // the queries within the shard's reach, compacted: thread tid tests queries tid + r * WG; a ballot per r
    // places them within the wave, the waves' totals (one barrier) place the waves (the order is free: rows carry
    // their qid). A workgroup with none in reach is done.
    uint32_t nnear;  // (block-uniform)
    {
        uint64_t mr[NR];
        uint32_t tw = 0;
#pragma unroll
        for (uint32_t r = 0; r < NR; r++) {
            const uint32_t j = r * WG + tid;
            bool in = false;
            if (j < nq) {
                Target th;
                th.hi = ((uint64_t)__builtin_bswap32(st[5 * j]) << 32) | __builtin_bswap32(st[5 * j + 1]);
                const uint32_t b = shard_bucket(S, th);
                in = b >= S.reach_lo && b < S.reach_hi;
            }
            mr[r] = __ballot(in);
            tw += (uint32_t)__builtin_popcountll(mr[r]);
        }
        if (lane == 0) c_w[w] = tw;
        __syncthreads();
        uint32_t pos = 0;
        nnear = 0;
        for (uint32_t k = 0; k < NW; k++) {
            pos += k < w ? c_w[k] : 0u;
            nnear += c_w[k];
        }
        if (nnear == 0) return;
#pragma unroll
        for (uint32_t r = 0; r < NR; r++) {
            if (mr[r] >> lane & 1u) cq[pos + lanes_below(mr[r])] = (uint16_t)(r * WG + tid);
            pos += (uint32_t)__builtin_popcountll(mr[r]);
        }
        __syncthreads();
    }
    // the compacted queries, WG at a time (block-uniform loop)
    for (uint32_t c0 = 0; c0 < nnear; c0 += WG) {
        const uint32_t k = c0 + tid;
        const bool act = k < nnear;
        const uint32_t j = act ? cq[k] : 0u;
        Target t{};
        uint32_t b = 0, i = 0;
        if (act) {
            const uint32_t* p = st + 5 * j;
            t.hi = ((uint64_t)__builtin_bswap32(p[0]) << 32) | __builtin_bswap32(p[1]);
            t.t2 = __builtin_bswap32(p[2]);
            t.t3 = __builtin_bswap32(p[3]);
            t.t4 = __builtin_bswap32(p[4]);
            b = shard_bucket(S, t);
            i = (uint32_t)base + j;
        }
        const bool line = LK && act && b >= S.s_lo + MARGIN && b + MARGIN <= S.s_hi && !(abl & 2);
        bool edge = act && !(abl & 3);
        if (LK) {  // (a round without line queries reserves nothing: its counts are zero and no wave has line work)
            // the row slots are reserved before the lines are read (one atomic per home block sb with line
            // queries in this round: its rows go to region sb % 8 of its home rank), so the atomic's round trip
            // overlaps the line loads; a query its line cannot answer leaves a tombstone row (qid KAD_NO_NODE, skipped
            // by the finish) and takes the wave path
            const uint32_t sb = act ? j / BLOCK : 0u;
            uint32_t slot = 0;
#pragma unroll
            for (uint32_t r = 0; r < NH; r++) {
                const uint64_t mb = __ballot(line && sb == r);
                if (lane == 0) wcnt[r][w] = (uint32_t)__builtin_popcountll(mb);
                if (line && sb == r) slot = lanes_below(mb);
            }
            __syncthreads();
            // one atomic per home rank among the workgroup's 256-query blocks (usually one), issued by thread 0
            // before its wave's line work; the bases are written to LDS after it, so that the atomic's round trip
            // overlaps the line loads of wave 0 too
            uint32_t tot[NH], hm[NH], ab[NH];
            if (tid == 0) {
#pragma unroll
                for (uint32_t r = 0; r < NH; r++) {
                    tot[r] = 0;
                    for (uint32_t x = 0; x < NW; x++) tot[r] += wcnt[r][x];
                    hm[r] = S.dests > 1 ? home_of_block((uint32_t)(base / BLOCK) + r, S.dests, S.nblk) : 0u;
                }
#pragma unroll
                for (uint32_t r = 0; r < NH; r++) {
                    ab[r] = 0;
                    if (r == 0 || hm[r] != hm[r - 1]) {  // (homes ascend with the block)
                        uint32_t run = 0;
                        for (uint32_t y = r; y < NH; y++) run += hm[y] == hm[r] ? tot[y] : 0u;
                        if (run)
                            ab[r] = atomicAdd(S.ctr + (uint64_t)hm[r] * S.dest_words +
                                              KAD_SHARD_COUNTER_STRIDE * (blockIdx.x & 7u), run);
                    }
                }
            }
            uint32_t o[LK ? LK : 1], m = 0;
            bool ok = false;
            if (__any(line)) {  // (a wave of idle lanes skips the line work)
                const uint32_t bl = line ? b - S.s_lo : 0u;
                if constexpr (LK == 8) ok = line8_answer(T, t, bl, count, line, line && (T.flags & TF_WS), o, m);
                else if constexpr (LK == 16) ok = wl16_answer(T, t, bl, count, line, o, m);
                else if constexpr (LK == 32) ok = wl32_answer(T, t, bl, count, line, o, m);
                ok = ok && line;
            }
            if (tid == 0) {
                uint32_t acc = 0;
#pragma unroll
                for (uint32_t r = 0; r < NH; r++) {
                    if (r == 0 || hm[r] != hm[r - 1]) acc = ab[r];
                    qbase_slot[r] = acc;
                    acc += tot[r];
                }
            }
            __syncthreads();
            if (line) {
                for (uint32_t x = 0; x < w; x++) slot += wcnt[sb][x];
                slot += qbase_slot[sb];
                const uint32_t kb = (uint32_t)(base / BLOCK) + sb;
                const uint64_t dof = S.dests > 1 ? (uint64_t)home_of_block(kb, S.dests, S.nblk) * S.dest_words : 0ull;
                if (slot < S.row_cap) {
                    uint32_t* row = S.rows + dof + ((size_t)(blockIdx.x & 7u) * S.row_cap + slot) * S.rs;
                    if (ok) {
                        reinterpret_cast<uint4*>(row)[0] = make_uint4(i, m, 0u, 0u);
                        if constexpr (LK == 8) store_row8(row + 4, o, count);
                        else if constexpr (LK == 16) store_row16(row + 4, o, count);
                        else if constexpr (LK == 32) store_row32(row + 4, o, count);
                        edge = false;
                    } else {
                        reinterpret_cast<uint4*>(row)[0] = make_uint4(NONE, 0u, 0u, 0u);  // tombstone
                    }
                } else {
                    atomicOr(S.ctr + dof + KAD_SHARD_COUNTER_STRIDE * 9u, 1u);
                }
            }
            if (c0 + WG < nnear) __syncthreads();  // (wcnt / qbase_slot reused by the next round; block-uniform)
        }
        for (uint64_t mm = __ballot(edge); mm; mm &= mm - 1) {
            const uint32_t l = (uint32_t)__builtin_ctzll(mm);
            Target u;
            u.hi = rdl64(t.hi, l);
            u.t2 = rdl(t.t2, l);
            u.t3 = rdl(t.t3, l);
            u.t4 = rdl(t.t4, l);
            wave_shard(T, S, u, rdl(i, l), count, blockIdx.x & 7u, xs[w]);
        }
    }
}

// A complete row's `count` indices (at src + 4) copied to dst by `lpr` lanes: lane `sub` moves the row's 16-byte
// pieces sub, sub + lpr, ... (counts that are multiples of 4, both ends 16-byte aligned), or its words sub, sub + lpr,
// ... otherwise. A row of k = 32 leaves as eight lanes' 16-byte stores instead of one lane's 32 dword stores into
// 64 different lines per instruction.
__host__ __device__ constexpr uint32_t scatter_lpr(uint32_t count) {
    return count <= 4 ? 1u : count <= 8 ? 2u : count <= 16 ? 4u : 8u;
}

__device__ __forceinline__ void copy_row(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t count,
                                         uint32_t sub, uint32_t lpr) {
    if ((count & 3u) == 0 && (((uintptr_t)(src + 4) | (uintptr_t)dst) & 15u) == 0) {
        for (uint32_t j = 4 * sub; j < count; j += 4 * lpr)
            *reinterpret_cast<uint4*>(dst + j) = *reinterpret_cast<const uint4*>(src + 4 + j);
    } else {
        for (uint32_t j = sub; j < count; j += lpr) dst[j] = src[4 + j];
    }
}

// Gathered complete rows -> out rows. Block r of n_blocks holds n_rows[r] rows of `stride` words at
// rows + r * block_cap * stride; scatter_lpr(count) lanes per row.
__global__ void scatter_rows_kernel(const uint32_t* __restrict__ rows, const uint32_t* __restrict__ n_rows,
                                    uint32_t n_rows_stride, uint32_t n_blocks, uint32_t block_cap, uint32_t stride,
                                    uint32_t count,
                                    uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    const uint32_t lpr = scatter_lpr(count);
    const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x, g = t / lpr;
    const uint32_t sub = (uint32_t)(t % lpr);
    const uint32_t r = (uint32_t)(g / block_cap), k = (uint32_t)(g % block_cap);
    if (r >= n_blocks || k >= min(n_rows[(size_t)r * n_rows_stride], block_cap)) return;
    const uint32_t* src = rows + ((size_t)r * block_cap + k) * stride;
    const uint32_t qid = src[0];
    if (qid == NONE) return;  // (a tombstone: the query's row comes from the wave path)
    if (out_cnt && sub == 0) out_cnt[qid] = (uint8_t)src[1];
    copy_row(src, out_idx + (size_t)qid * count, count, sub, lpr);
}

// Partial rows sorted by qid: the thread of a qid segment's first row merges the segment's sorted
// lists by (XOR distance, global index) and writes the first min(count, sum of m) entries.
__global__ void merge_parts_kernel(const uint32_t* __restrict__ parts, uint32_t n, uint32_t rs, uint32_t ps,
                                   uint32_t count, uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint32_t qid = parts[(size_t)i * ps];
    if (i > 0 && parts[(size_t)(i - 1) * ps] == qid) return;
    uint32_t e = i + 1;
    while (e < n && parts[(size_t)e * ps] == qid) e++;
    constexpr uint32_t MAXSEG = 16;
    uint32_t head[MAXSEG], total = 0;
    const uint32_t nseg = min(e - i, MAXSEG);
    for (uint32_t s = 0; s < nseg; s++) {
        head[s] = 0;
        total += parts[(size_t)(i + s) * ps + 1];
    }
    const uint32_t m = min(count, total);
    uint32_t* dst = out_idx + (size_t)qid * count;
    for (uint32_t p = 0; p < count; p++) {
        if (p >= m) {
            dst[p] = NONE;
            continue;
        }
        uint32_t best = NONE;
        for (uint32_t s = 0; s < nseg; s++) {
            const uint32_t* r = parts + (size_t)(i + s) * ps;
            if (head[s] >= r[1]) continue;
            if (best == NONE) { best = s; continue; }
            const uint32_t* rb = parts + (size_t)(i + best) * ps;
            const uint32_t* da = r + rs + 5 * head[s];
            const uint32_t* db = rb + rs + 5 * head[best];
            int c = 0;
            for (int w = 0; w < 5 && c == 0; w++) c = da[w] < db[w] ? -1 : da[w] > db[w] ? 1 : 0;
            if (c < 0 || (c == 0 && r[4 + head[s]] < rb[4 + head[best]])) best = s;
        }
        const uint32_t* rb = parts + (size_t)(i + best) * ps;
        dst[p] = rb[4 + head[best]];
        head[best]++;
    }
    if (out_cnt) out_cnt[qid] = (uint8_t)m;
}

// ---------------------------------------------------------------------------------------
// The all-gathered step of the north-star variant (kad_rt_gather_finish). A rank's send block is its
// kad_rt_shard_batch output in place: KAD_SHARD_REGIONS regions of row_cap complete rows, then part_cap
// partial rows, then the counters (KAD_SHARD_BLOCK_WORDS). After one all-gather of fixed-size blocks,
// block r of the received buffer is rank r's, and every count the kernels need is read on the device:
// no host read between the shard kernel, the collective and the merge, so a step can be captured in a
// graph. Parts of one query are chained through a per-query head word (atomicExch), merged by the
// thread of the chain's head, and the head is reset to NONE for the next step.
// ---------------------------------------------------------------------------------------
struct GatherCtx {
    const uint32_t* recv;
    uint64_t block;               // words per rank block
    uint64_t parts_off, ctr_off;  // word offsets of the parts and the counters inside a block
    uint32_t world, row_cap, part_cap, rs, ps, count, q;
    uint32_t qbase;               // rows of qids [qbase, qbase + q) (the home range; 0 for the all-gather)
};

__device__ __forceinline__ const uint32_t* gather_ctr(const GatherCtx& G, uint32_t r) {
    return G.recv + (size_t)r * G.block + G.ctr_off;
}

// The complete rows of (rank r, region g) = pair p, by the spb workgroups of that pair: each reads the region's count
// once and strides over its rows only, instead of one thread per row CAPACITY (a launch sized for the worst case, most
// of whose workgroups found nothing to copy: 8.4 us for ~131k rows at N = 8).
__device__ __forceinline__ void gather_scatter_pair(const GatherCtx& G, uint32_t b, uint32_t spb,
                                                    uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt,
                                                    uint32_t* __restrict__ overflow) {
    const uint32_t lpr = scatter_lpr(G.count), p = b / spb, j = b % spb;
    const uint32_t r = p / KAD_SHARD_REGIONS, region = p % KAD_SHARD_REGIONS;
    if (r >= G.world) return;
    const uint32_t* ctr = gather_ctr(G, r);
    if (region == 0 && j == 0 && threadIdx.x == 0 && ctr[KAD_SHARD_COUNTER_STRIDE * 9u] && overflow) atomicOr(overflow, 1u);
    const uint32_t n = min(ctr[KAD_SHARD_COUNTER_STRIDE * region], G.row_cap), rpb = BLOCK / lpr;
    const uint32_t sub = threadIdx.x % lpr;
    const uint32_t* base = G.recv + (size_t)r * G.block + (size_t)region * G.row_cap * G.rs;
    for (uint32_t k = j * rpb + threadIdx.x / lpr; k < n; k += spb * rpb) {
        const uint32_t* src = base + (size_t)k * G.rs;
        const uint32_t qid = src[0] - G.qbase;
        if (qid >= G.q) continue;  // (tombstones too: NONE - qbase >= q)
        if (out_cnt && sub == 0) out_cnt[qid] = (uint8_t)src[1];
        copy_row(src, out_idx + (size_t)qid * G.count, G.count, sub, lpr);
    }
}

// Workgroups per (rank, region) pair of gather_scatter_pair: about two rows per thread at a full region.
inline uint32_t scatter_spb(uint32_t row_cap, uint32_t count) {
    const uint64_t threads = (uint64_t)row_cap * scatter_lpr(count);
    return (uint32_t)std::min<uint64_t>(1024, std::max<uint64_t>(1, (threads + 2 * BLOCK - 1) / (2 * BLOCK)));
}

// The counters of `n` send blocks (block_words apart, the counters at ctr_off) zeroed before a step.
__global__ void zero_counters_kernel(uint32_t* send, uint32_t n, uint64_t block_words, uint64_t ctr_off) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    const uint32_t words = KAD_SHARD_COUNTERS * KAD_SHARD_COUNTER_STRIDE;
    if (j >= n * words) return;
    send[(uint64_t)(j / words) * block_words + ctr_off + j % words] = 0;
}

// Part x = (rank r, slot p) of the gathered buffer, or NULL if the slot is empty.
__device__ __forceinline__ const uint32_t* gather_part(const GatherCtx& G, uint64_t x) {
    const uint32_t r = (uint32_t)(x / G.part_cap), p = (uint32_t)(x % G.part_cap);
    if (r >= G.world || p >= min(gather_ctr(G, r)[KAD_SHARD_COUNTER_STRIDE * 8u], G.part_cap)) return nullptr;
    return G.recv + (size_t)r * G.block + G.parts_off + (size_t)p * G.ps;
}

// One launch for the two independent passes of a finish: blocks [0, sblocks) scatter the complete rows, the others
// link each part into its query's chain (the merge that walks the chains is the next launch).
__global__ __launch_bounds__(BLOCK) void gather_scatter_link_kernel(GatherCtx G, uint32_t sblocks, uint32_t spb,
                                                                    uint32_t* __restrict__ out_idx,
                                                                    uint8_t* __restrict__ out_cnt,
                                                                    uint32_t* __restrict__ overflow,
                                                                    uint32_t* __restrict__ head,
                                                                    uint32_t* __restrict__ next) {
    if (blockIdx.x < sblocks) {  // block-uniform
        gather_scatter_pair(G, blockIdx.x, spb, out_idx, out_cnt, overflow);
        return;
    }
    const uint64_t x = (uint64_t)(blockIdx.x - sblocks) * BLOCK + threadIdx.x;
    const uint32_t* part = gather_part(G, x);
    if (!part || part[0] - G.qbase >= G.q) return;
    next[x] = atomicExch(head + (part[0] - G.qbase), (uint32_t)x);
}

// (a, ai) < (b, bi): 160-bit XOR distance, then global index
__device__ __forceinline__ bool dist_idx_less(const uint32_t* a, uint32_t ai, const uint32_t* b, uint32_t bi) {
#pragma unroll
    for (int w = 0; w < 5; w++)
        if (a[w] != b[w]) return a[w] < b[w];
    return ai < bi;
}

// One query's parts (the chain from part xh: at most one per rank, KAD_SHARD_MAX_WORLD) merged by (XOR distance,
// global index) by the whole wave (wave-uniform arguments). Up to 64 entries in all: lane e loads entry e (one round
// of independent loads) and counts the entries before it, 6 words broadcast per entry; the row entry at that rank is
// the lane's. More entries: lane 0 merges the sorted parts serially, as merge_parts_kernel.
__device__ void wave_merge_chain(const GatherCtx& G, const uint32_t* __restrict__ next, uint32_t xh, uint32_t qid,
                                 uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    constexpr uint32_t MAXSEG = KAD_SHARD_MAX_WORLD;
    const uint32_t lane = threadIdx.x & 63u, count = G.count;
    uint32_t ys = NONE, nseg = 0;  // lane s < nseg: part slot of segment s
    for (uint32_t y = xh; y != NONE && nseg < MAXSEG; y = next[y]) {
        if (lane == nseg) ys = y;
        nseg++;
    }
    const uint32_t* myseg = lane < nseg ? gather_part(G, ys) : nullptr;
    const uint32_t cnt = myseg ? myseg[1] : 0u;
    uint32_t off = cnt;  // inclusive scan over the segments (nseg <= 16 lanes)
#pragma unroll
    for (int o = 1; o < (int)MAXSEG; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)off, o, 64);
        if (lane >= (uint32_t)o) off += y;
    }
    const uint32_t total = rdl(off, MAXSEG - 1), m = min(count, total);
    uint32_t* dst = out_idx + (size_t)qid * count;
    if (total <= 64) {
        // lane e: entry e of segment s (off[s-1] <= e < off[s])
        uint32_t s = 0;
        for (uint32_t k = 0; k + 1 < nseg; k++) s += rdl(off, k) <= lane ? 1u : 0u;
        const bool has = lane < total;
        const uintptr_t sp = (uintptr_t)myseg;  // (the shuffles run in every lane)
        const uint32_t* sg = reinterpret_cast<const uint32_t*>(
            (uintptr_t)(uint32_t)__shfl((int)(uint32_t)sp, (int)s, 64) |
            ((uintptr_t)(uint32_t)__shfl((int)(uint32_t)(sp >> 32), (int)s, 64) << 32));
        const uint32_t ofs = (uint32_t)__shfl((int)off, (int)(s ? s - 1 : 0), 64);
        const uint32_t e = lane - (s ? ofs : 0u);
        uint32_t d[5] = {0, 0, 0, 0, 0}, idx = NONE;
        if (has) {
            idx = sg[4 + e];
#pragma unroll
            for (int w = 0; w < 5; w++) d[w] = sg[G.rs + 5 * e + w];
        }
        uint32_t rank = 0;
        for (uint32_t j = 0; j < total; j++) {
            uint32_t b[5];
#pragma unroll
            for (int w = 0; w < 5; w++) b[w] = rdl(d[w], j);
            rank += dist_idx_less(b, rdl(idx, j), d, idx) ? 1u : 0u;
        }
        if (has && rank < m) dst[rank] = idx;
        if (lane >= m && lane < count) dst[lane] = NONE;
        if (count > 64)
            for (uint32_t p = 64 + lane; p < count; p += 64) dst[p] = NONE;
    } else if (lane == 0) {
        const uint32_t* seg[MAXSEG];
        uint32_t at[MAXSEG];
        {
            uint32_t k = 0;
            for (uint32_t y = xh; y != NONE && k < MAXSEG; y = next[y]) {
                seg[k] = gather_part(G, y);
                at[k++] = 0;
            }
        }
        for (uint32_t p = 0; p < count; p++) {
            if (p >= m) {
                dst[p] = NONE;
                continue;
            }
            uint32_t best = NONE;
            for (uint32_t k = 0; k < nseg; k++) {
                if (at[k] >= seg[k][1]) continue;
                if (best == NONE ||
                    dist_idx_less(seg[k] + G.rs + 5 * at[k], seg[k][4 + at[k]], seg[best] + G.rs + 5 * at[best],
                                  seg[best][4 + at[best]]))
                    best = k;
            }
            dst[p] = seg[best][4 + at[best]];
            at[best]++;
        }
    }
    if (lane == 0 && out_cnt) out_cnt[qid] = (uint8_t)m;
}

// The chain heads (the first part of each query's chain) merge their query's parts (wave_merge_chain) and reset the
// head. One WAVE per part slot (wave-uniform x): the chains merge side by side, each a few dependent memory round
// trips, instead of a wave walking the ~64 chain heads of its 64 slots one after another (8.5 us at N = 8 for a
// few thousand parts; profiles/r06/merge/).
constexpr uint32_t MERGE_WPB = BLOCK / 64;  // part slots per workgroup
__global__ __launch_bounds__(BLOCK) void gather_merge_kernel(GatherCtx G, uint32_t* __restrict__ head,
                                                             const uint32_t* __restrict__ next,
                                                             uint32_t* __restrict__ out_idx,
                                                             uint8_t* __restrict__ out_cnt, uint32_t mblocks,
                                                             uint32_t* __restrict__ zsend) {
    if (blockIdx.x >= mblocks) {  // kad_rt_home_finish_reset: the send blocks' counters for the next step
        const uint32_t j = (blockIdx.x - mblocks) * BLOCK + threadIdx.x, words = KAD_SHARD_COUNTERS * KAD_SHARD_COUNTER_STRIDE;
        if (j < G.world * words) zsend[(uint64_t)(j / words) * G.block + G.ctr_off + j % words] = 0;
        return;
    }
    const uint64_t x = (uint64_t)blockIdx.x * MERGE_WPB + (threadIdx.x >> 6);  // wave-uniform
    const uint32_t* part = gather_part(G, x);
    if (!part) return;
    const uint32_t qid = part[0] - G.qbase;
    if (qid >= G.q || head[qid] != (uint32_t)x) return;  // (parts are rare: queries whose window crosses a shard edge)
    wave_merge_chain(G, next, (uint32_t)x, qid, out_idx, out_cnt);
    if ((threadIdx.x & 63u) == 0) head[qid] = NONE;
}

// ---------------------------------------------------------------------------------------
// Wire step after the query
// NetworkEngine::bufferNodes (network_engine.cpp:942-974): a query's candidate nodes sorted by
// XOR distance to the target (std::sort on xorCmp, :945-947), the first SEND_NODES = 8 (:948),
// each packed as its 20-byte ID followed by the stored address + port bytes (26-byte v4 records,
// 38-byte v6 records). One lane per query: a register top-8 over the exact 160-bit distance
// (ties, i.e. duplicate IDs, keep input order), then byte stores of the records.
// ---------------------------------------------------------------------------------------
constexpr uint32_t SEND_NODES = 8;

// Per-node wire records, built once by kad_table_set_addrs: the node's 20-byte ID then its address
// + port bytes, padded to WREC4 = 32 / WREC6 = 48 bytes so a record is two or three aligned 16-byte
// loads. A query's candidates (one window of adjacent nodes) share a few lines of this array.
constexpr uint32_t WREC4 = 32, WREC6 = 48;

__global__ void wrec_build_kernel(const uint64_t* key, const uint32_t* tail, const uint8_t* addr, uint32_t al,
                                  uint32_t n, uint32_t* wrec) {
    const uint32_t v = blockIdx.x * BLOCK + threadIdx.x;
    if (v >= n) return;
    const uint32_t words = (al == KAD_ADDR4_LEN ? WREC4 : WREC6) / 4;
    uint32_t w[WREC6 / 4] = {0};
    const uint64_t k = key[v];
    w[0] = __builtin_bswap32((uint32_t)(k >> 32));
    w[1] = __builtin_bswap32((uint32_t)k);
    for (int x = 0; x < 3; x++) w[2 + x] = __builtin_bswap32(tail[3ull * v + x]);
    for (uint32_t b = 0; b < al; b++) w[(KAD_HASH_LEN + b) >> 2] |= (uint32_t)addr[(size_t)al * v + b] << (8 * (b & 3));
    for (uint32_t x = 0; x < words; x++) wrec[(size_t)words * v + x] = w[x];
}

// P lanes per query (P = the candidate count rounded up to a power of two, 8..32): lane j loads
// candidate j's wire record, ranks it against the other candidates of its query by the exact 160-bit
// XOR distance (shuffles within the segment; ties keep input order), and the 8 best write their
// records at byte rank * REC of the query's row in LDS; the block's rows, contiguous in `out`, then
// leave as coalesced 16-byte stores.
template <uint32_t AL, uint32_t P>
__global__ __launch_bounds__(BLOCK) void buffer_nodes_kernel(uint32_t n_nodes, uint32_t index_base,
                                                             const uint4* __restrict__ wrec,
                                                             const uint8_t* __restrict__ targets, uint32_t q,
                                                             const uint32_t* __restrict__ idx,
                                                             const uint8_t* __restrict__ cnt, uint32_t k,
                                                             uint8_t* __restrict__ out, uint8_t* __restrict__ out_n) {
    constexpr uint32_t RQ = (AL == KAD_ADDR4_LEN ? WREC4 : WREC6) / 16;  // 16-byte pieces per record
    constexpr uint32_t REC = KAD_HASH_LEN + AL;                          // 26 / 38 bytes
    constexpr uint32_t ROW = SEND_NODES * REC;                           // 208 / 304 bytes
    constexpr uint32_t QB = BLOCK / P;                                   // queries per block
    __shared__ uint4 rows[QB * ROW / 16];
    const uint32_t tid = threadIdx.x, ql = tid / P, j = tid % P;
    const uint32_t q0 = blockIdx.x * QB, qi = q0 + ql;
    const uint32_t nq = min(QB, q - q0);
    for (uint32_t x = tid; x < nq * ROW / 16; x += BLOCK) rows[x] = make_uint4(0, 0, 0, 0);
    bool valid = false;
    uint32_t r[RQ * 4];
    uint64_t d0 = ~0ull, d1 = ~0ull;
    uint32_t d2 = NONE;
    if (qi < q) {
        const uint32_t n = cnt ? min((uint32_t)cnt[qi], k) : k;
        const uint32_t g = j < n ? idx[(size_t)qi * k + j] : NONE;
        const uint32_t v = g - index_base;
        valid = j < n && g != NONE && v < n_nodes;
        if (valid) {
            const Target t = load_target(targets, qi);
#pragma unroll
            for (int x = 0; x < (int)RQ; x++) {
                const uint4 p = wrec[(size_t)RQ * v + x];
                r[4 * x] = p.x; r[4 * x + 1] = p.y; r[4 * x + 2] = p.z; r[4 * x + 3] = p.w;
            }
            d0 = (((uint64_t)__builtin_bswap32(r[0]) << 32) | __builtin_bswap32(r[1])) ^ t.hi;
            d1 = ((uint64_t)(__builtin_bswap32(r[2]) ^ t.t2) << 32) | (__builtin_bswap32(r[3]) ^ t.t3);
            d2 = __builtin_bswap32(r[4]) ^ t.t4;
        }
    }
    // rank within the segment of P lanes (invalid lanes sort last and never count)
    const uint64_t vm = __ballot(valid);
    const uint32_t seg = (tid & 63u) & ~(P - 1);
    uint32_t rank = 0;
#pragma unroll 4
    for (uint32_t p = 0; p < P; p++) {
        const int src = (int)(seg + p);
        const uint64_t e0 = ((uint64_t)(uint32_t)__shfl((int)(d0 >> 32), src, 64) << 32) | (uint32_t)__shfl((int)d0, src, 64);
        const uint64_t e1 = ((uint64_t)(uint32_t)__shfl((int)(d1 >> 32), src, 64) << 32) | (uint32_t)__shfl((int)d1, src, 64);
        const uint32_t e2 = (uint32_t)__shfl((int)d2, src, 64);
        const bool ev = (vm >> src) & 1ull;
        const bool less = e0 < d0 || (e0 == d0 && (e1 < d1 || (e1 == d1 && (e2 < d2 || (e2 == d2 && p < j)))));
        rank += ev && less;
    }
    __syncthreads();  // zero fill done
    if (valid && rank < SEND_NODES) {
        uint16_t* dst = reinterpret_cast<uint16_t*>(reinterpret_cast<uint8_t*>(rows) + ql * ROW + rank * REC);
#pragma unroll
        for (int h = 0; h < (int)REC / 2; h++) dst[h] = (uint16_t)(r[h >> 1] >> (16 * (h & 1)));
    }
    if (j == 0 && qi < q && out_n) {
        const uint32_t segm = (uint32_t)((vm >> seg) & (P == 64 ? ~0ull : ((1ull << P) - 1)));
        out_n[qi] = (uint8_t)min((uint32_t)__builtin_popcount(segm), SEND_NODES);
    }
    __syncthreads();
    uint4* dst = reinterpret_cast<uint4*>(out + (size_t)q0 * ROW);
    for (uint32_t x = tid; x < nq * ROW / 16; x += BLOCK) dst[x] = rows[x];
}

// NetworkEngine::isMartian (network_engine.cpp:308-339) on address + port bytes; v4prefix = ::ffff:0:0/96.
__device__ __forceinline__ bool is_martian(const uint8_t* a, uint32_t al) {
    if (al == 6) return (a[4] == 0 && a[5] == 0) || a[0] == 0 || a[0] == 127 || (a[0] & 0xE0) == 0xE0;
    bool z15 = true, v4m = a[10] == 0xFF && a[11] == 0xFF;
    for (int b = 0; b < 15; b++) z15 &= a[b] == 0;
    for (int b = 0; b < 10; b++) v4m &= a[b] == 0;
    return (a[16] == 0 && a[17] == 0) || a[0] == 0xFF || (a[0] == 0xFE && (a[1] & 0xC0) == 0x80) ||
           (z15 && (a[15] == 0 || a[15] == 1)) || v4m;
}

struct Id20 {
    uint8_t b[KAD_HASH_LEN];
};

// NetworkEngine::deserializeNodes' filter (network_engine.cpp:788-828): keep = not our own ID
// (:798-799) and not a martian address (:806, :822), per 26- or 38-byte record.
__global__ void parse_nodes_kernel(const uint8_t* __restrict__ in, uint32_t n, uint32_t rec_len, Id20 myid,
                                   uint8_t* __restrict__ keep) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    const uint8_t* r = in + (size_t)rec_len * i;
    bool mine = true;
    for (int b = 0; b < (int)KAD_HASH_LEN; b++) mine &= r[b] == myid.b[b];
    keep[i] = !(mine || is_martian(r + KAD_HASH_LEN, rec_len - KAD_HASH_LEN));
}

__global__ __launch_bounds__(BLOCK) void find_bucket_kernel(DevTable T, const uint8_t* __restrict__ targets,
                                                            uint32_t q, uint32_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    out[i] = T.B == 0 ? NONE : locate_bucket(T, load_target(targets, i));
}

// ---------------------------------------------------------------------------------------
// NodeCache::getCachedNodes, one query per lane (node_cache.cpp:36-66): two-pointer walk from
// lower_bound(t): p = lb-1 (or lb at begin), n = lb; take the closer (xorCmp(p, n) < 0 -> p);
// taking begin() exhausts p; emit non-expired nodes, stop at count. (Serial form: counts > 16 and
// the group kernel's rare fallback.) Inlined: as a call, the stack it needs made every kernel calling it ~2x slower
// (profiles/r06/ncl_lane/ncl_lane10).
__device__ void nc_serial(const DevTable& T, const Target& t, uint32_t count, uint32_t* row, uint8_t* cp) {
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
    if (cp) *cp = (uint8_t)min(m, 255u);  // saturates (a count above 255 reads the length off the padding)
}

__global__ __launch_bounds__(BLOCK) void nc_closest_kernel(DevTable T, const uint8_t* __restrict__ targets,
                                                           uint32_t q, uint32_t count,
                                                           uint32_t* __restrict__ out_idx,
                                                           uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    nc_serial(T, load_target(targets, i), count, out_idx + (size_t)i * count, out_cnt ? out_cnt + i : nullptr);
}

// Any count on the dual-family batch (counts above 64): the serial walk, one lane per query on its family's map.
__global__ __launch_bounds__(BLOCK) void nc_closest_dual_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ af,
                                                                const uint8_t* __restrict__ targets, uint32_t q,
                                                                uint32_t count, uint32_t* __restrict__ out_idx,
                                                                uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    nc_serial(af[i] ? T6 : T4, load_target(targets, i), count, out_idx + (size_t)i * count, out_cnt ? out_cnt + i : nullptr);
}

// NodeCache::getCachedNodes, one wave per query (count <= 32). The walk is a greedy merge of the
// left run a_k = lb-1-k and the right run b_k = lb+k by XOR distance (distinct IDs: no ties; the
// lb == 0 start takes node 0 from the right, which is the same walk with an empty left run). In a
// greedy merge an element's place is its index plus the number of elements of the other run whose
// PREFIX MAXIMUM distance is below its own prefix maximum (tests/test_nodecache_merge.py checks the
// lemma). Lanes 0-31 load a_0..31, lanes 32-63 b_0..31 (top-64 keys and status bytes), take prefix
// maxima with 5 shuffle steps, find their place by a 6-step binary search over the other run's
// (monotone) prefix maxima, and the non-expired ones rank themselves through an LDS bit mask.
// XOR-nearest nodes sit mostly on ONE side of lb (the target's dyadic subtree ends on one side): on
// the bench shard a k = 14 walk takes up to 20 nodes from one side, so each run gets 32 lanes. Lane 0
// walks serially (nc_serial) when a run is longer than 32 and the count-th emission does not come
// before its 32nd element, or when two prefix maxima tie on the top 64 bits (the 160-bit order is
// then needed).
__device__ __forceinline__ uint64_t shfl64(uint64_t v, int src) {
    return ((uint64_t)(uint32_t)__shfl((int)(v >> 32), src, 64) << 32) | (uint32_t)__shfl((int)(uint32_t)v, src, 64);
}

__global__ __launch_bounds__(BLOCK) void nc_group_v1_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                         uint32_t count, uint32_t* __restrict__ out_idx,
                                                         uint8_t* __restrict__ out_cnt) {
    constexpr uint32_t W = 32, G = 64;  // run window, lanes per query
    __shared__ unsigned long long emask[BLOCK / G];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, grp = tid / G;
    const uint32_t qi = blockIdx.x * (BLOCK / G) + grp;
    const bool right = lane >= W;
    const uint32_t k = lane & (W - 1);
    const bool act = qi < q && count > 0;
    const uint32_t N = T.n;
    Target t{};
    uint32_t lb = 0;
    if (act) {
        t = load_target(targets, qi);
        lb = N ? node_lower_bound(T, t) : 0u;
    }
    const uint32_t node = right ? lb + k : lb - 1 - k;
    const bool valid = act && (right ? lb + k < N : lb > k);
    uint64_t m = ~0ull;  // invalid lanes end their run: the maximum
    bool expired = true;
    if (valid) {
        m = T.key[node] ^ t.hi;
        expired = T.status[node] & KAD_STATUS_EXPIRED;
    }
    bool amb = valid && m == ~0ull;  // indistinguishable from the end-of-run sentinel
#pragma unroll
    for (uint32_t s = 1; s < W; s <<= 1) {  // prefix maxima along my run
        const uint64_t o = shfl64(m, (int)lane - (int)s);
        if (k >= s && o > m) m = o;  // unsigned (max() may pick a signed overload)
    }
    // place: my index + the other run's prefix maxima below mine (lower_bound over a monotone run)
    const uint32_t obase = right ? 0u : W;
    uint32_t lo = 0, hi = W;
#pragma unroll
    for (int it = 0; it < 6; it++) {  // 33 possible answers: 6 halvings (a settled lane stays put)
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t v = shfl64(m, (int)(obase + (mid < W ? mid : W - 1)));
        if (lo < hi) {
            if (v < m) lo = mid + 1; else hi = mid;
        }
    }
    const uint64_t at = shfl64(m, (int)(obase + (lo < W ? lo : W - 1)));
    amb |= valid && lo < W && at == m;  // equal top-64 prefix maxima: the 160-bit order decides
    const uint32_t pos = k + lo;
    const bool emit = valid && !expired;
    if (lane == 0) emask[grp] = 0;
    __syncthreads();
    if (emit) atomicOr(&emask[grp], 1ull << pos);
    __syncthreads();
    const uint64_t em = emask[grp];
    const uint32_t tot = (uint32_t)__builtin_popcountll(em);
    uint32_t pstar = 64;  // position of the count-th emission (64: not inside the window)
    if (tot >= count) {
        uint64_t e = em;
        for (uint32_t c = 1; c < count; c++) e &= e - 1;
        pstar = (uint32_t)__builtin_ctzll(e);
    }
    const uint32_t posA = (uint32_t)__shfl((int)pos, (int)(W - 1), 64);
    const uint32_t posB = (uint32_t)__shfl((int)pos, (int)(G - 1), 64);
    const bool ok = !__any(amb) && (lb <= W || posA > pstar) && (lb + W >= N || posB > pstar);
    if (act && ok) {
        uint32_t* row = out_idx + (size_t)qi * count;
        const uint32_t mm = min(tot, count);
        if (emit) {
            const uint32_t rank = (uint32_t)__builtin_popcountll(em & ((1ull << pos) - 1ull));
            if (rank < count) row[rank] = node + T.index_base;
        }
        if (lane >= mm && lane < count) row[lane] = NONE;
        if (lane == 0 && out_cnt) out_cnt[qi] = (uint8_t)mm;
    } else if (act && lane == 0) {
        nc_serial(T, t, count, out_idx + (size_t)qi * count, out_cnt ? out_cnt + qi : nullptr);
    }
}

// The same merge with the lower bound and the runs read from ONE window load (nc_window_kernel):
// the radix slot of t gives [r0, r1), the nodes whose top 64 bits share t's slot; lanes load the 96
// nodes r0-32 .. r0+63 (two loads per lane, independent, issued right after the slot lookup), lb =
// r0 + #(slot nodes < t) is one ballot, and the runs are shuffled out of the window (lb - r0 <= 32
// keeps both 32-runs inside it). This drops the binary search's dependent loads from the chain
// (target -> slot -> window -> answer). Emission ranks come from one ballot: a node's rank is the
// emitting nodes of its own run before it plus those of the other run placed before it (the first
// `lo` of them), so no LDS mask or block barrier. A slot of more than 32 nodes takes the binary
// search and per-lane loads.
// Slot range [r0, r1) of t's top 64 bits (wave-uniform loads).
__device__ __forceinline__ void nc_slot(const DevTable& T, const Target& t, uint32_t& r0, uint32_t& r1) {
    r0 = r1 = 0;
    if (T.n && t.hi >= T.nbase) {
        const uint64_t sl = (t.hi - T.nbase) >> T.nshift;
        if (sl >= T.nslots) {
            r0 = r1 = T.n;
        } else {
            r0 = T.nrdx[sl];
            r1 = T.nrdx[sl + 1];
        }
    }
}

// The window r0-32 .. r0+63: lane l holds nodes r0-32+l (k0, status byte 0 of st) and, for l < 32,
// r0+32+l (k1, status byte 1).
struct NcWindow {
    uint64_t k0, k1;
    uint32_t st;
};
__device__ __forceinline__ NcWindow nc_window(const DevTable& T, uint32_t r0, uint32_t lane) {
    NcWindow w{0, 0, 0};
    const int64_t p0 = (int64_t)r0 - 32 + lane, p1 = p0 + 64;
    if (p0 >= 0 && p0 < (int64_t)T.n) {
        w.k0 = T.key[p0];
        w.st = T.status[p0];
    }
    if (lane < 32 && p1 < (int64_t)T.n) {
        w.k1 = T.key[p1];
        w.st |= (uint32_t)T.status[p1] << 8;
    }
    return w;
}

// One query of the wave from its loaded window: lower bound, runs, merge, emission (see above).
__device__ __forceinline__ bool nc_answer(const DevTable& T, const Target& t, uint32_t r0, uint32_t r1,
                                          const NcWindow& w, uint32_t lane, uint32_t qi, uint32_t count,
                                          uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt,
                                          bool fallback = true) {
    constexpr uint32_t W = 32, G = 64;
    const bool right = lane >= W;
    const uint32_t k = lane & (W - 1);
    const uint32_t N = T.n;
    uint32_t lb;
    if (r1 - r0 <= 32) {
        bool lt = false;
        if (lane >= 32 && lane < 32 + (r1 - r0)) {
            if (w.k0 != t.hi) {
                lt = w.k0 < t.hi;
            } else {
                const uint32_t* tt = T.tail + 3ull * (r0 - 32 + lane);
                lt = cmp160(0, tt[0], tt[1], tt[2], 0, t.t2, t.t3, t.t4) < 0;
            }
        }
        lb = r0 + (uint32_t)__builtin_popcountll(__ballot(lt));
    } else {
        lb = node_lower_bound(T, t);
    }
    const uint32_t dl = lb - r0;
    const uint32_t node = right ? lb + k : lb - 1 - k;
    const bool valid = right ? lb + k < N : lb > k;
    uint64_t key;
    uint32_t sb;
    if (dl <= 32) {  // wave-uniform
        const uint32_t idx = right ? 32 + dl + k : 31 + dl - k;  // window slot of `node`, in [0, 96)
        const uint64_t a = shfl64(w.k0, (int)(idx & 63u)), b = shfl64(w.k1, (int)(idx & 63u));
        const uint32_t ss = (uint32_t)__shfl((int)w.st, (int)(idx & 63u), 64);
        key = idx < 64 ? a : b;
        sb = idx < 64 ? ss & 255u : ss >> 8;
    } else {
        key = valid ? T.key[node] : 0;
        sb = valid ? T.status[node] : 0u;
    }
    uint64_t m = valid ? key ^ t.hi : ~0ull;  // invalid lanes end their run: the maximum
    const bool expired = !valid || (sb & KAD_STATUS_EXPIRED);
    bool amb = valid && m == ~0ull;  // indistinguishable from the end-of-run sentinel
#pragma unroll
    for (uint32_t s = 1; s < W; s <<= 1) {  // prefix maxima along my run
        const uint64_t o = shfl64(m, (int)lane - (int)s);
        if (k >= s && o > m) m = o;
    }
    const uint32_t obase = right ? 0u : W;
    uint32_t lo = 0, hi = W;
#pragma unroll
    for (int it = 0; it < 6; it++) {  // 33 possible answers: 6 halvings (a settled lane stays put)
        const uint32_t mid = (lo + hi) >> 1;
        const uint64_t v = shfl64(m, (int)(obase + (mid < W ? mid : W - 1)));
        if (lo < hi) {
            if (v < m) lo = mid + 1; else hi = mid;
        }
    }
    const uint64_t at = shfl64(m, (int)(obase + (lo < W ? lo : W - 1)));
    amb |= valid && lo < W && at == m;
    const uint32_t pos = k + lo;
    const bool emit = valid && !expired;
    const uint64_t eb = __ballot(emit);
    const uint32_t mine = right ? (uint32_t)(eb >> 32) : (uint32_t)eb;
    const uint32_t other = right ? (uint32_t)eb : (uint32_t)(eb >> 32);
    const uint32_t rank = (uint32_t)__builtin_popcount(mine & ((1u << k) - 1u)) +
                          (uint32_t)__builtin_popcount(lo >= W ? other : other & ((1u << lo) - 1u));
    const uint32_t tot = (uint32_t)__builtin_popcountll(eb);
    uint32_t pstar = 64;  // position of the count-th emission (64: not inside the window)
    if (tot >= count) {
        const uint64_t wm = __ballot(emit && rank == count - 1);
        pstar = (uint32_t)__shfl((int)pos, (int)__builtin_ctzll(wm), 64);
    }
    const uint32_t posA = (uint32_t)__shfl((int)pos, (int)(W - 1), 64);
    const uint32_t posB = (uint32_t)__shfl((int)pos, (int)(G - 1), 64);
    const bool ok = !__any(amb) && (lb <= W || posA > pstar) && (lb + W >= N || posB > pstar);
    if (ok) {
        uint32_t* row = out_idx + (size_t)qi * count;
        const uint32_t mm = min(tot, count);
        if (emit && rank < count) row[rank] = node + T.index_base;
        if (lane >= mm && lane < count) row[lane] = NONE;
        if (lane == 0 && out_cnt) out_cnt[qi] = (uint8_t)mm;
    } else if (lane == 0 && fallback) {
        nc_serial(T, t, count, out_idx + (size_t)qi * count, out_cnt ? out_cnt + qi : nullptr);
    }
    return ok;
}

__global__ __launch_bounds__(BLOCK) void nc_group_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                         uint32_t count, uint32_t* __restrict__ out_idx,
                                                         uint8_t* __restrict__ out_cnt) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t qi = blockIdx.x * (BLOCK / 64) + threadIdx.x / 64;
    if (qi >= q) return;  // one query per wave: the whole wave leaves
    const Target t = load_target(targets, qi);
    uint32_t r0, r1;
    nc_slot(T, t, r0, r1);
    const NcWindow w = nc_window(T, r0, lane);
    nc_answer(T, t, r0, r1, w, lane, qi, count, out_idx, out_cnt);
}

// Q queries per wave with their loads interleaved by hand: the Q targets, then the Q slot ranges,
// then the Q windows are each loaded unconditionally (indices clamped, validity applied after), so
// the wave waits three memory round trips for Q queries instead of for one. The kernel is latency
// bound: at one query per wave the waves spent ~60% of their cycles waiting on loads with 8 waves
// per SIMD resident (PMC). Tables with nodes only (T.n > 0).
template <int Q>
__global__ __launch_bounds__(BLOCK) void nc_multi_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                         uint32_t count, uint32_t* __restrict__ out_idx,
                                                         uint8_t* __restrict__ out_cnt) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t q0 = (blockIdx.x * (BLOCK / 64) + threadIdx.x / 64) * Q;
    if (q0 >= q) return;
    const uint32_t N = T.n;
    Target t[Q];
#pragma unroll
    for (int j = 0; j < Q; j++) t[j] = load_target(targets, min(q0 + j, q - 1));
    uint32_t r0[Q], r1[Q];
#pragma unroll
    for (int j = 0; j < Q; j++) {
        const bool below = t[j].hi < T.nbase;
        const uint64_t sl = below ? 0 : (t[j].hi - T.nbase) >> T.nshift;
        const bool above = !below && sl >= T.nslots;
        const uint32_t c = above ? T.nslots - 1 : (uint32_t)sl;
        const uint32_t a = T.nrdx[c], b = T.nrdx[c + 1];
        r0[j] = below ? 0u : (above ? N : a);
        r1[j] = below ? 0u : (above ? N : b);
    }
    NcWindow w[Q];
#pragma unroll
    for (int j = 0; j < Q; j++) {
        const int64_t p0 = (int64_t)r0[j] - 32 + lane, p1 = p0 + 64;
        const uint32_t c0 = (uint32_t)min(max(p0, (int64_t)0), (int64_t)N - 1);
        const uint32_t c1 = (uint32_t)min(p1, (int64_t)N - 1);
        const uint64_t a = T.key[c0], b = T.key[c1];
        const uint32_t sa = T.status[c0], sb = T.status[c1];
        const bool v0 = p0 >= 0 && p0 < (int64_t)N, v1 = lane < 32 && p1 < (int64_t)N;
        w[j].k0 = v0 ? a : 0;
        w[j].k1 = v1 ? b : 0;
        w[j].st = (v0 ? sa : 0u) | (v1 ? sb << 8 : 0u);
    }
#pragma unroll
    for (int j = 0; j < Q; j++)
        if (q0 + j < q) nc_answer(T, t[j], r0[j], r1[j], w[j], lane, q0 + j, count, out_idx, out_cnt);
}

// NodeCache counts 17..64, one query per wave at a time, 64-node runs each side of lb (two per lane):
// lanes 0-31 hold left elements k and k+32 (a_k = lb-1-k), lanes 32-63 right elements k and k+32
// (b_k = lb+k). The same greedy-merge placement as nc_answer (place = index + the other run's
// elements whose prefix maximum is below mine) over runs twice as long, so a walk that takes a whole
// subtree from one side (common for 32 emissions) stays inside the runs; the serial walk remains the
// fallback. Merge and emission for one query whose elements are loaded:
__device__ __forceinline__ void nc64_answer(const DevTable& T, const Target& t, uint32_t lb, uint32_t lane, uint32_t qi,
                                            uint32_t count, uint32_t* __restrict__ out_idx,
                                            uint8_t* __restrict__ out_cnt, uint64_t (&m)[2], const uint32_t (&node)[2],
                                            const bool (&valid)[2], const bool (&emit)[2], bool amb, bool serial) {
    constexpr uint32_t W = 64;  // run length
    const uint32_t N = T.n;
    const bool right = lane >= 32;
    const uint32_t k = lane & 31u, base = right ? 32u : 0u, obase = right ? 0u : 32u;
#pragma unroll
    for (int e = 0; e < 2; e++)
#pragma unroll
        for (uint32_t s = 1; s < 32; s <<= 1) {  // prefix maxima along each half-run
            const uint64_t o = shfl64(m[e], (int)lane - (int)s);
            if (k >= s && o > m[e]) m[e] = o;
        }
    {
        const uint64_t top = shfl64(m[0], (int)(base + 31));  // the first half-run's maximum
        if (top > m[1]) m[1] = top;
    }
    uint32_t pos[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        uint32_t lo = 0, hi = W;
#pragma unroll
        for (int it = 0; it < 7; it++) {  // 65 possible answers: 7 halvings
            const uint32_t mid = (lo + hi) >> 1, mc = mid < W ? mid : W - 1;
            const uint64_t v0 = shfl64(m[0], (int)(obase + (mc & 31u))), v1 = shfl64(m[1], (int)(obase + (mc & 31u)));
            const uint64_t v = mc < 32 ? v0 : v1;
            if (lo < hi) {
                if (v < m[e]) lo = mid + 1; else hi = mid;
            }
        }
        const uint32_t lc = lo < W ? lo : W - 1;
        const uint64_t a0 = shfl64(m[0], (int)(obase + (lc & 31u))), a1 = shfl64(m[1], (int)(obase + (lc & 31u)));
        amb |= valid[e] && lo < W && (lc < 32 ? a0 : a1) == m[e];
        pos[e] = k + 32u * e + lo;
    }
    const uint64_t eb0 = __ballot(emit[0]), eb1 = __ballot(emit[1]);
    const uint32_t mine0 = (uint32_t)(eb0 >> base), mine1 = (uint32_t)(eb1 >> base);
    const uint32_t oth0 = (uint32_t)(eb0 >> obase), oth1 = (uint32_t)(eb1 >> obase);
    const uint32_t below = (1u << k) - 1u;
    uint32_t rank[2];
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const uint32_t lo = pos[e] - k - 32u * e;
        const uint32_t oth = lo >= 64 ? __builtin_popcount(oth0) + __builtin_popcount(oth1)
                             : lo >= 32 ? __builtin_popcount(oth0) + __builtin_popcount(oth1 & ((1u << (lo - 32)) - 1u))
                                        : __builtin_popcount(oth0 & ((1u << lo) - 1u));
        rank[e] = (e == 0 ? __builtin_popcount(mine0 & below)
                          : __builtin_popcount(mine0) + __builtin_popcount(mine1 & below)) + oth;
    }
    const uint32_t tot = (uint32_t)(__builtin_popcountll(eb0) + __builtin_popcountll(eb1));
    uint32_t pstar = 128;  // merge position of the count-th emission (128: not inside the runs)
    if (tot >= count) {
        const uint64_t w0 = __ballot(emit[0] && rank[0] == count - 1), w1 = __ballot(emit[1] && rank[1] == count - 1);
        pstar = w0 ? (uint32_t)__shfl((int)pos[0], (int)__builtin_ctzll(w0), 64)
                   : (uint32_t)__shfl((int)pos[1], (int)__builtin_ctzll(w1 | (1ull << 63)), 64);
    }
    const uint32_t posA = (uint32_t)__shfl((int)pos[1], 31, 64);  // left element 63
    const uint32_t posB = (uint32_t)__shfl((int)pos[1], 63, 64);  // right element 63
    const bool ok = !__any(amb) && (lb <= W || posA > pstar) && (lb + W >= N || posB > pstar);
    if (ok) {
        uint32_t* row = out_idx + (size_t)qi * count;
        const uint32_t mm = min(tot, count);
#pragma unroll
        for (int e = 0; e < 2; e++)
            if (emit[e] && rank[e] < count) row[rank[e]] = node[e] + T.index_base;
        if (lane >= mm && lane < count) row[lane] = NONE;
        if (lane == 0 && out_cnt) out_cnt[qi] = (uint8_t)mm;
    } else if (lane == 0 && serial) {
        nc_serial(T, t, count, out_idx + (size_t)qi * count, out_cnt ? out_cnt + qi : nullptr);
    }
}

// One query per wave: target -> slot -> lb (one ballot over the slot's nodes when it holds <= 64, else
// the binary search) -> the 128 run elements (direct loads; a 192-node window load around r0 read
// 1.5x the bytes and took 1036 against 890 us per 1M k = 32 queries, with no gain from interleaving two
// queries per wave: the kernel is bound by those bytes, not by latency).
// ABL 1 (timing ablation only, KAD_NC_KERNEL=w64_abl1; results wrong): no serial fallback.
__device__ __forceinline__ void nc64_query(const DevTable& T, const Target& t, uint32_t lane, uint32_t qi, uint32_t count,
                                           uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt, bool serial) {
    const uint32_t N = T.n;
    uint32_t r0, r1;
    nc_slot(T, t, r0, r1);
    uint32_t lb;
    if (r1 - r0 <= 64) {
        bool lt = false;
        if (lane < r1 - r0) {
            const uint32_t n = r0 + lane;
            const uint64_t kk = T.key[n];
            if (kk != t.hi) {
                lt = kk < t.hi;
            } else {
                const uint32_t* tt = T.tail + 3ull * n;
                lt = cmp160(0, tt[0], tt[1], tt[2], 0, t.t2, t.t3, t.t4) < 0;
            }
        }
        lb = r0 + (uint32_t)__builtin_popcountll(__ballot(lt));
    } else {
        lb = node_lower_bound(T, t);
    }
    const bool right = lane >= 32;
    const uint32_t k = lane & 31u;
    uint64_t m[2];
    uint32_t node[2];
    bool valid[2], emit[2], amb = false;
#pragma unroll
    for (int e = 0; e < 2; e++) {
        const uint32_t kk = k + 32u * e;
        node[e] = right ? lb + kk : lb - 1 - kk;
        valid[e] = right ? lb + kk < N : lb > kk;
        uint64_t key = 0;
        uint32_t sb = 0;
        if (valid[e]) {
            key = T.key[node[e]];
            sb = T.status[node[e]];
        }
        m[e] = valid[e] ? key ^ t.hi : ~0ull;
        emit[e] = valid[e] && !(sb & KAD_STATUS_EXPIRED);
        amb |= valid[e] && m[e] == ~0ull;
    }
    nc64_answer(T, t, lb, lane, qi, count, out_idx, out_cnt, m, node, valid, emit, amb, serial);
}

template <int ABL>
__global__ __launch_bounds__(BLOCK) void nc_wave64_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                          uint32_t count, uint32_t* __restrict__ out_idx,
                                                          uint8_t* __restrict__ out_cnt) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t qi = blockIdx.x * (BLOCK / 64) + threadIdx.x / 64;
    if (qi >= q) return;  // one query per wave: the whole wave leaves
    nc64_query(T, load_target(targets, qi), lane, qi, count, out_idx, out_cnt, ABL == 0);
}

// Counts 17..64, cheaper first pass: the 96-node window and 32-node runs (nc_answer, ~0.9 KB less per
// query); only the queries whose walk leaves those runs load the 64-node runs (nc64_query).
__global__ __launch_bounds__(BLOCK) void nc_two_pass_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                            uint32_t count, uint32_t* __restrict__ out_idx,
                                                            uint8_t* __restrict__ out_cnt) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t qi = blockIdx.x * (BLOCK / 64) + threadIdx.x / 64;
    if (qi >= q) return;  // one query per wave: the whole wave leaves
    const Target t = load_target(targets, qi);
    uint32_t r0, r1;
    nc_slot(T, t, r0, r1);
    const NcWindow w = nc_window(T, r0, lane);
    if (!nc_answer(T, t, r0, r1, w, lane, qi, count, out_idx, out_cnt, false))
        nc64_query(T, t, lane, qi, count, out_idx, out_cnt, true);
}

// ---------------------------------------------------------------------------------------
// NodeCache lines (TF_NCL): one 256-byte line per node radix slot s answers the count <= 16
// getCachedNodes queries whose target falls in s with one line load per lane (no lower_bound chain,
// no wave cooperation). Line s holds the 60-node window w0 = r0-28 .. r0+32 of the sorted node array,
// where [r0, r1) are the slot's nodes:
//   dw0      w0
//   dw1      ns = r1 - r0 | sh << 8
//   dw2      defer (clamped window / wide slot) | truncated left (w0 > 0) << 1 | truncated right (w0 + 60 < n) << 2
//   dw4..63  slot j: key24(node w0+j) << 8 | expired
// key24 = ID bits [40-sh, 64-sh) = (key >> sh) & 0xFFFFFF, starting at or above the window's common
// prefix: all window nodes share the bits above, so every XOR comparison between them (the walk's
// xorCmp) is decided inside those 24 bits unless the two nodes share them; key24 is monotone over the window,
// so a left-run and a right-run node can only share one if the two nodes either side of lb do, and only that
// pair sends the query to the exact path (round 4 deferred the whole line for any equal neighbours).
// The start is also at or above the slot's prefix, so "node < target" for the slot's nodes is a
// key24 comparison (equal key24: exact path). Windows clamped at the array ends and
// slots of more than 15 nodes are deferred (exact path): lb = r0 + x with x <= 15.
//
// The walk (node_cache.cpp:36-66) is the greedy merge by XOR distance of the left run lb-1, lb-2, ..
// and the right run lb, lb+1, ..; in a greedy merge an element's place is set by the maximum
// distance M along its run from lb to itself (tests/test_nodecache_merge.py), so the walk order is
// the order of (M, side, steps from lb), with no ties between the runs (distinct IDs). A lane shifts
// its window by x so that lb sits at slot 28 (four conditional shifts) and scans 28 left and 32-x
// right slots for M with static indices. Each run's keys ascend outward from lb, so the walk's first
// 32 steps are one top-32 bitonic merge of the two runs; the non-expired ones are then compacted. Nodes outside the window come after the window end of their side (larger
// M or more steps), so the keys up to min(end key of a truncated side) are exact; fewer than `count`
// of them means the walk leaves the window: the wave answers those lanes' queries one by one with
// nc_answer (32-node runs each side of lb, wave-cooperative).
// ---------------------------------------------------------------------------------------
#ifndef KAD_NCL_STRIDE
#define KAD_NCL_STRIDE 64u
#define KAD_NCL_LEFT 28u
#endif
constexpr uint32_t NCL_STRIDE = KAD_NCL_STRIDE, NCL_SLOTS = NCL_STRIDE - 4, NCL_LEFT = KAD_NCL_LEFT,
                   NCL_XMAX = 15;                 // dwords
constexpr uint32_t NCL_PIECES = NCL_STRIDE / 4;  // 16-byte pieces of a line
constexpr int NCL_NV = (int)NCL_SLOTS + 4;        // a lane's slot array (the slots, then NONE)
static_assert(NCL_STRIDE % 16 == 0 && NCL_STRIDE <= 64 && NCL_LEFT + NCL_XMAX < NCL_SLOTS, "NodeCache line");
// The 128-byte line of slot s (after all the 256-byte lines: dword NCL_STRIDE * nslots + NCL2_DWORDS * s), the 37-node
// window centred on the slot, read first (ncl2_build_line).
constexpr uint32_t NCL2_DWORDS = 32, NCL2_SLOTS = 37, NCL2_MID = 18, NCL2_XMAX = 15, NCL2_PMIN = NCL2_MID - NCL2_XMAX / 2,
                   NCL2_PMAX = NCL2_MID + (NCL2_XMAX + 1) / 2;
// counts up to 14 (SEARCH_NODES) read the 128-byte line and send its misses to the wave path; 15 and 16 walk past
// its 37 nodes for 1.6 % of the queries (k = 16) and read the 256-byte line instead
constexpr uint32_t NCL2_COUNT_MAX = 14;

// The answer from the lane's line (Lq: its 16 pieces, loaded by the wave): the node indices go to lrow[0..m) (the
// lane's LDS row) by emission rank.
__device__ __forceinline__ bool ncl_answer(const uint4 (&Lq)[16], uint32_t index_base, const Target& t,
                                           uint32_t count, uint32_t* lrow, uint32_t& m) {
    uint32_t v[NCL_NV];
    const uint4 hd = Lq[0];
#pragma unroll
    for (int x = 1; x < (int)NCL_PIECES; x++) {
        const uint4 u = Lq[x];
        v[4 * x - 4] = u.x; v[4 * x - 3] = u.y; v[4 * x - 2] = u.z; v[4 * x - 1] = u.w;
    }
    v[NCL_NV - 4] = v[NCL_NV - 3] = v[NCL_NV - 2] = v[NCL_NV - 1] = NONE;
    const uint32_t w0 = hd.x, ns = hd.y & 255u, sh = (hd.y >> 8) & 63u, fl = hd.z;
    const uint32_t tx = ((uint32_t)(t.hi >> sh) & 0xFFFFFFu) << 8;
    bool ex = fl & 1u;
    uint32_t x = 0;  // lb = r0 + x: the slot's nodes below the target
#pragma unroll
    for (int j = 0; j < (int)NCL_SLOTS; j++) {
        // a slot word is key24 << 8 | expired (bits 1..7 zero): key24 < t24 iff word < t24 << 8, and the XOR
        // with t24 << 8 is the distance inside the window's 24 bits | expired
        if (j >= (int)NCL_LEFT && j < (int)(NCL_LEFT + NCL_XMAX) && (uint32_t)j - NCL_LEFT < ns) {
            ex |= (v[j] ^ tx) < 256u;
            x += v[j] < tx ? 1u : 0u;
        }
        v[j] ^= tx;
    }
    // shift the window by x: lb at slot NCL_LEFT, the left run NCL_LEFT-1..0, the right run NCL_LEFT..NCL_SLOTS-1-x
    {
        uint32_t u[NCL_NV];
#pragma unroll
        for (int j = 0; j < NCL_NV; j++) u[j] = (x & 1u) ? (j < NCL_NV - 1 ? v[j + 1] : NONE) : v[j];
#pragma unroll
        for (int j = 0; j < NCL_NV; j++) v[j] = (x & 2u) ? (j < NCL_NV - 2 ? u[j + 2] : NONE) : u[j];
#pragma unroll
        for (int j = 0; j < NCL_NV; j++) u[j] = (x & 4u) ? (j < NCL_NV - 4 ? v[j + 4] : NONE) : v[j];
#pragma unroll
        for (int j = 0; j < NCL_NV; j++) v[j] = (x & 8u) ? (j < NCL_NV - 8 ? u[j + 8] : NONE) : u[j];
    }
    // equal key24 either side of lb: the runs may tie at 24 bits (the window's key24 values are monotone, so a
    // left and a right element can only share one if these two do); only the full IDs order them -> exact path
    ex |= (v[NCL_LEFT - 1] >> 8) == (v[NCL_LEFT] >> 8);
    const uint32_t nv = NCL_SLOTS - x;  // valid slots after the shift
    // keys: (M along the run) << 8 | side << 7 | steps from lb << 1 | expired. Each run's keys ascend
    // outward from lb (M never decreases, the steps grow), and the expired bit is below the steps.
    uint32_t run = 0;
#pragma unroll
    for (int j = (int)NCL_LEFT - 1; j >= 0; j--) {
        run = max(run, v[j] & ~255u);
        v[j] = run | ((uint32_t)(NCL_LEFT - 1 - j) << 1) | (v[j] & 1u);
    }
    const uint32_t endL = ((fl & 2u) || x > 0) ? v[0] : NONE;  // more nodes left of the window?
    run = 0;
    uint32_t endR = NONE;
#pragma unroll
    for (int j = (int)NCL_LEFT; j < (int)NCL_SLOTS; j++) {
        const bool in = (uint32_t)j < nv;
        run = max(run, in ? v[j] & ~255u : 0u);
        v[j] = in ? run | 128u | ((uint32_t)(j - NCL_LEFT) << 1) | (v[j] & 1u) : NONE;
        if (j >= (int)(NCL_SLOTS - NCL_XMAX - 1) && (uint32_t)j == nv - 1) endR = v[j];
    }
    if (!(fl & 4u)) endR = NONE;  // the window reaches the array end
    const uint32_t lim = min(endL, endR);  // keys <= lim are the walk's first steps
    // the walk's first 32 steps: top-32 merge of the two ascending runs (left NCL_LEFT reversed + NONE,
    // right up to 32 + NONE), then a bitonic half-cleaner cascade
    uint32_t w[32];
#pragma unroll
    for (int r = 0; r < 32; r++) {
        const uint32_t a = r < (int)NCL_LEFT ? v[NCL_LEFT - 1 - r] : NONE;              // left, ascending
        const int jr = (int)NCL_LEFT + 31 - r;
        w[r] = min(a, jr < (int)NCL_SLOTS ? v[jr < NCL_NV ? jr : 0] : NONE);              // right, descending
    }
#pragma unroll
    for (int h = 16; h >= 1; h >>= 1)
#pragma unroll
        for (int r = 0; r < 32; r++)
            if ((r & h) == 0) cx(w[r], w[r + h]);
    // emit the non-expired steps up to lim in walk order into the lane's LDS row (one pass, no rank arrays)
    const uint32_t base = w0 + x + index_base;
    uint32_t have = 0;
#pragma unroll
    for (int r = 0; r < 32; r++) {
        const bool keep = w[r] <= lim && !(w[r] & 1u);
        if (keep && have < count) {
            const uint32_t st = (w[r] >> 1) & 63u;
            lrow[have] = base + ((w[r] & 128u) ? NCL_LEFT + st : NCL_LEFT - 1 - st);
        }
        have += keep ? 1u : 0u;
    }
    m = min(count, have);
    ex |= have < count && (lim != NONE || w[31] != NONE);  // the walk goes on past the window / step 32
    return !ex;
}

// The answer from the lane's 128-byte line (Lq: its 8 pieces; layout at ncl2_build_line). The line's 37 nodes sit
// around the middle of the slot, so lb lies at window position p in [11, 26]: nodes before 11 are below every target of
// the slot, nodes from 26 on above it, and p = 11 + the nodes of positions 11..25 below the target. The window is
// shifted right by 26 - p (lb at 26; the left run 25..0 holds all p window nodes left of lb, then NONE; the right run
// 26.. the 37 - p others), then walked as ncl_answer walks the 256-byte line.
__device__ __forceinline__ bool ncl2_answer(const uint4 (&Lq)[8], uint32_t index_base, const Target& t,
                                            uint32_t count, uint32_t* lrow, uint32_t& m) {
    constexpr int S = (int)NCL2_SLOTS, PMIN = (int)NCL2_PMIN, PMAX = (int)NCL2_PMAX, NV = S + PMAX - PMIN;
    uint32_t d[32], v[NV];
#pragma unroll
    for (int x = 0; x < 8; x++) {
        d[4 * x] = Lq[x].x; d[4 * x + 1] = Lq[x].y; d[4 * x + 2] = Lq[x].z; d[4 * x + 3] = Lq[x].w;
    }
    const uint32_t w0 = d[0], sh = (d[1] >> 8) & 63u, fl = d[1] >> 16;
    const uint32_t tx = ((uint32_t)(t.hi >> sh) & 0xFFFFFFu) << 8;
    bool ex = fl & 1u;
    uint32_t p = PMIN;
#pragma unroll
    for (int e = 0; e < S; e++) {  // key24 of node w0 + e at byte 16 + 3e, its expired bit at bit e of dw2..3
        const int o = 3 * e, w = 4 + o / 4, b = 8 * (o % 4);
        const uint32_t k = b <= 8 ? d[w] >> b : __builtin_amdgcn_alignbit(d[w + 1], d[w], (uint32_t)b);
        const uint32_t val = (k << 8) | ((d[2 + e / 32] >> (e % 32)) & 1u);
        if (e >= PMIN && e < PMAX) {  // the slot's nodes and their neighbours: key24 < t24 iff val < t24 << 8
            ex |= (val ^ tx) < 256u;
            p += val < tx ? 1u : 0u;
        }
        v[e] = val ^ tx;
    }
#pragma unroll
    for (int e = S; e < NV; e++) v[e] = NONE;
    const uint32_t s = (uint32_t)PMAX - p;  // 0..15
    {
        uint32_t u[NV];
#pragma unroll
        for (int j = 0; j < NV; j++) u[j] = (s & 1u) ? (j >= 1 ? v[j - 1] : NONE) : v[j];
#pragma unroll
        for (int j = 0; j < NV; j++) v[j] = (s & 2u) ? (j >= 2 ? u[j - 2] : NONE) : u[j];
#pragma unroll
        for (int j = 0; j < NV; j++) u[j] = (s & 4u) ? (j >= 4 ? v[j - 4] : NONE) : v[j];
#pragma unroll
        for (int j = 0; j < NV; j++) v[j] = (s & 8u) ? (j >= 8 ? u[j - 8] : NONE) : u[j];
    }
    ex |= (v[PMAX - 1] >> 8) == (v[PMAX] >> 8);  // equal key24 either side of lb (ncl_answer)
    uint32_t run = 0, endL = NONE, endR = NONE;
#pragma unroll
    for (int j = PMAX - 1; j >= 0; j--) {
        const bool in = (uint32_t)j >= s;
        run = max(run, in ? v[j] & ~255u : 0u);
        v[j] = in ? run | ((uint32_t)(PMAX - 1 - j) << 1) | (v[j] & 1u) : NONE;
        if (j <= PMAX - PMIN && (uint32_t)j == s) endL = v[j];
    }
    if (!(fl & 2u)) endL = NONE;  // the window starts at node 0
    run = 0;
#pragma unroll
    for (int j = PMAX; j < NV; j++) {
        const bool in = (uint32_t)j < (uint32_t)S + s;
        run = max(run, in ? v[j] & ~255u : 0u);
        v[j] = in ? run | 128u | ((uint32_t)(j - PMAX) << 1) | (v[j] & 1u) : NONE;
        if (j >= S - 1 && (uint32_t)j == (uint32_t)S - 1 + s) endR = v[j];
    }
    if (!(fl & 4u)) endR = NONE;  // the window reaches the array end
    const uint32_t lim = min(endL, endR);
    uint32_t w[32];
#pragma unroll
    for (int r = 0; r < 32; r++) {
        const uint32_t a = r < PMAX ? v[PMAX - 1 - r] : NONE;
        const int jr = PMAX + 31 - r;
        w[r] = min(a, jr < NV ? v[jr] : NONE);
    }
#pragma unroll
    for (int h = 16; h >= 1; h >>= 1)
#pragma unroll
        for (int r = 0; r < 32; r++)
            if ((r & h) == 0) cx(w[r], w[r + h]);
    const uint32_t lbn = w0 + p + index_base;
    uint32_t have = 0;
#pragma unroll
    for (int r = 0; r < 32; r++) {
        const bool keep = w[r] <= lim && !(w[r] & 1u);
        if (keep && have < count) {
            const uint32_t st = (w[r] >> 1) & 63u;
            lrow[have] = (w[r] & 128u) ? lbn + st : lbn - 1 - st;
        }
        have += keep ? 1u : 0u;
    }
    m = min(count, have);
    ex |= have < count && (lim != NONE || w[31] != NONE);
    return !ex;
}

// Wave-level LDS ordering (the rocPRIM wave barrier): the wave's LDS writes before it are seen by its reads after.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Row r of the NodeCache line kernel's block inside its wave's staging region (64 x 8 uint4 = 2048 words per wave).
__device__ __forceinline__ uint32_t ncl_wrow(uint32_t r) { return (r >> 6) * 2048u + (r & 63u) * 16u; }

// The block's rows of count <= 16 from LDS (row r at rows[r * 16 + c], or rows[ncl_wrow(r) + c] with wrow; the first
// m[r] valid, the rest NONE) as one run of 16-byte stores; rows whose lane did not answer (ok false) are skipped
// dword by dword.
__device__ __forceinline__ void store_rows_lds16(uint32_t* __restrict__ out_idx, uint32_t q, uint32_t count,
                                                 const uint32_t* rows, const uint8_t* mrow, const uint32_t* okm,
                                                 bool wrow = false) {
    const uint32_t tid = threadIdx.x, q0 = blockIdx.x * BLOCK;
    const uint32_t nq = min((uint32_t)BLOCK, q - q0), nw = nq * count;
    uint32_t* dst = out_idx + (size_t)q0 * count;
    const bool al = ((uintptr_t)out_idx & 15u) == 0;  // BLOCK * count * 4 is a multiple of 16
    for (uint32_t c4 = tid; 4 * c4 < nw; c4 += BLOCK) {
        const uint32_t w0 = 4 * c4;
        uint32_t r = w0 / count, c = w0 - r * count, v[4];
        bool okv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const bool in = w0 + u < nw;
            okv[u] = in && ((okm[r >> 5] >> (r & 31)) & 1u);
            v[u] = in && c < mrow[r] ? rows[(wrow ? ncl_wrow(r) : r * 16) + c] : NONE;
            if (++c == count) { c = 0; r++; }
        }
        if (al && okv[0] && okv[1] && okv[2] && okv[3]) {
            st_row4(dst + w0, v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (okv[u]) st_row1(dst + w0 + u, v[u]);
        }
    }
}

// The block's rows from the waves' staging regions (2048 words each: row r's words at ncl_wrow(r), its meta word
// m | answered << 8 at word 1024 + (r & 63) of its wave's region) as one run of 16-byte stores; rows not answered
// are skipped dword by dword.
__device__ __forceinline__ void store_rows_wave16(uint32_t* __restrict__ out_idx, uint32_t q, uint32_t count,
                                                  const uint32_t* stgw) {
    const uint32_t tid = threadIdx.x, q0 = blockIdx.x * BLOCK;
    const uint32_t nq = min((uint32_t)BLOCK, q - q0), nw = nq * count;
    uint32_t* dst = out_idx + (size_t)q0 * count;
    const bool al = ((uintptr_t)out_idx & 15u) == 0;  // BLOCK * count * 4 is a multiple of 16
    for (uint32_t c4 = tid; 4 * c4 < nw; c4 += BLOCK) {
        const uint32_t w0 = 4 * c4;
        uint32_t r = w0 / count, c = w0 - r * count, v[4];
        bool okv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const bool in = w0 + u < nw;
            const uint32_t meta = in ? stgw[(r >> 6) * 2048u + 1024u + (r & 63u)] : 0u;
            okv[u] = in && ((meta >> 8) & 1u);
            v[u] = in && c < (meta & 255u) ? stgw[ncl_wrow(r) + c] : NONE;
            if (++c == count) { c = 0; r++; }
        }
        if (al && okv[0] && okv[1] && okv[2] && okv[3]) {
            st_row4(dst + w0, v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (okv[u]) st_row1(dst + w0 + u, v[u]);
        }
    }
}

// ABL 1 (timing ablation only, KAD_NC_KERNEL=lines_abl1; results wrong): the 256-byte lines alone (round 5's
// kernel), no exact path. ABL 2 (lines_abl2): the 256-byte line load and the row store only (every word of the line
// folded into one value), round 5's memory floor. ABL 3 (lines_abl3): the 128-byte lines alone (no second line, no
// exact path). ABL 5 (lines_stats): the product kernel with out_cnt = the step that answered (1: the 128-byte line,
// 2: the 256-byte line, 3: the wave path).
// DUAL: per-query family (af[i] = 0 -> T4, 1 -> T6; NodeCache::getCachedNodes picks cache_4 / cache_6 by
// sa_family, node_cache.cpp:37); an empty family map (n = 0) gives zero results.
// The lines are loaded by the wave, not by their lanes: a lane-private 256-byte line is 16 random 16-byte loads,
// each instruction touching 64 lines (64 address translations), and a 2 GB line table is bound by those
// translations (tools/nc_abl.py). The wave loads its 64 lines in two halves of 128 bytes, eight lanes per line
// (one translation per line per instruction), and hands each lane its line through LDS.
template <int ABL, bool DUAL, bool HALF>
__device__ __forceinline__ void nc_line_kernel_body(const DevTable& T4, const DevTable& T6, const uint8_t* __restrict__ af,
                                                        const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x, lane = threadIdx.x & 63u, tid = threadIdx.x;
    const bool act = i < q;
    const bool fam = DUAL && act && af[i] != 0;
    // a wave's 64 line halves, piece p of line q at [q][p ^ (q & 7)] (the XOR spreads a lane's 16-byte reads over
    // the banks without a pad: 8 KB per wave, 5 waves per SIMD); afterwards the wave's rows
    __shared__ uint4 stg[BLOCK / 64][64][8];  // 32 KB: five blocks per CU
    Target t{};
    bool ok = false;
    uint32_t m = 0, sl = NONE;  // this lane's line: radix slot | family << 31 (NONE: no line)
    if (act) {
        t = load_target(targets, i);
        // this lane's family: only the fields the line path reads
        const uint64_t nbase = fam ? T6.nbase : T4.nbase;
        const uint32_t nshift = fam ? T6.nshift : T4.nshift, nslots = fam ? T6.nslots : T4.nslots;
        const uint32_t n = fam ? T6.n : T4.n, flags = fam ? T6.flags : T4.flags;
        if (n == 0) {  // empty map: no nodes
            ok = true;
        } else if (flags & TF_NCL) {
            // below the first slot / past the last: lb = 0 / n, windows clamped at the ends (exact path)
            if (t.hi >= nbase && ((t.hi - nbase) >> nshift) < nslots)
                sl = (uint32_t)((t.hi - nbase) >> nshift) | (fam ? 0x80000000u : 0u);
        }
    }
    uint4 (*S)[8] = stg[tid >> 6];  // this wave's region: only wave-level ordering is needed
    // the wave's rows (64 x 16 words) reuse its region: row r of the block at rows + ncl_wrow(r)
    uint32_t* rows = reinterpret_cast<uint32_t*>(&stg[0][0][0]);
    uint32_t stage = 3;  // ABL 5: which step answered (1: the 128-byte line, 2: the 256-byte line, 3: the wave)
    uint32_t hr0 = NONE, hns = 0;  // the slot's first node and node count from a 128-byte line header (NONE: none)
    if ((ABL == 0 && HALF) || ABL == 3 || ABL == 5 || ABL == 6) {
        // the 128-byte lines first: round r, lane L loads piece (L & 7) of the line of query 8r + (L >> 3)
        uint4 ld[8], L2[8];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const uint32_t so = (uint32_t)__shfl((int)sl, 8 * r + (int)(lane >> 3), 64);
            uint4 a = make_uint4(0u, 0u, 0u, 0u);
            if (so != NONE) {
                const DevTable& T = (DUAL && (so >> 31)) ? T6 : T4;
                a = T.ncl[(size_t)NCL_PIECES * T.nslots + 8ull * (so & 0x7FFFFFFFu) + (lane & 7)];
            }
            ld[r] = a;
        }
#pragma unroll
        for (int r = 0; r < 8; r++) S[8 * r + (lane >> 3)][(lane & 7) ^ ((lane >> 3) & 7)] = ld[r];
        wave_sync();
#pragma unroll
        for (int x = 0; x < 8; x++) L2[x] = S[lane][x ^ (lane & 7)];
        wave_sync();
        const uint32_t ib = fam ? T6.index_base : T4.index_base;
        if (sl != NONE && !((L2[0].y >> 16) & 1u)) {  // the slot's node range from the line header (the wave path's)
            hns = L2[0].y & 255u;
            hr0 = L2[0].x + NCL2_MID - hns / 2;
        }
        if (sl != NONE) ok = ncl2_answer(L2, ib, t, count, rows + ncl_wrow(tid), m);
        if (ok) stage = 1;
        // the walks that leave the 37-node window (about one query in 150 at k = 14), deferred lines: the 256-byte
        // line, loaded by its lane
        if (ABL == 6 && sl != NONE && !ok) {
            const uint4* lp = (fam ? T6.ncl : T4.ncl) + (size_t)NCL_PIECES * (sl & 0x7FFFFFFFu);
            uint4 L[16];
#pragma unroll
            for (int x = 0; x < 16; x++) L[x] = x < (int)NCL_PIECES ? lp[x] : make_uint4(0u, 0u, 0u, 0u);
            ok = ncl_answer(L, ib, t, count, rows + ncl_wrow(tid), m);
            if (ok) stage = 2;
        }
    } else {
    // round r: lane L loads pieces (L & 7) and 8 + (L & 7) of the line of query 8r + (L >> 3)
    uint4 ld[16], L[16];
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const uint32_t so = (uint32_t)__shfl((int)sl, 8 * r + (int)(lane >> 3), 64);
        uint4 a = make_uint4(0u, 0u, 0u, 0u), b = a;
        if (so != NONE) {
            const uint4* lp = ((DUAL && (so >> 31)) ? T6.ncl : T4.ncl) + (size_t)NCL_PIECES * (so & 0x7FFFFFFFu);
            a = lp[lane & 7];
            if (NCL_PIECES == 16 || 8 + (lane & 7) < NCL_PIECES) b = lp[8 + (lane & 7)];
        }
        ld[r] = a;
        ld[8 + r] = b;
    }
#pragma unroll
    for (int h = 0; h < 2; h++) {
#pragma unroll
        for (int r = 0; r < 8; r++) S[8 * r + (lane >> 3)][(lane & 7) ^ ((lane >> 3) & 7)] = ld[8 * h + r];
        wave_sync();
#pragma unroll
        for (int x = 0; x < 8; x++) L[8 * h + x] = S[lane][x ^ (lane & 7)];
        wave_sync();
    }
    if (sl != NONE) {
        if (ABL == 2) {
            uint32_t f = 0;
#pragma unroll
            for (int x = 0; x < 16; x++) f ^= L[x].x + L[x].y + L[x].z + L[x].w;
            for (uint32_t c = 0; c < count; c++) rows[ncl_wrow(tid) + c] = f + c;
            m = count;
            ok = true;
        } else {
            ok = ncl_answer(L, fam ? T6.index_base : T4.index_base, t, count, rows + ncl_wrow(tid), m);
        }
    }
    }
    if (act && ok && out_cnt) out_cnt[i] = (uint8_t)m;
    rows[(tid >> 6) * 2048u + 1024u + lane] = m | (ok ? 256u : 0u);  // the row's meta word (its wave's region)
    __syncthreads();
    store_rows_wave16(out_idx, q, count, rows);
    // the lanes the lines could not answer: one query at a time by the whole wave (nc_answer: 32-node
    // runs each side of lb, itself falling back to lane 0's serial walk)
    uint64_t pend = (ABL == 0 || ABL == 5 || ABL == 6) ? __ballot(act && !ok) : 0ull;
    const uint64_t fm = DUAL ? __ballot(fam) : 0ull;
    while (pend) {
        const uint32_t l = (uint32_t)__builtin_ctzll(pend);
        pend &= pend - 1;
        Target u;
        u.hi = shfl64(t.hi, (int)l);
        u.t2 = (uint32_t)__shfl((int)t.t2, (int)l, 64);
        u.t3 = (uint32_t)__shfl((int)t.t3, (int)l, 64);
        u.t4 = (uint32_t)__shfl((int)t.t4, (int)l, 64);
        const DevTable& T = (DUAL && ((fm >> l) & 1ull)) ? T6 : T4;  // wave-uniform
        uint32_t r0 = (uint32_t)__shfl((int)hr0, (int)l, 64), r1;
        if (r0 != NONE) r1 = r0 + (uint32_t)__shfl((int)hns, (int)l, 64);  // no radix load
        else nc_slot(T, u, r0, r1);
        const NcWindow w = nc_window(T, r0, lane);
        nc_answer(T, u, r0, r1, w, lane, i - lane + l, count, out_idx, out_cnt);
    }
    if (ABL == 5 && act && out_cnt) out_cnt[i] = (uint8_t)stage;
}
template <int ABL, bool DUAL, bool HALF>
__global__ __launch_bounds__(BLOCK) void nc_line_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ af,
                                                        const uint8_t* __restrict__ targets, uint32_t q,
                                                        uint32_t count, uint32_t* __restrict__ out_idx,
                                                        uint8_t* __restrict__ out_cnt) {
    nc_line_kernel_body<ABL, DUAL, HALF>(T4, T6, af, targets, q, count, out_idx, out_cnt);
}

// ---------------------------------------------------------------------------------------
// NodeCache counts <= NCL2_COUNT_MAX, one lane per query reading its own 128-byte line (layout at ncl2_build_line).
// The line region of the bench shard is 1 GB (8M radix slots): at that size eight 16-byte loads per lane reach 37 us
// per 1M lines where the wave-loaded form (eight lanes per line, handed over through LDS) holds 45, and
// with no line staging the block's LDS is its rows alone, so eight waves per SIMD fit.
//
// The walk without shifting the window: along the line's positions e = 0..36 the left run's keys descend (each key
// ascends outward from lb) and the right run's ascend, so the 37 keys followed by NONE form a bitonic sequence of 64
// whatever lb is. One half-cleaner at h = 32 (five mins) keeps the 32 smallest as a bitonic 32, and five more levels
// sort them: the walk's first 32 steps, with no position-dependent indexing anywhere. The tie-break field is (63 - e)
// on the left and e on the right (the same order as the steps from lb), so the node of a key is w0 + e read straight
// from the key; the lane writes raw keys into its LDS row and the block's store decodes them.
// ---------------------------------------------------------------------------------------
constexpr uint32_t NCL2_RS = 17;  // LDS row stride in words (16 keys + 1: the lanes' rows fall into different banks)
#ifndef KAD_NCL2_STEPS
#define KAD_NCL2_STEPS 24u
#endif
constexpr uint32_t NCL2_STEPS = KAD_NCL2_STEPS;  // walk steps the lane kernel sorts (24, or 32: the whole lower half)
static_assert(NCL2_STEPS == 24 || NCL2_STEPS == 32, "lane kernel steps");

__device__ __forceinline__ uint32_t ncl2_key24x(const uint32_t (&d)[32], int e) {
    // key24 of line position e (bytes 16 + 3e .. 18 + 3e) as key24 << 8, low byte zero: one byte permute
    const int o = 3 * e, w = 4 + o / 4, b = o % 4;
    const uint32_t sel = 0x0Cu | ((uint32_t)b << 8) | ((uint32_t)(b + 1) << 16) | ((uint32_t)(b + 2) << 24);
    return __builtin_amdgcn_perm(w + 1 < 32 ? d[w + 1] : 0u, d[w], sel);
}

// The answer from the lane's 128-byte line d: raw walk keys (run max << 8 | side << 7 | tie-break << 1) into lrow[0..m),
// the row's node base (w0 + index_base) into *rbase. False: the walk leaves the line (or a tie needs the full IDs).
__device__ __forceinline__ bool ncl2_lane_answer(const uint32_t (&d)[32], uint64_t thi, uint32_t count, uint32_t* lrow,
                                                 uint32_t& m) {
    constexpr int S = (int)NCL2_SLOTS, PMIN = (int)NCL2_PMIN, PMAX = (int)NCL2_PMAX;
    const uint32_t sh = (d[1] >> 8) & 63u, fl = d[1] >> 16;
    const uint32_t tx = ((uint32_t)(thi >> sh) & 0xFFFFFFu) << 8;
    uint32_t k[S];
    uint32_t p = PMIN, z = NONE;
#pragma unroll
    for (int e = 0; e < S; e++) {
        const uint32_t val = ncl2_key24x(d, e);
        if (e >= PMIN && e < PMAX) p += val < tx ? 1u : 0u;  // the slot's nodes below the target (at 24 bits)
        // the distance's 24 bits << 8 | expired (node w0 + e at bit e of dw2..3), taken in here so that the header
        // dies with the line
        k[e] = (val ^ tx) | ((d[2 + e / 32] >> (e % 32)) & 1u);
        // a distance of zero at 24 bits in the slot (lb needs the full IDs) or just left of it (the runs may tie)
        if (e >= PMIN - 1 && e < PMAX) z = min(z, k[e]);
    }
    bool ex = (fl & 1u) || z < 256u;
    // runs: the left one from position PMAX - 1 down over the positions below p, the right one from PMIN up over the
    // others. The two sets are disjoint, so each position's distance turns into its side's key in place (the line's
    // keys and the walk fit in 64 VGPRs).
    uint32_t runL = 0, runR = 0, endL = NONE, endR = NONE;
#pragma unroll
    for (int e = PMAX - 1; e >= 0; e--) {
        const bool L = e < PMIN || (uint32_t)e < p;
        runL = max(runL, L ? k[e] : 0u);  // (the run's low byte is some node's expired bit: masked below)
        if (L) k[e] = (runL & ~255u) | ((uint32_t)(63 - e) << 1) | (k[e] & 1u);
    }
    if (fl & 2u) endL = k[0] | 1u;  // more nodes left of the line (the end node itself, expired or not, is in it)
#pragma unroll
    for (int e = PMIN; e < S; e++) {
        const bool R = e >= PMAX || (uint32_t)e >= p;
        runR = max(runR, R ? k[e] : 0u);
        if (R) k[e] = (runR & ~255u) | 128u | ((uint32_t)e << 1) | (k[e] & 1u);
    }
    if (fl & 4u) endR = k[S - 1] | 1u;  // more nodes right of the line
    const uint32_t lim = min(endL, endR);
    // the 32 smallest of the bitonic 64 (k, then NONE), sorted
#pragma unroll
    for (int r = 0; r + 32 < S; r++) k[r] = min(k[r], k[r + 32]);
    // the first NCL2_STEPS of those sorted: the 16 smallest (a half-cleaner at 16, then four levels), and the 8 next
    // (the upper 16 are bitonic: the smaller half of one more half-cleaner, then three levels). 24 walk steps hold
    // count <= 14 non-expired nodes unless more than 10 of them are expired (the wave path then answers)
    if (NCL2_STEPS == 32) {
#pragma unroll
        for (int h = 16; h >= 1; h >>= 1)
#pragma unroll
            for (int r = 0; r < 32; r++)
                if ((r & h) == 0) cx(k[r], k[r + h]);
    } else {
#pragma unroll
        for (int r = 0; r < 16; r++) cx(k[r], k[r + 16]);
#pragma unroll
        for (int h = 8; h >= 1; h >>= 1)
#pragma unroll
            for (int r = 0; r < 16; r++)
                if ((r & h) == 0) cx(k[r], k[r + h]);
#pragma unroll
        for (int r = 16; r < 24; r++) k[r] = min(k[r], k[r + 8]);
#pragma unroll
        for (int h = 4; h >= 1; h >>= 1)
#pragma unroll
            for (int r = 16; r < 24; r++)
                if ((r & h) == 0) cx(k[r], k[r + h]);
    }
    uint32_t have = 0;
#pragma unroll
    for (int r = 0; r < (int)NCL2_STEPS; r++) {
        const bool keep = k[r] <= lim && !(k[r] & 1u);
        if (keep && have < count) lrow[have] = k[r];
        have += keep ? 1u : 0u;
    }
    m = min(count, have);
    ex |= have < count && (lim != NONE || k[NCL2_STEPS - 1] != NONE);  // the walk goes on past the line / the steps
    return !ex;
}

// The block's rows from raw walk keys (row r's keys at rows[r * NCL2_RS ..], its meta word m | answered << 8 and its
// node base at meta[r] / base[r]) as one run of 16-byte stores; rows not answered are skipped dword by dword.
template <int NT>
__device__ __forceinline__ void store_rows_keys16(uint32_t* __restrict__ out_idx, uint32_t q, uint32_t count,
                                                  const uint32_t* rows, const uint32_t* meta, const uint32_t* base) {
    const uint32_t tid = threadIdx.x, q0 = blockIdx.x * NT;
    const uint32_t nq = min((uint32_t)NT, q - q0), nw = nq * count;
    uint32_t* dst = out_idx + (size_t)q0 * count;
    const bool al = ((uintptr_t)out_idx & 15u) == 0;  // NT * count * 4 is a multiple of 16
    for (uint32_t c4 = tid; 4 * c4 < nw; c4 += NT) {
        const uint32_t w0 = 4 * c4;
        uint32_t r = w0 / count, c = w0 - r * count, v[4];
        bool okv[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const bool in = w0 + u < nw;
            const uint32_t mt = in ? meta[r] : 0u;
            okv[u] = in && ((mt >> 8) & 1u);
            v[u] = NONE;
            if (in && c < (mt & 255u)) {
                const uint32_t key = rows[r * NCL2_RS + c], f = (key >> 1) & 63u;
                v[u] = base[r] + ((key & 128u) ? f : 63u - f);
            }
            if (++c == count) { c = 0; r++; }
        }
        if (al && okv[0] && okv[1] && okv[2] && okv[3]) {
            st_row4(dst + w0, v[0], v[1], v[2], v[3]);
        } else {
#pragma unroll
            for (int u = 0; u < 4; u++)
                if (okv[u]) st_row1(dst + w0 + u, v[u]);
        }
    }
}

// ABL 1 (timing ablation only, KAD_NC_KERNEL=lane_abl1; results wrong): the lines and the answer, no wave path. ABL 9
// (lane_abl9): the wave path's loads without its answers; ABL 11 (lane_abl11): the same and a whole row of plain stores
// per missed query; ABL 12 (lane_abl12): the wave path without its serial fallback (rows of walks past 32 steps a side
// missing). ABL 5 (lane_stats): out_cnt = the step that answered (1: the line, 2: the wave path, 3: the wave path's
// serial fallback).
// WPE: the waves per SIMD the register allocation aims at (5: 85 VGPRs, no spill; 6 and 8 spill: A/B only). NT: threads
// per workgroup (64: a wave that runs the wave path for a missed query holds only its own slot, not its block's).
template <int ABL, bool DUAL, int WPE, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void ncl2_lane_kernel(
    DevTable T4, DevTable T6, const uint8_t* __restrict__ af, const uint8_t* __restrict__ targets, uint32_t q,
    uint32_t count, uint32_t* __restrict__ out_idx, uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * NT + threadIdx.x, lane = threadIdx.x & 63u, tid = threadIdx.x;
    const bool act = i < q;
    const bool fam = DUAL && act && af[i] != 0;
    // 76 bytes per query. meta[r] = m | answered << 8 | header valid << 9 | the slot's node count << 16
    __shared__ uint32_t rows[NT * NCL2_RS], meta[NT], base[NT];
    bool ok = false;
    uint32_t m = 0, hv = 0;  // hv: header valid << 9 | the slot's node count << 16 (from the line header)
    if (act) {
        const uint64_t thi = load_target_hi(targets, i);  // the line path reads the top 64 bits alone
        const DevTable& T = fam ? T6 : T4;
        if (T.n == 0) {  // empty map: no nodes
            ok = true;
        } else if ((T.flags & TF_NCL) && thi >= T.nbase && ((thi - T.nbase) >> T.nshift) < T.nslots) {
            // below the first slot / past the last: lb = 0 / n, windows clamped at the ends (the wave path)
            const uint4* lp = T.ncl + (size_t)NCL_PIECES * T.nslots + 8ull * ((thi - T.nbase) >> T.nshift);
            uint32_t d[32];
#pragma unroll
            for (int x = 0; x < 8; x++) {
                const uint4 u = lp[x];
                d[4 * x] = u.x; d[4 * x + 1] = u.y; d[4 * x + 2] = u.z; d[4 * x + 3] = u.w;
            }
            if (!((d[1] >> 16) & 1u)) hv = 512u | ((d[1] & 255u) << 16);
            base[tid] = d[0] + T.index_base;
            ok = ncl2_lane_answer(d, thi, count, rows + tid * NCL2_RS, m);
        }
    }
    if (act && ok && out_cnt) out_cnt[i] = (uint8_t)(ABL == 5 ? 1u : m);
    meta[tid] = m | (ok ? 256u : 0u) | hv;
    if (NT > 64) __syncthreads(); else wave_sync();
    // the lanes the line could not answer (0.11 % of the queries at k = 14): one query at a time by the whole wave,
    // its target read again (wave-uniform) and its slot range from the line header when there is one. The first
    // one's target and window loads go out before the row store, each next one's before the current one's answer.
    // (Run before the row store instead, the wave path measured the same: profiles/r06/ncl_lane/ncl_lane11.)
    uint64_t pend = ABL == 1 ? 0ull : __ballot(act && !ok);
    const uint64_t fm = DUAL ? __ballot(fam) : 0ull;
    Target u{};
    NcWindow w{0, 0, 0};
    uint32_t qi = 0, r0 = 0, r1 = 0;
    bool f6 = false;
    auto fetch = [&](uint32_t l) {
        qi = i - lane + l;
        u = load_target(targets, qi);
        f6 = DUAL && ((fm >> l) & 1ull);  // wave-uniform
        const DevTable& T = f6 ? T6 : T4;
        const uint32_t mt = meta[tid - lane + l];
        if (mt & 512u) {  // no radix load
            const uint32_t ns = (mt >> 16) & 255u;
            r0 = base[tid - lane + l] - T.index_base + NCL2_MID - ns / 2;
            r1 = r0 + ns;
        } else {
            nc_slot(T, u, r0, r1);
        }
        w = nc_window(T, r0, lane);
    };
    if (pend) fetch((uint32_t)__builtin_ctzll(pend));
    store_rows_keys16<NT>(out_idx, q, count, rows, meta, base);
    uint64_t failed = 0;  // lanes whose query the wave path could not settle
    while (pend) {
        pend &= pend - 1;
        const Target uc = u;
        const NcWindow wc = w;
        const uint32_t qc = qi, a0 = r0, a1 = r1;
        const bool c6 = f6;
        if (pend) fetch((uint32_t)__builtin_ctzll(pend));
        if (ABL == 9) {  // the misses' loads without their answers (results wrong)
            if (lane == 0) out_idx[(size_t)qc * count] = (uint32_t)(wc.k0 ^ wc.k1 ^ uc.hi) + a0 + a1 + c6;
            continue;
        }
        if (ABL == 11) {  // the misses' loads and a whole row of plain stores, no answer (results wrong)
            if (lane < count) out_idx[(size_t)qc * count + lane] = (uint32_t)(wc.k0 ^ wc.k1 ^ uc.hi) + a0 + a1 + c6;
            continue;
        }
        const bool wok = nc_answer(c6 ? T6 : T4, uc, a0, a1, wc, lane, qc, count, out_idx, out_cnt, false);
        if (ABL == 5 && lane == 0 && out_cnt) out_cnt[qc] = wok ? 2 : 3;
        if (!wok) failed |= 1ull << (qc - (i - lane));  // (wave-uniform)
    }
    // the walks the wave path could not settle (longer than 32 steps a side, or 64-bit ties it cannot order: never on
    // the bench shard): lane 0's serial walk, after the loop (its code costs ~1 us per 1M at k = 14 although it never
    // runs, inside the loop or here: ABL 12, profiles/r06/ncl_lane/ncl_lane13)
    while (ABL != 12 && failed) {
        const uint32_t l = (uint32_t)__builtin_ctzll(failed);
        failed &= failed - 1;
        const uint32_t qf = i - lane + l;
        const DevTable& T = (DUAL && ((fm >> l) & 1ull)) ? T6 : T4;
        if (lane == 0) nc_serial(T, load_target(targets, qf), count, out_idx + (size_t)qf * count, out_cnt ? out_cnt + qf : nullptr);
    }
}

// NodeCache counts 17..64 for two families (af per query): nc_two_pass_kernel with the table chosen per
// wave (one query per wave); an empty family map gives zero results.
__global__ __launch_bounds__(BLOCK) void nc_two_pass_dual_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ af,
                                                                 const uint8_t* __restrict__ targets, uint32_t q,
                                                                 uint32_t count, uint32_t* __restrict__ out_idx,
                                                                 uint8_t* __restrict__ out_cnt) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t qi = blockIdx.x * (BLOCK / 64) + threadIdx.x / 64;
    if (qi >= q) return;  // one query per wave: the whole wave leaves
    const DevTable& T = af[qi] ? T6 : T4;
    if (T.n == 0) {
        if (lane < count) out_idx[(size_t)qi * count + lane] = NONE;
        if (lane == 0 && out_cnt) out_cnt[qi] = 0;
        return;
    }
    const Target t = load_target(targets, qi);
    uint32_t r0, r1;
    nc_slot(T, t, r0, r1);
    const NcWindow w = nc_window(T, r0, lane);
    if (!nc_answer(T, t, r0, r1, w, lane, qi, count, out_idx, out_cnt, false))
        nc64_query(T, t, lane, qi, count, out_idx, out_cnt, true);
}

// The 128-byte line of a slot ([r0, r1) its nodes, ns = r1 - r0 <= 15), the 37 nodes w0 = r0 + ns / 2 - 18 ..:
//   dw0      w0
//   dw1      ns | sh << 8 | (defer | truncated left << 1 | truncated right << 2) << 16
//   dw2..3   the expired bits of the 37 window nodes (node w0 + e at bit e)
//   bytes 16 + 3e .. 18 + 3e   key24 of node w0 + e (little-endian; key24 as in the 256-byte lines, from the window's
//            own common prefix)
// The slot's nodes sit at positions 18 - ns / 2 .. 17 + ns - ns / 2, inside [11, 26). A clamped window or a slot of
// more than 15 nodes is deferred (the 256-byte line answers).
__device__ __forceinline__ void ncl2_build_line(const uint64_t* key, const uint8_t* status, uint32_t r0, uint32_t r1,
                                                uint32_t n, uint32_t slot_prefix, uint4* L2) {
    const uint32_t ns = r1 - r0, c = r0 + ns / 2;
    if (ns > NCL2_XMAX || c < NCL2_MID || (uint64_t)c - NCL2_MID + NCL2_SLOTS > n) {
        L2[0] = make_uint4(0u, 1u << 16, 0u, 0u);
        return;
    }
    const uint32_t w0 = c - NCL2_MID;
    const uint32_t P = (uint32_t)__builtin_clzll((key[w0] ^ key[w0 + NCL2_SLOTS - 1]) | 1ull);
    const uint32_t Pp = min(min(P, slot_prefix), 40u), sh = 40 - Pp;
    uint32_t d[32];
#pragma unroll
    for (int x = 0; x < 32; x++) d[x] = 0;
#pragma unroll
    for (int e = 0; e < (int)NCL2_SLOTS; e++) {
        const uint32_t k24 = (uint32_t)(key[w0 + e] >> sh) & 0xFFFFFFu;
        const int o = 3 * e, w = 4 + o / 4, b = 8 * (o % 4);
        d[w] |= k24 << b;
        if (b > 8) d[w + 1] |= k24 >> (32 - b);
        d[2 + e / 32] |= ((status[w0 + e] & KAD_STATUS_EXPIRED) ? 1u : 0u) << (e % 32);
    }
    d[0] = w0;
    d[1] = ns | (sh << 8) | ((w0 > 0 ? 2u : 0u) | (w0 + NCL2_SLOTS < n ? 4u : 0u)) << 16;
#pragma unroll
    for (int x = 0; x < 8; x++) L2[x] = make_uint4(d[4 * x], d[4 * x + 1], d[4 * x + 2], d[4 * x + 3]);
}

// NodeCache lines after a status change (or at creation): one thread per radix slot, its 256-byte and its 128-byte
// line (lines: the 256-byte lines of all slots, then the 128-byte ones).
__global__ void ncl_build_kernel(const uint64_t* key, const uint8_t* status, const uint32_t* nrdx, uint32_t nslots,
                                 uint32_t n, uint32_t slot_prefix, uint32_t* lines, LineSel sel) {
    // one item per thread, grid-stride (an incremental rebuild launches a capped grid)
    for (uint32_t j_ = blockIdx.x * BLOCK + threadIdx.x;; j_ += gridDim.x * BLOCK) {
        uint32_t s;
        if (!sel.pick(j_, nslots, s)) return;
        [&] {
    uint32_t* L = lines + (size_t)NCL_STRIDE * s;
    const uint32_t r0 = nrdx[s], r1 = nrdx[s + 1], ns = r1 - r0;
    ncl2_build_line(key, status, r0, r1, n, slot_prefix,
                    reinterpret_cast<uint4*>(lines + (size_t)NCL_STRIDE * nslots + (size_t)NCL2_DWORDS * s));
    if (r0 < NCL_LEFT || (uint64_t)r0 - NCL_LEFT + NCL_SLOTS > n || ns > NCL_XMAX) {  // clamped window / wide slot
        L[0] = 0; L[1] = 0; L[2] = 1u; L[3] = 0;
        return;
    }
    const uint32_t w0 = r0 - NCL_LEFT;
    const uint32_t P = (uint32_t)__builtin_clzll((key[w0] ^ key[w0 + NCL_SLOTS - 1]) | 1ull);
    const uint32_t Pp = min(min(P, slot_prefix), 40u), sh = 40 - Pp;
    for (uint32_t j = 0; j < NCL_SLOTS; j++) {  // (equal neighbours: ncl_answer checks the pair around lb)
        const uint32_t k24 = (uint32_t)(key[w0 + j] >> sh) & 0xFFFFFFu;
        L[4 + j] = (k24 << 8) | ((status[w0 + j] & KAD_STATUS_EXPIRED) ? 1u : 0u);
    }
    L[0] = w0;
    L[1] = ns | (sh << 8);
    L[2] = (w0 > 0 ? 2u : 0u) | (w0 + NCL_SLOTS < n ? 4u : 0u);
    L[3] = 0;
        }();
    }
}

// ---------------------------------------------------------------------------------------
// NodeCache lines for counts 17..32 (TF_NCL32): one 384-byte line per node radix slot s, the 92-node window
// w0 = r0-44 .. r0+47 of the sorted node array ([r0, r1) = the slot's nodes, at most 15):
//   dw0      w0
//   dw1      ns = r1 - r0 | sh << 8
//   dw2      defer (a clamped or wide slot) | truncated left (w0 > 0) << 1 | truncated right (w0 + 92 < n) << 2
//   dw4..95  element e (node w0 + e): key24 << 8 | expired, key24 as in the 256-byte lines
// A query is answered by 8 lanes (an octet; 8 queries per wave). The octet stages its line in LDS with
// 16-byte loads, counts the slot's nodes below the target (lb = w0 + p, p = 44 + x), and reads the
// first 64 steps of each run: lane g holds left steps 8g..8g+7 (element p-1-step) and right steps
// 63-8g-u (element p+step). A run's prefix maxima of the XOR distance (in-lane, then across the octet)
// give each element the key (M << 8 | side << 7 | step << 1 | expired); each run's keys ascend with the
// step, the walk's order is the keys' order (node_cache.cpp:36-66, the greedy merge of the 256-byte
// lines), so the walk's first 64 steps are min(left[r], right[63-r]) followed by a bitonic half-cleaner
// cascade (three stages across lanes, three inside). The first `count` non-expired steps are the answer;
// a run cut by the window's truncated end limits the trusted keys to that end's key. A query with fewer
// than `count` trusted emissions, a deferred line, a target equal in key24 to a slot node, or equal key24
// either side of its position takes the two-pass wave path (nc_answer, then nc64_query / the serial walk).
// ---------------------------------------------------------------------------------------
// 384-byte lines, 44 nodes left of the slot: the count-32 walk rarely goes past 40 steps on a side
// (tools/nc32_walk_extent.py: p99 37, max 44 in 20k walks), and the 512-byte form (124 slots, 56 left) read a third more
// bytes for nothing: 121.9-122.9 -> 116.9-119.2 us at k = 32, 130-134 -> 119-122 at k = 24 (profiles/r05/nc96/)
#ifndef KAD_NC32_STRIDE
#define KAD_NC32_STRIDE 96u
#define KAD_NC32_LEFT 44u
#endif
constexpr uint32_t NC32_STRIDE = KAD_NC32_STRIDE, NC32_SLOTS = NC32_STRIDE - 4, NC32_LEFT = KAD_NC32_LEFT,
                   NC32_XMAX = 15;  // dwords
static_assert(NC32_STRIDE % 32 == 0 && NC32_STRIDE <= 128 && NC32_LEFT + NC32_XMAX < NC32_SLOTS, "NodeCache-32 line");

// Octet (8-lane group) cross-lane moves without address arithmetic: quad permutes and row shifts by DPP, the lane-4
// exchange and the octet broadcast by ds_swizzle's bit-mask mode (lane' = ((lane & and) | or) ^ xor within 32 lanes).
// __shfl_xor / __shfl_up with width 8 compiled to ds_bpermute with a per-lane address (several VALU ops each).
template <int O>  // the value of lane g ^ O of the octet (O = 1, 2, 4)
__device__ __forceinline__ uint32_t oct_xor(uint32_t v) {
    if constexpr (O == 1) return qdpp<QP_X1>(v);
    else if constexpr (O == 2) return qdpp<QP_X2>(v);
    else return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x1F | (4 << 10));
}
template <int O>  // the value of lane g - O (row_shr; the caller masks g < O, which read another octet or 0)
__device__ __forceinline__ uint32_t oct_up(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x110 | O, 0xF, 0xF, true);
}
template <int O>  // the value of lane g + O (row_shl; the caller masks g + O > 7)
__device__ __forceinline__ uint32_t oct_down(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x100 | O, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t oct_last(uint32_t v) {  // lane 7 of the octet
    return (uint32_t)__builtin_amdgcn_ds_swizzle((int)v, 0x18 | (0x07 << 5));
}

// One octet per radix slot: lane g builds dwords [16g, 16g + 16) of line s.
__global__ __launch_bounds__(BLOCK) void ncl32_build_kernel(const uint64_t* key, const uint8_t* status,
                                                             const uint32_t* nrdx, uint32_t nslots, uint32_t n,
                                                             uint32_t slot_prefix, uint32_t* lines, LineSel sel) {
    const uint32_t g = threadIdx.x & 7u;
    // one item per thread, grid-stride (an incremental rebuild launches a capped grid)
    for (uint32_t j_ = (blockIdx.x * BLOCK + threadIdx.x) >> 3;; j_ += (gridDim.x * BLOCK) >> 3) {
        uint32_t s;
        if (!sel.pick(j_, nslots, s)) return;
        [&] {
    uint4* dst = reinterpret_cast<uint4*>(lines + (size_t)NC32_STRIDE * s) + 4 * g;
    const uint32_t r0 = nrdx[s], r1 = nrdx[s + 1], ns = r1 - r0;
    if (r0 < NC32_LEFT || (uint64_t)r0 - NC32_LEFT + NC32_SLOTS > n || ns > NC32_XMAX) {  // clamped / wide slot
        if (g == 0) dst[0] = make_uint4(0u, 0u, 1u, 0u);
        return;
    }
    const uint32_t w0 = r0 - NC32_LEFT;
    const uint32_t P = (uint32_t)__builtin_clzll((key[w0] ^ key[w0 + NC32_SLOTS - 1]) | 1ull);
    const uint32_t Pp = min(min(P, slot_prefix), 40u), sh = 40 - Pp;
    // (equal key24 between neighbours no longer defers the line: nc32_line_kernel checks the one pair that can change
    // the walk's order, the two elements either side of the target's position)
    if (16 * g >= NC32_STRIDE) return;  // (a line of fewer than 128 dwords: its first NC32_STRIDE / 16 lanes)
    uint32_t v[16];
#pragma unroll
    for (int u = 0; u < 16; u++) {
        const int j = 16 * (int)g + u, e = j - 4;
        if (e < 0) { v[u] = 0; continue; }
        const uint32_t k24 = (uint32_t)(key[w0 + e] >> sh) & 0xFFFFFFu;
        v[u] = (k24 << 8) | ((status[w0 + e] & KAD_STATUS_EXPIRED) ? 1u : 0u);
    }
    if (g == 0) {
        v[0] = w0;
        v[1] = ns | (sh << 8);
        v[2] = (w0 > 0 ? 2u : 0u) | (w0 + NC32_SLOTS < n ? 4u : 0u);
        v[3] = 0;
    }
#pragma unroll
    for (int x = 0; x < 4; x++) dst[x] = make_uint4(v[4 * x], v[4 * x + 1], v[4 * x + 2], v[4 * x + 3]);
        }();
    }
}

// DUAL: the family per query (af[i] = 0 -> T4, 1 -> T6), an empty family map gives zero results.
// ABL 1 (timing ablations only, results wrong): no wave fallback; 2: also no merge (the line loads and one store);
// 3: path statistics (out_cnt = 250 for the queries the wave path answers).
template <int ABL, bool DUAL>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void nc32_line_kernel(DevTable T4, DevTable T6, const uint8_t* __restrict__ af,
                                                          const uint8_t* __restrict__ targets, uint32_t q,
                                                          uint32_t count, uint32_t* __restrict__ out_idx,
                                                          uint8_t* __restrict__ out_cnt) {
    // the octets' rows of NC32_STRIDE + 4 dwords, with padding before the first and after the last: the run steps
    // below read their elements at unclamped indices (NC32_LEFT - 60 .. NC32_LEFT + NC32_XMAX + 67 of a row) and mask
    // the ones outside
    constexpr uint32_t NC32_ROW = NC32_STRIDE + 4;
    constexpr uint32_t PADF = (64u - NC32_LEFT + 7u) & ~7u, PADB = NC32_LEFT + NC32_XMAX + 68u - NC32_ROW + 8u;
    __shared__ uint32_t ldsf[PADF + (BLOCK / 8) * NC32_ROW + PADB];
    const uint32_t lane = threadIdx.x & 63u, g = threadIdx.x & 7u;
    const uint32_t qi = (blockIdx.x * BLOCK + threadIdx.x) >> 3;
    const bool act = qi < q;
    const bool fam = DUAL && act && af[qi] != 0;
    const DevTable& T = fam ? T6 : T4;  // octet-uniform
    uint32_t* W = ldsf + PADF + (threadIdx.x >> 3) * NC32_ROW;
    bool ok = false, line = false;
    uint64_t thi = 0;
    uint32_t s = 0;
    if (act) {
        if (T.n == 0) {  // empty map
            for (uint32_t j = g; j < count; j += 8) out_idx[(size_t)qi * count + j] = NONE;
            if (g == 0 && out_cnt) out_cnt[qi] = 0;
            ok = true;
        } else if (T.flags & TF_NCL32) {
            thi = load_target_hi(targets, qi);
            line = thi >= T.nbase && ((thi - T.nbase) >> T.nshift) < T.nslots;
            s = line ? (uint32_t)((thi - T.nbase) >> T.nshift) : 0u;
        }
    }
    if (line) {  // load x: the octet reads 128 contiguous bytes, lane g the 16 at 128x + 16g
        const uint4* src = T.ncl32 + (size_t)(NC32_STRIDE / 4) * s + g;
        uint4 x4[NC32_STRIDE / 32];
#pragma unroll
        for (int x = 0; x < (int)NC32_STRIDE / 32; x++) x4[x] = src[8 * x];
#pragma unroll
        for (int x = 0; x < (int)NC32_STRIDE / 32; x++) {
            W[32 * x + 4 * g] = x4[x].x; W[32 * x + 4 * g + 1] = x4[x].y;
            W[32 * x + 4 * g + 2] = x4[x].z; W[32 * x + 4 * g + 3] = x4[x].w;
        }
    }
    // (the octet's row is its own: its wave's LDS order suffices — reads past the row into a neighbour's, which
    // another wave may still be writing, are masked out below)
    wave_sync();
    if (ABL == 2) {
        if (line) out_idx[(size_t)qi * count + g] = W[g] ^ W[64 + g] ^ W[NC32_STRIDE - 1 - g];
        return;
    }
    if (line) {
        const uint32_t w0 = W[0], ns = W[1] & 255u, sh = (W[1] >> 8) & 63u, fl = W[2];
        const uint32_t t24 = (uint32_t)(thi >> sh) & 0xFFFFFFu;
        // lb: the slot's nodes below the target (elements NC32_LEFT .. NC32_LEFT+ns-1, two per lane)
        uint32_t below = 0, eq = 0;
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t e = NC32_LEFT + 2 * g + u;
            if (e < NC32_LEFT + ns) {
                const uint32_t k24 = W[4 + e] >> 8;
                below += k24 < t24 ? 1u : 0u;
                eq |= k24 == t24 ? 1u : 0u;
            }
        }
        below += oct_xor<1>(below);
        eq |= oct_xor<1>(eq);
        below += oct_xor<2>(below);
        eq |= oct_xor<2>(eq);
        below += oct_xor<4>(below);
        eq |= oct_xor<4>(eq);
        const uint32_t p = NC32_LEFT + below;
        // the window's key24 values are monotone (its nodes share the top Pp bits), so equal ones are neighbours, and
        // a left-run and a right-run element can share one (a tie at 24 bits between the runs, which only the full IDs
        // order) only if elements p-1 and p do: then the exact path (the builder no longer defers a line for equal
        // neighbours elsewhere in the window: 0.5 % of count-32 queries took the wave path for that)
        bool ex = (fl & 1u) || eq || (W[4 + p - 1] >> 8) == (W[4 + p] >> 8);
        // the runs' first 64 steps: left step 8g+u = element p-1-step, right step 63-8g-u = element p+step. Key:
        // distance24 << 8 | side << 7 | step << 1 | expired. A step outside the line's window is NONE: it sorts
        // after every step inside, is never emitted (its expired bit is set), and (the outside steps are a suffix
        // of their run) the run maxima below pass it on only to other outside steps, so no step needs a validity
        // test after this.
        // (all 16 elements read first at unclamped indices — one base per side and constant offsets — then masked:
        // a clamped index per element had compiled to a branch and an LDS round trip per element)
        uint32_t ka[8], kb[8];
        {
            const uint32_t* Wa = W + 4 + (int)p - 1 - 8 * (int)g;   // element p-1-ra = Wa[-u]
            const uint32_t* Wb = W + 4 + (int)p + 63 - 8 * (int)g;  // element p+rb = Wb[-u]
            uint32_t xa[8], xb[8];
#pragma unroll
            for (int u = 0; u < 8; u++) {
                xa[u] = Wa[-u];
                xb[u] = Wb[-u];
            }
            // an element is key24 << 8 | expired (bits 1..7 clear), so x ^ t24 << 8 is the distance key with its expired
            // bit, and the step goes into bits 1..6 by an OR: ra << 1 = 16g | 2u, rb << 1 = 16(7 - g) | (14 - 2u).
            // Valid: ra < p <=> u < p - 8g; p + rb < NC32_SLOTS <=> u > p + 63 - NC32_SLOTS - 8g (four ops per element)
            const uint32_t T8 = t24 << 8, ga = 16u * g, gb = 128u | (16u * (7u - g));
            const int dA = (int)p - 8 * (int)g, dB = (int)p + 63 - (int)NC32_SLOTS - 8 * (int)g;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t a = (xa[u] ^ T8) | ga | (2u * u);
                const uint32_t b = (xb[u] ^ T8) | gb | (14u - 2u * u);
                ka[u] = u < dA ? a : NONE;
                kb[u] = u > dB ? b : NONE;
            }
        }
        // run maxima: in the lane (left: u ascending, right: u descending) over whole keys (their top 24 bits
        // are the distance maxima), then the runs' earlier lanes (left: lower g, right: higher g); a shuffle
        // from outside the octet returns the lane's own value, which max leaves alone
        uint32_t pa[8], pb[8], ca = 0, cb = 0;
#pragma unroll
        for (int u = 0; u < 8; u++) pa[u] = ca = max(ca, ka[u]);
#pragma unroll
        for (int u = 7; u >= 0; u--) pb[u] = cb = max(cb, kb[u]);
        // (lanes whose partner lies outside the octet take 0, which max leaves alone). Every lane runs the move and
        // then selects: a move under `cond ? move : 0` runs with the other lanes off, and a DPP read of an inactive
        // lane returns 0.
        {
            uint32_t ya = oct_up<1>(ca), yb = oct_down<1>(cb);
            ca = max(ca, g >= 1 ? ya : 0u);
            cb = max(cb, g + 1 <= 7 ? yb : 0u);
            ya = oct_up<2>(ca);
            yb = oct_down<2>(cb);
            ca = max(ca, g >= 2 ? ya : 0u);
            cb = max(cb, g + 2 <= 7 ? yb : 0u);
            ya = oct_up<4>(ca);
            yb = oct_down<4>(cb);
            ca = max(ca, g >= 4 ? ya : 0u);
            cb = max(cb, g + 4 <= 7 ? yb : 0u);
        }
        const uint32_t ua = oct_up<1>(ca), ub = oct_down<1>(cb);
        uint32_t inA = g > 0 ? ua : 0u, inB = g < 7 ? ub : 0u;
        asm volatile("" : "+v"(inA), "+v"(inB));  // (kept as values: folded into each max, the select ran per element)
#pragma unroll
        for (int u = 0; u < 8; u++) {  // the key's distance = the run maximum up to the step (bitfield insert)
            ka[u] = (max(pa[u], inA) & 0xFFFFFF00u) | (ka[u] & 255u);
            kb[u] = (max(pb[u], inB) & 0xFFFFFF00u) | (kb[u] & 255u);
        }
        // keys beyond a run cut short by the window's truncated end are not trusted: the run's last step inside
        // the window (left: step p-1, right: step NC32_SLOTS-1-p) bounds them
        uint32_t lim = NONE;
        if ((fl & 2u) && p <= 64) {
            const uint32_t r = p - 1, ux = r & 7u;
            uint32_t v = ka[0];
#pragma unroll
            for (int u = 1; u < 8; u++) v = ux == (uint32_t)u ? ka[u] : v;
            lim = min(lim, (uint32_t)__shfl((int)v, (int)((lane & ~7u) | (r >> 3)), 64));
        }
        if ((fl & 4u) && NC32_SLOTS - p <= 64) {
            const uint32_t r = 63u - (NC32_SLOTS - 1 - p), ux = r & 7u;  // that step sits at u = r & 7, g = r >> 3
            uint32_t v = kb[0];
#pragma unroll
            for (int u = 1; u < 8; u++) v = ux == (uint32_t)u ? kb[u] : v;
            lim = min(lim, (uint32_t)__shfl((int)v, (int)((lane & ~7u) | (r >> 3)), 64));
        }
        // the walk's first 64 steps: min(left[r], right[63-r]) is bitonic; half-cleaners sort it. Across lanes
        // the low lane of a pair keeps the min and the high one the max: med3(w, partner, 0 or ~0) in one op.
        uint32_t w[8];
#pragma unroll
        for (int u = 0; u < 8; u++) w[u] = min(ka[u], kb[u]);
        {
            const uint32_t hi4 = (g & 4u) ? 0xFFFFFFFFu : 0u, hi2 = (g & 2u) ? 0xFFFFFFFFu : 0u,
                           hi1 = (g & 1u) ? 0xFFFFFFFFu : 0u;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t y = oct_xor<4>(w[u]);
                w[u] = max(min(w[u], y), min(max(w[u], y), hi4));  // v_med3_u32
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t y = oct_xor<2>(w[u]);
                w[u] = max(min(w[u], y), min(max(w[u], y), hi2));
            }
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t y = oct_xor<1>(w[u]);
                w[u] = max(min(w[u], y), min(max(w[u], y), hi1));
            }
        }
#pragma unroll
        for (int h = 4; h >= 1; h >>= 1)
#pragma unroll
            for (int u = 0; u < 8; u++)
                if ((u & h) == 0) cx(w[u], w[u + h]);
        // emissions: non-expired steps up to lim (outside steps and NONE carry the expired bit), ranked across
        // the octet
        uint32_t kept = 0;
        bool keep[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            keep[u] = w[u] <= lim && !(w[u] & 1u);
            kept += keep[u];
        }
        uint32_t cr = kept;
        {
            uint32_t y = oct_up<1>(cr);  // (moves outside the select, as above)
            cr += g >= 1 ? y : 0u;
            y = oct_up<2>(cr);
            cr += g >= 2 ? y : 0u;
            y = oct_up<4>(cr);
            cr += g >= 4 ? y : 0u;
        }
        const uint32_t tot = oct_last(cr);
        ok = !ex && tot >= count;
        // the row through the octet's LDS row (the line is no longer read): entry `rank` at W[rank]
        __builtin_amdgcn_wave_barrier();
        if (ok) {  // (every step written: the ones not emitted into a dummy dword past the row's entries)
            uint32_t rank = cr - kept;
            const uint32_t bp = w0 + T.index_base + p;
#pragma unroll
            for (int u = 0; u < 8; u++) {
                const uint32_t st = (w[u] >> 1) & 63u;
                const uint32_t val = (w[u] & 128u) ? bp + st : bp - 1u - st;
                W[keep[u] ? rank : NC32_ROW - 1] = val;  // (rank < 64: entries past `count` are never read)
                rank += keep[u] ? 1u : 0u;
            }
        }
        __builtin_amdgcn_wave_barrier();
        if (ok) {
            uint32_t* row = out_idx + (size_t)qi * count;
            if ((count & 3u) == 0 && ((uintptr_t)out_idx & 15u) == 0) {
                if (4 * g < count) st_row4(row + 4 * g, W[4 * g], W[4 * g + 1], W[4 * g + 2], W[4 * g + 3]);
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (4 * g + j < count) st_row1(row + 4 * g + j, W[4 * g + j]);
            }
            if (g == 0 && out_cnt) out_cnt[qi] = (uint8_t)count;
        }
    }
    if (ABL == 1 || ABL == 2) return;
    // the queries the lines could not answer: one at a time by the whole wave (the two-pass path)
    for (uint64_t pend = __ballot(act && g == 0 && !ok); pend; pend &= pend - 1) {
        const uint32_t l = (uint32_t)__builtin_ctzll(pend);
        const uint32_t qj = rdl(qi, l);
        const DevTable& Tj = (DUAL && rdl(fam ? 1u : 0u, l)) ? T6 : T4;  // wave-uniform
        const Target u = load_target(targets, qj);
        uint32_t r0, r1;
        nc_slot(Tj, u, r0, r1);
        const NcWindow wn = nc_window(Tj, r0, lane);
        if (!nc_answer(Tj, u, r0, r1, wn, lane, qj, count, out_idx, out_cnt, false))
            nc64_query(Tj, u, lane, qj, count, out_idx, out_cnt, true);
        if (ABL == 3 && lane == 0 && out_cnt) out_cnt[qj] = 250;
    }
}

// ---------------------------------------------------------------------------------------
// Incremental device mirror: kad_table_apply re-lays the node arrays out on
// the device from a host plan of segments (an untouched bucket is one range of old nodes; an edited
// bucket an explicit handle list), then re-derives masks, prefix sums, dup masks and lines on the
// device. Handles: old node index, or MIRROR_NEW | slot for a node of the batch.
// ---------------------------------------------------------------------------
using kadplan::MIRROR_NEW;
using kadplan::MirrorSeg;

__global__ void mirror_gather_kernel(const MirrorSeg* __restrict__ seg, uint32_t nseg, const uint32_t* __restrict__ list,
                                     uint32_t n_out, const uint64_t* __restrict__ okey, const uint32_t* __restrict__ otail,
                                     const uint8_t* __restrict__ ost, const uint64_t* __restrict__ nkey,
                                     const uint32_t* __restrict__ ntail, const uint8_t* __restrict__ nst,
                                     uint64_t* __restrict__ key, uint32_t* __restrict__ tail, uint8_t* __restrict__ st,
                                     uint32_t* __restrict__ remap, uint32_t* __restrict__ newidx) {
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= n_out) return;
    uint32_t lo = 0, hi = nseg;  // last segment with start <= p
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg[mid].start <= p) lo = mid; else hi = mid;
    }
    const MirrorSeg s = seg[lo];
    const uint32_t h = s.kind == 0 ? s.src + (p - s.start) : list[s.src + (p - s.start)];
    if (h & MIRROR_NEW) {
        const uint32_t x = h & ~MIRROR_NEW;
        key[p] = nkey[x];
        tail[3ull * p] = ntail[3ull * x];
        tail[3ull * p + 1] = ntail[3ull * x + 1];
        tail[3ull * p + 2] = ntail[3ull * x + 2];
        st[p] = nst[x];
        newidx[x] = p;
    } else {
        key[p] = okey[h];
        tail[3ull * p] = otail[3ull * h];
        tail[3ull * p + 1] = otail[3ull * h + 1];
        tail[3ull * p + 2] = otail[3ull * h + 2];
        st[p] = ost[h];
        if (remap) remap[h] = p;
    }
}

// Nodes whose top 64 ID bits equal another node's of the same bucket (tables whose bucket firsts
// have zero low 96 bits cannot hold such a pair across buckets).
__global__ void mirror_dmask_kernel(const uint64_t* key, const uint2* dir, uint32_t B, uint32_t* dmask, uint32_t* any) {
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    if (b >= B) return;
    const uint32_t j0 = dir[b].x & ~WIDE, j1 = dir[b + 1].x & ~WIDE;
    uint32_t m = 0;
    if (j1 - j0 <= 32)
        for (uint32_t i = j0; i < j1; i++)
            for (uint32_t j = j0; j < j1; j++)
                if (i != j && key[i] == key[j]) m |= 1u << (i - j0);
    dmask[b] = m;
    if (m) atomicOr(any, 1u);
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
// NodeCache map mutations (kad_nc_apply; node_cache.cpp:91-115): the sorted node array of a NodeCache-only
// table merged with a sorted batch of new IDs (NodeMap::getNode's emplace) minus erased entries (a dead
// weak_ptr found by getNode, clearBadNodes). Every kept old node and every new node computes its new
// position by binary search in the other sorted list; the NodeCache radix is re-derived by a binary search
// per radix slot. No host copy of the IDs is needed.
// ---------------------------------------------------------------------------------------
// #elements of the sorted (key, tail) list [0, n) that are < (k, t2, t3, t4) (strict lower bound); *eq = an
// element equals it.
__device__ __forceinline__ uint32_t lower_bound160(const uint64_t* key, const uint32_t* tail, uint32_t n, uint64_t k,
                                                   uint32_t t2, uint32_t t3, uint32_t t4, bool* eq) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        const uint32_t* tm = tail + 3ull * mid;
        if (cmp160(key[mid], tm[0], tm[1], tm[2], k, t2, t3, t4) < 0) lo = mid + 1; else hi = mid;
    }
    if (eq) {
        const uint32_t* tl = tail + 3ull * lo;
        *eq = lo < n && cmp160(key[lo], tl[0], tl[1], tl[2], k, t2, t3, t4) == 0;
    }
    return lo;
}

__global__ void nc_merge_old_kernel(const uint64_t* key, const uint32_t* tail, const uint8_t* st, const uint8_t* eflag,
                                    const uint32_t* erased_before, uint32_t n, const uint64_t* ikey,
                                    const uint32_t* itail, uint32_t m, uint64_t* key1, uint32_t* tail1, uint8_t* st1,
                                    uint32_t* remap) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    if (eflag[i]) { remap[i] = NONE; return; }
    const uint32_t* tl = tail + 3ull * i;
    const uint32_t c = lower_bound160(ikey, itail, m, key[i], tl[0], tl[1], tl[2], nullptr);
    const uint32_t pos = i - erased_before[i] + c;
    key1[pos] = key[i];
    tail1[3ull * pos] = tl[0]; tail1[3ull * pos + 1] = tl[1]; tail1[3ull * pos + 2] = tl[2];
    st1[pos] = st[i];
    remap[i] = pos;
}

// err: set when a new ID is already a (kept) key of the map (the caller's emplace would not insert it)
__global__ void nc_merge_new_kernel(const uint64_t* key, const uint32_t* tail, const uint8_t* eflag,
                                    const uint32_t* erased_before, uint32_t n, const uint64_t* ikey,
                                    const uint32_t* itail, const uint8_t* ist, uint32_t m, uint64_t* key1,
                                    uint32_t* tail1, uint8_t* st1, uint32_t* new_index, uint32_t* err) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= m) return;
    const uint32_t* tl = itail + 3ull * j;
    bool eq = false;
    const uint32_t c = lower_bound160(key, tail, n, ikey[j], tl[0], tl[1], tl[2], &eq);
    if (eq && !eflag[c]) atomicOr(err, 1u);
    const uint32_t pos = j + c - erased_before[c];
    key1[pos] = ikey[j];
    tail1[3ull * pos] = tl[0]; tail1[3ull * pos + 1] = tl[1]; tail1[3ull * pos + 2] = tl[2];
    st1[pos] = ist[j];
    new_index[j] = pos;
}

// NodeCache radix over a sorted key array: rdx[s] = #keys whose top 64 bits are below slot s's start.
__global__ void nc_radix_kernel(const uint64_t* key, uint32_t n, uint64_t base, uint32_t shift, uint32_t slots,
                                uint32_t* rdx) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    if (s > slots) return;
    const unsigned __int128 start = (unsigned __int128)base + ((unsigned __int128)s << shift);
    uint32_t lo = 0, hi = n;
    if (start >> 64) {
        lo = n;
    } else {
        const uint64_t st64 = (uint64_t)start;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (key[mid] < st64) lo = mid + 1; else hi = mid;
        }
    }
    rdx[s] = lo;
}

__global__ void flags_from_list_kernel(const uint32_t* list, uint32_t m, uint32_t n, uint8_t* flags, uint32_t* cnt) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= m) return;
    flags[list[j]] = 1;
    cnt[list[j]] = 1;
}

// ---------------------------------------------------------------------------------------
// Table maintenance: status from times, per-bucket good counts, exclusive scan -> dir.y
// ---------------------------------------------------------------------------------------
// Where a status change must be re-derived (incremental refresh): bdirty[b] = bucket b's good set changed
// (its mask, count and every line whose window reaches it), ndirty[s] = a NodeCache line whose 60-node
// window holds a node whose expired bit changed. Any of the pointers may be NULL (no such structure).
struct StatusMarks {
    uint8_t* bdirty;     // B
    uint8_t* ndirty;     // NodeCache radix slots
    const uint2* dir;    // bucket starts (node -> bucket)
    uint32_t B;
    const uint64_t* key; // node -> NodeCache slot
    uint64_t nbase;
    uint32_t nshift, nslots, n;
    uint32_t nback, nfwd; // NodeCache lines hold nodes r0(s)-nfwd .. r0(s)+nback-1 (the widest line set present)
    uint32_t* any;        // set to 1 by any change: the incremental rebuild's kernels exit at once without one
};

__device__ __forceinline__ void mark_status_change(const StatusMarks& M, uint32_t i, uint32_t old_st, uint32_t st) {
    if (M.any && *M.any == 0) *M.any = 1;  // a plain store of the same value: at most one per wave instruction
    if (M.bdirty && ((old_st ^ st) & KAD_STATUS_GOOD)) {
        uint32_t lo = 0, hi = M.B;  // the last bucket whose first node is <= i (upper_bound - 1)
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if ((M.dir[mid].x & ~WIDE) <= i) lo = mid + 1; else hi = mid;
        }
        if (lo) M.bdirty[lo - 1] = 1;
    }
    if (M.ndirty && ((old_st ^ st) & KAD_STATUS_EXPIRED)) {
        // NodeCache line s holds nodes r0(s)-nfwd .. r0(s)+nback-1 (28 / 32 for the 256-byte lines, 56 / 68 with
        // the 512-byte ones): every slot from that of node i-nback to that of node i+nfwd (a superset of the
        // slots whose window holds i)
        const uint32_t a = i >= M.nback ? i - M.nback : 0u, e = min(M.n - 1, i + M.nfwd);
        const uint64_t ka = M.key[a], ke = M.key[e];
        const uint64_t sa = ka < M.nbase ? 0 : min<uint64_t>((ka - M.nbase) >> M.nshift, M.nslots - 1);
        const uint64_t se = ke < M.nbase ? 0 : min<uint64_t>((ke - M.nbase) >> M.nshift, M.nslots - 1);
        for (uint64_t x = sa; x <= se; x++) M.ndirty[x] = 1;
    }
}

// node.cpp:34-40 with NODE_GOOD_TIME = 120 min, NODE_EXPIRE_TIME = 10 min (node.h:91-94)
constexpr int64_t NODE_GOOD_NS = 120LL * 60 * 1000000000LL, NODE_EXPIRE_NS = 10LL * 60 * 1000000000LL;

struct NodeTimes {
    const int64_t* time_ns;
    const int64_t* reply_ns;
    const uint8_t* expired;
};

// The status byte of node i at `now`: Node::isGood(now) (node.cpp:34-40) and Node::isExpired() (node.h:67).
__device__ __forceinline__ uint32_t status_at(const NodeTimes& N, uint32_t i, int64_t now) {
    const bool ex = N.expired[i] != 0;
    const bool good = !ex && N.reply_ns[i] >= now - NODE_GOOD_NS && N.time_ns[i] >= now - NODE_EXPIRE_NS;
    return (good ? KAD_STATUS_GOOD : 0u) | (ex ? KAD_STATUS_EXPIRED : 0u);
}

__device__ __forceinline__ void refresh_node(const NodeTimes& N, uint32_t i, int64_t now, uint8_t* status,
                                             const StatusMarks& M) {
    const uint32_t st = status_at(N, i, now), old = status[i];
    if (old != st) {
        status[i] = (uint8_t)st;
        mark_status_change(M, i, old, st);
    }
}

__global__ void status_from_times_kernel(NodeTimes N, uint32_t n, int64_t now, uint8_t* status, StatusMarks M) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i < n) refresh_node(N, i, now, status, M);
}

// ---------------------------------------------------------------------------------------
// isGood(now) deadlines. A node that is good at `now` stays good exactly while now <= D with
// D = min(time + 10 min, reply_time + 120 min) (node.cpp:34-40); a later `now` can only turn it bad, and
// only new times (patch_times) can turn a node good. So a refresh at a later `now` has to look at the
// nodes whose D it passes and at the patched ones, nothing else. The deadlines are kept as two sorted
// runs of (key = D as an order-preserving unsigned, node): the main run (every node, built on the device
// by a radix sort at the first refresh after set_times) and a side run (the deadlines of patched nodes,
// merged on the host at patch time). A cursor per run separates the deadlines already passed. A refresh
// finds how far `now` moves each cursor with one 64-ary wave search, re-derives the status of the nodes
// in between and of the patched ones, and publishes the next deadline (the smallest unpassed key) to the
// host, which skips the next refresh entirely while `now` stays at or below it.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t sat_add(int64_t a, int64_t b /* > 0 */) {
    return a > INT64_MAX - b ? INT64_MAX : a + b;
}
__host__ __device__ __forceinline__ uint64_t dl_key(int64_t d) { return (uint64_t)d ^ 0x8000000000000000ull; }
constexpr uint64_t DL_NEVER = ~0ull;  // expired nodes: never good, whatever `now`

__global__ void deadline_kernel(NodeTimes N, uint32_t n, uint64_t* __restrict__ key, uint32_t* __restrict__ node) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= n) return;
    key[i] = N.expired[i] ? DL_NEVER
                          : dl_key(min(sat_add(N.time_ns[i], NODE_EXPIRE_NS), sat_add(N.reply_ns[i], NODE_GOOD_NS)));
    node[i] = i;
}

// The nodes whose deadline `now` passed (main run [ma, ma + mc), side run [sa, sa + sc), both found by the host
// on its copy of the run keys) and the patched nodes: status re-derived from their times (the large-refresh path:
// flags, then the O(buckets) passes of rebuild_good_prefix). A node listed twice gets the same status twice.
__global__ void dl_process_kernel(NodeTimes N, const uint32_t* __restrict__ mnode, uint32_t mc,
                                  const uint32_t* __restrict__ snode, uint32_t sc, const uint32_t* __restrict__ pend,
                                  uint32_t np, uint32_t n, int64_t now, uint8_t* status, StatusMarks M) {
    const uint64_t total = (uint64_t)mc + sc + np;
    for (uint64_t j = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; j < total; j += (uint64_t)gridDim.x * BLOCK) {
        const uint32_t i = j < mc ? mnode[j] : j < (uint64_t)mc + sc ? snode[j - mc] : pend[j - mc - sc];
        if (i < n) refresh_node(N, i, now, status, M);
    }
}

__device__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds, uint32_t& total);

// ---------------------------------------------------------------------------------------
// Small refresh (at most RF_CAP nodes to re-derive: the steady state of a table whose `now` follows the
// clock, where a few deadlines pass between two query batches). No pass over the buckets or the lines:
//   rf_nodes_kernel  phase 1, every block: each listed node's status from its times (or a given value);
//                    a good-bit change appends the node's bucket, an expired-bit change the NodeCache slot
//                    range whose lines hold the node (wave-aggregated appends);
//                    phase 2, the last block to finish (a completion counter, no grid barrier): the buckets
//                    sorted and made unique in LDS, their masks and good counts recounted, and per line set
//                    the union of the windows that can read them ([b-2, b+3] / [b-3, b+4] / [b-7, b+8]) written
//                    as a sorted list, and the union of the NodeCache ranges
//   line builders    the listed lines only (LineSel over those lists), grids sized by the host's bound.
// The window good counts come from the per-bucket counts (gcnt), so nothing is O(buckets).
// ---------------------------------------------------------------------------------------
constexpr uint32_t RF_CAP = 2048;
constexpr uint32_t RF_NB = 0, RF_NR = 1, RF_DONE = 2, RF_L8 = 3, RF_L16 = 4, RF_L32 = 5, RF_LNC = 6, RF_GO = 7;
// fused launches (FUSE 1 / 2): RF_DONE the completion word (blocks done, blocks that listed deferred lines,
// blocks that gave up waiting for block 0's list: RF_DONE_*); RF_NDEF window lines left to the last block
// (windows of more than 64 nodes); word 9 unused;
// sticky diagnostics, never reset by the device (kad_table_refresh_diag): RF_SPIN spin waits that timed out,
// RF_DEFB lines the last block built, RF_ERR bounds guards that fired (RF_ERR_* bits; zero unless a bug)
constexpr uint32_t RF_NDEF = 8, RF_SPIN = 10, RF_DEFB = 11, RF_ERR = 12, RF_CTRS = 13;
constexpr uint32_t RF_ERR_INB = 1, RF_ERR_RUN = 2, RF_ERR_LINE = 4, RF_ERR_NHR = 8, RF_ERR_DEF = 16;
constexpr uint32_t RF_DONE_BLOCK = 1u, RF_DONE_DEF = 1u << 12, RF_DONE_REDO = 1u << 22;  // fields of 12 / 10 / 10 bits
// a builder's wait for block 0's list: 1 s of the 100 MHz wall clock, then the last block does its work
constexpr uint64_t RF_SPIN_TICKS = 100000000ull;

struct RfCtx {
    NodeTimes N;
    const uint32_t* mnode; uint32_t mc;  // main-run nodes whose deadline passed
    const uint32_t* snode; uint32_t sc;  // side-run nodes whose deadline passed
    const uint32_t* pend; uint32_t np;   // patched nodes
    const uint8_t* vals;                 // NULL: every status from the times at `now`; else pend[j] gets vals[j]
    int64_t now;
    DevTable T;                          // locate (key, tail, radix, firsts), B, n
    uint8_t* status;
    uint2* dir;
    uint32_t* gcnt;
    uint32_t* blist;                     // RF_CAP appended buckets
    uint32_t* nrange;                    // RF_CAP NodeCache slot ranges (first, last)
    uint32_t* ctr;                       // RF_CTRS words
    uint32_t* list[4];                   // lines of the count <= 8, 9..16, 17..32 sets and NodeCache slots (NULL: none)
    uint32_t nback, nfwd;                // NodeCache windows, as StatusMarks
    uint32_t* wl;                        // fused count <= 8 builds (rf_nodes_kernel FUSE): the line sets written
    uint32_t* ws;
    uint32_t* gl;
    uint32_t* fl;                        // FUSE: the line list block 0 publishes to the builder blocks
    uint32_t epoch;                      // FUSE: this refresh's value of ctr[RF_GO] (the list is published)
    uint32_t ninl;                       // > 0: the nodes are inl[0, ninl) (the host's copies of the runs, sorted), no lists
    uint32_t inl[128];
    // with inline nodes, derived on the host from its copy of the bucket offsets (0: derived on the device):
    uint32_t nhb;                        // the listed nodes' buckets, sorted and distinct
    uint32_t hb[128];
    uint32_t inb[128];                   // nhb: node inl[j]'s bucket hb[inb[j] & 127] and, when that bucket holds at
                                         // most 32 nodes (a directory mask), 1 + its place in it (inb[j] >> 8)
    uint32_t nhl;                        // FUSE 1: the window lines to rebuild, as nhr runs of consecutive lines:
    uint32_t nhr;                        //   run r = lines hr[3r] .. hr[3r] + hr[3r+1] - 1, whose windows' bucket
    uint32_t hr[3 * 16];                 //   offsets h_off[max(0, first - 3) ..] start at hoff[hr[3r+2]]
    uint32_t hoff[256];
    uint32_t fin;                        // FUSE 1: 1 = some line's window may exceed RF_WCAP1 nodes (the host could
                                         // not rule it out): the blocks run the completion protocol (rf_fused_finish)
#ifdef KAD_ABLATIONS
    uint32_t abl;  // tools build (KAD_RF_ABL): 1 = builder blocks skip their work, 2 = block 0 skips its work,
                   // 3 = block 0 starts RF_SPIN_TICKS + 0.2 s late (the builders' wait times out)
#endif
};
constexpr uint32_t RF_INLINE = 128, RF_HOFF = 256;
static_assert(sizeof(RfCtx) <= 4096, "rf_nodes_kernel's arguments must fit the 4 KB kernel-argument limit");

// One atomic per wave for the lanes with `want` (wave-uniform call); returns each wanting lane's slot.
__device__ __forceinline__ uint32_t wave_append(uint32_t* ctr, bool want) {
    const uint64_t m = __ballot(want);
    if (!m) return 0;
    const uint32_t lane = threadIdx.x & 63u, leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(ctr, (uint32_t)__builtin_popcountll(m));
    base = __shfl(base, (int)leader, 64);
    return base + __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

// The bucket holding node i: the locate of its own ID (findBucket), checked against the directory; a table
// whose node lies outside its bucket's range falls back to the search over the bucket starts.
__device__ uint32_t node_bucket(const DevTable& T, const uint2* dir, uint32_t i, uint64_t key_i) {
    Target t;
    t.hi = key_i;
    if (T.flags & TF_WL) {  // window-line tables: every node lies in its bucket's dyadic range (checked at creation)
        t.t2 = t.t3 = t.t4 = 0;
        return locate_bucket(T, t);
    }
    const uint32_t* tl = T.tail + 3ull * i;
    t.t2 = tl[0]; t.t3 = tl[1]; t.t4 = tl[2];
    const uint32_t b = locate_bucket(T, t);
    if ((dir[b].x & ~WIDE) <= i && i < (dir[b + 1].x & ~WIDE)) return b;
    uint32_t lo = 0, hi = T.B;  // the last bucket whose first node is <= i
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if ((dir[mid].x & ~WIDE) <= i) lo = mid + 1; else hi = mid;
    }
    return lo ? lo - 1 : 0u;
}

// Ascending bitonic sort of a[0, P) in LDS by the block (P a power of two, block-uniform).
__device__ void block_sort_u64(uint64_t* a, uint32_t P) {
    for (uint32_t k = 2; k <= P; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t x = threadIdx.x; x < P; x += BLOCK) {
                const uint32_t y = x ^ j;
                if (y > x) {
                    const uint64_t u = a[x], v = a[y];
                    if ((x & k) == 0 ? u > v : u < v) { a[x] = v; a[y] = u; }
                }
            }
            __syncthreads();
        }
}

// Union of the sorted intervals [lo(u), hi(u)] (u < m, ascending lo) written as one sorted list of indices;
// returns its length. iv(u) gives the interval; the ends need not ascend (a running maximum covers them).
template <class IV>
__device__ uint32_t block_union(uint32_t m, IV iv, uint32_t* out, uint32_t* lds4) {
    uint32_t written = 0;
    int64_t reach = -1;  // the largest end so far (block-uniform between chunks)
    __shared__ int64_t chunk_end;
    for (uint32_t c = 0; c < m; c += BLOCK) {  // block-uniform
        const uint32_t u = c + threadIdx.x;
        int64_t lo = 0, hi = -1;
        if (u < m) { uint32_t a, e; iv(u, a, e); lo = a; hi = e; }
        // the running maximum of the ends before u: an inclusive max-scan over the chunk, shifted by one
        int64_t x = hi;
        const uint32_t lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(x, o, 64);
            if (lane >= (uint32_t)o) x = max(x, y);
        }
        __shared__ int64_t wmax[BLOCK / 64];
        if (lane == 63) wmax[wid] = x;
        __syncthreads();
        int64_t before = reach;
        for (uint32_t w = 0; w < wid; w++) before = max(before, wmax[w]);
        const int64_t incl = max(before, x);
        int64_t prev = __shfl_up(incl, 1, 64);
        if (lane == 0) prev = before;
        const int64_t s0 = max(lo, prev + 1);
        const uint32_t cnt = (u < m && hi >= s0) ? (uint32_t)(hi - s0 + 1) : 0u;
        uint32_t tot;
        const uint32_t off = block_exclusive_scan(cnt, lds4, tot);
        for (uint32_t k = 0; k < cnt; k++) out[written + off + k] = (uint32_t)(s0 + k);
        written += tot;
        if (threadIdx.x == BLOCK - 1) chunk_end = incl;
        __syncthreads();
        reach = chunk_end;
        __syncthreads();
    }
    return written;
}

// ---------------------------------------------------------------------------------------
// Window line b and its short copy built by a whole wave (the small refresh's few lines: one lane building
// a line serially waits on hundreds of dependent LDS and memory accesses, ~20 us). Bit for bit the lines
// of wl_build_line + ws_build_line, for windows W(2) = [b-3, b+2] of at most 64 nodes: lane l holds node
// n0 + l (key and status staged by the caller in the wave's registers), the bucket good counts are ballots
// over the status bytes, each stored good node finds its slot from the D ranks of the buckets and its rank
// in its bucket, and the key collisions the serial build resolves in processing order (D rank, node,
// earlier node) are found lane against lane in LDS:
//   pairs >= 2 or a pair equal in all 64 bits -> defer; the first pair (in that order) whose keys differ
//   -> the tie word. The short line's 23-bit slot fields are OR-ed into LDS words.
// ---------------------------------------------------------------------------------------
// LDS written by some lanes of a wave and read by others of the same wave: one wave's LDS accesses complete in
// order, so only the compiler must not move accesses across this point (no hardware wait, in particular none on
// the wave's outstanding global stores, which a workgroup-scope fence would drain).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

struct WaveLds {
    uint32_t L[32];    // the 128-byte line
    uint32_t S16[16];  // the short line
    uint32_t dx[8];    // first nodes of the staged buckets
    uint32_t hlo[32];  // collision prefilter: lanes (0..31, 32..63) per 5-bit hash
    uint32_t hhi[32];
    uint32_t pk[64];   // per lane: stored bit 31 | D rank << 24 | key21 (read by the lanes it may collide with)
    uint64_t key[64];
    uint32_t R[33 + 17];  // rows of the serial fallback (a window of more than 64 nodes)
};

__device__ __attribute__((always_inline)) void wl_ws_build_wave(uint32_t b, uint32_t B, uint32_t d, uint64_t pre0,
                                                                  uint32_t db, const uint32_t* dx,
                                 uint32_t n0, uint32_t n1, uint64_t key, uint32_t stat, uint32_t* wl_out,
                                 uint32_t* ws_out, WaveLds& W) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t below = (1ull << lane) - 1ull;
    const uint32_t n = n0 + lane;
    const bool have = n < n1;
    const uint32_t e = min(B, b + 3);  // buckets [db, e) staged; dx[i] = first node of bucket db + i (i <= e - db)
    const uint32_t dxv = lane < 8 ? dx[lane] : 0u;  // dx in registers: uniform reads by readlane
    uint32_t x = NONE, xfirst = 0;
    for (uint32_t i = 0; db + i < e; i++) {  // wave-uniform
        const uint32_t di = rdl(dxv, i);
        if (have && di <= n) { x = db + i; xfirst = di; }
    }
    const bool good = have && (stat & KAD_STATUS_GOOD);
    // good nodes per staged bucket (as gcnt / the masks: the same status bytes)
    uint32_t cnt[7];
#pragma unroll
    for (uint32_t i = 0; i < 7; i++)
        cnt[i] = db + i < e ? (uint32_t)__builtin_popcountll(__ballot(good && x == db + i)) : 0u;
    auto cnt_of = [&](uint32_t y) {  // y in [db, e)
        uint32_t c = 0;
#pragma unroll
        for (uint32_t i = 0; i < 7; i++) c = (db + i == y) ? cnt[i] : c;
        return c;
    };
    for (uint32_t k = lane; k < 32; k += 64) W.L[k] = NONE;
    uint32_t h = 0, R8 = 3, g = 0;
    for (uint32_t r = 0; r < 3; r++) {
        const uint32_t lo = b > r ? b - 1 - r : 0u, hi = min(B - 1, b + r);
        g += r == 0 ? cnt_of(b) + (b ? cnt_of(b - 1) : 0u)
                    : (b > r ? cnt_of(b - 1 - r) : 0u) + ((uint64_t)b + r < (uint64_t)B ? cnt_of(b + r) : 0u);
        const bool whole = lo == 0 && hi == B - 1;
        h |= (min(g, 63u) << (6 * r)) | ((whole ? 1u : 0u) << (18 + r));
        if (R8 == 3 && (g >= 8 || whole)) R8 = r;
    }
    uint32_t S = 0, rounds = 0, tie = 0, base = NONE;
    bool defer = false;
    if (R8 == 3) {
        if (lane == 0) { W.L[1] = WL_DEFER; W.L[3] = 0; }
    } else {
        const uint32_t lo = b > R8 ? b - 1 - R8 : 0u, hi = min(B - 1, b + R8), nb = hi - lo + 1;  // nb <= 6
        base = rdl(dxv, lo - db);
        // lane y < nb holds window bucket lo + y: its D rank (the order of (pre0 + y) ^ (pre0 + b)), its good
        // count, and the stored prefix in D order (whole buckets while the cumulative count fits WL_SLOTS)
        const uint32_t yb = lo + min(lane, nb - 1);
        const uint64_t dy = (pre0 + yb) ^ (pre0 + b);
        uint32_t ry = 0;
        for (uint32_t z = 0; z < nb; z++) ry += ((pre0 + lo + z) ^ (pre0 + b)) < dy;
        const uint32_t cy = cnt_of(yb);
        uint32_t excl = 0;
        for (uint32_t z = 0; z < nb; z++) excl += rdl(ry, z) < ry ? rdl(cy, z) : 0u;
        const bool sty = lane < nb && excl + cy <= WL_SLOTS;
        const uint32_t rb = lane < nb ? (yb >= b ? yb - b : b - 1 - yb) << (2 * ry) : 0u, sS = sty ? excl + cy : 0u;
        for (uint32_t z = 0; z < nb; z++) {  // (wave-uniform reads of the nb bucket lanes)
            rounds |= rdl(rb, z);
            S = max(S, rdl(sS, z));
        }
        const uint32_t info_y = (sty ? 0x80000000u : 0u) | (ry << 24) | excl;
        // my slot: my bucket's rank and start, my rank among its stored nodes (its nodes are consecutive lanes)
        const bool inw = good && x >= lo && x <= hi;
        const uint32_t info = (uint32_t)__shfl((int)info_y, (int)(inw ? x - lo : 0u), 64);
        const bool mine = inw && (info >> 31);
        const uint32_t rj = (info >> 24) & 7u, st0 = info & 0xFFFFFFu;
        const uint32_t k21 = (uint32_t)((key << d) >> (64 - WL_KBITS)), off = n - base;
        const uint64_t mm = __ballot(mine);
        const uint32_t fl = inw ? xfirst - n0 : 0u;  // first lane of my bucket
        const uint32_t inb = (uint32_t)__builtin_popcountll(mm & below & ~((1ull << fl) - 1ull));
        defer = __any(mine && off > 255u);
        // pairs: earlier stored nodes of my bucket (lower lanes, same D rank) with my key21, in lane order. A 5-bit
        // hash of (rank, key21) in LDS names the earlier lanes that can be equal; usually none, and the exact
        // comparison runs over those only.
        const uint32_t mypk = mine ? (0x80000000u | (rj << 24) | k21) : 0u;
        if (lane < 32) { W.hlo[lane] = 0; W.hhi[lane] = 0; }
        W.pk[lane] = mypk;
        W.key[lane] = key;
        wave_lds_sync();
        const uint32_t hs = (mypk * 0x9E3779B1u) >> 27;
        if (mine) atomicOr(lane < 32 ? &W.hlo[hs] : &W.hhi[hs], 1u << (lane & 31u));
        wave_lds_sync();
        uint64_t same = 0;
        if (mine) same = (((uint64_t)W.hhi[hs] << 32) | W.hlo[hs]) & below;
        uint32_t pairs = 0, my_tie = 0;
        bool zero = false, have_tie = false;
        for (uint64_t m = same; m; m &= m - 1) {  // per lane, ascending
            const uint32_t l2 = (uint32_t)__builtin_ctzll(m);
            const uint32_t v = W.pk[l2];  // (LDS: the lane l2 need not be active here)
            const uint64_t k2 = W.key[l2];
            if (v == mypk) {
                pairs++;
                const uint64_t x64 = key ^ k2;
                if (x64 == 0) {
                    zero = true;
                } else if (!have_tie) {
                    const uint32_t p = (uint32_t)__builtin_clzll(x64), bn = (uint32_t)(key >> (63 - p)) & 1u;
                    my_tie = WL_DEFER | (bn << 30) | (p << 16) | (((n0 + l2 - base) & 255u) << 8) | (off & 255u);
                    have_tie = true;
                }
            }
        }
        // two pairs or more in the line, or a pair equal in all 64 bits: defer
        defer = defer || __any(zero) || __any(pairs >= 2) || __builtin_popcountll(__ballot(pairs >= 1)) >= 2;
        // the tie of the first pair in processing order (D rank, then node index)
        for (uint32_t r = 0; r < nb; r++) {  // wave-uniform
            const uint64_t tm = __ballot(have_tie && rj == r);
            if (tm) {
                tie = rdl(my_tie, (uint32_t)__builtin_ctzll(tm));
                break;
            }
        }
        if (mine) W.L[WL_SLOT0 + st0 + inb] = (rj << 29) | (k21 << 8) | (off & 255u);
        if (lane == 0) {
            W.L[0] = base;
            W.L[2] = rounds;
            W.L[3] = tie;
        }
    }
    if (lane == 0 && R8 != 3) W.L[1] = h | (R8 << 21) | (S << 23) | (defer ? WL_DEFER : 0u);
    wave_lds_sync();
    if (lane < 8) reinterpret_cast<uint4*>(wl_out + 32ull * b)[lane] =
        make_uint4(W.L[4 * lane], W.L[4 * lane + 1], W.L[4 * lane + 2], W.L[4 * lane + 3]);
    if (!ws_out) return;
    // the short line (ws_build_line over W.L)
    const uint32_t hh = W.L[1], rnd = W.L[2], SS = (hh >> 23) & 31u;
    bool fb = (hh & WL_DEFER) != 0;
    const uint32_t vs = lane < SS ? W.L[WL_SLOT0 + lane] : 0u;
    const uint32_t vnext = (uint32_t)__shfl_down((int)vs, 1, 64), vprev = (uint32_t)__shfl_up((int)vs, 1, 64);
    const bool endb = lane < SS && lane < WS_SLOTS && (lane + 1 == SS || (vnext >> 29) != (vs >> 29));
    const uint64_t em = __ballot(endb);
    const uint32_t keep = em ? 64u - (uint32_t)__builtin_clzll(em) : 0u;  // the last bucket end + 1
    constexpr uint32_t KSH = 8 + WL_KBITS - WS_KBITS;
    const bool ks = lane < keep;
    const uint32_t jj = vs >> 29, k16 = (vs >> KSH) & 0xFFFFu, offs = vs & 255u;
    bool f = ks && offs >= 64u;
    {  // an earlier kept slot of the same bucket with my key16 (the same hash prefilter; kept slots are lanes < 19)
        const uint32_t jk = (jj << 16) | k16, hk = (jk * 0x9E3779B1u) >> 27;
        if (lane < 32) W.hlo[lane] = 0;
        wave_lds_sync();
        if (ks) atomicOr(&W.hlo[hk], 1u << lane);
        wave_lds_sync();
        uint32_t same = ks ? W.hlo[hk] & (uint32_t)below : 0u;
        for (; same; same &= same - 1) {
            const uint32_t u = W.L[WL_SLOT0 + __builtin_ctz(same)];
            f |= (u >> 29) == jj && ((u >> KSH) & 0xFFFFu) == k16;
        }
    }
    fb = fb || __any(f);
    const bool start = ks && (lane == 0 || (vprev >> 29) != jj);
    const uint64_t sm = __ballot(start);
    uint32_t rk = 0, kb = 0;
    for (uint64_t m = sm; m; m &= m - 1, kb++)  // wave-uniform: the rounds of the kept buckets, in slot order
        rk |= ((rnd >> (2 * rdl(jj, (uint32_t)__builtin_ctzll(m)))) & 3u) << (2 * kb);
    if (lane < 16) W.S16[lane] = 0;
    wave_lds_sync();
    if (ks) {  // the slot's 23 bits at bit WS_SLOT0 + 23 * lane
        const uint32_t v = (start ? 1u << 22 : 0u) | (k16 << 6) | offs, p = WS_SLOT0 + WS_SBITS * lane;
        const uint64_t w = (uint64_t)v << (p & 31);
        atomicOr(&W.S16[p >> 5], (uint32_t)w);
        if ((p & 31) + WS_SBITS > 32) atomicOr(&W.S16[(p >> 5) + 1], (uint32_t)(w >> 32));
    }
    wave_lds_sync();
    if (lane < 16) {
        const uint32_t G0 = min(hh & 63u, 15u), G1 = min((hh >> 6) & 63u, 15u), G2 = min((hh >> 12) & 63u, 15u);
        const uint32_t hw = G0 | (G1 << 4) | (G2 << 8) | (((hh >> 18) & 7u) << 12) | (((hh >> 21) & 3u) << 15) |
                            (keep << 17) | ((fb ? 1u : 0u) << 22);
        // bits [0, 32) base, [32, 55) hw, [55, 67) rk, slots from 67, ones from the first unused slot on
        const uint64_t hdr = (uint64_t)hw | ((uint64_t)rk << 23);  // bits 32 .. 66
        uint32_t v = W.S16[lane];
        if (lane == 0) v = W.L[0];
        if (lane == 1) v |= (uint32_t)hdr;
        if (lane == 2) v |= (uint32_t)(hdr >> 32);
        const uint32_t u0 = WS_SLOT0 + WS_SBITS * keep, lo_bit = 32 * lane;  // ones from bit u0
        if (lo_bit + 32 <= u0) {
        } else if (lo_bit >= u0) {
            v = NONE;
        } else {
            v |= NONE << (u0 - lo_bit);
        }
        W.S16[lane] = v;
    }
    wave_lds_sync();
    if (lane < 4) reinterpret_cast<uint4*>(ws_out + 16ull * b)[lane] =
        make_uint4(W.S16[4 * lane], W.S16[4 * lane + 1], W.S16[4 * lane + 2], W.S16[4 * lane + 3]);
}

// The listed window lines (and their short copies) built by one wave each (wl_ws_build_wave): an incremental
// rebuild's lines are few and scattered, so a line's latency (not the throughput of a thread per line) sets the
// time. Windows of more than 64 nodes are built by the wave's first lane.
__global__ __launch_bounds__(BLOCK) void wl_ws_wave_kernel(const uint64_t* __restrict__ key, const uint8_t* status,
                                                            const uint2* dir, const uint32_t* gcnt, uint32_t B,
                                                            uint32_t d, uint64_t pre0, uint32_t* wl, uint32_t* ws,
                                                            LineSel sel) {
    __shared__ WaveLds wv[BLOCK / 64];
    WaveLds& WV = wv[threadIdx.x >> 6];
    const uint32_t lane = threadIdx.x & 63u;
    for (uint32_t x = (blockIdx.x * BLOCK + threadIdx.x) >> 6;; x += (gridDim.x * BLOCK) >> 6) {  // wave-uniform
        uint32_t b;
        if (!sel.pick(x, B, b)) return;
        const uint32_t db = b >= 3 ? b - 3 : 0u, e = min(B, b + 3);
        if (db + lane <= e && lane < 8) WV.dx[lane] = dir[db + lane].x & ~WIDE;
        wave_lds_sync();
        const uint32_t n0 = WV.dx[0], n1 = WV.dx[e - db];
        if (n1 - n0 <= 64) {
            const bool have = n0 + lane < n1;
            const uint64_t kk = have ? key[n0 + lane] : 0ull;
            const uint32_t sv = have ? status[n0 + lane] : 0u;
            wl_ws_build_wave(b, B, d, pre0, db, WV.dx, n0, n1, kk, sv, wl, ws, WV);
        } else if (lane == 0) {
            wl_build_line(key, status, dir, gcnt, B, d, pre0, wl, b, WV.R);
            if (ws) ws_build_line(WV.R, ws, b, WV.R + 33);
        }
        wave_lds_sync();
    }
}

// SINGLE: one block (at most BLOCK listed nodes): the appends go to LDS and there is no completion counter.
// FUSE (implies SINGLE): the count <= 8 lines of the changed buckets are rebuilt in the same launch (1: window
// lines and their short copies, a wave per line; 2: general lines, a 16-lane group per line; the host fuses
// when at most RF_FUSE_LINES can be listed), so a refresh that passes a few deadlines is one launch. Block 0
// derives the nodes and the list, publishes it (ctr[RF_GO] = epoch, release at agent scope) and builds its share;
// blocks 1.. wait for the epoch (dispatched after block 0, so it is always resident) and build the rest, all
// lines in one round.
constexpr uint32_t RF_FUSE_LINES = 6 * 128;
// FUSE 1: a window of 65 .. RF_WCAP1 nodes is staged by its builder wave in LDS (keys, statuses derived as block 0
// derives them, the window's good counts and masks) and built from there by one lane (wl_build_line on the staged
// views), without waiting for block 0; only a larger one is left to the launch's last block.
constexpr uint32_t RF_WCAP1 = 1024;
struct RfStage {
    uint64_t key[RF_WCAP1];
    uint2 dir[8];
    uint32_t gc[8];
    uint8_t st[RF_WCAP1];
};

// p - n as a generic (flat) pointer: p[n + i] is then p[i] for the callee, whatever the address space of p.
template <class T>
__device__ __forceinline__ const T* flat_shift(const T* p, uint32_t n) {
    return reinterpret_cast<const T*>(reinterpret_cast<uintptr_t>(static_cast<const void*>(p)) - (uintptr_t)n * sizeof(T));
}
constexpr uint32_t RF_POOL = BLOCK * (33 + 17);  // dwords: phase 2's sort buffers, then phase 3's line rows

// KAD_RF_TRACE (diagnostic builds only): thread 0 of the phase-2 block stamps the device wall clock at the phase
// boundaries and prints them (tools/rf_trace.py).
#ifdef KAD_RF_TRACE
#define RF_STAMP(k) do { if (threadIdx.x == 0) rf_ts[k] = wall_clock64(); } while (0)
#else
#define RF_STAMP(k) do { } while (0)
#endif

// Builder blocks of a fused window-line refresh (FUSE 1, blocks 1..): independent of block 0. The lines to build
// are the union of [b-2, b+3] over the listed nodes' buckets (phase 2's count <= 8 list): given by the host with
// the bucket offsets their windows read (C.nhl), derived here from the host's buckets (C.nhb: a merge across the
// wave, then the directory), or, for nodes in device lists, derived from the nodes (their buckets located and
// sorted across wave 0). Every wave builds lines of that list (wl_ws_build_wave) with the listed nodes' statuses
// derived here as phase 1 derives them, so no line waits for block 0's status writes. Only a window of more than
// 64 nodes (the serial builder, which reads the table's statuses and good counts) waits for block 0's epoch
// (published after its good counts). A listed node whose status did not change rebuilds lines that come out the same.
__device__ __attribute__((always_inline)) bool rf_wl_builders(const RfCtx& C, uint32_t* pool) {
    const DevTable& T = C.T;
    const uint32_t B = T.B, lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
    const uint32_t total = C.ninl ? C.ninl : C.mc + C.sc + C.np;  // inline <= RF_INLINE, lists <= 64
    static_assert(4 * sizeof(WaveLds) + 4 * sizeof(RfStage) <= 4 * RF_POOL, "builder wave buffers");
    __shared__ uint32_t s_node[64];
    __shared__ uint32_t s_st[64];
    __shared__ uint32_t s_lines[RF_FUSE_LINES];
    __shared__ uint32_t s_nl;
    // the kernel arguments the line loop searches (inline nodes, runs, offsets), staged in LDS in one round of
    // independent loads: a wave-uniform search of them in the argument segment was a chain of dependent scalar loads
    __shared__ uint32_t s_inl[RF_INLINE], s_hr[3 * 16], s_hoff[RF_HOFF];
    // (the host checks every inline limit before the launch, rf_check_inline; the guards here only record a
    // violation in the sticky error word and skip the access)
    const bool host_lines = C.nhl != 0 && C.nhr <= 16;
    {
        const uint32_t tid = threadIdx.x;
        if (tid == 0 && C.nhl != 0 && C.nhr > 16) atomicOr(C.ctr + RF_ERR, RF_ERR_NHR);
        if (tid < min(C.ninl, RF_INLINE)) s_inl[tid] = C.inl[tid];
        if (host_lines) {
            if (tid < 3 * C.nhr) s_hr[tid] = C.hr[tid];
            for (uint32_t o = tid; o < RF_HOFF; o += BLOCK) s_hoff[o] = C.hoff[o];
        }
        __syncthreads();
    }
    if (!host_lines) {  // block-uniform
        if (wid == 0 && C.nhb) {
            // the host's buckets (sorted, distinct, <= RF_INLINE): merge [b-2, b+3] in passes of 64
            uint32_t carry = 0, base = 0;
            for (uint32_t p0 = 0; p0 < C.nhb; p0 += 64) {  // wave-uniform
                const uint32_t idx = p0 + lane;
                const bool keep = idx < C.nhb;
                const uint32_t v = keep ? C.hb[idx] : 0u;
                const uint32_t a0 = keep ? (v > 2 ? v - 2 : 0u) : 0u, e1 = keep ? min(B - 1, v + 3) + 1 : 0u;
                uint32_t mx = e1;  // inclusive running max of the interval ends (+1)
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)mx, o, 64);
                    if (lane >= (uint32_t)o) mx = max(mx, y);
                }
                uint32_t before = (uint32_t)__shfl_up((int)mx, 1, 64);
                before = max(lane == 0 ? 0u : before, carry);
                const uint32_t s0 = max(a0, before), cnt = keep && e1 > s0 ? e1 - s0 : 0u;
                uint32_t off = cnt;
#pragma unroll
                for (int o = 1; o < 64; o <<= 1) {
                    const uint32_t y = (uint32_t)__shfl_up((int)off, o, 64);
                    if (lane >= (uint32_t)o) off += y;
                }
                const uint32_t tot = rdl(off, 63);
                off = base + off - cnt;
                for (uint32_t k = 0; k < cnt; k++)
                    if (off + k < RF_FUSE_LINES) s_lines[off + k] = s0 + k;
                carry = max(carry, rdl(mx, 63));
                base += tot;
            }
            if (lane == 0) s_nl = min(base, RF_FUSE_LINES);
        } else if (wid == 0) {
            // nodes from device lists (<= 64): locate, derive, sort the buckets across the wave, merge
            const bool act = lane < total;
            uint32_t i = NONE, st = 0, b = NONE;
            if (act)
                i = C.ninl ? C.inl[lane] : lane < C.mc ? C.mnode[lane] : lane < C.mc + C.sc ? C.snode[lane - C.mc]
                                                                                           : C.pend[lane - C.mc - C.sc];
            if (act && i < T.n) {
                const uint64_t key_i = T.key[i];
                st = (!C.ninl && C.vals && lane >= C.mc + C.sc)
                         ? (uint32_t)(C.vals[lane - C.mc - C.sc] & (KAD_STATUS_GOOD | KAD_STATUS_EXPIRED))
                         : status_at(C.N, i, C.now);
                b = node_bucket(T, C.dir, i, key_i);
            } else {
                i = NONE;
            }
            s_node[lane] = i;
            s_st[lane] = st;
            uint32_t v = b;  // bitonic across the wave, NONE last
#pragma unroll
            for (uint32_t k = 2; k <= 64; k <<= 1)
#pragma unroll
                for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                    const uint32_t u = (uint32_t)__shfl_xor((int)v, (int)j, 64);
                    v = (((lane & j) == 0) == ((lane & k) == 0)) ? min(v, u) : max(v, u);
                }
            const uint32_t pv = (uint32_t)__shfl_up((int)v, 1, 64);
            const bool keep = v != NONE && (lane == 0 || v != pv);
            const uint32_t a0 = keep ? (v > 2 ? v - 2 : 0u) : 0u, e1 = keep ? min(B - 1, v + 3) + 1 : 0u;
            uint32_t mx = e1;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)mx, o, 64);
                if (lane >= (uint32_t)o) mx = max(mx, y);
            }
            uint32_t before = (uint32_t)__shfl_up((int)mx, 1, 64);
            if (lane == 0) before = 0;
            const uint32_t s0 = max(a0, before), cnt = keep && e1 > s0 ? e1 - s0 : 0u;
            uint32_t off = cnt;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)off, o, 64);
                if (lane >= (uint32_t)o) off += y;
            }
            const uint32_t nl = rdl(off, 63);
            off -= cnt;
            for (uint32_t k = 0; k < cnt; k++)
                if (off + k < RF_FUSE_LINES) s_lines[off + k] = s0 + k;
            if (lane == 0) s_nl = min(nl, RF_FUSE_LINES);
        }
        __syncthreads();
    }
    const uint32_t nl = host_lines ? C.nhl : s_nl;
    WaveLds& WV = reinterpret_cast<WaveLds*>(pool)[wid];
    RfStage& SG = reinterpret_cast<RfStage*>(pool + (4 * sizeof(WaveLds) + 15) / 16 * 4)[wid];
    bool deferred = false;  // (lane 0 of a wave that listed a line for the last block)
    // node n's status as this refresh derives it (the listed nodes: from their times or given values)
    auto derived = [&](uint32_t n) -> uint32_t {
        if (C.ninl) {
            uint32_t lo = 0, hi = C.ninl;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (s_inl[mid] < n) lo = mid + 1; else hi = mid;
            }
            return lo < C.ninl && s_inl[lo] == n ? status_at(C.N, n, C.now) : (uint32_t)C.status[n];
        }
        uint32_t sv = C.status[n];
        for (uint32_t j = 0; j < total; j++)
            if (s_node[j] == n) sv = s_st[j];
        return sv;
    };
    for (uint32_t x = (blockIdx.x - 1) * (BLOCK / 64) + wid; x < nl; x += (gridDim.x - 1) * (BLOCK / 64)) {
        uint32_t b, n0, n1;  // (wave-uniform)
        if (host_lines) {  // the run of line x and its offsets (kernel arguments)
            uint32_t r = 0, k = x;
            while (r + 1 < C.nhr && k >= s_hr[3 * r + 1]) k -= s_hr[3 * r + 1], r++;
            const uint32_t first = s_hr[3 * r];
            b = first + k;
            const uint32_t db = b >= 3 ? b - 3 : 0u, e = min(B, b + 3);
            const uint32_t o0 = s_hr[3 * r + 2] + (db - (first >= 3 ? first - 3 : 0u));
            if (b >= B || db < (first >= 3 ? first - 3 : 0u) || o0 + (e - db) >= RF_HOFF) {  // (never: rf_check_inline)
                if (lane == 0) atomicOr(C.ctr + RF_ERR, b >= B ? RF_ERR_LINE : RF_ERR_RUN);
                continue;
            }
            const uint32_t* hl = s_hoff + o0;
            if (lane < 8) WV.dx[lane] = hl[min(lane, e - db)];
            n0 = hl[0];
            n1 = hl[e - db];
        } else {
            b = s_lines[x];
            const uint32_t db = b >= 3 ? b - 3 : 0u, e = min(B, b + 3);
            if (db + lane <= e && lane < 8) WV.dx[lane] = C.dir[db + lane].x & ~WIDE;
            wave_lds_sync();
            n0 = WV.dx[0];
            n1 = WV.dx[e - db];
        }
        const uint32_t db = b >= 3 ? b - 3 : 0u;
        if (n1 - n0 <= 64) {
            const uint32_t n = n0 + lane;
            const bool have = n < n1;
            uint32_t sv;
#ifdef KAD_RF_TRACE
            const uint64_t tb0 = wall_clock64();
#endif
            const uint64_t kk = have ? T.key[n] : 0ull;
            if (C.ninl) {  // inline nodes (sorted by the host): those in [n0, n1) take their derived status
                uint32_t lo = 0, hi = C.ninl;
                while (lo < hi) {  // wave-uniform lower_bound of n0
                    const uint32_t mid = (lo + hi) >> 1;
                    if (s_inl[mid] < n0) lo = mid + 1; else hi = mid;
                }
                bool listed = false;
                for (uint32_t j = lo; j < C.ninl && s_inl[j] < n1; j++) listed |= s_inl[j] == n;
                sv = !have ? 0u : listed ? status_at(C.N, n, C.now) : (uint32_t)C.status[n];
            } else {  // device lists: the statuses wave 0 derived
                sv = have ? C.status[n] : 0u;
                for (uint32_t j = 0; j < total; j++) {
                    const uint32_t nj = s_node[j];
                    if (nj != NONE && nj - n0 == lane) sv = s_st[j];
                }
            }
            wave_lds_sync();
#ifdef KAD_RF_TRACE
            __builtin_amdgcn_s_waitcnt(0);
            const uint64_t tb1 = wall_clock64();
#endif
            wl_ws_build_wave(b, B, 64 - T.rshift, T.rbase >> T.rshift, db, WV.dx, n0, n1, kk, sv, C.wl, C.ws, WV);
#ifdef KAD_RF_TRACE
            const uint64_t tb2 = wall_clock64();
            __builtin_amdgcn_s_waitcnt(0);
            const uint64_t tb3 = wall_clock64();
            if (lane == 0)
                printf("RFWAVE blk=%u wave=%u line=%u nodes=%u loads=%llu build=%llu drain=%llu at=%llu\n", blockIdx.x,
                       wid, b, n1 - n0, (unsigned long long)(tb1 - tb0), (unsigned long long)(tb2 - tb1),
                       (unsigned long long)(tb3 - tb2), (unsigned long long)tb0);
#endif
        } else if (n1 - n0 <= RF_WCAP1) {
            // 65 .. RF_WCAP1 nodes: W(2) staged with this refresh's statuses, its buckets' good counts and masks
            // recounted from them, then the serial build over the staged views (no wait for block 0)
            const uint32_t e = min(B, b + 3), nbk = e - db;
            if (lane <= nbk) {
                const uint32_t f = WV.dx[lane], sz = lane < nbk ? WV.dx[lane + 1] - f : 0u;
                SG.dir[lane] = make_uint2(f | (sz > 32 ? WIDE : 0u), 0u);
                SG.gc[lane] = 0;
            }
            wave_lds_sync();
            for (uint32_t o = lane; o < n1 - n0; o += 64) {
                const uint32_t n = n0 + o, sv = derived(n);
                SG.key[o] = T.key[n];
                SG.st[o] = (uint8_t)sv;
                if (sv & KAD_STATUS_GOOD) {
                    uint32_t x = 0;
                    for (uint32_t y = 1; y < nbk; y++) x = WV.dx[y] <= n ? y : x;
                    atomicAdd(&SG.gc[x], 1u);
                    if (WV.dx[x + 1] - WV.dx[x] <= 32) atomicOr(&SG.dir[x].y, 1u << (n - WV.dx[x]));
                }
            }
            wave_lds_sync();
            if (lane == 0) {
                wl_build_line(flat_shift(SG.key, n0), flat_shift(SG.st, n0), flat_shift(SG.dir, db),
                              flat_shift(SG.gc, db), B, 64 - T.rshift, T.rbase >> T.rshift, C.wl, b, WV.R);
                if (C.ws) ws_build_line(WV.R, C.ws, b, WV.R + 33);
            }
        } else if (lane == 0) {
            // more: the serial build reads the table's statuses and good counts, which block 0 writes; the line goes
            // to the last block to finish (rf_fused_finish, which runs when the host could not rule this out: C.fin)
            const uint32_t o = atomicAdd(C.ctr + RF_NDEF, 1u);
            if (o < RF_FUSE_LINES && C.fin) C.blist[o] = b;
            else atomicOr(C.ctr + RF_ERR, RF_ERR_DEF);  // (never)
            deferred = true;
        }
        wave_lds_sync();
    }
    return deferred;
}

template <int FUSE>
__device__ void rf_fused_lines(const RfCtx& C, uint32_t* pool, uint32_t n8, const uint32_t* l8, uint32_t bx,
                               uint32_t nbx);

// End of a fused launch (FUSE 1 / 2), every block: the last block to finish (a completion counter; no block
// waits for another) builds what no builder could without block 0's statuses and good counts: FUSE 1, the
// window lines of more than 64 nodes the builders listed; FUSE 2, the whole line list again if a builder block
// gave up waiting for it (RF_DONE_REDO: its wait timed out, so block 0 was not running; rebuilding a line gives the
// same line). Then it resets the counters for the next refresh. Only the blocks whose writes the last block may
// read release them (block 0: statuses, counts, masks; a builder that listed a deferred line: the list): an
// agent-scope release writes back the XCD's L2 (buffer_wbl2), and one per builder block cost 2-6 us per
// refresh. The last block acquires (an L2 invalidate, buffer_inv) only when it has something to build.
template <int FUSE>
__device__ void rf_fused_finish(const RfCtx& C, uint32_t* pool, bool deferred, bool redo) {
    // one atomic per block: the returned word (plus this block's part) tells the last block whether any block
    // listed deferred lines or gave up waiting, so the common case reads nothing more
    __shared__ uint32_t s_last, s_ndef, s_redo, s_n8, s_pub;
    if (threadIdx.x == 0) s_pub = 0;
    __syncthreads();
    if (deferred) s_pub = 1;
    __syncthreads();
    const bool publish = s_pub || (FUSE == 1 && blockIdx.x == 0);  // block 0: statuses, counts, masks (FUSE 2
                                                                       // released them before its list)
    if (publish) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // (block-uniform)
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t mine = RF_DONE_BLOCK + (s_pub ? RF_DONE_DEF : 0u) + (redo ? RF_DONE_REDO : 0u);
        const uint32_t v = atomicAdd(C.ctr + RF_DONE, mine) + mine;
        s_last = (v & (RF_DONE_DEF - 1)) == gridDim.x;
        s_ndef = (v / RF_DONE_DEF) & 1023u;
        s_redo = v / RF_DONE_REDO;
    }
    __syncthreads();
    if (!s_last) return;
    if ((FUSE == 1 && s_ndef) || (FUSE == 2 && s_redo)) {  // (block-uniform)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        if (threadIdx.x == 0) {
            s_ndef = __hip_atomic_load(C.ctr + RF_NDEF, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_n8 = __hip_atomic_load(C.ctr + RF_L8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        __syncthreads();
    } else {
        if (threadIdx.x == 0) s_ndef = s_redo = 0;
        __syncthreads();
    }
    const DevTable& T = C.T;
    if (FUSE == 1 && s_ndef) {
        const uint32_t nd = min(s_ndef, RF_FUSE_LINES), lane = threadIdx.x & 63u, wid = threadIdx.x >> 6;
        WaveLds& WV = reinterpret_cast<WaveLds*>(pool)[wid];
        for (uint32_t x = wid; x < nd; x += BLOCK / 64) {  // wave-uniform
            if (lane == 0) {
                const uint32_t b = C.blist[x];
                wl_build_line(T.key, C.status, C.dir, C.gcnt, T.B, 64 - T.rshift, T.rbase >> T.rshift, C.wl, b, WV.R);
                if (C.ws) ws_build_line(WV.R, C.ws, b, WV.R + 33);
            }
            wave_lds_sync();
        }
    }
    if (FUSE == 2 && s_redo) rf_fused_lines<FUSE>(C, pool, s_n8, C.fl, 0u, 1u);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_ndef) {
            atomicAdd(C.ctr + RF_DEFB, s_ndef);
            C.ctr[RF_NDEF] = 0;
        }
        if (s_redo) atomicAdd(C.ctr + RF_DEFB, s_n8);
        C.ctr[RF_DONE] = 0;
    }
}

// Phase 3 of a fused general-line refresh (FUSE 2): lines l8[x] for x = this block's share (block bx of nbx:
// blockIdx.x of gridDim.x, or 0 of 1 for the last block's rebuild), after block 0 published the list.
template <int FUSE>
__device__ void rf_fused_lines(const RfCtx& C, uint32_t* pool, uint32_t n8, const uint32_t* l8, uint32_t bx,
                               uint32_t nbx) {
    const DevTable& T = C.T;
    const uint32_t B = T.B;
    if (FUSE == 2) {
        // phase 3: the count <= 8 general lines of the list, RF_GROUP lanes per line (the pool's sort buffers are free now).
        // A line reads only W(2) = [b-3, b+2] (its bucket counts, directory entries up to b+3 and their nodes),
        // which the group stages in LDS in two rounds of parallel loads; its first lane then builds the line from
        // there (a window larger than RF_WCAP nodes is read from HBM). A line built straight from HBM waits
        // for ~10 dependent loads (one per bucket of its window, and the keys eight at a time).
        constexpr uint32_t RF_GROUP = 16, NG = BLOCK / RF_GROUP, RF_WCAP = 128;
        static_assert(NG * (2 * RF_WCAP + RF_WCAP / 4 + 16 + 8 + 33 + 17) <= RF_POOL, "phase 3 staging");
        uint64_t* skey = reinterpret_cast<uint64_t*>(pool);                        // NG x RF_WCAP keys
        uint8_t* sst = reinterpret_cast<uint8_t*>(pool + NG * 2 * RF_WCAP);        // NG x RF_WCAP status bytes
        uint2* sdir = reinterpret_cast<uint2*>(pool + NG * (2 * RF_WCAP + RF_WCAP / 4));  // NG x 8
        uint32_t* sgc = pool + NG * (2 * RF_WCAP + RF_WCAP / 4 + 16);               // NG x 8
        uint32_t* rows = sgc + NG * 8;                                              // NG x (33 + 17)
        const uint32_t g = threadIdx.x / RF_GROUP, gl = threadIdx.x % RF_GROUP;
        for (uint32_t x0 = bx * NG; x0 < n8; x0 += nbx * NG) {  // block-uniform
            const uint32_t x = x0 + g;
            const bool act = x < n8;
            const uint32_t b = act ? l8[x] : 0u, db = b >= 3 ? b - 3 : 0u;
            // round 1: the counts of [db, db + 6) and the directory entries [db, db + 7)
            if (act && gl < 6 && db + gl < B) sgc[8 * g + gl] = C.gcnt[db + gl];
            if (act && gl >= 6 && gl < 13 && db + gl - 6 <= B) sdir[8 * g + gl - 6] = C.dir[db + gl - 6];
            __syncthreads();
            // round 2: the keys and status bytes of the nodes of buckets [db, min(B - 1, b + 2)]
            const uint32_t e = min(B, b + 3);
            const uint32_t n0 = sdir[8 * g].x & ~WIDE, n1 = sdir[8 * g + (e - db)].x & ~WIDE;
            const bool staged = act && n1 - n0 <= RF_WCAP;
            if (staged) {
#pragma unroll
                for (uint32_t k = 0; k < RF_WCAP / RF_GROUP; k++) {
                    const uint32_t o = gl + RF_GROUP * k;
                    if (o < n1 - n0) {
                        skey[RF_WCAP * g + o] = T.key[n0 + o];
                        sst[RF_WCAP * g + o] = C.status[n0 + o];
                    }
                }
            }
            __syncthreads();
            if (act && gl == 0) {
                // the staged copies as views indexed like the arrays (every index the build uses lies in W(2)):
                // the shift is applied to the generic address (an LDS-space pointer shifted below its base would
                // wrap in 32 bits and leave the LDS aperture once converted)
                const uint64_t* kp = staged ? flat_shift(skey + RF_WCAP * g, n0) : T.key;
                const uint8_t* sp = staged ? flat_shift(sst + RF_WCAP * g, n0) : C.status;
                const uint2* dp = flat_shift(sdir + 8 * g, db);
                const uint32_t* gp = flat_shift(sgc + 8 * g, db);
                uint32_t* rowA = rows + 50 * g;
                gl8_build_line(kp, sp, dp, gp, T.fkey, T.ftail, B, C.gl, b, rowA);
            }
            __syncthreads();
        }
    }
}

template <bool SINGLE, int FUSE>
__global__ __launch_bounds__(BLOCK) void rf_nodes_kernel(RfCtx C_arg) {
    static_assert(!FUSE || SINGLE, "a fused refresh derives its nodes in block 0");
    // the argument read in place through the segment pointer (it is the only one): indexed per lane, the by-value
    // argument was copied to scratch whole (3.2 KB per lane)
#if __HIP_DEVICE_COMPILE__
    const RfCtx& C = *(const RfCtx*)__builtin_amdgcn_kernarg_segment_ptr();
    (void)C_arg;
#else
    const RfCtx& C = C_arg;
#endif
    const DevTable& T = C.T;
#ifdef KAD_RF_TRACE
    uint64_t rf_ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#endif
    RF_STAMP(0);
    __shared__ __attribute__((aligned(16))) uint32_t pool[RF_POOL];
    __shared__ uint32_t lctr[2];
#ifdef KAD_ABLATIONS
    const bool skip = (C.abl == 1 && blockIdx.x > 0) || (C.abl == 2 && blockIdx.x == 0);
    if (skip && !FUSE) return;
    if (C.abl == 3 && blockIdx.x == 0) {  // block 0 starts late: the builders' wait for its list times out
        const uint64_t t0 = wall_clock64();
        while (wall_clock64() - t0 < RF_SPIN_TICKS + 20000000ull) __builtin_amdgcn_s_sleep(127);
    }
#else
    constexpr bool skip = false;
#endif
    if (FUSE == 1 && blockIdx.x > 0) {  // a window-line builder block (independent of block 0)
        const bool deferred = !skip && rf_wl_builders(C, pool);
#ifdef KAD_RF_TRACE
        __syncthreads();
        RF_STAMP(2);
        if (threadIdx.x == 0)
            printf("RFBUILD blk=%u start=%llu go=%llu end=%llu\n", blockIdx.x, (unsigned long long)rf_ts[0],
                   (unsigned long long)rf_ts[0], (unsigned long long)rf_ts[2]);
#endif
        if (C.fin) rf_fused_finish<FUSE>(C, pool, deferred, false);
        return;
    }
    if (FUSE == 2 && blockIdx.x > 0) {  // a general-line builder block: wait for block 0's list (block-uniform)
        if (threadIdx.x == 0) {
            // bounded: a list that does not come within RF_SPIN_TICKS (block 0 not running) is left to the last
            // block to finish (RF_DONE_REDO), which runs after block 0 whatever the order the blocks ran in
            const uint64_t t0 = wall_clock64();
            bool go = !skip;
            while (go && __hip_atomic_load(C.ctr + RF_GO, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) != C.epoch) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - t0 > RF_SPIN_TICKS) {
                    go = false;
                    atomicAdd(C.ctr + RF_SPIN, 1u);
                }
            }
            lctr[0] = go ? __hip_atomic_load(C.ctr + RF_L8, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
            lctr[1] = go || skip ? 0u : 1u;  // redo: the last block builds the list
        }
        __syncthreads();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        RF_STAMP(1);
        rf_fused_lines<FUSE>(C, pool, lctr[0], C.fl, blockIdx.x, gridDim.x);
#ifdef KAD_RF_TRACE
        __syncthreads();
        RF_STAMP(2);
        if (threadIdx.x == 0)
            printf("RFBUILD blk=%u start=%llu go=%llu end=%llu\n", blockIdx.x, (unsigned long long)rf_ts[0],
                   (unsigned long long)rf_ts[1], (unsigned long long)rf_ts[2]);
#endif
        rf_fused_finish<FUSE>(C, pool, false, lctr[1] != 0);
        return;
    }
    if (FUSE && skip) {  // (tools build) block 0 skips its work
        if (FUSE == 2 || C.fin) rf_fused_finish<FUSE>(C, pool, false, false);
        return;
    }
    uint64_t* srt = reinterpret_cast<uint64_t*>(pool);  // RF_CAP (phase 2)
    uint32_t* ub = pool + 2 * RF_CAP;                     // RF_CAP (phase 2)
    uint32_t* lb_ = SINGLE ? pool + 3 * RF_CAP : nullptr; // BLOCK appended buckets (phase 1, single block)
    uint32_t* lr_ = SINGLE ? pool + 3 * RF_CAP + BLOCK : nullptr;  // 2 x BLOCK NodeCache ranges
    static_assert(3 * RF_CAP + 3 * BLOCK <= RF_POOL, "pool");
    if (SINGLE && threadIdx.x < 2) lctr[threadIdx.x] = 0;
    if (SINGLE) __syncthreads();
    const uint32_t total = C.ninl ? C.ninl : C.mc + C.sc + C.np;
    for (uint32_t base = blockIdx.x * BLOCK; base < total; base += gridDim.x * BLOCK) {  // block-uniform
        const uint32_t j = base + threadIdx.x;
        bool act = j < total;
        uint32_t i = 0, st = 0, old = 0;
        if (act) {
            i = C.ninl ? C.inl[j] : j < C.mc ? C.mnode[j] : j < C.mc + C.sc ? C.snode[j - C.mc] : C.pend[j - C.mc - C.sc];
            act = i < T.n;
        }
        uint64_t key_i = 0;
        if (act) {
            if (T.B && !C.nhb) key_i = T.key[i];  // issued with the times: the locate needs it only if the good bit flips
            st = (!C.ninl && C.vals && j >= C.mc + C.sc)
                     ? (uint32_t)(C.vals[j - C.mc - C.sc] & (KAD_STATUS_GOOD | KAD_STATUS_EXPIRED))
                     : status_at(C.N, i, C.now);
            old = C.status[i];
            if (st != old) C.status[i] = (uint8_t)st;
        }
        const bool gchg = act && T.B && !C.nhb && ((st ^ old) & KAD_STATUS_GOOD);  // (nhb: the host's buckets)
        if (act && T.B && C.nhb && ((st ^ old) & KAD_STATUS_GOOD)) {
            // the host's buckets: the flip patches its bucket's good count and mask in place (no recount: the
            // nodes are distinct, the atomics return nothing, block 0's release below orders them before RF_GO)
            const uint32_t e = C.inb[j];
            if ((e & 127u) < min(C.nhb, RF_INLINE) && C.hb[e & 127u] < T.B && (e >> 8) <= 32) {  // (rf_check_inline)
                const uint32_t hbk = C.hb[e & 127u];
                atomicAdd(C.gcnt + hbk, (st & KAD_STATUS_GOOD) ? 1u : ~0u);
                if (e >> 8) atomicXor(reinterpret_cast<uint32_t*>(C.dir + hbk) + 1, 1u << ((e >> 8) - 1));
            } else {
                atomicOr(C.ctr + RF_ERR, RF_ERR_INB);
            }
        }
        const uint32_t b = gchg ? node_bucket(T, C.dir, i, key_i) : 0u;
        const bool echg = act && C.list[3] && ((st ^ old) & KAD_STATUS_EXPIRED);
        uint32_t sa = 0, se = 0;
        if (echg) {  // every NodeCache slot from that of node i - nback to that of node i + nfwd (as mark_status_change)
            const uint32_t a = i >= C.nback ? i - C.nback : 0u, e = min(T.n - 1, i + C.nfwd);
            const uint64_t ka = T.key[a], ke = T.key[e];
            sa = ka < T.nbase ? 0u : (uint32_t)min<uint64_t>((ka - T.nbase) >> T.nshift, T.nslots - 1);
            se = ke < T.nbase ? 0u : (uint32_t)min<uint64_t>((ke - T.nbase) >> T.nshift, T.nslots - 1);
        }
        if (SINGLE) {  // LDS appends (total <= BLOCK)
            if (gchg) lb_[atomicAdd(&lctr[0], 1u)] = b;
            if (echg) { const uint32_t o = atomicAdd(&lctr[1], 1u); lr_[2 * o] = sa; lr_[2 * o + 1] = se; }
        } else {
            const uint32_t ob = wave_append(C.ctr + RF_NB, gchg);
            if (gchg && ob < RF_CAP) C.blist[ob] = b;
            const uint32_t orr = wave_append(C.ctr + RF_NR, echg);
            if (echg && orr < RF_CAP) { C.nrange[2 * orr] = sa; C.nrange[2 * orr + 1] = se; }
        }
    }
    uint32_t nb, nr;
    const uint32_t* blist;
    const uint32_t* nrange;
    if (SINGLE) {
        __syncthreads();
        nb = lctr[0];
        nr = lctr[1];
        blist = lb_;
        nrange = lr_;
    } else {
        // the last block to finish takes phase 2 (every other block's appends are visible after the acquire)
        __shared__ uint32_t last;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (threadIdx.x == 0) last = atomicAdd(C.ctr + RF_DONE, 1u) == gridDim.x - 1;
        __syncthreads();
        if (!last) return;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        nb = min(__hip_atomic_load(C.ctr + RF_NB, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), RF_CAP);
        nr = min(__hip_atomic_load(C.ctr + RF_NR, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT), RF_CAP);
        blist = C.blist;
        nrange = C.nrange;
    }
    RF_STAMP(1);
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t l8[FUSE ? RF_FUSE_LINES : 1];
    __shared__ uint32_t n8_s;
    // NodeCache ranges first (sorted in the same buffer as the buckets next)
    uint32_t nrs = 0;
    uint64_t* rsrt = srt;
    if (C.list[3]) {  // block-uniform
        uint32_t P = 1;
        while (P < nr) P <<= 1;
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < P; x += BLOCK)  // (single mode: the appends lie above the sort buffer)
            rsrt[x] = x < nr ? ((uint64_t)nrange[2 * x] << 32) | nrange[2 * x + 1] : ~0ull;
        __syncthreads();
        block_sort_u64(rsrt, P);
        const uint32_t n = block_union(nr, [&](uint32_t u, uint32_t& a, uint32_t& e) {
            a = (uint32_t)(rsrt[u] >> 32);
            e = (uint32_t)rsrt[u];
        }, C.list[3], lds4);
        if (threadIdx.x == 0) C.ctr[RF_LNC] = n;
        nrs = n;
    }
    (void)nrs;
    RF_STAMP(2);
    // buckets: sort, unique (or the host's list: every listed node's bucket, changed or not; a recount of an
    // unchanged bucket and a rebuild of its lines give the same values)
    uint32_t nu = 0;
    if (C.nhb) {  // block-uniform
        __syncthreads();
        nu = min(C.nhb, RF_INLINE);
        if (threadIdx.x < nu) ub[threadIdx.x] = C.hb[threadIdx.x];
        __syncthreads();
    } else {
        uint32_t P = 1;
        while (P < nb) P <<= 1;
        __syncthreads();
        for (uint32_t x = threadIdx.x; x < P; x += BLOCK) srt[x] = x < nb ? (uint64_t)blist[x] : ~0ull;
        __syncthreads();
        block_sort_u64(srt, P);
        for (uint32_t c = 0; c < nb; c += BLOCK) {
            const uint32_t x = c + threadIdx.x;
            const bool keep = x < nb && (x == 0 || srt[x] != srt[x - 1]);
            uint32_t tot;
            const uint32_t off = block_exclusive_scan(keep ? 1u : 0u, lds4, tot);
            if (keep) ub[nu + off] = (uint32_t)srt[x];
            nu += tot;
        }
        __syncthreads();
    }
    RF_STAMP(3);
    // their masks and good counts (bucket_good_kernel for these buckets; the host's buckets were patched in phase 1)
    for (uint32_t u = threadIdx.x; u < (C.nhb ? 0u : nu); u += BLOCK) {
        const uint32_t b = ub[u];
        const uint32_t j0 = C.dir[b].x & ~WIDE, j1 = C.dir[b + 1].x & ~WIDE;
        uint32_t g = 0, mask = 0;
        for (uint32_t jj = j0; jj < j1; jj++) {
            const uint32_t gb = C.status[jj] & KAD_STATUS_GOOD;
            g += gb;
            if (jj - j0 < 32) mask |= gb << (jj - j0);
        }
        C.gcnt[b] = g;
        C.dir[b].y = (j1 - j0 <= 32) ? mask : 0u;
    }
    RF_STAMP(4);
    // per line set: the union of the windows that can read a changed bucket (the count <= 8 set into LDS when fused)
    const uint32_t B = T.B;
    const uint32_t below[3] = {2, 3, 7}, above[3] = {3, 4, 8};
    for (int k = 0; k < 3; k++) {
        if (!C.list[k] && !(FUSE == 2 && k == 0)) continue;  // block-uniform (FUSE 1: the builders list their own)
        const uint32_t lb = below[k], la = above[k];
        const uint32_t n = block_union(nu, [&](uint32_t u, uint32_t& a, uint32_t& e) {
            const uint32_t b = ub[u];
            a = b > lb ? b - lb : 0u;
            e = min(B - 1, b + la);
        }, (FUSE == 2 && k == 0) ? l8 : C.list[k], lds4);
        if (threadIdx.x == 0) {
            if (FUSE == 2 && k == 0) n8_s = n; else C.ctr[RF_L8 + k] = n;
        }
    }
    if (!SINGLE && threadIdx.x == 0) {  // the next refresh starts from empty appends
        C.ctr[RF_NB] = 0;
        C.ctr[RF_NR] = 0;
        C.ctr[RF_DONE] = 0;
    }
    RF_STAMP(5);
    if (FUSE == 2) {
        // publish the list to the builder blocks, then build this block's share
        __syncthreads();
        const uint32_t n8 = n8_s;
        for (uint32_t x = threadIdx.x; x < n8; x += BLOCK) C.fl[x] = l8[x];
        if (threadIdx.x == 0) C.ctr[RF_L8] = n8;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __syncthreads();
        if (threadIdx.x == 0 && gridDim.x > 1)
            __hip_atomic_store(C.ctr + RF_GO, C.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        RF_STAMP(6);
        rf_fused_lines<FUSE>(C, pool, n8, l8, blockIdx.x, gridDim.x);
    }
#ifdef KAD_RF_TRACE
    __syncthreads();
    RF_STAMP(7);
    if (threadIdx.x == 0)
        printf("RFTRACE single=%d fuse=%d total=%u nb=%u nu=%u n8=%u grid=%u ts=%llu %llu %llu %llu %llu %llu %llu %llu\n",
               (int)SINGLE, FUSE, total, nb, nu, FUSE == 2 ? n8_s : 0u, gridDim.x, (unsigned long long)rf_ts[0],
               (unsigned long long)(rf_ts[1] - rf_ts[0]), (unsigned long long)(rf_ts[2] - rf_ts[0]),
               (unsigned long long)(rf_ts[3] - rf_ts[0]), (unsigned long long)(rf_ts[4] - rf_ts[0]),
               (unsigned long long)(rf_ts[5] - rf_ts[0]), (unsigned long long)(rf_ts[6] - rf_ts[0]),
               (unsigned long long)(rf_ts[7] - rf_ts[0]));
#endif
    // block 0's statuses, counts and masks, for the last block: FUSE 2 released them before publishing the list
    if (FUSE == 2 || (FUSE == 1 && C.fin)) rf_fused_finish<FUSE>(C, pool, false, false);
}

// New status bytes: all n nodes (nodes == NULL) or the m listed ones; only changes are written and marked.
__global__ void status_patch_kernel(const uint32_t* nodes, const uint8_t* vals, uint32_t m, uint8_t* status,
                                    StatusMarks M) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= m) return;
    const uint32_t i = nodes ? nodes[j] : j;
    if (i >= M.n) return;
    const uint32_t st = vals[j] & (KAD_STATUS_GOOD | KAD_STATUS_EXPIRED), old = status[i];
    if (old != st) {
        status[i] = (uint8_t)st;
        mark_status_change(M, i, old, st);
    }
}

// Node times of the m listed nodes (Node::received / setExpired on the host side).
__global__ void times_patch_kernel(const uint32_t* nodes, const int64_t* t, const int64_t* rt, const uint8_t* ex,
                                   uint32_t m, uint32_t n, int64_t* time_ns, int64_t* reply_ns, uint8_t* expired) {
    const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
    if (j >= m || nodes[j] >= n) return;
    time_ns[nodes[j]] = t[j];
    reply_ns[nodes[j]] = rt[j];
    expired[nodes[j]] = ex[j];
}

// Incremental form of bucket_good_kernel: only flagged buckets get a new mask and count (cnt keeps every
// other bucket's count from the last rebuild); each flags the lines whose window can reach it and is
// cleared. A line of bucket c reads buckets [c-3, c+2] (count <= 8: W(r <= 2)), [c-4, c+3] (9..16:
// W(r <= 3)) or [c-8, c+7] (17..32: W(r <= 7)), so bucket b dirties lines [b-2, b+3], [b-3, b+4], [b-7, b+8].
__global__ void bucket_good_dirty_kernel(const uint8_t* status, uint2* dir, uint32_t B, uint32_t* cnt,
                                         uint8_t* bdirty, uint8_t* ld8, uint8_t* ld16, uint8_t* ld32,
                                         const uint32_t* any) {
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    if (!*any || b >= B || !bdirty[b]) return;
    bdirty[b] = 0;
    const uint32_t j0 = dir[b].x & ~WIDE, j1 = dir[b + 1].x & ~WIDE;
    uint32_t g = 0, mask = 0;
    for (uint32_t j = j0; j < j1; j++) {
        const uint32_t gb = status[j] & KAD_STATUS_GOOD;
        g += gb;
        if (j - j0 < 32) mask |= gb << (j - j0);
    }
    cnt[b] = g;
    dir[b].y = (j1 - j0 <= 32) ? mask : 0u;
    auto flag = [&](uint8_t* f, uint32_t below, uint32_t above) {
        if (!f) return;
        const uint32_t c0 = b >= below ? b - below : 0u, c1 = min(B - 1, b + above);
        for (uint32_t c = c0; c <= c1; c++) f[c] = 1;
    };
    flag(ld8, 2, 3);
    flag(ld16, 3, 4);
    flag(ld32, 7, 8);
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

// *acc += sum of a[0, m) (grid-stride; *acc zeroed by the caller).
__global__ __launch_bounds__(BLOCK) void sum_u32_kernel(const uint32_t* a, uint32_t m, uint32_t* acc) {
    uint32_t s = 0;
    for (uint32_t j = blockIdx.x * BLOCK + threadIdx.x; j < m; j += gridDim.x * BLOCK) s += a[j];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63u) == 0 && s) atomicAdd(acc, s);
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

// Flags -> a compact list of their indices, flags cleared. Each thread takes 16 flags (one 16-byte load;
// flag arrays are padded to 16 bytes), the block scans the counts in LDS and claims its range with ONE
// atomic (a single counter hit by every wave saturates at ~90 adds per microsecond).
// any: NULL, or a word that is 0 when no flag can be set (the kernel exits at once).
__global__ __launch_bounds__(BLOCK) void compact_flags_kernel(uint8_t* flags, uint32_t m, uint32_t* list, uint32_t* ctr,
                                                              const uint32_t* any) {
    __shared__ uint32_t lds[4];
    __shared__ uint32_t base_s;
    if (any && !*any) return;  // grid-uniform
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x, i0 = 16 * g;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (i0 < m) v = reinterpret_cast<const uint4*>(flags)[g];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t c = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) c += __popc(w[k] & 0x01010101u);  // flags are 0 or 1
    uint32_t total;
    const uint32_t ex = block_exclusive_scan(c, lds, total);
    if (total == 0) return;  // block-uniform
    if (threadIdx.x == 0) base_s = atomicAdd(ctr, total);
    __syncthreads();
    if (!c) return;
    uint32_t o = base_s + ex;
#pragma unroll
    for (int k = 0; k < 16; k++)
        if ((w[k >> 2] >> (8 * (k & 3))) & 1u) list[o++] = i0 + k;
    reinterpret_cast<uint4*>(flags)[g] = make_uint4(0, 0, 0, 0);
}

// Tile-local exclusive scan of cnt[0..m) written to out; tile sums to sums[tile].
// any (scan kernels): NULL, or a word that is 0 when the counts did not change (the kernel exits at once).
__global__ __launch_bounds__(BLOCK) void scan_tiles_kernel(const uint32_t* cnt, uint32_t m, uint32_t* out, uint32_t* sums,
                                                           const uint32_t* any) {
    __shared__ uint32_t lds[4];
    if (any && !*any) return;
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
__global__ __launch_bounds__(BLOCK) void scan_sums_kernel(uint32_t* sums, uint32_t m, const uint32_t* any) {
    __shared__ uint32_t lds[4];
    if (any && !*any) return;
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

__global__ void scan_apply_kernel(const uint32_t* part, const uint32_t* sums, uint32_t m, uint32_t* gpre,
                                  const uint32_t* any) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if ((any && !*any) || i >= m) return;
    gpre[i] = part[i] + sums[i / SCAN_TILE];
}

inline uint32_t grid_for(uint64_t n) { return (uint32_t)((n + BLOCK - 1) / BLOCK); }
inline uint32_t grid64(uint64_t n) { return (uint32_t)((n + 63) / 64); }  // one-wave workgroups


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
// One pass over the items (their slot by a shift) and one over the slots: O(items + slots), 64-bit arithmetic.
std::vector<uint32_t> build_radix(const Radix& r, uint32_t m, const uint8_t* items, bool exact_flag) {
    std::vector<uint32_t> rdx(r.slots + 1, 0);
    // rdx[s + 1] counts the items of slot s, rdx[0] the items below the base; items past the last slot count
    // in no slot (rdx[slots] = #items below the end of the last slot)
    uint32_t below = 0;
    for (uint32_t j = 0; j < m; j++) {
        const uint64_t hi = id_hi(items + 20ull * j);
        if (hi < r.base) { below++; continue; }
        const uint64_t sl = (hi - r.base) >> r.shift;
        if (sl < r.slots) rdx[sl + 1]++;
    }
    rdx[0] = below;
    for (uint32_t sl = 0; sl < r.slots; sl++) rdx[sl + 1] += rdx[sl];
    if (exact_flag)
        for (uint32_t sl = 0; sl < r.slots; sl++) {
            const uint32_t j = rdx[sl];
            if (j >= m) continue;
            const uint8_t* it = items + 20ull * j;
            const uint64_t start = r.base + ((uint64_t)sl << r.shift);  // sl < slots: inside 64 bits
            if (id_hi(it) == start && id_low_zero(it)) rdx[sl] |= RDX_EXACT;
        }
    return rdx;
}

// ---------------------------------------------------------------------------------------
// Resident query service (kad_table_serve): single Dht requests without a kernel launch. One workgroup of
// BLOCK threads stays on the GPU and polls a mailbox in pinned host memory. The request header and the first
// target share one 64-byte line, which wave 0 reads with one 16-lane load per poll; the host writes the
// targets, then `seq2`, then `seq`, and a header read with seq == seq2 is whole. The workgroup then runs the
// same kernel body the launch path would run for the table's line sets (the bodies index queries from
// blockIdx.x = 0, so a request of up to SVC_Q <= BLOCK queries is one block of them), with the targets in LDS
// and the rows and counts written straight into the pinned reply; counts above 32 and NodeCache queries
// without lines take the wave paths. Every wave fences its rows to system scope before thread 0 publishes
// the request number. A launch ends on its own: when the host sets `stop`, after `idle` ticks without a
// request, or after `life` ticks in all (the host launches it again on the next request), so no wave
// outlives its process.
// ---------------------------------------------------------------------------------------
constexpr uint32_t SVC_Q = 64, SVC_COUNT = 64;
constexpr uint64_t KAD_SERVE_LIFE_MS = 50;  // one launch's longest life (bounds head-of-line blocking)
static_assert(SVC_Q <= BLOCK, "a request is one block of queries");

struct SvcMail {             // host writes, the service reads (system-scope loads)
    uint32_t seq;            // dw0: request number, written last
    uint32_t stop;           // dw1: nonzero: leave
    uint32_t q, count, kind; // dw2-4: kind 0: RoutingTable::findClosestNodes, 1: NodeCache::getCachedNodes
    uint32_t pad[2];
    uint32_t seq2;           // dw7: the request number, written before seq (a torn header read shows seq != seq2)
    uint32_t targets[SVC_Q * 5];  // from dw8: target 0 shares the header's 64-byte line
};
struct SvcReply {            // the service writes, the host reads
    uint32_t done;           // the last request answered: written after the rows and counts
    uint32_t polls;          // header reads before the last request was seen
    uint64_t t_seen, t_done; // device wall clock: the last request seen, its rows fenced (tools/latency)
    uint32_t pad[10];
    uint8_t cnt[SVC_Q];
    uint32_t idx[SVC_Q * SVC_COUNT];
};

__global__ __launch_bounds__(BLOCK) void svc_kernel(DevTable T, const SvcMail* __restrict__ mail,
                                                     SvcReply* __restrict__ reply, uint32_t last, uint64_t idle,
                                                     uint64_t life) {
    __shared__ uint32_t req[4];  // go, q, count, kind
    __shared__ uint32_t tg[SVC_Q * 5];
    __shared__ uint64_t xs[BLOCK / 64][192];
    const uint32_t tid = threadIdx.x, lane = tid & 63u, w = tid >> 6;
    const uint32_t* mw = reinterpret_cast<const uint32_t*>(mail);
    const uint64_t t0 = wall_clock64();
    uint64_t heard = t0;
    for (;;) {
        if (w == 0) {  // wave 0 polls the header line (wave-uniform loop)
            uint32_t v = 0, s = last, go = 0, polls = 0;
            for (;;) {
                polls++;
                v = lane < 16 ? __hip_atomic_load(mw + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
                s = rdl(v, 0);
                const uint32_t stop = rdl(v, 1), s2 = rdl(v, 7);
                if (s != last && s == s2) { go = 1; break; }
                const uint64_t now = wall_clock64();
                if (stop || now - heard > idle || now - t0 > life) break;
                __builtin_amdgcn_s_sleep(1);
            }
            if (go) {
                // seq == seq2 shows the header words were read together, not that the rest of the line was: after an
                // acquire at system scope (synchronising with the host's release of seq) the line is read again, and
                // holds the request the host wrote before seq (it writes no other until this one is answered)
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
                v = lane < 16 ? __hip_atomic_load(mw + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : 0u;
            }
            if (lane == 0) {
                if (go) {  // the statistics of a request (an idle or stop exit leaves them alone)
                    reply->polls = polls;
                    reply->t_seen = wall_clock64();
                }
                req[0] = go;
                req[1] = min(rdl(v, 2), SVC_Q);
                req[2] = min(rdl(v, 3), SVC_COUNT);
                req[3] = rdl(v, 4);
            }
            if (lane >= 8 && lane < 16) tg[lane - 8] = v;  // target 0 and the start of target 1
            last = s;
            heard = wall_clock64();
        }
        __syncthreads();
        if (req[0] == 0) return;  // block-uniform: stop or timeout with nothing posted
        // the other targets: system-scope loads issued after the header was seen (the host wrote them before seq)
        const uint32_t q = req[1], count = req[2], kind = req[3];
        for (uint32_t j = 8 + tid; j < 5 * q; j += BLOCK)  // the other targets (targets start at dw8)
            tg[j] = __hip_atomic_load(&mail->targets[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __syncthreads();
        const uint8_t* tq = reinterpret_cast<const uint8_t*>(tg);
        uint32_t* idx = reply->idx;
        uint8_t* cnt = reply->cnt;
        // the launch path's kernel choice (launch_rt) for the line sets this table has: block-uniform branches
        if (kind == 0 && count >= 1 && count <= 8) {
            if (T.flags & TF_WS) rt_ws_kernel_body<0>(T, tq, q, count, idx, cnt);
            else if (T.flags & TF_WL) rt_wl_kernel_body<0>(T, tq, q, count, idx, cnt);
            else if (T.flags & TF_SL) rt_sl_kernel_body<0>(T, tq, q, count, idx, cnt);
            else if (T.flags & TF_GL) rt_gl_kernel_body(T, tq, q, count, idx, cnt);
            else rt_closest_kernel_body<8>(T, tq, q, count, idx, cnt);
        } else if (kind == 0 && count >= 9 && count <= 16) {
            if (T.flags & TF_WL16) rt_wl16_kernel_body<0>(T, tq, q, count, idx, cnt);
            else if (T.flags & TF_SL16) rt_sl16_kernel_body(T, tq, q, count, idx, cnt);
            else if (T.flags & TF_GL16) rt_gl16_kernel_body(T, tq, q, count, idx, cnt);
            else if (T.flags & TF_GL32) rt_gl32_kernel_body(T, tq, q, count, idx, cnt);
            else rt_closest_kernel_body<16>(T, tq, q, count, idx, cnt);
        } else if (kind == 0 && count >= 17 && count <= 32) {
            if (T.flags & TF_WL32) rt_wl32_kernel_body(T, tq, q, count, idx, cnt);
            else if (T.flags & TF_GL32) rt_gl32_kernel_body(T, tq, q, count, idx, cnt);
            else rt_closest_kernel_body<32>(T, tq, q, count, idx, cnt);
        } else if (kind == 1 && count >= 1 && count <= 16 && (T.flags & TF_NCL)) {
            nc_line_kernel_body<0, false, false>(T, T, nullptr, tq, q, count, idx, cnt);
        } else {
            // count 0, counts above 32, NodeCache without lines: one query per wave
            for (uint32_t i = w; i < q; i += BLOCK / 64) {  // wave-uniform
                const Target t = load_target(tq, i);
                uint32_t* row = idx + (size_t)i * count;
                uint8_t* cp = cnt + i;
                if (count == 0) {
                    if (lane == 0) *cp = 0;
                } else if (kind == 0) {
                    if (T.B == 0) {  // an empty table: an empty result (routing_table.cpp:73)
                        if (lane < count) row[lane] = NONE;
                        if (lane == 0) *cp = 0;
                    } else {
                        uint32_t lo, hi, good;
                        wave_window(T.gcnt, T.B, locate_bucket(T, t), count, lo, hi, good);
                        wave_rank_any(T, t, T.dir[lo].x & ~WIDE, T.dir[hi + 1].x & ~WIDE, good, count, row, cp, xs[w]);
                    }
                } else if (T.n > 0) {
                    // the placement rounds use all 64 lanes; the serial walk (lane 0) answers what the runs cannot
                    nc64_query(T, t, lane, i, count, idx, cnt, true);
                } else if (lane == 0) {
                    nc_serial(T, t, count, row, cp);
                }
            }
        }
        __threadfence_system();  // this wave's rows and counts reach host memory before `done`
        __syncthreads();
        if (tid == 0) {
            reply->t_done = wall_clock64();
            __hip_atomic_store(&reply->done, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
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

// Host-pointer batches (kad_*_closest_batch_host): pinned staging and device buffers kept with the table, and a
// chunked pipeline per worker thread: host copy into pinned memory, H2D, kernel, D2H, host copy out. Each worker has
// two slots on their own streams, so one slot's copies and kernel overlap the other slot's host copies, and the
// workers split the batch so that the pageable host copies run on several cores.
struct HostPipe {
    static constexpr uint32_t CHUNK = 1u << 16;  // queries per slot
    static constexpr int WORKERS = 4, SLOTS = 2;
    struct Slot {
        uint8_t *ht = nullptr, *hc = nullptr, *dt = nullptr, *dc = nullptr;  // pinned / device: targets, counts
        uint32_t *hi = nullptr, *di = nullptr;                               // pinned / device: indices
        hipStream_t s = nullptr;
        hipEvent_t done = nullptr;
        uint32_t c0 = 0, n = 0;
        bool pending = false;
    };
    Slot slot[WORKERS][SLOTS];
    hipEvent_t start = nullptr;  // recorded on the null stream: the slots' streams wait for prior device work
    std::mutex mu;      // one host batch per table at a time
    // Small batches (single Dht requests): one launch on pinned host memory the kernel reads and writes
    // directly (mapped into the device's address space), no copies, one stream synchronise.
    static constexpr uint32_t SMALL = 1024, SMALL_COUNT = 64;
    uint8_t *st = nullptr, *sc = nullptr;  // pinned: targets, counts
    uint32_t* si = nullptr;                // pinned: rows
    uint8_t *dst = nullptr, *dsc = nullptr;  // their device addresses
    uint32_t* dsi = nullptr;
    hipStream_t ss = nullptr;
    // Resident query service (kad_table_serve, svc_kernel): mailbox and reply in mapped pinned memory
    SvcMail* vm = nullptr;   // host view / device view
    SvcMail* dvm = nullptr;
    SvcReply* vr = nullptr;
    SvcReply* dvr = nullptr;
    hipStream_t vs = nullptr;
    uint32_t vseq = 0;       // the last request number posted
    uint64_t vlaunches = 0, vrequests = 0;  // kad_table_serve_stats
    int vkhz = 0;            // device wall clock rate
    uint32_t idle_us = 0;    // 0: the service is off
    bool vrun = false;       // a launch may still be running on vs
    ~HostPipe() {
        if (vs) {
            if (vm) __atomic_store_n(&vm->stop, 1u, __ATOMIC_RELEASE);
            (void)hipStreamSynchronize(vs);
            (void)hipStreamDestroy(vs);
        }
        for (void* p : {(void*)vm, (void*)vr}) if (p) (void)hipHostFree(p);
        if (ss) { (void)hipStreamSynchronize(ss); (void)hipStreamDestroy(ss); }
        for (void* p : {(void*)st, (void*)sc, (void*)si}) if (p) (void)hipHostFree(p);
        for (auto& w : slot)
            for (Slot& S : w) {
                if (S.s) (void)hipStreamSynchronize(S.s);
                for (void* p : {(void*)S.ht, (void*)S.hc, (void*)S.hi}) if (p) (void)hipHostFree(p);
                for (void* p : {(void*)S.dt, (void*)S.dc, (void*)S.di}) if (p) (void)hipFree(p);
                if (S.done) (void)hipEventDestroy(S.done);
                if (S.s) (void)hipStreamDestroy(S.s);
            }
        if (start) (void)hipEventDestroy(start);
    }
};

// isGood(now) deadlines of a table with node times (kad_table_refresh_status; the device side is at
// deadline_kernel). valid: the runs, cursors and status bytes agree with the device times at last_now. The host
// keeps a copy of both runs' keys, so it finds the passed ranges itself (no device search, no read-back) and
// knows the next deadline at once.
struct Deadlines {
    bool valid = false;
    int64_t last_now = INT64_MIN;
    uint64_t* km = nullptr;        // main run: keys and nodes, n entries (device)
    uint32_t* kn = nullptr;
    uint32_t nm = 0, mcap = 0;
    std::vector<uint64_t> hkm;     // the main run's keys and nodes (host copies)
    std::vector<uint32_t> hkn;
    uint32_t cm = 0, cs = 0;       // cursors: the first unpassed entry of each run
    uint64_t* ks = nullptr;        // side run: deadlines of patched nodes (device), kept sorted on the host
    uint32_t* sn = nullptr;
    uint32_t ns = 0, scap = 0;
    std::vector<uint64_t> hks;
    std::vector<uint32_t> hsn;
    uint32_t* pend = nullptr;      // nodes patched since the last refresh (device), re-derived at the next one
    uint32_t np = 0, pcap = 0;
    std::vector<uint32_t> hpend;
    uint64_t next = 0;             // the smallest unpassed key (valid runs)
    void* tmp = nullptr;           // radix-sort scratch: keys, nodes, hipcub temp storage
    size_t tmp_bytes = 0;
    ~Deadlines() {
        for (void* p : {(void*)km, (void*)kn, (void*)ks, (void*)sn, (void*)pend, tmp})
            if (p) (void)hipFree(p);
    }
    void invalidate() {
        valid = false;
        np = 0;
        ns = 0;
        cs = 0;
        hpend.clear();
        hks.clear();
        hsn.clear();
    }
    void set_next() {
        const uint64_t a = cm < hkm.size() ? hkm[cm] : ~0ull, b = cs < hks.size() ? hks[cs] : ~0ull;
        next = std::min(a, b);
    }
};

struct kad_table {
    int device = 0;
    uint32_t flags = 0;
    DevTable d{};
    std::vector<void*> owned;
    uint64_t bytes = 0;
    uint32_t rbits = 0, nbits = 0;
    uint8_t* status_mut = nullptr;
    uint2* dir_mut = nullptr;
    uint32_t* wl_mut = nullptr;
    uint32_t* ws_mut = nullptr;
    uint32_t* wl16_mut = nullptr;
    uint32_t* wl32_mut = nullptr;
    uint32_t* ncl_mut = nullptr;
    uint32_t* ncl32_mut = nullptr;
    uint32_t* gl_mut = nullptr;
    uint32_t* gl32_mut = nullptr;
    uint32_t* gl16_mut = nullptr;
    uint32_t* sl_mut = nullptr;     // slot lines (TF_SL) and the bucket of every coarse slot
    uint32_t* slb = nullptr;
    uint32_t* sl16_mut = nullptr;   // slot lines for counts 9..16 (TF_SL16)
    uint8_t* gdirty = nullptr;      // B: general lines rebuilt by an incremental refresh (slot-line transcode)
    // host copies of the bucket directory, for the incremental mirror (kad_table_apply)
    std::vector<uint32_t> h_off;
    std::vector<uint8_t> h_first;
    int8_t firsts_low_zero = -1, firsts_low_zero_next = -1;  // all h_first low 96 bits zero (-1: not known yet)
    uint32_t* wrec = nullptr;  // per-node wire records: ID + address + port (kad_table_set_addrs)
    uint32_t addr_len = 0;
    int64_t* time_ns = nullptr;
    int64_t* reply_ns = nullptr;
    uint8_t* expired = nullptr;
    uint32_t* gcnt_mut = nullptr;   // B+1: the per-bucket good counts (d.gcnt), kept current by every rebuild
    // incremental status refresh (allocated on first use, see StatusMarks)
    uint8_t* bdirty = nullptr;      // B
    uint8_t* ld8 = nullptr;         // B each, per line set present: lines to rebuild
    uint8_t* ld16 = nullptr;
    uint8_t* ld32 = nullptr;
    uint8_t* ndirty = nullptr;      // NodeCache radix slots (only with NodeCache lines)
    uint32_t* dlist = nullptr;      // compacted dirty lists: 3 x B line indices + NodeCache slots
    uint32_t* dctr = nullptr;       // 4 list lengths
    void* stage = nullptr;          // host -> device staging of patch lists
    size_t stage_bytes = 0;
    mutable std::mutex pipe_mu;     // creates `pipe` on the first host-pointer batch
    mutable HostPipe* pipe = nullptr;
    Deadlines dl;                   // isGood(now) deadlines (kad_table_refresh_status)
    uint32_t* rf_ctr = nullptr;     // small refresh (rf_nodes_kernel): counters, appended buckets, NodeCache ranges
    uint32_t rf_epoch = 0;          // the last fused refresh's list epoch (rf_ctr[RF_GO])
    // FUSE 2's builder blocks spin for block 0's list; when other work holds the CUs that spin can time out (a
    // latency cliff of up to RF_SPIN_TICKS). rf_spin_host: pinned mirror of rf_ctr[RF_SPIN],
    // copied after every fused general-line refresh and read by the next one; once non-zero the table never fuses
    // the general-line builds again (rf_no_fuse2: they go out as stream-ordered launches after the node kernel).
    uint32_t* rf_spin_host = nullptr;
    bool rf_no_fuse2 = false;
    uint32_t* rf_blist = nullptr;
    uint32_t* rf_nrange = nullptr;
    hipStream_t ss[2] = {nullptr, nullptr};  // side streams of an incremental rebuild (side_streams)
    hipEvent_t mut_ev = nullptr;    // recorded after the last asynchronous status refresh (the host batches wait on it)
    bool mut_async = false;
    // line sets built on first use (ensure_lines): the sets built or found not to apply to this table's shape,
    // and each one's bytes and build time
    std::atomic<uint32_t> ls_done{0};
    std::mutex ls_mu;
    uint64_t ls_bytes[8] = {};
    float ls_ms[8] = {};
    hipEvent_t ev_fork = nullptr, ev_join[2] = {nullptr, nullptr};
    hipStream_t bs = nullptr;       // line-set builds (ensure_lines): a non-blocking stream of the table's own
    ~kad_table() {
        if (bs) { (void)hipStreamSynchronize(bs); (void)hipStreamDestroy(bs); }
        for (hipStream_t x : ss)
            if (x) { (void)hipStreamSynchronize(x); (void)hipStreamDestroy(x); }
        for (hipEvent_t e : {ev_fork, ev_join[0], ev_join[1], mut_ev})
            if (e) (void)hipEventDestroy(e);
        delete pipe;
        for (void* p : owned) (void)hipFree(p);
        for (void* p : {(void*)bdirty, (void*)ld8, (void*)ld16, (void*)ld32, (void*)ndirty, (void*)dlist, (void*)dctr, stage,
                        (void*)rf_ctr, (void*)rf_blist, (void*)rf_nrange})
            if (p) (void)hipFree(p);
        if (rf_spin_host) (void)hipHostFree(rf_spin_host);
    }
};

static int svc_quiesce(const kad_table* t);  // ends the resident query service's launch (kad_table_serve)

namespace {

bool is_gfx950(int dev) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, dev) != hipSuccess) return false;
    return std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
}

// Re-derive what depends on the status bytes: good masks, per-bucket good counts, the good prefix sums,
// the window lines and the NodeCache lines. full: every bucket and line; otherwise only what the
// StatusMarks of the last status change flagged (kad_table_refresh_status / update / patch; ensure_marks
// must have run). Async on stream.
// The table's two side streams and the fork / join events of an incremental rebuild (created on first use).
int side_streams(kad_table* t) {
    for (hipStream_t& x : t->ss)
        if (!x) HIP_TRY(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    if (!t->ev_fork) HIP_TRY(hipEventCreateWithFlags(&t->ev_fork, hipEventDisableTiming));
    for (hipEvent_t& e : t->ev_join)
        if (!e) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return KAD_OK;
}

// The table's build stream (created on first use; the null stream if that fails). Line-set builds run there and
// wait for it alone, not for the whole device (a resident service or another thread's graph capture).
hipStream_t build_stream(kad_table* t) {
    if (!t->bs && hipStreamCreateWithFlags(&t->bs, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        t->bs = nullptr;
    }
    return t->bs;
}

int rebuild_good_prefix_(kad_table* t, hipStream_t s, bool full);
int rebuild_good_prefix(kad_table* t, hipStream_t s, bool full = true) {
    const int rc = rebuild_good_prefix_(t, s, full);
    // the change flag of the marks just consumed (StatusMarks::any)
    if (rc == KAD_OK && t->dctr) HIP_TRY(hipMemsetAsync(t->dctr + 4, 0, sizeof(uint32_t), s));
    return rc;
}
int rebuild_good_prefix_(kad_table* t, hipStream_t s, bool full) {
    const uint32_t B = t->d.B;
    uint32_t* ctr = t->dctr;
    // incremental: every kernel exits at once when no status changed (dctr[4], set by mark_status_change)
    const uint32_t* any = full ? nullptr : t->dctr + 4;
    if (!full) HIP_TRY(hipMemsetAsync(ctr, 0, 4 * sizeof(uint32_t), s));
    // line builders loop over their items: an incremental rebuild (a dirty list whose length only the device
    // knows) launches at most one chip-filling grid instead of one thread per line
    auto lgrid = [&](uint64_t threads) { return dim3(full ? grid_for(threads) : std::min(grid_for(threads), 2048u)); };
    if (t->ncl_mut) {  // NodeCache lines carry the expired bits
        LineSel sel{};
        if (!full) {
            uint32_t* lst = t->dlist + 3ull * B;
            hipLaunchKernelGGL(compact_flags_kernel, dim3(grid_for((t->d.nslots + 15) / 16)), dim3(BLOCK), 0, s,
                               t->ndirty, t->d.nslots, lst, ctr + 3, any);
            sel = LineSel{lst, ctr + 3};
        }
        hipLaunchKernelGGL(ncl_build_kernel, lgrid(t->d.nslots), dim3(BLOCK), 0, s, t->d.key, t->d.status,
                           t->d.nrdx, t->d.nslots, t->d.n, 64 - t->d.nshift, t->ncl_mut, sel);
        if (t->ncl32_mut)  // the same slots: the marks cover the wider windows when these lines exist
            hipLaunchKernelGGL(ncl32_build_kernel, lgrid(8ull * t->d.nslots), dim3(BLOCK), 0, s, t->d.key,
                               t->d.status, t->d.nrdx, t->d.nslots, t->d.n, 64 - t->d.nshift, t->ncl32_mut, sel);
    }
    if (B == 0) return KAD_OK;
    const uint32_t m = B + 1;
    if (full)
        hipLaunchKernelGGL(bucket_good_kernel, dim3(grid_for(m)), dim3(BLOCK), 0, s, t->d.status, t->dir_mut, B,
                           t->gcnt_mut);
    else
        hipLaunchKernelGGL(bucket_good_dirty_kernel, dim3(grid_for(B)), dim3(BLOCK), 0, s, t->d.status, t->dir_mut, B,
                           t->gcnt_mut, t->bdirty, (t->wl_mut || t->gl_mut) ? t->ld8 : nullptr,
                           (t->wl16_mut || t->gl16_mut) ? t->ld16 : nullptr, (t->wl32_mut || t->gl32_mut) ? t->ld32 : nullptr,
                           any);
    // the lines of every bucket (full) or only the compacted dirty ones
    auto sel_for = [&](uint8_t* flags, uint32_t k, hipStream_t st) -> LineSel {
        if (full) return LineSel{};
        hipLaunchKernelGGL(compact_flags_kernel, dim3(grid_for((B + 15) / 16)), dim3(BLOCK), 0, st, flags, B,
                           t->dlist + (size_t)k * B, ctr + k, any);
        return LineSel{t->dlist + (size_t)k * B, ctr + k};
    };
    // Three independent chains (an incremental rebuild is a few latency-bound items per builder, so they
    // overlap): A = count <= 8 lines and everything that shares the general tables' gdirty flags, on s;
    // B = the uniform count 9..16 lines and C = the count 17..32 lines on the table's side streams, forked
    // from s after the prefix sums and joined back into s.
    hipStream_t sB = s, sC = s;
    const bool fork = !full && t->wl16_mut && (t->wl32_mut || t->gl32_mut) && side_streams(t) == KAD_OK;
    if (fork) {
        HIP_TRY(hipEventRecord(t->ev_fork, s));
        sB = t->ss[0];
        sC = t->ss[1];
        HIP_TRY(hipStreamWaitEvent(sB, t->ev_fork, 0));
        HIP_TRY(hipStreamWaitEvent(sC, t->ev_fork, 0));
    }
    if (t->wl16_mut)
        hipLaunchKernelGGL(wl16_build_kernel, lgrid(B), dim3(BLOCK), 0, sB, t->d.key, t->d.status, t->d.dir,
                           t->d.gcnt, B, 64 - t->d.rshift, t->d.rbase >> t->d.rshift, t->wl16_mut, sel_for(t->ld16, 1, sB));
    if (t->wl32_mut)
        hipLaunchKernelGGL(wl32_build_kernel, lgrid(B), dim3(BLOCK), 0, sC, t->d.key, t->d.status, t->d.dir,
                           t->d.gcnt, B, 64 - t->d.rshift, t->d.rbase >> t->d.rshift, t->wl32_mut, sel_for(t->ld32, 2, sC));
    if (t->gl32_mut)
        hipLaunchKernelGGL(gl32_build_kernel, lgrid(B), dim3(BLOCK), 0, sC, t->d.key, t->d.status, t->d.dir,
                           t->d.gcnt, t->d.fkey, t->d.ftail, B, t->gl32_mut, sel_for(t->ld32, 2, sC));
    LineSel s8{};
    if (t->wl_mut || t->gl_mut) s8 = sel_for(t->ld8, 0, s);
    if (t->wl_mut && !full)  // a few scattered lines: a wave per line (wl_ws_wave_kernel), the short copies with it
        hipLaunchKernelGGL(wl_ws_wave_kernel, lgrid(64ull * B), dim3(BLOCK), 0, s, t->d.key, t->d.status, t->d.dir,
                           t->d.gcnt, B, 64 - t->d.rshift, t->d.rbase >> t->d.rshift, t->wl_mut, t->ws_mut, s8);
    else if (t->wl_mut && t->ws_mut)  // the short lines transcoded from the 128-byte lines in the same thread
        hipLaunchKernelGGL(wl_build_kernel<true>, lgrid(B), dim3(BLOCK), 0, s, t->d.key, t->d.status, t->d.dir,
                           t->d.gcnt, B, 64 - t->d.rshift, t->d.rbase >> t->d.rshift, t->wl_mut, t->ws_mut, s8);
    else if (t->wl_mut)
        hipLaunchKernelGGL(wl_build_kernel<false>, lgrid(B), dim3(BLOCK), 0, s, t->d.key, t->d.status, t->d.dir,
                           t->d.gcnt, B, 64 - t->d.rshift, t->d.rbase >> t->d.rshift, t->wl_mut, nullptr, s8);
    if (t->gl_mut)
        hipLaunchKernelGGL(gl_build_kernel, lgrid(B), dim3(BLOCK), 0, s, t->d.key, t->d.status, t->d.dir,
                           t->d.gcnt, t->d.fkey, t->d.ftail, B, t->gl_mut, s8);
    if (t->sl_mut) {  // slot lines: transcoded from the general lines just rebuilt (all, or the flagged buckets')
        if (!full) hipLaunchKernelGGL(mark_sel_kernel, lgrid(B), dim3(BLOCK), 0, s, s8, B, t->gdirty, (uint8_t)1);
        hipLaunchKernelGGL(sl_build_kernel, lgrid(t->d.slslots), dim3(BLOCK), 0, s, t->gl_mut, t->slb, t->d.slslots,
                           full ? nullptr : t->gdirty, t->d.rrdx, t->d.rslots, t->d.slshift - t->d.rshift, t->d.fkey,
                           t->d.ftail, t->sl_mut);
        if (!full) hipLaunchKernelGGL(mark_sel_kernel, lgrid(B), dim3(BLOCK), 0, s, s8, B, t->gdirty, (uint8_t)0);
    }
    if (t->gl16_mut) {
        const LineSel s16 = sel_for(t->ld16, 1, s);
        hipLaunchKernelGGL(gl16_build_kernel, lgrid(B), dim3(BLOCK), 0, s, t->d.key, t->d.status, t->d.dir,
                           t->d.gcnt, t->d.fkey, t->d.ftail, B, t->gl16_mut, s16);
        if (t->sl16_mut) {  // their slot-indexed copies: all, or the flagged buckets'
            if (!full) hipLaunchKernelGGL(mark_sel_kernel, lgrid(B), dim3(BLOCK), 0, s, s16, B, t->gdirty, (uint8_t)1);
            hipLaunchKernelGGL(sl16_build_kernel, lgrid(8ull * t->d.slslots), dim3(BLOCK), 0, s, t->gl16_mut, t->slb,
                               t->d.slslots, full ? nullptr : t->gdirty, t->d.rrdx, t->d.rslots,
                               t->d.slshift - t->d.rshift, t->d.fkey, t->d.ftail, t->sl16_mut);
            if (!full) hipLaunchKernelGGL(mark_sel_kernel, lgrid(B), dim3(BLOCK), 0, s, s16, B, t->gdirty, (uint8_t)0);
        }
    }
    if (fork) {
        HIP_TRY(hipEventRecord(t->ev_join[0], sB));
        HIP_TRY(hipEventRecord(t->ev_join[1], sC));
        HIP_TRY(hipStreamWaitEvent(s, t->ev_join[0], 0));
        HIP_TRY(hipStreamWaitEvent(s, t->ev_join[1], 0));
    }
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

// Slot lines (TF_SL) for a table with general lines: the coarsening k (coarse slot = 2^k locate slots) is the
// coarsest (smallest table) at which at most 1/32 of the coarse slots hold a bucket start (their queries take a
// fallback line), provided the lines fit 512 MiB; otherwise no slot lines. Synchronous; a failure leaves the
// table without them.
int build_sl16(kad_table* t);

int setup_slot_lines(kad_table* t) {
    DevTable& d = t->d;
    if (!(d.flags & TF_GL) || !t->gl_mut || d.B == 0 || d.rslots == 0 || t->h_first.size() < 20ull * d.B) return KAD_OK;
    if (t->flags & KAD_TABLE_NO_SLOT_LINES) return KAD_OK;  // general lines alone (the caller's choice)
    const uint32_t B = d.B;
    const uint8_t* f = t->h_first.data();
    int pick = -1;
    for (uint32_t k = 0; k <= 4 && d.rshift + k <= 63; k++) {
        const uint32_t sh = d.rshift + k;
        const uint64_t slots = ((uint64_t)d.rslots + (1ull << k) - 1) >> k;
        uint64_t inner = 0, last = ~0ull;
        for (uint32_t b = 0; b < B; b++) {
            const uint64_t rel = id_hi(f + 20ull * b) - d.rbase;
            if ((rel & ((1ull << sh) - 1)) == 0 && id_low_zero(f + 20ull * b)) continue;  // starts at a slot start
            const uint64_t j = rel >> sh;
            if (j != last) { inner++; last = j; }
        }
        const bool few = inner * 32 <= slots;
        if (std::getenv("KAD_DEBUG"))
            std::fprintf(stderr, "slot lines: k=%u slots=%llu inner=%llu\n", k, (unsigned long long)slots,
                         (unsigned long long)inner);
        if (few && slots * 64 <= (512ull << 20)) pick = (int)k;  // the coarsest (smallest) that qualifies
    }
    if (pick < 0) return KAD_OK;
    const uint32_t k = (uint32_t)pick;
    const uint32_t slslots = (uint32_t)(((uint64_t)d.rslots + (1ull << k) - 1) >> k);
    uint32_t *lines = nullptr, *slb = nullptr;
    uint8_t* gd = nullptr;
    std::vector<void*> fresh;
    uint64_t fb = 0;
    auto drop = [&]() { for (void* p : fresh) (void)hipFree(p); };
    if (dev_upload(&lines, nullptr, 16ull * slslots, fresh, fb) || dev_upload(&slb, nullptr, slslots, fresh, fb) ||
        dev_upload(&gd, nullptr, B, fresh, fb) || hipMemset(gd, 0, B) != hipSuccess) {
        drop();
        return KAD_OK;
    }
    hipLaunchKernelGGL(sl_index_kernel, dim3(grid_for(slslots)), dim3(BLOCK), 0, build_stream(t), d.rrdx, d.rslots, k, slslots, slb);
    hipLaunchKernelGGL(sl_build_kernel, dim3(grid_for(slslots)), dim3(BLOCK), 0, build_stream(t), t->gl_mut, slb, slslots, nullptr,
                       d.rrdx, d.rslots, k, d.fkey, d.ftail, lines);
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(build_stream(t)) != hipSuccess) {
        drop();
        return set_err(KAD_ERR_HIP, "slot-line build failed");
    }
    if (std::getenv("KAD_DEBUG")) {
        uint32_t* dc = nullptr;
        uint32_t hc[2] = {0, 0};
        if (hipMalloc(&dc, 8) == hipSuccess && hipMemset(dc, 0, 8) == hipSuccess) {
            hipLaunchKernelGGL(sl_count_kernel, dim3(grid_for(slslots)), dim3(BLOCK), 0, build_stream(t), lines, slslots, dc);
            (void)hipMemcpy(hc, dc, 8, hipMemcpyDeviceToHost);
        }
        if (dc) (void)hipFree(dc);
        std::fprintf(stderr, "slot lines: k=%u, %u slots, %u fallback lines (%u without a bucket)\n", k, slslots, hc[0], hc[1]);
    }
    t->owned.insert(t->owned.end(), fresh.begin(), fresh.end());
    t->bytes += fb;
    t->sl_mut = lines; t->slb = slb; t->gdirty = gd;
    d.sl = reinterpret_cast<const uint4*>(lines);
    d.slb = slb;
    d.slshift = d.rshift + k;
    d.slslots = slslots;
    d.flags |= TF_SL;
    return build_sl16(t);
}

// Counts 9..16 on a table with slot lines: copies of the gl16 lines at the same slots (optional: without them,
// locate + gl16). Synchronous.
int build_sl16(kad_table* t) {
    DevTable& d = t->d;
    if (!t->gl16_mut || !t->sl_mut || t->sl16_mut) return KAD_OK;
    std::vector<void*> f16;
    uint64_t b16 = 0;
    uint32_t* l16 = nullptr;
    if (dev_upload(&l16, nullptr, (size_t)GL16_STRIDE * d.slslots, f16, b16) == KAD_OK) {
        hipLaunchKernelGGL(sl16_build_kernel, dim3(grid_for(8ull * d.slslots)), dim3(BLOCK), 0, build_stream(t), t->gl16_mut, t->slb,
                           d.slslots, nullptr, d.rrdx, d.rslots, d.slshift - d.rshift, d.fkey, d.ftail, l16);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(build_stream(t)) != hipSuccess) {
            for (void* p : f16) (void)hipFree(p);
            return set_err(KAD_ERR_HIP, "slot-line (16) build failed");
        }
        t->owned.insert(t->owned.end(), f16.begin(), f16.end());
        t->bytes += b16;
        t->sl16_mut = l16;
        d.sl16 = reinterpret_cast<const uint4*>(l16);
        d.flags |= TF_SL16;
    }
    return KAD_OK;
}

// General window lines for count <= 8 (TF_GL) for a table without uniform-depth lines: allocated, built from the
// current status, and kept only when at most 1/16 of them are deferred (otherwise the lane kernel is the faster
// path); then the slot lines. Synchronous. A failure leaves the table without general lines (still correct).
// The count 9..32 general lines are built on first use (build_gl32, build_gl16).
int count_deferred(const uint32_t* lines, uint32_t stride, uint32_t hdr_word, uint32_t B, uint32_t& nd,
                   hipStream_t s) {
    uint32_t* cnt = nullptr;
    HIP_TRY(hipMalloc(&cnt, 4));
    hipError_t e = hipMemsetAsync(cnt, 0, 4, s);
    if (e == hipSuccess) {
        hipLaunchKernelGGL(count_deferred_kernel, dim3(grid_for(B)), dim3(BLOCK), 0, s, lines, stride, hdr_word, B, cnt);
        e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpyAsync(&nd, cnt, 4, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    (void)hipFree(cnt);
    if (e != hipSuccess) return set_err(KAD_ERR_HIP, "deferred-line count failed: %s", hipGetErrorString(e));
    return KAD_OK;
}

int setup_general_lines(kad_table* t) {
    DevTable& d = t->d;
    if (d.B == 0 || (d.flags & TF_WL) || !d.fkey) return KAD_OK;
    const uint32_t B = d.B;
    uint32_t* lp = nullptr;
    std::vector<void*> fresh;
    uint64_t fb = 0;
    if (dev_upload(&lp, nullptr, (size_t)GL_STRIDE * B, fresh, fb)) return KAD_OK;
    hipLaunchKernelGGL(gl_build_kernel, dim3(grid_for(B)), dim3(BLOCK), 0, build_stream(t), d.key, d.status, d.dir, d.gcnt, d.fkey,
                       d.ftail, B, lp, LineSel{});
    uint32_t nd = B;
    int rc;
    if (hipGetLastError() != hipSuccess || (rc = count_deferred(lp, GL_STRIDE, 1u, B, nd, build_stream(t)))) {
        (void)hipFree(lp);
        return set_err(KAD_ERR_HIP, "general window-line build failed");
    }
    if (std::getenv("KAD_DEBUG")) std::fprintf(stderr, "general lines: B=%u deferred %u (count <= 8)\n", B, nd);
    if ((uint64_t)nd * 16 > B) {
        (void)hipFree(lp);
        return KAD_OK;
    }
    t->owned.push_back(lp); t->bytes += fb;
    t->gl_mut = lp; d.gl = reinterpret_cast<const uint4*>(lp); d.flags |= TF_GL;
    return setup_slot_lines(t);
}

// The 256-byte general lines (counts 9..32), kept when at most 1/16 are deferred. Synchronous.
int build_gl32(kad_table* t) {
    DevTable& d = t->d;
    if (d.B == 0 || (d.flags & TF_WL) || !d.fkey || t->gl32_mut) return KAD_OK;
    const uint32_t B = d.B;
    uint32_t* lp = nullptr;
    std::vector<void*> fresh;
    uint64_t fb = 0;
    int rc;
    if ((rc = dev_upload(&lp, nullptr, (size_t)GL32_STRIDE * B, fresh, fb))) return rc;
    hipLaunchKernelGGL(gl32_build_kernel, dim3(grid_for(B)), dim3(BLOCK), 0, build_stream(t), d.key, d.status, d.dir, d.gcnt, d.fkey,
                       d.ftail, B, lp, LineSel{});
    uint32_t nd = B;
    if (hipGetLastError() != hipSuccess || (rc = count_deferred(lp, GL32_STRIDE, 3u, B, nd, build_stream(t)))) {
        (void)hipFree(lp);
        return set_err(KAD_ERR_HIP, "general window-line (32) build failed");
    }
    if (std::getenv("KAD_DEBUG")) std::fprintf(stderr, "general lines 32: B=%u deferred %u\n", B, nd);
    if ((uint64_t)nd * 16 > B) { (void)hipFree(lp); return KAD_OK; }
    t->owned.push_back(lp); t->bytes += fb;
    t->gl32_mut = lp; d.gl32 = reinterpret_cast<const uint4*>(lp); d.flags |= TF_GL32;
    return KAD_OK;
}

// The 128-byte general lines of counts 9..16 (the 256-byte lines are their fallback, so only with those), kept
// when at most 1/16 are deferred, and their slot-indexed copies when the table has slot lines. Synchronous.
int build_gl16(kad_table* t) {
    DevTable& d = t->d;
    if (d.B == 0 || (d.flags & TF_WL) || !d.fkey || t->gl16_mut || !t->gl32_mut) return KAD_OK;
    const uint32_t B = d.B;
    uint32_t* lp = nullptr;
    std::vector<void*> fresh;
    uint64_t fb = 0;
    int rc;
    if ((rc = dev_upload(&lp, nullptr, (size_t)GL16_STRIDE * B, fresh, fb))) return rc;
    hipLaunchKernelGGL(gl16_build_kernel, dim3(grid_for(B)), dim3(BLOCK), 0, build_stream(t), d.key, d.status, d.dir, d.gcnt, d.fkey,
                       d.ftail, B, lp, LineSel{});
    uint32_t nd = B;
    if (hipGetLastError() != hipSuccess || (rc = count_deferred(lp, GL16_STRIDE, 1u, B, nd, build_stream(t)))) {
        (void)hipFree(lp);
        return set_err(KAD_ERR_HIP, "general window-line (16) build failed");
    }
    if (std::getenv("KAD_DEBUG")) std::fprintf(stderr, "general lines 16: B=%u deferred %u\n", B, nd);
    if ((uint64_t)nd * 16 > B) { (void)hipFree(lp); return KAD_OK; }
    t->owned.push_back(lp); t->bytes += fb;
    t->gl16_mut = lp; d.gl16 = reinterpret_cast<const uint4*>(lp); d.flags |= TF_GL16;
    return build_sl16(t);
}

// Allocate (zeroed) the incremental-refresh flags for the table's current shape.
int ensure_marks(kad_table* t) {
    auto alloc = [](uint8_t** p, size_t n) -> int {
        if (*p || n == 0) return KAD_OK;
        n = (n + 15) & ~(size_t)15;  // compact_flags_kernel reads 16 flags at a time
        void* q = nullptr;
        hipError_t e = hipMalloc(&q, n);
        if (e != hipSuccess) return set_err(KAD_ERR_NOMEM, "hipMalloc(%zu) failed: %s", n, hipGetErrorString(e));
        e = hipMemset(q, 0, n);
        if (e != hipSuccess) { (void)hipFree(q); return set_err(KAD_ERR_HIP, "hipMemset failed: %s", hipGetErrorString(e)); }
        *p = static_cast<uint8_t*>(q);
        return KAD_OK;
    };
    int rc;
    if ((rc = alloc(&t->bdirty, t->d.B))) return rc;
    if ((t->wl_mut || t->gl_mut) && (rc = alloc(&t->ld8, t->d.B))) return rc;
    if ((t->wl16_mut || t->gl16_mut) && (rc = alloc(&t->ld16, t->d.B))) return rc;
    if ((t->wl32_mut || t->gl32_mut) && (rc = alloc(&t->ld32, t->d.B))) return rc;
    if (t->ncl_mut && (rc = alloc(&t->ndirty, t->d.nslots))) return rc;
    uint8_t *l = reinterpret_cast<uint8_t*>(t->dlist), *c = reinterpret_cast<uint8_t*>(t->dctr);
    if ((rc = alloc(&l, 4 * (3ull * t->d.B + (t->ncl_mut ? t->d.nslots : 0u) + 1)))) return rc;
    if ((rc = alloc(&c, 8 * sizeof(uint32_t)))) return rc;  // 4 list lengths, [4] the change flag
    t->dlist = reinterpret_cast<uint32_t*>(l);
    t->dctr = reinterpret_cast<uint32_t*>(c);
    return KAD_OK;
}

// Drop the incremental-refresh flags (the table's shape changed: kad_table_apply).
void drop_marks(kad_table* t) {
    for (uint8_t** p : {&t->bdirty, &t->ld8, &t->ld16, &t->ld32, &t->ndirty})
        if (*p) { (void)hipFree(*p); *p = nullptr; }
    if (t->dlist) { (void)hipFree(t->dlist); t->dlist = nullptr; }
    if (t->dctr) { (void)hipFree(t->dctr); t->dctr = nullptr; }
}

StatusMarks marks_of(const kad_table* t) {
    StatusMarks M{};
    M.bdirty = t->d.B ? t->bdirty : nullptr;
    M.ndirty = t->ncl_mut ? t->ndirty : nullptr;
    M.dir = t->d.dir;
    M.B = t->d.B;
    M.key = t->d.key;
    M.nbase = t->d.nbase;
    M.nshift = t->d.nshift;
    M.nslots = t->d.nslots;
    M.n = t->d.n;
    M.nback = t->ncl32_mut ? NC32_SLOTS - NC32_LEFT : NCL_SLOTS - NCL_LEFT;
    M.nfwd = t->ncl32_mut ? NC32_LEFT : NCL_LEFT;
    M.any = t->dctr ? t->dctr + 4 : nullptr;
    return M;
}

// Device staging buffer of at least `bytes` (host patch lists).
int stage_reserve(kad_table* t, size_t bytes) {
    if (t->stage_bytes >= bytes) return KAD_OK;
    if (t->stage) { (void)hipFree(t->stage); t->stage = nullptr; t->stage_bytes = 0; }
    hipError_t e = hipMalloc(&t->stage, std::max<size_t>(bytes, 4096));
    if (e != hipSuccess) { t->stage = nullptr; return set_err(KAD_ERR_NOMEM, "hipMalloc(%zu) failed", bytes); }
    t->stage_bytes = std::max<size_t>(bytes, 4096);
    return KAD_OK;
}

// The table's state changed asynchronously on stream s (kad_table_refresh_status): the host batches, on their
// own streams, wait for the event recorded here.
int mark_async(kad_table* t, hipStream_t s) {
    if (!t->mut_ev) HIP_TRY(hipEventCreateWithFlags(&t->mut_ev, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(t->mut_ev, s));
    t->mut_async = true;
    return KAD_OK;
}

// ---- small refresh (rf_nodes_kernel) ----
NodeTimes times_of(const kad_table* t) { return NodeTimes{t->time_ns, t->reply_ns, t->expired}; }

int rf_ready(kad_table* t) {
    if (t->rf_ctr) return KAD_OK;
    void *c = nullptr, *bl = nullptr, *nr = nullptr;
    hipError_t e = hipMalloc(&c, RF_CTRS * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&bl, RF_CAP * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&nr, 2 * RF_CAP * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMemset(c, 0, RF_CTRS * sizeof(uint32_t));
    void* sh = nullptr;
    if (e == hipSuccess) e = hipHostMalloc(&sh, sizeof(uint32_t), hipHostMallocDefault);
    if (e != hipSuccess) {
        for (void* p : {c, bl, nr}) if (p) (void)hipFree(p);
        if (sh) (void)hipHostFree(sh);
        return set_err(KAD_ERR_NOMEM, "small refresh buffers: %s", hipGetErrorString(e));
    }
    *static_cast<uint32_t*>(sh) = 0;
    t->rf_spin_host = static_cast<uint32_t*>(sh);
    t->rf_ctr = static_cast<uint32_t*>(c);
    t->rf_blist = static_cast<uint32_t*>(bl);
    t->rf_nrange = static_cast<uint32_t*>(nr);
    return KAD_OK;
}

// Re-derive the status of at most RF_CAP listed nodes (main-run, side-run and patched nodes; vals: the patched
// nodes' new status bytes instead of their times) and rebuild only what they change: rf_nodes_kernel, then the
// line builders over its lists. ensure_marks must have run (the lists live in dlist). Async on s.
// The bucket holding node i (the last b with off[b] <= i; off = the B + 1 bucket offsets, off[B] = n): a galloping
// search from the proportional guess i * B / n, so a few cache lines of the 4 (B + 1)-byte array per node.
uint32_t bucket_of_node(const std::vector<uint32_t>& off, uint32_t n, uint32_t i) {
    const uint32_t B = (uint32_t)off.size() - 1;
    uint64_t lo, hi;  // off[lo] <= i < off[hi] (hi may be B + 1: past the end)
    uint64_t g = n ? std::min<uint64_t>((uint64_t)i * B / n, B - 1) : 0;
    if (off[g] <= i) {
        uint64_t step = 1;
        lo = g;
        while (lo + step <= B && off[lo + step] <= i) { lo += step; step <<= 1; }
        hi = std::min<uint64_t>(lo + step, B + 1);
    } else {
        uint64_t step = 1;
        hi = g;
        while (hi >= step && off[hi - step] > i) { hi -= step; step <<= 1; }
        lo = hi >= step ? hi - step : 0;
        if (off[lo] > i) return 0;  // (i below every offset: bucket 0)
    }
    while (hi - lo > 1) {
        const uint64_t mid = (lo + hi) >> 1;
        if (off[mid] <= i) lo = mid; else hi = mid;
    }
    return (uint32_t)std::min<uint64_t>(lo, B - 1);
}

// Every index the kernel derives from its inline arguments, checked on the host before the launch (at most
// RF_INLINE nodes, 16 runs and RF_HOFF offsets: a few hundred compares). The kernel's guards only record a
// violation (RF_ERR); this check refuses the launch, so a wrong argument never reaches the device.
int rf_check_inline(const RfCtx& C, const std::vector<uint32_t>& off, uint32_t n, uint32_t B) {
    auto bad = [](const char* what, uint32_t a, uint32_t b) {
        return set_err(KAD_ERR_INVALID, "small refresh: inline argument out of range (%s: %u, %u)", what, a, b);
    };
    if (C.ninl > RF_INLINE) return bad("ninl", C.ninl, RF_INLINE);
    for (uint32_t j = 1; j < C.ninl; j++)
        if (C.inl[j] <= C.inl[j - 1]) return bad("inl order", j, C.inl[j]);
    if (C.nhb == 0) return C.nhl ? bad("nhl without nhb", C.nhl, 0) : KAD_OK;
    if (C.nhb > RF_INLINE) return bad("nhb", C.nhb, RF_INLINE);
    if (off.size() != (size_t)B + 1) return bad("offsets", (uint32_t)off.size(), B);
    for (uint32_t u = 0; u < C.nhb; u++)
        if (C.hb[u] >= B || (u && C.hb[u] <= C.hb[u - 1])) return bad("hb", u, C.hb[u]);
    for (uint32_t j = 0; j < C.ninl; j++) {
        const uint32_t i = C.inl[j];
        if (i >= n) continue;
        const uint32_t u = C.inb[j] & 127u, p = C.inb[j] >> 8;
        if ((C.inb[j] & 0xFFu) >= C.nhb || u >= C.nhb) return bad("inb bucket", j, C.inb[j]);
        const uint32_t b = C.hb[u];
        if (!(off[b] <= i && i < off[b + 1])) return bad("inb not the node's bucket", j, b);
        if (p > 32 || (p && off[b] + p - 1 != i) || (!p && off[b + 1] - off[b] <= 32)) return bad("inb place", j, p);
    }
    if (C.nhl == 0) return C.nhr ? bad("nhr without nhl", C.nhr, 0) : KAD_OK;
    if (C.nhr == 0 || C.nhr > 16) return bad("nhr", C.nhr, 16);
    uint32_t lines = 0, next = 0, prev_end = 0;
    for (uint32_t r = 0; r < C.nhr; r++) {
        const uint32_t first = C.hr[3 * r], len = C.hr[3 * r + 1], o = C.hr[3 * r + 2];
        if (len == 0 || (uint64_t)first + len > B || (r && first <= prev_end)) return bad("run lines", r, first);
        const uint32_t o0 = first >= 3 ? first - 3 : 0u, o1 = std::min(B, first + len - 1 + 3) + 1;
        if (o != next || (uint64_t)o + (o1 - o0) > RF_HOFF) return bad("run offsets", r, o);
        for (uint32_t k = o0; k < o1; k++)
            if (C.hoff[o + (k - o0)] != off[k]) return bad("hoff", r, k);
        next = o + (o1 - o0);
        lines += len;
        prev_end = first + len;
    }
    if (lines != C.nhl) return bad("nhl", C.nhl, lines);
    return KAD_OK;
}

int small_refresh(kad_table* t, hipStream_t s, const uint32_t* mnode, uint32_t mc, const uint32_t* snode, uint32_t sc,
                  const uint32_t* pend, uint32_t np, const uint8_t* vals, int64_t now, const uint32_t* inl = nullptr,
                  uint32_t ninl = 0) {
    const uint32_t total = ninl ? ninl : mc + sc + np;
    if (total == 0) return KAD_OK;
    int rc;
    if ((rc = rf_ready(t))) return rc;
    const DevTable& d = t->d;
    const uint32_t B = d.B;
    const bool has8 = t->wl_mut || t->gl_mut, has16 = t->wl16_mut || t->gl16_mut, has32 = t->wl32_mut || t->gl32_mut;
    RfCtx C{};
    C.N = times_of(t);
    C.mnode = mnode; C.mc = mc;
    C.snode = snode; C.sc = sc;
    C.pend = pend; C.np = np;
    C.vals = vals;
    C.now = now;
    C.T = d;
    C.status = t->status_mut;
    C.dir = t->dir_mut;
    C.gcnt = t->gcnt_mut;
    C.blist = t->rf_blist;
    C.nrange = t->rf_nrange;
    C.ctr = t->rf_ctr;
    C.list[0] = B && has8 ? t->dlist : nullptr;
    C.list[1] = B && has16 ? t->dlist + (size_t)B : nullptr;
    C.list[2] = B && has32 ? t->dlist + 2ull * B : nullptr;
    C.list[3] = t->ncl_mut ? t->dlist + 3ull * B : nullptr;
    C.nback = t->ncl32_mut ? NC32_SLOTS - NC32_LEFT : NCL_SLOTS - NCL_LEFT;
    C.nfwd = t->ncl32_mut ? NC32_LEFT : NCL_LEFT;
    if (ninl) {  // the node ids as kernel arguments (host copies of the runs): no list load before the times
        C.ninl = std::min(ninl, RF_INLINE);
        std::memcpy(C.inl, inl, 4ull * C.ninl);
        std::sort(C.inl, C.inl + C.ninl);  // (the builders search them by node)
        C.ninl = (uint32_t)(std::unique(C.inl, C.inl + C.ninl) - C.inl);  // (each flip patches its bucket once)
        // their buckets from the host's copy of the bucket offsets (no locate on the device), and for the window
        // lines the lines to rebuild with the offsets their builders read (no directory load before the keys)
        if (B && t->h_off.size() == (size_t)B + 1) {
            uint32_t nh = 0, nb_[RF_INLINE];
            for (uint32_t j = 0; j < C.ninl; j++)
                if (C.inl[j] < d.n) C.hb[nh++] = nb_[j] = bucket_of_node(t->h_off, d.n, C.inl[j]);
            std::sort(C.hb, C.hb + nh);
            C.nhb = (uint32_t)(std::unique(C.hb, C.hb + nh) - C.hb);
            if (C.nhb == 0) C.hb[C.nhb++] = 0;  // (no valid node: one harmless recount)
            for (uint32_t j = 0; j < C.ninl; j++) {
                if (C.inl[j] >= d.n) continue;
                const uint32_t b = nb_[j], u = (uint32_t)(std::lower_bound(C.hb, C.hb + C.nhb, b) - C.hb);
                const uint32_t a = t->h_off[b], sz = t->h_off[b + 1] - a;
                C.inb[j] = u | (sz <= 32 ? (C.inl[j] - a + 1) << 8 : 0u);
            }
            // the union of [b-2, b+3] (ascending) as runs of consecutive lines, with the bucket offsets their
            // windows [l-3, l+3] read
            uint32_t nl = 0, nr = 0, no = 0;
            bool fits = true;
            for (uint32_t u = 0; u < C.nhb && fits; u++) {
                const uint32_t b = C.hb[u], lo = b > 2 ? b - 2 : 0u, hi = std::min(B - 1, b + 3);
                if (nr && lo <= C.hr[3 * (nr - 1)] + C.hr[3 * (nr - 1) + 1]) {  // extends the last run
                    uint32_t* R = C.hr + 3 * (nr - 1);
                    const uint32_t end = std::max(R[0] + R[1], hi + 1), add = end - (R[0] + R[1]);
                    const uint32_t o_end = std::min(B, end - 1 + 3) + 1;  // offsets [.., min(B, last + 3)]
                    const uint32_t have = R[2] + ((std::min(B, R[0] + R[1] - 1 + 3) + 1) - (R[0] >= 3 ? R[0] - 3 : 0u));
                    const uint32_t want = R[2] + (o_end - (R[0] >= 3 ? R[0] - 3 : 0u));
                    if (want > RF_HOFF) { fits = false; break; }
                    for (uint32_t o = have; o < want; o++) C.hoff[o] = t->h_off[(R[0] >= 3 ? R[0] - 3 : 0u) + (o - R[2])];
                    no = want;
                    R[1] += add;
                    nl += add;
                } else {
                    if (nr == 16) { fits = false; break; }
                    const uint32_t o0 = lo >= 3 ? lo - 3 : 0u, o1 = std::min(B, hi + 3) + 1;
                    if (no + (o1 - o0) > RF_HOFF) { fits = false; break; }
                    uint32_t* R = C.hr + 3 * nr++;
                    R[0] = lo;
                    R[1] = hi - lo + 1;
                    R[2] = no;
                    for (uint32_t o = o0; o < o1; o++) C.hoff[no++] = t->h_off[o];
                    nl += R[1];
                }
            }
            C.nhl = fits ? nl : 0;
            C.nhr = fits ? nr : 0;
        }
        if ((rc = rf_check_inline(C, t->h_off, d.n, B))) return rc;
    }
    // one block when it holds every listed node; the count <= 8 lines built by it when at most RF_FUSE_LINES can
    // be listed (6 per changed bucket) and no slot lines depend on them
    const bool single = total <= BLOCK;
    // (window-line builders derive the lines of nodes in device lists with one wave: at most 64 of them)
    int fuse = (!B || 6ull * total > RF_FUSE_LINES || t->sl_mut) ? 0 : t->wl_mut ? 1 : t->gl_mut ? 2 : 0;
    if (fuse == 1 && !C.nhb && total > 64) fuse = 0;
    // (the mirror of an earlier fused refresh's spin-timeout count: a copy that has not landed yet reads as the one
    // before it, so the demotion can come one refresh late, never wrongly)
    if (t->rf_spin_host && __atomic_load_n(t->rf_spin_host, __ATOMIC_RELAXED)) t->rf_no_fuse2 = true;
    if (fuse == 2 && t->rf_no_fuse2) fuse = 0;
    dim3 g1(std::min<uint32_t>((total + BLOCK - 1) / BLOCK, 64u));
    if (fuse) {  // (6 * total <= RF_FUSE_LINES: one block derives every node) + builder blocks, all lines in one round
        C.list[0] = nullptr;
        C.wl = t->wl_mut;
        C.ws = t->ws_mut;
        C.gl = t->gl_mut;
        C.fl = t->dlist;
        if (++t->rf_epoch == 0) t->rf_epoch = 1;  // ctr[RF_GO] starts at 0
        C.epoch = t->rf_epoch;
        // FUSE 1: block 0 + builder blocks of one line per wave; FUSE 2: 16 lines per block, block 0 included
        const uint32_t lines = C.nhl ? C.nhl : std::min<uint32_t>(B, 6u * total);
        // FUSE 1: the completion protocol only if some window may exceed RF_WCAP1 nodes (the largest W(2) of the
        // lines around the host's buckets, from its copy of the offsets; unknown without them)
        C.fin = 1;
        if (fuse == 1 && C.nhb && t->h_off.size() == (size_t)B + 1) {
            uint32_t wmax = 0;
            for (uint32_t u = 0; u < C.nhb; u++)
                for (uint32_t l = C.hb[u] > 2 ? C.hb[u] - 2 : 0u; l <= std::min(B - 1, C.hb[u] + 3); l++)
                    wmax = std::max(wmax, t->h_off[std::min(B, l + 3)] - t->h_off[l >= 3 ? l - 3 : 0u]);
            C.fin = wmax > RF_WCAP1;
        }
        g1 = fuse == 1 ? dim3(1 + (lines + BLOCK / 64 - 1) / (BLOCK / 64))
                       : dim3(std::max<uint32_t>(1, (lines + BLOCK / 16 - 1) / (BLOCK / 16)));
    }
#ifdef KAD_ABLATIONS
    if (const char* e = std::getenv("KAD_RF_ABL")) C.abl = (uint32_t)std::atoi(e);
#endif
    if (fuse == 1) hipLaunchKernelGGL((rf_nodes_kernel<true, 1>), g1, dim3(BLOCK), 0, s, C);
    else if (fuse == 2) {
        hipLaunchKernelGGL((rf_nodes_kernel<true, 2>), g1, dim3(BLOCK), 0, s, C);
        HIP_TRY(hipMemcpyAsync(t->rf_spin_host, t->rf_ctr + RF_SPIN, sizeof(uint32_t), hipMemcpyDeviceToHost, s));
    }
    else if (single) hipLaunchKernelGGL((rf_nodes_kernel<true, 0>), g1, dim3(BLOCK), 0, s, C);
    else hipLaunchKernelGGL((rf_nodes_kernel<false, 0>), g1, dim3(BLOCK), 0, s, C);
    HIP_TRY(hipGetLastError());
    // the builders over the lists; grids from the host's bound on each list
    auto grid = [&](uint64_t items) { return dim3((uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((items + BLOCK - 1) / BLOCK, 2048))); };
    const uint64_t u8 = std::min<uint64_t>(B, 6ull * total), u16 = std::min<uint64_t>(B, 8ull * total),
                   u32 = std::min<uint64_t>(B, 16ull * total), unc = d.nslots;
    const LineSel s8{C.list[0], t->rf_ctr + RF_L8}, s16{C.list[1], t->rf_ctr + RF_L16}, s32{C.list[2], t->rf_ctr + RF_L32};
    if (t->ncl_mut) {
        const LineSel snc{C.list[3], t->rf_ctr + RF_LNC};
        hipLaunchKernelGGL(ncl_build_kernel, grid(unc), dim3(BLOCK), 0, s, d.key, d.status, d.nrdx, d.nslots, d.n,
                           64 - d.nshift, t->ncl_mut, snc);
        if (t->ncl32_mut)
            hipLaunchKernelGGL(ncl32_build_kernel, grid(8 * unc), dim3(BLOCK), 0, s, d.key, d.status, d.nrdx, d.nslots,
                               d.n, 64 - d.nshift, t->ncl32_mut, snc);
    }
    if (B == 0) return KAD_OK;
    // the count 9..16 and 17..32 sets on the side streams (independent of the count <= 8 chain), joined back
    hipStream_t sB = s, sC = s;
    const bool fork = (has16 || has32) && side_streams(t) == KAD_OK;
    if (fork) {
        HIP_TRY(hipEventRecord(t->ev_fork, s));
        sB = t->ss[0];
        sC = t->ss[1];
        HIP_TRY(hipStreamWaitEvent(sB, t->ev_fork, 0));
        HIP_TRY(hipStreamWaitEvent(sC, t->ev_fork, 0));
    }
    if (t->wl16_mut)
        hipLaunchKernelGGL(wl16_build_kernel, grid(u16), dim3(BLOCK), 0, sB, d.key, d.status, d.dir, d.gcnt, B,
                           64 - d.rshift, d.rbase >> d.rshift, t->wl16_mut, s16);
    if (t->wl32_mut)
        hipLaunchKernelGGL(wl32_build_kernel, grid(u32), dim3(BLOCK), 0, sC, d.key, d.status, d.dir, d.gcnt, B,
                           64 - d.rshift, d.rbase >> d.rshift, t->wl32_mut, s32);
    if (t->gl32_mut)
        hipLaunchKernelGGL(gl32_build_kernel, grid(u32), dim3(BLOCK), 0, sC, d.key, d.status, d.dir, d.gcnt, d.fkey,
                           d.ftail, B, t->gl32_mut, s32);
    if (fuse) {
        // built by rf_nodes_kernel
    } else if (t->wl_mut) {  // a wave per listed line
        hipLaunchKernelGGL(wl_ws_wave_kernel, grid(64ull * u8), dim3(BLOCK), 0, s, d.key, d.status, d.dir, d.gcnt, B,
                           64 - d.rshift, d.rbase >> d.rshift, t->wl_mut, t->ws_mut, s8);
    }
    if (t->gl_mut && !fuse) {
        hipLaunchKernelGGL(gl_build_kernel, grid(u8), dim3(BLOCK), 0, s, d.key, d.status, d.dir, d.gcnt, d.fkey, d.ftail,
                           B, t->gl_mut, s8);
        if (t->sl_mut) {  // slot lines: transcoded from the general lines just rebuilt (the flagged buckets')
            hipLaunchKernelGGL(mark_sel_kernel, grid(u8), dim3(BLOCK), 0, s, s8, B, t->gdirty, (uint8_t)1);
            hipLaunchKernelGGL(sl_build_kernel, grid(d.slslots), dim3(BLOCK), 0, s, t->gl_mut, t->slb, d.slslots,
                               t->gdirty, d.rrdx, d.rslots, d.slshift - d.rshift, d.fkey, d.ftail, t->sl_mut);
            hipLaunchKernelGGL(mark_sel_kernel, grid(u8), dim3(BLOCK), 0, s, s8, B, t->gdirty, (uint8_t)0);
        }
    }
    if (t->gl16_mut) {  // on s: its slot copies share the gdirty flags with the count <= 8 slot lines
        hipLaunchKernelGGL(gl16_build_kernel, grid(u16), dim3(BLOCK), 0, s, d.key, d.status, d.dir, d.gcnt, d.fkey,
                           d.ftail, B, t->gl16_mut, s16);
        if (t->sl16_mut) {
            hipLaunchKernelGGL(mark_sel_kernel, grid(u16), dim3(BLOCK), 0, s, s16, B, t->gdirty, (uint8_t)1);
            hipLaunchKernelGGL(sl16_build_kernel, grid(8ull * d.slslots), dim3(BLOCK), 0, s, t->gl16_mut, t->slb,
                               d.slslots, t->gdirty, d.rrdx, d.rslots, d.slshift - d.rshift, d.fkey, d.ftail, t->sl16_mut);
            hipLaunchKernelGGL(mark_sel_kernel, grid(u16), dim3(BLOCK), 0, s, s16, B, t->gdirty, (uint8_t)0);
        }
    }
    if (fork) {
        HIP_TRY(hipEventRecord(t->ev_join[0], sB));
        HIP_TRY(hipEventRecord(t->ev_join[1], sC));
        HIP_TRY(hipStreamWaitEvent(s, t->ev_join[0], 0));
        HIP_TRY(hipStreamWaitEvent(s, t->ev_join[1], 0));
    }
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

// ---- isGood(now) deadlines, host side (see deadline_kernel) ----

int dl_alloc(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, std::max<size_t>(bytes, 16));
    if (e != hipSuccess) { *p = nullptr; return set_err(KAD_ERR_NOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(e)); }
    return KAD_OK;
}

// lower_bound of x in k[from, n) by galloping from the cursor (a refresh passes few deadlines).
uint32_t gallop_lower_bound(const std::vector<uint64_t>& k, uint32_t from, uint64_t x) {
    const uint32_t n = (uint32_t)k.size();
    if (from >= n || k[from] >= x) return from;
    uint32_t lo = from, step = 1;  // k[lo] < x
    while (lo + step < n && k[lo + step] < x) {
        lo += step;
        step <<= 1;
    }
    const uint32_t hi = std::min<uint64_t>(n, (uint64_t)lo + step);
    return (uint32_t)(std::lower_bound(k.begin() + lo + 1, k.begin() + hi, x) - k.begin());
}

// Main run of every node's deadline from the device times (radix sort by key), its keys copied to the host
// (synchronous on s), the side run emptied, the cursors at the first deadline >= nowk (everything before it
// counts as passed).
int dl_build_main(kad_table* t, hipStream_t s, uint64_t nowk) {
    Deadlines& D = t->dl;
    const uint32_t n = t->d.n;
    int rc;
    if (D.mcap < n) {
        if (D.km) { (void)hipFree(D.km); D.km = nullptr; }
        if (D.kn) { (void)hipFree(D.kn); D.kn = nullptr; }
        if (D.tmp) { (void)hipFree(D.tmp); D.tmp = nullptr; D.tmp_bytes = 0; }
        D.mcap = 0;
        if ((rc = dl_alloc((void**)&D.km, 8ull * n)) || (rc = dl_alloc((void**)&D.kn, 4ull * n))) return rc;
        size_t cub = 0;
        HIP_TRY(hipcub::DeviceRadixSort::SortPairs(nullptr, cub, (const uint64_t*)nullptr, (uint64_t*)nullptr,
                                                   (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n, 0, 64, s));
        const size_t kb = (8ull * n + 255) & ~255ull, nb = (4ull * n + 255) & ~255ull;
        if ((rc = dl_alloc(&D.tmp, kb + nb + cub))) return rc;
        D.tmp_bytes = kb + nb + cub;
        D.mcap = n;
    }
    try {
        D.hkm.resize(n);
        D.hkn.resize(n);
    } catch (...) {
        return set_err(KAD_ERR_NOMEM, "deadline keys: out of host memory");
    }
    const size_t kb = (8ull * n + 255) & ~255ull, nb = (4ull * n + 255) & ~255ull;
    uint64_t* tk = static_cast<uint64_t*>(D.tmp);
    uint32_t* tn = reinterpret_cast<uint32_t*>(static_cast<uint8_t*>(D.tmp) + kb);
    void* ct = static_cast<uint8_t*>(D.tmp) + kb + nb;
    size_t cb = D.tmp_bytes - kb - nb;
    hipLaunchKernelGGL(deadline_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, s, times_of(t), n, tk, tn);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipcub::DeviceRadixSort::SortPairs(ct, cb, tk, D.km, tn, D.kn, (int)n, 0, 64, s));
    HIP_TRY(hipMemcpyAsync(D.hkm.data(), D.km, 8ull * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(D.hkn.data(), D.kn, 4ull * n, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    D.nm = n;
    D.ns = 0;
    D.hks.clear();
    D.hsn.clear();
    D.cm = (uint32_t)(std::lower_bound(D.hkm.begin(), D.hkm.end(), nowk) - D.hkm.begin());
    D.cs = 0;
    D.set_next();
    return KAD_OK;
}

// patch_times on the deadline runs (synchronous; the device times are already updated): the patched nodes
// join the pending list (re-derived at the next refresh, whatever `now`), their new deadlines the side run.
// Side entries below last_now are dropped (passed; the pending list covers them). A side run grown past an
// eighth of the main run is folded into a rebuilt main run.
int dl_patch(kad_table* t, uint32_t m, const uint32_t* nodes, const int64_t* time_ns, const int64_t* reply_ns,
             const uint8_t* expired) {
    Deadlines& D = t->dl;
    if (!D.valid) return KAD_OK;
    if ((uint64_t)D.hpend.size() + m > t->d.n) {  // more patched than nodes: a full refresh is cheaper
        D.invalidate();
        return KAD_OK;
    }
    const uint64_t lk = dl_key(D.last_now);
    auto sat = [](int64_t a, int64_t b) { return a > INT64_MAX - b ? INT64_MAX : a + b; };
    std::vector<std::pair<uint64_t, uint32_t>> add;
    add.reserve(m);
    for (uint32_t j = 0; j < m; j++) {
        D.hpend.push_back(nodes[j]);
        const uint64_t k = expired[j] ? DL_NEVER
                                      : dl_key(std::min(sat(time_ns[j], NODE_EXPIRE_NS), sat(reply_ns[j], NODE_GOOD_NS)));
        if (k >= lk) add.emplace_back(k, nodes[j]);
    }
    std::sort(add.begin(), add.end());
    std::vector<uint64_t> nk;
    std::vector<uint32_t> nn;
    nk.reserve(D.hks.size() + add.size());
    nn.reserve(D.hks.size() + add.size());
    size_t x = 0, y = 0;
    while (x < D.hks.size() || y < add.size()) {
        const bool take_old = y == add.size() || (x < D.hks.size() && D.hks[x] <= add[y].first);
        const uint64_t k = take_old ? D.hks[x] : add[y].first;
        const uint32_t v = take_old ? D.hsn[x] : add[y].second;
        if (take_old) x++; else y++;
        if (k >= lk) { nk.push_back(k); nn.push_back(v); }
    }
    D.hks.swap(nk);
    D.hsn.swap(nn);
    int rc;
    // (re)allocate a pair of device arrays to hold `need` entries; on failure both are freed and cap is 0
    auto grow = [&](void** a, size_t ea, void** b, size_t eb, uint32_t& cap, size_t need) -> int {
        if (cap >= need) return KAD_OK;
        const size_t c = std::max<size_t>(need + need / 2, 4096);
        for (void** p : {a, b})
            if (p && *p) { (void)hipFree(*p); *p = nullptr; }
        cap = 0;
        int r = dl_alloc(a, c * ea);
        if (r == KAD_OK && b) r = dl_alloc(b, c * eb);
        if (r != KAD_OK) {
            for (void** p : {a, b})
                if (p && *p) { (void)hipFree(*p); *p = nullptr; }
            return r;
        }
        cap = (uint32_t)c;
        return KAD_OK;
    };
    if ((rc = grow((void**)&D.pend, 4, nullptr, 0, D.pcap, D.hpend.size()))) return rc;
    HIP_TRY(hipMemcpy(D.pend, D.hpend.data(), 4ull * D.hpend.size(), hipMemcpyHostToDevice));
    D.np = (uint32_t)D.hpend.size();
    if (D.hks.size() > D.nm / 8 + 65536) {  // fold the side run into a rebuilt main run
        if ((rc = dl_build_main(t, nullptr, lk))) return rc;
        HIP_TRY(hipDeviceSynchronize());
        return KAD_OK;
    }
    if ((rc = grow((void**)&D.ks, 8, (void**)&D.sn, 4, D.scap, D.hks.size()))) return rc;
    if (!D.hks.empty()) {
        HIP_TRY(hipMemcpy(D.ks, D.hks.data(), 8ull * D.hks.size(), hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(D.sn, D.hsn.data(), 4ull * D.hsn.size(), hipMemcpyHostToDevice));
    }
    D.ns = (uint32_t)D.hks.size();
    D.cs = 0;  // every side entry is unpassed
    D.set_next();
    return KAD_OK;
}

// ---- line sets built on first use --------------------------------------------------------------------------
// kad_table_create builds the count <= 8 lines (the headline path) and, with KAD_TABLE_EAGER, every other set;
// otherwise a set is built by the first query that needs it (ensure_lines), which synchronises the device once.
int build_wl16(kad_table* t) {
    DevTable& d = t->d;
    if (!(d.flags & TF_WL) || t->wl16_mut) return KAD_OK;
    uint32_t* lp = nullptr;
    std::vector<void*> fresh;
    uint64_t fb = 0;
    int rc;
    if ((rc = dev_upload(&lp, nullptr, (size_t)WL16_STRIDE * d.B, fresh, fb))) return rc;
    hipLaunchKernelGGL(wl16_build_kernel, dim3(grid_for(d.B)), dim3(BLOCK), 0, build_stream(t), d.key, d.status, d.dir, d.gcnt, d.B,
                       64 - d.rshift, d.rbase >> d.rshift, lp, LineSel{});
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(build_stream(t)) != hipSuccess) {
        (void)hipFree(lp);
        return set_err(KAD_ERR_HIP, "window-line (16) build failed");
    }
    t->owned.push_back(lp); t->bytes += fb;
    d.wl16 = reinterpret_cast<const uint4*>(lp); t->wl16_mut = lp; d.flags |= TF_WL16;
    return KAD_OK;
}

int build_wl32(kad_table* t) {
    DevTable& d = t->d;
    if (!(d.flags & TF_WL) || t->wl32_mut || 64 - d.rshift > 44) return KAD_OK;  // 20-bit in-bucket keys
    uint32_t* lp = nullptr;
    std::vector<void*> fresh;
    uint64_t fb = 0;
    int rc;
    if ((rc = dev_upload(&lp, nullptr, (size_t)WL32_STRIDE * d.B, fresh, fb))) return rc;
    hipLaunchKernelGGL(wl32_build_kernel, dim3(grid_for(d.B)), dim3(BLOCK), 0, build_stream(t), d.key, d.status, d.dir, d.gcnt, d.B,
                       64 - d.rshift, d.rbase >> d.rshift, lp, LineSel{});
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(build_stream(t)) != hipSuccess) {
        (void)hipFree(lp);
        return set_err(KAD_ERR_HIP, "window-line (32) build failed");
    }
    t->owned.push_back(lp); t->bytes += fb;
    d.wl32 = reinterpret_cast<const uint4*>(lp); t->wl32_mut = lp; d.flags |= TF_WL32;
    return KAD_OK;
}

int build_ncl(kad_table* t) {
    DevTable& d = t->d;
    if (!(t->flags & KAD_TABLE_SORTED) || !d.nrdx || d.n == 0 || t->ncl_mut) return KAD_OK;
    uint32_t* lp = nullptr;
    std::vector<void*> fresh;
    uint64_t fb = 0;
    int rc;
    if ((rc = dev_upload(&lp, nullptr, (size_t)(NCL_STRIDE + NCL2_DWORDS) * d.nslots, fresh, fb))) return rc;
    hipLaunchKernelGGL(ncl_build_kernel, dim3(grid_for(d.nslots)), dim3(BLOCK), 0, build_stream(t), d.key, d.status, d.nrdx, d.nslots,
                       d.n, 64 - d.nshift, lp, LineSel{});
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(build_stream(t)) != hipSuccess) {
        (void)hipFree(lp);
        return set_err(KAD_ERR_HIP, "NodeCache line build failed");
    }
    t->owned.push_back(lp); t->bytes += fb;
    d.ncl = reinterpret_cast<const uint4*>(lp); t->ncl_mut = lp; d.flags |= TF_NCL;
    return KAD_OK;
}

int build_ncl32(kad_table* t) {
    DevTable& d = t->d;
    if (!(t->flags & KAD_TABLE_SORTED) || !d.nrdx || d.n == 0 || t->ncl32_mut) return KAD_OK;
    uint32_t* lp = nullptr;
    std::vector<void*> fresh;
    uint64_t fb = 0;
    int rc;
    if ((rc = dev_upload(&lp, nullptr, (size_t)NC32_STRIDE * d.nslots, fresh, fb))) return rc;
    hipLaunchKernelGGL(ncl32_build_kernel, dim3(grid_for(8ull * d.nslots)), dim3(BLOCK), 0, build_stream(t), d.key, d.status, d.nrdx,
                       d.nslots, d.n, 64 - d.nshift, lp, LineSel{});
    if (hipGetLastError() != hipSuccess || hipStreamSynchronize(build_stream(t)) != hipSuccess) {
        (void)hipFree(lp);
        return set_err(KAD_ERR_HIP, "NodeCache line (32) build failed");
    }
    t->owned.push_back(lp); t->bytes += fb;
    d.ncl32 = reinterpret_cast<const uint4*>(lp); t->ncl32_mut = lp; d.flags |= TF_NCL32;
    return KAD_OK;
}

constexpr uint32_t LS_WL16 = KAD_LINES_RT16, LS_WL32 = KAD_LINES_RT32, LS_NCL = KAD_LINES_NC16,
                   LS_NCL32 = KAD_LINES_NC32, LS_ALL = KAD_LINES_ALL;

// The line sets `need` (KAD_LINES_*) of a table, built now if they are not yet (the count 9..16 sets bring the
// 17..32 ones, their fallback). Nothing is built inside a stream capture (no allocation there): the kernels
// answer exactly without the set, on their slower paths. An allocation failure leaves the set unbuilt (the
// same fallbacks), any other failure is returned.
int ensure_lines(const kad_table* ct, uint32_t need, hipStream_t s) {
    kad_table* t = const_cast<kad_table*>(ct);  // the sets are caches of the table's state
    if (need & LS_WL16) need |= LS_WL32;
    if (need & LS_NCL32) need |= LS_NCL;  // the refresh rebuilds the 512-byte lines along with the 256-byte ones
    if (!(need & ~t->ls_done.load(std::memory_order_acquire))) return KAD_OK;
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (s) {  // the null stream is never captured (and the query would fail with the runtime's last error set)
        if (hipStreamIsCapturing(s, &cs) != hipSuccess) (void)hipGetLastError();
        else if (cs != hipStreamCaptureStatusNone) return KAD_OK;
    }
    std::lock_guard<std::mutex> lk(t->ls_mu);
    need &= ~t->ls_done.load(std::memory_order_relaxed);
    if (!need) return KAD_OK;
    DeviceGuard g(t->device);
    // built from the current status: after the last asynchronous refresh (every other change is synchronous);
    // the table's own streams only, never the whole device
    if (t->mut_async) HIP_TRY(hipEventSynchronize(t->mut_ev));
    for (hipStream_t x : t->ss)
        if (x) HIP_TRY(hipStreamSynchronize(x));
    const uint32_t bits[4] = {LS_WL32, LS_WL16, LS_NCL, LS_NCL32};
    int (*uni[4])(kad_table*) = {build_wl32, build_wl16, build_ncl, build_ncl32};
    int (*gen[4])(kad_table*) = {build_gl32, build_gl16, build_ncl, build_ncl32};
    const bool general = !(t->d.flags & TF_WL);
    int rc = KAD_OK;
    for (int k = 0; k < 4 && rc == KAD_OK; k++) {
        if (!(need & bits[k])) continue;
        const uint64_t b0 = t->bytes;
        const auto a = std::chrono::steady_clock::now();
        rc = (general ? gen[k] : uni[k])(t);
        if (rc == KAD_ERR_NOMEM) rc = KAD_OK;  // unbuilt: the fallbacks answer
        t->ls_ms[k] = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - a).count();
        t->ls_bytes[k] = t->bytes - b0;
        t->ls_done.fetch_or(bits[k], std::memory_order_release);
    }
    drop_marks(t);  // the incremental-refresh flags are re-allocated with the new sets'
    return rc;
}

// After a structural change (kad_table_apply, kad_nc_apply): a set the table still has stays built; the others
// may be built again on first use.
void reset_line_sets(kad_table* t) {
    uint32_t done = 0;
    if (t->wl16_mut || t->gl16_mut) done |= LS_WL16;
    if (t->wl32_mut || t->gl32_mut) done |= LS_WL32;
    if (t->ncl_mut) done |= LS_NCL;
    if (t->ncl32_mut) done |= LS_NCL32;
    t->ls_done.store(done, std::memory_order_release);
}

int check_count(uint32_t count) {
    if (count > KAD_MAX_COUNT) return set_err(KAD_ERR_UNSUPPORTED, "count %u > KAD_MAX_COUNT (%u)", count, KAD_MAX_COUNT);
    return KAD_OK;
}

// KAD_RT_KERNEL=lane forces the lane-per-query kernel where the window-line kernel would run, =wl the
// 128-byte window lines where the short ones would (A/B timing, tools/ab_bench.py); read per call so one
// process can time both.
template <int K>
int launch_rt(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out, uint8_t* cnt,
              hipStream_t s) {
    const DevTable& d = t->d;
    const char* ev = std::getenv("KAD_RT_KERNEL");
    if (K == 8 && (d.flags & TF_WS) && !(ev && (std::strcmp(ev, "lane") == 0 || std::strcmp(ev, "wl") == 0 ||
                                                 std::strncmp(ev, "wl_abl", 6) == 0))) {
#ifdef KAD_ABLATIONS
        if (ev && std::strcmp(ev, "ws_abl1") == 0)
            hipLaunchKernelGGL(rt_ws_kernel<1>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else if (ev && std::strcmp(ev, "ws_abl2") == 0)
            hipLaunchKernelGGL(rt_ws_kernel<2>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else if (ev && std::strcmp(ev, "ws_abl3") == 0)
            hipLaunchKernelGGL(rt_ws_kernel<3>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else if (ev && std::strcmp(ev, "ws_abl5") == 0)
            hipLaunchKernelGGL(rt_ws_kernel<5>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else if (ev && std::strcmp(ev, "ws_stats") == 0)
            hipLaunchKernelGGL(rt_ws_kernel<4>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else
#endif
        if (ev && std::strcmp(ev, "ws_plain") == 0)  // A/B: the streams with the plain policy
            hipLaunchKernelGGL(rt_ws_kernel<0>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else if (ev && std::strcmp(ev, "ws_nocr") == 0)  // A/B: rows stored by their lanes (round-3 form before CR)
            hipLaunchKernelGGL((rt_ws_kernel<0, true>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out,
                               cnt);
        else  // rows through LDS as coalesced runs: 31.85 -> 31.0 us per 1M (profiles/r03/ab_ws_cr/)
            hipLaunchKernelGGL((rt_ws_kernel<0, true, true>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count,
                               out, cnt);
    } else if (K == 8 && (d.flags & TF_WL) && !(ev && std::strcmp(ev, "lane") == 0)) {
#ifdef KAD_ABLATIONS  // timing ablations with WRONG results: only in the tools build (Makefile target `ablations`)
        if (ev && std::strcmp(ev, "wl_abl1") == 0)
            hipLaunchKernelGGL(rt_wl_kernel<1>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else if (ev && std::strcmp(ev, "wl_abl2") == 0)
            hipLaunchKernelGGL(rt_wl_kernel<2>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else
#endif
            hipLaunchKernelGGL(rt_wl_kernel<0>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    } else if (K == 16 && (d.flags & TF_WL16) && !(ev && std::strcmp(ev, "lane") == 0)) {
#ifdef KAD_ABLATIONS
        if (ev && std::strcmp(ev, "wl16_abl1") == 0)
            hipLaunchKernelGGL(rt_wl16_kernel<1>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else if (ev && std::strcmp(ev, "wl16_stats") == 0)
            hipLaunchKernelGGL(rt_wl16_kernel<3>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else
#endif
            hipLaunchKernelGGL(rt_wl16_kernel<0>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    } else if (K == 32 && (d.flags & TF_WL32) && !(ev && std::strcmp(ev, "lane") == 0)) {
        // the quad form ranks faster for long rows stored as 16-byte pieces (counts 28 and 32), the one-lane
        // form for the others (tools/ab_kernels.py, profiles/r03/ab_wl32.json)
        // the quad form with its per-quad LDS row store is faster for rows of 24, 28 and 32 entries (16-byte
        // pieces), the one-lane form for the others (tools/ab_kernels.py, profiles/r03/ab_wl32_qs.json)
        const bool quad = count >= 24 && (count & 3u) == 0;
#ifdef KAD_ABLATIONS
        if (ev && std::strcmp(ev, "wl32qs_abl1") == 0) {  // no ranking: the kernel's memory floor (results wrong)
            hipLaunchKernelGGL((rt_wl32q_kernel<1, true>), dim3(grid_for(4ull * q)), dim3(BLOCK), 0, s, d, targets, q,
                               count, out, cnt);
        } else
#endif
        if (ev && std::strcmp(ev, "wl32quad") == 0)  // A/B: the quad form with the register / block-staged stores
            hipLaunchKernelGGL((rt_wl32q_kernel<0, false>), dim3(grid_for(4ull * q)), dim3(BLOCK), 0, s, d, targets, q,
                               count, out, cnt);
        else if ((!quad && !(ev && std::strcmp(ev, "wl32qs") == 0)) || (ev && std::strcmp(ev, "wl32lane") == 0))
            hipLaunchKernelGGL(rt_wl32_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        else
            hipLaunchKernelGGL((rt_wl32q_kernel<0, true>), dim3(grid_for(4ull * q)), dim3(BLOCK), 0, s, d, targets, q,
                               count, out, cnt);
    } else if (K == 8 && (d.flags & TF_SL) && !(ev && (std::strcmp(ev, "lane") == 0 || std::strcmp(ev, "gl") == 0 ||
                                                        std::strcmp(ev, "sl_abl1") == 0))) {
        hipLaunchKernelGGL(rt_sl_kernel<0>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
#ifdef KAD_ABLATIONS
    } else if (K == 8 && (d.flags & TF_SL) && ev && std::strcmp(ev, "sl_abl1") == 0) {
        hipLaunchKernelGGL(rt_sl_kernel<1>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
#endif
    } else if (K == 8 && (d.flags & TF_GL) && !(ev && std::strcmp(ev, "lane") == 0)) {
        hipLaunchKernelGGL(rt_gl_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    } else if (K == 16 && (d.flags & TF_SL16) && !(ev && (std::strcmp(ev, "lane") == 0 || std::strcmp(ev, "gl32") == 0 ||
                                                          std::strcmp(ev, "gl") == 0))) {
        hipLaunchKernelGGL(rt_sl16_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    } else if (K == 16 && (d.flags & TF_GL16) && !(ev && (std::strcmp(ev, "lane") == 0 || std::strcmp(ev, "gl32") == 0))) {
        hipLaunchKernelGGL(rt_gl16_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    } else if (K == 32 && (d.flags & TF_GL32) && count >= 24 && (count & 3u) == 0 &&
               !(ev && (std::strcmp(ev, "lane") == 0 || std::strcmp(ev, "gl32lane") == 0))) {
        // four lanes per query for rows of 24, 28 and 32 entries (as the uniform lines' rt_wl32q_kernel)
        void (*kq)(DevTable, const uint8_t*, uint32_t, uint32_t, uint32_t*, uint8_t*) = rt_gl32q_kernel<0>;
#ifdef KAD_ABLATIONS
        if (ev && std::strcmp(ev, "gl32q_abl1") == 0) kq = rt_gl32q_kernel<1>;
        if (ev && std::strcmp(ev, "gl32q_stats") == 0) kq = rt_gl32q_kernel<3>;
#endif
        hipLaunchKernelGGL(kq, dim3(grid_for(4ull * q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    } else if (K > 8 && (d.flags & TF_GL32) && !(ev && std::strcmp(ev, "lane") == 0)) {
        hipLaunchKernelGGL(rt_gl32_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
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
    int rc = KAD_OK;
    if (count > 8 && count <= KAD_MAX_COUNT && (rc = ensure_lines(t, count <= 16 ? LS_WL16 : LS_WL32, s))) return rc;
    if (count > KAD_MAX_COUNT) {
        if ((uint64_t)q > 0xFFFFFFFFull / 4 * BLOCK / 64) return set_err(KAD_ERR_INVALID, "batch too large");
        hipLaunchKernelGGL(rt_wave_kernel, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0, s, t->d, t->d,
                           nullptr, targets, q, count, out, cnt);
    } else if (count <= 8) rc = launch_rt<8>(t, targets, q, count, out, cnt, s);
    else if (count <= 16) rc = launch_rt<16>(t, targets, q, count, out, cnt, s);
    else rc = launch_rt<32>(t, targets, q, count, out, cnt, s);
    if (rc) return rc;
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

}  // namespace

extern "C" {

const char* kad_last_error(void) { return g_err.c_str(); }
}  // extern "C"

// Internal, for the other translation units of libkadgpu.so (kad_swarm.hip): the thread-local
// error of kad_last_error() and the gfx950 check.
namespace kadgpu_internal {
int set_error(int code, const char* msg) { return set_err(code, "%s", msg); }
bool device_ok(int dev) { return is_gfx950(dev); }
}  // namespace kadgpu_internal

extern "C" {
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
    if (n_buckets) {
        t->h_off.assign(bucket_offset, bucket_offset + n_buckets + 1);
        t->h_first.assign(bucket_first, bucket_first + 20ull * n_buckets);
    }
    std::vector<uint64_t>().swap(key);
    std::vector<uint32_t>().swap(tail);

    // bucket directory
    if (n_buckets) {
        std::vector<uint2> dir(n_buckets + 1);
        std::vector<uint32_t> cnt(n_buckets + 1, 0), dmask(any_dup ? n_buckets : 0);
        for (uint32_t b = 0; b <= n_buckets; b++) {
            dir[b].x = bucket_offset[b];
            dir[b].y = 0;
            if (b < n_buckets) {
                const uint32_t j0 = bucket_offset[b], j1 = bucket_offset[b + 1];
                if (j1 - j0 > 32) dir[b].x |= WIDE;
                for (uint32_t j = j0; j < j1; j++) {
                    const uint32_t gb = status[j] & KAD_STATUS_GOOD;
                    cnt[b] += gb;
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
        uint2* ddir; uint64_t* dfk; uint32_t *dft, *drdx, *ddm = nullptr;
        if ((rc = dev_upload(&ddir, dir.data(), n_buckets + 1, t->owned, t->bytes)) ||
            (any_dup && (rc = dev_upload(&ddm, dmask.data(), n_buckets, t->owned, t->bytes))) ||
            (rc = dev_upload(&dfk, fkey.data(), n_buckets, t->owned, t->bytes)) ||
            (rc = dev_upload(&dft, ftail.data(), 3ull * n_buckets, t->owned, t->bytes)) ||
            (rc = dev_upload(&drdx, rdx.data(), rdx.size(), t->owned, t->bytes)) ||
            (rc = dev_upload(&t->gcnt_mut, cnt.data(), n_buckets + 1, t->owned, t->bytes))) {
            delete t;
            return rc;
        }
        d.dir = ddir; t->dir_mut = ddir; d.gcnt = t->gcnt_mut; d.dmask = ddm; d.fkey = dfk; d.ftail = dft; d.rrdx = drdx;
        d.rbase = r.base; d.rshift = r.shift; d.rslots = r.slots; t->rbits = r.bits;
        // window lines (rt_wl_kernel): direct-mapped, uniform depth 1..43, every node inside its
        // bucket's dyadic range
        if (direct && depth >= 1 && depth <= 43) {
            bool inside = true;
            const uint64_t pre0 = r.base >> r.shift;
            for (uint32_t b = 0; b < n_buckets && inside; b++)
                for (uint32_t j = bucket_offset[b]; j < bucket_offset[b + 1] && inside; j++)
                    inside = (id_hi(ids + 20ull * j) >> r.shift) == pre0 + b;
            if (inside) {
                uint32_t *lp, *lps;
                if ((rc = dev_upload(&lp, nullptr, 32ull * n_buckets, t->owned, t->bytes)) ||
                    (rc = dev_upload(&lps, nullptr, 16ull * n_buckets, t->owned, t->bytes))) {
                    delete t;
                    return rc;
                }
                hipLaunchKernelGGL(wl_build_kernel<true>, dim3(grid_for(n_buckets)), dim3(BLOCK), 0, 0, d.key, d.status,
                                   d.dir, d.gcnt, n_buckets, depth, pre0, lp, lps, LineSel{});
                if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
                    delete t;
                    return set_err(KAD_ERR_HIP, "window-line build failed");
                }
                d.wl = reinterpret_cast<const uint4*>(lp);
                t->wl_mut = lp;
                d.flags |= TF_WL;
                d.ws = reinterpret_cast<const uint4*>(lps);
                t->ws_mut = lps;
                d.flags |= TF_WS;
            }
        }
    }
    // general window lines for every other bucket shape (split policy, per-peer tables, shards)
    if (n_buckets && !(d.flags & TF_WL) && (rc = setup_general_lines(t))) {
        delete t;
        return rc;
    }
    // NodeCache radix
    if ((flags & KAD_TABLE_SORTED) && n_nodes) {
        uint32_t tb = 1, tb_max = 23;
        if (const char* e = std::getenv("KAD_NC_RADIX_BITS")) tb_max = (uint32_t)std::max(1, std::min(23, std::atoi(e)));
        while ((1u << tb) < n_nodes && tb < tb_max) tb++;
        const Radix r = choose_radix(id_hi(ids), id_hi(ids + 20ull * (n_nodes - 1)), tb);
        std::vector<uint32_t> rdx = build_radix(r, n_nodes, ids, false);
        uint32_t* dn;
        if ((rc = dev_upload(&dn, rdx.data(), rdx.size(), t->owned, t->bytes))) { delete t; return rc; }
        d.nrdx = dn; d.nbase = r.base; d.nshift = r.shift; d.nslots = r.slots; t->nbits = r.bits;
    }
    // the line sets of counts above 8 and of NodeCache queries: now (KAD_TABLE_EAGER) or on first use
    if ((flags & KAD_TABLE_EAGER) && (rc = ensure_lines(t, LS_ALL, nullptr))) {
        delete t;
        return rc;
    }
    *out = t;
    return KAD_OK;
}

int kad_table_destroy(kad_table* t) {
    if (!t) return KAD_OK;
    DeviceGuard g(t->device);
    (void)svc_quiesce(t);  // the resident service ends before the device-wide synchronise
    (void)hipDeviceSynchronize();
    delete t;
    return KAD_OK;
}

int kad_table_get_info(const kad_table* t, kad_table_info* out) {
    if (!t || !out) return set_err(KAD_ERR_INVALID, "NULL argument");
    out->n_nodes = t->d.n;
    out->n_buckets = t->d.B;
    out->index_base = t->d.index_base;
    out->flags = t->flags | ((t->d.flags & TF_WL) ? KAD_INFO_WINDOW_LINES : 0u) |
                 ((t->d.flags & TF_GL) ? KAD_INFO_GENERAL_LINES : 0u) | ((t->d.flags & TF_GL32) ? KAD_INFO_GENERAL_LINES32 : 0u) |
                 ((t->d.flags & TF_GL16) ? KAD_INFO_GENERAL_LINES16 : 0u) |
                 ((t->d.flags & TF_SL16) ? KAD_INFO_SLOT_LINES16 : 0u) |
                 ((t->d.flags & TF_WS) ? KAD_INFO_SHORT_LINES : 0u) |
                 ((t->d.flags & TF_NCL32) ? KAD_INFO_NODECACHE_LINES32 : 0u) |
                 ((t->d.flags & TF_SL) ? KAD_INFO_SLOT_LINES : 0u);
    out->device = t->device;
    out->rt_radix_bits = t->rbits;
    out->nc_radix_bits = t->nbits;
    out->device_bytes = t->bytes;
    out->n_good = 0;
    if (t->d.B) {  // the sum of the per-bucket good counts
        DeviceGuard g(t->device);
        if (t->mut_async) HIP_TRY(hipEventSynchronize(t->mut_ev));  // after the last asynchronous refresh
        uint32_t* acc = nullptr;
        HIP_TRY(hipMalloc(&acc, sizeof(uint32_t)));
        uint32_t last = 0;
        hipError_t e = hipMemset(acc, 0, sizeof(uint32_t));
        if (e == hipSuccess) {
            hipLaunchKernelGGL(sum_u32_kernel, dim3(std::min(grid_for(t->d.B), 1024u)), dim3(BLOCK), 0, 0, t->d.gcnt,
                               t->d.B, acc);
            e = hipGetLastError();
        }
        if (e == hipSuccess) e = hipMemcpy(&last, acc, sizeof last, hipMemcpyDeviceToHost);  // after the table's refreshes
        (void)hipFree(acc);
        if (e != hipSuccess) return set_err(KAD_ERR_HIP, "good count: %s", hipGetErrorString(e));
        out->n_good = last;
    }
    return KAD_OK;
}

int kad_table_prepare(kad_table* t, uint32_t sets) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (sets & ~KAD_LINES_ALL) return set_err(KAD_ERR_INVALID, "unknown line sets 0x%x", sets);
    DeviceGuard g(t->device);
    if (int rc = svc_quiesce(t)) return rc;
    return ensure_lines(t, sets, nullptr);
}

int kad_table_line_sets(const kad_table* t, uint32_t* built, uint64_t* bytes, float* build_ms) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    const uint32_t bits[4] = {LS_WL32, LS_WL16, LS_NCL, LS_NCL32};
    if (built) {
        *built = ((t->wl16_mut || t->gl16_mut) ? LS_WL16 : 0u) | ((t->wl32_mut || t->gl32_mut) ? LS_WL32 : 0u) |
                 (t->ncl_mut ? LS_NCL : 0u) | (t->ncl32_mut ? LS_NCL32 : 0u);
    }
    for (int k = 0; k < 4; k++) {  // in the order of the KAD_LINES_* bits
        const int j = bits[k] == LS_WL16 ? 0 : bits[k] == LS_WL32 ? 1 : bits[k] == LS_NCL ? 2 : 3;
        if (bytes) bytes[j] = t->ls_bytes[k];
        if (build_ms) build_ms[j] = t->ls_ms[k];
    }
    return KAD_OK;
}

int kad_table_update_status(kad_table* t, const uint8_t* status) {
    if (!t || (!status && t->d.n)) return set_err(KAD_ERR_INVALID, "NULL argument");
    return kad_table_patch_status(t, t->d.n, nullptr, status);
}

int kad_table_patch_status(kad_table* t, uint32_t m, const uint32_t* nodes, const uint8_t* status) {
    if (!t || (m && !status)) return set_err(KAD_ERR_INVALID, "NULL argument");
    if (!nodes && m != t->d.n) return set_err(KAD_ERR_INVALID, "nodes NULL needs m = n_nodes");
    if (nodes)
        for (uint32_t j = 0; j < m; j++)
            if (nodes[j] >= t->d.n) return set_err(KAD_ERR_INVALID, "node %u out of range (n=%u)", nodes[j], t->d.n);
    DeviceGuard g(t->device);
    int rc;
    if ((rc = svc_quiesce(t))) return rc;
    if ((rc = ensure_marks(t))) return rc;
    t->dl.invalidate();  // status bytes set directly: the next refresh_status re-derives every node from its times
    if (m) {
        const size_t ib = nodes ? ((4ull * m + 15) & ~15ull) : 0;
        if ((rc = stage_reserve(t, ib + m))) return rc;
        uint8_t* st = static_cast<uint8_t*>(t->stage);
        if (nodes) HIP_TRY(hipMemcpy(st, nodes, 4ull * m, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy(st + ib, status, m, hipMemcpyHostToDevice));
        if (nodes && m <= RF_CAP) {  // a few nodes: the small refresh (no pass over the buckets or the lines)
            if ((rc = small_refresh(t, nullptr, nullptr, 0, nullptr, 0, reinterpret_cast<const uint32_t*>(st), m, st + ib,
                                    0)))
                return rc;
            HIP_TRY(hipDeviceSynchronize());
            return KAD_OK;
        }
        hipLaunchKernelGGL(status_patch_kernel, dim3(grid_for(m)), dim3(BLOCK), 0, 0,
                           nodes ? reinterpret_cast<const uint32_t*>(st) : nullptr, st + ib, m, t->status_mut,
                           marks_of(t));
        HIP_TRY(hipGetLastError());
    }
    if ((rc = rebuild_good_prefix(t, nullptr, false))) return rc;
    HIP_TRY(hipDeviceSynchronize());
    return KAD_OK;
}

int kad_table_patch_times(kad_table* t, uint32_t m, const uint32_t* nodes, const int64_t* time_ns,
                          const int64_t* reply_ns, const uint8_t* expired) {
    if (!t || (m && (!nodes || !time_ns || !reply_ns || !expired))) return set_err(KAD_ERR_INVALID, "NULL argument");
    if (!t->time_ns) return set_err(KAD_ERR_INVALID, "kad_table_set_times was not called");
    for (uint32_t j = 0; j < m; j++)
        if (nodes[j] >= t->d.n) return set_err(KAD_ERR_INVALID, "node %u out of range (n=%u)", nodes[j], t->d.n);
    if (!m) return KAD_OK;
    DeviceGuard g(t->device);
    int rc;
    if ((rc = svc_quiesce(t))) return rc;
    HIP_TRY(hipDeviceSynchronize());  // a refresh still running reads the staging and the deadline runs
    const size_t a = (4ull * m + 15) & ~15ull, b = 8ull * m;
    if ((rc = stage_reserve(t, a + 2 * b + m))) return rc;
    uint8_t* st = static_cast<uint8_t*>(t->stage);
    HIP_TRY(hipMemcpy(st, nodes, 4ull * m, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(st + a, time_ns, b, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(st + a + b, reply_ns, b, hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(st + a + 2 * b, expired, m, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(times_patch_kernel, dim3(grid_for(m)), dim3(BLOCK), 0, 0, reinterpret_cast<const uint32_t*>(st),
                       reinterpret_cast<const int64_t*>(st + a), reinterpret_cast<const int64_t*>(st + a + b),
                       st + a + 2 * b, m, t->d.n, t->time_ns, t->reply_ns, t->expired);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipDeviceSynchronize());
    if ((rc = dl_patch(t, m, nodes, time_ns, reply_ns, expired))) {
        t->dl.invalidate();  // the next refresh re-derives every node: still exact
        return rc;
    }
    return KAD_OK;
}

int kad_table_set_times(kad_table* t, const int64_t* time_ns, const int64_t* reply_ns, const uint8_t* expired) {
    if (!t || (t->d.n && (!time_ns || !reply_ns || !expired))) return set_err(KAD_ERR_INVALID, "NULL argument");
    DeviceGuard g(t->device);
    int rc;
    if ((rc = svc_quiesce(t))) return rc;
    if (!t->time_ns) {
        if ((rc = dev_upload(&t->time_ns, nullptr, t->d.n, t->owned, t->bytes)) ||
            (rc = dev_upload(&t->reply_ns, nullptr, t->d.n, t->owned, t->bytes)) ||
            (rc = dev_upload(&t->expired, nullptr, t->d.n, t->owned, t->bytes)))
            return rc;
    }
    t->dl.invalidate();  // the next refresh re-derives every node and rebuilds the deadline runs
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
    int rc;
    Deadlines& D = t->dl;
    const uint32_t n = t->d.n;
    const uint64_t nowk = dl_key(now_ns);
    if (D.valid && now_ns >= D.last_now) {
        if (D.np == 0 && nowk <= D.next) {  // no deadline passed, nothing patched: no status can change
            D.last_now = now_ns;
            return KAD_OK;
        }
        // the nodes whose deadline `now` passes (both runs, found on the host copies of their keys) and the patched ones
        const uint32_t hm = gallop_lower_bound(D.hkm, D.cm, nowk);
        const uint32_t hs = (uint32_t)(std::lower_bound(D.hks.begin() + D.cs, D.hks.end(), nowk) - D.hks.begin());
        const uint32_t mc = hm - D.cm, sc = hs - D.cs;
        // the resident service reads what changes: its launch ends (the next one waits for mut_ev)
        if ((rc = svc_quiesce(t)) || (rc = ensure_marks(t))) return rc;
        if ((uint64_t)mc + sc + D.np <= RF_INLINE && D.hkn.size() == D.hkm.size()) {
            uint32_t inl[RF_INLINE], k = 0;
            for (uint32_t x = D.cm; x < hm; x++) inl[k++] = D.hkn[x];
            for (uint32_t x = D.cs; x < hs; x++) inl[k++] = D.hsn[x];
            for (uint32_t x : D.hpend) inl[k++] = x;
            rc = small_refresh(t, s, nullptr, 0, nullptr, 0, nullptr, 0, nullptr, now_ns, inl, k);
        } else if ((uint64_t)mc + sc + D.np <= RF_CAP) {
            rc = small_refresh(t, s, D.kn + D.cm, mc, D.sn + D.cs, sc, D.pend, D.np, nullptr, now_ns);
        } else {
            hipLaunchKernelGGL(dl_process_kernel, dim3(512), dim3(BLOCK), 0, s, times_of(t), D.kn + D.cm, mc, D.sn + D.cs,
                               sc, D.pend, D.np, n, now_ns, t->status_mut, marks_of(t));
            rc = hipGetLastError() == hipSuccess ? rebuild_good_prefix(t, s, false)
                                                 : set_err(KAD_ERR_HIP, "status refresh launch failed");
        }
        if (rc) { D.invalidate(); return rc; }
        D.cm = hm;
        D.cs = hs;
        D.np = 0;
        D.hpend.clear();
        D.last_now = now_ns;
        D.set_next();
        return mark_async(t, s);
    }
    // first refresh after set_times / a status patch, or `now` moved back: every node, then the runs
    if ((rc = svc_quiesce(t)) || (rc = ensure_marks(t))) return rc;
    D.invalidate();
    if (n)
        hipLaunchKernelGGL(status_from_times_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, s, times_of(t), n, now_ns,
                           t->status_mut, marks_of(t));
    HIP_TRY(hipGetLastError());
    if ((rc = rebuild_good_prefix(t, s, false))) return rc;
    if (n && dl_build_main(t, s, nowk) == KAD_OK) {  // without the runs (no memory) every refresh takes this path
        D.valid = true;
        D.last_now = now_ns;
    }
    return mark_async(t, s);
}

int kad_rt_closest_batch(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                         uint8_t* out_cnt, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (q == 0) return KAD_OK;
    if (!targets || (!out_idx && count)) return set_err(KAD_ERR_INVALID, "NULL buffer");
    if (count == 0 && !out_cnt) return KAD_OK;
    if (((uintptr_t)targets & 3) || ((uintptr_t)out_idx & 3)) return set_err(KAD_ERR_INVALID, "device buffers must be 4-byte aligned");
    DeviceGuard g(t->device);
    return rt_dispatch(t, targets, q, count, out_idx, out_cnt, (hipStream_t)stream);
}

int kad_rt_closest_batch_packed(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count,
                                uint32_t* packed, uint32_t* escape, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (count != 8 || !(t->d.flags & TF_WS) || std::getenv("KAD_RT_KERNEL"))
        return set_err(KAD_ERR_UNSUPPORTED, "packed rows: count 8 on tables with short window lines only");
    if (q == 0) return KAD_OK;
    if (!targets || !packed || !escape) return set_err(KAD_ERR_INVALID, "NULL buffer");
    if (((uintptr_t)targets & 3) || ((uintptr_t)packed & 3)) return set_err(KAD_ERR_INVALID, "device buffers must be 4-byte aligned");
    DeviceGuard g(t->device);
    hipLaunchKernelGGL(rt_ws_packed_kernel<false>, dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d, targets,
                       q, packed, escape, nullptr);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_rt_closest_keys_packed(const kad_table* t, const uint64_t* keys, uint32_t q, uint32_t count, uint32_t* packed,
                               uint32_t* escape, uint32_t* tail, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (count != 8 || !(t->d.flags & TF_WS) || std::getenv("KAD_RT_KERNEL"))
        return set_err(KAD_ERR_UNSUPPORTED, "key-only rows: count 8 on tables with short window lines only");
    if (q == 0) return KAD_OK;
    if (!keys || !packed || !escape || !tail) return set_err(KAD_ERR_INVALID, "NULL buffer");
    if (((uintptr_t)keys & 7) || ((uintptr_t)packed & 3)) return set_err(KAD_ERR_INVALID, "keys must be 8-byte aligned, rows 4-byte");
    DeviceGuard g(t->device);
    hipLaunchKernelGGL(rt_ws_packed_kernel<true>, dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d,
                       reinterpret_cast<const uint8_t*>(keys), q, packed, escape, tail);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_rt_closest_batch_dual(const kad_table* t4, const kad_table* t6, const uint8_t* targets, const uint8_t* af,
                              uint32_t q, uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, void* stream) {
    if (!t4 && !t6) return set_err(KAD_ERR_INVALID, "both tables NULL");
    if (t4 && t6 && t4->device != t6->device) return set_err(KAD_ERR_INVALID, "tables on different devices");
    if (q == 0) return KAD_OK;
    if (!targets || !af || (!out_idx && count)) return set_err(KAD_ERR_INVALID, "NULL buffer");
    // A missing family behaves as an empty table (zero results), as an empty RoutingTable does.
    DevTable empty{};
    const DevTable& d4 = t4 ? t4->d : empty;
    const DevTable& d6 = t6 ? t6->d : empty;
    DeviceGuard g(t4 ? t4->device : t6->device);
    hipStream_t s = (hipStream_t)stream;
    if (count == 0) {
        if (out_cnt) HIP_TRY(hipMemsetAsync(out_cnt, 0, q, s));
        return KAD_OK;
    }
    if (count > 8 && count <= KAD_MAX_COUNT) {
        const uint32_t need = count <= 16 ? LS_WL16 : LS_WL32;
        int rc;
        if ((t4 && (rc = ensure_lines(t4, need, s))) || (t6 && (rc = ensure_lines(t6, need, s)))) return rc;
    }
    // LEAN kernels where every family has the line set the count needs or is empty (config 4's two uniform tables)
    auto lean = [&](uint32_t f) { return (d4.B == 0 || (d4.flags & f)) && (d6.B == 0 || (d6.flags & f)); };
    if (count > KAD_MAX_COUNT)
        hipLaunchKernelGGL(rt_wave_kernel, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0, s, d4, d6, af,
                           targets, q, count, out_idx, out_cnt);
    else if (count <= 8 && ((d4.flags | d6.flags) & TF_WL) && lean(TF_WL))
        hipLaunchKernelGGL(rt_dual_wl_lean_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                           out_idx, out_cnt);
    else if (count <= 8 && ((d4.flags | d6.flags) & TF_WL))
        hipLaunchKernelGGL(rt_dual_wl_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                           out_idx, out_cnt);
    else if (count <= 8 && ((d4.flags | d6.flags) & TF_SL) && lean(TF_SL))
        hipLaunchKernelGGL(rt_dual_sl_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                           out_idx, out_cnt);
    else if (count <= 8 && ((d4.flags | d6.flags) & TF_GL))
        hipLaunchKernelGGL(rt_dual_gl_kernel<8>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                           out_idx, out_cnt);
    else if (count <= 8) launch_rt_dual<8>(d4, d6, targets, af, q, count, out_idx, out_cnt, s);
    else if (count <= 16 && ((d4.flags | d6.flags) & TF_WL16) && lean(TF_WL16))
        hipLaunchKernelGGL(rt_dual_wl16_kernel<true>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q,
                           count, out_idx, out_cnt);
    else if (count <= 16 && ((d4.flags | d6.flags) & TF_WL16))
        hipLaunchKernelGGL(rt_dual_wl16_kernel<false>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q,
                           count, out_idx, out_cnt);
    else if (count <= 16 && ((d4.flags | d6.flags) & TF_SL16) && lean(TF_SL16))
        hipLaunchKernelGGL(rt_dual_sl16_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                           out_idx, out_cnt);
    else if (count <= 16 && ((d4.flags | d6.flags) & TF_GL16))
        hipLaunchKernelGGL(rt_dual_gl_kernel<16>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                           out_idx, out_cnt);
    else if (count <= 16) launch_rt_dual<16>(d4, d6, targets, af, q, count, out_idx, out_cnt, s);
    else if (((d4.flags | d6.flags) & TF_WL32) && lean(TF_WL32) && count >= 24 && (count & 3u) == 0)
        hipLaunchKernelGGL(rt_dual_wl32q_kernel<false>, dim3(grid_for(4ull * q)), dim3(BLOCK), 0, s, d4, d6, targets, af,
                           q, count, out_idx, out_cnt);
    else if (((d4.flags | d6.flags) & TF_WL32) && lean(TF_WL32))
        hipLaunchKernelGGL(rt_dual_wl32_kernel<true>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q,
                           count, out_idx, out_cnt);
    else if ((d4.flags | d6.flags) & TF_WL32)
        hipLaunchKernelGGL(rt_dual_wl32_kernel<false>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q,
                           count, out_idx, out_cnt);
    else if (((d4.flags | d6.flags) & TF_GL32) && lean(TF_GL32) && count >= 24 && (count & 3u) == 0)
        hipLaunchKernelGGL(rt_dual_wl32q_kernel<true>, dim3(grid_for(4ull * q)), dim3(BLOCK), 0, s, d4, d6, targets, af,
                           q, count, out_idx, out_cnt);
    else if ((d4.flags | d6.flags) & TF_GL32)
        hipLaunchKernelGGL(rt_dual_gl_kernel<32>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                           out_idx, out_cnt);
    else launch_rt_dual<32>(d4, d6, targets, af, q, count, out_idx, out_cnt, s);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

static int shard_batch(const kad_table* t, const uint32_t* global_good_prefix, uint32_t global_buckets,
                       uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                       uint32_t reach_hi, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* rows,
                       uint32_t row_cap, uint32_t* parts, uint32_t part_cap, uint32_t* counters, uint32_t dests,
                       uint64_t dest_words, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    int rc = check_count(count);
    if (rc) return rc;
    if (count == 0) return set_err(KAD_ERR_INVALID, "count 0: nothing to answer (the caller writes empty rows)");
    if (depth < 1 || depth > 63) return set_err(KAD_ERR_INVALID, "depth %u outside 1..63", depth);
    if ((uint64_t)shard_first_bucket + t->d.B > global_buckets)
        return set_err(KAD_ERR_INVALID, "shard buckets [%u, %u) exceed the %u global buckets", shard_first_bucket,
                       shard_first_bucket + t->d.B, global_buckets);
    if (q == 0) return KAD_OK;
    if (!global_good_prefix || !targets || !rows || !parts || !counters) return set_err(KAD_ERR_INVALID, "NULL buffer");
    if (t->d.B == 0) return KAD_OK;
    ShardCtx S{};
    S.gpre = global_good_prefix;
    S.gbase = global_base_hi;
    S.gshift = 64 - depth;
    S.GB = global_buckets;
    S.s_lo = shard_first_bucket;
    S.s_hi = shard_first_bucket + t->d.B;
    S.reach_lo = reach_lo;
    S.reach_hi = reach_hi;
    S.rows = rows;
    S.parts = parts;
    S.ctr = counters;
    S.row_cap = row_cap;
    S.part_cap = part_cap;
    S.rs = KAD_ROW_WORDS(count);
    S.ps = KAD_PART_WORDS(count);
    S.dests = dests;
    S.nblk = (q + BLOCK - 1) / BLOCK;
    S.dest_words = dest_words;
    // the window lines are valid for a shard of a uniform table of the same depth (built on first use for
    // counts 9..32, as for the unsharded query)
    const bool uni = (t->d.flags & TF_WL) && (64 - t->d.rshift) == depth;
    if (uni && count > 8 && (rc = ensure_lines(t, count <= 16 ? LS_WL16 : LS_WL32, (hipStream_t)stream))) return rc;
    const uint32_t fl = t->d.flags;
    const int lk = !uni ? 0 : count <= 8 ? 8 : count <= 16 ? ((fl & TF_WL16) ? 16 : 0) : ((fl & TF_WL32) ? 32 : 0);
    DeviceGuard g(t->device);
    void (*kern)(DevTable, ShardCtx, const uint8_t*, uint32_t, uint32_t, uint32_t, uint32_t) =
        lk == 8 ? rt_shard_kernel<8, shard_qb(8), shard_wg(8)> : lk == 16 ? rt_shard_kernel<16, shard_qb(16), shard_wg(16)>
        : lk == 32 ? rt_shard_kernel<32, shard_qb(32), shard_wg(32)> : rt_shard_kernel<0, shard_qb(0), shard_wg(0)>;
    uint32_t qb = shard_qb(lk), wg = shard_wg(lk);
    const uint32_t aligned16 = ((uintptr_t)targets & 15u) == 0;
    uint32_t abl = 0;
#ifdef KAD_ABLATIONS
    if (const char* e = std::getenv("KAD_SHARD_ABL")) abl = (uint32_t)std::atoi(e);
    if (abl & 16) {  // 2,048 queries per workgroup of 256 threads (A/B)
        qb = 8u * BLOCK;
        wg = BLOCK;
        kern = lk == 8 ? rt_shard_kernel<8, 8u * BLOCK, BLOCK> : lk == 16 ? rt_shard_kernel<16, 8u * BLOCK, BLOCK>
               : lk == 32 ? rt_shard_kernel<32, 8u * BLOCK, BLOCK> : rt_shard_kernel<0, 8u * BLOCK, BLOCK>;
    }
#endif
    hipLaunchKernelGGL(kern, dim3((uint32_t)(((uint64_t)q + qb - 1) / qb)), dim3(wg), 0,
                       (hipStream_t)stream, t->d, S, targets, q, count, aligned16, abl);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_rt_shard_batch(const kad_table* t, const uint32_t* global_good_prefix, uint32_t global_buckets,
                       uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                       uint32_t reach_hi, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* rows,
                       uint32_t row_cap, uint32_t* parts, uint32_t part_cap, uint32_t* counters, void* stream) {
    return shard_batch(t, global_good_prefix, global_buckets, global_base_hi, depth, shard_first_bucket, reach_lo,
                       reach_hi, targets, q, count, rows, row_cap, parts, part_cap, counters, 1, 0, stream);
}

void kad_home_range(uint32_t q, uint32_t world, uint32_t rank, uint32_t* lo, uint32_t* hi) {
    // the query blocks k with home_of_block(k) == rank: k in [ceil(rank * nblk / world), ceil((rank+1) * nblk / world))
    const uint32_t nblk = (q + BLOCK - 1) / BLOCK;
    auto first = [&](uint32_t r) { return (uint32_t)(((uint64_t)r * nblk + world - 1) / world); };
    const uint64_t a = (uint64_t)first(rank) * BLOCK, e = (uint64_t)first(rank + 1) * BLOCK;
    *lo = (uint32_t)std::min<uint64_t>(a, q);
    *hi = (uint32_t)std::min<uint64_t>(e, q);
}

static int shard_home(const kad_table* t, const uint32_t* global_good_prefix, uint32_t global_buckets,
                      uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                      uint32_t reach_hi, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t world,
                      uint32_t* send, uint32_t row_cap, uint32_t part_cap, void* stream, bool zero) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (world == 0 || world > KAD_SHARD_MAX_WORLD)
        return set_err(KAD_ERR_INVALID, "world %u outside 1..%u", world, KAD_SHARD_MAX_WORLD);
    if (row_cap == 0 || part_cap == 0) return set_err(KAD_ERR_INVALID, "row_cap and part_cap must be > 0");
    if (!send) return set_err(KAD_ERR_INVALID, "NULL buffer");
    const uint64_t bw = KAD_SHARD_BLOCK_WORDS(count, row_cap, part_cap);
    const uint64_t parts_off = (uint64_t)KAD_SHARD_REGIONS * row_cap * KAD_ROW_WORDS(count);
    const uint64_t ctr_off = parts_off + (uint64_t)part_cap * KAD_PART_WORDS(count);
    DeviceGuard g(t->device);
    if (zero) {
        hipLaunchKernelGGL(zero_counters_kernel, dim3(grid_for((uint64_t)world * KAD_SHARD_COUNTERS * KAD_SHARD_COUNTER_STRIDE)),
                           dim3(BLOCK), 0, (hipStream_t)stream, send, world, bw, ctr_off);
        HIP_TRY(hipGetLastError());
    }
    return shard_batch(t, global_good_prefix, global_buckets, global_base_hi, depth, shard_first_bucket, reach_lo,
                       reach_hi, targets, q, count, send, row_cap, send + parts_off, part_cap, send + ctr_off, world, bw,
                       stream);
}

int kad_rt_shard_batch_home(const kad_table* t, const uint32_t* global_good_prefix, uint32_t global_buckets,
                            uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                            uint32_t reach_hi, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t world,
                            uint32_t* send, uint32_t row_cap, uint32_t part_cap, void* stream) {
    return shard_home(t, global_good_prefix, global_buckets, global_base_hi, depth, shard_first_bucket, reach_lo,
                      reach_hi, targets, q, count, world, send, row_cap, part_cap, stream, true);
}

int kad_rt_shard_step_home(const kad_table* t, const uint32_t* global_good_prefix, uint32_t global_buckets,
                           uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                           uint32_t reach_hi, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t world,
                           uint32_t* send, uint32_t row_cap, uint32_t part_cap, void* stream) {
    return shard_home(t, global_good_prefix, global_buckets, global_base_hi, depth, shard_first_bucket, reach_lo,
                      reach_hi, targets, q, count, world, send, row_cap, part_cap, stream, false);
}

int kad_rt_scatter_rows(const uint32_t* rows, const uint32_t* n_rows, uint32_t n_rows_stride, uint32_t n_blocks,
                        uint32_t block_cap, uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, int device,
                        void* stream) {
    int rc = check_count(count);
    if (rc) return rc;
    if (n_blocks == 0 || block_cap == 0) return KAD_OK;
    if (!rows || !n_rows || !out_idx) return set_err(KAD_ERR_INVALID, "NULL buffer");
    DeviceGuard g(device);
    hipLaunchKernelGGL(scatter_rows_kernel, dim3(grid_for((uint64_t)n_blocks * block_cap * scatter_lpr(count))), dim3(BLOCK), 0,
                       (hipStream_t)stream, rows, n_rows, n_rows_stride ? n_rows_stride : 1u, n_blocks, block_cap,
                       (uint32_t)KAD_ROW_WORDS(count), count,
                       out_idx, out_cnt);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_rt_merge_parts(const uint32_t* parts, uint32_t n_parts, uint32_t count, uint32_t* out_idx, uint8_t* out_cnt,
                       int device, void* stream) {
    int rc = check_count(count);
    if (rc) return rc;
    if (n_parts == 0) return KAD_OK;
    if (!parts || !out_idx) return set_err(KAD_ERR_INVALID, "NULL buffer");
    DeviceGuard g(device);
    hipLaunchKernelGGL(merge_parts_kernel, dim3(grid_for(n_parts)), dim3(BLOCK), 0, (hipStream_t)stream, parts, n_parts,
                       (uint32_t)KAD_ROW_WORDS(count), (uint32_t)KAD_PART_WORDS(count), count, out_idx, out_cnt);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

static int gather_finish(const uint32_t* recv, uint32_t world, uint32_t row_cap, uint32_t part_cap, uint32_t qbase,
                         uint32_t q, uint32_t head_words, uint32_t count, uint32_t* scratch, uint32_t* out_idx,
                         uint8_t* out_cnt, uint32_t* overflow, int device, void* stream, uint32_t* zsend = nullptr) {
    int rc = check_count(count);
    if (rc) return rc;
    if (count == 0) return set_err(KAD_ERR_INVALID, "count 0: nothing to answer (the caller writes empty rows)");
    if (world == 0 || world > KAD_SHARD_MAX_WORLD)
        return set_err(KAD_ERR_INVALID, "world %u outside 1..%u", world, KAD_SHARD_MAX_WORLD);
    if (row_cap == 0 || part_cap == 0) return set_err(KAD_ERR_INVALID, "row_cap and part_cap must be > 0");
    if (q == 0) return KAD_OK;
    if (!recv || !scratch || !out_idx) return set_err(KAD_ERR_INVALID, "NULL buffer");
    GatherCtx G{};
    G.recv = recv;
    G.rs = KAD_ROW_WORDS(count);
    G.ps = KAD_PART_WORDS(count);
    G.parts_off = (uint64_t)KAD_SHARD_REGIONS * row_cap * G.rs;
    G.ctr_off = G.parts_off + (uint64_t)part_cap * G.ps;
    G.block = KAD_SHARD_BLOCK_WORDS(count, row_cap, part_cap);
    G.world = world;
    G.row_cap = row_cap;
    G.part_cap = part_cap;
    G.count = count;
    G.q = q;
    G.qbase = qbase;
    uint32_t* head = scratch;
    uint32_t* next = scratch + head_words;  // the same offset for every rank of a step: one scratch can serve them all
    DeviceGuard g(device);
    hipStream_t s = (hipStream_t)stream;
    const uint64_t nparts = (uint64_t)world * part_cap;
    if (nparts >= 0xFFFFFFFFull) return set_err(KAD_ERR_INVALID, "buffers too large");
    const uint32_t spb = scatter_spb(row_cap, count), sb = world * KAD_SHARD_REGIONS * spb, lb = grid_for(nparts);
    if ((uint64_t)sb + lb > 0x7FFFFFFFull) return set_err(KAD_ERR_INVALID, "buffers too large");
    hipLaunchKernelGGL(gather_scatter_link_kernel, dim3(sb + lb), dim3(BLOCK), 0, s, G, sb, spb, out_idx, out_cnt,
                       overflow, head, next);
    const uint32_t mb = (uint32_t)((nparts + MERGE_WPB - 1) / MERGE_WPB),
                   zb = zsend ? grid_for((uint64_t)world * KAD_SHARD_COUNTERS * KAD_SHARD_COUNTER_STRIDE) : 0u;
    hipLaunchKernelGGL(gather_merge_kernel, dim3(mb + zb), dim3(BLOCK), 0, s, G, head, next, out_idx, out_cnt, mb, zsend);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_rt_gather_finish(const uint32_t* recv, uint32_t world, uint32_t row_cap, uint32_t part_cap, uint32_t q,
                         uint32_t count, uint32_t* scratch, uint32_t* out_idx, uint8_t* out_cnt, uint32_t* overflow,
                         int device, void* stream) {
    return gather_finish(recv, world, row_cap, part_cap, 0, q, q, count, scratch, out_idx, out_cnt, overflow, device,
                         stream);
}

int kad_rt_home_finish(const uint32_t* recv, uint32_t world, uint32_t rank, uint32_t row_cap, uint32_t part_cap,
                       uint32_t q, uint32_t count, uint32_t* scratch, uint32_t* out_idx, uint8_t* out_cnt,
                       uint32_t* overflow, int device, void* stream) {
    if (world == 0 || rank >= world) return set_err(KAD_ERR_INVALID, "rank %u of world %u", rank, world);
    uint32_t lo, hi, lo0, hi0;
    kad_home_range(q, world, rank, &lo, &hi);
    kad_home_range(q, world, 0, &lo0, &hi0);  // rank 0's range is the largest
    return gather_finish(recv, world, row_cap, part_cap, lo, hi - lo, hi0 - lo0, count, scratch, out_idx, out_cnt,
                         overflow, device, stream);
}

int kad_rt_home_finish_reset(const uint32_t* recv, uint32_t* send, uint32_t world, uint32_t rank, uint32_t row_cap,
                             uint32_t part_cap, uint32_t q, uint32_t count, uint32_t* scratch, uint32_t* out_idx,
                             uint8_t* out_cnt, uint32_t* overflow, int device, void* stream) {
    if (world == 0 || rank >= world) return set_err(KAD_ERR_INVALID, "rank %u of world %u", rank, world);
    if (!send || send == recv) return set_err(KAD_ERR_INVALID, "send must be a buffer of its own (not recv)");
    uint32_t lo, hi, lo0, hi0;
    kad_home_range(q, world, rank, &lo, &hi);
    kad_home_range(q, world, 0, &lo0, &hi0);
    if (q == 0) {  // (nothing to finish: the counters are zeroed all the same)
        const uint64_t bw = KAD_SHARD_BLOCK_WORDS(count, row_cap, part_cap);
        const uint64_t ctr_off = (uint64_t)KAD_SHARD_REGIONS * row_cap * KAD_ROW_WORDS(count) +
                                 (uint64_t)part_cap * KAD_PART_WORDS(count);
        DeviceGuard g(device);
        hipLaunchKernelGGL(zero_counters_kernel, dim3(grid_for((uint64_t)world * KAD_SHARD_COUNTERS * KAD_SHARD_COUNTER_STRIDE)),
                           dim3(BLOCK), 0, (hipStream_t)stream, send, world, bw, ctr_off);
        HIP_TRY(hipGetLastError());
        return KAD_OK;
    }
    return gather_finish(recv, world, row_cap, part_cap, lo, hi - lo, hi0 - lo0, count, scratch, out_idx, out_cnt,
                         overflow, device, stream, send);
}

int kad_table_set_addrs(kad_table* t, uint32_t addr_len, const uint8_t* addrs) {
    if (!t || (t->d.n && !addrs)) return set_err(KAD_ERR_INVALID, "NULL argument");
    if (addr_len != KAD_ADDR4_LEN && addr_len != KAD_ADDR6_LEN)
        return set_err(KAD_ERR_INVALID, "addr_len %u: 6 (in_addr + port) or 18 (in6_addr + port)", addr_len);
    DeviceGuard g(t->device);
    if (int rc = svc_quiesce(t)) return rc;
    if (t->wrec && t->addr_len != addr_len) return set_err(KAD_ERR_INVALID, "address length changed");
    const uint32_t rec = addr_len == KAD_ADDR4_LEN ? WREC4 : WREC6;
    int rc;
    if (!t->wrec && (rc = dev_upload(&t->wrec, nullptr, (size_t)rec / 4 * t->d.n + 4, t->owned, t->bytes))) return rc;
    t->addr_len = addr_len;
    if (t->d.n) {
        uint8_t* da = nullptr;
        HIP_TRY(hipMalloc(&da, (size_t)addr_len * t->d.n));
        hipError_t e = hipMemcpy(da, addrs, (size_t)addr_len * t->d.n, hipMemcpyHostToDevice);
        if (e == hipSuccess) {
            hipLaunchKernelGGL(wrec_build_kernel, dim3(grid_for(t->d.n)), dim3(BLOCK), 0, 0, t->d.key, t->d.tail, da,
                               addr_len, t->d.n, t->wrec);
            e = hipGetLastError();
            if (e == hipSuccess) e = hipDeviceSynchronize();
        }
        (void)hipFree(da);
        if (e != hipSuccess) return set_err(KAD_ERR_HIP, "wire record build failed: %s", hipGetErrorString(e));
    }
    return KAD_OK;
}

int kad_buffer_nodes_batch(const kad_table* t, const uint8_t* targets, uint32_t q, const uint32_t* idx,
                           const uint8_t* cnt, uint32_t k, uint8_t* out, uint8_t* out_n, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (!t->wrec) return set_err(KAD_ERR_INVALID, "kad_table_set_addrs was not called");
    if (q == 0) return KAD_OK;
    if (!targets || (!idx && k) || !out) return set_err(KAD_ERR_INVALID, "NULL buffer");
    if (((uintptr_t)out & 15u) != 0) return set_err(KAD_ERR_INVALID, "out must be 16-byte aligned");
    DeviceGuard g(t->device);
    const uint4* w = reinterpret_cast<const uint4*>(t->wrec);
    if (k > KAD_MAX_COUNT) return set_err(KAD_ERR_UNSUPPORTED, "k %u > KAD_MAX_COUNT", k);
    hipStream_t st = (hipStream_t)stream;
#define KAD_BUF_LAUNCH(AL, P)                                                                                      \
    hipLaunchKernelGGL((buffer_nodes_kernel<AL, P>), dim3((q + BLOCK / P - 1) / (BLOCK / P)), dim3(BLOCK), 0, st, \
                       t->d.n, t->d.index_base, w, targets, q, idx, cnt, k, out, out_n)
    if (t->addr_len == KAD_ADDR4_LEN) {
        if (k <= 8) KAD_BUF_LAUNCH(KAD_ADDR4_LEN, 8);
        else if (k <= 16) KAD_BUF_LAUNCH(KAD_ADDR4_LEN, 16);
        else KAD_BUF_LAUNCH(KAD_ADDR4_LEN, 32);
    } else {
        if (k <= 8) KAD_BUF_LAUNCH(KAD_ADDR6_LEN, 8);
        else if (k <= 16) KAD_BUF_LAUNCH(KAD_ADDR6_LEN, 16);
        else KAD_BUF_LAUNCH(KAD_ADDR6_LEN, 32);
    }
#undef KAD_BUF_LAUNCH
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_parse_nodes_batch(const uint8_t* records, uint32_t n, uint32_t rec_len, const uint8_t* myid, uint8_t* keep,
                          int device, void* stream) {
    if (rec_len != KAD_NODE4_INFO_LEN && rec_len != KAD_NODE6_INFO_LEN)
        return set_err(KAD_ERR_INVALID, "rec_len %u: 26 or 38", rec_len);
    if (n == 0) return KAD_OK;
    if (!records || !myid || !keep) return set_err(KAD_ERR_INVALID, "NULL buffer");
    Id20 me;
    std::memcpy(me.b, myid, KAD_HASH_LEN);
    DeviceGuard g(device);
    hipLaunchKernelGGL(parse_nodes_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, (hipStream_t)stream, records, n, rec_len,
                       me, keep);
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

// The count <= 14 NodeCache kernel's form for A/B (KAD_NCL2_WPE = 6: aimed at six waves per SIMD, spills; 256: blocks of
// four waves; default: five waves per SIMD, one-wave blocks).
static int ncl2_wpe() {
    const char* e = std::getenv("KAD_NCL2_WPE");
    return e ? std::atoi(e) : 5;
}

int kad_nc_closest_batch(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                         uint8_t* out_cnt, void* stream) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (!(t->flags & KAD_TABLE_SORTED)) return set_err(KAD_ERR_NOT_SORTED, "NodeCache query needs a KAD_TABLE_SORTED table");
    if (q == 0) return KAD_OK;
    if (!targets || (!out_idx && count)) return set_err(KAD_ERR_INVALID, "NULL buffer");
    DeviceGuard g(t->device);
    if (count >= 1 && count <= 32) {
        const int rc = ensure_lines(t, count <= 16 ? LS_NCL : LS_NCL32, (hipStream_t)stream);
        if (rc) return rc;
    }
    const char* ev = std::getenv("KAD_NC_KERNEL");
    const bool lines = (t->d.flags & TF_NCL) && !ev;  // KAD_NC_KERNEL=<kernel> picks another one (A/B timing)
#ifdef KAD_ABLATIONS  // timing ablations with WRONG results: only in the tools build
    if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lines_abl1") == 0 && count >= 1 && count <= 16)
        hipLaunchKernelGGL((nc_line_kernel<1, false, false>), dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d,
                           t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lines_abl2") == 0 && count >= 1 && count <= 16)
        hipLaunchKernelGGL((nc_line_kernel<2, false, false>), dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d,
                           t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL32) && ev && std::strcmp(ev, "l32_abl1") == 0 && count > 16 && count <= 32)
        hipLaunchKernelGGL((nc32_line_kernel<1, false>), dim3(grid_for(8ull * q)), dim3(BLOCK), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL32) && ev && std::strcmp(ev, "l32_stats") == 0 && count > 16 && count <= 32)
        hipLaunchKernelGGL((nc32_line_kernel<3, false>), dim3(grid_for(8ull * q)), dim3(BLOCK), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL32) && ev && std::strcmp(ev, "l32_abl2") == 0 && count > 16 && count <= 32)
        hipLaunchKernelGGL((nc32_line_kernel<2, false>), dim3(grid_for(8ull * q)), dim3(BLOCK), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if (count > 16 && count <= 64 && t->d.n > 0 && ev && std::strcmp(ev, "w64_abl1") == 0)
        hipLaunchKernelGGL(nc_wave64_kernel<1>, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0,
                           (hipStream_t)stream, t->d, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lines_abl3") == 0 && count >= 1 && count <= 16)
        hipLaunchKernelGGL((nc_line_kernel<3, false, true>), dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d,
                           t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lines_stats") == 0 && count >= 1 && count <= 16)
        hipLaunchKernelGGL((nc_line_kernel<5, false, true>), dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d,
                           t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lines_p2") == 0 && count >= 1 && count <= 16)
        hipLaunchKernelGGL((nc_line_kernel<6, false, true>), dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lines_wave") == 0 && count >= 1 && count <= NCL2_COUNT_MAX)
        hipLaunchKernelGGL((nc_line_kernel<0, false, true>), dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lane_abl1") == 0 && count >= 1 && count <= NCL2_COUNT_MAX)
        hipLaunchKernelGGL((ncl2_lane_kernel<1, false, 5, 64>), dim3(grid64(q)), dim3(64), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lane_abl9") == 0 && count >= 1 && count <= NCL2_COUNT_MAX)
        hipLaunchKernelGGL((ncl2_lane_kernel<9, false, 5, 64>), dim3(grid64(q)), dim3(64), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lane_abl11") == 0 && count >= 1 && count <= NCL2_COUNT_MAX)
        hipLaunchKernelGGL((ncl2_lane_kernel<11, false, 5, 64>), dim3(grid64(q)), dim3(64), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lane_abl12") == 0 && count >= 1 && count <= NCL2_COUNT_MAX)
        hipLaunchKernelGGL((ncl2_lane_kernel<12, false, 5, 64>), dim3(grid64(q)), dim3(64), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lane_stats") == 0 && count >= 1 && count <= NCL2_COUNT_MAX)
        hipLaunchKernelGGL((ncl2_lane_kernel<5, false, 5, 64>), dim3(grid64(q)), dim3(64), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL) && ev && std::strcmp(ev, "lines_one") == 0 && count >= 1 && count <= 16)
        hipLaunchKernelGGL((nc_line_kernel<0, false, false>), dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else
#endif
    if (lines && count >= 1 && count <= NCL2_COUNT_MAX) {
        const int wpe = ncl2_wpe();
        if (wpe == 6)
            hipLaunchKernelGGL((ncl2_lane_kernel<0, false, 6, 64>), dim3(grid64(q)), dim3(64), 0,
                               (hipStream_t)stream, t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
        else if (wpe == 256)
            hipLaunchKernelGGL((ncl2_lane_kernel<0, false, 5, 256>), dim3(grid_for(q)), dim3(256), 0,
                               (hipStream_t)stream, t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
        else
            hipLaunchKernelGGL((ncl2_lane_kernel<0, false, 5, 64>), dim3(grid64(q)), dim3(64), 0,
                               (hipStream_t)stream, t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    }
    else if (lines && count > NCL2_COUNT_MAX && count <= 16)
        hipLaunchKernelGGL((nc_line_kernel<0, false, false>), dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if ((t->d.flags & TF_NCL32) && !ev && count > 16 && count <= 32)
        hipLaunchKernelGGL((nc32_line_kernel<0, false>), dim3(grid_for(8ull * q)), dim3(BLOCK), 0, (hipStream_t)stream,
                           t->d, t->d, nullptr, targets, q, count, out_idx, out_cnt);
    else if (count >= 1 && count <= 16 && ev && std::strcmp(ev, "group1") == 0)
        hipLaunchKernelGGL(nc_group_v1_kernel, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0,
                           (hipStream_t)stream, t->d, targets, q, count, out_idx, out_cnt);
    else if (count >= 1 && count <= 16 && ev && std::strcmp(ev, "group2") == 0)
        hipLaunchKernelGGL(nc_group_kernel, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0,
                           (hipStream_t)stream, t->d, targets, q, count, out_idx, out_cnt);
    else if (count >= 1 && count <= 16 && t->d.n > 0 && ev && std::strcmp(ev, "multi4") == 0)
        hipLaunchKernelGGL(nc_multi_kernel<4>, dim3((q + 4 * (BLOCK / 64) - 1) / (4 * (BLOCK / 64))), dim3(BLOCK), 0,
                           (hipStream_t)stream, t->d, targets, q, count, out_idx, out_cnt);
    else if (count > 16 && count <= 64 && t->d.n > 0 && ev && std::strcmp(ev, "wave64") == 0)
        hipLaunchKernelGGL(nc_wave64_kernel<0>, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0,
                           (hipStream_t)stream, t->d, targets, q, count, out_idx, out_cnt);
    else if (count > 16 && count <= 64 && t->d.n > 0 && !(ev && std::strcmp(ev, "serial") == 0) &&
             !(ev && std::strcmp(ev, "multi2") == 0))
        hipLaunchKernelGGL(nc_two_pass_kernel, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0,
                           (hipStream_t)stream, t->d, targets, q, count, out_idx, out_cnt);
    else if (count >= 1 && count <= 32 && t->d.n > 0 && !(ev && std::strcmp(ev, "serial") == 0))
        hipLaunchKernelGGL(nc_multi_kernel<2>, dim3((q + 2 * (BLOCK / 64) - 1) / (2 * (BLOCK / 64))), dim3(BLOCK), 0,
                           (hipStream_t)stream, t->d, targets, q, count, out_idx, out_cnt);
    else if (count >= 1 && count <= 32 && !(ev && std::strcmp(ev, "serial") == 0))
        hipLaunchKernelGGL(nc_group_kernel, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0,
                           (hipStream_t)stream, t->d, targets, q, count, out_idx, out_cnt);
    else
        hipLaunchKernelGGL(nc_closest_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, t->d, targets, q,
                           count, out_idx, out_cnt);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_nc_closest_batch_dual(const kad_table* t4, const kad_table* t6, const uint8_t* targets, const uint8_t* af,
                              uint32_t q, uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, void* stream) {
    if (!t4 && !t6) return set_err(KAD_ERR_INVALID, "both tables NULL");
    if (t4 && t6 && t4->device != t6->device) return set_err(KAD_ERR_INVALID, "tables on different devices");
    for (const kad_table* t : {t4, t6})
        if (t && t->d.n && !(t->flags & KAD_TABLE_SORTED))
            return set_err(KAD_ERR_NOT_SORTED, "NodeCache query needs KAD_TABLE_SORTED tables");
    if (q == 0) return KAD_OK;
    if (!targets || !af || (!out_idx && count)) return set_err(KAD_ERR_INVALID, "NULL buffer");
    DevTable empty{};  // a missing family behaves as an empty map (no results)
    const DevTable& d4 = t4 ? t4->d : empty;
    const DevTable& d6 = t6 ? t6->d : empty;
    DeviceGuard g(t4 ? t4->device : t6->device);
    hipStream_t s = (hipStream_t)stream;
    if (count == 0) {
        if (out_cnt) HIP_TRY(hipMemsetAsync(out_cnt, 0, q, s));
        return KAD_OK;
    }
    if (count <= 32) {
        const uint32_t need = count <= 16 ? LS_NCL : LS_NCL32;
        int rc;
        if ((t4 && (rc = ensure_lines(t4, need, s))) || (t6 && (rc = ensure_lines(t6, need, s)))) return rc;
    }
    if (count <= NCL2_COUNT_MAX)
        hipLaunchKernelGGL((ncl2_lane_kernel<0, true, 5, 64>), dim3(grid64(q)), dim3(64), 0, s, d4, d6, af, targets, q,
                           count, out_idx, out_cnt);
    else if (count <= 16)
        hipLaunchKernelGGL((nc_line_kernel<0, true, false>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, af, targets, q,
                           count, out_idx, out_cnt);
    else if (count <= 32 && ((d4.flags | d6.flags) & TF_NCL32))  // a family without the lines takes the wave path
        hipLaunchKernelGGL((nc32_line_kernel<0, true>), dim3(grid_for(8ull * q)), dim3(BLOCK), 0, s, d4, d6, af, targets,
                           q, count, out_idx, out_cnt);
    else if (count <= 64)
        hipLaunchKernelGGL(nc_two_pass_dual_kernel, dim3((q + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK), 0, s, d4, d6,
                           af, targets, q, count, out_idx, out_cnt);
    else  // any larger count (node_cache.h:32 takes a size_t): the serial walk
        hipLaunchKernelGGL(nc_closest_dual_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, af, targets, q, count,
                           out_idx, out_cnt);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

// Pinned and device buffers of every slot (index buffers of 32 * CHUNK words: a chunk holds CHUNK queries of count
// <= 32, fewer of a larger count).
static int pipe_ready(HostPipe& P) {
    if (!P.start) HIP_TRY(hipEventCreateWithFlags(&P.start, hipEventDisableTiming));
    for (auto& w : P.slot)
        for (HostPipe::Slot& S : w) {
            // each piece on its own, so that a call after a failed one completes the slot
            if (!S.s) HIP_TRY(hipStreamCreateWithFlags(&S.s, hipStreamNonBlocking));
            if (!S.done) HIP_TRY(hipEventCreateWithFlags(&S.done, hipEventDisableTiming));
            if (!S.ht) HIP_TRY(hipHostMalloc((void**)&S.ht, 20ull * HostPipe::CHUNK, hipHostMallocDefault));
            if (!S.hc) HIP_TRY(hipHostMalloc((void**)&S.hc, HostPipe::CHUNK, hipHostMallocDefault));
            if (!S.hi) HIP_TRY(hipHostMalloc((void**)&S.hi, 4ull * 32 * HostPipe::CHUNK, hipHostMallocDefault));
            if (!S.dt) HIP_TRY(hipMalloc(&S.dt, 20ull * HostPipe::CHUNK));
            if (!S.dc) HIP_TRY(hipMalloc(&S.dc, HostPipe::CHUNK));
            if (!S.di) HIP_TRY(hipMalloc(&S.di, 4ull * 32 * HostPipe::CHUNK));
        }
    return KAD_OK;
}

static int small_ready(HostPipe& P) {
    if (!P.start) HIP_TRY(hipEventCreateWithFlags(&P.start, hipEventDisableTiming));
    if (!P.ss) HIP_TRY(hipStreamCreateWithFlags(&P.ss, hipStreamNonBlocking));
    if (!P.st) {
        HIP_TRY(hipHostMalloc((void**)&P.st, 20ull * HostPipe::SMALL, hipHostMallocMapped));
        HIP_TRY(hipHostGetDevicePointer((void**)&P.dst, P.st, 0));
    }
    if (!P.sc) {
        HIP_TRY(hipHostMalloc((void**)&P.sc, HostPipe::SMALL, hipHostMallocMapped));
        HIP_TRY(hipHostGetDevicePointer((void**)&P.dsc, P.sc, 0));
    }
    if (!P.si) {
        HIP_TRY(hipHostMalloc((void**)&P.si, 4ull * HostPipe::SMALL * HostPipe::SMALL_COUNT, hipHostMallocMapped));
        HIP_TRY(hipHostGetDevicePointer((void**)&P.dsi, P.si, 0));
    }
    return KAD_OK;
}

// q <= SMALL, count <= SMALL_COUNT: the kernel reads the targets from and writes the rows to mapped pinned memory.
static int small_query(const kad_table* t, HostPipe& P, const uint8_t* targets, uint32_t q, uint32_t count,
                       uint32_t* out_idx, uint8_t* out_cnt, bool nc) {
    int rc = small_ready(P);
    if (rc) return rc;
    std::memcpy(P.st, targets, 20ull * q);
    const char* mode = std::getenv("KAD_SMALL_SYNC");  // A/B of the synchronisation (tools/latency_floor.hip)
    // ordered after the table's last asynchronous status refresh, whatever its stream (every other change to a
    // table is synchronous); an event on the null stream would cost a whole round trip (13 us on MI355X)
    if (t->mut_async) HIP_TRY(hipStreamWaitEvent(P.ss, t->mut_ev, 0));
    rc = nc ? kad_nc_closest_batch(t, P.dst, q, count, P.dsi, P.dsc, P.ss)
            : kad_rt_closest_batch(t, P.dst, q, count, P.dsi, P.dsc, P.ss);
    hipError_t e = hipSuccess;
    if (mode && std::strstr(mode, "spin")) {
        while ((e = hipStreamQuery(P.ss)) == hipErrorNotReady) {
        }
    } else {
        e = hipStreamSynchronize(P.ss);
    }
    if (rc) return rc;
    if (e != hipSuccess) return set_err(KAD_ERR_HIP, "host batch: %s", hipGetErrorString(e));
    if (count) std::memcpy(out_idx, P.si, 4ull * q * count);
    if (out_cnt) std::memcpy(out_cnt, P.sc, q);
    return KAD_OK;
}

// ---- the resident query service (svc_kernel) ----
static int svc_launch(const kad_table* t, HostPipe& P) {
    if (!P.vs) HIP_TRY(hipStreamCreateWithFlags(&P.vs, hipStreamNonBlocking));
    if (!P.vm) {
        HIP_TRY(hipHostMalloc((void**)&P.vm, sizeof(SvcMail), hipHostMallocMapped));
        std::memset((void*)P.vm, 0, sizeof(SvcMail));
        HIP_TRY(hipHostGetDevicePointer((void**)&P.dvm, P.vm, 0));
    }
    if (!P.vr) {
        HIP_TRY(hipHostMalloc((void**)&P.vr, sizeof(SvcReply), hipHostMallocMapped));
        std::memset((void*)P.vr, 0, sizeof(SvcReply));
        HIP_TRY(hipHostGetDevicePointer((void**)&P.dvr, P.vr, 0));
    }
    if (!P.vkhz) HIP_TRY(hipDeviceGetAttribute(&P.vkhz, hipDeviceAttributeWallClockRate, t->device));
    const int khz = P.vkhz;  // the device wall clock (wall_clock64)
    if (khz <= 0) return set_err(KAD_ERR_HIP, "no device wall clock rate");
    const uint64_t idle = (uint64_t)P.idle_us * (uint64_t)khz / 1000u, life = (uint64_t)khz * KAD_SERVE_LIFE_MS;
    // the first request of a launch sees the table after its last asynchronous status refresh
    if (t->mut_async) HIP_TRY(hipStreamWaitEvent(P.vs, t->mut_ev, 0));
    __atomic_store_n(&P.vm->stop, 0u, __ATOMIC_RELEASE);
    hipLaunchKernelGGL(svc_kernel, dim3(1), dim3(BLOCK), 0, P.vs, t->d, P.dvm, P.dvr,
                       __atomic_load_n(&P.vr->done, __ATOMIC_ACQUIRE), idle, life);
    HIP_TRY(hipGetLastError());
    P.vrun = true;
    P.vlaunches++;
    return KAD_OK;
}

// Ends the running launch, if any (the caller holds P.mu).
static int svc_halt(HostPipe& P) {
    if (!P.vrun) return KAD_OK;
    __atomic_store_n(&P.vm->stop, 1u, __ATOMIC_RELEASE);
    const hipError_t e = hipStreamSynchronize(P.vs);
    __atomic_store_n(&P.vm->stop, 0u, __ATOMIC_RELEASE);
    P.vrun = false;
    if (e != hipSuccess) return set_err(KAD_ERR_HIP, "query service: %s", hipGetErrorString(e));
    return KAD_OK;
}

// Before any call that changes or frees what the service reads (or synchronises the whole device).
static int svc_quiesce(const kad_table* t) {
    std::lock_guard<std::mutex> lk(t->pipe_mu);
    if (!t->pipe) return KAD_OK;
    std::lock_guard<std::mutex> lk2(t->pipe->mu);
    DeviceGuard g(t->device);
    return svc_halt(*t->pipe);
}

// One request of q <= SVC_Q queries, count <= SVC_COUNT (the caller holds P.mu and has validated the call).
static int svc_query(const kad_table* t, HostPipe& P, const uint8_t* targets, uint32_t q, uint32_t count,
                     uint32_t* out_idx, uint8_t* out_cnt, bool nc) {
    if (t->mut_async) {  // ordered after the table's last asynchronous status refresh, whatever its stream
        const hipError_t e = hipEventQuery(t->mut_ev);
        if (e == hipErrorNotReady) HIP_TRY(hipEventSynchronize(t->mut_ev));
        else if (e != hipSuccess) return set_err(KAD_ERR_HIP, "status refresh: %s", hipGetErrorString(e));
    }
    int rc;
    if (!P.vrun && (rc = svc_launch(t, P))) return rc;
    std::memcpy(P.vm->targets, targets, 20ull * q);
    P.vm->q = q;
    P.vm->count = count;
    P.vm->kind = nc ? 1u : 0u;
    const uint32_t s = ++P.vseq;
    __atomic_store_n(&P.vm->seq2, s, __ATOMIC_RELEASE);  // the targets, then seq2, then seq (svc_kernel)
    __atomic_store_n(&P.vm->seq, s, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    int relaunched = 0;
    for (uint64_t it = 1;; it++) {
        if (__atomic_load_n(&P.vr->done, __ATOMIC_ACQUIRE) == s) break;
        if ((it & 255u) == 0) {
            const hipError_t e = hipStreamQuery(P.vs);
            if (e == hipSuccess) {  // the launch ended (idle or life time) before it saw the request
                P.vrun = false;
                if (__atomic_load_n(&P.vr->done, __ATOMIC_ACQUIRE) == s) break;
                if (++relaunched > 3) return set_err(KAD_ERR_HIP, "query service: request %u not answered", s);
                if ((rc = svc_launch(t, P))) return rc;
            } else if (e != hipErrorNotReady) {
                P.vrun = false;
                return set_err(KAD_ERR_HIP, "query service: %s", hipGetErrorString(e));
            }
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
                (void)svc_halt(P);
                return set_err(KAD_ERR_HIP, "query service: request %u timed out", s);
            }
        }
    }
    if (count) std::memcpy(out_idx, (const void*)P.vr->idx, 4ull * q * count);
    if (out_cnt) std::memcpy(out_cnt, (const void*)P.vr->cnt, q);
    P.vrequests++;
    return KAD_OK;
}

static int host_query(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                      uint8_t* out_cnt, bool nc) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (q == 0) return KAD_OK;
    if (!targets || (!out_idx && count)) return set_err(KAD_ERR_INVALID, "NULL buffer");
    // every check the per-chunk calls make, once, before anything is queued
    if (nc && !(t->flags & KAD_TABLE_SORTED)) return set_err(KAD_ERR_NOT_SORTED, "NodeCache query needs a KAD_TABLE_SORTED table");
    {
        std::lock_guard<std::mutex> lk(t->pipe_mu);
        if (!t->pipe) {
            try {
                t->pipe = new HostPipe();
            } catch (...) {
                return set_err(KAD_ERR_NOMEM, "host batch: out of host memory");
            }
        }
    }
    HostPipe& P = *t->pipe;
    std::lock_guard<std::mutex> lk(P.mu);
    DeviceGuard g(t->device);
    if (P.idle_us && q <= SVC_Q && count <= SVC_COUNT) return svc_query(t, P, targets, q, count, out_idx, out_cnt, nc);
    if (q <= HostPipe::SMALL && count <= HostPipe::SMALL_COUNT)
        return small_query(t, P, targets, q, count, out_idx, out_cnt, nc);
    int rc = pipe_ready(P);
    if (rc) return rc;
    // ordered after the table's last asynchronous status refresh, whatever its stream
    if (t->mut_async)
        for (auto& w : P.slot)
            for (HostPipe::Slot& S : w) HIP_TRY(hipStreamWaitEvent(S.s, t->mut_ev, 0));
    if (count > 32u * HostPipe::CHUNK)
        return set_err(KAD_ERR_UNSUPPORTED, "count %u exceeds a host-batch chunk row (%u): use the device-pointer batch",
                       count, 32u * HostPipe::CHUNK);
    const uint32_t chunk = count <= 32 ? HostPipe::CHUNK : 32u * HostPipe::CHUNK / count;
    // worker w takes chunks [w * nch / W, (w + 1) * nch / W) of the batch
    const uint32_t nch = (q + chunk - 1) / chunk;
    const int W = (int)std::min<uint32_t>(HostPipe::WORKERS, nch);
    std::vector<int> wrc;
    std::vector<std::string> werr;
    try {
        wrc.assign(W, KAD_OK);
        werr.resize(W);
    } catch (...) {
        return set_err(KAD_ERR_NOMEM, "host batch: out of host memory");
    }
    auto work = [&](int w) {
        DeviceGuard gw(t->device);
        const uint32_t lo = (uint32_t)((uint64_t)w * nch / W * chunk);
        const uint32_t hi = (uint32_t)std::min<uint64_t>((uint64_t)(w + 1) * nch / W * chunk, q);
        auto finish = [&](HostPipe::Slot& S) -> int {  // the slot's chunk out to the caller's buffers
            if (!S.pending) return KAD_OK;
            S.pending = false;
            if (hipEventSynchronize(S.done) != hipSuccess) return set_err(KAD_ERR_HIP, "host batch: chunk failed");
            if (count) std::memcpy(out_idx + (size_t)S.c0 * count, S.hi, 4ull * S.n * count);
            if (out_cnt) std::memcpy(out_cnt + S.c0, S.hc, S.n);
            return KAD_OK;
        };
        int r = KAD_OK;
        uint32_t j = 0;
        for (uint32_t c0 = lo; c0 < hi && !r; c0 += chunk, j++) {
            HostPipe::Slot& S = P.slot[w][j & 1u];
            if ((r = finish(S))) break;
            const uint32_t n = std::min(chunk, hi - c0);
            std::memcpy(S.ht, targets + 20ull * c0, 20ull * n);
            if (hipMemcpyAsync(S.dt, S.ht, 20ull * n, hipMemcpyHostToDevice, S.s) != hipSuccess) {
                r = set_err(KAD_ERR_HIP, "host batch: H2D failed");
                break;
            }
            r = nc ? kad_nc_closest_batch(t, S.dt, n, count, S.di, S.dc, S.s)
                   : kad_rt_closest_batch(t, S.dt, n, count, S.di, S.dc, S.s);
            if (r) {
                (void)hipStreamSynchronize(S.s);  // the H2D copy out of the pinned slot may still run
                break;
            }
            if ((count && hipMemcpyAsync(S.hi, S.di, 4ull * n * count, hipMemcpyDeviceToHost, S.s) != hipSuccess) ||
                hipMemcpyAsync(S.hc, S.dc, n, hipMemcpyDeviceToHost, S.s) != hipSuccess ||
                hipEventRecord(S.done, S.s) != hipSuccess) {
                r = set_err(KAD_ERR_HIP, "host batch: D2H failed");
                (void)hipStreamSynchronize(S.s);
                break;
            }
            S.c0 = c0;
            S.n = n;
            S.pending = true;
        }
        for (HostPipe::Slot& S : P.slot[w]) {  // drain: no copy may still target the pinned buffers
            const int r2 = finish(S);
            if (!r) r = r2;
        }
        wrc[w] = r;
        if (r) werr[w] = kad_last_error();
    };
    std::vector<std::thread> th;
    bool inline_w[HostPipe::WORKERS] = {};  // workers whose thread could not be started run here
    try {
        th.reserve(W);
    } catch (...) {
    }
    for (int w = 1; w < W; w++) {
        try {
            th.emplace_back(work, w);
        } catch (...) {
            inline_w[w] = true;
        }
    }
    work(0);
    for (int w = 1; w < W; w++)
        if (inline_w[w]) work(w);
    for (auto& x : th) x.join();
    for (int w = 0; w < W; w++)
        if (wrc[w]) return set_err(wrc[w], "%s", werr[w].c_str());
    return KAD_OK;
}

int kad_rt_closest_batch_host(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                              uint8_t* out_cnt) {
    return host_query(t, targets, q, count, out_idx, out_cnt, false);
}

int kad_table_serve_stats(const kad_table* t, kad_serve_stats* out) {
    if (!t || !out) return set_err(KAD_ERR_INVALID, "NULL argument");
    *out = kad_serve_stats{};
    std::lock_guard<std::mutex> lk(t->pipe_mu);
    if (!t->pipe) return KAD_OK;
    HostPipe& P = *t->pipe;
    std::lock_guard<std::mutex> lk2(P.mu);
    out->idle_us = P.idle_us;
    out->launches = P.vlaunches;
    out->requests = P.vrequests;
    if (P.vr && P.vkhz > 0 && P.vrequests) {
        out->last_polls = P.vr->polls;
        const uint64_t a = P.vr->t_seen, b = P.vr->t_done;
        out->last_busy_ns = b > a ? (uint64_t)((double)(b - a) * 1e6 / P.vkhz) : 0u;
    }
    return KAD_OK;
}

int kad_table_refresh_diag(const kad_table* t, kad_refresh_diag* out) {
    if (!t || !out) return set_err(KAD_ERR_INVALID, "NULL argument");
    *out = kad_refresh_diag{};
    if (!t->rf_ctr) return KAD_OK;
    DeviceGuard g(t->device);
    uint32_t c[RF_CTRS];
    HIP_TRY(hipDeviceSynchronize());
    HIP_TRY(hipMemcpy(c, t->rf_ctr, sizeof(c), hipMemcpyDeviceToHost));
    out->spin_timeouts = c[RF_SPIN];
    out->last_block_lines = c[RF_DEFB];
    out->guard_errors = c[RF_ERR];
    return KAD_OK;
}

int kad_table_serve(kad_table* t, uint32_t idle_us) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    if (idle_us > KAD_SERVE_MAX_IDLE_US)
        return set_err(KAD_ERR_INVALID, "idle_us %u above %u", idle_us, (uint32_t)KAD_SERVE_MAX_IDLE_US);
    {
        std::lock_guard<std::mutex> lk(t->pipe_mu);
        if (!t->pipe) {
            if (!idle_us) return KAD_OK;
            try {
                t->pipe = new HostPipe();
            } catch (...) {
                return set_err(KAD_ERR_NOMEM, "query service: out of host memory");
            }
        }
    }
    HostPipe& P = *t->pipe;
    std::lock_guard<std::mutex> lk(P.mu);
    DeviceGuard g(t->device);
    const int rc = svc_halt(P);  // a launch with the old idle time ends
    P.idle_us = idle_us;
    if (rc) return rc;
    return idle_us ? svc_launch(t, P) : KAD_OK;  // running before the first request
}
int kad_nc_closest_batch_host(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out_idx,
                              uint8_t* out_cnt) {
    return host_query(t, targets, q, count, out_idx, out_cnt, true);
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

namespace {

void release(kad_table* t, void* p) {
    if (!p) return;
    auto it = std::find(t->owned.begin(), t->owned.end(), p);
    if (it != t->owned.end()) t->owned.erase(it);
    size_t sz = 0;
    if (hipMemPtrGetInfo(p, &sz) == hipSuccess && sz <= t->bytes) t->bytes -= sz;
    (void)hipFree(p);
}

// Bucket firsts -> fkey/ftail, the locate radix and TF_DIRECT (as kad_table_create builds them), uploaded into
// new buffers listed in `fresh` (the table is not touched: kad_table_apply commits them only once every
// allocation has succeeded).
struct BucketIndex {
    uint64_t* fkey = nullptr;
    uint32_t* ftail = nullptr;
    uint32_t* rrdx = nullptr;
    Radix r;
    bool direct = false;
};

int make_bucket_index(const std::vector<uint8_t>& h_first, uint32_t B, BucketIndex& out, std::vector<void*>& fresh,
                      uint64_t& fresh_bytes) {
    const uint8_t* first = h_first.data();
    std::vector<uint64_t> fkey(B);
    std::vector<uint32_t> ftail(3ull * B);
    for (uint32_t b = 0; b < B; b++) {
        fkey[b] = id_hi(first + 20ull * b);
        for (int w = 0; w < 3; w++) ftail[3ull * b + w] = id_word(first + 20ull * b, 2 + w);
    }
    uint32_t tb = 1;
    while ((1u << tb) < B && tb < 24) tb++;
    Radix r = choose_radix(fkey[0], fkey[B - 1], std::min<uint32_t>(tb + 1, 24));
    if (B >= 2) {
        const uint64_t step = fkey[1] - fkey[0];
        bool uni = step && (step & (step - 1)) == 0 && (fkey[0] & (step - 1)) == 0;
        for (uint32_t b = 0; b < B && uni; b++)
            uni = (b == 0 || fkey[b] - fkey[b - 1] == step) && !ftail[3ull * b] && !ftail[3ull * b + 1] && !ftail[3ull * b + 2];
        if (uni) { r.shift = (uint32_t)__builtin_ctzll(step); r.base = fkey[0]; r.slots = B; r.bits = tb; }
    }
    std::vector<uint32_t> rdx = build_radix(r, B, first, true);
    bool direct = r.slots == B;
    for (uint32_t sl = 0; sl < r.slots && direct; sl++) direct = rdx[sl] == (sl | RDX_EXACT);
    int rc;
    if ((rc = dev_upload(&out.fkey, fkey.data(), B, fresh, fresh_bytes)) ||
        (rc = dev_upload(&out.ftail, ftail.data(), 3ull * B, fresh, fresh_bytes)) ||
        (rc = dev_upload(&out.rrdx, rdx.data(), rdx.size(), fresh, fresh_bytes)))
        return rc;
    out.r = r;
    out.direct = direct;
    return KAD_OK;
}

}  // namespace

extern "C" {

int kad_table_apply(kad_table* t, const uint32_t* ops, uint32_t n_ops, const uint8_t* new_ids, const uint8_t* new_status,
                    uint32_t n_new, uint32_t* remap, uint32_t* new_index) {
    if (!t || (n_ops && !ops) || (n_new && (!new_ids || !new_status))) return set_err(KAD_ERR_INVALID, "NULL argument");
    if (t->d.B == 0 || t->h_off.empty()) return set_err(KAD_ERR_INVALID, "the mirror needs a RoutingTable (buckets)");
    if ((uint64_t)t->d.n + n_new >= 0x7FFFFFFFull) return set_err(KAD_ERR_INVALID, "table too large");
    DeviceGuard g(t->device);
    if (int rc = svc_quiesce(t)) return rc;  // the resident service reads the arrays this call replaces
    DevTable& d = t->d;
    const uint32_t B0 = d.B, n0 = d.n;
    // KAD_DEBUG: the phases' wall times (host plan, layout, gather, directory, line rebuild)
    const bool dbg = std::getenv("KAD_DEBUG") != nullptr;
    auto tp = std::chrono::steady_clock::now();
    auto phase = [&](const char* what) {
        if (!dbg) return;
        const auto now = std::chrono::steady_clock::now();
        std::fprintf(stderr, "kad_table_apply %s: %.3f ms\n", what, std::chrono::duration<double, std::milli>(now - tp).count());
        tp = now;
    };
    // the host plan (kad_mirror_plan.cpp): the new layout as segments of old-node ranges and handle lists
    const std::vector<uint32_t>& off0 = t->h_off;
    const uint8_t* first0 = t->h_first.data();
    kadplan::MirrorPlan plan;
    std::string perr;
    const kadplan::OldIds old_ids = [&](uint32_t a, uint32_t e, uint8_t* out) -> int {  // IDs of old nodes [a, e)
        std::vector<uint64_t> k(e - a);
        std::vector<uint32_t> tl(3ull * (e - a));
        HIP_TRY(hipMemcpy(k.data(), d.key + a, 8ull * (e - a), hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(tl.data(), d.tail + 3ull * a, 12ull * (e - a), hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < e - a; i++) {
            uint8_t* b = out + 20ull * i;
            for (int x = 0; x < 8; x++) b[x] = (uint8_t)(k[i] >> (56 - 8 * x));
            for (int w = 0; w < 3; w++)
                for (int x = 0; x < 4; x++) b[8 + 4 * w + x] = (uint8_t)(tl[3ull * i + w] >> (24 - 8 * x));
        }
        return KAD_OK;
    };
    const bool wl_table = (d.flags & TF_WL) != 0;
    int rc = kadplan::mirror_plan(off0, first0, n0, ops, n_ops, new_ids, n_new, wl_table ? (int)d.rshift : -1,
                                  wl_table ? d.rbase >> d.rshift : 0, old_ids, plan, perr);
    if (rc) return perr.empty() ? rc : set_err(rc, "%s", perr.c_str());
    const bool structural = n_ops > 0;  // node indices move: the NodeCache radix no longer applies
    // window lines need every node inside its bucket's dyadic range
    const bool lines_ok = wl_table && plan.B1 == B0 && plan.new_in_range;
    const uint32_t B1 = plan.B1, n1 = plan.n1;
    std::vector<MirrorSeg>& segs = plan.segs;
    std::vector<uint32_t>& list = plan.list;
    std::vector<uint32_t>& off1 = plan.off1;
    phase("plan (ops, layout)");
    // new nodes' device rows
    std::vector<uint64_t> nkey(n_new);
    std::vector<uint32_t> ntail(3ull * n_new);
    for (uint32_t s = 0; s < n_new; s++) {
        nkey[s] = id_hi(new_ids + 20ull * s);
        for (int w = 0; w < 3; w++) ntail[3ull * s + w] = id_word(new_ids + 20ull * s, 2 + w);
    }
    // Everything the new layout needs is allocated and filled first (`fresh`: owned by the table only once
    // all of it exists; `tmp`: scratch). Until the commit below the table is untouched, so any failure
    // leaves it exactly as it was.
    std::vector<void*> tmp, fresh;
    uint64_t tmpb = 0, freshb = 0;
    auto fail = [&](int code) {
        for (void* p : tmp) (void)hipFree(p);
        for (void* p : fresh) (void)hipFree(p);
        return code;
    };
    MirrorSeg* dseg; uint32_t *dlist, *dntail, *dnidx, *dremap = nullptr; uint64_t* dnkey; uint8_t* dnst;
    uint64_t* key1; uint32_t* tail1; uint8_t* st1;
    if ((rc = dev_upload(&dseg, segs.data(), segs.size(), tmp, tmpb)) ||
        (rc = dev_upload(&dlist, list.data(), list.size(), tmp, tmpb)) ||
        (rc = dev_upload(&dnkey, nkey.data(), n_new, tmp, tmpb)) ||
        (rc = dev_upload(&dntail, ntail.data(), 3ull * n_new, tmp, tmpb)) ||
        (rc = dev_upload(&dnst, new_status, n_new, tmp, tmpb)) || (rc = dev_upload(&dnidx, nullptr, n_new, tmp, tmpb)) ||
        (remap && (rc = dev_upload(&dremap, nullptr, n0, tmp, tmpb))))
        return fail(rc);
    if ((rc = dev_upload(&key1, nullptr, n1 + KEY_PAD, fresh, freshb)) ||
        (rc = dev_upload(&tail1, nullptr, 3ull * n1, fresh, freshb)) ||
        (rc = dev_upload(&st1, nullptr, n1, fresh, freshb)))
        return fail(rc);
    if (hipMemset(key1, 0xFF, 8ull * (n1 + KEY_PAD)) != hipSuccess || hipMemset(dnidx, 0xFF, 4ull * n_new) != hipSuccess ||
        (remap && n0 && hipMemset(dremap, 0xFF, 4ull * n0) != hipSuccess))
        return fail(set_err(KAD_ERR_HIP, "hipMemset failed"));
    if (n1)
        hipLaunchKernelGGL(mirror_gather_kernel, dim3(grid_for(n1)), dim3(BLOCK), 0, 0, dseg, (uint32_t)segs.size(), dlist, n1,
                           d.key, d.tail, d.status, dnkey, dntail, dnst, key1, tail1, st1, dremap, dnidx);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return fail(set_err(KAD_ERR_HIP, "mirror gather failed"));
    phase("upload + gather");
    // bucket directory (always a new array, so the old one stays valid until the commit)
    std::vector<uint2> dir(B1 + 1);
    for (uint32_t c = 0; c <= B1; c++) {
        dir[c].x = off1[c] | (c < B1 && off1[c + 1] - off1[c] > 32 ? WIDE : 0u);
        dir[c].y = 0;
    }
    uint2* ddir; uint32_t *scnt = nullptr, *ddm, *dany;
    if ((rc = dev_upload(&ddir, dir.data(), B1 + 1, fresh, freshb))) return fail(rc);
    const bool reshape = B1 != B0;
    BucketIndex bix;
    if (reshape &&
        (rc = dev_upload(&scnt, nullptr, B1 + 1, fresh, freshb)))
        return fail(rc);
    std::vector<uint8_t>& first1 = plan.first1;  // the new bucket firsts (only splits change them)
    if (reshape && (rc = make_bucket_index(first1, B1, bix, fresh, freshb))) return fail(rc);
    const uint8_t* fnew = reshape ? first1.data() : first0;
    // duplicate top-64 masks of the new layout
    if ((rc = dev_upload(&ddm, nullptr, B1, fresh, freshb)) || (rc = dev_upload(&dany, nullptr, 1, tmp, tmpb)))
        return fail(rc);
    if (reshape || t->firsts_low_zero < 0) {  // every bucket first is 64-bit granular (cached until a split)
        bool lz = true;
        for (uint32_t c = 0; c < B1 && lz; c++) lz = id_low_zero(fnew + 20ull * c);
        t->firsts_low_zero_next = lz ? 1 : 0;
    } else {
        t->firsts_low_zero_next = t->firsts_low_zero;
    }
    const bool low_zero = t->firsts_low_zero_next == 1;
    uint32_t any = 0;
    if (low_zero) {
        if (hipMemset(dany, 0, 4) != hipSuccess) return fail(set_err(KAD_ERR_HIP, "hipMemset failed"));
        hipLaunchKernelGGL(mirror_dmask_kernel, dim3(grid_for(B1)), dim3(BLOCK), 0, 0, key1, ddir, B1, ddm, dany);
        if (hipGetLastError() != hipSuccess || hipMemcpy(&any, dany, 4, hipMemcpyDeviceToHost) != hipSuccess)
            return fail(set_err(KAD_ERR_HIP, "dup mask failed"));
    } else {  // a bucket first below 64-bit granularity: flag every node (exact path, always correct)
        if (hipMemset(ddm, 0xFF, 4ull * B1) != hipSuccess) return fail(set_err(KAD_ERR_HIP, "hipMemset failed"));
        any = 1;
    }
    if ((new_index && n_new && hipMemcpy(new_index, dnidx, 4ull * n_new, hipMemcpyDeviceToHost) != hipSuccess) ||
        (remap && n0 && hipMemcpy(remap, dremap, 4ull * n0, hipMemcpyDefault) != hipSuccess))
        return fail(set_err(KAD_ERR_HIP, "copy of new indices failed"));
    for (void* p : tmp) (void)hipFree(p);

    phase("directory, bucket index, dup masks");
    // ---- commit: nothing below can fail before the derived state is rebuilt ----
    release(t, const_cast<uint64_t*>(d.key));
    release(t, const_cast<uint32_t*>(d.tail));
    release(t, t->status_mut);
    d.key = key1; d.tail = tail1; d.status = st1; t->status_mut = st1; d.n = n1;
    // derived state that no longer matches the nodes: NodeCache order, wire records, node times
    if (structural) {
        t->flags &= ~KAD_TABLE_SORTED;
        release(t, const_cast<uint32_t*>(d.nrdx)); d.nrdx = nullptr; t->nbits = 0;
        release(t, t->ncl_mut); t->ncl_mut = nullptr; d.ncl = nullptr; d.flags &= ~TF_NCL;
        release(t, t->ncl32_mut); t->ncl32_mut = nullptr; d.ncl32 = nullptr; d.flags &= ~TF_NCL32;
    }
    release(t, t->wrec); t->wrec = nullptr; t->addr_len = 0;
    release(t, t->time_ns); release(t, t->reply_ns); release(t, t->expired);
    t->time_ns = nullptr; t->reply_ns = nullptr; t->expired = nullptr;
    t->dl.invalidate();
    t->h_off.swap(off1);
    if (reshape) t->h_first.swap(first1);
    t->firsts_low_zero = t->firsts_low_zero_next;
    release(t, t->dir_mut);
    d.dir = ddir; t->dir_mut = ddir;
    if (reshape) {
        release(t, t->gcnt_mut);
        d.gcnt = scnt; t->gcnt_mut = scnt; d.B = B1;
        release(t, const_cast<uint64_t*>(d.fkey));
        release(t, const_cast<uint32_t*>(d.ftail));
        release(t, const_cast<uint32_t*>(d.rrdx));
        d.fkey = bix.fkey; d.ftail = bix.ftail; d.rrdx = bix.rrdx;
        d.rbase = bix.r.base; d.rshift = bix.r.shift; d.rslots = bix.r.slots; t->rbits = bix.r.bits;
        d.flags = bix.direct ? (d.flags | TF_DIRECT) : (d.flags & ~TF_DIRECT);
    }
    if (reshape || !lines_ok) {  // a split (or a new node outside its dyadic range) breaks the uniform depth
        release(t, t->wl_mut); t->wl_mut = nullptr; d.wl = nullptr; d.flags &= ~TF_WL;
        release(t, t->ws_mut); t->ws_mut = nullptr; d.ws = nullptr; d.flags &= ~TF_WS;
        release(t, t->wl16_mut); t->wl16_mut = nullptr; d.wl16 = nullptr; d.flags &= ~TF_WL16;
        release(t, t->wl32_mut); t->wl32_mut = nullptr; d.wl32 = nullptr; d.flags &= ~TF_WL32;
    }
    if (reshape) {  // general lines are per bucket: re-created below for the new bucket count
        release(t, t->gl_mut); t->gl_mut = nullptr; d.gl = nullptr; d.flags &= ~TF_GL;
        release(t, t->gl32_mut); t->gl32_mut = nullptr; d.gl32 = nullptr; d.flags &= ~TF_GL32;
        release(t, t->gl16_mut); t->gl16_mut = nullptr; d.gl16 = nullptr; d.flags &= ~TF_GL16;
        release(t, t->sl_mut); release(t, t->slb); release(t, t->gdirty);
        t->sl_mut = nullptr; t->slb = nullptr; t->gdirty = nullptr; d.sl = nullptr; d.slb = nullptr; d.slslots = 0;
        d.flags &= ~TF_SL;
        release(t, t->sl16_mut); t->sl16_mut = nullptr; d.sl16 = nullptr; d.flags &= ~TF_SL16;
    }
    release(t, const_cast<uint32_t*>(d.dmask));
    d.dmask = ddm;
    d.flags = any ? (d.flags | TF_HAS_DUP) : (d.flags & ~TF_HAS_DUP);
    t->owned.insert(t->owned.end(), fresh.begin(), fresh.end());
    t->bytes += freshb;
    drop_marks(t);  // the incremental-refresh flags are sized for the old shape
    // masks, good prefix sums, window lines
    if ((rc = rebuild_good_prefix(t, nullptr))) return rc;
    HIP_TRY(hipDeviceSynchronize());
    phase("masks, prefix sums, lines");
    // a table that lost (or never had) uniform-depth lines gets general ones (built from the new state)
    if (!(d.flags & TF_WL) && !t->gl_mut && !t->gl32_mut && (rc = setup_general_lines(t))) return rc;
    phase("general lines");
    reset_line_sets(t);
    return KAD_OK;
}

int kad_nc_apply(kad_table* t, const uint32_t* erase, uint32_t n_erase, const uint8_t* ins_ids,
                 const uint8_t* ins_status, uint32_t n_ins, uint32_t* remap, uint32_t* new_index) {
    if (!t || (n_erase && !erase) || (n_ins && (!ins_ids || !ins_status))) return set_err(KAD_ERR_INVALID, "NULL argument");
    if (t->d.B != 0 || !(t->flags & KAD_TABLE_SORTED))
        return set_err(KAD_ERR_INVALID, "kad_nc_apply needs a NodeCache-only table (no buckets, KAD_TABLE_SORTED)");
    DevTable& d = t->d;
    const uint32_t n0 = d.n;
    std::vector<uint8_t> seen(n0, 0);
    for (uint32_t j = 0; j < n_erase; j++) {
        if (erase[j] >= n0) return set_err(KAD_ERR_INVALID, "erase: node %u out of range (n=%u)", erase[j], n0);
        if (seen[erase[j]]++) return set_err(KAD_ERR_INVALID, "erase: node %u listed twice", erase[j]);
    }
    if ((uint64_t)n0 - n_erase + n_ins >= 0x7FFFFFFFull) return set_err(KAD_ERR_INVALID, "table too large");
    // the insert batch, sorted (remember each slot's place for new_index), strictly ascending
    std::vector<uint32_t> order(n_ins);
    for (uint32_t j = 0; j < n_ins; j++) order[j] = j;
    std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) {
        return std::memcmp(ins_ids + 20ull * a, ins_ids + 20ull * b, 20) < 0;
    });
    std::vector<uint64_t> ik(n_ins);
    std::vector<uint32_t> it(3ull * n_ins);
    std::vector<uint8_t> ist(n_ins);
    for (uint32_t j = 0; j < n_ins; j++) {
        const uint8_t* p = ins_ids + 20ull * order[j];
        if (j && std::memcmp(ins_ids + 20ull * order[j - 1], p, 20) == 0)
            return set_err(KAD_ERR_INVALID, "insert: an ID is listed twice");
        ik[j] = id_hi(p);
        for (int w = 0; w < 3; w++) it[3ull * j + w] = id_word(p, 2 + w);
        ist[j] = ins_status[order[j]];
    }
    const uint32_t n1 = n0 - n_erase + n_ins;
    DeviceGuard g(t->device);
    if (int rc = svc_quiesce(t)) return rc;  // the resident service reads the arrays this call replaces
    std::vector<void*> tmp, fresh;
    uint64_t tmpb = 0, freshb = 0;
    auto fail = [&](int code) {
        for (void* p : tmp) (void)hipFree(p);
        for (void* p : fresh) (void)hipFree(p);
        return code;
    };
    uint64_t *dik, *key1; uint32_t *dit, *del, *dcnt, *dpre, *dsums, *dremap, *dnew, *derr, *tail1, *rdx1;
    uint32_t* ncl1 = nullptr;
    uint8_t *dist, *deflag, *st1;
    const uint32_t tiles = (n0 + 1 + SCAN_TILE - 1) / SCAN_TILE;
    int rc;
    if ((rc = dev_upload(&dik, ik.data(), n_ins, tmp, tmpb)) || (rc = dev_upload(&dit, it.data(), 3ull * n_ins, tmp, tmpb)) ||
        (rc = dev_upload(&dist, ist.data(), n_ins, tmp, tmpb)) || (rc = dev_upload(&del, erase, n_erase, tmp, tmpb)) ||
        (rc = dev_upload(&deflag, nullptr, n0 + 1, tmp, tmpb)) || (rc = dev_upload(&dcnt, nullptr, n0 + 1, tmp, tmpb)) ||
        (rc = dev_upload(&dpre, nullptr, n0 + 1, tmp, tmpb)) || (rc = dev_upload(&dsums, nullptr, tiles, tmp, tmpb)) ||
        (rc = dev_upload(&dremap, nullptr, n0, tmp, tmpb)) || (rc = dev_upload(&dnew, nullptr, n_ins, tmp, tmpb)) ||
        (rc = dev_upload(&derr, nullptr, 1, tmp, tmpb)))
        return fail(rc);
    if ((rc = dev_upload(&key1, nullptr, n1 + KEY_PAD, fresh, freshb)) ||
        (rc = dev_upload(&tail1, nullptr, 3ull * n1, fresh, freshb)) ||
        (rc = dev_upload(&st1, nullptr, n1, fresh, freshb)))
        return fail(rc);
    if (hipMemset(deflag, 0, n0 + 1) != hipSuccess || hipMemset(dcnt, 0, 4ull * (n0 + 1)) != hipSuccess ||
        hipMemset(derr, 0, 4) != hipSuccess || hipMemset(key1, 0xFF, 8ull * (n1 + KEY_PAD)) != hipSuccess)
        return fail(set_err(KAD_ERR_HIP, "hipMemset failed"));
    if (n_erase)
        hipLaunchKernelGGL(flags_from_list_kernel, dim3(grid_for(n_erase)), dim3(BLOCK), 0, 0, del, n_erase, n0, deflag, dcnt);
    // erased_before[i] = erased nodes below i (exclusive scan of the flags, n0 + 1 entries)
    hipLaunchKernelGGL(scan_tiles_kernel, dim3(tiles), dim3(BLOCK), 0, 0, dcnt, n0 + 1, dpre, dsums, nullptr);
    hipLaunchKernelGGL(scan_sums_kernel, dim3(1), dim3(BLOCK), 0, 0, dsums, tiles, nullptr);
    hipLaunchKernelGGL(scan_apply_kernel, dim3(grid_for(n0 + 1)), dim3(BLOCK), 0, 0, dpre, dsums, n0 + 1, dpre, nullptr);
    if (n0)
        hipLaunchKernelGGL(nc_merge_old_kernel, dim3(grid_for(n0)), dim3(BLOCK), 0, 0, d.key, d.tail, d.status, deflag, dpre,
                           n0, dik, dit, n_ins, key1, tail1, st1, dremap);
    if (n_ins)
        hipLaunchKernelGGL(nc_merge_new_kernel, dim3(grid_for(n_ins)), dim3(BLOCK), 0, 0, d.key, d.tail, deflag, dpre, n0,
                           dik, dit, dist, n_ins, key1, tail1, st1, dnew, derr);
    uint32_t err = 0;
    uint64_t kmin = 0, kmax = 0;
    if (hipGetLastError() != hipSuccess || hipMemcpy(&err, derr, 4, hipMemcpyDeviceToHost) != hipSuccess ||
        (n1 && (hipMemcpy(&kmin, key1, 8, hipMemcpyDeviceToHost) != hipSuccess ||
                hipMemcpy(&kmax, key1 + (n1 - 1), 8, hipMemcpyDeviceToHost) != hipSuccess)))
        return fail(set_err(KAD_ERR_HIP, "NodeCache merge failed"));
    if (err) return fail(set_err(KAD_ERR_INVALID, "insert: an ID is already in the map"));
    // NodeCache radix and lines of the new array
    Radix r;
    uint32_t tb = 1;
    while ((1u << tb) < n1 && tb < 23) tb++;
    if (n1) r = choose_radix(kmin, kmax, tb);
    uint32_t* ncl32 = nullptr;
    // the line sets the table has are rebuilt for the new array; the others stay unbuilt until first use
    const bool has_ncl = t->ncl_mut != nullptr, has_ncl32 = t->ncl32_mut != nullptr;
    if (n1 && ((rc = dev_upload(&rdx1, nullptr, (size_t)r.slots + 1, fresh, freshb)) ||
               (has_ncl && (rc = dev_upload(&ncl1, nullptr, (size_t)(NCL_STRIDE + NCL2_DWORDS) * r.slots, fresh, freshb))) ||
               (has_ncl32 && (rc = dev_upload(&ncl32, nullptr, (size_t)NC32_STRIDE * r.slots, fresh, freshb)))))
        return fail(rc);
    if (n1) {
        hipLaunchKernelGGL(nc_radix_kernel, dim3(grid_for((uint64_t)r.slots + 1)), dim3(BLOCK), 0, 0, key1, n1, r.base,
                           r.shift, r.slots, rdx1);
        if (has_ncl)
            hipLaunchKernelGGL(ncl_build_kernel, dim3(grid_for(r.slots)), dim3(BLOCK), 0, 0, key1, st1, rdx1, r.slots, n1,
                               64 - r.shift, ncl1, LineSel{});
        if (has_ncl32)
            hipLaunchKernelGGL(ncl32_build_kernel, dim3(grid_for(8ull * r.slots)), dim3(BLOCK), 0, 0, key1, st1, rdx1,
                               r.slots, n1, 64 - r.shift, ncl32, LineSel{});
    }
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess)
        return fail(set_err(KAD_ERR_HIP, "NodeCache radix / line build failed"));
    if ((remap && n0 && hipMemcpy(remap, dremap, 4ull * n0, hipMemcpyDeviceToHost) != hipSuccess))
        return fail(set_err(KAD_ERR_HIP, "copy of the remap failed"));
    if (new_index && n_ins) {
        std::vector<uint32_t> sorted_idx(n_ins);
        if (hipMemcpy(sorted_idx.data(), dnew, 4ull * n_ins, hipMemcpyDeviceToHost) != hipSuccess)
            return fail(set_err(KAD_ERR_HIP, "copy of the new indices failed"));
        for (uint32_t j = 0; j < n_ins; j++) new_index[order[j]] = sorted_idx[j];
    }
    for (void* p : tmp) (void)hipFree(p);
    // ---- commit ----
    release(t, const_cast<uint64_t*>(d.key));
    release(t, const_cast<uint32_t*>(d.tail));
    release(t, t->status_mut);
    release(t, const_cast<uint32_t*>(d.nrdx));
    release(t, t->ncl_mut);
    release(t, t->ncl32_mut);
    d.key = key1; d.tail = tail1; d.status = st1; t->status_mut = st1; d.n = n1;
    if (n1) {
        d.nrdx = rdx1; d.nbase = r.base; d.nshift = r.shift; d.nslots = r.slots; t->nbits = r.bits;
        d.ncl = reinterpret_cast<const uint4*>(ncl1); t->ncl_mut = ncl1;
        d.flags = has_ncl ? (d.flags | TF_NCL) : (d.flags & ~TF_NCL);
        d.ncl32 = reinterpret_cast<const uint4*>(ncl32); t->ncl32_mut = ncl32;
        d.flags = has_ncl32 ? (d.flags | TF_NCL32) : (d.flags & ~TF_NCL32);
    } else {
        d.nrdx = nullptr; d.nslots = 0; t->nbits = 0; d.ncl = nullptr; t->ncl_mut = nullptr; d.flags &= ~TF_NCL;
        d.ncl32 = nullptr; t->ncl32_mut = nullptr; d.flags &= ~TF_NCL32;
    }
    release(t, t->wrec); t->wrec = nullptr; t->addr_len = 0;
    release(t, t->time_ns); release(t, t->reply_ns); release(t, t->expired);
    t->time_ns = nullptr; t->reply_ns = nullptr; t->expired = nullptr;
    t->dl.invalidate();
    t->owned.insert(t->owned.end(), fresh.begin(), fresh.end());
    t->bytes += freshb;
    drop_marks(t);
    reset_line_sets(t);
    return KAD_OK;
}

int kad_table_export(const kad_table* t, uint8_t* ids, uint8_t* status, uint8_t* bucket_first, uint32_t* bucket_offset) {
    if (!t) return set_err(KAD_ERR_INVALID, "NULL table");
    DeviceGuard g(t->device);
    const uint32_t n = t->d.n, B = t->d.B;
    if (ids && n) {
        std::vector<uint64_t> k(n);
        std::vector<uint32_t> tl(3ull * n);
        HIP_TRY(hipMemcpy(k.data(), t->d.key, 8ull * n, hipMemcpyDeviceToHost));
        HIP_TRY(hipMemcpy(tl.data(), t->d.tail, 12ull * n, hipMemcpyDeviceToHost));
        for (uint32_t i = 0; i < n; i++) {
            uint8_t* b = ids + 20ull * i;
            for (int x = 0; x < 8; x++) b[x] = (uint8_t)(k[i] >> (56 - 8 * x));
            for (int w = 0; w < 3; w++)
                for (int x = 0; x < 4; x++) b[8 + 4 * w + x] = (uint8_t)(tl[3ull * i + w] >> (24 - 8 * x));
        }
    }
    if (status && n) {
        if (t->mut_async) HIP_TRY(hipEventSynchronize(t->mut_ev));  // after the last asynchronous refresh
        HIP_TRY(hipMemcpy(status, t->d.status, n, hipMemcpyDeviceToHost));
    }
    if (bucket_first && B) std::memcpy(bucket_first, t->h_first.data(), 20ull * B);
    if (bucket_offset && B) std::memcpy(bucket_offset, t->h_off.data(), 4ull * (B + 1));
    return KAD_OK;
}

int kad_table_export_lines(const kad_table* t, uint32_t set, void* out, uint64_t* bytes) {
    if (!t || !bytes) return set_err(KAD_ERR_INVALID, "NULL argument");
    const DevTable& d = t->d;
    const void* src = nullptr;
    uint64_t nb = 0;
    switch (set) {
        case KAD_LINESET_WL: src = d.wl; nb = 128ull * d.B; break;
        case KAD_LINESET_WS: src = d.ws; nb = 64ull * d.B; break;
        case KAD_LINESET_WL16: src = d.wl16; nb = 4ull * WL16_STRIDE * d.B; break;
        case KAD_LINESET_WL32: src = d.wl32; nb = 4ull * WL32_STRIDE * d.B; break;
        case KAD_LINESET_GL: src = d.gl; nb = 4ull * GL_STRIDE * d.B; break;
        case KAD_LINESET_GL16: src = d.gl16; nb = 4ull * GL16_STRIDE * d.B; break;
        case KAD_LINESET_GL32: src = d.gl32; nb = 4ull * GL32_STRIDE * d.B; break;
        case KAD_LINESET_SL: src = d.sl; nb = 64ull * d.slslots; break;
        case KAD_LINESET_SL16: src = d.sl16; nb = 128ull * d.slslots; break;
        case KAD_LINESET_NCL: src = d.ncl; nb = 4ull * (NCL_STRIDE + NCL2_DWORDS) * d.nslots; break;
        case KAD_LINESET_NCL32: src = d.ncl32; nb = 4ull * NC32_STRIDE * d.nslots; break;
        case KAD_LINESET_GCNT: src = d.gcnt; nb = 4ull * d.B; break;
        case KAD_LINESET_DIR: src = d.dir; nb = 8ull * (d.B + 1); break;
        default: return set_err(KAD_ERR_INVALID, "unknown line set %u", set);
    }
    if (!src) nb = 0;
    if (!out) { *bytes = nb; return KAD_OK; }
    if (*bytes < nb) return set_err(KAD_ERR_INVALID, "buffer of %llu bytes for %llu", (unsigned long long)*bytes,
                                    (unsigned long long)nb);
    *bytes = nb;
    if (!nb) return KAD_OK;
    DeviceGuard g(t->device);
    if (t->mut_async) HIP_TRY(hipEventSynchronize(t->mut_ev));
    HIP_TRY(hipMemcpy(out, src, nb, hipMemcpyDeviceToHost));
    return KAD_OK;
}

}  // extern "C"

