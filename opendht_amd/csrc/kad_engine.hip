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
    const uint4* bl;  // bucket lines (TF_BL): 64 bytes per bucket, see rt_bl_kernel
    uint64_t rbase, nbase;
    uint32_t rshift, rslots, nshift, nslots;
    uint32_t n, B, index_base, flags;
};

constexpr uint32_t TF_DIRECT = 1u;   // radix slot s holds exactly bucket s (no locate load)
constexpr uint32_t TF_HAS_DUP = 2u;  // some nodes share their top 64 ID bits
constexpr uint32_t TF_BL = 4u;       // bucket-line layout present (direct-mapped, depth <= 32)
constexpr uint32_t BL_CAP = 14;      // node keys per 64-byte bucket line
constexpr uint32_t BL_OVF = 31;      // n field of a bucket that does not fit its line
constexpr uint32_t BL_OFF_MASK = (1u << 27) - 1;
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

// Is node a strictly before node b in the reference's result order, given equal top-64
// XOR distance? Full-width XOR compare on the tails, then insertion order (= index order
// within one bucket, the only place equal IDs can meet: routing_table.cpp:75-87).
__device__ __forceinline__ bool tail_less(const DevTable& T, const Target& t, uint32_t a, uint32_t b) {
    const uint32_t* ta = T.tail + 3ull * a;
    const uint32_t* tb = T.tail + 3ull * b;
    uint32_t a2 = ta[0] ^ t.t2, a3 = ta[1] ^ t.t3, a4 = ta[2] ^ t.t4;
    uint32_t b2 = tb[0] ^ t.t2, b3 = tb[1] ^ t.t3, b4 = tb[2] ^ t.t4;
    if (a2 != b2) return a2 < b2;
    if (a3 != b3) return a3 < b3;
    if (a4 != b4) return a4 < b4;
    return a < b;
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
    // Exact order: equal top-64 distances fall back to the 96-bit tails, then to the index.
    __device__ __forceinline__ void insert_exact(const DevTable& T, const Target& t, uint64_t cd, uint32_t ci) {
        bool sh = false;
#pragma unroll
        for (int s = 0; s < K; s++) {
            bool lt;
            if (sh) lt = true;
            else if (di[s] == NONE) lt = true;
            else if (cd != dk[s]) lt = cd < dk[s];
            else lt = tail_less(T, t, ci, di[s]);
            sh = lt;
            const uint64_t nd = lt ? dk[s] : cd;
            const uint32_t ni = lt ? di[s] : ci;
            dk[s] = lt ? cd : dk[s];
            di[s] = lt ? ci : di[s];
            cd = nd;
            ci = ni;
        }
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

// Slow path: any window (unbounded rounds, wide buckets), per-node status reads.
template <int K>
__device__ __forceinline__ void rt_query_slow(const DevTable& T, const Target& t, uint32_t b, uint32_t count,
                                           uint32_t* __restrict__ out_row, uint8_t* out_cnt_p) {
    const uint32_t B = T.B;
    uint32_t lo = b > 0 ? b - 1 : 0, hi = b;
    uint32_t good = T.gpre[hi + 1] - T.gpre[lo];
    while (good < count && (lo > 0 || hi < B - 1)) {
        if (hi < B - 1) hi++;
        if (lo > 0) lo--;
        good = T.gpre[hi + 1] - T.gpre[lo];
    }
    const uint2 dl = T.dir[lo], dh = T.dir[hi + 1];
    TopK<K> L;
    L.init();
    const uint32_t beg = dl.x & ~WIDE, end = dh.x & ~WIDE;
    for (uint32_t j = beg; j < end; j++) {
        const uint8_t st = T.status[j];
        if (!(st & KAD_STATUS_GOOD)) continue;
        L.insert_exact(T, t, T.key[j] ^ t.hi, j);
    }
    write_row<K>(L, T, count, min(good, count), out_row, out_cnt_p);
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

// Deferral marker: out_cnt[i] = DEFER_CNT when the caller asked for counts, else row[0] = DEFER_IDX.
constexpr uint8_t DEFER_CNT = 0xFF;
constexpr uint32_t DEFER_IDX = 0xFFFFFFFEu;

__device__ __forceinline__ void mark_deferred(uint32_t* out_row, uint8_t* out_cnt_p) {
    if (out_cnt_p) *out_cnt_p = DEFER_CNT;
    else out_row[0] = DEFER_IDX;
}
__device__ __forceinline__ bool is_deferred(const uint32_t* out_row, const uint8_t* out_cnt_p) {
    return out_cnt_p ? *out_cnt_p == DEFER_CNT : out_row[0] == DEFER_IDX;
}

// ---------------------------------------------------------------------------------------
// Block-cooperative RoutingTable kernel (K = 8, 16). Ranking stays one query per lane, but every
// global read is issued cooperatively so that an instruction touches few lines (a lane-per-query
// load touches 64 distinct lines and keeps the texture-address unit busy), and the block's 256
// queries are counting-sorted by window length so that a wave ranks windows of equal length:
//   1. the block's 256 targets (5 KB, contiguous) -> LDS with 16-byte loads
//   2. bucket per query; directory records of 16 queries per instruction (4 lanes x 16 B each)
//   3. window per query (rt_window); class = number of 8-node chunks (0: done or deferred)
//   4. counting sort of the 256 queries by class (wave ballots), query state -> LDS slot
//   5. per wave: key chunks of 16 queries per instruction (4 lanes x 16 B = one 64-byte line
//      each) -> swizzled LDS tile -> each lane ranks its own query's 8 nodes
//   6. result rows -> LDS in query order -> fully coalesced row stores
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ __forceinline__ uint32_t lane_rank(uint64_t mask) {  // set bits of mask below this lane
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// LDS key tile slot: query j of the wave, 16-byte part x; parts rotated so that the 16 lanes of a
// ds_read_b128 group and the 8 of a ds_write_b128 group hit 16 / 8 distinct bank quads.
__device__ __forceinline__ uint32_t ktile(uint32_t j, uint32_t x) { return j * 4u + (x ^ ((j >> 2) & 3u)); }

template <int K>
__global__ __launch_bounds__(BLOCK) void rt_block_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                         uint32_t count, uint32_t* __restrict__ out_idx,
                                                         uint8_t* __restrict__ out_cnt) {
    static_assert(K <= 16, "block kernel: K <= 16");
    constexpr int P = 2;  // R <= 2 covers all but ~1e-6 of k <= 16 windows on 80%-good uniform tables
    constexpr int NR = 2 * P + 3;
    constexpr int RQ = (NR + 2) / 2;  // 16-byte directory pieces per query (even-aligned cover of NR records)
    constexpr uint32_t NCLS = 9;      // classes 0..8: 8-node chunks per window (MW = 1: <= 64 nodes)
    __shared__ uint4 lds[1024 + 512 + 64 + 32];
    uint4* stage = lds;                                   // 16 KB: targets / directory / key tiles / rows
    uint4* state = lds + 1024;                            // 256 slots x 32 B
    uint32_t* b_arr = reinterpret_cast<uint32_t*>(lds + 1536);
    uint32_t* cls = reinterpret_cast<uint32_t*>(lds + 1600);  // [4][NCLS] counts, then [4][NCLS] starts

    const uint32_t tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const uint32_t q0 = blockIdx.x * BLOCK;
    const uint32_t nq = min((uint32_t)BLOCK, q - q0);
    const bool active = tid < nq;
    const bool trivial = (T.B == 0) | (count == 0);
    const uint32_t B = T.B;

    // 1. targets -> LDS
    {
        const uint32_t* src32 = reinterpret_cast<const uint32_t*>(targets + 20ull * q0);
        if (nq == BLOCK && ((uintptr_t)targets & 15u) == 0) {
            const uint4* src = reinterpret_cast<const uint4*>(src32);
            stage[tid] = src[tid];
            if (tid < 64) stage[256 + tid] = src[256 + tid];
        } else {
            uint32_t* tw = reinterpret_cast<uint32_t*>(stage);
            for (uint32_t k = tid; k < nq * 5; k += BLOCK) tw[k] = src32[k];
        }
    }
    __syncthreads();
    Target t{};
    if (active) {
        const uint32_t* tw = reinterpret_cast<const uint32_t*>(stage) + 5 * tid;
        const uint32_t w0 = __builtin_bswap32(tw[0]), w1 = __builtin_bswap32(tw[1]);
        t.hi = ((uint64_t)w0 << 32) | w1;
        t.t2 = __builtin_bswap32(tw[2]);
        t.t3 = __builtin_bswap32(tw[3]);
        t.t4 = __builtin_bswap32(tw[4]);
    }
    // 2. bucket, then cooperative directory loads (each query's pieces come from its own wave)
    const uint32_t b = (active && !trivial) ? locate_bucket(T, t) : 0u;
    b_arr[tid] = b;
    __syncthreads();  // targets consumed; buckets visible
    if (!trivial) {
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const uint32_t qs = wid * 64 + 16 * i + (lane >> 2), part = lane & 3;
            const uint32_t bq = b_arr[qs];
            const int64_t r0 = (int64_t)bq - (P + 1);
            const int64_t a = r0 & ~(int64_t)1;
            if (part < (uint32_t)RQ && qs < nq && r0 >= 0 && a + 2 * RQ - 1 <= (int64_t)B)
                stage[qs * RQ + part] = reinterpret_cast<const uint4*>(T.dir + a)[part];
        }
    }
    wave_lds_sync();
    Window<K> W{};
    int st = 0;
    if (active && !trivial) {
        uint2 rec[NR];
        const int64_t r0 = (int64_t)b - (P + 1);
        if (r0 >= 0 && (r0 & ~(int64_t)1) + 2 * RQ - 1 <= (int64_t)B) {
            // the query's pieces start at an even record; the odd shift is applied in the LDS address
            const uint2* u = reinterpret_cast<const uint2*>(stage + tid * RQ) + (r0 & 1);
#pragma unroll
            for (int i = 0; i < NR; i++) rec[i] = u[i];
        } else {
            load_recs<P>(T, b, rec);  // first / last buckets of the table: clamped per-lane loads
        }
        st = rt_window<K, P>(T, b, rec, count, W);
    }
    uint8_t* cp_own = (out_cnt && active) ? out_cnt + q0 + tid : nullptr;
    if (active && trivial && cp_own) *cp_own = 0;
    if (st == WIN_DEFER && cp_own) *cp_own = DEFER_CNT;
    // 3/4. counting sort by class
    const uint32_t M = st == WIN_READY ? W.chunks() : 0u;
    uint32_t myrank = 0;
#pragma unroll
    for (uint32_t v = 0; v < NCLS; v++) {
        const uint64_t m = __ballot(M == v);
        if (M == v) myrank = lane_rank(m);
        if (lane == 0) cls[wid * NCLS + v] = (uint32_t)__builtin_popcountll(m);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t acc = 0;
        for (uint32_t v = 0; v < NCLS; v++)
            for (uint32_t w = 0; w < 4; w++) {
                const uint32_t c = cls[w * NCLS + v];
                cls[4 * NCLS + w * NCLS + v] = acc;
                acc += c;
            }
    }
    __syncthreads();
    const uint32_t start1 = cls[4 * NCLS + 1];  // first slot of class 1 (= class-0 population)
    if (M) {
        const uint32_t pos = cls[4 * NCLS + wid * NCLS + M] + myrank;
        state[2 * pos] = make_uint4(q0 + tid, (uint32_t)t.hi, (uint32_t)(t.hi >> 32), W.base);
        state[2 * pos + 1] = make_uint4(W.ne, W.good, (uint32_t)W.gm[0], (uint32_t)(W.gm[0] >> 32));
    }
    __syncthreads();
    // 5. rank: slot tid's query, key tiles loaded cooperatively per wave
    const bool mine = tid >= start1;
    uint32_t qid = 0, sgood = 0;
    Window<K> S{};
    uint64_t th = 0;
    if (mine) {
        const uint4 a0 = state[2 * tid], a1 = state[2 * tid + 1];
        qid = a0.x;
        th = ((uint64_t)a0.z << 32) | a0.y;
        S.base = a0.w;
        S.ne = a1.x;
        sgood = a1.y;
        S.gm[0] = ((uint64_t)a1.w << 32) | a1.z;
    }
    const uint32_t Ms = mine ? S.chunks() : 0u;
    uint32_t lbase[4], lM[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t si = wid * 64 + 16 * i + (lane >> 2);
        const uint4 a0 = state[2 * si], a1 = state[2 * si + 1];
        lbase[i] = a0.w;
        lM[i] = si >= start1 ? (a1.x - a0.w + 7) >> 3 : 0u;
    }
    uint4* tile = stage + wid * 256;
    TopK<K> L;
    L.init();
    bool ones = false;
    for (uint32_t c = 0; __ballot(c < Ms) != 0; c++) {
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (c < lM[i])
                tile[ktile(16 * i + (lane >> 2), lane & 3)] =
                    reinterpret_cast<const uint4*>(T.key + lbase[i] + 8 * c)[lane & 3];
        wave_lds_sync();
        if (c < Ms) {
            uint4 kv[4];
#pragma unroll
            for (int x = 0; x < 4; x++) kv[x] = tile[ktile(lane, x)];
            rank_chunk<K>(L, kv, th, chunk_bits<K>(S, 8 * c), S.base + 8 * c, ones);
        }
        wave_lds_sync();
    }
    // 6. rows -> LDS (query order) -> coalesced stores
    __syncthreads();
    uint32_t* rows = reinterpret_cast<uint32_t*>(stage);
    if (mine) {
        const uint32_t loc = qid - q0;
        if (ones) {
            if (out_cnt) out_cnt[qid] = DEFER_CNT;
            else rows[loc * count] = DEFER_IDX;
        } else {
            const uint32_t m = min(sgood, count);
#pragma unroll
            for (int s2 = 0; s2 < K; s2++)
                if ((uint32_t)s2 < count) rows[loc * count + s2] = (uint32_t)s2 < m ? L.di[s2] + T.index_base : NONE;
            if (out_cnt) out_cnt[qid] = (uint8_t)m;
        }
    }
    if (active && M == 0) {  // trivial (NONE rows) or deferred (marker row when there are no counts)
        for (uint32_t s2 = 0; s2 < count; s2++) rows[tid * count + s2] = NONE;
        if (st == WIN_DEFER && !out_cnt && count) rows[tid * count] = DEFER_IDX;
    }
    __syncthreads();
    uint32_t* dst = out_idx + (size_t)q0 * count;
    for (uint32_t k = tid; k < nq * count; k += BLOCK) dst[k] = rows[k];
}

template <int K>
__global__ __launch_bounds__(BLOCK) void rt_closest_kernel(DevTable T, const uint8_t* __restrict__ targets,
                                                           uint32_t q, uint32_t count,
                                                           uint32_t* __restrict__ out_idx,
                                                           uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    const Target t = load_target(targets, i);
    uint32_t* row = out_idx + (size_t)i * count;
    uint8_t* cp = out_cnt ? out_cnt + i : nullptr;
    if (!rt_query_fast<K, (K > 16 ? 6 : 3)>(T, t, count, row, cp)) mark_deferred(row, cp);
}

// Debug ablation of the lane kernel (KAD_RT_KERNEL=abl1|abl2|abl3): 1 = target + locate + store,
// 2 = + directory window, 3 = + key loads without ranking. Results are garbage; timing only.
template <int K, int ABL>
__global__ __launch_bounds__(BLOCK) void rt_ablate_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                          uint32_t count, uint32_t* __restrict__ out_idx,
                                                          uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    const Target t = load_target(targets, i);
    uint32_t* row = out_idx + (size_t)i * count;
    const uint32_t b = locate_bucket(T, t);
    uint32_t acc = b ^ (uint32_t)t.hi;
    if (ABL >= 2) {
        uint2 rec[7];
        load_recs<2>(T, b, rec);
        Window<K> W;
        const int st = rt_window<K, 2>(T, b, rec, count, W);
        acc += st + W.base + W.ne + (uint32_t)W.gm[0];
        if (ABL >= 3 && st == WIN_READY) {
            const uint4* kp = reinterpret_cast<const uint4*>(T.key + W.base);
            const uint32_t M = W.chunks();
            for (uint32_t c = 0; c < M; c++) {
                uint4 kv[4];
#pragma unroll
                for (int x = 0; x < 4; x++) kv[x] = kp[4 * c + x];
#pragma unroll
                for (int x = 0; x < 4; x++) acc += kv[x].x ^ kv[x].y ^ kv[x].z ^ kv[x].w;
            }
        }
    }
    uint4 v = make_uint4(acc, acc, acc, acc);
    *reinterpret_cast<uint4*>(row) = v;
    *reinterpret_cast<uint4*>(row + 4) = v;
    if (out_cnt) out_cnt[i] = 0;
}

// ---------------------------------------------------------------------------------------
// Bucket-line RoutingTable kernel (direct-mapped tables of uniform depth d <= 32, the U(d) shape).
//
// Random gathers on MI355X cost per 128-byte line touched (~50 G random lines/s whether 32, 64 or
// 128 bytes of it are used: tools/microbench.py), so the window is laid out to touch as few lines
// as possible. Each bucket is one 64-byte record:
//   w0 = first node index (27 bits) | n << 27 (n = BL_OVF if the bucket does not fit)
//   w1 = good bitmask (bits 0..13) | "needs the exact compare" bitmask (bits 16..29)
//   w2..w15 = key32 of each node = ID bits [d, d + 32), right after the bucket's d-bit prefix.
// The round-0 window {b-1, b} is 128 contiguous bytes. Buckets are dyadic, so a node's XOR distance
// is ordered by (bucket prefix XOR target prefix, key32 XOR target bits [d, d+32)): that 64-bit
// rank key is exact in the top d+32 distance bits; two nodes can tie only inside one bucket on
// equal key32, and those nodes carry the exact-compare bit (the query is deferred).
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t bl_key_word(const uint4& a, const uint4& b, const uint4& c, const uint4& e, int s) {
    switch (s) {  // slot s lives in dword 2 + s of the line (static after unrolling)
        case 0: return a.z; case 1: return a.w;
        case 2: return b.x; case 3: return b.y; case 4: return b.z; case 5: return b.w;
        case 6: return c.x; case 7: return c.y; case 8: return c.z; case 9: return c.w;
        case 10: return e.x; case 11: return e.y; case 12: return e.z; default: return e.w;
    }
}

// One bucket line held in registers, with its rank-relevant values.
struct BlLine {
    uint4 v[4];
    uint32_t gm, off, good;  // good bitmask, first node index, good count
    uint64_t D;              // bucket prefix XOR target prefix (orders whole buckets)
    bool present;
};

__device__ __forceinline__ void bl_load(const DevTable& T, uint32_t w, BlLine& L) {
    const uint4* p = T.bl + 4ull * w;
#pragma unroll
    for (int x = 0; x < 4; x++) L.v[x] = p[x];
}

__device__ __forceinline__ void bl_header(BlLine& L, uint64_t D, bool present, bool& bad) {
    L.present = present;
    L.D = D;
    const uint32_t nf = L.v[0].x >> 27, xm = L.v[0].y >> 16;
    L.gm = present ? (L.v[0].y & 0xFFFFu) : 0u;
    L.off = L.v[0].x & BL_OFF_MASK;
    L.good = __builtin_popcount(L.gm);
    bad |= present & ((nf == BL_OVF) | ((L.gm & xm) != 0));
}

// Rank every good node of line L among the good nodes of its own bucket (32-bit keys suffice: the
// nodes of one bucket share its prefix) and place it at base + rank among the K output slots.
template <int K>
__device__ __forceinline__ void bl_place(const BlLine& L, uint32_t base, uint32_t t32, uint32_t (&out)[K]) {
    uint32_t k[BL_CAP];
#pragma unroll
    for (int s2 = 0; s2 < (int)BL_CAP; s2++) k[s2] = bl_key_word(L.v[0], L.v[1], L.v[2], L.v[3], s2) ^ t32;
    uint32_t ns = 0;  // one past the highest good slot over the wave: bounds both loops
#pragma unroll
    for (int s2 = 0; s2 < (int)BL_CAP; s2++) ns = __any((L.gm >> s2) != 0) ? (uint32_t)s2 + 1 : ns;
#pragma unroll
    for (int s2 = 0; s2 < (int)BL_CAP; s2++) {
        if ((uint32_t)s2 >= ns) break;
        uint32_t r = base;
#pragma unroll
        for (int u = 0; u < (int)BL_CAP; u++) {
            if ((uint32_t)u >= ns) break;
            r += ((L.gm >> u) & 1u) & (uint32_t)(k[u] < k[s2]);
        }
        const bool g = (L.gm >> s2) & 1u;
#pragma unroll
        for (int j = 0; j < K; j++) out[j] = (g & (r == (uint32_t)j)) ? L.off + s2 : out[j];
    }
}

template <int K>
__global__ __launch_bounds__(BLOCK) void rt_bl_kernel(DevTable T, const uint8_t* __restrict__ targets, uint32_t q,
                                                      uint32_t count, uint32_t* __restrict__ out_idx,
                                                      uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    uint32_t* row = out_idx + (size_t)i * count;
    uint8_t* cp = out_cnt ? out_cnt + i : nullptr;
    if (count == 0) {
        if (cp) *cp = 0;
        return;
    }
    const Target t = load_target(targets, i);
    const uint32_t B = T.B, d = 64 - T.rshift;
    const uint32_t b = locate_bucket(T, t);
    const uint64_t pre0 = T.rbase >> T.rshift, tp = t.hi >> T.rshift;
    const uint32_t t32 = (uint32_t)((t.hi << d) >> 32);
    bool bad = false;
    // Round 0 window {b-1, b}: both lines in flight together. Round 1 adds {b-2, b+1}; later
    // rounds (~0.3% of k=8 queries on an 80%-good U(24) shard) are deferred.
    BlLine Lb, Ll, Lh, Ll2;
    const bool hasl = b > 0;
    bl_load(T, b, Lb);
    bl_load(T, hasl ? b - 1 : b, Ll);
    bl_header(Lb, (pre0 + b) ^ tp, true, bad);
    bl_header(Ll, (pre0 + b - 1) ^ tp, hasl, bad);
    uint32_t good = Lb.good + Ll.good;
    const bool whole0 = (b <= 1) & (b >= B - 1);
    const bool r1 = (good < count) & !whole0;
    const bool hash = r1 & (b + 1 < B), hasl2 = r1 & (b >= 2);
    if (r1) {
        bl_load(T, hash ? b + 1 : b, Lh);
        bl_load(T, hasl2 ? b - 2 : b, Ll2);
    }
    bl_header(Lh, (pre0 + b + 1) ^ tp, hash, bad);
    bl_header(Ll2, (pre0 + b - 2) ^ tp, hasl2, bad);
    good += Lh.good + Ll2.good;
    const bool whole1 = (b <= 2) & (b + 1 >= B - 1);
    bad |= r1 & (good < count) & !whole1;
    if (bad) {
        mark_deferred(row, cp);
        return;
    }
    // whole buckets are ordered by D (the XOR images of disjoint dyadic buckets are disjoint intervals)
    auto base_of = [&](const BlLine& X) {
        return (Ll.present & (Ll.D < X.D) ? Ll.good : 0u) + (Lb.D < X.D ? Lb.good : 0u) +
               (Lh.present & (Lh.D < X.D) ? Lh.good : 0u) + (Ll2.present & (Ll2.D < X.D) ? Ll2.good : 0u);
    };
    uint32_t out[K];
#pragma unroll
    for (int j = 0; j < K; j++) out[j] = NONE;
    bl_place<K>(Lb, base_of(Lb), t32, out);
    bl_place<K>(Ll, base_of(Ll), t32, out);
    if (__any(r1)) {
        bl_place<K>(Lh, base_of(Lh), t32, out);
        bl_place<K>(Ll2, base_of(Ll2), t32, out);
    }
    const uint32_t m = min(good, count);
    if (count == (uint32_t)K && (K % 4) == 0) {
#pragma unroll
        for (int j = 0; j < K; j += 4)
            *reinterpret_cast<uint4*>(row + j) =
                make_uint4((uint32_t)j < m ? out[j] + T.index_base : NONE,
                           (uint32_t)j + 1 < m ? out[j + 1] + T.index_base : NONE,
                           (uint32_t)j + 2 < m ? out[j + 2] + T.index_base : NONE,
                           (uint32_t)j + 3 < m ? out[j + 3] + T.index_base : NONE);
    } else {
#pragma unroll
        for (int j = 0; j < K; j++)
            if ((uint32_t)j < count) row[j] = (uint32_t)j < m ? out[j] + T.index_base : NONE;
    }
    if (cp) *cp = (uint8_t)m;
}

// Good bitmasks of the bucket lines after a status change (exact-compare bits are kept).
__global__ void bl_good_kernel(const uint8_t* status, uint4* bl, uint32_t B) {
    const uint32_t b = blockIdx.x * BLOCK + threadIdx.x;
    if (b >= B) return;
    uint4 h = bl[4ull * b];
    const uint32_t off = h.x & BL_OFF_MASK, nf = h.x >> 27;
    if (nf == BL_OVF) return;
    uint32_t gm = 0;
    for (uint32_t s2 = 0; s2 < nf; s2++) gm |= (uint32_t)(status[off + s2] & KAD_STATUS_GOOD) << s2;
    h.y = (h.y & 0xFFFF0000u) | gm;
    bl[4ull * b] = h;
}

// Second pass over the batch: the (rare) queries the fast kernel deferred, exact per-node path.
template <int K>
__global__ __launch_bounds__(BLOCK) void rt_closest_deferred_kernel(DevTable T, const uint8_t* __restrict__ targets,
                                                                    uint32_t q, uint32_t count,
                                                                    uint32_t* __restrict__ out_idx,
                                                                    uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    uint32_t* row = out_idx + (size_t)i * count;
    uint8_t* cp = out_cnt ? out_cnt + i : nullptr;
    if (!is_deferred(row, cp)) return;
    const Target t = load_target(targets, i);
    rt_query_slow<K>(T, t, locate_bucket(T, t), count, row, cp);
}

template <int K>
__global__ __launch_bounds__(BLOCK) void rt_closest_dual_kernel(DevTable T4, DevTable T6,
                                                                const uint8_t* __restrict__ targets,
                                                                const uint8_t* __restrict__ af, uint32_t q,
                                                                uint32_t count, uint32_t* __restrict__ out_idx,
                                                                uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    const Target t = load_target(targets, i);
    const DevTable& T = af[i] ? T6 : T4;
    uint32_t* row = out_idx + (size_t)i * count;
    uint8_t* cp = out_cnt ? out_cnt + i : nullptr;
    if (!rt_query_fast<K, (K > 16 ? 6 : 3)>(T, t, count, row, cp)) mark_deferred(row, cp);
}

template <int K>
__global__ __launch_bounds__(BLOCK) void rt_closest_dual_deferred_kernel(DevTable T4, DevTable T6,
                                                                         const uint8_t* __restrict__ targets,
                                                                         const uint8_t* __restrict__ af, uint32_t q,
                                                                         uint32_t count, uint32_t* __restrict__ out_idx,
                                                                         uint8_t* __restrict__ out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    uint32_t* row = out_idx + (size_t)i * count;
    uint8_t* cp = out_cnt ? out_cnt + i : nullptr;
    if (!is_deferred(row, cp)) return;
    const Target t = load_target(targets, i);
    const DevTable& T = af[i] ? T6 : T4;
    rt_query_slow<K>(T, t, locate_bucket(T, t), count, row, cp);
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

// KAD_RT_KERNEL=lane (default) | block | bl | abl1..3 selects the RoutingTable kernel variant (A/B
// benching, tools/ab_bench.py); read per call so one process can time several.
bool force_lane() {
    const char* e = std::getenv("KAD_RT_KERNEL");
    return !e || std::strcmp(e, "block") != 0;
}

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
    uint4* bl_mut = nullptr;
    int64_t* time_ns = nullptr;
    int64_t* reply_ns = nullptr;
    uint8_t* expired = nullptr;
    uint32_t* scan_cnt = nullptr;   // B+1
    uint32_t* scan_part = nullptr;  // B+1
    uint32_t* scan_sums = nullptr;  // tiles
    ~kad_table() {
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
    if (t->bl_mut) hipLaunchKernelGGL(bl_good_kernel, dim3(grid_for(B)), dim3(BLOCK), 0, s, t->d.status, t->bl_mut, B);
    HIP_TRY(hipGetLastError());
    return KAD_OK;
}

int check_count(uint32_t count) {
    if (count > KAD_MAX_COUNT) return set_err(KAD_ERR_UNSUPPORTED, "count %u > KAD_MAX_COUNT (%u)", count, KAD_MAX_COUNT);
    return KAD_OK;
}

template <int K>
void launch_rt(const DevTable& d, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out, uint8_t* cnt,
               hipStream_t s) {
    const char* ev = std::getenv("KAD_RT_KERNEL");
    if (K == 8 && ev && std::strncmp(ev, "abl", 3) == 0) {
        const int a = ev[3] - '0';
        if (a == 1) hipLaunchKernelGGL((rt_ablate_kernel<8, 1>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        if (a == 2) hipLaunchKernelGGL((rt_ablate_kernel<8, 2>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        if (a == 3) hipLaunchKernelGGL((rt_ablate_kernel<8, 3>), dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
        return;
    }
    if ((d.flags & TF_BL) && ev && std::strcmp(ev, "bl") == 0)
        hipLaunchKernelGGL(rt_bl_kernel<K>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    else if (K <= 16 && !force_lane())
        hipLaunchKernelGGL(rt_block_kernel<(K <= 16 ? K : 16)>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count,
                           out, cnt);
    else
        hipLaunchKernelGGL(rt_closest_kernel<K>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out, cnt);
    hipLaunchKernelGGL(rt_closest_deferred_kernel<K>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d, targets, q, count, out,
                       cnt);
}
template <int K>
void launch_rt_dual(const DevTable& d4, const DevTable& d6, const uint8_t* targets, const uint8_t* af, uint32_t q,
                    uint32_t count, uint32_t* out, uint8_t* cnt, hipStream_t s) {
    hipLaunchKernelGGL(rt_closest_dual_kernel<K>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q, count,
                       out, cnt);
    hipLaunchKernelGGL(rt_closest_dual_deferred_kernel<K>, dim3(grid_for(q)), dim3(BLOCK), 0, s, d4, d6, targets, af, q,
                       count, out, cnt);
}

int rt_dispatch(const DevTable& d, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t* out, uint8_t* cnt,
                hipStream_t s) {
    if (count <= 8) launch_rt<8>(d, targets, q, count, out, cnt, s);
    else if (count <= 16) launch_rt<16>(d, targets, q, count, out, cnt, s);
    else launch_rt<32>(d, targets, q, count, out, cnt, s);
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
        // bucket lines for direct-mapped tables of depth <= 32 (see rt_bl_kernel)
        const uint32_t depth = 64 - r.shift;
        if (direct && depth >= 1 && depth <= 32 && n_nodes <= BL_OFF_MASK) {
            std::vector<uint32_t> bl(16ull * n_buckets, 0u);
            const uint64_t pre0 = r.base >> r.shift;
            for (uint32_t b = 0; b < n_buckets; b++) {
                uint32_t* L = &bl[16ull * b];
                const uint32_t j0 = bucket_offset[b], j1 = bucket_offset[b + 1], nb = j1 - j0;
                bool fits = nb <= BL_CAP;
                for (uint32_t j = j0; j < j1 && fits; j++) fits = (id_hi(ids + 20ull * j) >> r.shift) == pre0 + b;
                L[0] = j0 | ((fits ? nb : BL_OVF) << 27);
                if (!fits) continue;
                uint32_t gm = 0, xm = 0;
                for (uint32_t s2 = 0; s2 < nb; s2++) {
                    const uint64_t hi = id_hi(ids + 20ull * (j0 + s2));
                    L[2 + s2] = (uint32_t)((hi << depth) >> 32);
                    gm |= (uint32_t)(status[j0 + s2] & KAD_STATUS_GOOD) << s2;
                }
                for (uint32_t a = 0; a < nb; a++)
                    for (uint32_t c = a + 1; c < nb; c++)
                        if (L[2 + a] == L[2 + c]) xm |= (1u << a) | (1u << c);
                L[1] = gm | (xm << 16);
            }
            uint4* dbl;
            if ((rc = dev_upload(&dbl, bl.data(), 4ull * n_buckets, t->owned, t->bytes))) { delete t; return rc; }
            d.bl = dbl;
            t->bl_mut = dbl;
            d.flags |= TF_BL;
        }
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
    return rt_dispatch(t->d, targets, q, count, out_idx, out_cnt, (hipStream_t)stream);
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
