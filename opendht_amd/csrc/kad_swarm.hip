// kad_swarm.hip — config 5: a simulated swarm of n peers, each with its
// own shape-K routing table in HBM, and synchronous-round iterative lookups over it.
//
// BUILD-DEFINED MODEL (the reference has no swarm simulator); parity is pinned per hop against the
// oracle's restatement (oracle/kad_oracle.cpp "Config 5 swarm model"):
//   * peer tables of shape K (Dht::onNewNode, dht.cpp:867-936: only my bucket splits, a full bucket
//     caches newcomers away): peer p of top-64 key k has depth D = the least D with at most 8 other
//     peers sharing >= D leading bits (capped at KAD_SWARM_LEVELS-1); level d < D holds min(8, |S_d|)
//     peers of S_d (peers sharing exactly d bits) at positions lo + (off + j|S_d|/8) % |S_d|,
//     off = mix(k ^ (d+1)*GOLDEN) % |S_d|; my bucket (level D) the first 8 other peers sharing >= D
//     bits. All peers good.
//   * a hop queries the first <= 4 unqueried nodes of a search's list (MAX_REQUESTED_SEARCH_NODES,
//     dht.h:327); each answers RoutingTable::findClosestNodes(t, 8) (routing_table.cpp:67-111) from
//     its own table; answers equal to the source are dropped (network_engine.cpp:798-799); the rest
//     go through Search::insertNode (dht.cpp:961-1047: sorted insert, trim to SEARCH_NODES = 14).
//     Done when the first min(8, |list|) nodes have been queried (Search::isSynced, dht.cpp:1467-1478);
//     stalled when no unqueried node is left.
//
// HBM layout (n peers, L = KAD_SWARM_LEVELS levels, 8 entries per bucket):
//   key[n] u64 (ID bits 0..63 of the sorted peer IDs), tail[n][3] u32 (bits 64..159, exact ties only)
//   hdr[n]: one 64-byte line (key, depth D, the L level counts); lvl[n][L]: one 128-byte line per bucket (the 8
//   entries' peer indices, then their keys inline), so a findClosestNodes reads the header and one line per window
//   bucket and does no per-node gathers
// A peer's buckets sorted by `first` (the RoutingTable order) follow from k's bits: the levels whose
// bit of k is 1 (their bucket lies below k) in ascending d, my bucket, then the levels whose bit is
// 0 in descending d. The bucket holding a target is level commonBits(k, t) (or my bucket).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstdarg>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kadgpu.h"

namespace kadgpu_internal {
int set_error(int code, const char* msg);
bool device_ok(int dev);
}  // namespace kadgpu_internal

namespace {

constexpr uint32_t NONE = 0xFFFFFFFFu;
constexpr uint32_t L = KAD_SWARM_LEVELS;
constexpr uint32_t BK = 8;   // TARGET_NODES per bucket
constexpr uint32_t SN = 14;  // SEARCH_NODES (dht.h:314)
constexpr uint32_t SNP = 16; // per-peer answer width (count <= 16)
constexpr uint32_t LST = KAD_SEARCH_LIST;  // search list capacity: SEARCH_NODES non-bad nodes + the bad ones
constexpr uint32_t MAX_BAD = 25;           // SEARCH_MAX_BAD_NODES (dht.h:316-324)
constexpr uint32_t ALPHA = 4;
#ifndef SW_NARROW_WPE
#define SW_NARROW_WPE 1
#endif
#ifndef SW_QUERY_WPE
#define SW_QUERY_WPE 1
#endif
constexpr int BLOCK = 256;

int err(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    return kadgpu_internal::set_error(code, buf);
}

#define SW_TRY(expr)                                                                          \
    do {                                                                                      \
        hipError_t e_ = (expr);                                                               \
        if (e_ != hipSuccess) return err(KAD_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

inline uint32_t grid_for(uint64_t n) { return (uint32_t)((n + BLOCK - 1) / BLOCK); }

// A peer's table as one 64-byte header line (HDR_WORDS: its key, depth and the L level counts) and one 128-byte line
// per level (LVL_WORDS: the 8 entries' keys, then the rule giving their peer indices — a bucket's entries are a run of
// the sorted peers or an even sample of one: first index a, run length m, sample offset, and the index skipped in my
// own bucket (mine) — then the indices themselves for the host): a findClosestNodes on a peer's table reads the
// header and the first 80 bytes of one line per window bucket, 3 random lines for the usual 2-bucket window, where
// separate key, depth, count, index and key arrays took 7 (the query kernel is bound by its random line requests).
constexpr uint32_t HDR_WORDS = 16, LVL_WORDS = 32;  // header: dw0-1 key, byte 8 depth, bytes 16.. counts
constexpr uint32_t LVL_RULE = 16, LVL_IDX = 20;      // level line: dw 0-15 keys, 16-19 index rule, 20-27 indices

// Entry j's peer index from a level line's rule (a, m, off, skip) — the build's choice (swarm_build_kernel): a run of
// m <= 8 sorted peers from a, or my own bucket's run from a without me (skip), or 8 evenly spaced of m > 8 from an
// offset: a + (off + j m / 8) mod m, where off < m and j m / 8 < m make the mod one subtraction.
__device__ __forceinline__ uint32_t lvl_index(const uint4& r, uint32_t j) {
    if (r.y <= 8u || r.w != 0xFFFFFFFFu) {
        const uint32_t x = r.x + j;
        return x + (x >= r.w ? 1u : 0u);
    }
    const uint32_t o = r.z + (uint32_t)(((uint64_t)j * r.y) >> 3);
    return r.x + (o >= r.y ? o - r.y : o);
}
struct SwarmDev {
    const uint64_t* key;
    const uint32_t* tail;
    uint32_t* hdr;  // [n][HDR_WORDS]
    uint32_t* lvl;  // [n][L][LVL_WORDS]: dw 0-15 keys (lo, hi), dw 16-19 the index rule, dw 20-27 indices, 28-31 zero
    uint32_t n;
};

struct Tgt {
    uint64_t hi;
    uint32_t t2, t3, t4;
};

__device__ __forceinline__ Tgt load_tgt(const uint8_t* targets, uint32_t i) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(targets + 20ull * i);
    Tgt t;
    t.hi = ((uint64_t)__builtin_bswap32(p[0]) << 32) | __builtin_bswap32(p[1]);
    t.t2 = __builtin_bswap32(p[2]);
    t.t3 = __builtin_bswap32(p[3]);
    t.t4 = __builtin_bswap32(p[4]);
    return t;
}

__device__ __forceinline__ uint64_t mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

__device__ __forceinline__ uint32_t lower_bound(const uint64_t* key, uint32_t n, uint64_t v) {
    uint32_t lo = 0, hi = n;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (key[mid] < v) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// peers whose key starts with the Lb-bit prefix P (Lb <= 63): [lo, hi)
__device__ __forceinline__ void prefix_range(const SwarmDev& W, uint64_t P, uint32_t Lb, uint32_t& lo, uint32_t& hi) {
    if (Lb == 0) { lo = 0; hi = W.n; return; }
    lo = lower_bound(W.key, W.n, P << (64 - Lb));
    hi = (P + 1 == (1ull << Lb)) ? W.n : lower_bound(W.key, W.n, (P + 1) << (64 - Lb));
}

// One thread per peer: depth, level buckets, my bucket (see the header).
__global__ void swarm_build_kernel(SwarmDev W) {
    const uint32_t p = blockIdx.x * BLOCK + threadIdx.x;
    if (p >= W.n) return;
    const uint64_t k = W.key[p];
    uint32_t D = 0, lo = 0, hi = W.n;
    for (;; D++) {
        prefix_range(W, D ? k >> (64 - D) : 0ull, D, lo, hi);
        if (hi - lo - 1 <= BK || D == L - 1) break;
    }
    uint32_t* hp = W.hdr + (size_t)p * HDR_WORDS;
    uint8_t cp[L];
    for (uint32_t d = 0; d < L; d++) cp[d] = 0;
    // a level line: 8 keys, the index rule (lvl_index), 8 indices, padding
    auto put = [&](uint32_t d, const uint32_t (&ei)[BK], uint32_t a, uint32_t m, uint32_t off, uint32_t skip) {
        uint32_t* lp = W.lvl + ((size_t)p * L + d) * LVL_WORDS;
        for (uint32_t j = 0; j < BK; j++) {
            const uint64_t kk = ei[j] != NONE ? W.key[ei[j]] : ~0ull;
            lp[2 * j] = (uint32_t)kk;
            lp[2 * j + 1] = (uint32_t)(kk >> 32);
            lp[LVL_IDX + j] = ei[j];
        }
        lp[LVL_RULE] = a;
        lp[LVL_RULE + 1] = m;
        lp[LVL_RULE + 2] = off;
        lp[LVL_RULE + 3] = skip;
        for (uint32_t j = LVL_IDX + BK; j < LVL_WORDS; j++) lp[j] = 0;
    };
    for (uint32_t d = 0; d < L; d++) {
        uint32_t ei[BK], ra = 0, rm = 0, roff = 0, rskip = NONE;
        for (uint32_t j = 0; j < BK; j++) ei[j] = NONE;
        if (d < D) {
            uint32_t a, e;
            prefix_range(W, (k >> (63 - d)) ^ 1ull, d + 1, a, e);
            const uint32_t m = e - a, c = min(m, BK);
            const uint64_t off = m > BK ? mix(k ^ ((uint64_t)(d + 1) * 0x9E3779B97F4A7C15ull)) % m : 0ull;
            for (uint32_t j = 0; j < c; j++) ei[j] = m > BK ? a + (uint32_t)((off + (uint64_t)j * m / BK) % m) : a + j;
            cp[d] = (uint8_t)c;
            ra = a;
            rm = m;
            roff = (uint32_t)off;
        } else if (d == D) {
            uint32_t c = 0;
            for (uint32_t x = lo; x < hi && c < BK; x++)
                if (x != p) ei[c++] = x;
            cp[D] = (uint8_t)c;
            ra = lo;
            rm = hi - lo;
            rskip = p;
        }
        put(d, ei, ra, rm, roff, rskip);  // (levels past my bucket: empty lines)
    }
    hp[0] = (uint32_t)k;
    hp[1] = (uint32_t)(k >> 32);
    hp[2] = D;
    hp[3] = 0;
    for (uint32_t w = 0; w < HDR_WORDS - 4; w++) {
        uint32_t v = 0;
        for (uint32_t b = 0; b < 4; b++)
            if (4 * w + b < L) v |= (uint32_t)cp[4 * w + b] << (8 * b);
        hp[4 + w] = v;
    }
}
static_assert(L <= 4 * (HDR_WORDS - 4), "the level counts fit the header line");

// The i-th set bit (ascending) of m (i < popcount(m)).
__device__ __forceinline__ uint32_t nth_bit(uint32_t m, uint32_t i) {
    for (uint32_t k = 0; k < i; k++) m &= m - 1;
    return (uint32_t)__builtin_ctz(m);
}

// Exact order of two candidates with equal top-64 distance: the 96-bit tail XOR the target's tail.
__device__ __forceinline__ bool tail_less(const SwarmDev& W, const Tgt& t, uint32_t a, uint32_t b) {
    const uint32_t* ta = W.tail + 3ull * a;
    const uint32_t* tb = W.tail + 3ull * b;
    const uint32_t a2 = ta[0] ^ t.t2, a3 = ta[1] ^ t.t3, a4 = ta[2] ^ t.t4;
    const uint32_t b2 = tb[0] ^ t.t2, b3 = tb[1] ^ t.t3, b4 = tb[2] ^ t.t4;
    if (a2 != b2) return a2 < b2;
    if (a3 != b3) return a3 < b3;
    return a4 < b4;
}

// (key, id) compare-exchange: the smaller key first (equal keys stay: the caller sends ties to the sequential form)
__device__ __forceinline__ void cx_kid(uint64_t& ka, uint32_t& ia, uint64_t& kb, uint32_t& ib) {
    const bool sw = kb < ka;
    const uint64_t k0 = sw ? kb : ka, k1 = sw ? ka : kb;
    const uint32_t i0 = sw ? ib : ia, i1 = sw ? ia : ib;
    ka = k0; kb = k1; ia = i0; ib = i1;
}

// Batcher's odd-even merge sort of 8 (key, id) pairs, 19 compare-exchanges
__device__ __forceinline__ void sort8_kid(uint64_t (&bk)[BK], uint32_t (&bi)[BK]) {
    cx_kid(bk[0], bi[0], bk[1], bi[1]); cx_kid(bk[2], bi[2], bk[3], bi[3]);
    cx_kid(bk[4], bi[4], bk[5], bi[5]); cx_kid(bk[6], bi[6], bk[7], bi[7]);
    cx_kid(bk[0], bi[0], bk[2], bi[2]); cx_kid(bk[1], bi[1], bk[3], bi[3]);
    cx_kid(bk[4], bi[4], bk[6], bi[6]); cx_kid(bk[5], bi[5], bk[7], bi[7]);
    cx_kid(bk[1], bi[1], bk[2], bi[2]); cx_kid(bk[5], bi[5], bk[6], bi[6]);
    cx_kid(bk[0], bi[0], bk[4], bi[4]); cx_kid(bk[1], bi[1], bk[5], bi[5]);
    cx_kid(bk[2], bi[2], bk[6], bi[6]); cx_kid(bk[3], bi[3], bk[7], bi[7]);
    cx_kid(bk[2], bi[2], bk[4], bi[4]); cx_kid(bk[3], bi[3], bk[5], bi[5]);
    cx_kid(bk[1], bi[1], bk[2], bi[2]); cx_kid(bk[3], bi[3], bk[4], bi[4]); cx_kid(bk[5], bi[5], bk[6], bi[6]);
}

// RoutingTable::findClosestNodes(t, count) on peer p's table, count <= K. Writes the result's peer
// indices and keys (sorted by XOR distance) and returns their number.
// NET (K = 8): the window's nodes ranked by a sorting network instead of one insert each: each bucket's 8 slots are
// sorted (19 compare-exchanges) and merged with the running top 8 (a bitonic half-cleaner and three levels), ~250 VALU
// operations a bucket where the inserts took ~100 a node. The network orders by the top 64 bits of the distance only,
// so a result whose order or cut needs the 160-bit tails (two of its distances equal, or its last equal to the
// nearest node left out) returns TIE and the caller ranks it again with inserts (NET = false).
constexpr uint32_t TIE = 0xFFFFFFFFu;
template <uint32_t K, bool NET = false>
__device__ uint32_t peer_closest(const SwarmDev& W, uint32_t p, const Tgt& t, uint32_t count, uint32_t* oi, uint64_t* ok) {
    const uint32_t* hp = W.hdr + (size_t)p * HDR_WORDS;
    // key, depth and the level counts: the header line's first 48 bytes in one round of 16-byte loads, so the window
    // rounds below read counts from registers, not one dependent cache round trip each
    const uint4 h0 = reinterpret_cast<const uint4*>(hp)[0], h1 = reinterpret_cast<const uint4*>(hp)[1],
                h2 = reinterpret_cast<const uint4*>(hp)[2];
    const uint64_t k = ((uint64_t)h0.y << 32) | h0.x;
    const uint32_t D = h0.z;
    static_assert(L <= 32, "the counts are header bytes 16..47");
    const uint32_t cw[8] = {h1.x, h1.y, h1.z, h1.w, h2.x, h2.y, h2.z, h2.w};
    auto cnt = [&](uint32_t d) -> uint32_t {  // (a select chain: the words stay in registers)
        uint32_t w = cw[0];
#pragma unroll
        for (uint32_t y = 1; y < (L + 3) / 4; y++) w = (d >> 2) == y ? cw[y] : w;
        return (w >> (8 * (d & 3u))) & 255u;
    };
    const uint32_t lv = (uint32_t)(__builtin_bitreverse64(k) & ((1ull << D) - 1));  // bit d = bit d of k from the top
    const uint32_t m1 = lv, m0 = ~lv & (uint32_t)((1ull << D) - 1);
    const uint32_t M = (uint32_t)__builtin_popcount(m1), B = D + 1;
    // position of the target's bucket
    const uint64_t x = k ^ t.hi;
    const uint32_t c = x ? (uint32_t)__builtin_clzll(x) : 64u;
    uint32_t b;
    if (c >= D) b = M;
    else if ((m1 >> c) & 1u) b = (uint32_t)__builtin_popcount(m1 & ((1u << c) - 1u));
    else b = M + 1 + (uint32_t)__builtin_popcount(m0 & ~((2u << c) - 1u));
    // level of a position
    const uint32_t n0 = (uint32_t)__builtin_popcount(m0);
    auto level = [&](uint32_t P) -> uint32_t {
        if (P < M) return nth_bit(m1, P);
        if (P == M) return D;
        return nth_bit(m0, n0 - 1 - (P - M - 1));
    };
    // window rounds (routing_table.cpp:89-104)
    uint32_t lo = b > 0 ? b - 1 : 0, hi = b, good = cnt(level(b)) + (b > 0 ? cnt(level(b - 1)) : 0u);
    while (good < count && !(lo == 0 && hi == B - 1)) {
        if (hi < B - 1) { hi++; good += cnt(level(hi)); }
        if (lo > 0) { lo--; good += cnt(level(lo)); }
    }
    // top-count of the window's nodes by (XOR distance, insertion order)
    uint64_t L0[K];
    uint32_t LI[K];
#pragma unroll
    for (uint32_t s = 0; s < K; s++) { L0[s] = ~0ull; LI[s] = NONE; }
    uint32_t nl = 0;
    uint64_t nin = ~0ull;  // (NET) the nearest node left out
    bool tie = false;
    static_assert(!NET || K == BK, "the network ranks 8");
    static_assert(BK == 8, "a level's slots are four 16-byte key loads and one 16-byte index rule");
    // a level's 8 slots in one round of 16-byte loads (the slots from its count on are padding, skipped); the next
    // window bucket's slots are loaded before the current one's are ranked, so the window costs one round trip, not
    // one per bucket
    struct Slots {
        uint64_t k[BK];
        uint4 rule;
        uint32_t nb;
    };
    auto load_level = [&](uint32_t P, Slots& S) {
        const uint32_t d = level(P);
        S.nb = cnt(d);
        const uint4* kp4 = reinterpret_cast<const uint4*>(W.lvl + ((size_t)p * L + d) * LVL_WORDS);
        S.rule = kp4[LVL_RULE / 4];
#pragma unroll
        for (int x = 0; x < 4; x++) {
            const uint4 u = kp4[x];
            S.k[2 * x] = ((uint64_t)u.y << 32) | u.x;
            S.k[2 * x + 1] = ((uint64_t)u.w << 32) | u.z;
        }
    };
    Slots cur, nxt;
    load_level(lo, cur);
    for (uint32_t P = lo; P <= hi; P++) {
        if (P < hi) load_level(P + 1, nxt);
        const uint32_t nb = cur.nb;
        const uint64_t* ek = cur.k;
        if constexpr (NET) {  // (in place in cur's registers; the first bucket merges with an empty top as well)
            uint32_t ej[BK];  // the slots travel through the network, their peer indices are derived after it
#pragma unroll
            for (uint32_t j = 0; j < BK; j++) {
                cur.k[j] = j < nb ? cur.k[j] ^ t.hi : ~0ull;
                ej[j] = j;
                tie |= j < nb && cur.k[j] == ~0ull;  // (a node as far as the padding)
            }
            sort8_kid(cur.k, ej);
#pragma unroll
            for (uint32_t s = 0; s < K; s++) {  // the 8 smallest of (top ascending, bucket descending)
                const bool sw = cur.k[K - 1 - s] < L0[s];
                nin = min(nin, sw ? L0[s] : cur.k[K - 1 - s]);
                L0[s] = sw ? cur.k[K - 1 - s] : L0[s];
                LI[s] = sw ? (cur.k[K - 1 - s] != ~0ull ? lvl_index(cur.rule, ej[K - 1 - s]) : NONE) : LI[s];
            }
#pragma unroll
            for (uint32_t h = K / 2; h >= 1; h >>= 1)
#pragma unroll
                for (uint32_t r = 0; r < K; r++)
                    if ((r & h) == 0) cx_kid(L0[r], LI[r], L0[r + h], LI[r + h]);
            nl = min(nl + nb, K);
            if (P < hi) cur = nxt;
            continue;
        }
        uint32_t ei[BK];
#pragma unroll
        for (uint32_t j = 0; j < BK; j++) ei[j] = lvl_index(cur.rule, j);
#pragma unroll 1
        for (uint32_t j = 0; j < nb; j++) {
            uint64_t cd = ek[0];
            uint32_t ci = ei[0];
#pragma unroll
            for (uint32_t y = 1; y < BK; y++) {  // (a select chain: the slots stay in registers)
                cd = j == y ? ek[y] : cd;
                ci = j == y ? ei[y] : ci;
            }
            cd ^= t.hi;
            bool sh = false;
#pragma unroll
            for (uint32_t s = 0; s < K; s++) {
                const bool lt = sh || s >= nl || cd < L0[s] || (cd == L0[s] && tail_less(W, t, ci, LI[s]));
                sh = lt;
                const uint64_t n0_ = lt ? L0[s] : cd;
                const uint32_t n1_ = lt ? LI[s] : ci;
                if (lt) { L0[s] = cd; LI[s] = ci; }
                cd = n0_;
                ci = n1_;
            }
            nl = min(nl + 1, K);
        }
        if (P < hi) cur = nxt;
    }
    if constexpr (NET) {
#pragma unroll
        for (uint32_t s = 0; s + 1 < K; s++) tie |= L0[s] != ~0ull && L0[s] == L0[s + 1];
        tie |= nin != ~0ull && L0[K - 1] == nin;
        if (tie) return TIE;
    }
    const uint32_t m = min(nl, count);
#pragma unroll
    for (uint32_t s = 0; s < K; s++) {  // (every slot, statically: entries from m on are padding)
        oi[s] = LI[s];
        ok[s] = L0[s] ^ t.hi;
    }
    return m;
}

__global__ __launch_bounds__(BLOCK) void swarm_closest_kernel(SwarmDev W, const uint32_t* peers, const uint8_t* targets, uint32_t q, uint32_t count,
                                     uint32_t* out_idx, uint8_t* out_cnt) {
    const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
    if (i >= q) return;
    uint32_t oi[SNP];
    uint64_t ok[SNP];
    const uint32_t p = peers[i];
    const uint32_t m = p < W.n ? peer_closest<SNP>(W, p, load_tgt(targets, i), count, oi, ok) : 0u;
    for (uint32_t s = 0; s < count; s++) out_idx[(size_t)i * count + s] = s < m ? oi[s] : NONE;
    if (out_cnt) out_cnt[i] = (uint8_t)m;
}

// ---- search state ------------------------------------------------------------------------
struct SearchDev {
    const uint32_t* src;
    const uint8_t* targets;
    uint32_t* li;   // [S][LST] list peer indices
    uint64_t* lk;   // [S][LST] their keys
    uint8_t* lq;    // [S][LST] queried
    uint8_t* lb;    // [S][LST] bad (SearchNode::isBad: expired)
    uint8_t* ln;    // [S] list length
    uint32_t* hops; // [S]
    uint8_t* done;  // [S] 0 running, 1 synced, 2 stalled, 3 expired
    uint32_t* sel;  // [S][ALPHA] nodes queried this hop (NONE padded)
    uint32_t* ri;   // [S][ALPHA][BK] answers
    uint64_t* rk;
    uint8_t* rn;    // [S][ALPHA]
    uint32_t* active;
    uint32_t* overflow;  // lists that hit LST entries (a bad node was dropped from the end)
    uint32_t* xo;   // [S][XO_CAP] the search's queried peers that stayed silent: their nodes are expired
    uint8_t* xn;    // [S] how many
    uint32_t S;
    uint32_t offline;    // peers offline per 10,000 (swarm_offline)
};

__device__ __forceinline__ uint64_t sw_mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// Whether peer p is offline (never answers) in a lookup run: a fixed share of the peers by a hash of the index.
__device__ __forceinline__ bool swarm_offline(uint32_t p, uint32_t per10k) {
    return per10k && (uint32_t)(sw_mix((uint64_t)p * 0x9E37ull + 0xBADull) % 10000ull) < per10k;
}

// first <= ALPHA nodes in list order that are neither queried nor bad (searchSendGetValues / canGet,
// dht.cpp:302-304, 1171-1235) -> sel, marked queried; none -> stalled. The queried and bad flags are bit masks (bit k:
// list entry k; bits from n on are don't-care) and every list index is static, so the lists stay in registers.
__device__ __forceinline__ uint32_t lo_mask(uint32_t n) { return n >= 32 ? ~0u : (1u << n) - 1u; }

template <uint32_t N>
__device__ __forceinline__ void select_next(const SearchDev& X, uint32_t s, uint32_t n, uint32_t& qm, uint32_t bm,
                                            const uint32_t (&li)[N]) {
    uint32_t rest = ~(qm | bm) & lo_mask(min(n, N)), pick = 0;
#pragma unroll
    for (uint32_t a = 0; a < ALPHA; a++) {
        pick |= rest & (0u - rest);
        rest &= rest - 1u;
    }
    qm |= pick;
    uint32_t sel[ALPHA] = {NONE, NONE, NONE, NONE};
#pragma unroll
    for (uint32_t j = 0; j < N; j++) {
        const uint32_t rk = (uint32_t)__builtin_popcount(pick & ((1u << j) - 1u));
        if ((pick >> j) & 1u)
#pragma unroll
            for (uint32_t a = 0; a < ALPHA; a++)
                if (a == rk) sel[a] = li[j];
    }
    reinterpret_cast<uint4*>(X.sel)[s] = make_uint4(sel[0], sel[1], sel[2], sel[3]);  // (ALPHA = 4)
    if (!pick) X.done[s] = 2;
}

// the list's flag bytes (queried or bad) of search s as a bit mask, and back (entries from n on: 0); only the 16-byte
// pieces holding entries below n are read (a list is ~14-17 entries: one piece of two)
__device__ __forceinline__ uint32_t load_flags(const uint8_t* f, uint32_t s, uint32_t n = LST) {
    const uint4* p = reinterpret_cast<const uint4*>(f + (size_t)s * LST);
    uint32_t m = 0;
#pragma unroll
    for (int x = 0; x < (int)LST / 16; x++) {
        const uint4 u = 16u * x < n ? p[x] : make_uint4(0, 0, 0, 0);
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int y = 0; y < 4; y++)
#pragma unroll
            for (int z = 0; z < 4; z++) m |= (((w[y] >> (8 * z)) & 255u) ? 1u : 0u) << (16 * x + 4 * y + z);
    }
    return m;
}
// w: the pieces to write are those below max(n, the previous length): the ones above hold zeros already
__device__ __forceinline__ void store_flags(uint8_t* f, uint32_t s, uint32_t m, uint32_t n, uint32_t w = LST) {
    m &= lo_mask(n);
    uint4* p = reinterpret_cast<uint4*>(f + (size_t)s * LST);
#pragma unroll
    for (int x = 0; x < (int)LST / 16; x++) {
        if (16u * x >= w) continue;
        uint32_t w[4];
#pragma unroll
        for (int y = 0; y < 4; y++) {
            w[y] = 0;
#pragma unroll
            for (int z = 0; z < 4; z++) w[y] |= ((m >> (16 * x + 4 * y + z)) & 1u) << (8 * z);
        }
        p[x] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}
static_assert(LST == 32 && ALPHA == 4, "the flag masks are 32 bits, the selection one 16-byte store");

__global__ __launch_bounds__(BLOCK) void search_init_kernel(SwarmDev W, SearchDev X) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    if (s >= X.S) return;
    uint32_t li[SNP];
    uint64_t lk[SNP];
    uint32_t qm = 0;
    const uint32_t p = X.src[s];
    const uint32_t n = p < W.n ? peer_closest<SNP>(W, p, load_tgt(X.targets, s), SN, li, lk) : 0u;
    X.done[s] = n ? 0 : 2;
    X.hops[s] = 0;
    X.ln[s] = (uint8_t)n;
    if (n) select_next(X, s, n, qm, 0u, li);
#pragma unroll
    for (uint32_t j = 0; j < LST; j++) {
        X.li[(size_t)s * LST + j] = j < SNP && j < n ? li[j < SNP ? j : 0] : NONE;
        X.lk[(size_t)s * LST + j] = j < SNP && j < n ? lk[j < SNP ? j : 0] : ~0ull;
    }
    store_flags(X.lq, s, qm, n);
    store_flags(X.lb, s, 0u, n);
}

// one lane per (search, queried node): its findClosestNodes(t, 8), or nothing if it is offline
// NET: findClosestNodes by the sorting network (peer_closest<BK, true>), by inserts where it returns TIE (a 64-bit tie
// in the answer). ~1-2 % a hop over inserts alone (profiles/r06/swarm_qnet/: the kernel waits on its level loads, not
// on VALU); deferring the ties to a second kernel, so that this one does not carry the insert code's registers (134
// against 138 VGPRs), or aiming it at four waves a SIMD (5 VGPRs spilled) was no faster.
template <bool NET>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(SW_QUERY_WPE, 8))) void search_query_kernel(SwarmDev W, SearchDev X) {
    const uint32_t g = blockIdx.x * BLOCK + threadIdx.x;
    if (g >= X.S * ALPHA) return;
    const uint32_t s = g / ALPHA;
    // (the selection, the state and the target loaded together: the selection read whatever the state, so that the
    // peer's header load waits on one round trip, not two)
    const uint32_t sv = X.sel[g];
    const Tgt t = load_tgt(X.targets, s);
    const uint32_t v = X.done[s] ? NONE : sv;
    uint32_t oi[BK];
    uint64_t ok[BK];
    const bool up = v < W.n && !swarm_offline(v, X.offline);
    uint32_t m = up ? (NET ? peer_closest<BK, true>(W, v, t, BK, oi, ok) : TIE) : 0u;
    if (m == TIE) m = peer_closest<BK>(W, v, t, BK, oi, ok);
    // the answers as whole 16-byte pieces (entries from m on are never read: the merge reads rn of them)
    if (m) {
        uint4* pi = reinterpret_cast<uint4*>(X.ri + (size_t)g * BK);
        uint4* pk = reinterpret_cast<uint4*>(X.rk + (size_t)g * BK);
#pragma unroll
        for (uint32_t x = 0; x < BK / 4; x++)
            if (4 * x < m) pi[x] = make_uint4(oi[4 * x], oi[4 * x + 1], oi[4 * x + 2], oi[4 * x + 3]);
#pragma unroll
        for (uint32_t x = 0; x < BK / 2; x++)
            if (2 * x < m)
                pk[x] = make_uint4((uint32_t)ok[2 * x], (uint32_t)(ok[2 * x] >> 32), (uint32_t)ok[2 * x + 1],
                                   (uint32_t)(ok[2 * x + 1] >> 32));
    }
    X.rn[g] = (uint8_t)m;
}

constexpr uint32_t XO_CAP = 64;  // silent peers remembered per lookup (4 per hop; beyond it: counted in overflow)

// Search::insertNode of node r at top-64 distance rd (dht.cpp:961-1047, expired search = false); rbad: r's node
// is expired (a peer this search queried and that stayed silent), so it joins the list as a bad node
// (`if (node.isExpired()) bad++`, dht.cpp:1023-1025):
// its place is after every closer entry; if the list already holds SEARCH_NODES non-bad nodes it is first cut
// after the last prefix with SEARCH_NODES non-bad nodes (an insert beyond that point is refused), then
// trimmed from the end while it holds more than SEARCH_NODES non-bad nodes. Static indices only; the queried and
// bad flags are bit masks (qm, bm).
// N: the list's register width (LST, or 16 for a wave whose lists hold no bad node and no silent peer: at most
// SEARCH_NODES + 1 entries then, so the capacity branch is never taken).
template <uint32_t N>
__device__ __forceinline__ void search_insert(const SwarmDev& W, const Tgt& t, uint32_t (&li)[N], uint64_t (&ld)[N],
                                              uint32_t& qm, uint32_t& bm, uint32_t& n, uint32_t r, uint64_t rd, bool rbad,
                                              bool& ovf) {
    bool found = false, anyeq = false;
    uint32_t pos = 0;
#pragma unroll
    for (uint32_t k = 0; k < N; k++) {
        if (k < n) {
            found |= li[k] == r;
            pos += ld[k] < rd;
            anyeq |= ld[k] == rd;
        }
    }
    if (found) return;
    uint32_t tie = 0;
    if (anyeq) {  // equal top 64 bits (rare): which entries, for the full 160-bit order below
#pragma unroll
        for (uint32_t k = 0; k < N; k++)
            if (k < n) tie |= (ld[k] == rd && li[k] != r ? 1u : 0u) << k;
    }
    while (tie) {  // the full 160-bit order (a select chain keeps the index static)
        const uint32_t k = (uint32_t)__builtin_ctz(tie);
        tie &= tie - 1u;
        uint32_t lk = 0;
#pragma unroll
        for (uint32_t x = 0; x < N; x++) lk = x == k ? li[x] : lk;
        pos += tail_less(W, t, lk, r);
    }
    uint32_t bad = (uint32_t)__builtin_popcount(bm & lo_mask(n));
    const bool full = n - bad >= SN;
    if (full) {
        // tt = the largest t <= n whose prefix [0, t) holds at most SEARCH_NODES non-bad nodes: the prefix ends
        // just before the (SN + 1)-th non-bad entry (or at n)
        uint32_t good = ~bm & lo_mask(n);
#pragma unroll
        for (uint32_t k = 0; k < SN; k++) good &= good - 1u;  // drop the first SN non-bad entries
        const uint32_t tt = good ? (uint32_t)__builtin_ctz(good) : n;
        n = tt;
        bad = (uint32_t)__builtin_popcount(bm & lo_mask(n));
        if (pos >= tt) return;
    }
    if (n == N) {  // capacity: drop the farthest entry (counted; never reached in the tests)
        bad -= (bm >> (N - 1)) & 1u;
        n--;
        ovf = true;
        if (pos >= n) return;
    }
    // insert at pos: entries from pos on move up one (selects, not conditional stores: those became stores through
    // a selected pointer and put the lists in scratch); entries from n + 1 on are don't-care
#pragma unroll
    for (uint32_t k = N - 1; k > 0; k--) {
        li[k] = k > pos ? li[k - 1] : k == pos ? r : li[k];
        ld[k] = k > pos ? ld[k - 1] : k == pos ? rd : ld[k];
    }
    li[0] = pos == 0 ? r : li[0];
    ld[0] = pos == 0 ? rd : ld[0];
    const uint32_t low = lo_mask(pos), bit = 1u << pos;
    qm = (qm & low) | ((qm & ~low) << 1);
    bm = (bm & low) | ((bm & ~low) << 1) | (rbad ? bit : 0u);
    n++;
    bad += rbad ? 1u : 0u;
    // while more than SEARCH_NODES non-bad nodes: drop the last one (dropping from the end stops right after the
    // (SN + 1)-th non-bad entry goes: the list ends just before it, the bad entries ahead of it kept). In closed form
    // from the masks instead of a 32-step loop over the entries (~190 of the insert's ~600 VALU instructions)
    if (n - bad > SN) {
        uint32_t good = ~bm & lo_mask(n);
#pragma unroll
        for (uint32_t k = 0; k < SN; k++) good &= good - 1u;  // drop the first SN non-bad entries
        n = (uint32_t)__builtin_ctz(good);                    // (non-empty: n - bad > SN)
        bad = (uint32_t)__builtin_popcount(bm & lo_mask(n));
    }
}

// One queried node's answers (<= BK peer indices and keys), loaded as whole 16-byte pieces (predicated on its count)
struct Answers {
    uint32_t r[BK];
    uint64_t k[BK];
};
__device__ __forceinline__ void load_answers(const SearchDev& X, uint32_t g, uint32_t rn, Answers& A) {
    const uint4* pi = reinterpret_cast<const uint4*>(X.ri + (size_t)g * BK);
    const uint4* pk = reinterpret_cast<const uint4*>(X.rk + (size_t)g * BK);
#pragma unroll
    for (uint32_t x = 0; x < BK / 4; x++) {
        const uint4 u = 4 * x < rn ? pi[x] : make_uint4(NONE, NONE, NONE, NONE);
        A.r[4 * x] = u.x; A.r[4 * x + 1] = u.y; A.r[4 * x + 2] = u.z; A.r[4 * x + 3] = u.w;
    }
#pragma unroll
    for (uint32_t x = 0; x < BK / 2; x++) {
        const uint4 u = 2 * x < rn ? pk[x] : make_uint4(0, 0, 0, 0);
        A.k[2 * x] = ((uint64_t)u.y << 32) | u.x;
        A.k[2 * x + 1] = ((uint64_t)u.w << 32) | u.z;
    }
}

// one lane per search: Search::insertNode of every answer in the order of the queried nodes, then the
// offline queried nodes turn bad (expired), then the isSynced / expired checks and the next hop's selection.
// Memory: the list, its flags and the answers are read as 16-byte pieces below their lengths only, all of them before
// the inserts (the next queried node's answers in flight while the current one's are inserted), and the list is
// written back below max(new, old length): the round-5 form read every answer by a dependent 4 + 8-byte load inside
// the insert loop (32 round trips per lookup) and moved whole 32-entry lists.
// FUSED (search_hop_kernel): the hop in one lane per lookup — each queried node's findClosestNodes(t, 8) computed in
// place (peer_closest, the query kernel's code) and inserted at once, so the answers never go through HBM (the split
// form writes and reads 4 x 96 bytes per lookup and hop) and the hop is one launch.
// N: the list's register width (search_insert); n0, bm0, xn: the list length, its bad flags and the silent-peer count.
template <uint32_t N, bool FUSED>
__device__ __forceinline__ bool merge_lookup(const SwarmDev& W, const SearchDev& X, uint32_t s, uint32_t n0, uint32_t bm0,
                                             uint32_t xn) {
    {
        const Tgt t = load_tgt(X.targets, s);
        uint32_t li[N];
        uint64_t ld[N];  // top-64 XOR distances
        uint32_t n = n0;
        const uint4 sv = reinterpret_cast<const uint4*>(X.sel)[s];
        const uint32_t sel[ALPHA] = {sv.x, sv.y, sv.z, sv.w};
        const uint32_t rn4 = FUSED ? 0u : *reinterpret_cast<const uint32_t*>(X.rn + (size_t)s * ALPHA);  // (ALPHA = 4)
        Answers A[2];
        if (!FUSED) load_answers(X, s * ALPHA, rn4 & 255u, A[0]);
        {
            const uint4* pi = reinterpret_cast<const uint4*>(X.li + (size_t)s * LST);
            const uint4* pk = reinterpret_cast<const uint4*>(X.lk + (size_t)s * LST);
#pragma unroll
            for (uint32_t x = 0; x < N / 4; x++) {
                const uint4 u = 4 * x < n0 ? pi[x] : make_uint4(NONE, NONE, NONE, NONE);
                li[4 * x] = u.x; li[4 * x + 1] = u.y; li[4 * x + 2] = u.z; li[4 * x + 3] = u.w;
            }
#pragma unroll
            for (uint32_t x = 0; x < N / 2; x++) {
                const uint4 u = 2 * x < n0 ? pk[x] : make_uint4(~0u, ~0u, ~0u, ~0u);
                ld[2 * x] = (((uint64_t)u.y << 32) | u.x) ^ t.hi;
                ld[2 * x + 1] = (((uint64_t)u.w << 32) | u.z) ^ t.hi;
            }
        }
        uint32_t qm = load_flags(X.lq, s, n0), bm = bm0;
        const uint32_t src = X.src[s];
        bool ovf = false;
        const uint32_t* xo = X.xo + (size_t)s * XO_CAP;
#pragma unroll
        for (uint32_t a = 0; a < ALPHA; a++) {
            uint32_t rn;
            if (FUSED) {
                const uint32_t v = sel[a];
                const bool up = v < W.n && !swarm_offline(v, X.offline);
                rn = up ? peer_closest<BK>(W, v, t, BK, A[a & 1].r, A[a & 1].k) : 0u;
            } else {
                if (a + 1 < ALPHA) load_answers(X, s * ALPHA + a + 1, (rn4 >> (8 * (a + 1))) & 255u, A[(a + 1) & 1]);
                rn = (rn4 >> (8 * a)) & 255u;
            }
            const Answers& C = A[a & 1];
            for (uint32_t j = 0; j < rn; j++) {
                uint32_t r = C.r[0];
                uint64_t rk = C.k[0];
#pragma unroll
                for (uint32_t x = 1; x < BK; x++) {  // (a select chain: the answers stay in registers)
                    r = j == x ? C.r[x] : r;
                    rk = j == x ? C.k[x] : rk;
                }
                if (r == src) continue;  // deserializeNodes drops our own ID (network_engine.cpp:798-799)
                bool rbad = false;
                if (swarm_offline(r, X.offline))
                    for (uint32_t e = 0; e < xn && !rbad; e++) rbad = xo[e] == r;
                search_insert(W, t, li, ld, qm, bm, n, r, rk ^ t.hi, rbad, ovf);
            }
        }
#pragma unroll
        for (uint32_t a = 0; a < ALPHA; a++) {  // the silent ones: expired after their tries -> bad
            const uint32_t v = sel[a];
            if (v == NONE || !swarm_offline(v, X.offline)) continue;
            if (xn < XO_CAP) X.xo[(size_t)s * XO_CAP + xn++] = v;  // its node is expired from now on
            else ovf = true;
#pragma unroll
            for (uint32_t k = 0; k < N; k++)
                if (k < n && li[k] == v) bm |= 1u << k;
        }
        X.xn[s] = (uint8_t)xn;
        X.hops[s] += 1;
        // Search::isSynced: the first TARGET_NODES non-bad nodes answered; consecutive bad nodes from the front
        const uint32_t nm = lo_mask(n), good = ~bm & nm;
        uint32_t first8 = good;  // the first BK non-bad entries
        {
            uint32_t rest = good;
#pragma unroll
            for (uint32_t k = 0; k < BK; k++) rest &= rest - 1u;
            first8 &= ~rest;
        }
        const bool synced = (first8 & ~qm) == 0;
        const uint32_t lead = ~(bm & nm), cb = lead ? (uint32_t)__builtin_ctz(lead) : 32u;  // leading bad entries
        if (synced && first8) X.done[s] = 1;
        else if (n > 0 && cb >= min(n, MAX_BAD)) X.done[s] = 3;
        else select_next(X, s, n, qm, bm, li);
        X.ln[s] = (uint8_t)n;
        const uint32_t wn = max(n, n0);  // pieces above it hold the padding already
        {
            uint4* pi = reinterpret_cast<uint4*>(X.li + (size_t)s * LST);
            uint4* pk = reinterpret_cast<uint4*>(X.lk + (size_t)s * LST);
#pragma unroll
            for (uint32_t x = 0; x < N / 4; x++)
                if (4 * x < wn)
                    pi[x] = make_uint4(4 * x < n ? li[4 * x] : NONE, 4 * x + 1 < n ? li[4 * x + 1] : NONE,
                                       4 * x + 2 < n ? li[4 * x + 2] : NONE, 4 * x + 3 < n ? li[4 * x + 3] : NONE);
#pragma unroll
            for (uint32_t x = 0; x < N / 2; x++) {
                if (2 * x >= wn) continue;
                const uint64_t k0 = 2 * x < n ? ld[2 * x] ^ t.hi : ~0ull, k1 = 2 * x + 1 < n ? ld[2 * x + 1] ^ t.hi : ~0ull;
                pk[x] = make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
            }
        }
        store_flags(X.lq, s, qm, n, wn);
        store_flags(X.lb, s, bm, n, wn);
        if (ovf) atomicAdd(X.overflow, 1u);
        return !X.done[s];
    }
}

// The all-online hop's merge as a sorting network (runs where every peer answers). With no bad node and no silent
// peer, Search::insertNode's sequential inserts (dht.cpp:961-1047) keep exactly the SEARCH_NODES closest of the list
// and the answers (an insert beyond a full list is refused, a full list drops its farthest after an insert, a node
// already in the list is skipped): the result does not depend on the order of the inserts. So each queried node's
// block of <= 8 answers (sorted, from findClosestNodes) loses our own ID and the nodes already in the list (index
// compares), is re-sorted (19 compare-exchanges), and merges with the 16-slot list as one bitonic half-cleaner (the
// list ascending, the block descending) and four levels: ~560 VALU operations a block where the sequential inserts
// took ~250 each answer. Equal 64-bit distances of different nodes (their order needs the 160-bit tails) are adjacent
// after each merge; a lookup that has one is left untouched with done = 4 and the sequential form merges it next.
// Queried flags travel in bit 31 of the node index.
// PF: the next queried node's answers loaded before the current block is merged (a second Answers in registers).
template <bool PF>
__device__ __forceinline__ bool merge_lookup_net(const SwarmDev& W, const SearchDev& X, uint32_t s) {
    constexpr uint32_t QB = 0x80000000u, IM = 0x7FFFFFFFu;
    const uint64_t MAXK = ~0ull;
    const Tgt t = load_tgt(X.targets, s);
    const uint32_t n0 = X.ln[s];
    uint32_t li[16];
    uint64_t lk[16];
    {
        const uint4* pi = reinterpret_cast<const uint4*>(X.li + (size_t)s * LST);
        const uint4* pk = reinterpret_cast<const uint4*>(X.lk + (size_t)s * LST);
#pragma unroll
        for (uint32_t x = 0; x < 4; x++) {
            const uint4 u = 4 * x < n0 ? pi[x] : make_uint4(NONE, NONE, NONE, NONE);
            li[4 * x] = u.x; li[4 * x + 1] = u.y; li[4 * x + 2] = u.z; li[4 * x + 3] = u.w;
        }
#pragma unroll
        for (uint32_t x = 0; x < 8; x++) {
            const uint4 u = 2 * x < n0 ? pk[x] : make_uint4(~0u, ~0u, ~0u, ~0u);
            lk[2 * x] = 2 * x < n0 ? (((uint64_t)u.y << 32) | u.x) ^ t.hi : MAXK;
            lk[2 * x + 1] = 2 * x + 1 < n0 ? (((uint64_t)u.w << 32) | u.z) ^ t.hi : MAXK;
        }
    }
    const uint32_t qm0 = load_flags(X.lq, s, n0);
#pragma unroll
    for (uint32_t k = 0; k < 16; k++)
        if (k < n0 && ((qm0 >> k) & 1u)) li[k] |= QB;
    const uint32_t rn4 = *reinterpret_cast<const uint32_t*>(X.rn + (size_t)s * ALPHA);  // (ALPHA = 4)
    const uint32_t src = X.src[s];
    bool tie = false;
#pragma unroll
    for (uint32_t k = 0; k + 1 < 16; k++) tie |= li[k + 1] != NONE && lk[k] == lk[k + 1];
    Answers A, An;
    if (PF) load_answers(X, s * ALPHA, rn4 & 255u, A);
#pragma unroll 1
    for (uint32_t a = 0; a < ALPHA; a++) {  // (not unrolled: one or two blocks' answers in registers at a time)
        const uint32_t rn = (rn4 >> (8 * a)) & 255u;
        if (!PF) load_answers(X, s * ALPHA + a, rn, A);
        else if (a + 1 < ALPHA) load_answers(X, s * ALPHA + a + 1, (rn4 >> (8 * (a + 1))) & 255u, An);
        uint64_t bk[BK];
        uint32_t bi[BK];
#pragma unroll
        for (uint32_t j = 0; j < BK; j++) {
            const uint32_t r = A.r[j];
            bool drop = j >= rn || r == src;  // deserializeNodes drops our own ID (network_engine.cpp:798-799)
#pragma unroll
            for (uint32_t k = 0; k < 16; k++) drop |= (li[k] & IM) == r;  // already in the list (empty slots: IM)
            bk[j] = drop ? MAXK : A.k[j] ^ t.hi;
            bi[j] = drop ? NONE : r;
        }
        sort8_kid(bk, bi);  // (the block was sorted; the dropped entries leave MAX holes)
        // the 16 smallest of (list ascending, block descending): one half-cleaner, then four levels
#pragma unroll
        for (uint32_t i = 8; i < 16; i++) {
            const bool sw = bk[15 - i] < lk[i];
            lk[i] = sw ? bk[15 - i] : lk[i];
            li[i] = sw ? bi[15 - i] : li[i];
        }
#pragma unroll
        for (uint32_t h = 8; h >= 1; h >>= 1)
#pragma unroll
            for (uint32_t r = 0; r < 16; r++)
                if ((r & h) == 0) cx_kid(lk[r], li[r], lk[r + h], li[r + h]);
#pragma unroll
        for (uint32_t k = 0; k + 1 < 16; k++) tie |= li[k + 1] != NONE && lk[k] == lk[k + 1];
        if (PF) A = An;
    }
    if (tie) {  // the sequential form (search_merge_kernel<false, 16, true>) merges this lookup
        X.done[s] = 4;
        return false;
    }
    uint32_t n = 0, qm = 0;
#pragma unroll
    for (uint32_t k = 0; k < SN; k++) {
        n += li[k] != NONE ? 1u : 0u;
        qm |= (li[k] != NONE && (li[k] & QB)) ? 1u << k : 0u;
        li[k] = li[k] != NONE ? li[k] & IM : NONE;
    }
    X.hops[s] += 1;
    // Search::isSynced: the first TARGET_NODES nodes answered (no bad node here)
    const uint32_t nm = lo_mask(n);
    uint32_t first8 = nm;
    {
        uint32_t rest = nm;
#pragma unroll
        for (uint32_t k = 0; k < BK; k++) rest &= rest - 1u;
        first8 &= ~rest;
    }
    const bool synced = (first8 & ~qm) == 0;
    if (synced && first8) X.done[s] = 1;
    else select_next(X, s, n, qm, 0u, li);
    X.ln[s] = (uint8_t)n;
    const uint32_t wn = max(n, n0);  // pieces above it hold the padding already
    {
        uint4* pi = reinterpret_cast<uint4*>(X.li + (size_t)s * LST);
        uint4* pk = reinterpret_cast<uint4*>(X.lk + (size_t)s * LST);
#pragma unroll
        for (uint32_t x = 0; x < 4; x++)
            if (4 * x < wn)
                pi[x] = make_uint4(4 * x < n ? li[4 * x] : NONE, 4 * x + 1 < n ? li[4 * x + 1] : NONE,
                                   4 * x + 2 < n ? li[4 * x + 2] : NONE, 4 * x + 3 < n ? li[4 * x + 3] : NONE);
#pragma unroll
        for (uint32_t x = 0; x < 8; x++) {
            if (2 * x >= wn) continue;
            const uint64_t k0 = 2 * x < n ? lk[2 * x] ^ t.hi : ~0ull, k1 = 2 * x + 1 < n ? lk[2 * x + 1] ^ t.hi : ~0ull;
            pk[x] = make_uint4((uint32_t)k0, (uint32_t)(k0 >> 32), (uint32_t)k1, (uint32_t)(k1 >> 32));
        }
    }
    store_flags(X.lq, s, qm, n, wn);
    store_flags(X.lb, s, 0u, n, wn);
    return !X.done[s];
}

template <bool PF>
__global__ __launch_bounds__(BLOCK) void search_merge_net_kernel(SwarmDev W, SearchDev X) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    const bool running = s < X.S && !X.done[s] && merge_lookup_net<PF>(W, X, s);
    const uint64_t m = __ballot(running);
    if ((threadIdx.x & 63u) == 0 && m) atomicAdd(X.active, (uint32_t)__builtin_popcountll(m));
}

// N = 16 (the narrow form): for runs where every peer answers (swarm_offline never true), so that no list holds a bad
// node and no lookup meets a silent peer: a list keeps at most SEARCH_NODES + 1 entries through a hop, in 16
// registers instead of LST (and the kernel in a quarter of the VGPRs). N = LST: any run.
// RETRY: only the lookups search_merge_net_kernel left with done = 4 (a 64-bit distance tie), this hop.
template <bool FUSED, uint32_t N, bool RETRY = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(N == 16 ? SW_NARROW_WPE : 1, 8))) void search_merge_kernel(SwarmDev W, SearchDev X) {
    const uint32_t s = blockIdx.x * BLOCK + threadIdx.x;
    const bool live = s < X.S && X.done[s] == (RETRY ? 4u : 0u);
    if (RETRY && live) X.done[s] = 0;
    bool running = false;
    if (live) {
        const uint32_t n0 = X.ln[s];
        running = merge_lookup<N, FUSED>(W, X, s, n0, N == LST ? load_flags(X.lb, s, n0) : 0u, N == LST ? X.xn[s] : 0u);
    }
    const uint64_t m = __ballot(running);
    if ((threadIdx.x & 63u) == 0 && m) atomicAdd(X.active, (uint32_t)__builtin_popcountll(m));
}

}  // namespace

// A search's device state (lists, flags, answers, its copies of the sources and targets) for up to `cap` lookups.
// The swarm keeps the largest one a destroyed search left (kad_search_destroy) and the next kad_search_create of at
// most that many lookups takes it instead of making its ~700 bytes per lookup of hipMalloc calls again (17 of them:
// ~2.5 ms of a 1M-lookup run that converges in ~8 ms of kernels, tools/bench_swarm.py).
struct SearchBufs {
    std::vector<void*> owned;
    SearchDev X{};
    uint32_t* src = nullptr;
    uint8_t* targets = nullptr;
    uint32_t cap = 0;
    void release() {
        for (void* p : owned) (void)hipFree(p);
        owned.clear();
        cap = 0;
    }
};
struct kad_swarm {
    int device = 0;
    SwarmDev W{};
    std::vector<void*> owned;
    uint64_t bytes = 0;
    mutable std::mutex pool_mu;
    mutable SearchBufs pool;  // (searches must not outlive their swarm: they read its tables)
    ~kad_swarm() {
        pool.release();
        for (void* p : owned) (void)hipFree(p);
    }
};

struct kad_search {
    int device = 0;
    const kad_swarm* sw = nullptr;
    SearchDev X{};
    hipStream_t stream = nullptr;
    SearchBufs bufs;
    ~kad_search() { bufs.release(); }
};

namespace {
template <class T>
int alloc(T** p, size_t count, std::vector<void*>& owned, uint64_t* bytes = nullptr) {
    void* q = nullptr;
    const size_t nb = std::max<size_t>(count * sizeof(T), 16);
    hipError_t e = hipMalloc(&q, nb);
    if (e != hipSuccess) return err(KAD_ERR_NOMEM, "hipMalloc(%zu) failed: %s", nb, hipGetErrorString(e));
    owned.push_back(q);
    if (bytes) *bytes += nb;
    *p = static_cast<T*>(q);
    return KAD_OK;
}

struct Guard {
    int prev = -1;
    explicit Guard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~Guard() {
        int cur;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};
}  // namespace

extern "C" {

int kad_swarm_create(kad_swarm** out, int device, uint32_t n, const uint8_t* sorted_ids) {
    if (!out || (n && !sorted_ids)) return err(KAD_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (n < 2) return err(KAD_ERR_INVALID, "a swarm needs at least 2 peers");
    if (!kadgpu_internal::device_ok(device)) return err(KAD_ERR_NO_DEVICE, "device %d is not a gfx950 GPU", device);
    std::vector<uint64_t> key(n);
    std::vector<uint32_t> tail(3ull * n);
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t* p = sorted_ids + 20ull * i;
        uint64_t k = 0;
        for (int b = 0; b < 8; b++) k = (k << 8) | p[b];
        key[i] = k;
        for (int w = 0; w < 3; w++)
            tail[3ull * i + w] = ((uint32_t)p[8 + 4 * w] << 24) | ((uint32_t)p[9 + 4 * w] << 16) |
                                 ((uint32_t)p[10 + 4 * w] << 8) | p[11 + 4 * w];
        if (i && std::memcmp(sorted_ids + 20ull * (i - 1), p, 20) >= 0)
            return err(KAD_ERR_INVALID, "peer IDs must be strictly ascending (index %u)", i);
    }
    Guard g(device);
    kad_swarm* s = new kad_swarm;
    s->device = device;
    uint64_t* dk;
    uint32_t* dt;
    int rc;
    if ((rc = alloc(&dk, n, s->owned, &s->bytes)) || (rc = alloc(&dt, 3ull * n, s->owned, &s->bytes)) ||
        (rc = alloc(&s->W.hdr, (size_t)n * HDR_WORDS, s->owned, &s->bytes)) ||
        (rc = alloc(&s->W.lvl, (size_t)n * L * LVL_WORDS, s->owned, &s->bytes))) {
        delete s;
        return rc;
    }
    if (hipMemcpy(dk, key.data(), 8ull * n, hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(dt, tail.data(), 12ull * n, hipMemcpyHostToDevice) != hipSuccess) {
        delete s;
        return err(KAD_ERR_HIP, "upload failed");
    }
    s->W.key = dk;
    s->W.tail = dt;
    s->W.n = n;
    hipLaunchKernelGGL(swarm_build_kernel, dim3(grid_for(n)), dim3(BLOCK), 0, 0, s->W);
    if (hipGetLastError() != hipSuccess || hipDeviceSynchronize() != hipSuccess) {
        delete s;
        return err(KAD_ERR_HIP, "swarm table build failed");
    }
    *out = s;
    return KAD_OK;
}

int kad_swarm_destroy(kad_swarm* s) {
    if (!s) return KAD_OK;
    Guard g(s->device);
    (void)hipDeviceSynchronize();
    delete s;
    return KAD_OK;
}

int kad_swarm_info(const kad_swarm* s, uint32_t* n_peers, uint64_t* device_bytes) {
    if (!s) return err(KAD_ERR_INVALID, "NULL swarm");
    if (n_peers) *n_peers = s->W.n;
    if (device_bytes) *device_bytes = s->bytes;
    return KAD_OK;
}

int kad_swarm_get_table(const kad_swarm* s, uint32_t peer, uint32_t* depth, uint8_t* counts, uint32_t* entries) {
    if (!s || !depth || !counts || !entries) return err(KAD_ERR_INVALID, "NULL argument");
    if (peer >= s->W.n) return err(KAD_ERR_INVALID, "peer %u >= %u", peer, s->W.n);
    Guard g(s->device);
    uint32_t h[HDR_WORDS];
    std::vector<uint32_t> lv((size_t)L * LVL_WORDS);
    SW_TRY(hipMemcpy(h, s->W.hdr + (size_t)peer * HDR_WORDS, sizeof h, hipMemcpyDeviceToHost));
    SW_TRY(hipMemcpy(lv.data(), s->W.lvl + (size_t)peer * L * LVL_WORDS, 4 * lv.size(), hipMemcpyDeviceToHost));
    *depth = h[2];
    for (uint32_t d = 0; d < L; d++) {
        counts[d] = (uint8_t)(h[4 + d / 4] >> (8 * (d % 4)));
        for (uint32_t j = 0; j < BK; j++) entries[d * BK + j] = lv[(size_t)d * LVL_WORDS + LVL_IDX + j];
    }
    return KAD_OK;
}

int kad_swarm_closest_batch(const kad_swarm* s, const uint32_t* peers, const uint8_t* targets, uint32_t q,
                            uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, void* stream) {
    if (!s) return err(KAD_ERR_INVALID, "NULL swarm");
    if (count > SNP) return err(KAD_ERR_UNSUPPORTED, "count %u > %u", count, SNP);
    if (q == 0) return KAD_OK;
    if (!peers || !targets || !out_idx) return err(KAD_ERR_INVALID, "NULL buffer");
    Guard g(s->device);
    hipLaunchKernelGGL(swarm_closest_kernel, dim3(grid_for(q)), dim3(BLOCK), 0, (hipStream_t)stream, s->W, peers,
                       targets, q, count, out_idx, out_cnt);
    SW_TRY(hipGetLastError());
    return KAD_OK;
}

int kad_search_create(kad_search** out, const kad_swarm* s, uint32_t S, const uint32_t* src, const uint8_t* targets,
                      uint32_t offline_per_10k, void* stream) {
    if (!out || !s || (S && (!src || !targets))) return err(KAD_ERR_INVALID, "NULL argument");
    *out = nullptr;
    Guard g(s->device);
    kad_search* x = new kad_search;
    x->device = s->device;
    x->sw = s;
    x->stream = (hipStream_t)stream;
    SearchDev& X = x->X;
    X.S = S;
    if (offline_per_10k > 10000) {
        delete x;
        return err(KAD_ERR_INVALID, "offline_per_10k %u > 10000", offline_per_10k);
    }
    X.offline = offline_per_10k;
    {
        std::lock_guard<std::mutex> lk(s->pool_mu);
        if (S && s->pool.cap >= S) std::swap(x->bufs, s->pool);  // (the pool is left empty)
    }
    SearchBufs& B = x->bufs;
    if (!B.cap) {
        SearchDev& Y = B.X;
        std::vector<void*>& o = B.owned;
        const uint32_t C = S;
        int rc;
        if ((rc = alloc(&B.src, C, o)) || (rc = alloc(&B.targets, 20ull * C, o)) ||
            (rc = alloc(&Y.li, (size_t)C * LST, o)) || (rc = alloc(&Y.lk, (size_t)C * LST, o)) ||
            (rc = alloc(&Y.lq, (size_t)C * LST, o)) || (rc = alloc(&Y.lb, (size_t)C * LST, o)) ||
            (rc = alloc(&Y.ln, C, o)) || (rc = alloc(&Y.overflow, 1, o)) || (rc = alloc(&Y.hops, C, o)) ||
            (rc = alloc(&Y.done, C, o)) || (rc = alloc(&Y.sel, (size_t)C * ALPHA, o)) ||
            (rc = alloc(&Y.ri, (size_t)C * ALPHA * BK, o)) || (rc = alloc(&Y.rk, (size_t)C * ALPHA * BK, o)) ||
            (rc = alloc(&Y.rn, (size_t)C * ALPHA, o)) || (rc = alloc(&Y.active, 1, o)) ||
            (rc = alloc(&Y.xo, (size_t)C * XO_CAP, o)) || (rc = alloc(&Y.xn, C, o))) {
            delete x;
            return rc;
        }
        B.cap = std::max<uint32_t>(C, 1);
    }
    {
        const uint32_t S0 = X.S, off0 = X.offline;
        X = B.X;
        X.S = S0;
        X.offline = off0;
    }
    uint32_t* dsrc = B.src;
    uint8_t* dt = B.targets;
    if (S && (hipMemcpyAsync(dsrc, src, 4ull * S, hipMemcpyDefault, x->stream) != hipSuccess ||
              hipMemcpyAsync(dt, targets, 20ull * S, hipMemcpyDefault, x->stream) != hipSuccess)) {
        delete x;
        return err(KAD_ERR_HIP, "search upload failed");
    }
    X.src = dsrc;
    X.targets = dt;
    if (hipMemsetAsync(X.overflow, 0, 4, x->stream) != hipSuccess ||
        hipMemsetAsync(X.xn, 0, std::max<uint32_t>(S, 1), x->stream) != hipSuccess) {
        delete x;
        return err(KAD_ERR_HIP, "search init failed");
    }
    if (S) hipLaunchKernelGGL(search_init_kernel, dim3(grid_for(S)), dim3(BLOCK), 0, x->stream, s->W, X);
    if (hipGetLastError() != hipSuccess) {
        delete x;
        return err(KAD_ERR_HIP, "search init launch failed");
    }
    *out = x;
    return KAD_OK;
}

// KAD_SWARM_WIDE=1 (A/B): the LST-wide merge even where every peer answers.
static bool narrow_off() {
    static const bool off = std::getenv("KAD_SWARM_WIDE") != nullptr;
    return off;
}

// KAD_SWARM_SEQ=1 (A/B): the sequential 16-entry merge where every peer answers, not the sorting network.
static bool net_off() {
    static const bool off = std::getenv("KAD_SWARM_SEQ") != nullptr;
    return off;
}

// KAD_SWARM_NETPF=0 (A/B): the merge network without the next block's answers loaded ahead.
static bool net_pf_off() {
    static const bool off = [] {
        const char* e = std::getenv("KAD_SWARM_NETPF");
        return e && !std::strcmp(e, "0");
    }();
    return off;
}

// KAD_SWARM_QUERY=ins (A/B): the query kernel's findClosestNodes by inserts, not the sorting network.
static bool qnet_off() {
    static const bool off = [] {
        const char* e = std::getenv("KAD_SWARM_QUERY");
        return e && !std::strcmp(e, "ins");
    }();
    return off;
}

int kad_search_hop(kad_search* x, uint32_t* n_active) {
    if (!x) return err(KAD_ERR_INVALID, "NULL search");
    Guard g(x->device);
    const SearchDev& X = x->X;
    SW_TRY(hipMemsetAsync(X.active, 0, 4, x->stream));
    if (X.S) {
        // the two-kernel hop (query kernel, answers through HBM, merge kernel). KAD_SWARM_FUSED=1 (tools): the fused
        // kernel, measured slower — 48-50 against 73 M lookups/s at 10M peers (profiles/r06/swarm_fused/): the peer
        // walks run on a quarter of the lanes, behind the merge's registers, with their round trips no longer hidden
        static const bool split = std::getenv("KAD_SWARM_FUSED") == nullptr;
        if (split) {
            const dim3 qg(grid_for((uint64_t)X.S * ALPHA));
            if (qnet_off())
                hipLaunchKernelGGL(search_query_kernel<false>, qg, dim3(BLOCK), 0, x->stream, x->sw->W, X);
            else
                hipLaunchKernelGGL(search_query_kernel<true>, qg, dim3(BLOCK), 0, x->stream, x->sw->W, X);
            if (X.offline == 0 && !narrow_off() && !net_off()) {
                if (net_pf_off())
                    hipLaunchKernelGGL(search_merge_net_kernel<false>, dim3(grid_for(X.S)), dim3(BLOCK), 0, x->stream,
                                       x->sw->W, X);
                else
                    hipLaunchKernelGGL(search_merge_net_kernel<true>, dim3(grid_for(X.S)), dim3(BLOCK), 0, x->stream,
                                       x->sw->W, X);
                hipLaunchKernelGGL((search_merge_kernel<false, 16, true>), dim3(grid_for(X.S)), dim3(BLOCK), 0,
                                   x->stream, x->sw->W, X);
            } else if (X.offline == 0 && !narrow_off())
                hipLaunchKernelGGL((search_merge_kernel<false, 16>), dim3(grid_for(X.S)), dim3(BLOCK), 0, x->stream,
                                   x->sw->W, X);
            else
                hipLaunchKernelGGL((search_merge_kernel<false, LST>), dim3(grid_for(X.S)), dim3(BLOCK), 0, x->stream,
                                   x->sw->W, X);
        } else {
            hipLaunchKernelGGL((search_merge_kernel<true, LST>), dim3(grid_for(X.S)), dim3(BLOCK), 0, x->stream, x->sw->W, X);
        }
    }
    SW_TRY(hipGetLastError());
    if (n_active) {
        SW_TRY(hipMemcpyAsync(n_active, X.active, 4, hipMemcpyDeviceToHost, x->stream));
        SW_TRY(hipStreamSynchronize(x->stream));
    }
    return KAD_OK;
}

int kad_search_get(const kad_search* x, uint32_t* list, uint8_t* queried, uint8_t* bad, uint8_t* n, uint32_t* hops,
                   uint8_t* done, uint32_t* overflow) {
    if (!x) return err(KAD_ERR_INVALID, "NULL search");
    Guard g(x->device);
    const SearchDev& X = x->X;
    SW_TRY(hipStreamSynchronize(x->stream));
    const size_t S = X.S;
    if (list) SW_TRY(hipMemcpy(list, X.li, 4 * S * LST, hipMemcpyDeviceToHost));
    if (queried) SW_TRY(hipMemcpy(queried, X.lq, S * LST, hipMemcpyDeviceToHost));
    if (bad) SW_TRY(hipMemcpy(bad, X.lb, S * LST, hipMemcpyDeviceToHost));
    if (n) SW_TRY(hipMemcpy(n, X.ln, S, hipMemcpyDeviceToHost));
    if (hops) SW_TRY(hipMemcpy(hops, X.hops, 4 * S, hipMemcpyDeviceToHost));
    if (done) SW_TRY(hipMemcpy(done, X.done, S, hipMemcpyDeviceToHost));
    if (overflow) SW_TRY(hipMemcpy(overflow, X.overflow, 4, hipMemcpyDeviceToHost));
    return KAD_OK;
}

int kad_search_destroy(kad_search* x) {
    if (!x) return KAD_OK;
    Guard g(x->device);
    if (hipStreamSynchronize(x->stream) == hipSuccess && x->sw && x->bufs.cap) {
        // the buffers back to the swarm's pool (the larger of the two stays)
        std::lock_guard<std::mutex> lk(x->sw->pool_mu);
        if (x->bufs.cap > x->sw->pool.cap) std::swap(x->bufs, x->sw->pool);
    }
    delete x;
    return KAD_OK;
}

}  // extern "C"
