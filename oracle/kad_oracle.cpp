/*
 * kad_oracle.cpp — CPU ORACLE for the Kademlia closest-node path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / the timed CPU baseline. The product path
 * (opendht_amd/, libkadgpu.so) never links or calls it.
 *
 * PARITY STATUS: "parity unpinned". The reference (OpenDHT 1.2.1 at /root/reference)
 * cannot be compiled here without stand-in msgpack/GnuTLS headers, which the rules of
 * this build forbid, its Python binding cannot be built, and it ships no tests or golden
 * vectors for this path. This file is therefore a restatement of the
 * reference's algorithm, written from reading its source, with every function citing the
 * file:line it follows. Two independent restatements are kept and cross-checked by the
 * tests: (1) a structure-faithful one (std::list of Buckets holding std::list of
 * shared_ptr<Node>, linear findBucket, find_if insertion sort, std::map NodeCache) and
 * (2) a closed-form flat-array one (binary-search bucket locate, window rounds from good
 * counts, sort). The structure-faithful one is also the "port" CPU baseline that
 * bench.py times on the GPU box's host cores.
 *
 * All paths below cite /root/reference/... relative paths.
 */
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <list>
#include <map>
#include <memory>
#include <random>
#include <thread>
#include <vector>

namespace orc {

static constexpr unsigned HASH_LEN = 20;  // include/opendht/infohash.h:49

// ---------------------------------------------------------------------------
// InfoHash restatement (include/opendht/infohash.h:58-180). Byte 0 is most significant.
// ---------------------------------------------------------------------------
struct Id : std::array<uint8_t, HASH_LEN> {
    Id() { fill(0); }
    explicit Id(const uint8_t* p) { std::memcpy(data(), p, HASH_LEN); }

    // infohash.h:84-95 lowbit(): index (MSB = 0) of the lowest set bit, (unsigned)-1 if zero
    unsigned lowbit() const {
        int i, j;
        for (i = HASH_LEN - 1; i >= 0; i--)
            if ((*this)[i] != 0) break;
        if (i < 0) return (unsigned)-1;
        for (j = 7; j >= 0; j--)
            if (((*this)[i] & (0x80 >> j)) != 0) break;
        return 8 * i + j;
    }
    // infohash.h:101-103 cmp(): memcmp order
    static int cmp(const Id& a, const Id& b) { return std::memcmp(a.data(), b.data(), HASH_LEN); }
    // infohash.h:106-128 commonBits()
    static unsigned commonBits(const Id& a, const Id& b) {
        unsigned i;
        for (i = 0; i < HASH_LEN; i++)
            if (a[i] != b[i]) break;
        if (i == HASH_LEN) return 8 * HASH_LEN;
        uint8_t x = a[i] ^ b[i];
        unsigned j = 0;
        while ((x & 0x80) == 0) { x <<= 1; j++; }
        return 8 * i + j;
    }
    // infohash.h:131-146 xorCmp(): which of id1/id2 is closer to *this
    int xorCmp(const Id& id1, const Id& id2) const {
        for (unsigned i = 0; i < HASH_LEN; i++) {
            if (id1[i] == id2[i]) continue;
            uint8_t x1 = id1[i] ^ (*this)[i], x2 = id2[i] ^ (*this)[i];
            return x1 < x2 ? -1 : 1;
        }
        return 0;
    }
    // infohash.h:148-162 getBit/setBit
    bool getBit(unsigned n) const { return ((*this)[n / 8] >> (7 - n % 8)) & 1; }
    void setBit(unsigned n, bool b) {
        uint8_t& num = (*this)[n / 8];
        unsigned bit = 7 - (n % 8);
        num ^= (-(int)b ^ num) & (1 << bit);
    }
    // infohash.h:173-180 operator<
    bool operator<(const Id& o) const { return cmp(*this, o) < 0; }
};

// ---------------------------------------------------------------------------
// Node (include/opendht/node.h:35-105, src/node.cpp:34-40)
// ---------------------------------------------------------------------------
using clock_ns = std::chrono::nanoseconds;
struct Node {
    Id id;
    uint32_t idx;  // snapshot index (the engine's result currency)
    int64_t time = INT64_MIN, reply_time = INT64_MIN;  // time_point::min()
    bool expired_ = false;
    static constexpr int64_t NODE_GOOD_TIME = 120LL * 60 * 1000000000LL;   // node.h:91
    static constexpr int64_t NODE_EXPIRE_TIME = 10LL * 60 * 1000000000LL;  // node.h:94
    bool isExpired() const { return expired_; }                          // node.h:67
    bool isGood(int64_t now) const {                                     // node.cpp:34-40
        return !expired_ && reply_time >= now - NODE_GOOD_TIME && time >= now - NODE_EXPIRE_TIME;
    }
};

// Status byte -> node times at `now` (SURVEY.md §8d status mix): good -> time = reply_time = now;
// expired -> setExpired(); dubious -> time = now - 11 min.
static void apply_status(Node& n, uint8_t st, int64_t now) {
    n.time = n.reply_time = now;
    n.expired_ = false;
    if (st & 2) n.expired_ = true;
    else if (!(st & 1)) n.time = now - 11LL * 60 * 1000000000LL;
}

// ---------------------------------------------------------------------------
// Structure-faithful RoutingTable (include/opendht/routing_table.h:28-79,
// src/routing_table.cpp:47-163)
// ---------------------------------------------------------------------------
struct Bucket {
    Id first;
    std::list<std::shared_ptr<Node>> nodes;
};

struct RoutingTable : std::list<Bucket> {
    // routing_table.cpp:113-127 findBucket(): linear walk from begin()
    iterator findBucket(const Id& id) {
        if (empty()) return end();
        auto b = begin();
        while (true) {
            auto next = std::next(b);
            if (next == end()) return b;
            if (Id::cmp(id, next->first) < 0) return b;
            b = next;
        }
    }
    const_iterator findBucket(const Id& id) const {  // routing_table.cpp:129-135
        return const_cast<RoutingTable*>(this)->findBucket(id);
    }
    // routing_table.cpp:59-65 depth()
    unsigned depth(const_iterator it) const {
        int bit1 = (int)it->first.lowbit();
        int bit2 = std::next(it) != end() ? (int)std::next(it)->first.lowbit() : -1;
        return std::max(bit1, bit2) + 1;
    }
    // routing_table.cpp:47-57 middle(); returns false where the reference throws out_of_range
    bool middle(const_iterator it, Id& out) const {
        unsigned bit = depth(it);
        if (bit >= 8 * HASH_LEN) return false;
        out = it->first;
        out.setBit(bit, 1);
        return true;
    }
    // routing_table.cpp:137-163 split()
    bool split(iterator b) {
        Id new_id;
        if (!middle(b, new_id)) return false;
        insert(std::next(b), Bucket{new_id, {}});
        std::list<std::shared_ptr<Node>> nodes;
        nodes.splice(nodes.begin(), b->nodes);
        while (!nodes.empty()) {
            auto n = nodes.begin();
            auto nb = findBucket((*n)->id);
            if (nb == end()) nodes.erase(n);
            else nb->nodes.splice(nb->nodes.begin(), nodes, n);
        }
        return true;
    }
    // routing_table.cpp:67-111 findClosestNodes()
    std::vector<std::shared_ptr<Node>> findClosestNodes(const Id& id, int64_t now, size_t count) const {
        std::vector<std::shared_ptr<Node>> nodes;
        auto bucket = findBucket(id);
        if (bucket == end()) return nodes;
        auto sortedBucketInsert = [&](const Bucket& b) {
            for (auto n : b.nodes) {
                if (!n->isGood(now)) continue;
                auto here = std::find_if(nodes.begin(), nodes.end(), [&](std::shared_ptr<Node>& node) {
                    return id.xorCmp(n->id, node->id) < 0;
                });
                nodes.insert(here, n);
            }
        };
        auto itn = bucket;
        // std::prev(begin()) is the list sentinel end() in libstdc++ (routing_table.cpp:90)
        auto itp = bucket == begin() ? end() : std::prev(bucket);
        while (nodes.size() < count && (itn != end() || itp != end())) {
            if (itn != end()) {
                sortedBucketInsert(*itn);
                itn = std::next(itn);
            }
            if (itp != end()) {
                sortedBucketInsert(*itp);
                if (itp == begin()) { itp = end(); continue; }
                itp = std::prev(itp);
            }
        }
        if (nodes.size() > count) nodes.resize(count);
        return nodes;
    }
};

// Structure-faithful NodeCache map for one family (include/opendht/node_cache.h:42-50,
// src/node_cache.cpp:36-66 getCachedNodes()).
struct NodeMap : std::map<Id, std::weak_ptr<Node>> {
    std::vector<std::shared_ptr<Node>> getCachedNodes(const Id& id, size_t count) const {
        const auto& c = *this;
        auto it_p = c.lower_bound(id), it_n = it_p;
        std::vector<std::shared_ptr<Node>> nodes;
        nodes.reserve(std::min(c.size(), count));
        const_iterator it;
        if (it_p != c.begin()) --it_p;
        while (nodes.size() < count && (it_n != c.end() || it_p != c.end())) {
            if (it_p == c.end()) it = it_n++;
            else if (it_n == c.end()) { it = it_p; it_p = (it_p == c.begin()) ? c.end() : std::prev(it_p); }
            else if (id.xorCmp(it_p->first, it_n->first) < 0) {
                it = it_p; it_p = (it_p == c.begin()) ? c.end() : std::prev(it_p);
            } else it = it_n++;
            // node_cache.cpp:57-58: taking begin() exhausts the p side
            if (it == c.begin()) it_p = c.end();
            if (auto n = it->second.lock())
                if (!n->isExpired()) nodes.emplace_back(std::move(n));
        }
        return nodes;
    }
};

// The faithful table owns its nodes (the reference's Dht owns them through the buckets).
struct FaithfulTable {
    RoutingTable rt;
    NodeMap nc;
    std::vector<std::shared_ptr<Node>> all;
    int64_t now = 0;
};

// ---------------------------------------------------------------------------
// Closed-form flat restatement (verified there against the
// compiled reference): W(r) = [max(0,b-1-r), min(B-1,b+r)], R = least r with
// good(W(r)) >= count or W(r) = whole table; result = first min(count, good(W(R)))
// good nodes of W(R) by (XOR distance, snapshot index).
// ---------------------------------------------------------------------------
struct Flat {
    uint32_t n = 0, B = 0;
    const uint8_t* ids = nullptr;
    const uint8_t* st = nullptr;
    const uint8_t* first = nullptr;
    const uint32_t* off = nullptr;
    const uint8_t* id(uint32_t i) const { return ids + (size_t)i * HASH_LEN; }
};

static inline int cmp20(const uint8_t* a, const uint8_t* b) { return std::memcmp(a, b, HASH_LEN); }
static inline int xorcmp20(const uint8_t* t, const uint8_t* a, const uint8_t* b) {
    for (unsigned i = 0; i < HASH_LEN; i++) {
        if (a[i] == b[i]) continue;
        return (uint8_t)(a[i] ^ t[i]) < (uint8_t)(b[i] ^ t[i]) ? -1 : 1;
    }
    return 0;
}

// routing_table.cpp:113-127 as upper_bound(first, t) - 1, clamped to 0 (the walk never
// tests the first bucket's lower bound).
static uint32_t flat_find_bucket(const Flat& f, const uint8_t* t) {
    uint32_t lo = 0, hi = f.B;  // count of firsts <= t
    while (lo < hi) {
        uint32_t mid = (lo + hi) / 2;
        if (cmp20(f.first + (size_t)mid * HASH_LEN, t) <= 0) lo = mid + 1; else hi = mid;
    }
    return lo == 0 ? 0 : lo - 1;
}

static uint32_t flat_rt_closest(const Flat& f, const uint8_t* t, uint32_t count, uint32_t* out) {
    if (f.B == 0 || count == 0) return 0;
    uint32_t b = flat_find_bucket(f, t);
    auto good_in = [&](uint32_t bk) {
        uint32_t g = 0;
        for (uint32_t i = f.off[bk]; i < f.off[bk + 1]; i++) g += f.st[i] & 1;
        return g;
    };
    // rounds
    int64_t lo = b, hi = b;  // current window [lo, hi]
    uint64_t good = good_in(b);
    if (b >= 1) { lo = b - 1; good += good_in(b - 1); }
    for (uint32_t r = 1; good < count && (lo > 0 || hi < (int64_t)f.B - 1); r++) {
        if (hi < (int64_t)f.B - 1) { hi++; good += good_in((uint32_t)hi); }
        if (lo > 0) { lo--; good += good_in((uint32_t)lo); }
    }
    std::vector<uint32_t> cand;
    for (uint32_t i = f.off[lo]; i < f.off[hi + 1]; i++)
        if (f.st[i] & 1) cand.push_back(i);
    std::sort(cand.begin(), cand.end(), [&](uint32_t x, uint32_t y) {
        int c = xorcmp20(t, f.id(x), f.id(y));
        return c != 0 ? c < 0 : x < y;
    });
    uint32_t m = (uint32_t)std::min<size_t>(count, cand.size());
    std::copy(cand.begin(), cand.begin() + m, out);
    return m;
}

// node_cache.cpp:36-66 over a sorted flat array; emits non-expired (status bit1 clear).
static uint32_t flat_nc_closest(const Flat& f, const uint8_t* t, uint32_t count, uint32_t* out) {
    uint32_t lo = 0, hi = f.n;  // lower_bound
    while (lo < hi) {
        uint32_t mid = (lo + hi) / 2;
        if (cmp20(f.id(mid), t) < 0) lo = mid + 1; else hi = mid;
    }
    const int64_t END = -1;
    int64_t n = lo < f.n ? (int64_t)lo : END;       // it_n (END == c.end())
    int64_t p = f.n == 0 ? END : (lo > 0 ? (int64_t)lo - 1 : (lo < f.n ? (int64_t)lo : END));
    uint32_t m = 0;
    while (m < count && (n != END || p != END)) {
        int64_t it;
        if (p == END) { it = n; n = (n + 1 < (int64_t)f.n) ? n + 1 : END; }
        else if (n == END) { it = p; p = p > 0 ? p - 1 : END; }
        else if (xorcmp20(t, f.id((uint32_t)p), f.id((uint32_t)n)) < 0) { it = p; p = p > 0 ? p - 1 : END; }
        else { it = n; n = (n + 1 < (int64_t)f.n) ? n + 1 : END; }
        if (it == 0) p = END;
        if (!(f.st[it] & 2)) out[m++] = (uint32_t)it;
    }
    return m;
}

template <class F>
static void parallel_for(uint32_t q, int nthreads, F fn) {
    if (nthreads <= 1 || q < 64) { fn(0u, q); return; }
    std::vector<std::thread> th;
    uint32_t per = (q + nthreads - 1) / nthreads;
    for (int k = 0; k < nthreads; k++) {
        uint32_t a = k * per, e = std::min(q, a + per);
        if (a >= e) break;
        th.emplace_back([=] { fn(a, e); });
    }
    for (auto& x : th) x.join();
}

}  // namespace orc

using namespace orc;

extern "C" {

// ---- primitives ----
int orc_cmp(const uint8_t* a, const uint8_t* b) {
    int c = Id::cmp(Id(a), Id(b));
    return c < 0 ? -1 : (c > 0 ? 1 : 0);
}
int orc_xor_cmp(const uint8_t* t, const uint8_t* a, const uint8_t* b) { return Id(t).xorCmp(Id(a), Id(b)); }
unsigned orc_common_bits(const uint8_t* a, const uint8_t* b) { return Id::commonBits(Id(a), Id(b)); }
unsigned orc_lowbit(const uint8_t* a) { return Id(a).lowbit(); }
int orc_get_bit(const uint8_t* a, unsigned n) { return Id(a).getBit(n); }
void orc_set_bit(uint8_t* a, unsigned n, int b) {
    Id x(a); x.setBit(n, b != 0); std::memcpy(a, x.data(), HASH_LEN);
}

// ---- synthetic IDs, identical recipe to the engine's kad_synth_ids ----
int orc_synth_ids(uint64_t seed, uint32_t n, uint8_t* out) {
    std::mt19937_64 g(seed);
    std::map<Id, int> seen;  // a different dedupe structure than the engine's, on purpose
    uint32_t i = 0;
    while (i < n) {
        uint64_t d[3] = {g(), g(), g()};
        uint8_t* p = out + (size_t)i * HASH_LEN;
        for (int k = 0; k < 8; k++) p[k] = (uint8_t)(d[0] >> (56 - 8 * k));
        for (int k = 0; k < 8; k++) p[8 + k] = (uint8_t)(d[1] >> (56 - 8 * k));
        for (int k = 0; k < 4; k++) p[16 + k] = (uint8_t)(d[2] >> (56 - 8 * k));
        if (seen.emplace(Id(p), 1).second) i++;
    }
    return 0;
}
int orc_synth_status(uint64_t seed, uint32_t n, uint32_t good_pct, uint32_t exp_pct, uint8_t* out) {
    std::mt19937_64 g(seed);
    for (uint32_t i = 0; i < n; i++) {
        uint32_t u = (uint32_t)(g() % 100);
        out[i] = u < good_pct ? 1 : (u < good_pct + exp_pct ? 2 : 0);
    }
    return 0;
}

// ---- structure-faithful table ----
void* orc_table_build(uint32_t n, const uint8_t* ids, const uint8_t* status, uint32_t B,
                      const uint8_t* first, const uint32_t* off, int with_nc) {
    auto* T = new FaithfulTable();
    T->now = 1000LL * 3600 * 1000000000LL;  // arbitrary steady_clock point (1000 h)
    T->all.reserve(n);
    for (uint32_t i = 0; i < n; i++) {
        auto nd = std::make_shared<Node>();
        nd->id = Id(ids + (size_t)i * HASH_LEN);
        nd->idx = i;
        apply_status(*nd, status[i], T->now);
        T->all.push_back(nd);
    }
    for (uint32_t b = 0; b < B; b++) {
        Bucket bk;
        bk.first = Id(first + (size_t)b * HASH_LEN);
        for (uint32_t i = off[b]; i < off[b + 1]; i++) bk.nodes.push_back(T->all[i]);
        T->rt.push_back(std::move(bk));
    }
    if (with_nc)
        for (uint32_t i = 0; i < n; i++) T->nc.emplace(T->all[i]->id, T->all[i]);
    return T;
}
void orc_table_free(void* h) { delete (FaithfulTable*)h; }

int orc_table_rt_closest(void* h, uint32_t q, const uint8_t* targets, uint32_t count,
                         uint32_t* out_idx, uint8_t* out_cnt, int nthreads) {
    auto* T = (FaithfulTable*)h;
    parallel_for(q, nthreads, [&](uint32_t a, uint32_t e) {
        for (uint32_t i = a; i < e; i++) {
            auto r = T->rt.findClosestNodes(Id(targets + (size_t)i * HASH_LEN), T->now, count);
            for (uint32_t j = 0; j < count; j++)
                out_idx[(size_t)i * count + j] = j < r.size() ? r[j]->idx : 0xFFFFFFFFu;
            out_cnt[i] = (uint8_t)r.size();
        }
    });
    return 0;
}
int orc_table_nc_closest(void* h, uint32_t q, const uint8_t* targets, uint32_t count,
                         uint32_t* out_idx, uint8_t* out_cnt, int nthreads) {
    auto* T = (FaithfulTable*)h;
    parallel_for(q, nthreads, [&](uint32_t a, uint32_t e) {
        for (uint32_t i = a; i < e; i++) {
            auto r = T->nc.getCachedNodes(Id(targets + (size_t)i * HASH_LEN), count);
            for (uint32_t j = 0; j < count; j++)
                out_idx[(size_t)i * count + j] = j < r.size() ? r[j]->idx : 0xFFFFFFFFu;
            out_cnt[i] = (uint8_t)r.size();
        }
    });
    return 0;
}
int orc_table_find_bucket(void* h, uint32_t q, const uint8_t* targets, uint32_t* out) {
    auto* T = (FaithfulTable*)h;
    for (uint32_t i = 0; i < q; i++) {
        auto it = T->rt.findBucket(Id(targets + (size_t)i * HASH_LEN));
        out[i] = it == T->rt.end() ? 0xFFFFFFFFu : (uint32_t)std::distance(T->rt.begin(), it);
    }
    return 0;
}

// ---- closed-form flat restatement ----
int orc_flat_rt_closest(uint32_t n, const uint8_t* ids, const uint8_t* status, uint32_t B,
                        const uint8_t* first, const uint32_t* off, uint32_t q, const uint8_t* targets,
                        uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, int nthreads) {
    Flat f; f.n = n; f.B = B; f.ids = ids; f.st = status; f.first = first; f.off = off;
    parallel_for(q, nthreads, [&](uint32_t a, uint32_t e) {
        std::vector<uint32_t> buf(count + 1);
        for (uint32_t i = a; i < e; i++) {
            uint32_t m = flat_rt_closest(f, targets + (size_t)i * HASH_LEN, count, buf.data());
            for (uint32_t j = 0; j < count; j++) out_idx[(size_t)i * count + j] = j < m ? buf[j] : 0xFFFFFFFFu;
            out_cnt[i] = (uint8_t)m;
        }
    });
    return 0;
}
int orc_flat_nc_closest(uint32_t n, const uint8_t* ids, const uint8_t* status, uint32_t q,
                        const uint8_t* targets, uint32_t count, uint32_t* out_idx, uint8_t* out_cnt,
                        int nthreads) {
    Flat f; f.n = n; f.ids = ids; f.st = status;
    parallel_for(q, nthreads, [&](uint32_t a, uint32_t e) {
        std::vector<uint32_t> buf(count + 1);
        for (uint32_t i = a; i < e; i++) {
            uint32_t m = flat_nc_closest(f, targets + (size_t)i * HASH_LEN, count, buf.data());
            for (uint32_t j = 0; j < count; j++) out_idx[(size_t)i * count + j] = j < m ? buf[j] : 0xFFFFFFFFu;
            out_cnt[i] = (uint8_t)m;
        }
    });
    return 0;
}
// Algorithmic bytes of a RoutingTable query: 20 + sum over W(R) of
// (8 + n_b + 20 g_b) + 4 count. Returns the total over the batch; also the number of
// visited buckets / nodes / good nodes (sums) through the out pointers.
uint64_t orc_flat_rt_bytes(uint32_t n, const uint8_t* ids, const uint8_t* status, uint32_t B,
                           const uint8_t* first, const uint32_t* off, uint32_t q, const uint8_t* targets,
                           uint32_t count, uint64_t* s_buckets, uint64_t* s_nodes, uint64_t* s_good) {
    Flat f; f.n = n; f.B = B; f.ids = ids; f.st = status; f.first = first; f.off = off;
    uint64_t tot = 0, sb = 0, sn = 0, sg = 0;
    for (uint32_t i = 0; i < q; i++) {
        tot += 20 + 4ull * count;
        if (B == 0 || count == 0) continue;
        const uint8_t* t = targets + (size_t)i * HASH_LEN;
        uint32_t b = flat_find_bucket(f, t);
        auto good_in = [&](uint32_t bk) {
            uint32_t g = 0;
            for (uint32_t k = off[bk]; k < off[bk + 1]; k++) g += status[k] & 1;
            return g;
        };
        int64_t lo = b, hi = b;
        uint64_t good = good_in(b);
        if (b >= 1) { lo = b - 1; good += good_in(b - 1); }
        while (good < count && (lo > 0 || hi < (int64_t)B - 1)) {
            if (hi < (int64_t)B - 1) { hi++; good += good_in((uint32_t)hi); }
            if (lo > 0) { lo--; good += good_in((uint32_t)lo); }
        }
        for (int64_t bk = lo; bk <= hi; bk++) {
            uint64_t nb = off[bk + 1] - off[bk], gb = good_in((uint32_t)bk);
            tot += 8 + nb + 20 * gb;
            sb++; sn += nb; sg += gb;
        }
    }
    if (s_buckets) *s_buckets = sb;
    if (s_nodes) *s_nodes = sn;
    if (s_good) *s_good = sg;
    return tot;
}

// ---- split-policy table builder, structure-faithful (dht.cpp:903-934 minus the my-bucket
// restriction; routing_table.cpp:137-163). Emits nodes grouped by bucket in list order.
int orc_split_table(uint32_t n, const uint8_t* ids, uint32_t cap, uint32_t* out_perm,
                    uint8_t* out_first, uint32_t* out_off, uint32_t* out_B) {
    RoutingTable rt;
    rt.push_back(Bucket{Id(), {}});
    std::vector<std::shared_ptr<Node>> all(n);
    for (uint32_t i = 0; i < n; i++) {
        all[i] = std::make_shared<Node>();
        all[i]->id = Id(ids + (size_t)i * HASH_LEN);
        all[i]->idx = i;
    }
    for (uint32_t i = 0; i < n; i++) {
        while (true) {
            auto b = rt.findBucket(all[i]->id);
            if (b->nodes.size() >= cap) {
                if (rt.split(b)) continue;
            }
            b->nodes.emplace_front(all[i]);  // dht.cpp:934
            break;
        }
    }
    uint32_t B = 0, k = 0;
    for (auto& b : rt) {
        std::memcpy(out_first + (size_t)B * HASH_LEN, b.first.data(), HASH_LEN);
        out_off[B] = k;
        for (auto& nd : b.nodes) out_perm[k++] = nd->idx;
        B++;
    }
    out_off[B] = k;
    *out_B = B;
    return 0;
}

// ---------------------------------------------------------------------------
// Wire step after the query
// ---------------------------------------------------------------------------
// NetworkEngine::bufferNodes(af, id, nodes) (src/network_engine.cpp:942-974): std::sort of the
// nodes by id.xorCmp (:945-947), truncation to SEND_NODES = 8 (:59, :948), then per node the
// 20-byte ID followed by sin_addr (4 bytes) + sin_port (2 bytes) for AF_INET (26-byte records,
// :950-960) or sin6_addr (16) + sin6_port (2) for AF_INET6 (38-byte records, :961-971).
// addr: per node addr_len = 6 or 18 bytes (address then port bytes, as stored in the sockaddr).
// Rows: q queries, candidate list idx[i*k .. i*k + cnt[i]) (node indices); out: q x 8 records.
uint32_t orc_buffer_nodes(uint32_t q, const uint8_t* targets, const uint8_t* ids, const uint8_t* addr,
                          uint32_t addr_len, const uint32_t* idx, const uint8_t* cnt, uint32_t k, uint8_t* out,
                          uint8_t* out_n) {
    const uint32_t rec = HASH_LEN + addr_len;
    for (uint32_t i = 0; i < q; i++) {
        const Id t(targets + (size_t)HASH_LEN * i);
        std::vector<uint32_t> nodes(idx + (size_t)i * k, idx + (size_t)i * k + cnt[i]);
        std::sort(nodes.begin(), nodes.end(), [&](uint32_t a, uint32_t b) {
            return t.xorCmp(Id(ids + (size_t)HASH_LEN * a), Id(ids + (size_t)HASH_LEN * b)) < 0;
        });
        const uint32_t nn = std::min<uint32_t>(8, (uint32_t)nodes.size());
        uint8_t* dst = out + (size_t)i * 8 * rec;
        for (uint32_t j = 0; j < nn; j++) {
            std::memcpy(dst + j * rec, ids + (size_t)HASH_LEN * nodes[j], HASH_LEN);
            std::memcpy(dst + j * rec + HASH_LEN, addr + (size_t)addr_len * nodes[j], addr_len);
        }
        out_n[i] = (uint8_t)nn;
    }
    return 0;
}

// NetworkEngine::isMartian (src/network_engine.cpp:308-339) on a 6-byte (v4) / 18-byte (v6)
// address + port record; v4prefix = ::ffff:0:0/96 (:55-57).
int orc_is_martian(const uint8_t* a, uint32_t addr_len) {
    if (addr_len == 6) {
        const bool port0 = a[4] == 0 && a[5] == 0;
        return port0 || a[0] == 0 || a[0] == 127 || (a[0] & 0xE0) == 0xE0;
    }
    static const uint8_t v4prefix[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0xFF, 0xFF};
    static const uint8_t z[15] = {0};
    const bool port0 = a[16] == 0 && a[17] == 0;
    return port0 || a[0] == 0xFF || (a[0] == 0xFE && (a[1] & 0xC0) == 0x80) ||
           (std::memcmp(a, z, 15) == 0 && (a[15] == 0 || a[15] == 1)) || std::memcmp(a, v4prefix, 12) == 0;
}

// NetworkEngine::deserializeNodes (src/network_engine.cpp:788-828) up to the table insertion:
// records of rec_len = 26 / 38 bytes, keep[i] = 0 for the sender's own ID (:798-799) or a martian
// address (:806, :822). (The blacklist and cache.getNode / onNewNode are host state.)
int orc_parse_nodes(uint32_t n, const uint8_t* in, uint32_t rec_len, const uint8_t* myid, uint8_t* keep) {
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t* r = in + (size_t)rec_len * i;
        keep[i] = !(std::memcmp(r, myid, HASH_LEN) == 0 || orc_is_martian(r + HASH_LEN, rec_len - HASH_LEN));
    }
    return 0;
}

}  // extern "C"
