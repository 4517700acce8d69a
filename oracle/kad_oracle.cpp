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
#include <mutex>
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

// ---------------------------------------------------------------------------
// Config 5 swarm model (SURVEY.md §8d "Config 5", §8f row 2). BUILD-DEFINED: the reference has no
// swarm simulator; parity is pinned per hop (RoutingTable::findClosestNodes on each peer's table,
// routing_table.cpp:67-111, and the Search::insertNode ordering, dht.cpp:961-1047).
//   Peer tables, shape K (Dht::onNewNode, dht.cpp:867-936: only my bucket splits, a full bucket
//   caches newcomers away): peer p with top-64 key k has depth D = the least D with at most 8 other
//   peers sharing >= D leading bits with it (capped at SW_LEVELS-1); for d < D the level-d bucket
//   holds min(8, |S_d|) peers of S_d (peers sharing exactly d bits), picked at positions
//   lo + (off + j*|S_d|/8) % |S_d|, off = mix(k ^ (d+1)*GOLDEN) % |S_d|; my bucket holds the first 8
//   other peers sharing >= D bits, in ID order. All peers good.
//   Lookup: the source's findClosestNodes(t, SEARCH_NODES=14) seeds the list; each synchronous hop
//   queries the first <= 4 (MAX_REQUESTED_SEARCH_NODES, dht.h:327) unqueried nodes in list order,
//   each answers findClosestNodes(t, TARGET_NODES=8) from its own table, answers equal to the source
//   are dropped (deserializeNodes, network_engine.cpp:798-799), the rest go through insertNode (sorted
//   insert, trim to 14). Done when the first min(8, |list|) nodes have all been queried
//   (Search::isSynced, dht.cpp:1467-1478), or stalled when no unqueried node is left.
// ---------------------------------------------------------------------------
static constexpr uint32_t SW_LEVELS = 28, SW_BUCKET = 8, SW_SEARCH = 14, SW_ALPHA = 4;

static inline uint64_t sw_mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

struct Swarm {
    uint32_t n;
    const uint8_t* ids;
    std::vector<uint64_t> key;
    std::unique_ptr<uint8_t[]> depth, counts;  // counts[p*SW_LEVELS + level]
    std::unique_ptr<uint32_t[]> ent;           // ent[(p*SW_LEVELS + level)*SW_BUCKET + j]
    std::unique_ptr<std::once_flag[]> once;    // lazy model: each peer's table built on first use
    void ensure(uint32_t p) const {
        if (once) std::call_once(once[p], [&] { const_cast<Swarm*>(this)->build(p); });
    }
    // peers whose top-64 key starts with the L-bit prefix P: [lo, hi)
    void range(uint64_t P, uint32_t L, uint32_t& lo, uint32_t& hi) const {
        if (L == 0) { lo = 0; hi = n; return; }
        const uint64_t a = P << (64 - L);
        lo = (uint32_t)(std::lower_bound(key.begin(), key.end(), a) - key.begin());
        if (P + 1 == (L == 64 ? 0 : (1ull << L))) { hi = n; return; }
        hi = (uint32_t)(std::lower_bound(key.begin(), key.end(), (P + 1) << (64 - L)) - key.begin());
    }
    void build(uint32_t p) {
        const uint64_t k = key[p];
        uint32_t D = 0, lo, hi;
        for (;; D++) {
            range(D ? k >> (64 - D) : 0, D, lo, hi);
            if (hi - lo - 1 <= SW_BUCKET || D == SW_LEVELS - 1) break;
        }
        depth[p] = (uint8_t)D;
        for (uint32_t d = 0; d < SW_LEVELS; d++) {
            counts[(size_t)p * SW_LEVELS + d] = 0;
            for (uint32_t j = 0; j < SW_BUCKET; j++) ent[((size_t)p * SW_LEVELS + d) * SW_BUCKET + j] = 0xFFFFFFFFu;
        }
        for (uint32_t d = 0; d < D; d++) {
            uint32_t a, e;
            range((k >> (63 - d)) ^ 1ull, d + 1, a, e);
            const uint32_t m = e - a, c = std::min(m, SW_BUCKET);
            uint32_t* out = &ent[((size_t)p * SW_LEVELS + d) * SW_BUCKET];
            const uint64_t off = m > SW_BUCKET ? sw_mix(k ^ ((uint64_t)(d + 1) * 0x9E3779B97F4A7C15ull)) % m : 0;
            for (uint32_t j = 0; j < c; j++) out[j] = m > SW_BUCKET ? a + (uint32_t)((off + (uint64_t)j * m / SW_BUCKET) % m) : a + j;
            counts[(size_t)p * SW_LEVELS + d] = (uint8_t)c;
        }
        uint32_t* out = &ent[((size_t)p * SW_LEVELS + D) * SW_BUCKET];
        uint32_t c = 0;
        for (uint32_t x = lo; x < hi && c < SW_BUCKET; x++)
            if (x != p) out[c++] = x;
        counts[(size_t)p * SW_LEVELS + D] = (uint8_t)c;
    }
    // p's table as a RoutingTable (buckets sorted by first) -> findClosestNodes(t, count)
    void closest(uint32_t p, const Id& t, uint32_t count, std::vector<uint32_t>& out) const {
        ensure(p);
        out.clear();
        const Id me(ids + (size_t)HASH_LEN * p);
        const uint32_t D = depth[p];
        struct Bk { Id first; uint32_t level; };
        std::vector<Bk> bk;
        for (uint32_t d = 0; d <= D; d++) {
            Id f;  // first: my first d bits, bit d flipped (levels), zeros after; my bucket: my first D bits
            for (uint32_t b = 0; b < d; b++) f.setBit(b, me.getBit(b));
            if (d < D) f.setBit(d, !me.getBit(d));
            bk.push_back({f, d});
        }
        std::sort(bk.begin(), bk.end(), [](const Bk& a, const Bk& b) { return a.first < b.first; });
        const uint32_t B = (uint32_t)bk.size();
        uint32_t b = 0;  // upper_bound(first, t) - 1, clamped (routing_table.cpp:113-127)
        while (b + 1 < B && !(t < bk[b + 1].first)) b++;
        auto cnt = [&](uint32_t i) { return (uint32_t)counts[(size_t)p * SW_LEVELS + bk[i].level]; };
        uint32_t r = 0, lo, hi;
        for (;; r++) {
            lo = b > r ? b - 1 - r : 0;
            hi = std::min(B - 1, b + r);
            uint32_t g = 0;
            for (uint32_t i = lo; i <= hi; i++) g += cnt(i);
            if (g >= count || (lo == 0 && hi == B - 1)) break;
        }
        std::vector<uint32_t> cand;
        for (uint32_t i = lo; i <= hi; i++)
            for (uint32_t j = 0; j < cnt(i); j++) cand.push_back(ent[((size_t)p * SW_LEVELS + bk[i].level) * SW_BUCKET + j]);
        std::stable_sort(cand.begin(), cand.end(), [&](uint32_t x, uint32_t y) {
            return t.xorCmp(Id(ids + (size_t)HASH_LEN * x), Id(ids + (size_t)HASH_LEN * y)) < 0;
        });
        if (cand.size() > count) cand.resize(count);
        out = cand;
    }
};

extern "C" {
static Swarm* swarm_alloc(uint32_t n, const uint8_t* sorted_ids) {
    Swarm* s = new Swarm;
    s->n = n;
    s->ids = sorted_ids;
    s->key.resize(n);
    for (uint32_t i = 0; i < n; i++) {
        uint64_t k = 0;
        for (int b = 0; b < 8; b++) k = (k << 8) | sorted_ids[(size_t)HASH_LEN * i + b];
        s->key[i] = k;
    }
    // not value-initialised: a lazy model touches only the pages of the peers it builds
    s->depth.reset(new uint8_t[n]);
    s->counts.reset(new uint8_t[(size_t)n * SW_LEVELS]);
    s->ent.reset(new uint32_t[(size_t)n * SW_LEVELS * SW_BUCKET]);
    return s;
}
void* orc_swarm_build(uint32_t n, const uint8_t* sorted_ids, int nthreads) {
    Swarm* s = swarm_alloc(n, sorted_ids);
    parallel_for(n, nthreads, [&](uint32_t a, uint32_t e) { for (uint32_t p = a; p < e; p++) s->build(p); });
    return s;
}
// The same model with each peer's table built when a query first reaches it (swarms of 10M peers, of which a
// sample of lookups touches a few thousand).
void* orc_swarm_build_lazy(uint32_t n, const uint8_t* sorted_ids) {
    Swarm* s = swarm_alloc(n, sorted_ids);
    s->once.reset(new std::once_flag[n]);
    return s;
}
void orc_swarm_free(void* h) { delete (Swarm*)h; }
void orc_swarm_table(void* h, uint32_t p, uint32_t* depth, uint8_t* counts, uint32_t* ent) {
    const Swarm* s = (const Swarm*)h;
    s->ensure(p);
    *depth = s->depth[p];
    std::memcpy(counts, &s->counts[(size_t)p * SW_LEVELS], SW_LEVELS);
    std::memcpy(ent, &s->ent[(size_t)p * SW_LEVELS * SW_BUCKET], 4ull * SW_LEVELS * SW_BUCKET);
}
int orc_swarm_closest(void* h, uint32_t q, const uint32_t* peers, const uint8_t* targets, uint32_t count,
                      uint32_t* out_idx, uint8_t* out_cnt, int nthreads) {
    const Swarm* s = (const Swarm*)h;
    parallel_for(q, nthreads, [&](uint32_t a, uint32_t e) {
        std::vector<uint32_t> r;
        for (uint32_t i = a; i < e; i++) {
            s->closest(peers[i], Id(targets + (size_t)HASH_LEN * i), count, r);
            for (uint32_t j = 0; j < count; j++) out_idx[(size_t)i * count + j] = j < r.size() ? r[j] : 0xFFFFFFFFu;
            out_cnt[i] = (uint8_t)r.size();
        }
    });
    return 0;
}
// Lookups for S (source, target) pairs, at most max_hops hops each, with a share of the peers offline
// (offline_per_10k / 10000 of them, by a hash of the peer index: swarm_offline). Outputs: list S x
// SW_LIST (NO_NODE padded), queried flags and bad flags S x SW_LIST, list length, hops done, done
// (0 running, 1 synced, 2 stalled, 3 expired). Search::insertNode (dht.cpp:961-1047) with its bad-node
// accounting: the list keeps SEARCH_NODES non-bad nodes and the bad ones among them, an insert beyond the
// trim point is refused. A queried peer that is offline does not answer; after the hop its node is
// expired (the request's MAX_ATTEMPT_COUNT = 3 tries ran out, network_engine.cpp:243-247) and it is a bad
// search node (SearchNode::isBad, dht.cpp:458-460). Within a hop the answers are merged in the order of the
// queried nodes, then the silent ones turn bad. The next hop queries the first <= 4 nodes in list order
// that are neither queried nor bad (searchSendGetValues / canGet, dht.cpp:302-304, 1171-1235). Synced:
// the first TARGET_NODES non-bad nodes have all answered (Search::isSynced, dht.cpp:1467-1478). Expired:
// the first min(size, SEARCH_MAX_BAD_NODES = 25) nodes are all bad (searchStep, dht.cpp:1451-1457).
// Not modelled (documented in DESIGN.md §7.2): removeExpiredNode needs a node expired for 10 minutes,
// longer than a lookup; `candidate` only matters after a search is synced.
static constexpr uint32_t SW_LIST = 32, SW_MAX_BAD = 25;

static inline bool swarm_offline(uint32_t p, uint32_t per10k) {
    return per10k && (uint32_t)(sw_mix((uint64_t)p * 0x9E37ull + 0xBADull) % 10000ull) < per10k;
}

int orc_swarm_search_ex(void* h, uint32_t S, const uint32_t* src, const uint8_t* targets, uint32_t max_hops,
                        uint32_t offline_per_10k, uint32_t* out_list, uint8_t* out_q, uint8_t* out_bad, uint8_t* out_n,
                        uint32_t* out_hops, uint8_t* out_done, int nthreads) {
    const Swarm* s = (const Swarm*)h;
    struct SN { uint32_t idx; uint8_t queried, bad; };
    parallel_for(S, nthreads, [&](uint32_t a, uint32_t e) {
      for (uint32_t i = a; i < e; i++) {
        const Id t(targets + (size_t)HASH_LEN * i);
        std::vector<SN> L;
        std::vector<uint32_t> init;
        s->closest(src[i], t, SW_SEARCH, init);
        for (uint32_t v : init) L.push_back(SN{v, 0, 0});
        uint32_t hops = 0;
        uint8_t done = 0;
        auto id_of = [&](uint32_t v) { return Id(s->ids + (size_t)HASH_LEN * v); };
        // the peers this search queried that stayed silent: their nodes are expired from then on
        std::vector<uint32_t> silent;
        // Search::insertNode(node) (dht.cpp:961-1047, expired search = false); an expired node joins as a bad
        // search node (`if (node.isExpired()) bad++`, :1023-1025)
        auto insert = [&](uint32_t r) {
            const Id rid = id_of(r);
            size_t n = L.size();
            bool found = false;
            while (n > 0) {
                --n;
                if (L[n].idx == r) { found = true; break; }
                if (t.xorCmp(rid, id_of(L[n].idx)) > 0) { ++n; break; }
            }
            if (found) return;
            size_t bad = 0;
            for (const SN& x : L) bad += x.bad;
            const bool full = L.size() - bad >= SW_SEARCH;
            size_t tt = L.size();
            while (tt - bad > SW_SEARCH) {
                --tt;
                if (L[tt].bad) bad--;
            }
            if (full) {
                if (tt != L.size()) L.resize(tt);
                if (n >= tt) return;
            }
            const bool rbad = std::find(silent.begin(), silent.end(), r) != silent.end();
            L.insert(L.begin() + n, SN{r, 0, (uint8_t)(rbad ? 1 : 0)});
            bad += rbad ? 1 : 0;
            while (L.size() - bad > SW_SEARCH) {
                if (L.back().bad) bad--;
                L.pop_back();
            }
        };
        std::vector<uint32_t> sel;
        auto select = [&]() {
            sel.clear();
            for (size_t j = 0; j < L.size() && sel.size() < SW_ALPHA; j++)
                if (!L[j].queried && !L[j].bad) { sel.push_back(L[j].idx); L[j].queried = 1; }
            if (sel.empty()) done = 2;  // stalled
        };
        select();
        while (!done && hops < max_hops) {
            hops++;
            std::vector<uint32_t> rep;
            for (uint32_t v : sel) {
                if (swarm_offline(v, offline_per_10k)) continue;  // no answer this hop
                s->closest(v, t, SW_BUCKET, rep);
                for (uint32_t r : rep)
                    if (r != src[i]) insert(r);  // deserializeNodes drops our own ID (network_engine.cpp:798-799)
            }
            for (uint32_t v : sel)  // the silent ones: expired after their tries, bad search nodes
                if (swarm_offline(v, offline_per_10k)) {
                    silent.push_back(v);
                    for (SN& x : L)
                        if (x.idx == v) x.bad = 1;
                }
            uint32_t good = 0;  // Search::isSynced
            bool synced = true;
            for (const SN& x : L) {
                if (x.bad) continue;
                if (!x.queried) { synced = false; break; }
                if (++good == SW_BUCKET) break;
            }
            uint32_t cb = 0;  // getNumberOfConsecutiveBadNodes
            while (cb < L.size() && L[cb].bad) cb++;
            if (synced && good > 0) done = 1;
            else if (!L.empty() && cb >= std::min<size_t>(L.size(), SW_MAX_BAD)) done = 3;
            else select();
        }
        for (uint32_t j = 0; j < SW_LIST; j++) {
            out_list[(size_t)i * SW_LIST + j] = j < L.size() ? L[j].idx : 0xFFFFFFFFu;
            out_q[(size_t)i * SW_LIST + j] = j < L.size() ? L[j].queried : 0;
            out_bad[(size_t)i * SW_LIST + j] = j < L.size() ? L[j].bad : 0;
        }
        out_n[i] = (uint8_t)std::min<size_t>(L.size(), 255);
        out_hops[i] = hops;
        out_done[i] = done;
      }
    });
    return 0;
}

// All peers online (the round-1 interface): lists of SEARCH_NODES.
int orc_swarm_search(void* h, uint32_t S, const uint32_t* src, const uint8_t* targets, uint32_t max_hops,
                     uint32_t* out_list, uint8_t* out_q, uint8_t* out_n, uint32_t* out_hops, uint8_t* out_done,
                     int nthreads) {
    std::vector<uint32_t> l((size_t)S * SW_LIST);
    std::vector<uint8_t> q((size_t)S * SW_LIST), bad((size_t)S * SW_LIST);
    orc_swarm_search_ex(h, S, src, targets, max_hops, 0, l.data(), q.data(), bad.data(), out_n, out_hops, out_done,
                        nthreads);
    for (size_t i = 0; i < S; i++)
        for (uint32_t j = 0; j < SW_SEARCH; j++) {
            out_list[i * SW_SEARCH + j] = l[i * SW_LIST + j];
            out_q[i * SW_SEARCH + j] = q[i * SW_LIST + j];
        }
    return 0;
}
}  // extern "C" (swarm)

// ---------------------------------------------------------------------------
// InfoHash::get (src/infohash.cpp:46-61): GnuTLS SHA-1 of the data (HASH_LEN 20 -> GNUTLS_DIG_SHA1).
// GnuTLS is absent here; this is FIPS 180-4 SHA-1, pinned by the standard's test vectors
// (tests/test_sha1.py). SURVEY.md §8f row 4.
// ---------------------------------------------------------------------------
static inline uint32_t rol(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }
static void sha1(const uint8_t* m, uint64_t len, uint8_t* out) {
    uint32_t h[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
    const uint64_t nblk = (len + 8) / 64 + 1;
    for (uint64_t b = 0; b < nblk; b++) {
        uint8_t blk[64];
        for (int i = 0; i < 64; i++) {
            const uint64_t j = 64 * b + i;
            blk[i] = j < len ? m[j] : (j == len ? 0x80 : 0);
        }
        if (b == nblk - 1)
            for (int i = 0; i < 8; i++) blk[56 + i] = (uint8_t)((len * 8) >> (56 - 8 * i));
        uint32_t w[80];
        for (int i = 0; i < 16; i++) w[i] = (uint32_t)blk[4 * i] << 24 | (uint32_t)blk[4 * i + 1] << 16 | (uint32_t)blk[4 * i + 2] << 8 | blk[4 * i + 3];
        for (int i = 16; i < 80; i++) w[i] = rol(w[i - 3] ^ w[i - 8] ^ w[i - 14] ^ w[i - 16], 1);
        uint32_t a = h[0], bb = h[1], c = h[2], d = h[3], e = h[4];
        for (int i = 0; i < 80; i++) {
            uint32_t f, k;
            if (i < 20) { f = (bb & c) | (~bb & d); k = 0x5A827999u; }
            else if (i < 40) { f = bb ^ c ^ d; k = 0x6ED9EBA1u; }
            else if (i < 60) { f = (bb & c) | (bb & d) | (c & d); k = 0x8F1BBCDCu; }
            else { f = bb ^ c ^ d; k = 0xCA62C1D6u; }
            const uint32_t t = rol(a, 5) + f + e + k + w[i];
            e = d; d = c; c = rol(bb, 30); bb = a; a = t;
        }
        h[0] += a; h[1] += bb; h[2] += c; h[3] += d; h[4] += e;
    }
    for (int i = 0; i < 5; i++)
        for (int j = 0; j < 4; j++) out[4 * i + j] = (uint8_t)(h[i] >> (24 - 8 * j));
}

extern "C" int orc_infohash_get(uint32_t n, const uint8_t* data, const uint64_t* off, uint8_t* out) {
    for (uint32_t i = 0; i < n; i++) sha1(data + off[i], off[i + 1] - off[i], out + (size_t)HASH_LEN * i);
    return 0;
}

// ---------------------------------------------------------------------------
// Incremental mirror ops on the structure-faithful table. Ops are applied in
// order; node operands are indices of the table at the batch start, `slot` operands index the
// batch's new nodes:
//   REMOVE  a     the old node a leaves its bucket (Dht::expireBuckets remove_if, dht.cpp:942-956)
//   REPLACE a s   new node s takes old node a's place (onNewNode's expired replacement, dht.cpp:917-921)
//   INSERT  s     new node s is emplace_front'ed into findBucket(id) (dht.cpp:934)
//   SPLIT   b     RoutingTable::split of the bucket at current index b (routing_table.cpp:137-163)
// Then the table is written out: ids/status in bucket then list order, firsts, offsets, the new
// index of every old node (NO_NODE if removed or replaced) and of every new node.
// ---------------------------------------------------------------------------
extern "C" int orc_table_apply(void* h, uint32_t n_ops, const uint32_t* ops, uint32_t n_new, const uint8_t* new_ids,
                               const uint8_t* new_status, uint32_t* out_n, uint32_t* out_B, uint8_t* out_ids,
                               uint8_t* out_status, uint8_t* out_first, uint32_t* out_off, uint32_t* out_remap,
                               uint32_t* out_new_idx) {
    auto* T = (FaithfulTable*)h;
    const uint32_t n_old = (uint32_t)T->all.size();
    std::vector<std::shared_ptr<Node>> fresh(n_new);
    for (uint32_t s = 0; s < n_new; s++) {
        fresh[s] = std::make_shared<Node>();
        fresh[s]->id = Id(new_ids + (size_t)s * HASH_LEN);
        fresh[s]->idx = n_old + s;
        apply_status(*fresh[s], new_status[s], T->now);
    }
    auto locate = [&](uint32_t old) {  // (bucket, node) iterators of an old node
        for (auto b = T->rt.begin(); b != T->rt.end(); ++b)
            for (auto n = b->nodes.begin(); n != b->nodes.end(); ++n)
                if ((*n)->idx == old) return std::make_pair(b, n);
        return std::make_pair(T->rt.end(), std::list<std::shared_ptr<Node>>::iterator());
    };
    for (uint32_t o = 0; o < n_ops; o++) {
        const uint32_t kind = ops[3 * o], a = ops[3 * o + 1], b = ops[3 * o + 2];
        if (kind == 1) {  // REMOVE
            auto p = locate(a);
            if (p.first != T->rt.end()) p.first->nodes.erase(p.second);
        } else if (kind == 2) {  // REPLACE
            auto p = locate(a);
            if (p.first != T->rt.end()) *p.second = fresh[b];
        } else if (kind == 3) {  // INSERT
            auto bk = T->rt.findBucket(fresh[a]->id);
            if (bk != T->rt.end()) bk->nodes.emplace_front(fresh[a]);
        } else if (kind == 4) {  // SPLIT
            auto bk = T->rt.begin();
            std::advance(bk, a);
            T->rt.split(bk);
        }
    }
    for (uint32_t i = 0; i < n_old; i++) out_remap[i] = 0xFFFFFFFFu;
    for (uint32_t s = 0; s < n_new; s++) out_new_idx[s] = 0xFFFFFFFFu;
    uint32_t k = 0, B = 0;
    for (auto& bk : T->rt) {
        std::memcpy(out_first + (size_t)B * HASH_LEN, bk.first.data(), HASH_LEN);
        out_off[B++] = k;
        for (auto& nd : bk.nodes) {
            std::memcpy(out_ids + (size_t)k * HASH_LEN, nd->id.data(), HASH_LEN);
            out_status[k] = (nd->isExpired() ? 2 : 0) | (nd->isGood(T->now) ? 1 : 0);
            if (nd->idx < n_old) out_remap[nd->idx] = k;
            else out_new_idx[nd->idx - n_old] = k;
            k++;
        }
    }
    out_off[B] = k;
    *out_n = k;
    *out_B = B;
    return 0;
}
