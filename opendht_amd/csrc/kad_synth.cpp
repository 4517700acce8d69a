// kad_synth.cpp — synthetic routing tables for the bench and the tests (host C++).
//
// Table shapes of SURVEY.md §8d:
//   U(d)  uniform depth: bucket firsts prefix << (160-d)                  kad_uniform_buckets
//   S     reference split policy: insert in order, split a full bucket    kad_split_table
//         (Dht::onNewNode dht.cpp:903-934 without the my-bucket restriction,
//          RoutingTable::split/middle/depth routing_table.cpp:47-65,137-163)
//   swarm counter-based U(d) shard: any bucket range reproducible alone   kad_synth_uniform_shard
// IDs: std::mt19937_64 recipe of SURVEY.md §8d                            kad_synth_ids
#include <algorithm>
#include <atomic>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <random>
#include <set>
#include <thread>

#include <vector>

#include "../../include/kadgpu.h"

namespace {

using Id = std::array<uint8_t, 20>;

inline int cmp_id(const uint8_t* a, const uint8_t* b) { return std::memcmp(a, b, 20); }

// InfoHash::lowbit (infohash.h:84-95) on raw bytes; -1 for zero.
int lowbit(const uint8_t* p) {
    int i;
    for (i = 19; i >= 0; i--)
        if (p[i]) break;
    if (i < 0) return -1;
    int j;
    for (j = 7; j >= 0; j--)
        if (p[i] & (0x80 >> j)) break;
    return 8 * i + j;
}

void write_draws(uint8_t* p, uint64_t d0, uint64_t d1, uint64_t d2) {
    for (int k = 0; k < 8; k++) p[k] = (uint8_t)(d0 >> (56 - 8 * k));
    for (int k = 0; k < 8; k++) p[8 + k] = (uint8_t)(d1 >> (56 - 8 * k));
    for (int k = 0; k < 4; k++) p[16 + k] = (uint8_t)(d2 >> (56 - 8 * k));
}

inline uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

int nthreads() {
    unsigned h = std::thread::hardware_concurrency();
    return (int)std::max(1u, std::min(h, 16u));
}

template <class F>
void par_for(uint64_t n, F fn) {
    int T = n < 4096 ? 1 : nthreads();
    if (T == 1) { fn(0, n); return; }
    std::vector<std::thread> th;
    uint64_t per = (n + T - 1) / T;
    for (int k = 0; k < T; k++) {
        uint64_t a = k * per, e = std::min(n, a + per);
        if (a >= e) break;
        th.emplace_back([=] { fn(a, e); });
    }
    for (auto& x : th) x.join();
}

// Poisson(mean) by multiplication (Knuth); deterministic for a given stream.
uint32_t poisson(uint64_t& st, double mean) {
    const double L = std::exp(-mean);
    uint32_t k = 0;
    double p = 1.0;
    do {
        k++;
        p *= (double)(splitmix64(st) >> 11) * (1.0 / 9007199254740992.0);
    } while (p > L);
    return k - 1;
}

}  // namespace

extern "C" {

int kad_synth_ids(uint64_t seed, uint32_t n, uint8_t* out) {
    if (n && !out) return KAD_ERR_INVALID;
    std::mt19937_64 g(seed);
    for (uint32_t i = 0; i < n; i++) {
        uint64_t d0 = g(), d1 = g(), d2 = g();
        write_draws(out + 20ull * i, d0, d1, d2);
    }
    // Duplicates among 160-bit draws are (astronomically) rare: detect them by sorting an
    // index and, only if one exists, redo the exact sequential reject-and-redraw procedure.
    std::vector<uint32_t> ord(n);
    for (uint32_t i = 0; i < n; i++) ord[i] = i;
    std::sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return cmp_id(out + 20ull * a, out + 20ull * b) < 0; });
    bool dup = false;
    for (uint32_t i = 1; i < n && !dup; i++) dup = cmp_id(out + 20ull * ord[i - 1], out + 20ull * ord[i]) == 0;
    if (!dup) return KAD_OK;
    std::set<Id> seen;
    std::mt19937_64 h(seed);
    uint32_t i = 0;
    while (i < n) {
        Id x;
        uint64_t d0 = h(), d1 = h(), d2 = h();
        write_draws(x.data(), d0, d1, d2);
        if (seen.insert(x).second) std::memcpy(out + 20ull * i++, x.data(), 20);
    }
    return KAD_OK;
}

int kad_synth_status(uint64_t seed, uint32_t n, uint32_t good_pct, uint32_t expired_pct, uint8_t* out) {
    if (n && !out) return KAD_ERR_INVALID;
    std::mt19937_64 g(seed);
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t u = (uint32_t)(g() % 100);
        out[i] = u < good_pct ? KAD_STATUS_GOOD : (u < good_pct + expired_pct ? KAD_STATUS_EXPIRED : 0);
    }
    return KAD_OK;
}

int kad_sort_ids(uint32_t n, uint8_t* ids, uint32_t* out_perm) {
    if (n && !ids) return KAD_ERR_INVALID;
    std::vector<uint32_t> ord(n);
    for (uint32_t i = 0; i < n; i++) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return cmp_id(ids + 20ull * a, ids + 20ull * b) < 0; });
    std::vector<uint8_t> tmp((size_t)n * 20);
    for (uint32_t i = 0; i < n; i++) std::memcpy(tmp.data() + 20ull * i, ids + 20ull * ord[i], 20);
    if (n == 0) return KAD_OK;  // (memcpy from an empty vector's NULL data() is undefined)
    std::memcpy(ids, tmp.data(), tmp.size());
    if (out_perm) std::memcpy(out_perm, ord.data(), 4ull * n);
    return KAD_OK;
}

int kad_uniform_buckets(uint32_t n, const uint8_t* ids, uint32_t depth, uint64_t prefix_lo, uint64_t prefix_hi,
                        uint8_t* out_first, uint32_t* out_offset) {
    if (depth == 0 || depth > 63) return KAD_ERR_INVALID;
    if (prefix_hi == 0) prefix_hi = 1ull << depth;
    if (prefix_hi <= prefix_lo || prefix_hi > (1ull << depth)) return KAD_ERR_INVALID;
    const uint64_t B = prefix_hi - prefix_lo;
    if (B >= 0x7FFFFFFFull || !out_first || !out_offset) return KAD_ERR_INVALID;
    par_for(B, [&](uint64_t a, uint64_t e) {
        for (uint64_t j = a; j < e; j++) {
            uint8_t* f = out_first + 20ull * j;
            std::memset(f, 0, 20);
            const uint64_t hi = (prefix_lo + j) << (64 - depth);
            for (int k = 0; k < 8; k++) f[k] = (uint8_t)(hi >> (56 - 8 * k));
            // node offset = lower_bound(first_j); bucket 0 also takes ids below its first
            // (findBucket clamps to begin(), routing_table.cpp:113-127)
            uint32_t lo = 0, h = n;
            while (lo < h) {
                uint32_t mid = (lo + h) / 2;
                if (cmp_id(ids + 20ull * mid, f) < 0) lo = mid + 1; else h = mid;
            }
            out_offset[j] = j == 0 ? 0 : lo;
        }
    });
    out_offset[B] = n;
    return KAD_OK;
}

int kad_split_table(uint32_t n, const uint8_t* ids, uint32_t cap, uint32_t* out_perm, uint8_t* out_first,
                    uint32_t* out_offset, uint32_t* out_n_buckets) {
    if (n && !ids) return KAD_ERR_INVALID;
    if (!out_perm || !out_first || !out_offset || !out_n_buckets || cap == 0) return KAD_ERR_INVALID;
    // The list of buckets as an ordered map first -> node list (RoutingTable list order inside a bucket:
    // front = most recently emplaced, dht.cpp:934); O(log B) per findBucket and per split.
    struct IdLess {
        bool operator()(const Id& a, const Id& b) const { return cmp_id(a.data(), b.data()) < 0; }
    };
    using Map = std::map<Id, std::vector<uint32_t>, IdLess>;
    Map buckets;
    Id zero;
    zero.fill(0);  // the initial bucket covers the whole space from zeroes
    buckets.emplace(zero, std::vector<uint32_t>());
    auto find_bucket = [&](const uint8_t* id) -> Map::iterator {
        // routing_table.cpp:113-127: last bucket with first <= id, clamped to the first bucket
        Id key;
        std::memcpy(key.data(), id, 20);
        auto it = buckets.upper_bound(key);
        return it == buckets.begin() ? it : std::prev(it);
    };
    auto split = [&](Map::iterator b) -> bool {
        // depth (routing_table.cpp:59-65), middle (:47-57), split (:137-163)
        const auto next = std::next(b);
        const int bit1 = lowbit(b->first.data());
        const int bit2 = next != buckets.end() ? lowbit(next->first.data()) : -1;
        const int bit = std::max(bit1, bit2) + 1;
        if (bit >= 160) return false;
        Id mid = b->first;
        mid[bit / 8] |= (uint8_t)(0x80 >> (bit % 8));
        auto nb = buckets.emplace_hint(next, mid, std::vector<uint32_t>());
        std::vector<uint32_t> moving;
        moving.swap(b->second);
        for (uint32_t idx : moving) {  // each spliced to the FRONT of its bucket, in list order
            auto& dst = cmp_id(ids + 20ull * idx, mid.data()) < 0 ? b->second : nb->second;
            dst.insert(dst.begin(), idx);
        }
        return true;
    };
    for (uint32_t i = 0; i < n; i++) {
        const uint8_t* id = ids + 20ull * i;
        bool placed = true;
        auto b = find_bucket(id);
        while (b->second.size() >= cap) {
            if (!split(b)) { placed = false; break; }  // unsplittable: the node is cached away, not added
            b = find_bucket(id);
        }
        if (placed) b->second.insert(b->second.begin(), i);
    }
    uint32_t k = 0, j = 0;
    for (const auto& kv : buckets) {
        std::memcpy(out_first + 20ull * j, kv.first.data(), 20);
        out_offset[j++] = k;
        for (uint32_t idx : kv.second) out_perm[k++] = idx;
    }
    out_offset[j] = k;
    *out_n_buckets = j;
    return KAD_OK;
}

int kad_synth_uniform_shard(uint64_t seed, uint32_t depth, uint64_t prefix_lo, uint64_t prefix_hi,
                            double mean_per_bucket, uint32_t good_pct, uint32_t expired_pct, uint32_t* out_n,
                            uint8_t* out_ids, uint8_t* out_status, uint32_t* out_offset) {
    if (depth == 0 || depth > 63 || !out_n || !(mean_per_bucket > 0) || mean_per_bucket > 64) return KAD_ERR_INVALID;
    if (prefix_hi == 0) prefix_hi = 1ull << depth;
    if (prefix_hi <= prefix_lo || prefix_hi > (1ull << depth)) return KAD_ERR_INVALID;
    const uint64_t B = prefix_hi - prefix_lo;
    if (B >= 0x7FFFFFFFull) return KAD_ERR_INVALID;
    // per-bucket counts from a counting stream keyed by (seed, prefix)
    std::vector<uint32_t> cnt(B);
    par_for(B, [&](uint64_t a, uint64_t e) {
        for (uint64_t j = a; j < e; j++) {
            uint64_t st = seed * 0x2545F4914F6CDD1Dull ^ ((prefix_lo + j) * 0x9E3779B97F4A7C15ull) ^ 0xC0FFEEull;
            (void)splitmix64(st);
            cnt[j] = poisson(st, mean_per_bucket);
        }
    });
    uint64_t total = 0;
    for (uint64_t j = 0; j < B; j++) total += cnt[j];
    if (total >= 0x7FFFFFFFull) return KAD_ERR_INVALID;
    *out_n = (uint32_t)total;
    if (!out_ids) return KAD_OK;
    if (!out_status || !out_offset) return KAD_ERR_INVALID;
    uint32_t acc = 0;
    for (uint64_t j = 0; j < B; j++) { out_offset[j] = acc; acc += cnt[j]; }
    out_offset[B] = acc;
    const uint32_t sh = 64 - depth;
    par_for(B, [&](uint64_t a, uint64_t e) {
        std::vector<Id> tmp;
        for (uint64_t j = a; j < e; j++) {
            const uint64_t p = prefix_lo + j;
            uint64_t st = seed * 0x94D049BB133111EBull ^ (p * 0xBF58476D1CE4E5B9ull) ^ 0x1D5ull;
            (void)splitmix64(st);
            tmp.resize(cnt[j]);
            for (uint32_t k = 0; k < cnt[j]; k++) {
                while (true) {
                    uint64_t hi = splitmix64(st), mid = splitmix64(st), lo = splitmix64(st);
                    hi = (p << sh) | (hi & ((1ull << sh) - 1));
                    write_draws(tmp[k].data(), hi, mid, lo);
                    bool dup = false;
                    for (uint32_t m = 0; m < k && !dup; m++) dup = tmp[m] == tmp[k];
                    if (!dup) break;
                }
            }
            std::sort(tmp.begin(), tmp.end());
            const uint32_t o = out_offset[j];
            for (uint32_t k = 0; k < cnt[j]; k++) {
                std::memcpy(out_ids + 20ull * (o + k), tmp[k].data(), 20);
                const uint32_t u = (uint32_t)(splitmix64(st) % 100);
                out_status[o + k] = u < good_pct ? KAD_STATUS_GOOD : (u < good_pct + expired_pct ? KAD_STATUS_EXPIRED : 0);
            }
        }
    });
    return KAD_OK;
}

// SURVEY.md §8d recipe (kad_synth_ids + kad_synth_status over n nodes: ID i from draws 3i..3i+2 of mt19937_64(seed_ids),
// status of node i from draw i of mt19937_64(seed_status)) restricted to the U(depth) buckets [prefix_lo, prefix_hi):
// one sequential pass over the n draws, sorted by ID, with the bucket offsets and the number of IDs below the range
// (the global index of the range's first node). kad_synth_ids rejects and redraws a duplicate ID; among 1e8 random
// 160-bit IDs one has probability < 1e-30, so this pass fails (KAD_ERR_INVALID) on a duplicate instead. With
// out_ids == NULL: counts only (*out_n, *out_below); more than cap nodes in the range: KAD_ERR_NOMEM with the
// count in *out_n.
int kad_synth_recipe_range(uint64_t seed_ids, uint64_t seed_status, uint64_t n, uint32_t depth, uint64_t prefix_lo,
                           uint64_t prefix_hi, uint32_t good_pct, uint32_t expired_pct, uint64_t cap, uint32_t* out_n,
                           uint64_t* out_below, uint8_t* out_ids, uint8_t* out_status, uint32_t* out_offset) {
    if (depth == 0 || depth > 63 || !out_n || !out_below) return KAD_ERR_INVALID;
    if (prefix_hi == 0) prefix_hi = 1ull << depth;
    if (prefix_hi <= prefix_lo || prefix_hi > (1ull << depth) || prefix_hi - prefix_lo >= 0x7FFFFFFFull)
        return KAD_ERR_INVALID;
    const uint64_t B = prefix_hi - prefix_lo;
    const uint32_t sh = 64 - depth;
    struct Rec {
        uint64_t hi, mid;
        uint32_t lo;
        uint8_t st;
    };
    std::vector<Rec> keep;
    if (out_ids) keep.reserve(cap);
    std::mt19937_64 g(seed_ids), h(seed_status);
    uint64_t below = 0, kept = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t d0 = g(), d1 = g(), d2 = g();
        const uint32_t u = (uint32_t)(h() % 100);
        const uint64_t p = d0 >> sh;
        if (p < prefix_lo) { below++; continue; }
        if (p >= prefix_hi) continue;
        kept++;
        if (out_ids && kept <= cap)
            keep.push_back(Rec{d0, d1, (uint32_t)(d2 >> 32),
                               (uint8_t)(u < good_pct ? KAD_STATUS_GOOD : (u < good_pct + expired_pct ? KAD_STATUS_EXPIRED : 0))});
    }
    if (kept >= 0x7FFFFFFFull) return KAD_ERR_INVALID;
    *out_n = (uint32_t)kept;
    *out_below = below;
    if (!out_ids) return KAD_OK;
    if (!out_status || !out_offset) return KAD_ERR_INVALID;
    if (kept > cap) return KAD_ERR_NOMEM;  // *out_n holds the count: call again with cap >= it
    // counting sort by bucket, then by ID inside each bucket
    std::vector<uint32_t> pos(B + 1, 0);
    for (const Rec& r : keep) pos[(r.hi >> sh) - prefix_lo + 1]++;
    for (uint64_t j = 0; j < B; j++) pos[j + 1] += pos[j];
    for (uint64_t j = 0; j <= B; j++) out_offset[j] = pos[j];
    std::vector<uint32_t> order(keep.size());
    for (uint32_t k = 0; k < (uint32_t)keep.size(); k++) order[pos[(keep[k].hi >> sh) - prefix_lo]++] = k;
    std::atomic<bool> dup{false};
    par_for(B, [&](uint64_t a, uint64_t e) {
        for (uint64_t j = a; j < e; j++) {
            auto lt = [&](uint32_t x, uint32_t y) {
                const Rec &p = keep[x], &q = keep[y];
                return p.hi != q.hi ? p.hi < q.hi : p.mid != q.mid ? p.mid < q.mid : p.lo < q.lo;
            };
            std::sort(order.begin() + out_offset[j], order.begin() + out_offset[j + 1], lt);
            for (uint32_t k = out_offset[j]; k < out_offset[j + 1]; k++) {
                const Rec& r = keep[order[k]];
                write_draws(out_ids + 20ull * k, r.hi, r.mid, (uint64_t)r.lo << 32);
                out_status[k] = r.st;
                if (k > out_offset[j] && !lt(order[k - 1], order[k])) dup = true;
            }
        }
    });
    return dup ? KAD_ERR_INVALID : KAD_OK;
}

}  // extern "C"
