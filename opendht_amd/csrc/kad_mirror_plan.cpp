// Host plan of the incremental device mirror; see kad_mirror_plan.h.
#include "kad_mirror_plan.h"

#include <algorithm>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <unordered_map>

#include "../../include/kadgpu.h"

namespace kadplan {
namespace {

int fail(std::string& err, const char* fmt, ...) {
    char buf[256];
    va_list ap;
    va_start(ap, fmt);
    std::vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    err = buf;
    return KAD_ERR_INVALID;
}

int lowbit20(const uint8_t* p) {  // InfoHash::lowbit (infohash.h:84-95), -1 for zero
    for (int i = 19; i >= 0; i--)
        if (p[i])
            for (int j = 7; j >= 0; j--)
                if (p[i] & (0x80 >> j)) return 8 * i + j;
    return -1;
}

uint64_t top64(const uint8_t* p) {
    uint64_t x = 0;
    for (int k = 0; k < 8; k++) x = (x << 8) | p[k];
    return x;
}

// A current bucket of a touched origin: an untouched range of old nodes (raw) or an explicit handle list.
struct PB {
    bool raw;
    uint32_t src, len;
    std::vector<uint32_t> h;
    std::array<uint8_t, 20> first;
};

}  // namespace

// Sparse plan: an origin bucket (a bucket of the table at the batch start) that an op touches gets the
// list of its current buckets (splits add some); every other origin stays one untouched range. Host work
// is proportional to the batch, except the new offsets (one O(buckets) pass).
int mirror_plan(const std::vector<uint32_t>& off0, const uint8_t* first0, uint32_t n0, const uint32_t* ops,
                uint32_t n_ops, const uint8_t* new_ids, uint32_t n_new, int range_shift, uint64_t range_pre0,
                const OldIds& old_ids, MirrorPlan& out, std::string& err) {
    if (off0.size() < 2) return fail(err, "the mirror needs a RoutingTable (buckets)");
    const uint32_t B0 = (uint32_t)off0.size() - 1;
    std::unordered_map<uint32_t, std::vector<PB>> tb;  // touched origin -> its current buckets
    std::map<uint32_t, uint32_t> extra;                // split origin -> buckets its splits added
    uint32_t Bcur = B0;
    auto touch = [&](uint32_t o) -> std::vector<PB>& {
        auto it = tb.find(o);
        if (it == tb.end()) {
            PB p{true, off0[o], off0[o + 1] - off0[o], {}, {}};
            std::memcpy(p.first.data(), first0 + 20ull * o, 20);
            it = tb.emplace(o, std::vector<PB>(1, std::move(p))).first;
        }
        return it->second;
    };
    auto mat = [](PB& p) {
        if (p.raw) {
            p.h.resize(p.len);
            for (uint32_t i = 0; i < p.len; i++) p.h[i] = p.src + i;
            p.raw = false;
        }
    };
    // current bucket index c -> (origin, index among the origin's current buckets)
    auto origin_of = [&](uint32_t c, uint32_t& o, uint32_t& sub) {
        uint32_t shift = 0;  // buckets added by the splits of the origins below
        for (const auto& e : extra) {
            if (c < e.first + shift) break;
            if (c <= e.first + shift + e.second) {
                o = e.first;
                sub = c - e.first - shift;
                return;
            }
            shift += e.second;
        }
        o = c - shift;
        sub = 0;
    };
    // IDs of old nodes, fetched per origin bucket on first use (splits only)
    std::unordered_map<uint32_t, uint32_t> oid_at;
    std::vector<uint8_t> oid;
    auto id_of = [&](uint32_t h, uint32_t origin, uint8_t* id) -> int {
        if (h & MIRROR_NEW) {
            std::memcpy(id, new_ids + 20ull * (h & ~MIRROR_NEW), 20);
            return KAD_OK;
        }
        auto it = oid_at.find(origin);
        if (it == oid_at.end()) {
            const uint32_t a = off0[origin], e = off0[origin + 1];
            const size_t at = oid.size();
            oid.resize(at + 20ull * (e - a));
            if (e > a) {
                const int rc = old_ids(a, e, oid.data() + at);
                if (rc) return rc;
            }
            it = oid_at.emplace(origin, (uint32_t)(at / 20)).first;
        }
        std::memcpy(id, oid.data() + 20ull * (it->second + (h - off0[origin])), 20);
        return KAD_OK;
    };
    // node a (index at the batch start) -> its origin, current bucket and position
    auto locate = [&](uint32_t a, uint32_t& o, uint32_t& sub, uint32_t& pos) -> bool {
        if (a >= n0) return false;
        o = (uint32_t)(std::upper_bound(off0.begin(), off0.end(), a) - off0.begin()) - 1;
        auto it = tb.find(o);
        if (it == tb.end()) {
            sub = 0;
            pos = a - off0[o];
            return true;
        }
        for (sub = 0; sub < it->second.size(); sub++) {
            const PB& p = it->second[sub];
            if (p.raw) {
                if (a >= p.src && a < p.src + p.len) {
                    pos = a - p.src;
                    return true;
                }
            } else {
                auto f = std::find(p.h.begin(), p.h.end(), a);
                if (f != p.h.end()) {
                    pos = (uint32_t)(f - p.h.begin());
                    return true;
                }
            }
        }
        return false;
    };
    for (uint32_t k = 0; k < n_ops; k++) {
        const uint32_t kind = ops[3ull * k], a = ops[3ull * k + 1], b = ops[3ull * k + 2];
        uint32_t o = 0, sub = 0, pos = 0;
        if (kind == KAD_OP_REMOVE || kind == KAD_OP_REPLACE) {
            if (!locate(a, o, sub, pos)) return fail(err, "op %u: node %u is not in the table", k, a);
            if (kind == KAD_OP_REPLACE) {
                if (b >= n_new) return fail(err, "op %u: new slot %u", k, b);
                // onNewNode replaces inside findBucket(id) (dht.cpp:908-921): the new node must belong there
                const auto it = tb.find(o);
                const uint8_t* lo = it == tb.end() ? first0 + 20ull * o : it->second[sub].first.data();
                const uint8_t* hi = it != tb.end() && sub + 1 < it->second.size() ? it->second[sub + 1].first.data()
                                    : o + 1 < B0                                  ? first0 + 20ull * (o + 1)
                                                                                  : nullptr;
                const uint8_t* id = new_ids + 20ull * b;
                if (std::memcmp(lo, id, 20) > 0 || (hi && std::memcmp(id, hi, 20) >= 0))
                    return fail(err, "op %u: new node %u does not belong to node %u's bucket", k, b, a);
            }
            PB& p = touch(o)[sub];
            mat(p);
            if (kind == KAD_OP_REMOVE) p.h.erase(p.h.begin() + pos);
            else p.h[pos] = MIRROR_NEW | b;
        } else if (kind == KAD_OP_INSERT) {
            if (a >= n_new) return fail(err, "op %u: new slot %u", k, a);
            // RoutingTable::findBucket (routing_table.cpp:113-127): last bucket with first <= id
            const uint8_t* id = new_ids + 20ull * a;
            uint32_t lo = 0, hi = B0;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (std::memcmp(first0 + 20ull * mid, id, 20) <= 0) lo = mid + 1;
                else hi = mid;
            }
            o = lo ? lo - 1 : 0;
            std::vector<PB>& v = touch(o);
            sub = 0;
            while (sub + 1 < v.size() && std::memcmp(v[sub + 1].first.data(), id, 20) <= 0) sub++;
            mat(v[sub]);
            v[sub].h.insert(v[sub].h.begin(), MIRROR_NEW | a);  // emplace_front (dht.cpp:934)
        } else if (kind == KAD_OP_SPLIT) {
            if (a >= Bcur) return fail(err, "op %u: bucket %u of %u", k, a, Bcur);
            origin_of(a, o, sub);
            std::vector<PB>& v = touch(o);
            // RoutingTable::depth / middle / split (routing_table.cpp:47-65, 137-163)
            const uint8_t* nf = sub + 1 < v.size() ? v[sub + 1].first.data() : o + 1 < B0 ? first0 + 20ull * (o + 1) : nullptr;
            const int b1 = lowbit20(v[sub].first.data()), b2 = nf ? lowbit20(nf) : -1;
            const int depth = std::max(b1, b2) + 1;
            if (depth >= 160) continue;  // middle() throws: split returns false
            std::array<uint8_t, 20> mid = v[sub].first;
            mid[depth / 8] |= (uint8_t)(0x80 >> (depth % 8));
            mat(v[sub]);
            std::vector<uint32_t> keep, move;
            for (uint32_t h : v[sub].h) {  // splice each node to the FRONT of its new bucket
                uint8_t id[20];
                const int rc = id_of(h, o, id);
                if (rc) return rc;
                auto& dst = std::memcmp(id, mid.data(), 20) >= 0 ? move : keep;
                dst.insert(dst.begin(), h);
            }
            v[sub].h = std::move(keep);
            v.insert(v.begin() + sub + 1, PB{false, 0, 0, std::move(move), mid});
            extra[o]++;
            Bcur++;
        } else {
            return fail(err, "op %u: unknown kind %u", k, kind);
        }
    }
    std::vector<uint32_t> tk;  // touched origins, ascending
    tk.reserve(tb.size());
    for (const auto& e : tb) tk.push_back(e.first);
    std::sort(tk.begin(), tk.end());
    const uint32_t B1 = Bcur;
    out = MirrorPlan{};
    out.B1 = B1;
    if (range_shift >= 0 && B1 == B0)
        for (uint32_t o : tk)
            for (const PB& p : tb[o])
                if (!p.raw)
                    for (uint32_t h : p.h)
                        if (h & MIRROR_NEW) {
                            const uint64_t hi = top64(new_ids + 20ull * (h & ~MIRROR_NEW));
                            out.new_in_range &= (range_shift < 64 ? hi >> range_shift : 0) == range_pre0 + o;
                        }
    // new layout: untouched origins between touched ones are one range of old nodes
    std::vector<MirrorSeg>& segs = out.segs;
    std::vector<uint32_t>& off1 = out.off1;
    off1.resize(B1 + 1);
    uint32_t acc = 0, c = 0, prev = 0;
    auto raw_seg = [&](uint32_t src, uint32_t len) {
        if (!len) return;
        MirrorSeg* last = segs.empty() ? nullptr : &segs.back();
        if (last && last->kind == 0 && last->src + last->len == src && last->start + last->len == acc) last->len += len;
        else segs.push_back(MirrorSeg{acc, src, len, 0});
    };
    auto untouched = [&](uint32_t e) {  // origins [prev, e)
        const uint32_t base = off0[prev];
        for (uint32_t u = prev; u < e; u++) off1[c++] = acc + (off0[u] - base);
        raw_seg(base, off0[e] - base);
        acc += off0[e] - base;
    };
    for (uint32_t o : tk) {
        untouched(o);
        for (const PB& p : tb[o]) {
            off1[c++] = acc;
            const uint32_t len = p.raw ? p.len : (uint32_t)p.h.size();
            if (p.raw) {
                raw_seg(p.src, len);
            } else if (len) {
                segs.push_back(MirrorSeg{acc, (uint32_t)out.list.size(), len, 1});
                out.list.insert(out.list.end(), p.h.begin(), p.h.end());
            }
            acc += len;
        }
        prev = o + 1;
    }
    untouched(B0);
    off1[B1] = acc;
    out.n1 = acc;
    if (B1 != B0) {  // the new bucket firsts (only splits change them)
        out.first1.resize(20ull * B1);
        uint32_t j = 0, pv = 0;
        for (uint32_t o : tk) {
            if (o > pv) std::memcpy(out.first1.data() + 20ull * j, first0 + 20ull * pv, 20ull * (o - pv));
            j += o - pv;
            for (const PB& p : tb[o]) std::memcpy(out.first1.data() + 20ull * j++, p.first.data(), 20);
            pv = o + 1;
        }
        if (B0 > pv) std::memcpy(out.first1.data() + 20ull * j, first0 + 20ull * pv, 20ull * (B0 - pv));
    }
    return KAD_OK;
}

}  // namespace kadplan
