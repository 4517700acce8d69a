// C++ test of include/kadgpu.hpp against test doubles shaped like OpenDHT's types
// (InfoHash = std::array<uint8_t,20>, Node with time / reply_time / isGood(now) / isExpired(),
// Bucket{first, list<shared_ptr<Node>>}, RoutingTable = std::list<Bucket>, NodeCache family map =
// std::map<InfoHash, weak_ptr<Node>>). Expected results come from the CPU oracle (test infrastructure)
// on the host objects' state at each query's `now`. Needs a GPU. Exit 0 = pass.
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <list>
#include <map>
#include <memory>
#include <random>
#include <vector>

#include "kadgpu.hpp"

extern "C" int orc_flat_rt_closest(uint32_t, const uint8_t*, const uint8_t*, uint32_t, const uint8_t*, const uint32_t*,
                                   uint32_t, const uint8_t*, uint32_t, uint32_t*, uint8_t*, int);
extern "C" int orc_flat_nc_closest(uint32_t, const uint8_t*, const uint8_t*, uint32_t, const uint8_t*, uint32_t,
                                   uint32_t*, uint8_t*, int);

namespace mock {
using clock = std::chrono::steady_clock;
using time_point = clock::time_point;
struct InfoHash : std::array<uint8_t, 20> {
    bool operator<(const InfoHash& o) const { return std::memcmp(data(), o.data(), 20) < 0; }
};
// node.h:35-105 / node.cpp:34-40, 82-108 in miniature
struct Node {
    InfoHash id;
    time_point time{time_point::min()}, reply_time{time_point::min()};
    bool expired_ = false;
    uint32_t idx = 0;
    bool isExpired() const { return expired_; }
    bool isGood(time_point now) const {
        return !expired_ && reply_time >= now - std::chrono::minutes(120) && time >= now - std::chrono::minutes(10);
    }
    void received(time_point now, bool reply) {
        time = now;
        if (reply) { reply_time = now; expired_ = false; }
    }
    void setExpired() { expired_ = true; }
};
struct Bucket {
    InfoHash first;
    std::list<std::shared_ptr<Node>> nodes;
};
using RoutingTable = std::list<Bucket>;
using NodeMap = std::map<InfoHash, std::weak_ptr<Node>>;
}  // namespace mock

static int fails = 0;
#define EXPECT(c, ...) do { if (!(c)) { fails++; if (fails < 30) { std::fprintf(stderr, __VA_ARGS__); std::fprintf(stderr, "\n"); } } } while (0)

using namespace mock;

// The oracle's answer on the host table as it is now, compared with the mirror's result vectors.
static void check_rt(const RoutingTable& rt, const std::vector<std::vector<std::shared_ptr<Node>>>& got,
                     const std::vector<InfoHash>& targets, uint32_t count, time_point now, const char* what) {
    std::vector<uint8_t> ids, st, first;
    std::vector<uint32_t> off;
    std::vector<const Node*> flat;
    for (auto& b : rt) {
        off.push_back((uint32_t)flat.size());
        first.insert(first.end(), b.first.begin(), b.first.end());
        for (auto& nd : b.nodes) {
            ids.insert(ids.end(), nd->id.begin(), nd->id.end());
            st.push_back((uint8_t)((nd->isGood(now) ? 1 : 0) | (nd->isExpired() ? 2 : 0)));
            flat.push_back(nd.get());
        }
    }
    off.push_back((uint32_t)flat.size());
    const uint32_t q = (uint32_t)targets.size();
    std::vector<uint32_t> want(q * count);
    std::vector<uint8_t> wcnt(q);
    orc_flat_rt_closest((uint32_t)flat.size(), ids.data(), st.data(), (uint32_t)rt.size(), first.data(), off.data(), q,
                        reinterpret_cast<const uint8_t*>(targets.data()), count, want.data(), wcnt.data(), 4);
    for (uint32_t i = 0; i < q; i++) {
        uint32_t m = wcnt[i];  // the oracle's count byte wraps above 255: the row's padding gives the length
        if (count > 255)
            for (m = 0; m < count && want[(size_t)i * count + m] != 0xFFFFFFFFu; m++) {}
        EXPECT(got[i].size() == m, "%s: rt count q=%u k=%u (%zu vs %u)", what, i, count, got[i].size(), m);
        for (uint32_t j = 0; j < got[i].size() && j < m; j++)
            EXPECT(got[i][j].get() == flat[want[(size_t)i * count + j]], "%s: rt node q=%u k=%u j=%u", what, i, count, j);
    }
}

static void check_nc(const NodeMap& nm, const std::vector<std::vector<std::shared_ptr<Node>>>& got,
                     const std::vector<InfoHash>& targets, size_t count_in, const char* what) {
    std::vector<uint8_t> ids, st;
    std::vector<const Node*> flat;
    for (auto& kv : nm) {
        auto n = kv.second.lock();
        ids.insert(ids.end(), kv.first.begin(), kv.first.end());
        st.push_back((!n || n->isExpired()) ? 2 : 0);
        flat.push_back(n.get());
    }
    const uint32_t q = (uint32_t)targets.size();
    const uint32_t count = (uint32_t)std::min<size_t>(count_in, flat.size());  // a result holds at most the map
    EXPECT(got.size() == q, "%s: nc rows", what);
    if (count == 0) {
        for (uint32_t i = 0; i < q; i++) EXPECT(got[i].empty(), "%s: nc empty q=%u", what, i);
        return;
    }
    std::vector<uint32_t> want((size_t)q * count);
    std::vector<uint8_t> wcnt(q);
    orc_flat_nc_closest((uint32_t)flat.size(), ids.data(), st.data(), q, reinterpret_cast<const uint8_t*>(targets.data()),
                        count, want.data(), wcnt.data(), 4);
    for (uint32_t i = 0; i < q; i++) {
        uint32_t m = 0;  // the row's entries before the padding (the count byte wraps above 255)
        while (m < count && want[(size_t)i * count + m] != 0xFFFFFFFFu) m++;
        EXPECT(got[i].size() == m, "%s: nc count q=%u k=%zu", what, i, count_in);
        for (uint32_t j = 0; j < got[i].size() && j < m; j++)
            EXPECT(got[i][j].get() == flat[want[(size_t)i * count + j]], "%s: nc node q=%u j=%u", what, i, j);
    }
}

int main() {
    const uint32_t n = 20000, q = 3000;
    std::vector<uint8_t> ids(20ull * n);
    kadgpu::check(kad_synth_ids(0xC0FFEE, n, ids.data()), "synth");
    std::vector<uint32_t> perm(n), off(n + 2);
    std::vector<uint8_t> first(20ull * (n + 1));
    uint32_t B = 0;
    kadgpu::check(kad_split_table(n, ids.data(), 8, perm.data(), first.data(), off.data(), &B), "split");
    const time_point t0 = clock::now();
    std::mt19937_64 g(7);
    std::vector<std::shared_ptr<Node>> nodes(n);
    const auto MIN = std::chrono::minutes(1);
    for (uint32_t i = 0; i < n; i++) {
        auto nd = std::make_shared<Node>();
        std::memcpy(nd->id.data(), &ids[20ull * i], 20);
        nd->idx = i;
        const unsigned u = g() % 100;
        // heard 0..9.9 min and replied 0..119 min before t0; edges: exactly 10 and 120 min
        nd->time = t0 - std::chrono::milliseconds(g() % 594000);
        nd->reply_time = t0 - std::chrono::seconds(g() % 7140);
        if (u < 3) nd->time = t0 - 10 * MIN;                // good at t0, dubious 1 ns later
        else if (u < 6) nd->reply_time = t0 - 120 * MIN;    // likewise through reply_time
        else if (u < 8) nd->reply_time = time_point::min(); // never replied
        else if (u >= 85 && u < 95) nd->expired_ = true;
        nodes[i] = nd;
    }
    RoutingTable rt;
    for (uint32_t b = 0; b < B; b++) {
        Bucket bk;
        std::memcpy(bk.first.data(), &first[20ull * b], 20);
        for (uint32_t j = off[b]; j < off[b + 1]; j++) bk.nodes.push_back(nodes[perm[j]]);
        rt.push_back(bk);
    }
    std::vector<InfoHash> targets(q);
    for (auto& t : targets)
        for (auto& x : t) x = (uint8_t)g();
    targets[0] = nodes[5]->id;
    targets[1].fill(0);
    targets[2].fill(0xFF);

    // RoutingTable::findClosestNodes(id, now, count) at a moving `now` (routing_table.h:48)
    kadgpu::RoutingTableMirror<RoutingTable> mirror(rt, t0, 0);
    EXPECT(mirror.bucketCount() == B, "bucket count");
    const std::chrono::nanoseconds steps[] = {std::chrono::nanoseconds(0), std::chrono::nanoseconds(1),
                                              std::chrono::seconds(30), std::chrono::minutes(3), std::chrono::minutes(9),
                                              std::chrono::minutes(11), std::chrono::minutes(125)};
    for (auto dt : steps) {
        const time_point now = t0 + dt;
        for (uint32_t count : {1u, 8u, 14u, 32u, 33u, 100u, 300u}) {
            auto got = mirror.findClosestNodesBatch(targets, now, count);
            check_rt(rt, got, targets, count, now, "moving now");
        }
        auto one = mirror.findClosestNodes(targets[3], now, 8);  // one request: the host path
        mirror.setHostPath(0);  // every batch to the device
        auto ref = mirror.findClosestNodesBatch(&targets[3], 2, now, 8);
        mirror.setHostPath(kadgpu::RoutingTableMirror<RoutingTable>::kHostPathAuto);
        EXPECT(one == ref[0], "single query (host path) equals the device batch");
        // the host path (single requests below the crossover) for every target and count, against the oracle
        for (uint32_t count : {1u, 8u, 14u, 33u, 300u}) {
            std::vector<std::vector<std::shared_ptr<Node>>> hg;
            for (auto& t : targets) hg.push_back(mirror.findClosestNodesHost(t, now, count));
            check_rt(rt, hg, targets, count, now, "host path");
        }
    }
    // a count above the table's size (any size_t, routing_table.h:48): every good node, closest first
    {
        const time_point now = t0 + std::chrono::seconds(30);
        auto all = mirror.findClosestNodes(targets[7], now, (size_t)1 << 40);
        size_t good = 0;
        for (auto& nd : nodes) good += nd->isGood(now);
        EXPECT(all.size() == good, "count > n: %zu of %zu good nodes", all.size(), good);
        std::vector<std::vector<std::shared_ptr<Node>>> g1{all};
        std::vector<InfoHash> t1{targets[7]};
        check_rt(rt, g1, t1, n, now, "count > n");
    }
    // going back in time is allowed too (the status is a function of now)
    {
        auto got = mirror.findClosestNodesBatch(targets, t0, 8);
        check_rt(rt, got, targets, 8, t0, "now moved back");
    }
    // liveness changes on the host, reported with nodeUpdated: Node::received / setExpired
    {
        const time_point now = t0 + 11 * MIN;
        for (uint32_t i = 0; i < n; i += 7) {
            nodes[i]->received(now, i % 2 == 0);
            mirror.nodeUpdated(nodes[i]);
        }
        for (uint32_t i = 3; i < n; i += 29) {
            nodes[i]->setExpired();
            mirror.nodeUpdated(nodes[i]);
        }
        for (uint32_t count : {1u, 8u, 14u, 32u}) {
            auto got = mirror.findClosestNodesBatch(targets, now, count);
            check_rt(rt, got, targets, count, now, "nodeUpdated");
        }
        // the same changes through syncTimes()
        for (uint32_t i = 1; i < n; i += 13) nodes[i]->received(now, true);
        mirror.syncTimes();
        auto got = mirror.findClosestNodesBatch(targets, now, 8);
        check_rt(rt, got, targets, 8, now, "syncTimes");
    }

    // NodeCache::getCachedNodes(id, sa_family_t, count) over both families (node_cache.h:32)
    {
        NodeMap c4, c6;
        std::vector<std::shared_ptr<Node>> extra;  // cache-only nodes, some of which die
        for (auto& nd : nodes) (nd->idx % 3 == 0 ? c6 : c4).emplace(nd->id, nd);
        for (int k = 0; k < 3000; k++) {
            auto nd = std::make_shared<Node>();
            for (auto& x : nd->id) x = (uint8_t)g();
            nd->idx = 100000 + k;
            nd->time = nd->reply_time = t0;
            extra.push_back(nd);
            c4.emplace(nd->id, nd);
        }
        kadgpu::NodeCacheMirror<NodeMap> nc;
        nc.snapshot(c4, c6, 0);
        for (uint32_t count : {8u, 14u, 32u}) {
            std::vector<std::vector<std::shared_ptr<Node>>> g4, g6;
            for (auto& t : targets) {
                g4.push_back(nc.getCachedNodes(t, AF_INET, count));
                g6.push_back(nc.getCachedNodes(t, AF_INET6, count));
            }
            check_nc(c4, g4, targets, count, "nc v4");
            check_nc(c6, g6, targets, count, "nc v6");
        }
        // deaths and expiries need no notification (detected on the results, re-run)
        for (size_t k = 0; k < extra.size(); k += 3) extra[k].reset();
        for (uint32_t i = 0; i < n; i += 17) nodes[i]->setExpired();
        // an expired node that answers again must be reported
        for (uint32_t i = 0; i < n; i += 31)
            if (nodes[i]->isExpired()) { nodes[i]->received(t0, true); nc.nodeUpdated(nodes[i]); }
        for (uint32_t count : {8u, 14u}) {
            auto b4 = nc.family(AF_INET).getCachedNodesBatch(targets, count);
            auto b6 = nc.family(AF_INET6).getCachedNodesBatch(targets, count);
            check_nc(c4, b4, targets, count, "nc v4 after deaths");
            check_nc(c6, b6, targets, count, "nc v6 after expiries");
        }
        // the maps change: NodeMap::getNode(id, addr, now, confirm) emplaces new IDs (node_cache.cpp:91-103),
        // getNode(id) erases entries whose node died (:79-89); the mirror follows with sync() (kad_nc_apply)
        for (int k = 0; k < 2000; k++) {
            auto nd = std::make_shared<Node>();
            for (auto& x : nd->id) x = (uint8_t)g();
            nd->idx = 200000 + k;
            nd->time = nd->reply_time = t0;
            if (k % 4 == 0) nd->expired_ = true;
            extra.push_back(nd);
            (k % 2 ? c6 : c4).emplace(nd->id, nd);
        }
        for (auto it = c4.begin(); it != c4.end();)  // erase dead entries, as getNode(id) does on lookup
            if (it->second.expired() && (g() % 2)) it = c4.erase(it); else ++it;
        nc.sync(c4, c6);
        for (uint32_t count : {8u, 14u, 32u}) {
            auto b4 = nc.family(AF_INET).getCachedNodesBatch(targets, count);
            auto b6 = nc.family(AF_INET6).getCachedNodesBatch(targets, count);
            check_nc(c4, b4, targets, count, "nc v4 after sync");
            check_nc(c6, b6, targets, count, "nc v6 after sync");
        }
        EXPECT(nc.family(AF_INET).size() == c4.size() && nc.family(AF_INET6).size() == c6.size(), "nc sizes after sync");
        // any size_t count (node_cache.h:32): above the kernels' 64, above the count byte's 255, above the map's size
        for (size_t count : {size_t(300), c6.size() + 5, size_t(1) << 40}) {
            std::vector<InfoHash> few(targets.begin(), targets.begin() + 40);
            auto b4 = nc.family(AF_INET).getCachedNodesBatch(few, count);
            auto b6 = nc.family(AF_INET6).getCachedNodesBatch(few, count);
            check_nc(c4, b4, few, count, "nc v4 large count");
            check_nc(c6, b6, few, count, "nc v6 large count");
        }
    }

    // Incremental mirror: Dht::onNewNode (replace an expired node / emplace_front / split my bucket)
    // and Dht::expireBuckets on the host table, recorded on the mirror and flushed to the device.
    {
        const time_point now = t0 + 12 * MIN;
        auto find_bucket = [&](const InfoHash& id) {  // routing_table.cpp:113-127
            auto b = rt.begin();
            while (std::next(b) != rt.end() && !(id < std::next(b)->first)) ++b;
            return b;
        };
        auto lowbit = [](const InfoHash& h) {
            for (int i = 19; i >= 0; i--)
                if (h[i])
                    for (int j = 7; j >= 0; j--)
                        if (h[i] & (0x80 >> j)) return 8 * i + j;
            return -1;
        };
        auto split = [&](RoutingTable::iterator b) {  // routing_table.cpp:137-163
            const int depth = std::max(lowbit(b->first), std::next(b) != rt.end() ? lowbit(std::next(b)->first) : -1) + 1;
            if (depth >= 160) return false;
            InfoHash mid = b->first;
            mid[depth / 8] |= (uint8_t)(0x80 >> (depth % 8));
            rt.insert(std::next(b), Bucket{mid, {}});
            std::list<std::shared_ptr<Node>> tmp;
            tmp.splice(tmp.begin(), b->nodes);
            while (!tmp.empty()) {
                auto it = tmp.begin();
                auto dst = find_bucket((*it)->id);
                dst->nodes.splice(dst->nodes.begin(), tmp, it);
            }
            return true;
        };
        const InfoHash myid = nodes[123]->id;
        uint32_t replaced = 0, added = 0, splits = 0, removed = 0, next_idx = n;
        for (int k = 0; k < 3000; k++) {
            auto nd = std::make_shared<Node>();
            for (auto& x : nd->id) x = (uint8_t)g();
            if (k % 5 == 0) {  // some land next to myid, to make my bucket split
                nd->id = myid;
                for (int x = 6; x < 20; x++) nd->id[x] = (uint8_t)g();
            }
            nd->time = nd->reply_time = now;
            nd->idx = next_idx++;
            while (true) {  // Dht::onNewNode (dht.cpp:867-936), confirm = 0, all new nodes good
                auto b = find_bucket(nd->id);
                auto exp = std::find_if(b->nodes.begin(), b->nodes.end(), [](const std::shared_ptr<Node>& x) { return x->isExpired(); });
                if (exp != b->nodes.end()) {
                    mirror.nodeReplaced(*exp, nd);
                    *exp = nd;
                    replaced++;
                    break;
                }
                if (b->nodes.size() >= 8) {
                    // my bucket splits when full (the reference also requires no dubious node,
                    // dht.cpp:923; the mirror replays whatever the host does either way)
                    const bool mine = !(myid < b->first) && (std::next(b) == rt.end() || myid < std::next(b)->first);
                    if (mine) {
                        const size_t bi = (size_t)std::distance(rt.begin(), b);
                        if (split(b)) {
                            mirror.bucketSplit(bi);
                            splits++;
                            continue;
                        }
                    }
                    break;  // cached away
                }
                b->nodes.emplace_front(nd);
                mirror.nodeAdded(nd);
                added++;
                break;
            }
            if (k == 1500) mirror.flush(now);  // two batches
        }
        for (auto& b : rt)  // Dht::expireBuckets (dht.cpp:942-956)
            b.nodes.remove_if([&](const std::shared_ptr<Node>& x) {
                if (x->isExpired()) { mirror.nodeRemoved(x); removed++; return true; }
                return false;
            });
        mirror.flush(now);
        EXPECT(mirror.bucketCount() == rt.size(), "mirror buckets %zu vs %zu", mirror.bucketCount(), rt.size());
        size_t total = 0;
        for (auto& b : rt) total += b.nodes.size();
        EXPECT(mirror.nodeCount() == total, "mirror nodes %zu vs %zu", mirror.nodeCount(), total);
        for (uint32_t count : {1u, 8u, 14u}) {
            auto got = mirror.findClosestNodesBatch(targets, now, count);
            check_rt(rt, got, targets, count, now, "mirror");
        }
        // and the mirrored table keeps tracking `now` after the flush
        const time_point later = now + 10 * MIN;
        auto got = mirror.findClosestNodesBatch(targets, later, 8);
        check_rt(rt, got, targets, 8, later, "mirror later");
        std::printf("mirror: %u replaced, %u added, %u splits, %u removed\n", replaced, added, splits, removed);
        EXPECT(replaced && added && splits && removed, "every mutation kind exercised");
    }

    // Dht::findClosestNodes(id, af, count) with exactly three arguments; `now` from the mirror's clock
    {
        kadgpu::DhtMirror<RoutingTable> dht;
        RoutingTable empty6;
        time_point sched = t0 + 12 * MIN;
        dht.snapshot(rt, empty6, sched, 0);
        dht.setClock([&] { return sched; });  // Dht's scheduler.time()
        for (time_point at : {t0 + 12 * MIN, t0 + 20 * MIN, t0 + 200 * MIN}) {
            sched = at;
            std::vector<std::vector<std::shared_ptr<Node>>> got;
            for (auto& t : targets) got.push_back(dht.findClosestNodes(t, AF_INET, 8));
            check_rt(rt, got, targets, 8, at, "dht v4");
            EXPECT(dht.findClosestNodes(targets[4], AF_INET6, 8).empty(), "dht v6 empty table");
        }
    }
    // latency of one call through the shim on a live-sized table (~170 nodes, the reference's per-request
    // case): median of single findClosestNodes calls and of 64-query batches
    {
        const uint32_t m = 170;
        std::vector<uint8_t> lid(20ull * m);
        kadgpu::check(kad_synth_ids(0x1A7, m, lid.data()), "synth");
        std::vector<uint32_t> lperm(m), loff(m + 2);
        std::vector<uint8_t> lfirst(20ull * (m + 1));
        uint32_t LB = 0;
        kadgpu::check(kad_split_table(m, lid.data(), 8, lperm.data(), lfirst.data(), loff.data(), &LB), "split");
        RoutingTable lrt;
        std::vector<std::shared_ptr<Node>> keep;
        for (uint32_t b = 0; b < LB; b++) {
            Bucket bk;
            std::memcpy(bk.first.data(), &lfirst[20ull * b], 20);
            for (uint32_t j = loff[b]; j < loff[b + 1]; j++) {
                auto nd = std::make_shared<Node>();
                std::memcpy(nd->id.data(), &lid[20ull * lperm[j]], 20);
                nd->time = nd->reply_time = t0;
                keep.push_back(nd);
                bk.nodes.push_back(nd);
            }
            lrt.push_back(bk);
        }
        kadgpu::RoutingTableMirror<RoutingTable> lm(lrt, t0, 0);
        auto med = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v[v.size() / 2]; };
        std::vector<double> host_us;
        for (int r = 0; r < 2000; r++) {  // single requests on the host path (the default below the crossover)
            const auto a = clock::now();
            auto res = lm.findClosestNodes(targets[r % q], t0, 8);
            host_us.push_back(std::chrono::duration<double, std::micro>(clock::now() - a).count());
            EXPECT(res.size() == 8, "latency table result (host)");
        }
        lm.setHostPath(0);  // the device paths from here
        std::vector<double> one_us, b64_us;
        for (int r = 0; r < 2000; r++) {
            const auto a = clock::now();
            auto res = lm.findClosestNodes(targets[r % q], t0, 8);
            one_us.push_back(std::chrono::duration<double, std::micro>(clock::now() - a).count());
            EXPECT(res.size() == 8, "latency table result");
        }
        for (int r = 0; r < 500; r++) {
            const auto a = clock::now();
            auto res = lm.findClosestNodesBatch(&targets[(r * 64) % (q - 64)], 64, t0, 8);
            b64_us.push_back(std::chrono::duration<double, std::micro>(clock::now() - a).count());
        }
        // the same calls answered by the resident query service (kad_table_serve): the same nodes, in order
        auto before = lm.findClosestNodesBatch(&targets[0], 64, t0, 14);
        lm.serve(100000);
        EXPECT(lm.findClosestNodesBatch(&targets[0], 64, t0, 14) == before, "served batch equals the launch path");
        for (int j = 0; j < 64; j++)
            EXPECT(lm.findClosestNodes(targets[j], t0, 14) == before[j], "served single call equals the launch path");
        std::vector<double> s1_us, s64_us;
        for (int r = 0; r < 2000; r++) {
            const auto a = clock::now();
            auto res = lm.findClosestNodes(targets[r % q], t0, 8);
            s1_us.push_back(std::chrono::duration<double, std::micro>(clock::now() - a).count());
            EXPECT(res.size() == 8, "latency table result (served)");
        }
        for (int r = 0; r < 500; r++) {
            const auto a = clock::now();
            auto res = lm.findClosestNodesBatch(&targets[(r * 64) % (q - 64)], 64, t0, 8);
            s64_us.push_back(std::chrono::duration<double, std::micro>(clock::now() - a).count());
        }
        lm.serve(0);
        std::printf("LATENCY {\"nodes\": %u, \"buckets\": %u, \"host_single_call_us\": %.2f, \"single_call_us\": %.2f, "
                    "\"batch64_call_us\": %.2f, \"served_single_call_us\": %.2f, \"served_batch64_call_us\": %.2f}\n",
                    m, LB, med(host_us), med(one_us), med(b64_us), med(s1_us), med(s64_us));
    }
    std::printf("%s (%d failures)\n", fails ? "FAIL" : "PASS", fails);
    return fails ? 1 : 0;
}
