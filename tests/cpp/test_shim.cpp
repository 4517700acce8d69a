// C++ test of include/kadgpu.hpp against test doubles shaped like OpenDHT's types
// (InfoHash = std::array<uint8_t,20>, Node with isGood/isExpired, Bucket{first, list<shared_ptr<Node>>},
// RoutingTable = std::list<Bucket>, NodeCache family map = std::map<InfoHash, weak_ptr<Node>>).
// Expected results come from the CPU oracle (test infrastructure). Needs a GPU. Exit 0 = pass.
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
struct Node {
    InfoHash id;
    time_point time{time_point::min()}, reply_time{time_point::min()};
    bool expired_ = false;
    uint32_t idx = 0;
    bool isExpired() const { return expired_; }
    bool isGood(time_point now) const {
        return !expired_ && reply_time >= now - std::chrono::minutes(120) && time >= now - std::chrono::minutes(10);
    }
};
struct Bucket {
    InfoHash first;
    std::list<std::shared_ptr<Node>> nodes;
};
using RoutingTable = std::list<Bucket>;
using NodeMap = std::map<InfoHash, std::weak_ptr<Node>>;
}  // namespace mock

static int fails = 0;
#define EXPECT(c, ...) do { if (!(c)) { fails++; std::fprintf(stderr, __VA_ARGS__); std::fprintf(stderr, "\n"); } } while (0)

int main() {
    using namespace mock;
    const uint32_t n = 20000, q = 3000;
    std::vector<uint8_t> ids(20ull * n);
    kadgpu::check(kad_synth_ids(0xC0FFEE, n, ids.data()), "synth");
    std::vector<uint32_t> perm(n), off(n + 2);
    std::vector<uint8_t> first(20ull * (n + 1));
    uint32_t B = 0;
    kadgpu::check(kad_split_table(n, ids.data(), 8, perm.data(), first.data(), off.data(), &B), "split");
    const time_point now = clock::now();
    std::mt19937_64 g(7);
    std::vector<std::shared_ptr<Node>> nodes(n);
    for (uint32_t i = 0; i < n; i++) {
        auto nd = std::make_shared<Node>();
        std::memcpy(nd->id.data(), &ids[20ull * i], 20);
        nd->idx = i;
        const unsigned u = g() % 100;
        nd->time = nd->reply_time = now;
        if (u >= 80 && u < 90) nd->expired_ = true;
        else if (u >= 90) nd->time = now - std::chrono::minutes(11);
        nodes[i] = nd;
    }
    RoutingTable rt;
    std::vector<uint8_t> fids, fst;  // flattened in list order for the oracle
    for (uint32_t b = 0; b < B; b++) {
        Bucket bk;
        std::memcpy(bk.first.data(), &first[20ull * b], 20);
        for (uint32_t j = off[b]; j < off[b + 1]; j++) bk.nodes.push_back(nodes[perm[j]]);
        rt.push_back(bk);
    }
    std::vector<uint32_t> flat_to_node;
    for (auto& b : rt)
        for (auto& nd : b.nodes) {
            fids.insert(fids.end(), nd->id.begin(), nd->id.end());
            fst.push_back((uint8_t)((nd->isGood(now) ? 1 : 0) | (nd->isExpired() ? 2 : 0)));
            flat_to_node.push_back(nd->idx);
        }
    std::vector<InfoHash> targets(q);
    for (auto& t : targets)
        for (auto& x : t) x = (uint8_t)g();
    targets[0] = nodes[5]->id;
    targets[1].fill(0);
    targets[2].fill(0xFF);

    kadgpu::RoutingTableMirror<RoutingTable> mirror(rt, now, 0);
    EXPECT(mirror.bucketCount() == B, "bucket count");
    for (uint32_t count : {1u, 8u, 14u, 32u}) {
        auto got = mirror.findClosestNodesBatch(targets, count);
        std::vector<uint32_t> want(q * count);
        std::vector<uint8_t> wcnt(q);
        orc_flat_rt_closest(n, fids.data(), fst.data(), B, first.data(), off.data(), q,
                            reinterpret_cast<const uint8_t*>(targets.data()), count, want.data(), wcnt.data(), 4);
        for (uint32_t i = 0; i < q; i++) {
            EXPECT(got[i].size() == wcnt[i], "rt count q=%u k=%u", i, count);
            for (uint32_t j = 0; j < got[i].size() && j < wcnt[i]; j++)
                EXPECT(got[i][j]->idx == flat_to_node[want[i * count + j]], "rt node q=%u k=%u j=%u", i, count, j);
        }
        auto one = mirror.findClosestNodes(targets[3], count);
        EXPECT(one.size() == got[3].size(), "single query");
    }
    // NodeCache family map
    NodeMap nm;
    for (auto& nd : nodes) nm.emplace(nd->id, nd);
    std::vector<uint8_t> sids, sst;
    std::vector<uint32_t> sorted_to_node;
    for (auto& kv : nm) {
        sids.insert(sids.end(), kv.first.begin(), kv.first.end());
        sst.push_back(kv.second.lock()->isExpired() ? 2 : 0);
        sorted_to_node.push_back(kv.second.lock()->idx);
    }
    kadgpu::NodeCacheMirror<NodeMap> nc(nm, 0);
    for (uint32_t count : {8u, 14u}) {
        auto got = nc.getCachedNodesBatch(targets, count);
        std::vector<uint32_t> want(q * count);
        std::vector<uint8_t> wcnt(q);
        orc_flat_nc_closest(n, sids.data(), sst.data(), q, reinterpret_cast<const uint8_t*>(targets.data()), count,
                            want.data(), wcnt.data(), 4);
        for (uint32_t i = 0; i < q; i++) {
            EXPECT(got[i].size() == wcnt[i], "nc count q=%u", i);
            for (uint32_t j = 0; j < got[i].size() && j < wcnt[i]; j++)
                EXPECT(got[i][j]->idx == sorted_to_node[want[i * count + j]], "nc node q=%u j=%u", i, j);
        }
    }
    // Incremental mirror: Dht::onNewNode (replace an expired node / emplace_front / split my bucket)
    // and Dht::expireBuckets on the host table, recorded on the mirror and flushed to the device.
    {
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
            auto nb = rt.insert(std::next(b), Bucket{mid, {}});
            std::list<std::shared_ptr<Node>> tmp;
            tmp.splice(tmp.begin(), b->nodes);
            while (!tmp.empty()) {
                auto it = tmp.begin();
                auto dst = find_bucket((*it)->id);
                dst->nodes.splice(dst->nodes.begin(), tmp, it);
            }
            (void)nb;
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
        std::vector<uint8_t> mids, mst, mfirst;
        std::vector<uint32_t> moff;
        std::vector<const Node*> mnode;
        for (auto& b : rt) {
            moff.push_back((uint32_t)mnode.size());
            mfirst.insert(mfirst.end(), b.first.begin(), b.first.end());
            for (auto& nd : b.nodes) {
                mids.insert(mids.end(), nd->id.begin(), nd->id.end());
                mst.push_back((uint8_t)((nd->isGood(now) ? 1 : 0) | (nd->isExpired() ? 2 : 0)));
                mnode.push_back(nd.get());
            }
        }
        moff.push_back((uint32_t)mnode.size());
        EXPECT(mirror.nodeCount() == mnode.size(), "mirror nodes %zu vs %zu", mirror.nodeCount(), mnode.size());
        for (uint32_t count : {1u, 8u, 14u}) {
            auto got = mirror.findClosestNodesBatch(targets, count);
            std::vector<uint32_t> want(q * count);
            std::vector<uint8_t> wcnt(q);
            orc_flat_rt_closest((uint32_t)mnode.size(), mids.data(), mst.data(), (uint32_t)rt.size(), mfirst.data(),
                                moff.data(), q, reinterpret_cast<const uint8_t*>(targets.data()), count, want.data(),
                                wcnt.data(), 4);
            for (uint32_t i = 0; i < q; i++) {
                EXPECT(got[i].size() == wcnt[i], "mirror count q=%u k=%u", i, count);
                for (uint32_t j = 0; j < got[i].size() && j < wcnt[i]; j++)
                    EXPECT(got[i][j].get() == mnode[want[i * count + j]], "mirror node q=%u k=%u j=%u", i, count, j);
            }
        }
        std::printf("mirror: %u replaced, %u added, %u splits, %u removed\n", replaced, added, splits, removed);
        EXPECT(replaced && added && splits && removed, "every mutation kind exercised");
    }
    // Dht-style accessor over two families
    kadgpu::DhtMirror<RoutingTable> dht;
    RoutingTable empty6;
    dht.snapshot(rt, empty6, now, 0);
    EXPECT(dht.findClosestNodes(targets[4], 2 /*AF_INET*/, 8, 2).size() == 8, "dht v4");
    EXPECT(dht.findClosestNodes(targets[4], 10 /*AF_INET6*/, 8, 2).empty(), "dht v6 empty table");
    std::printf("%s (%d failures)\n", fails ? "FAIL" : "PASS", fails);
    return fails ? 1 : 0;
}
