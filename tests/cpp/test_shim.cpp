// C++ test of include/kadgpu.hpp against test doubles shaped like OpenDHT's types
// (InfoHash = std::array<uint8_t,20>, Node with isGood/isExpired, Bucket{first, list<shared_ptr<Node>>},
// RoutingTable = std::list<Bucket>, NodeCache family map = std::map<InfoHash, weak_ptr<Node>>).
// Expected results come from the CPU oracle (test infrastructure). Needs a GPU. Exit 0 = pass.
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
    // Dht-style accessor over two families
    kadgpu::DhtMirror<RoutingTable> dht;
    RoutingTable empty6;
    dht.snapshot(rt, empty6, now, 0);
    EXPECT(dht.findClosestNodes(targets[4], 2 /*AF_INET*/, 8, 2).size() == 8, "dht v4");
    EXPECT(dht.findClosestNodes(targets[4], 10 /*AF_INET6*/, 8, 2).empty(), "dht v6 empty table");
    std::printf("%s (%d failures)\n", fails ? "FAIL" : "PASS", fails);
    return fails ? 1 : 0;
}
