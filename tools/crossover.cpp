// The single-request crossover (verdict r03 item 4): RoutingTableMirror::findClosestNodes through the shim on
// reference-shaped test doubles (the split policy of Dht::onNewNode, tables of 170 .. 1M nodes), for q requests
// of count 8: the host path (findClosestNodesHost: closed form over the bucket directory, isGood read from the
// Node objects), the resident query service (kad_table_serve) and one kernel launch per call. Median of many
// calls, microseconds. Prints one JSON object.
// Build: g++ -O2 -std=c++17 -Iinclude -o tools/crossover tools/crossover.cpp -Lopendht_amd -lkadgpu
//        -Wl,-rpath,'$ORIGIN/../opendht_amd'
#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <list>
#include <memory>
#include <random>
#include <vector>

#include "kadgpu.hpp"

namespace mock {
using clock = std::chrono::steady_clock;
using time_point = clock::time_point;
struct InfoHash : std::array<uint8_t, 20> {};
struct Node {  // node.h:35-105 / node.cpp:34-40 in miniature
    InfoHash id;
    time_point time{time_point::min()}, reply_time{time_point::min()};
    bool expired_ = false;
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
}  // namespace mock
using namespace mock;

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

int main() {
    const time_point t0 = clock::now();
    std::mt19937_64 g(0xC05);
    std::printf("{\"count\": 8, \"tables\": [");
    bool firstt = true;
    for (uint32_t m : {170u, 1000u, 10000u, 100000u, 1000000u}) {
        std::vector<uint8_t> lid(20ull * m);
        kadgpu::check(kad_synth_ids(0x1A7 + m, m, lid.data()), "synth");
        std::vector<uint32_t> perm(m), off(m + 2);
        std::vector<uint8_t> first(20ull * (m + 1));
        uint32_t B = 0;
        kadgpu::check(kad_split_table(m, lid.data(), 8, perm.data(), first.data(), off.data(), &B), "split");
        RoutingTable rt;
        std::vector<std::shared_ptr<Node>> keep;
        for (uint32_t b = 0; b < B; b++) {
            Bucket bk;
            std::memcpy(bk.first.data(), &first[20ull * b], 20);
            for (uint32_t j = off[b]; j < off[b + 1]; j++) {
                auto nd = std::make_shared<Node>();
                std::memcpy(nd->id.data(), &lid[20ull * perm[j]], 20);
                nd->time = nd->reply_time = t0 - std::chrono::seconds(g() % 500);  // good, heard over ~8 min
                keep.push_back(nd);
                bk.nodes.push_back(nd);
            }
            rt.push_back(bk);
        }
        std::vector<InfoHash> targets(4096);
        for (auto& t : targets)
            for (auto& x : t) x = (uint8_t)g();
        kadgpu::RoutingTableMirror<RoutingTable> mir(rt, t0, 0);
        const int reps = m >= 1000000 ? 300 : 1000;
        auto time_q = [&](uint32_t q) {  // median microseconds of one findClosestNodesBatch of q requests
            std::vector<double> us;
            for (int r = 0; r < reps; r++) {
                const auto a = clock::now();
                auto res = mir.findClosestNodesBatch(&targets[(r * q) % (4096 - q)], q, t0, 8);
                us.push_back(std::chrono::duration<double, std::micro>(clock::now() - a).count());
                if (res.size() != q) std::abort();
            }
            return med(us);
        };
        const uint32_t qs[] = {1, 2, 4, 8, 16, 32, 64};
        double host[7], served[7], launch[7];
        mir.setHostPath(64);  // every q below on the host path
        for (int k = 0; k < 7; k++) host[k] = time_q(qs[k]);
        mir.setHostPath(0);
        for (int k = 0; k < 7; k++) launch[k] = time_q(qs[k]);
        mir.serve(100000);
        for (int k = 0; k < 7; k++) served[k] = time_q(qs[k]);
        mir.serve(0);
        std::printf("%s{\"nodes\": %u, \"buckets\": %u, \"q\": [1, 2, 4, 8, 16, 32, 64], \"host_us\": [", firstt ? "" : ", ",
                    m, B);
        for (int k = 0; k < 7; k++) std::printf("%s%.2f", k ? ", " : "", host[k]);
        std::printf("], \"served_us\": [");
        for (int k = 0; k < 7; k++) std::printf("%s%.2f", k ? ", " : "", served[k]);
        std::printf("], \"launch_us\": [");
        for (int k = 0; k < 7; k++) std::printf("%s%.2f", k ? ", " : "", launch[k]);
        int cross = 0;  // the largest q for which the host path is the fastest
        for (int k = 0; k < 7; k++)
            if (host[k] <= std::min(served[k], launch[k])) cross = (int)qs[k];
        std::printf("], \"host_fastest_up_to_q\": %d}", cross);
        std::fflush(stdout);
        firstt = false;
    }
    std::printf("]}\n");
    return 0;
}
