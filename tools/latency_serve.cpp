// One Dht request through the C ABI with no Python in the way: kad_rt_closest_batch_host /
// kad_nc_closest_batch_host on a ~170-node split-policy table (SURVEY.md §6's live-sized table), through
// the launch path and through the resident query service (kad_table_serve), with the service's own
// device-side time per request (kad_table_serve_stats). Build (tools/README.md):
//   g++ -O2 -std=c++17 -Iinclude -o tools/latency_serve tools/latency_serve.cpp -Lopendht_amd -lkadgpu \
//       -Wl,-rpath,'$ORIGIN/../opendht_amd'
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kadgpu.h"

#define CK(x)                                                                         \
    do {                                                                              \
        int rc_ = (x);                                                                \
        if (rc_) {                                                                    \
            std::fprintf(stderr, "%s: %d %s\n", #x, rc_, kad_last_error());           \
            std::exit(1);                                                             \
        }                                                                             \
    } while (0)

static double pct(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(p * (v.size() - 1))];
}

int main(int argc, char** argv) {
    const uint32_t n = argc > 1 ? (uint32_t)std::atoi(argv[1]) : 170, reps = 5000;
    std::vector<uint8_t> ids(20ull * n), st(n), sid(20ull * n), sst(n), first(20ull * n);
    std::vector<uint32_t> perm(n), off(n + 1);
    uint32_t B = 0;
    CK(kad_synth_ids(0x1A7, n, ids.data()));
    CK(kad_synth_status(0x1A8, n, 80, 10, st.data()));
    CK(kad_split_table(n, ids.data(), 8, perm.data(), first.data(), off.data(), &B));
    for (uint32_t i = 0; i < n; i++) {
        std::copy(&ids[20ull * perm[i]], &ids[20ull * perm[i] + 20], &sid[20ull * i]);
        sst[i] = st[perm[i]];
    }
    kad_table* t = nullptr;
    CK(kad_table_create(&t, 0, n, sid.data(), sst.data(), B, first.data(), off.data(), 0, 0));
    std::vector<uint8_t> tg(20ull * 4096);
    CK(kad_synth_ids(0x1A9, 4096, tg.data()));
    std::vector<uint32_t> idx(64 * 64);
    std::vector<uint8_t> cnt(64);
    std::printf("{\"nodes\": %u, \"buckets\": %u", n, B);
    for (int serve = 0; serve < 2; serve++) {
        if (serve) CK(kad_table_serve(t, 100000));
        for (uint32_t q : {1u, 64u}) {
            std::vector<double> us, busy;
            for (uint32_t r = 0; r < reps; r++) {
                const uint8_t* x = &tg[20ull * ((r * q) % (4096 - q))];
                const auto a = std::chrono::steady_clock::now();
                CK(kad_rt_closest_batch_host(t, x, q, 8, idx.data(), cnt.data()));
                us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - a).count());
                if (serve) {
                    kad_serve_stats s;
                    CK(kad_table_serve_stats(t, &s));
                    busy.push_back(s.last_busy_ns / 1e3);
                }
            }
            const char* k = serve ? "serve" : "launch";
            std::printf(", \"%s_q%u_us\": %.2f, \"%s_q%u_p99_us\": %.2f", k, q, pct(us, 0.5), k, q, pct(us, 0.99));
            if (serve) std::printf(", \"serve_q%u_device_us\": %.2f", q, pct(busy, 0.5));
        }
    }
    kad_serve_stats s;
    CK(kad_table_serve_stats(t, &s));
    std::printf(", \"launches\": %llu, \"requests\": %llu}\n", (unsigned long long)s.launches,
                (unsigned long long)s.requests);
    CK(kad_table_destroy(t));
    return 0;
}
