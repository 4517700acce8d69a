// Host code under AddressSanitizer + UndefinedBehaviorSanitizer (CPU only, no GPU): the native table
// builders of libkadgpu.so (opendht_amd/csrc/kad_synth.cpp: synthetic IDs and status, sort, U(d) and
// split-policy tables, counter-based shards), the mirror's host plan (kad_mirror_plan.cpp, checked
// against the oracle's std::list table after random op batches) and the CPU oracle (oracle/kad_oracle.cpp: both
// restatements, NodeCache walk, mirror ops, swarm model, wire filter, SHA-1), compiled from source with
// -fsanitize=address,undefined and exercised on tables from 0 to 60k nodes. Built and run by
// tests/test_sanitizers.py (make -C tests/cpp sanitize_host). Exit 0 and "PASS" = no report.
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <random>
#include <string>
#include <vector>

#include "kadgpu.h"
#include "../../opendht_amd/csrc/kad_mirror_plan.h"

extern "C" {
int orc_flat_rt_closest(uint32_t, const uint8_t*, const uint8_t*, uint32_t, const uint8_t*, const uint32_t*, uint32_t,
                        const uint8_t*, uint32_t, uint32_t*, uint8_t*, int);
int orc_flat_nc_closest(uint32_t, const uint8_t*, const uint8_t*, uint32_t, const uint8_t*, uint32_t, uint32_t*, uint8_t*,
                        int);
void* orc_table_build(uint32_t, const uint8_t*, const uint8_t*, uint32_t, const uint8_t*, const uint32_t*, int);
void orc_table_free(void*);
int orc_table_rt_closest(void*, uint32_t, const uint8_t*, uint32_t, uint32_t*, uint8_t*, int);
int orc_table_nc_closest(void*, uint32_t, const uint8_t*, uint32_t, uint32_t*, uint8_t*, int);
int orc_table_apply(void*, uint32_t, const uint32_t*, uint32_t, const uint8_t*, const uint8_t*, uint32_t*, uint32_t*,
                    uint8_t*, uint8_t*, uint8_t*, uint32_t*, uint32_t*, uint32_t*);
int orc_split_table(uint32_t, const uint8_t*, uint32_t, uint32_t*, uint8_t*, uint32_t*, uint32_t*);
void* orc_swarm_build(uint32_t, const uint8_t*, int);
void orc_swarm_free(void*);
int orc_swarm_search(void*, uint32_t, const uint32_t*, const uint8_t*, uint32_t, uint32_t*, uint8_t*, uint8_t*, uint32_t*,
                     uint8_t*, int);
int orc_parse_nodes(uint32_t, const uint8_t*, uint32_t, const uint8_t*, uint8_t*);
int orc_infohash_get(uint32_t, const uint8_t*, const uint64_t*, uint8_t*);
}

static int fails = 0;
#define EXPECT(c, ...) do { if (!(c)) { fails++; std::fprintf(stderr, __VA_ARGS__); std::fprintf(stderr, "\n"); } } while (0)

// Random batches of removals, replacements, insertions and splits: kad_table_apply's host plan, with its
// segments resolved to IDs on the host, against orc_table_apply on the structure-faithful table.
static void check_mirror_plan(std::mt19937_64& g, uint32_t n, const std::vector<uint8_t>& sid,
                              const std::vector<uint8_t>& sst, uint32_t B, const std::vector<uint8_t>& first,
                              const std::vector<uint32_t>& off) {
    const std::vector<uint32_t> off0(off.begin(), off.begin() + B + 1);
    for (int trial = 0; trial < 6; trial++) {
        const uint32_t n_new = 1 + (uint32_t)(g() % 40), n_rm = (uint32_t)(g() % 30), n_split = (uint32_t)(g() % 6);
        std::vector<uint8_t> nid(20ull * n_new), nst(n_new, 1);
        for (auto& x : nid) x = (uint8_t)g();
        std::vector<uint32_t> pick(n);  // distinct old nodes for removals / replacements
        for (uint32_t i = 0; i < n; i++) pick[i] = i;
        std::shuffle(pick.begin(), pick.end(), g);
        std::vector<uint32_t> ops;
        uint32_t used = 0, slot = 0;
        for (uint32_t r = 0; r < n_rm && used < n; r++) ops.insert(ops.end(), {KAD_OP_REMOVE, pick[used++], 0});
        for (; slot < n_new / 2 && used < n; slot++) {  // the new ID: the old one's top 96 bits (same bucket)
            std::memcpy(&nid[20ull * slot], &sid[20ull * pick[used]], 12);
            ops.insert(ops.end(), {KAD_OP_REPLACE, pick[used++], slot});
        }
        for (; slot < n_new; slot++) ops.insert(ops.end(), {KAD_OP_INSERT, slot, 0});
        for (uint32_t s = 0; s < n_split; s++) ops.insert(ops.end(), {KAD_OP_SPLIT, (uint32_t)(g() % B), 0});
        // shuffle the op rows (node operands stay batch-start indices)
        const uint32_t n_ops = (uint32_t)(ops.size() / 3);
        std::vector<uint32_t> ord(n_ops);
        for (uint32_t i = 0; i < n_ops; i++) ord[i] = i;
        std::shuffle(ord.begin(), ord.end(), g);
        std::vector<uint32_t> rows(3ull * n_ops);
        for (uint32_t i = 0; i < n_ops; i++) std::memcpy(&rows[3ull * i], &ops[3ull * ord[i]], 12);
        kadplan::MirrorPlan plan;
        std::string err;
        const kadplan::OldIds old_ids = [&](uint32_t a, uint32_t e, uint8_t* out) {
            std::memcpy(out, sid.data() + 20ull * a, 20ull * (e - a));
            return KAD_OK;
        };
        const int rc = kadplan::mirror_plan(off0, first.data(), n, rows.data(), n_ops, nid.data(), n_new, -1, 0, old_ids,
                                            plan, err);
        EXPECT(rc == KAD_OK, "mirror plan n=%u: %s", n, err.c_str());
        if (rc) continue;
        if (trial == 0 && B > 1 && off[1] > 0 && off[B] > off[B - 1]) {  // a replacement from another bucket is refused
            std::vector<uint8_t> far(sid.begin() + 20ull * off[B - 1], sid.begin() + 20ull * off[B - 1] + 20);
            far[19] ^= 1;
            const uint32_t bad[] = {KAD_OP_REPLACE, 0, 0};
            kadplan::MirrorPlan p2;
            std::string e2;
            EXPECT(kadplan::mirror_plan(off0, first.data(), n, bad, 1, far.data(), 1, -1, 0, old_ids, p2, e2) ==
                       KAD_ERR_INVALID,
                   "out-of-bucket replacement accepted n=%u", n);
        }
        // the plan's layout as IDs
        std::vector<uint8_t> got(20ull * plan.n1 + 1);
        uint32_t at = 0;
        for (const auto& sg : plan.segs) {
            EXPECT(sg.start == at, "segment start %u, expected %u", sg.start, at);
            for (uint32_t i = 0; i < sg.len; i++) {
                const uint32_t h = sg.kind ? plan.list[sg.src + i] : sg.src + i;
                const uint8_t* src = h & kadplan::MIRROR_NEW ? nid.data() + 20ull * (h & ~kadplan::MIRROR_NEW)
                                                             : sid.data() + 20ull * h;
                std::memcpy(&got[20ull * at++], src, 20);
            }
        }
        EXPECT(at == plan.n1, "segments cover %u of %u nodes", at, plan.n1);
        // the same ops on the oracle
        void* T = orc_table_build(n, sid.data(), sst.data(), B, first.data(), off.data(), 1);
        const uint32_t cap = n + n_new + 1, capB = B + n_split + 1;
        std::vector<uint8_t> oid(20ull * cap), ost(cap), of(20ull * capB);
        std::vector<uint32_t> oo(capB + 1), rm(n + 1), ni(n_new);
        uint32_t on = 0, oB = 0;
        orc_table_apply(T, n_ops, rows.data(), n_new, nid.data(), nst.data(), &on, &oB, oid.data(), ost.data(), of.data(),
                        oo.data(), rm.data(), ni.data());
        orc_table_free(T);
        const uint8_t* f1 = plan.B1 != B ? plan.first1.data() : first.data();
        EXPECT(on == plan.n1 && oB == plan.B1, "mirror plan n=%u trial %d: %u nodes / %u buckets, oracle %u / %u", n, trial,
               plan.n1, plan.B1, on, oB);
        if (on == plan.n1 && oB == plan.B1) {
            EXPECT(std::memcmp(got.data(), oid.data(), 20ull * on) == 0, "mirror plan n=%u trial %d: node order", n, trial);
            EXPECT(std::equal(oo.begin(), oo.begin() + oB + 1, plan.off1.begin()), "mirror plan n=%u: offsets", n);
            EXPECT(std::memcmp(f1, of.data(), 20ull * oB) == 0, "mirror plan n=%u: firsts", n);
        }
    }
}

int main() {
    std::mt19937_64 g(11);
    for (uint32_t n : {0u, 1u, 3u, 50u, 5000u, 60000u}) {
        std::vector<uint8_t> ids(20ull * n + 1), st(n + 1);
        EXPECT(kad_synth_ids(0xA5A5 + n, n, ids.data()) == KAD_OK, "synth ids");
        EXPECT(kad_synth_status(0x5A5A, n, 70, 20, st.data()) == KAD_OK, "synth status");
        // split-policy table: the native builder against the oracle's list-of-lists builder
        std::vector<uint32_t> perm(n + 1), off(n + 2), perm2(n + 1), off2(n + 2);
        std::vector<uint8_t> first(20ull * (n + 1)), first2(20ull * (n + 1));
        uint32_t B = 0, B2 = 0;
        EXPECT(kad_split_table(n, ids.data(), 8, perm.data(), first.data(), off.data(), &B) == KAD_OK, "split");
        EXPECT(orc_split_table(n, ids.data(), 8, perm2.data(), first2.data(), off2.data(), &B2) == 0, "orc split");
        EXPECT(B == B2 && std::memcmp(first.data(), first2.data(), 20ull * B) == 0, "split tables differ n=%u", n);
        std::vector<uint8_t> sid(20ull * n + 1), sst(n + 1);
        for (uint32_t i = 0; i < n; i++) {
            std::memcpy(&sid[20ull * i], &ids[20ull * perm[i]], 20);
            sst[i] = st[perm[i]];
        }
        const uint32_t q = 700;
        std::vector<uint8_t> tg(20ull * q);
        for (auto& x : tg) x = (uint8_t)g();
        for (uint32_t k : {1u, 8u, 14u, 32u}) {
            std::vector<uint32_t> a(q * k), b(q * k);
            std::vector<uint8_t> ca(q), cb(q);
            orc_flat_rt_closest(n, sid.data(), sst.data(), B, first.data(), off.data(), q, tg.data(), k, a.data(),
                                ca.data(), 2);
            void* T = orc_table_build(n, sid.data(), sst.data(), B, first.data(), off.data(), 1);
            orc_table_rt_closest(T, q, tg.data(), k, b.data(), cb.data(), 2);
            EXPECT(a == b && ca == cb, "restatements differ n=%u k=%u", n, k);
            orc_table_nc_closest(T, q, tg.data(), k, b.data(), cb.data(), 2);
            // mirror ops: remove, insert, split on the structure-faithful table
            if (n >= 50 && k == 8) {
                std::vector<uint8_t> nid(20 * 4);
                for (auto& x : nid) x = (uint8_t)g();
                const uint32_t ops[] = {KAD_OP_REMOVE, 3, 0, KAD_OP_INSERT, 0, 0, KAD_OP_INSERT, 1, 0, KAD_OP_SPLIT, 0, 0};
                const uint8_t nst[4] = {1, 1, 0, 2};
                const uint32_t cap = n + 8, capB = B + 8;
                std::vector<uint8_t> oid(20ull * cap), ost(cap), of(20ull * capB);
                std::vector<uint32_t> oo(capB + 1), rm(n), ni(4);
                uint32_t on = 0, oB = 0;
                orc_table_apply(T, 4, ops, 4, nid.data(), nst, &on, &oB, oid.data(), ost.data(), of.data(), oo.data(),
                                rm.data(), ni.data());
                EXPECT(on == n + 1, "apply node count %u", on);
            }
            orc_table_free(T);
        }
        if (n >= 50) check_mirror_plan(g, n, sid, sst, B, first, off);
        // uniform buckets + NodeCache walk over the sorted array
        std::vector<uint8_t> srt(ids.begin(), ids.begin() + 20ull * n);
        srt.push_back(0);
        std::vector<uint32_t> sp(n + 1);
        kad_sort_ids(n, srt.data(), sp.data());
        if (n) {
            const uint32_t d = 6;
            std::vector<uint8_t> uf(20ull << d);
            std::vector<uint32_t> uo((1u << d) + 1);
            EXPECT(kad_uniform_buckets(n, srt.data(), d, 0, 0, uf.data(), uo.data()) == KAD_OK, "uniform");
            std::vector<uint32_t> a(q * 14);
            std::vector<uint8_t> ca(q);
            orc_flat_nc_closest(n, srt.data(), st.data(), q, tg.data(), 14, a.data(), ca.data(), 2);
            orc_flat_rt_closest(n, srt.data(), st.data(), 1u << d, uf.data(), uo.data(), q, tg.data(), 8, a.data(),
                                ca.data(), 2);
        }
        if (n >= 50) {  // swarm model and lookups
            void* sw = orc_swarm_build(n, srt.data(), 2);
            const uint32_t S = 64;
            std::vector<uint32_t> src(S), L(S * 14), hops(S);
            std::vector<uint8_t> qf(S * 14), ln(S), done(S), t2(20ull * S);
            for (uint32_t i = 0; i < S; i++) src[i] = (uint32_t)(g() % n);
            for (auto& x : t2) x = (uint8_t)g();
            orc_swarm_search(sw, S, src.data(), t2.data(), 32, L.data(), qf.data(), ln.data(), hops.data(), done.data(), 2);
            orc_swarm_free(sw);
        }
    }
    // counter-based shard generator
    uint32_t cnt = 0;
    EXPECT(kad_synth_uniform_shard(7, 12, 100, 300, 6.0, 80, 10, &cnt, nullptr, nullptr, nullptr) == KAD_OK, "shard count");
    std::vector<uint8_t> si(20ull * cnt + 1), ss(cnt + 1);
    std::vector<uint32_t> so(201);
    EXPECT(kad_synth_uniform_shard(7, 12, 100, 300, 6.0, 80, 10, &cnt, si.data(), ss.data(), so.data()) == KAD_OK, "shard");
    // wire filter and SHA-1
    std::vector<uint8_t> rec(26 * 100), keep(100), my(20, 7);
    for (auto& x : rec) x = (uint8_t)g();
    orc_parse_nodes(100, rec.data(), 26, my.data(), keep.data());
    std::vector<uint8_t> data(1000);
    for (auto& x : data) x = (uint8_t)g();
    std::vector<uint64_t> koff = {0, 0, 3, 64, 65, 1000};
    std::vector<uint8_t> h(20 * 5);
    orc_infohash_get(5, data.data(), koff.data(), h.data());
    std::printf("%s (%d failures)\n", fails ? "FAIL" : "PASS", fails);
    return fails ? 1 : 0;
}
