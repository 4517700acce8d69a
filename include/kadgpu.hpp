/*
 * kadgpu.hpp — C++11 host shim over the kadgpu C ABI, with OpenDHT's own signatures.
 *
 * Drop-in for the reference path (OpenDHT 1.2.1):
 *   RoutingTable::findClosestNodes(const InfoHash, time_point, size_t)   routing_table.h:48
 *   RoutingTable::findBucket(const InfoHash&)                            routing_table.h:50-51
 *   NodeCache::getCachedNodes(const InfoHash&, sa_family_t, size_t)      node_cache.h:32
 *   Dht::findClosestNodes(id, af, count) -- the accessor SURVEY.md §0.3 asks for, equal to
 *   buckets(af).findClosestNodes(id, scheduler.time(), count)             dht.h:437-438
 *
 * The shim is generic over the reference's types, so it compiles against OpenDHT's own headers
 * without modifying them (and against test doubles of the same shape):
 *   RoutingTableT : iterable of Buckets in ascending `first` order (std::list<Bucket>)
 *   Bucket        : `first` (20 contiguous bytes via .data()), `nodes` (iterable of shared_ptr<NodeT>)
 *   NodeT         : `id` (20 bytes via .data()), `bool isGood(time_point) const`, `bool isExpired() const`
 *   NodeMapT      : std::map<InfoHash, std::weak_ptr<NodeT>> (one NodeCache family, node_cache.h:42-50)
 *
 * A mirror holds the table's node IDs, bucket directory and every node's liveness (Node::time,
 * reply_time, isExpired(); node.h:39-40, 67) on the device. findClosestNodes(id, now, count) evaluates
 * Node::isGood(now) for the `now` it is given, as the reference does per call (routing_table.cpp:77):
 * when `now` moves, kad_table_refresh_status re-derives the status on the device and rebuilds only what
 * flipped. Results come back as the same shared_ptr<NodeT> objects the table holds, in the reference's
 * order. What the mirror cannot observe must be reported:
 *   - liveness changes of a node (Node::received, setExpired, reset, a search writing node->time):
 *     nodeUpdated(node) before the next query (or syncTimes() to re-read every node);
 *   - table mutations (Dht::onNewNode / expireBuckets / split): nodeRemoved / nodeReplaced / nodeAdded /
 *     bucketSplit, then flush(now): kad_table_apply replays them on the device copy; or re-snapshot.
 */
#ifndef KADGPU_HPP
#define KADGPU_HPP

#include <sys/socket.h>  // AF_INET (sa_family_t), as OpenDHT's sockaddr.h

#include <algorithm>
#include <chrono>
#include <climits>
#include <cstdint>
#include <functional>
#include <unordered_map>
#include <cstring>
#include <iterator>
#include <memory>
#include <stdexcept>
#include <string>
#include <type_traits>
#include <utility>
#include <vector>

#include "kadgpu.h"

namespace kadgpu {

class Error : public std::runtime_error {
public:
    Error(int code, const std::string& what) : std::runtime_error(what), code_(code) {}
    int code() const { return code_; }

private:
    int code_;
};

inline void check(int rc, const char* where) {
    if (rc != KAD_OK) throw Error(rc, std::string(where) + ": " + kad_last_error());
}

/* RAII owner of one device table (kad_table_create / kad_table_destroy). */
class DeviceTable {
public:
    DeviceTable() {}
    DeviceTable(int device, const std::vector<uint8_t>& ids, const std::vector<uint8_t>& status,
                const std::vector<uint8_t>& bucket_first, const std::vector<uint32_t>& bucket_offset,
                uint32_t index_base = 0, bool sorted = false) {
        const uint32_t n = (uint32_t)(ids.size() / KAD_HASH_LEN);
        const uint32_t B = (uint32_t)(bucket_first.size() / KAD_HASH_LEN);
        check(kad_table_create(&t_, device, n, ids.data(), status.data(), B, B ? bucket_first.data() : nullptr,
                               B ? bucket_offset.data() : nullptr, index_base, sorted ? KAD_TABLE_SORTED : 0u),
              "kad_table_create");
    }
    ~DeviceTable() { reset(); }
    DeviceTable(const DeviceTable&) = delete;
    DeviceTable& operator=(const DeviceTable&) = delete;
    DeviceTable(DeviceTable&& o) : t_(o.t_) { o.t_ = nullptr; }
    DeviceTable& operator=(DeviceTable&& o) {
        if (this != &o) { reset(); t_ = o.t_; o.t_ = nullptr; }
        return *this;
    }
    void reset() {
        if (t_) kad_table_destroy(t_);
        t_ = nullptr;
    }
    kad_table* get() const { return t_; }
    explicit operator bool() const { return t_ != nullptr; }

    /* Resident query service for single requests (kad_table_serve); idle_us = 0 turns it off. */
    void serve(uint32_t idle_us) const { check(kad_table_serve(t_, idle_us), "kad_table_serve"); }

    /* Host-buffer batch queries (synchronous). Rows of `count` indices, KAD_NO_NODE padded. */
    void findClosestNodesBatch(const uint8_t* targets, size_t q, size_t count, std::vector<uint32_t>& idx,
                               std::vector<uint8_t>& cnt) const {
        idx.resize(q * count);
        cnt.resize(q);
        if (q) check(kad_rt_closest_batch_host(t_, targets, (uint32_t)q, (uint32_t)count, idx.data(), cnt.data()),
                     "kad_rt_closest_batch_host");
    }
    void getCachedNodesBatch(const uint8_t* targets, size_t q, size_t count, std::vector<uint32_t>& idx,
                             std::vector<uint8_t>& cnt) const {
        idx.resize(q * count);
        cnt.resize(q);
        if (q) check(kad_nc_closest_batch_host(t_, targets, (uint32_t)q, (uint32_t)count, idx.data(), cnt.data()),
                     "kad_nc_closest_batch_host");
    }

    /* Node liveness (kad_table_set_times / kad_table_patch_times) and the device-side isGood(now)
     * refresh (kad_table_refresh_status, incremental). */
    void setTimes(const std::vector<int64_t>& time_ns, const std::vector<int64_t>& reply_ns,
                  const std::vector<uint8_t>& expired) {
        check(kad_table_set_times(t_, time_ns.data(), reply_ns.data(), expired.data()), "kad_table_set_times");
    }
    void patchTimes(const std::vector<uint32_t>& nodes, const std::vector<int64_t>& time_ns,
                    const std::vector<int64_t>& reply_ns, const std::vector<uint8_t>& expired) {
        if (!nodes.empty())
            check(kad_table_patch_times(t_, (uint32_t)nodes.size(), nodes.data(), time_ns.data(), reply_ns.data(),
                                        expired.data()), "kad_table_patch_times");
    }
    void patchStatus(const std::vector<uint32_t>& nodes, const std::vector<uint8_t>& status) {
        if (!nodes.empty())
            check(kad_table_patch_status(t_, (uint32_t)nodes.size(), nodes.data(), status.data()),
                  "kad_table_patch_status");
    }
    void refreshStatus(int64_t now_ns) {
        check(kad_table_refresh_status(t_, now_ns, nullptr), "kad_table_refresh_status");
    }

private:
    kad_table* t_ = nullptr;
};

/* time_point -> int64 nanoseconds of its clock, time_point::min()/max() -> INT64_MIN/MAX (Node::time and
 * reply_time start at time_point::min(), node.h:39-40). */
template <class TimePoint>
inline int64_t to_ns(TimePoint tp) {
    if (tp == TimePoint::min()) return INT64_MIN;
    if (tp == TimePoint::max()) return INT64_MAX;
    return (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tp.time_since_epoch()).count();
}

/* Status byte of a node at `now`: Node::isGood(now) | Node::isExpired() << 1 (node.cpp:34-40, node.h:67). */
template <class NodePtr, class TimePoint>
inline uint8_t status_of(const NodePtr& n, TimePoint now) {
    return (uint8_t)((n->isGood(now) ? KAD_STATUS_GOOD : 0u) | (n->isExpired() ? KAD_STATUS_EXPIRED : 0u));
}

template <class T>
inline const uint8_t* id_bytes(const T& id) {
    static_assert(sizeof(id) == KAD_HASH_LEN, "InfoHash must be 20 contiguous bytes");
    return reinterpret_cast<const uint8_t*>(id.data());
}

/* Device mirror of one RoutingTable (one address family). */
template <class RoutingTableT>
class RoutingTableMirror {
public:
    using BucketT = typename std::decay<decltype(*std::declval<const RoutingTableT&>().begin())>::type;
    using NodePtr = typename std::decay<decltype(*std::declval<const BucketT&>().nodes.begin())>::type;

    RoutingTableMirror() {}

    template <class TimePoint>
    RoutingTableMirror(const RoutingTableT& rt, TimePoint now, int device = 0) {
        snapshot(rt, now, device);
    }

    /* Snapshot `rt`: nodes grouped by bucket in list order, their liveness, status at `now`. */
    template <class TimePoint>
    void snapshot(const RoutingTableT& rt, TimePoint now, int device = 0) {
        std::vector<uint8_t> ids, status, first;
        std::vector<uint32_t> off;
        nodes_.clear();
        for (const auto& b : rt) {
            off.push_back((uint32_t)nodes_.size());
            first.insert(first.end(), id_bytes(b.first), id_bytes(b.first) + KAD_HASH_LEN);
            for (const auto& n : b.nodes) {
                nodes_.push_back(n);
                ids.insert(ids.end(), id_bytes(n->id), id_bytes(n->id) + KAD_HASH_LEN);
                status.push_back(status_of(n, now));
            }
        }
        off.push_back((uint32_t)nodes_.size());
        buckets_ = (uint32_t)(off.size() - 1);
        table_ = DeviceTable(device, ids, status, first, off);
        first_.swap(first);
        off_.swap(off);
        reindex();
        syncTimes();
        now_ns_ = to_ns(now);
        refresh_ = false;
    }

    /* RoutingTable::findClosestNodes(id, now, count) (routing_table.h:48, routing_table.cpp:67-111). */
    template <class InfoHashT, class TimePoint>
    std::vector<NodePtr> findClosestNodes(const InfoHashT& id, TimePoint now, size_t count = KAD_TARGET_NODES) const {
        std::vector<std::vector<NodePtr>> r = findClosestNodesBatch(&id, 1, now, count);
        return std::move(r[0]);
    }

    /* Batched form: one result vector per target, all at the same `now`. */
    template <class InfoHashT, class TimePoint>
    std::vector<std::vector<NodePtr>> findClosestNodesBatch(const InfoHashT* ids, size_t q, TimePoint now,
                                                            size_t count = KAD_TARGET_NODES) const {
        if (q <= hostBatchLimit() && count <= host_count_) {  // a few requests: the host path (no device round trip)
            std::vector<std::vector<NodePtr>> out(q);
            for (size_t i = 0; i < q; i++) out[i] = findClosestNodesHost(ids[i], now, count);
            return out;
        }
        advance(to_ns(now));
        std::vector<std::vector<NodePtr>> out(q);
        // any size_t count, as routing_table.h:48: a result never holds more than the table's nodes
        count = std::min(count, nodes_.size());
        if (count == 0 || q == 0) return out;
        std::vector<uint8_t> targets(q * KAD_HASH_LEN);
        for (size_t i = 0; i < q; i++) std::memcpy(&targets[i * KAD_HASH_LEN], id_bytes(ids[i]), KAD_HASH_LEN);
        std::vector<uint32_t> idx;
        std::vector<uint8_t> cnt;
        table_.findClosestNodesBatch(targets.data(), q, count, idx, cnt);
        for (size_t i = 0; i < q; i++) {
            size_t m = cnt[i];
            if (count > 255)  // the count byte saturates: the row's padding gives the length
                for (m = 0; m < count && idx[i * count + m] != KAD_NO_NODE; m++) {}
            out[i].reserve(m);
            for (size_t j = 0; j < m; j++) out[i].push_back(nodes_[idx[i * count + j]]);
        }
        return out;
    }
    template <class InfoHashT, class TimePoint>
    std::vector<std::vector<NodePtr>> findClosestNodesBatch(const std::vector<InfoHashT>& ids, TimePoint now,
                                                            size_t count = KAD_TARGET_NODES) const {
        return findClosestNodesBatch(ids.data(), ids.size(), now, count);
    }

    /* A mirrored node's time / reply_time / expired_ changed (Node::received, setExpired, reset,
     * Search::insertNode writing node->time): re-read at the next query. */
    void nodeUpdated(const NodePtr& n) { updated_.push_back(index_of(n)); }
    /* Re-read every mirrored node's liveness (kad_table_set_times); status re-derived at the next query. */
    void syncTimes() {
        std::vector<int64_t> t(nodes_.size()), r(nodes_.size());
        std::vector<uint8_t> e(nodes_.size());
        for (size_t i = 0; i < nodes_.size(); i++) {
            t[i] = to_ns(nodes_[i]->time);
            r[i] = to_ns(nodes_[i]->reply_time);
            e[i] = nodes_[i]->isExpired() ? 1 : 0;
        }
        if (!nodes_.empty()) table_.setTimes(t, r, e);
        updated_.clear();
        refresh_ = true;
    }

    /* Incremental mirror (kad_table_apply): record the mutations the Dht makes to the host table, in
     * the order it makes them, then flush(now). Nodes named by nodeRemoved / nodeReplaced must be in
     * the last snapshot or flush (flush in between otherwise). */
    void nodeRemoved(const NodePtr& n) {  // Dht::expireBuckets remove_if (dht.cpp:942-956)
        op(KAD_OP_REMOVE, index_of(n), 0);
    }
    void nodeReplaced(const NodePtr& old, const NodePtr& n) {  // onNewNode: `n = node` (dht.cpp:917-921)
        op(KAD_OP_REPLACE, index_of(old), slot(n));
    }
    void nodeAdded(const NodePtr& n) {  // onNewNode: b->nodes.emplace_front(node) (dht.cpp:934)
        op(KAD_OP_INSERT, slot(n), 0);
    }
    void bucketSplit(size_t bucket_index) {  // RoutingTable::split (routing_table.cpp:137-163)
        op(KAD_OP_SPLIT, (uint32_t)bucket_index, 0);
        buckets_++;
    }
    template <class TimePoint>
    void flush(TimePoint now) {
        if (ops_.empty()) return;
        std::vector<uint8_t> ids, status;
        for (const auto& n : added_) {
            ids.insert(ids.end(), id_bytes(n->id), id_bytes(n->id) + KAD_HASH_LEN);
            status.push_back(status_of(n, now));
        }
        std::vector<uint32_t> remap(nodes_.size()), idx(added_.size());
        check(kad_table_apply(table_.get(), ops_.data(), (uint32_t)(ops_.size() / 3), ids.data(), status.data(),
                              (uint32_t)added_.size(), remap.data(), idx.data()),
              "kad_table_apply");
        kad_table_info inf;
        check(kad_table_get_info(table_.get(), &inf), "kad_table_get_info");
        std::vector<NodePtr> next(inf.n_nodes);
        for (size_t i = 0; i < nodes_.size(); i++)
            if (remap[i] != KAD_NO_NODE) next[remap[i]] = nodes_[i];
        for (size_t s = 0; s < added_.size(); s++)
            if (idx[s] != KAD_NO_NODE) next[idx[s]] = added_[s];
        nodes_.swap(next);
        buckets_ = inf.n_buckets;
        first_.assign((size_t)KAD_HASH_LEN * buckets_, 0);
        off_.assign(buckets_ + 1, 0);
        check(kad_table_export(table_.get(), nullptr, nullptr, buckets_ ? first_.data() : nullptr, off_.data()),
              "kad_table_export");
        ops_.clear();
        added_.clear();
        reindex();
        syncTimes();  // kad_table_apply drops the node times (the layout moved)
        now_ns_ = to_ns(now);
        refresh_ = true;
    }

    /* RoutingTable::findClosestNodes(id, now, count) on the host, over the mirror's bucket directory and the
     * table's own Node objects (isGood(now) read from them, as routing_table.cpp:77 does): the closed form of
     * routing_table.cpp:67-111 -- findBucket by binary search over the bucket firsts, the window W(r) grown ring
     * by ring until it holds `count` good nodes or the whole table, its good nodes ordered by (XOR distance,
     * index) -- no pass over the table and no device round trip. For a few single requests it answers faster
     * than a launch or the resident service (the crossover, tools/crossover.cpp); batches go to the device. */
    template <class InfoHashT, class TimePoint>
    std::vector<NodePtr> findClosestNodesHost(const InfoHashT& id, TimePoint now, size_t count = KAD_TARGET_NODES) const {
        std::vector<NodePtr> out;
        const uint32_t B = (uint32_t)(off_.size() ? off_.size() - 1 : 0);
        if (B == 0 || count == 0) return out;
        const uint8_t* t = id_bytes(id);
        // findBucket (routing_table.cpp:113-127): the last bucket whose first is <= t, the first if none
        uint32_t lo = 0, hi = B;
        while (lo < hi) {
            const uint32_t mid = (lo + hi) / 2;
            if (std::memcmp(&first_[(size_t)KAD_HASH_LEN * mid], t, KAD_HASH_LEN) <= 0) lo = mid + 1; else hi = mid;
        }
        const uint32_t b = lo ? lo - 1 : 0;
        // the window: W(0) = [b-1, b], each round one bucket more on either side (routing_table.cpp:89-104)
        struct Cand { uint32_t idx; const uint8_t* id; };
        std::vector<Cand> cand;
        size_t good = 0;
        auto take = [&](uint32_t x) {
            for (uint32_t j = off_[x]; j < off_[x + 1]; j++)
                if (nodes_[j]->isGood(now)) { cand.push_back(Cand{j, id_bytes(nodes_[j]->id)}); good++; }
        };
        uint32_t wl = b ? b - 1 : 0, wh = b;
        for (uint32_t x = wl; x <= wh; x++) take(x);
        while (good < count && !(wl == 0 && wh == B - 1)) {
            if (wh + 1 < B) take(++wh);
            if (wl > 0) take(--wl);
        }
        auto closer = [&](const Cand& a, const Cand& c) {  // InfoHash::xorCmp (infohash.h:131-146), then index
            for (unsigned k = 0; k < KAD_HASH_LEN; k++) {
                const uint8_t da = a.id[k] ^ t[k], dc = c.id[k] ^ t[k];
                if (da != dc) return da < dc;
            }
            return a.idx < c.idx;
        };
        const size_t m = std::min(count, cand.size());
        std::partial_sort(cand.begin(), cand.begin() + m, cand.end(), closer);
        out.reserve(m);
        for (size_t k = 0; k < m; k++) out.push_back(nodes_[cand[k].idx]);
        return out;
    }
    /* Batches of at most q requests with count <= max_count take the host path (0: never; kHostPathAuto, the
       default: q from the table size, below).
       The two paths read liveness differently: the host path evaluates isGood(now) on the table's own Node objects
       (as routing_table.cpp:77 does), the device path the liveness mirrored through nodeUpdated / syncTimes. They
       agree when every change is reported (the mirror's contract); a change that is not reported shows up only in
       the answers of device batches (more than hostBatchLimit() requests, or count above max_count). */
    static constexpr size_t kHostPathAuto = ~size_t(0);
    void setHostPath(size_t q, size_t max_count = 64) {
        host_q_ = q;
        host_count_ = max_count;
    }
    /* The largest batch the host path answers: set by setHostPath, else the crossover measured on MI355X
       (tools/crossover.cpp, profiles/r04/r04j/crossover.json: the host path beats both device paths up to 32
       requests on tables of up to 10k nodes, 16 at 100k, 8 at 1M). */
    size_t hostBatchLimit() const {
        if (host_q_ != kHostAuto) return host_q_;
        const size_t n = nodes_.size();
        return n <= 20000 ? 32 : n <= 200000 ? 16 : 8;
    }

    size_t bucketCount() const { return buckets_; }
    size_t nodeCount() const { return nodes_.size(); }
    const DeviceTable& table() const { return table_; }
    /* Single findClosestNodes calls answered by the resident query service (kad_table_serve); 0 turns it off. */
    void serve(uint32_t idle_us = 2000) const { table_.serve(idle_us); }

private:
    // status at the query's `now`: reported liveness changes first, then the device refresh
    void advance(int64_t now_ns) const {
        if (nodes_.empty()) {  // nothing to evaluate (and no times on the device)
            now_ns_ = now_ns;
            return;
        }
        if (!updated_.empty()) {
            std::vector<int64_t> t, r;
            std::vector<uint8_t> e;
            for (uint32_t i : updated_) {
                t.push_back(to_ns(nodes_[i]->time));
                r.push_back(to_ns(nodes_[i]->reply_time));
                e.push_back(nodes_[i]->isExpired() ? 1 : 0);
            }
            table_.patchTimes(updated_, t, r, e);
            updated_.clear();
            refresh_ = true;
        }
        if (refresh_ || now_ns != now_ns_) {
            table_.refreshStatus(now_ns);
            now_ns_ = now_ns;
            refresh_ = false;
        }
    }
    void reindex() {
        index_.clear();
        for (size_t i = 0; i < nodes_.size(); i++) index_[nodes_[i].get()] = (uint32_t)i;
    }
    void op(uint32_t kind, uint32_t a, uint32_t b) {
        ops_.push_back(kind);
        ops_.push_back(a);
        ops_.push_back(b);
    }
    uint32_t index_of(const NodePtr& n) const {
        auto it = index_.find(n.get());
        if (it == index_.end()) throw Error(KAD_ERR_INVALID, "node not in the mirrored snapshot (flush first)");
        return it->second;
    }
    uint32_t slot(const NodePtr& n) {
        added_.push_back(n);
        return (uint32_t)(added_.size() - 1);
    }

    mutable DeviceTable table_;
    std::vector<NodePtr> nodes_;
    std::unordered_map<const void*, uint32_t> index_;
    uint32_t buckets_ = 0;
    std::vector<uint8_t> first_;  // the bucket directory on the host (the host path)
    std::vector<uint32_t> off_;
    static constexpr size_t kHostAuto = ~size_t(0);
    size_t host_q_ = kHostAuto, host_count_ = 64;  // small batches take the host path (hostBatchLimit)
    std::vector<uint32_t> ops_;
    std::vector<NodePtr> added_;
    mutable std::vector<uint32_t> updated_;
    mutable int64_t now_ns_ = INT64_MIN;
    mutable bool refresh_ = false;
};

/* Device mirror of one NodeCache family map (node_cache.h:42-50: std::map<InfoHash, weak_ptr<Node>>). */
template <class NodeMapT>
class NodeCacheFamilyMirror {
public:
    using WeakPtr = typename std::decay<decltype(std::declval<const NodeMapT&>().begin()->second)>::type;
    using NodePtr = decltype(std::declval<const WeakPtr&>().lock());

    NodeCacheFamilyMirror() {}
    explicit NodeCacheFamilyMirror(const NodeMapT& m, int device = 0) { snapshot(m, device); }

    /* Snapshot: map order (ascending ID); dead weak_ptrs and expired nodes are walked over but never
     * emitted (node_cache.cpp:60-62), so both get the "expired" status bit. */
    void snapshot(const NodeMapT& m, int device = 0) {
        std::vector<uint8_t> status;
        ids_.clear();
        nodes_.clear();
        for (const auto& kv : m) {
            NodePtr n = kv.second.lock();
            ids_.insert(ids_.end(), id_bytes(kv.first), id_bytes(kv.first) + KAD_HASH_LEN);
            status.push_back(status_of(n));
            nodes_.push_back(kv.second);
        }
        table_ = DeviceTable(device, ids_, status, std::vector<uint8_t>(), std::vector<uint32_t>(), 0, true);
        reindex();
    }

    /* Bring the device copy in line with the host map after NodeMap::getNode emplaced new IDs or erased
     * dead entries, or clearBadNodes erased them (node_cache.cpp:79-115): a sorted diff of the map against
     * the mirrored IDs, then one kad_nc_apply (a device merge, no re-snapshot). An entry whose weak_ptr now
     * names another Node (getNode recreated it) or whose expiry changed gets its status patched. */
    void sync(const NodeMapT& m) {
        std::vector<uint32_t> erase, changed;
        std::vector<uint8_t> ins, ist, chst;
        std::vector<WeakPtr> added;
        size_t i = 0;
        auto it = m.begin();
        const size_t n = nodes_.size();
        while (i < n || it != m.end()) {
            const int c = i == n ? 1 : it == m.end() ? -1 : std::memcmp(&ids_[i * KAD_HASH_LEN], id_bytes(it->first), KAD_HASH_LEN);
            if (c < 0) {
                erase.push_back((uint32_t)i++);
            } else if (c > 0) {
                ins.insert(ins.end(), id_bytes(it->first), id_bytes(it->first) + KAD_HASH_LEN);
                ist.push_back(status_of(it->second.lock()));
                added.push_back(it->second);
                ++it;
            } else {
                const bool same = !nodes_[i].owner_before(it->second) && !it->second.owner_before(nodes_[i]);
                if (!same) {
                    nodes_[i] = it->second;
                    changed.push_back((uint32_t)i);
                    chst.push_back(status_of(it->second.lock()));
                }
                ++i;
                ++it;
            }
        }
        if (!changed.empty()) table_.patchStatus(changed, chst);
        if (erase.empty() && added.empty()) {
            if (!changed.empty()) reindex();
            return;
        }
        std::vector<uint32_t> remap(n ? n : 1), idx(added.empty() ? 1 : added.size());
        check(kad_nc_apply(table_.get(), erase.data(), (uint32_t)erase.size(), ins.data(), ist.data(),
                           (uint32_t)added.size(), remap.data(), idx.data()), "kad_nc_apply");
        const size_t n1 = n - erase.size() + added.size();
        std::vector<WeakPtr> next(n1);
        std::vector<uint8_t> ids1(n1 * KAD_HASH_LEN);
        for (size_t k = 0; k < n; k++)
            if (remap[k] != KAD_NO_NODE) {
                next[remap[k]] = nodes_[k];
                std::memcpy(&ids1[remap[k] * KAD_HASH_LEN], &ids_[k * KAD_HASH_LEN], KAD_HASH_LEN);
            }
        for (size_t k = 0; k < added.size(); k++) {
            next[idx[k]] = added[k];
            std::memcpy(&ids1[idx[k] * KAD_HASH_LEN], &ins[k * KAD_HASH_LEN], KAD_HASH_LEN);
        }
        nodes_.swap(next);
        ids_.swap(ids1);
        reindex();
    }

    /* NodeCache::getCachedNodes(id, af, count) for this family (node_cache.cpp:36-66). */
    template <class InfoHashT>
    std::vector<NodePtr> getCachedNodes(const InfoHashT& id, size_t count) const {
        std::vector<std::vector<NodePtr>> r = getCachedNodesBatch(&id, 1, count);
        return std::move(r[0]);
    }
    /* Batched form. A returned node found dead or expired on the host (the reference skips it without
     * counting it) is marked expired on the device and its queries re-run, so results stay exact without
     * a notification for deaths and expiries; an expired node that comes back (Node::received with a
     * reply, reset(), clearBadNodes) must be reported with nodeUpdated. */
    template <class InfoHashT>
    std::vector<std::vector<NodePtr>> getCachedNodesBatch(const InfoHashT* ids, size_t q, size_t count) const {
        std::vector<std::vector<NodePtr>> out(q);
        // any size_t count, as node_cache.h:32: a result never holds more than the map's nodes
        count = std::min(count, nodes_.size());
        if (count == 0 || q == 0) return out;
        std::vector<size_t> todo(q);
        for (size_t i = 0; i < q; i++) todo[i] = i;
        while (!todo.empty()) {
            std::vector<uint8_t> targets(todo.size() * KAD_HASH_LEN);
            for (size_t k = 0; k < todo.size(); k++)
                std::memcpy(&targets[k * KAD_HASH_LEN], id_bytes(ids[todo[k]]), KAD_HASH_LEN);
            std::vector<uint32_t> idx, stale;
            std::vector<uint8_t> cnt;
            table_.getCachedNodesBatch(targets.data(), todo.size(), count, idx, cnt);
            std::vector<size_t> again;
            for (size_t k = 0; k < todo.size(); k++) {
                std::vector<NodePtr>& o = out[todo[k]];
                o.clear();
                bool ok = true;
                size_t m = cnt[k];
                if (count > 255)  // the count byte saturates: the row's padding gives the length
                    for (m = 0; m < count && idx[k * count + m] != KAD_NO_NODE; m++) {}
                for (size_t j = 0; j < m; j++) {
                    const uint32_t x = idx[k * count + j];
                    NodePtr n = nodes_[x].lock();
                    if (!n || n->isExpired()) { stale.push_back(x); ok = false; continue; }
                    o.push_back(std::move(n));
                }
                if (!ok) again.push_back(todo[k]);
            }
            if (!stale.empty()) {
                std::sort(stale.begin(), stale.end());
                stale.erase(std::unique(stale.begin(), stale.end()), stale.end());
                table_.patchStatus(stale, std::vector<uint8_t>(stale.size(), (uint8_t)KAD_STATUS_EXPIRED));
            }
            todo.swap(again);
        }
        return out;
    }
    template <class InfoHashT>
    std::vector<std::vector<NodePtr>> getCachedNodesBatch(const std::vector<InfoHashT>& ids, size_t count) const {
        return getCachedNodesBatch(ids.data(), ids.size(), count);
    }
    /* A cached node's isExpired() changed (setExpired, Node::received with a reply, reset()). */
    void nodeUpdated(const NodePtr& n) {
        auto it = index_.find(n.get());
        if (it == index_.end()) return;  // not in this family's map
        table_.patchStatus(std::vector<uint32_t>{it->second},
                           std::vector<uint8_t>{(uint8_t)(n->isExpired() ? KAD_STATUS_EXPIRED : 0u)});
    }
    size_t size() const { return nodes_.size(); }

private:
    static uint8_t status_of(const NodePtr& n) {
        return (uint8_t)((!n || n->isExpired()) ? KAD_STATUS_EXPIRED : 0u);
    }
    void reindex() {
        index_.clear();
        for (size_t i = 0; i < nodes_.size(); i++)
            if (NodePtr n = nodes_[i].lock()) index_[n.get()] = (uint32_t)i;
    }

    mutable DeviceTable table_;
    std::vector<uint8_t> ids_;  // the mirrored map's keys, in map order
    std::vector<WeakPtr> nodes_;
    std::unordered_map<const void*, uint32_t> index_;
};

/* Device mirror of a whole NodeCache (cache_4 and cache_6, node_cache.h:49-50). */
template <class NodeMapT>
class NodeCacheMirror {
public:
    using NodePtr = typename NodeCacheFamilyMirror<NodeMapT>::NodePtr;

    void snapshot(const NodeMapT& cache4, const NodeMapT& cache6, int device = 0) {
        v4_.snapshot(cache4, device);
        v6_.snapshot(cache6, device);
    }
    /* NodeCache::getCachedNodes(const InfoHash&, sa_family_t, size_t) (node_cache.h:32, node_cache.cpp:36-66). */
    template <class InfoHashT>
    std::vector<NodePtr> getCachedNodes(const InfoHashT& id, sa_family_t sa_f, size_t count) const {
        return family(sa_f).getCachedNodes(id, count);
    }
    void nodeUpdated(const NodePtr& n) {
        v4_.nodeUpdated(n);
        v6_.nodeUpdated(n);
    }
    /* After NodeCache::getNode / clearBadNodes changed the maps (inserted or erased entries). */
    void sync(const NodeMapT& cache4, const NodeMapT& cache6) {
        v4_.sync(cache4);
        v6_.sync(cache6);
    }
    const NodeCacheFamilyMirror<NodeMapT>& family(sa_family_t sa_f) const { return sa_f == AF_INET ? v4_ : v6_; }
    NodeCacheFamilyMirror<NodeMapT>& family(sa_family_t sa_f) { return sa_f == AF_INET ? v4_ : v6_; }

private:
    NodeCacheFamilyMirror<NodeMapT> v4_, v6_;
};

/* Dht-level accessor over both families: findClosestNodes(id, af, count)
 * = buckets(af).findClosestNodes(id, scheduler.time(), count) (dht.h:437-438; call sites dht.cpp:3196-3217).
 * `now` comes from the mirror's clock: steady_clock::now() by default, or the Dht scheduler's time
 * (setClock([&]{ return scheduler.time(); })). */
template <class RoutingTableT, class Clock = std::chrono::steady_clock>
class DhtMirror {
public:
    using NodePtr = typename RoutingTableMirror<RoutingTableT>::NodePtr;
    using time_point = typename Clock::time_point;

    DhtMirror() : clock_([] { return Clock::now(); }) {}

    void snapshot(const RoutingTableT& buckets4, const RoutingTableT& buckets6, time_point now, int device = 0) {
        v4_.snapshot(buckets4, now, device);
        v6_.snapshot(buckets6, now, device);
    }
    void setClock(std::function<time_point()> clock) { clock_ = std::move(clock); }

    template <class InfoHashT>
    std::vector<NodePtr> findClosestNodes(const InfoHashT& id, sa_family_t af, size_t count = KAD_TARGET_NODES) const {
        return buckets(af).findClosestNodes(id, clock_(), count);
    }
    /* Dht::buckets(af) (dht.h:437-438) */
    const RoutingTableMirror<RoutingTableT>& buckets(sa_family_t af) const { return af == AF_INET ? v4_ : v6_; }
    RoutingTableMirror<RoutingTableT>& buckets(sa_family_t af) { return af == AF_INET ? v4_ : v6_; }

private:
    RoutingTableMirror<RoutingTableT> v4_, v6_;
    std::function<time_point()> clock_;
};

}  // namespace kadgpu

#endif /* KADGPU_HPP */
