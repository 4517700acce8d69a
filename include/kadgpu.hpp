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
 * A mirror is a snapshot of the table at `now` (the status byte of every node is Node::isGood(now)
 * / isExpired() evaluated once, on the host thread that owns the table, as the reference does on its
 * dht thread). Results come back as the same shared_ptr<NodeT> objects the table holds, in the
 * reference's order. After table mutations (Dht::onNewNode / expireBuckets / split), either
 * re-snapshot or record them on the mirror (nodeRemoved / nodeReplaced / nodeAdded / bucketSplit)
 * and flush(now): kad_table_apply replays them on the device copy.
 */
#ifndef KADGPU_HPP
#define KADGPU_HPP

#include <algorithm>
#include <cstdint>
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

private:
    kad_table* t_ = nullptr;
};

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

    /* Snapshot `rt` at `now`: nodes grouped by bucket in list order, status = isGood(now) | isExpired()<<1. */
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
                status.push_back((uint8_t)((n->isGood(now) ? KAD_STATUS_GOOD : 0u) |
                                           (n->isExpired() ? KAD_STATUS_EXPIRED : 0u)));
            }
        }
        off.push_back((uint32_t)nodes_.size());
        buckets_ = (uint32_t)(off.size() - 1);
        table_ = DeviceTable(device, ids, status, first, off);
    }

    /* RoutingTable::findClosestNodes(id, now, count) at the snapshot's `now` (routing_table.cpp:67-111). */
    template <class InfoHashT>
    std::vector<NodePtr> findClosestNodes(const InfoHashT& id, size_t count = KAD_TARGET_NODES) const {
        std::vector<std::vector<NodePtr>> r = findClosestNodesBatch(&id, 1, count);
        return std::move(r[0]);
    }

    /* Batched form: one result vector per target. */
    template <class InfoHashT>
    std::vector<std::vector<NodePtr>> findClosestNodesBatch(const InfoHashT* ids, size_t q,
                                                            size_t count = KAD_TARGET_NODES) const {
        std::vector<uint8_t> targets(q * KAD_HASH_LEN);
        for (size_t i = 0; i < q; i++) std::memcpy(&targets[i * KAD_HASH_LEN], id_bytes(ids[i]), KAD_HASH_LEN);
        std::vector<uint32_t> idx;
        std::vector<uint8_t> cnt;
        table_.findClosestNodesBatch(targets.data(), q, count, idx, cnt);
        std::vector<std::vector<NodePtr>> out(q);
        for (size_t i = 0; i < q; i++) {
            out[i].reserve(cnt[i]);
            for (size_t j = 0; j < cnt[i]; j++) out[i].push_back(nodes_[idx[i * count + j]]);
        }
        return out;
    }
    template <class InfoHashT>
    std::vector<std::vector<NodePtr>> findClosestNodesBatch(const std::vector<InfoHashT>& ids,
                                                            size_t count = KAD_TARGET_NODES) const {
        return findClosestNodesBatch(ids.data(), ids.size(), count);
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
            status.push_back((uint8_t)((n->isGood(now) ? KAD_STATUS_GOOD : 0u) | (n->isExpired() ? KAD_STATUS_EXPIRED : 0u)));
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
        ops_.clear();
        added_.clear();
    }

    size_t bucketCount() const { return buckets_; }
    size_t nodeCount() const { return nodes_.size(); }
    const DeviceTable& table() const { return table_; }

private:
    void op(uint32_t kind, uint32_t a, uint32_t b) {
        ops_.push_back(kind);
        ops_.push_back(a);
        ops_.push_back(b);
    }
    uint32_t index_of(const NodePtr& n) const {
        auto it = std::find(nodes_.begin(), nodes_.end(), n);
        if (it == nodes_.end()) throw Error(KAD_ERR_INVALID, "node not in the mirrored snapshot (flush first)");
        return (uint32_t)(it - nodes_.begin());
    }
    uint32_t slot(const NodePtr& n) {
        added_.push_back(n);
        return (uint32_t)(added_.size() - 1);
    }

    DeviceTable table_;
    std::vector<NodePtr> nodes_;
    uint32_t buckets_ = 0;
    std::vector<uint32_t> ops_;
    std::vector<NodePtr> added_;
};

/* Device mirror of one NodeCache family map (node_cache.h:42-50). */
template <class NodeMapT>
class NodeCacheMirror {
public:
    using NodePtr = decltype(std::declval<const NodeMapT&>().begin()->second.lock());

    NodeCacheMirror() {}
    explicit NodeCacheMirror(const NodeMapT& m, int device = 0) { snapshot(m, device); }

    /* Snapshot: map order (ascending ID); dead weak_ptrs and expired nodes are walked over but never
     * emitted (node_cache.cpp:60-62), so both get the "expired" status bit. */
    void snapshot(const NodeMapT& m, int device = 0) {
        std::vector<uint8_t> ids, status;
        nodes_.clear();
        for (const auto& kv : m) {
            NodePtr n = kv.second.lock();
            ids.insert(ids.end(), id_bytes(kv.first), id_bytes(kv.first) + KAD_HASH_LEN);
            status.push_back((uint8_t)((!n || n->isExpired()) ? KAD_STATUS_EXPIRED : 0u));
            nodes_.push_back(n);
        }
        table_ = DeviceTable(device, ids, status, std::vector<uint8_t>(), std::vector<uint32_t>(), 0, true);
    }

    /* NodeCache::getCachedNodes(id, af, count) for this family (node_cache.cpp:36-66). */
    template <class InfoHashT>
    std::vector<NodePtr> getCachedNodes(const InfoHashT& id, size_t count) const {
        std::vector<uint32_t> idx;
        std::vector<uint8_t> cnt;
        table_.getCachedNodesBatch(id_bytes(id), 1, count, idx, cnt);
        std::vector<NodePtr> out;
        for (size_t j = 0; j < cnt[0]; j++) out.push_back(nodes_[idx[j]]);
        return out;
    }
    template <class InfoHashT>
    std::vector<std::vector<NodePtr>> getCachedNodesBatch(const std::vector<InfoHashT>& ids, size_t count) const {
        const size_t q = ids.size();
        std::vector<uint8_t> targets(q * KAD_HASH_LEN);
        for (size_t i = 0; i < q; i++) std::memcpy(&targets[i * KAD_HASH_LEN], id_bytes(ids[i]), KAD_HASH_LEN);
        std::vector<uint32_t> idx;
        std::vector<uint8_t> cnt;
        table_.getCachedNodesBatch(targets.data(), q, count, idx, cnt);
        std::vector<std::vector<NodePtr>> out(q);
        for (size_t i = 0; i < q; i++)
            for (size_t j = 0; j < cnt[i]; j++) out[i].push_back(nodes_[idx[i * count + j]]);
        return out;
    }

private:
    DeviceTable table_;
    std::vector<NodePtr> nodes_;
};

/* Dht-level accessor over both families: findClosestNodes(id, af, count)
 * = buckets(af).findClosestNodes(id, now, count) (dht.h:437-438; call sites dht.cpp:3196-3217). */
template <class RoutingTableT>
class DhtMirror {
public:
    using NodePtr = typename RoutingTableMirror<RoutingTableT>::NodePtr;

    template <class TimePoint>
    void snapshot(const RoutingTableT& buckets4, const RoutingTableT& buckets6, TimePoint now, int device = 0) {
        v4_.snapshot(buckets4, now, device);
        v6_.snapshot(buckets6, now, device);
    }
    /* af: the caller's AF_INET / AF_INET6 values (passed in so this header needs no socket headers). */
    template <class InfoHashT>
    std::vector<NodePtr> findClosestNodes(const InfoHashT& id, int af, size_t count, int af_inet) const {
        return (af == af_inet ? v4_ : v6_).findClosestNodes(id, count);
    }
    const RoutingTableMirror<RoutingTableT>& family4() const { return v4_; }
    const RoutingTableMirror<RoutingTableT>& family6() const { return v6_; }

private:
    RoutingTableMirror<RoutingTableT> v4_, v6_;
};

}  // namespace kadgpu

#endif /* KADGPU_HPP */
