/*
 * kadgpu.h — C ABI of the MI355X-native batched Kademlia closest-node engine.
 *
 * This is the drop-in boundary for OpenDHT's XOR-distance lookup path. The
 * reference exposes no C API/FFI for this path: its interface
 * is the C++ member
 *     std::vector<std::shared_ptr<Node>>
 *     RoutingTable::findClosestNodes(const InfoHash id, time_point now,
 *                                    size_t count) const
 *         (reference: include/opendht/routing_table.h:48, src/routing_table.cpp:67-111)
 *     RoutingTable::findBucket(const InfoHash&)
 *         (reference: include/opendht/routing_table.h:50-51, src/routing_table.cpp:113-135)
 *     std::vector<std::shared_ptr<Node>>
 *     NodeCache::getCachedNodes(const InfoHash&, sa_family_t, size_t)
 *         (reference: include/opendht/node_cache.h:32, src/node_cache.cpp:36-66)
 * and the InfoHash primitives (include/opendht/infohash.h:84-162).
 *
 * Every entry point below replaces one of those; each cites the reference
 * interface it stands in for. The C++11 shim in kadgpu.hpp wraps these with
 * the reference's own signatures (RoutingTable::findClosestNodes, the new
 * Dht-style findClosestNodes(id, af, count) accessor, NodeCache::getCachedNodes).
 *
 * Conventions
 *  - IDs cross the ABI as raw InfoHash bytes: 20 bytes per ID, byte 0 most
 *    significant (InfoHash::data() layout, reference infohash.h:58).
 *  - A table is a snapshot of one address family's RoutingTable (and/or its
 *    NodeCache map) at a chosen `now`: a flat node array grouped by bucket,
 *    a bucket directory, and one status byte per node (bit0 = Node::isGood(now),
 *    bit1 = Node::isExpired(); reference src/node.cpp:34-40, node.h:67).
 *  - Results are uint32 node indices into the snapshot's node array plus
 *    `index_base` (so shards can return global indices), padded with
 *    KAD_NO_NODE beyond the per-query result count.
 *  - Every function returns an int status (KAD_OK = 0, negative on error);
 *    kad_last_error() gives a thread-local message. No C++ exception crosses
 *    this ABI. Empty table -> zero results (reference routing_table.cpp:73).
 *  - `*_batch` entry points take DEVICE pointers and enqueue on `stream`
 *    (a hipStream_t, NULL = default stream); they do not synchronise.
 *    `*_batch_host` entry points take HOST pointers and are synchronous
 *    (H2D, kernel, D2H on an internal stream).
 *  - A table handle is not safe for concurrent mutation; concurrent const
 *    queries on distinct streams are safe (as in the reference, where
 *    findClosestNodes is const: SURVEY.md §8b "Threading").
 */
#ifndef KADGPU_H
#define KADGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define KAD_HASH_LEN 20u            /* reference infohash.h:49 HASH_LEN */
#define KAD_TARGET_NODES 8u         /* reference routing_table.h:26 TARGET_NODES */
#define KAD_SEARCH_NODES 14u        /* reference dht.h:314 SEARCH_NODES */
#define KAD_MAX_COUNT 32u           /* largest `count` of the line kernels; RoutingTable queries take any
                                       count (larger ones run one wave per query); the shard / wire
                                       entry points stay at <= KAD_MAX_COUNT */
#define KAD_NO_NODE 0xFFFFFFFFu     /* padding index in result rows */

/* status byte bits (snapshot of Node state at `now`) */
#define KAD_STATUS_GOOD 0x01u       /* Node::isGood(now)   reference node.cpp:34-40 */
#define KAD_STATUS_EXPIRED 0x02u    /* Node::isExpired()   reference node.h:67       */

/* kad_table_create flags */
#define KAD_TABLE_SORTED 0x01u      /* node array ascending by ID (enables NodeCache queries) */
#define KAD_TABLE_EAGER 0x02u       /* build every line set at creation (default: those of count <= 8 RoutingTable
                                       queries; the others on first use, kad_table_prepare) */
#define KAD_TABLE_NO_SLOT_LINES 0x04u /* general-line tables: no slot lines (count <= 8 / 9..16 queries locate
                                         their bucket and read its general line; a status refresh then rebuilds
                                         the count <= 8 general lines in its one fused launch) */

/* line sets built on first use (kad_table_prepare, kad_table_line_sets) */
#define KAD_LINES_RT16 0x01u        /* RoutingTable counts 9..16 (brings KAD_LINES_RT32, their fallback) */
#define KAD_LINES_RT32 0x02u        /* RoutingTable counts 17..32 */
#define KAD_LINES_NC16 0x04u        /* NodeCache counts 1..16 */
#define KAD_LINES_NC32 0x08u        /* NodeCache counts 17..32 (brings KAD_LINES_NC16) */
#define KAD_LINES_ALL 0x0Fu
/* kad_table_info.flags, reported only */
#define KAD_INFO_WINDOW_LINES 0x100u /* uniform-depth table: count <= 8 queries use one 128-byte
                                        window line per query (rt_wl_kernel) */
#define KAD_INFO_GENERAL_LINES 0x200u /* any other bucket shape: count <= 8 queries use one 128-byte
                                         general window line per query (rt_gl_kernel) */
#define KAD_INFO_GENERAL_LINES32 0x400u /* ... and counts 9..32 one 256-byte line (rt_gl32_kernel) */
#define KAD_INFO_GENERAL_LINES16 0x4000u /* ... and counts 9..16 one 128-byte line (rt_gl16_kernel) */
#define KAD_INFO_SLOT_LINES16 0x8000u /* ... read through a 128-byte copy indexed by the target's top bits (rt_sl16_kernel) */
#define KAD_INFO_SLOT_LINES 0x2000u /* other bucket shapes: count <= 8 queries read one 64-byte line indexed by
                                       the target's top bits (rt_sl_kernel), the locate + 128-byte line only
                                       as fallback */
#define KAD_INFO_NODECACHE_LINES32 0x1000u /* sorted table: NodeCache counts 17..32 read one 384-byte line
                                             per query, 8 lanes per query (nc32_line_kernel) */
#define KAD_INFO_SHORT_LINES 0x800u /* uniform-depth table: count <= 8 queries read one 64-byte short
                                       window line (rt_ws_kernel), the 128-byte line only as fallback */

/* error codes */
#define KAD_OK 0
#define KAD_ERR_INVALID -1          /* bad argument / shape */
#define KAD_ERR_HIP -2              /* HIP runtime error */
#define KAD_ERR_NOMEM -3            /* device allocation failed */
#define KAD_ERR_UNSUPPORTED -4      /* e.g. count > KAD_MAX_COUNT */
#define KAD_ERR_NOT_SORTED -5       /* NodeCache query on a table without KAD_TABLE_SORTED */
#define KAD_ERR_NO_DEVICE -6        /* no usable gfx950 device */

typedef struct kad_table kad_table;

typedef struct kad_table_info {
    uint32_t n_nodes;
    uint32_t n_buckets;
    uint32_t index_base;
    uint32_t flags;
    int32_t device;
    uint32_t rt_radix_bits;         /* log2 of the bucket-locate radix table size */
    uint32_t nc_radix_bits;         /* log2 of the NodeCache lower_bound radix table size (0 if unsorted) */
    uint32_t n_good;                /* good nodes under the current status snapshot */
    uint64_t device_bytes;          /* HBM held by the table */
} kad_table_info;

/* ---- library ---------------------------------------------------------- */
const char* kad_last_error(void);
int kad_version(void);                                  /* 10000*major + 100*minor + patch */
int kad_device_count(int* out_n);                       /* gfx950 devices visible */

/* ---- table lifetime ----------------------------------------------------- */
/* Snapshot a RoutingTable (reference routing_table.h:28-79) and/or NodeCache map
 * (node_cache.h:42-50) into device memory.
 *   ids           host, n_nodes x 20 bytes; bucket b owns [bucket_offset[b], bucket_offset[b+1])
 *                 (RoutingTable list order inside a bucket; ties between equal IDs resolve by index)
 *   status        host, n_nodes status bytes (KAD_STATUS_*)
 *   bucket_first  host, n_buckets x 20 bytes, ascending (Bucket::first, routing_table.h:33)
 *   bucket_offset host, n_buckets+1 offsets, bucket_offset[0]=0, bucket_offset[n_buckets]=n_nodes
 *   n_buckets = 0 builds a NodeCache-only table (requires KAD_TABLE_SORTED).
 *   flags         KAD_TABLE_SORTED if ids are strictly ascending (checked) */
int kad_table_create(kad_table** out, int device,
                     uint32_t n_nodes, const uint8_t* ids, const uint8_t* status,
                     uint32_t n_buckets, const uint8_t* bucket_first, const uint32_t* bucket_offset,
                     uint32_t index_base, uint32_t flags);
int kad_table_destroy(kad_table* t);
int kad_table_get_info(const kad_table* t, kad_table_info* out);
/* Build the line sets `sets` (KAD_LINES_*) now, if not yet: a query builds the set it needs on first use
 * (synchronising the device once, and never inside a stream capture, where it answers on its slower exact
 * path instead), so a caller about to capture a HIP graph prepares them first. Synchronous. */
int kad_table_prepare(kad_table* t, uint32_t sets);
/* Which line sets are built (KAD_LINES_* mask), and per set in bit order (RT16, RT32, NC16, NC32) the HBM
 * bytes and the build time in ms of its first build (any output may be NULL). */
int kad_table_line_sets(const kad_table* t, uint32_t* built, uint64_t* bytes, float* build_ms);

/* Replace the status snapshot (host bytes, n_nodes). Synchronous. Incremental: only the buckets whose
 * good set changed get new masks and good counts, and only the window / NodeCache lines whose window reaches
 * a changed node are rebuilt. */
int kad_table_update_status(kad_table* t, const uint8_t* status);
/* Incremental status update for a changed-node list (reference: the isGood/isExpired flips that
 * Node::received / setExpired cause, node.cpp:82-108; network_engine.cpp:245): node nodes[j] gets
 * status[j] (host arrays, m entries; nodes == NULL means all n_nodes in order). Rebuilds only what
 * the flips touch, as kad_table_update_status. Synchronous. */
int kad_table_patch_status(kad_table* t, uint32_t m, const uint32_t* nodes, const uint8_t* status);

/* Upload Node liveness (reference node.h:39-40,105: time, reply_time, expired_)
 * as int64 nanoseconds of steady_clock + expired flag bytes; host arrays, n_nodes each.
 * INT64_MIN encodes time_point::min(). Synchronous. */
int kad_table_set_times(kad_table* t, const int64_t* time_ns, const int64_t* reply_time_ns,
                        const uint8_t* expired);
/* Update the uploaded liveness of m listed nodes (Node::received / setExpired on the host: node.cpp:82-108):
 * host arrays of m entries. Takes effect at the next kad_table_refresh_status. Synchronous. */
int kad_table_patch_times(kad_table* t, uint32_t m, const uint32_t* nodes, const int64_t* time_ns,
                          const int64_t* reply_time_ns, const uint8_t* expired);
/* Recompute the status snapshot on the device at `now_ns` from the uploaded times:
 * good = !expired && reply_time >= now-120min && time >= now-10min (node.cpp:34-40,
 * node.h:91-94). A good node stays good while now <= min(time + 10 min, reply_time + 120 min), so the
 * table keeps every node's deadline sorted: the first refresh after kad_table_set_times (or after a
 * direct status change, or with `now` earlier than the last refresh's) re-derives every node and sorts
 * the deadlines; later ones re-derive only the nodes whose deadline `now` passed since the last refresh
 * and the nodes patched by kad_table_patch_times, and a refresh whose `now` has not reached the next
 * deadline (with nothing patched) returns at once without touching the GPU. The host keeps a copy of the
 * sorted deadlines (8 bytes per node) and finds the passed ones itself. Up to 2,048 such nodes take the
 * small path: one kernel re-derives them and lists the changed buckets and the lines whose windows reach
 * them, then the line builders rebuild only those (no pass over the buckets or the lines); up to 128 of them
 * on a table with window lines are one launch in all (block 0 re-derives the nodes, the other blocks rebuild
 * the count <= 8 lines at the same time, the host having found the nodes' buckets and the lines). More take
 * the flag-and-compact path. Async on `stream` (the first refresh after set_times waits for the sort);
 * later refreshes and device batches must be ordered after it by the caller (the host-pointer batches
 * order themselves). A refresh that changes anything ends the table's resident query service launch
 * (kad_table_serve) first. */
int kad_table_refresh_status(kad_table* t, int64_t now_ns, void* stream);
/* Counters of the small refresh since the table was created (synchronises the device):
 *   spin_timeouts     builder blocks of a fused general-line refresh that waited RF_SPIN_TICKS (1 s) for the
 *                     line list block 0 publishes and gave up (block 0 not running: the GPU busy with other
 *                     work); their lines were then built by the launch's last block, so results stay exact. After
 *                     the first timeout the table stops fusing those builds (they go out as stream-ordered
 *                     launches after the node kernel), so the wait cannot recur
 *   last_block_lines  lines built by a fused launch's last block (windows of more than 64 nodes, and the lists
 *                     of timed-out builders)
 *   guard_errors      bounds guards of the kernel that fired (bit mask; the host validates every inline
 *                     argument before a launch, so this is 0 unless the engine has a bug) */
typedef struct kad_refresh_diag {
    uint32_t spin_timeouts;
    uint32_t last_block_lines;
    uint32_t guard_errors;
} kad_refresh_diag;
int kad_table_refresh_diag(const kad_table* t, kad_refresh_diag* out);

/* ---- incremental device mirror ----------------------
 * Replays the table mutations of a live Dht on the device instead of re-snapshotting. Ops are rows
 * of three uint32 (kind, a, b) applied in order; `a` names a node by its index at the start of
 * the batch, `b` / `a` of INSERT a slot of the batch's new nodes (new_ids / new_status, host):
 *   KAD_OP_REMOVE  a     node a leaves its bucket (Dht::expireBuckets, dht.cpp:942-956)
 *   KAD_OP_REPLACE a b   new node b takes node a's place (onNewNode's expired slot, dht.cpp:917-921);
 *                        b must belong to a's bucket (findBucket(id_b)), else KAD_ERR_INVALID
 *   KAD_OP_INSERT  a     new node a is emplace_front'ed into findBucket(id) (dht.cpp:934)
 *   KAD_OP_SPLIT   a     RoutingTable::split of the bucket at current index a (routing_table.cpp:137-163;
 *                        nodes re-spliced to the front of their new bucket: list order reverses)
 * The node arrays are re-laid out on the device (one gather over the plan's segments); masks,
 * prefix sums, dup masks and window lines are re-derived there (a split turns window lines off).
 * Outputs: remap (host or device, old n entries, may be NULL) = new index of every old node, KAD_NO_NODE
 * if removed or replaced; new_index (host, n_new, may be NULL) = index of every new node,
 * KAD_NO_NODE if unused. Any op clears KAD_TABLE_SORTED (NodeCache queries need a new snapshot);
 * wire records and node times must be set again. Synchronous. */
#define KAD_OP_REMOVE 1u
#define KAD_OP_REPLACE 2u
#define KAD_OP_INSERT 3u
#define KAD_OP_SPLIT 4u
int kad_table_apply(kad_table* t, const uint32_t* ops, uint32_t n_ops, const uint8_t* new_ids,
                    const uint8_t* new_status, uint32_t n_new, uint32_t* remap, uint32_t* new_index);
/* NodeCache map mutations (node_cache.cpp:91-115) on a NodeCache-only table (n_buckets = 0,
 * KAD_TABLE_SORTED), without a re-snapshot: erase the n_erase listed nodes (indices at the call, each at
 * most once: NodeMap::getNode(id) erasing a dead weak_ptr, clearBadNodes' erase of dead entries), then
 * insert n_ins new IDs (host, any order, none already a kept key: NodeMap::getNode(id, addr, now, confirm)'s
 * emplace) with their status bytes. The node array is merged on the device and stays sorted; the NodeCache
 * radix and lines are re-derived there. remap (host, old n entries, may be NULL): new index of every old
 * node, KAD_NO_NODE if erased; new_index (host, n_ins, may be NULL): index of every new node. Node times and
 * wire records must be set again. Failure leaves the table unchanged. Synchronous. */
int kad_nc_apply(kad_table* t, const uint32_t* erase, uint32_t n_erase, const uint8_t* ins_ids,
                 const uint8_t* ins_status, uint32_t n_ins, uint32_t* remap, uint32_t* new_index);
/* The table as host arrays (any may be NULL): ids n x 20 and status in bucket/list order, bucket
 * firsts B x 20 and offsets B+1 (sizes from kad_table_get_info). */
int kad_table_export(const kad_table* t, uint8_t* ids, uint8_t* status, uint8_t* bucket_first,
                     uint32_t* bucket_offset);
/* A derived array of the table as raw bytes (tests: an incrementally maintained set must equal the one a fresh
 * table builds from the same status). out == NULL: *bytes = the size (0 if the table has no such set). */
#define KAD_LINESET_WL 0u     /* 128-byte window lines (count <= 8) */
#define KAD_LINESET_WS 1u     /* 64-byte short window lines */
#define KAD_LINESET_WL16 2u
#define KAD_LINESET_WL32 3u
#define KAD_LINESET_GL 4u     /* general lines */
#define KAD_LINESET_GL16 5u
#define KAD_LINESET_GL32 6u
#define KAD_LINESET_SL 7u     /* slot lines */
#define KAD_LINESET_SL16 8u
#define KAD_LINESET_NCL 9u    /* NodeCache lines */
#define KAD_LINESET_NCL32 10u
#define KAD_LINESET_GCNT 11u  /* per-bucket good counts */
#define KAD_LINESET_DIR 12u   /* bucket directory: first node (bit 31: wide), good mask */
int kad_table_export_lines(const kad_table* t, uint32_t set, void* out, uint64_t* bytes);

/* ---- queries: RoutingTable::findClosestNodes ---------------------------- */
/* Batched RoutingTable::findClosestNodes(target, now, count) (routing_table.cpp:67-111)
 * on the table's status snapshot. Device pointers:
 *   targets  q x 20 bytes; out_idx q x count uint32; out_cnt q uint8 (may be NULL).
 * Row i of out_idx holds the result in the reference's order (ascending XOR
 * distance), out_cnt[i] entries, padded with KAD_NO_NODE. Any count, as the reference's
 * size_t count (routing_table.h:48): counts up to KAD_MAX_COUNT run the line kernels, larger
 * ones one wave per query; out_cnt saturates at 255 (for count > 255 the result length is the
 * row's entries before the first KAD_NO_NODE). */
int kad_rt_closest_batch(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count,
                         uint32_t* out_idx, uint8_t* out_cnt, void* stream);
/* The same on host buffers (any memory), synchronous, and ordered after every change made to the table
 * before the call (the asynchronous kad_table_refresh_status on whatever stream it ran; every other change
 * is synchronous). Batches of up to 1024 queries with count <= 64 are one kernel launch that reads the
 * targets from and writes the rows to mapped pinned memory (one round trip); larger ones run as 64k-query
 * chunks pipelined over four host threads through ~80 MB of pinned staging and device buffers the table
 * keeps (allocated on first use, freed with it). One host batch per table at a time.
 * count <= 2,097,152 (one chunk row; larger counts: the device-pointer batch). */
int kad_rt_closest_batch_host(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count,
                              uint32_t* out_idx, uint8_t* out_cnt);

/* Resident query service for single requests (the per-request calls of dht.cpp:3196-3217, 1650): with
 * idle_us > 0 one workgroup stays on the GPU and answers host batches of up to KAD_SERVE_MAX_Q queries with
 * count <= KAD_SERVE_MAX_COUNT (kad_rt_closest_batch_host, kad_nc_closest_batch_host) from a mailbox in
 * pinned host memory: no kernel launch and no stream synchronise per call. Same results, same ordering
 * (after the table's last asynchronous status refresh). A launch ends by itself after idle_us without a
 * request or after 50 ms in all, and the next request launches it again. Calls that change or free what
 * it reads (patch/update_status, patch/set_times, a refresh_status that changes anything, apply, nc_apply,
 * set_addrs, prepare, destroy) end it first. While it runs it holds one CU, and:
 *   - device-wide synchronisation (hipDeviceSynchronize, torch.cuda.synchronize) waits for it to go idle
 *     (up to idle_us after the last request, or the rest of its 50 ms life);
 *   - HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default): work queued on a stream that
 *     shares the service's queue waits behind the resident launch the same way. With more than four
 *     streams in the process, keep idle_us short (a few hundred microseconds) or call kad_table_serve(t, 0)
 *     before long device work.
 * idle_us = 0 ends it and turns it off (the default). idle_us <= KAD_SERVE_MAX_IDLE_US. */
#define KAD_SERVE_MAX_Q 64
#define KAD_SERVE_MAX_COUNT 64
#define KAD_SERVE_MAX_IDLE_US 1000000
int kad_table_serve(kad_table* t, uint32_t idle_us);
/* The service's counters: launches so far (the first request after an idle exit launches again), requests
 * answered, and for the last request the header reads it took to be seen and the device time from seen to
 * its rows fenced (the rest of a call's latency is the PCIe round trip and the host). */
typedef struct kad_serve_stats {
    uint32_t idle_us;
    uint32_t last_polls;
    uint64_t launches;
    uint64_t requests;
    uint64_t last_busy_ns;
} kad_serve_stats;
int kad_table_serve_stats(const kad_table* t, kad_serve_stats* out);

/* Batched RoutingTable::findBucket (routing_table.cpp:113-135): bucket index per
 * target (0 for targets below the first bucket, as the reference's list walk). */
int kad_rt_find_bucket_batch(const kad_table* t, const uint8_t* targets, uint32_t q,
                             uint32_t* out_bucket, void* stream);

/* ---- queries: NodeCache::getCachedNodes --------------------------------- */
/* Batched NodeCache::getCachedNodes(target, af, count) (node_cache.cpp:36-66) over
 * one family's map, snapshotted as a KAD_TABLE_SORTED table. Emits non-expired
 * nodes in the reference's two-pointer walk order (NOT sorted by distance). Any count, as the
 * reference's size_t count (node_cache.h:32): counts up to 16 / 32 run the NodeCache line kernels,
 * 33..64 one wave per query, larger ones the serial walk (a lane per query); out_cnt saturates at 255
 * (for count > 255 the result length is the row's entries before the first KAD_NO_NODE). */
int kad_nc_closest_batch(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count,
                         uint32_t* out_idx, uint8_t* out_cnt, void* stream);
int kad_nc_closest_batch_host(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count,
                              uint32_t* out_idx, uint8_t* out_cnt);

/* ---- dual-family batch (Dht::onGetValues asks both tables, dht.cpp:3216-3217) ---- */
/* Per-query family select: af[i] = 0 -> table4, 1 -> table6 (either may be NULL
 * if no query selects it). Device pointers. */
int kad_rt_closest_batch_dual(const kad_table* table4, const kad_table* table6,
                              const uint8_t* targets, const uint8_t* af, uint32_t q, uint32_t count,
                              uint32_t* out_idx, uint8_t* out_cnt, void* stream);

/* Per-query family select for NodeCache::getCachedNodes(id, sa_family, count) (node_cache.cpp:36-66:
 * cache_4 or cache_6 by family; Dht::refill asks the search's family, dht.cpp:1650): af[i] = 0 -> table4,
 * 1 -> table6 (KAD_TABLE_SORTED tables; either may be NULL = an empty map). Any count (as kad_nc_closest_batch).
 * Device pointers. */
int kad_nc_closest_batch_dual(const kad_table* table4, const kad_table* table6,
                              const uint8_t* targets, const uint8_t* af, uint32_t q, uint32_t count,
                              uint32_t* out_idx, uint8_t* out_cnt, void* stream);

/* ---- sharded table without halo: the north-star multi-GPU variant ----
 * A global uniform-depth table U(depth) (bucket b's first ID = global_base + b << (160-depth)) is
 * cut into contiguous bucket ranges, one table per GPU, with global node indices (index_base).
 * Every rank holds the global good prefix sums, computes each query's global window W(R)
 * (routing_table.cpp:89-104) and answers W(R) ∩ its shard for a replicated batch of targets:
 *   W(R) inside the shard -> a final row appended to one of KAD_SHARD_REGIONS regions of `rows`
 *                            (region r: row_cap rows at rows + r*row_cap*KAD_ROW_WORDS(count);
 *                            a row is qid, m, 0, 0, idx[count] padded to 4 words)
 *   W(R) crosses an edge  -> this shard's part appended to `parts` (KAD_PART_WORDS(count) each:
 *                            the row, then the entries' 160-bit XOR distances, 5 words each)
 *   W(R) misses the shard -> nothing (queries with a bucket outside [reach_lo, reach_hi) exit early;
 *                            reach must cover every bucket whose window can touch the shard).
 * counters (device, KAD_SHARD_COUNTERS x KAD_SHARD_COUNTER_STRIDE uint32, zeroed by the caller;
 * counter k at word k*KAD_SHARD_COUNTER_STRIDE): rows appended per region (k < 8), parts appended
 * (k = 8), overflow flag (k = 9: a region or the parts buffer was full: grow and run again).
 * Rows of the queries [QB w, QB w + QB) go to region w % 8 (QB = 1024, or 256 for counts 17..32; 2048 in a
 * tools-build A/B). A query takes at most two rows: a query whose window line cannot answer it leaves a tombstone row (qid
 * KAD_NO_NODE, skipped by every finish) beside its wave-path row or part, so row_cap >= 2*ceil(ceil(q/QB)/8)*QB
 * never overflows (home layout: W = ceil(ceil(q/256)/world/(QB/256)) + 1 workgroups per home range,
 * row_cap >= 2*ceil(W/8)*QB).
 * The ranks' rows and parts are all-gathered by the caller (RCCL); kad_rt_scatter_rows and
 * kad_rt_merge_parts (parts sorted by qid) then give every query's findClosestNodes result.
 * All pointers are device pointers; count in 1..KAD_MAX_COUNT. Queries far enough inside the shard
 * answer from the window lines of their count (counts 9..32: the 16/32-count sets, built on first
 * use as for kad_rt_closest_batch; kad_table_prepare builds them ahead of a stream capture). */
#define KAD_ROW_WORDS(count) (4u + (((count) + 3u) & ~3u))
#define KAD_PART_WORDS(count) (KAD_ROW_WORDS(count) + 5u * (count))
#define KAD_SHARD_REGIONS 8u
#define KAD_SHARD_COUNTERS 10u
#define KAD_SHARD_COUNTER_STRIDE 32u
int kad_rt_shard_batch(const kad_table* shard, const uint32_t* global_good_prefix, uint32_t global_buckets,
                       uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket,
                       uint32_t reach_lo, uint32_t reach_hi, const uint8_t* targets, uint32_t q,
                       uint32_t count, uint32_t* rows, uint32_t row_cap, uint32_t* parts,
                       uint32_t part_cap, uint32_t* counters, void* stream);
/* n_blocks row blocks (block r: n_rows[r * n_rows_stride] rows at rows + r*block_cap*KAD_ROW_WORDS)
 * -> out_idx[qid] / out_cnt[qid]. n_rows_stride 0 means 1 (gathered counts); pass
 * KAD_SHARD_COUNTER_STRIDE to scatter a single rank's regions straight from its counters. */
int kad_rt_scatter_rows(const uint32_t* rows, const uint32_t* n_rows, uint32_t n_rows_stride, uint32_t n_blocks,
                        uint32_t block_cap, uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, int device,
                        void* stream);
/* n_parts partial rows sorted by qid -> the first min(count, sum of m) entries by (XOR distance,
 * global index) of each query (exact: parts come from disjoint buckets). */
int kad_rt_merge_parts(const uint32_t* parts, uint32_t n_parts, uint32_t count, uint32_t* out_idx,
                       uint8_t* out_cnt, int device, void* stream);
/* The device-only exchange step (no host read between the shard kernel, the collective and the merge,
 * so a step can be captured in a HIP graph). Every rank lays out ONE send block of
 * KAD_SHARD_BLOCK_WORDS(count, row_cap, part_cap) words and passes its pieces to kad_rt_shard_batch:
 *   rows     = block                                        (KAD_SHARD_REGIONS regions of row_cap rows)
 *   parts    = block + KAD_SHARD_REGIONS*row_cap*KAD_ROW_WORDS(count)      (part_cap partial rows)
 *   counters = parts + part_cap*KAD_PART_WORDS(count)       (zeroed before kad_rt_shard_batch)
 * The blocks of all `world` ranks are all-gathered in rank order (one fixed-size all_gather, RCCL)
 * into `recv`; kad_rt_gather_finish then writes every query's findClosestNodes row: complete rows
 * scattered by qid, the parts of edge-crossing windows merged by (XOR distance, global index).
 *   q        queries of the replicated batch (qids < q)
 *   scratch  device, q + world*part_cap words; its first q words must be KAD_NO_NODE (0xFFFFFFFF)
 *            before the first call, and every call leaves them so
 *   overflow device word: set to 1 (never cleared here) when any rank's region or part buffer was
 *            full, i.e. some rows are missing: grow row_cap / part_cap and run the batch again. A
 *            caller checks it once per batch or once per K steps.
 * world <= KAD_SHARD_MAX_WORLD. All pointers are device pointers; count in 1..KAD_MAX_COUNT. */
#define KAD_SHARD_MAX_WORLD 16u
#define KAD_SHARD_BLOCK_WORDS(count, row_cap, part_cap)                                                \
    ((uint64_t)KAD_SHARD_REGIONS * (row_cap) * KAD_ROW_WORDS(count) +                                  \
     (uint64_t)(part_cap) * KAD_PART_WORDS(count) + (uint64_t)KAD_SHARD_COUNTERS * KAD_SHARD_COUNTER_STRIDE)
int kad_rt_gather_finish(const uint32_t* recv, uint32_t world, uint32_t row_cap, uint32_t part_cap, uint32_t q,
                         uint32_t count, uint32_t* scratch, uint32_t* out_idx, uint8_t* out_cnt,
                         uint32_t* overflow, int device, void* stream);
/* The home-rank exchange (the default north-star step; the all-gather above moves every row to every rank).
 * Query block k (KAD_SHARD_QUERY_BLOCK queries of the replicated batch) has the home rank k * world / nblk:
 * kad_home_range gives rank r's queries [lo, hi). A rank's rows and parts go only to their query's home rank,
 * so one all_to_all of fixed-size blocks (RCCL) moves ~q/world rows into each rank instead of q:
 *   send     device, world blocks of KAD_SHARD_BLOCK_WORDS(count, row_cap, part_cap) words: block d holds what
 *            goes to rank d (its regions, parts and counters; the counters are zeroed by the call first)
 *   recv     after all_to_all_single(recv, send) with equal splits: block s = what rank s sent here
 * kad_rt_home_finish then writes rank `rank`'s rows: out_idx (hi - lo) x count and out_cnt (hi - lo) for qids
 * lo + i. scratch: H + world*part_cap words, H = the size of rank 0's range (the largest; the same for every rank,
 * so one scratch can serve the ranks of a step one after the other), the first H KAD_NO_NODE before the first call
 * (every call leaves them so). overflow: set to 1 when a block sent here was full; it only sees this rank's blocks, so
 * callers combine it over the ranks (all_reduce MAX) before deciding to grow and run again. */
#define KAD_SHARD_QUERY_BLOCK 256u
void kad_home_range(uint32_t q, uint32_t world, uint32_t rank, uint32_t* lo, uint32_t* hi);
int kad_rt_shard_batch_home(const kad_table* shard, const uint32_t* global_good_prefix, uint32_t global_buckets,
                            uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                            uint32_t reach_hi, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t world,
                            uint32_t* send, uint32_t row_cap, uint32_t part_cap, void* stream);
int kad_rt_home_finish(const uint32_t* recv, uint32_t world, uint32_t rank, uint32_t row_cap, uint32_t part_cap,
                       uint32_t q, uint32_t count, uint32_t* scratch, uint32_t* out_idx, uint8_t* out_cnt,
                       uint32_t* overflow, int device, void* stream);
/* The same step without the counter-zeroing launch: kad_rt_shard_step_home is kad_rt_shard_batch_home on send blocks
 * whose counters are already zero (a zero-filled buffer, or the previous step's kad_rt_home_finish_reset);
 * kad_rt_home_finish_reset is kad_rt_home_finish that also zeroes the counters of the `world` send blocks in its last
 * launch (the exchange has delivered them by then). send must not be recv (at world 1 without a collective, use the
 * zeroing pair above). */
int kad_rt_shard_step_home(const kad_table* shard, const uint32_t* global_good_prefix, uint32_t global_buckets,
                           uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                           uint32_t reach_hi, const uint8_t* targets, uint32_t q, uint32_t count, uint32_t world,
                           uint32_t* send, uint32_t row_cap, uint32_t part_cap, void* stream);
int kad_rt_home_finish_reset(const uint32_t* recv, uint32_t* send, uint32_t world, uint32_t rank, uint32_t row_cap,
                             uint32_t part_cap, uint32_t q, uint32_t count, uint32_t* scratch, uint32_t* out_idx,
                             uint8_t* out_cnt, uint32_t* overflow, int device, void* stream);

#define KAD_ROUTE_PACKED 1u /* mode bits of kad_route_run / kad_route_pack_ex */
#define KAD_ROUTE_KEYS 2u
#define KAD_ROUTE_ZEROED 4u

/* ---- owner routing of a serving front end ----
 * The headline form shards the table by ID range, one GPU per range, and answers every query on the GPU owning its
 * target (the reference answers each request where it arrives: Dht::onFindNode / onGetValues, dht.cpp:3189-3217).
 * A front end spreading arbitrary targets over N GPUs sends each target to its owner and the rows back, as
 * all_to_all_single of fixed-size blocks (no host read per batch):
 * kad_route_pack: targets (device, q x 20 bytes) into `world` send blocks of `cap` records of 20 bytes (send:
 *   world * cap * 20 bytes): target i goes to block d = (byte 0 >> (8 - shard_bits)) % world (d = 0 when
 *   shard_bits = 0). A block is KAD_ROUTE_SUBS sub-blocks of cap / KAD_ROUTE_SUBS records (cap a multiple of
 *   KAD_ROUTE_SUBS): the targets of workgroup w (KAD_ROUTE_QPW queries) go to sub-block w % KAD_ROUTE_SUBS, so that
 *   the workgroups' appends spread over KAD_ROUTE_SUBS counters per block (one counter hit by every workgroup
 *   serialised them: 24 us against 15 per 1M targets). slot[i] = d * cap + its record (KAD_NO_NODE when its
 *   sub-block is full, which sets the sticky word ctr[KAD_ROUTE_OVERFLOW_WORD(world)]). ctr:
 *   KAD_ROUTE_CTR_WORDS(world) words, zeroed by the call; ctr[(d * KAD_ROUTE_SUBS + r) * KAD_ROUTE_CSTRIDE] ends as
 *   sub-block r of block d's record count (it may exceed its capacity). The order of the records inside a sub-block
 *   is unspecified; records past a sub-block's count are left as they were (the owner answers them too; their rows
 *   are never read back). targets, send, slot and ctr must be 4-byte aligned (KAD_ERR_INVALID otherwise). Async on
 *   stream.
 * kad_route_unpack: rows returned in the send layout (back_idx: world * cap rows of `count` uint32, back_cnt: world *
 *   cap bytes) back to each query's position: out_idx row i = back_idx row slot[i], out_cnt[i] = back_cnt[slot[i]]
 *   (KAD_NO_NODE and 0 for slot KAD_NO_NODE). Async on stream. All pointers are device pointers. */
#define KAD_ROUTE_CSTRIDE 32u
#define KAD_ROUTE_MAX_WORLD 16u
#define KAD_ROUTE_SUBS 8u
#define KAD_ROUTE_QPW 1024u
#define KAD_ROUTE_CTR_WORDS(world) (((world) * KAD_ROUTE_SUBS + 1u) * KAD_ROUTE_CSTRIDE)
#define KAD_ROUTE_OVERFLOW_WORD(world) ((world) * KAD_ROUTE_SUBS * KAD_ROUTE_CSTRIDE)
int kad_route_pack(const uint8_t* targets, uint32_t q, uint32_t world, uint32_t shard_bits, uint32_t cap,
                   uint8_t* send, uint32_t* slot, uint32_t* ctr, int device, void* stream);
/* kad_route_pack_keys: kad_route_pack with each record the target's top 64 bits as one native uint64 key (send_keys:
 * world * cap keys, 8-byte aligned) instead of its 20 bytes: owner routing's key-only exchange, 8 bytes per query on
 * the links instead of 20 (answered by kad_rt_closest_keys_packed). */
int kad_route_pack_keys(const uint8_t* targets, uint32_t q, uint32_t world, uint32_t shard_bits, uint32_t cap,
                        uint64_t* send_keys, uint32_t* slot, uint32_t* ctr, int device, void* stream);
/* kad_route_pack_ex: kad_route_pack / kad_route_pack_keys by `mode`: KAD_ROUTE_KEYS (8-byte key records),
 * KAD_ROUTE_ZEROED (ctr is already zero — kad_route_unpack_packed_fold of the buffer set's previous batch leaves it so
 * — and is not zeroed by the call: no memset before the kernel). */
int kad_route_pack_ex(const uint8_t* targets, uint32_t q, uint32_t world, uint32_t shard_bits, uint32_t cap, void* send,
                      uint32_t* slot, uint32_t* ctr, uint32_t mode, int device, void* stream);
int kad_route_unpack(const uint32_t* slot, uint32_t q, uint32_t count, const uint32_t* back_idx,
                     const uint8_t* back_cnt, uint32_t* out_idx, uint8_t* out_cnt, int device, void* stream);
/* Packed rows for the way back (count <= KAD_ROUTE_PACKED_MAX_COUNT): a row's indices lie in one window of the
 * sorted table, so they travel as word 0 = the row's smallest index (KAD_NO_NODE for an empty row) and one byte
 * per entry = the entry's index minus word 0 (0xFF past the row's count), KAD_ROUTE_PACKED_WORDS(count) words
 * (count 8: 12 bytes instead of 33).
 * kad_route_compress: n rows (idx: n x count uint32, cnt: n bytes, the send layout) -> packed (n x
 *   KAD_ROUTE_PACKED_WORDS(count) uint32). A row whose indices span more than 254 cannot be packed: it sets the
 *   sticky word *escape (not cleared by the call; kad_route_pack's ctr[KAD_ROUTE_OVERFLOW_WORD(world) + 1] is meant
 *   for it), and the caller runs the batch's way back unpacked.
 * kad_route_unpack_packed: as kad_route_unpack, from packed rows in the send layout. Async on stream. */
#define KAD_ROUTE_PACKED_MAX_COUNT 32u
#define KAD_ROUTE_PACKED_WORDS(count) (1u + ((count) + 3u) / 4u)
int kad_route_compress(const uint32_t* idx, const uint8_t* cnt, uint32_t n, uint32_t count, uint32_t* packed,
                       uint32_t* escape, int device, void* stream);
int kad_route_unpack_packed(const uint32_t* slot, uint32_t q, uint32_t count, const uint32_t* back_packed,
                            uint32_t* out_idx, uint8_t* out_cnt, int device, void* stream);
/* kad_route_unpack_packed_fold: kad_route_unpack_packed, and in the same launch the batch's counters folded and zeroed
 * for the next KAD_ROUTE_ZEROED pack: flags[0..2] |= ctr[KAD_ROUTE_OVERFLOW_WORD(world) + 0..2] (overflow, escape,
 * tail), flags[3] = max(flags[3], KAD_ROUTE_SUBS x the fullest sub-block count: the capacity the batch needed), then
 * ctr[0 .. KAD_ROUTE_CTR_WORDS(world)) = 0. q = 0: the fold and reset alone. */
int kad_route_unpack_packed_fold(const uint32_t* slot, uint32_t q, uint32_t count, const uint32_t* back_packed,
                                 uint32_t* out_idx, uint8_t* out_cnt, uint32_t* ctr, uint32_t world, uint32_t* flags,
                                 int device, void* stream);
/* kad_rt_closest_batch_packed: kad_rt_closest_batch with each row written packed (the layout above, word 0 a base
 * no larger than any entry) by the query kernel itself: no full row is written and read back by kad_route_compress.
 * Count 8 on tables with short window lines only (KAD_ERR_UNSUPPORTED otherwise: use kad_rt_closest_batch +
 * kad_route_compress). A row whose indices span more than 254 sets *escape and writes nothing for it: the caller
 * answers the batch again unpacked. Async on stream. */
int kad_rt_closest_batch_packed(const kad_table* t, const uint8_t* targets, uint32_t q, uint32_t count,
                                uint32_t* packed, uint32_t* escape, void* stream);
/* kad_rt_closest_keys_packed: kad_rt_closest_batch_packed from 8-byte keys (the targets' top 64 bits, native uint64:
 * kad_route_pack_keys' records), which is all the short and 128-byte window lines read. The exact path (the few queries
 * no line answers) runs with the targets' low 96 bits taken as zero: the same rows as from the full targets unless two
 * nodes of its window share their top 64 bits (XOR order then depends on the low bits, infohash.h:131-146), which sets
 * the sticky word *tail (not cleared; ctr[KAD_ROUTE_OVERFLOW_WORD(world) + 2] is meant for it): the caller answers
 * that batch again from full targets. keys 8-byte aligned. Count 8 on tables with short window lines only. */
int kad_rt_closest_keys_packed(const kad_table* t, const uint64_t* keys, uint32_t q, uint32_t count, uint32_t* packed,
                               uint32_t* escape, uint32_t* tail, void* stream);
/* kad_route_fold_flags: flags[0..2] |= ctr[KAD_ROUTE_OVERFLOW_WORD(world) + 0..2] — overflow, packing escape, key-only
 * tail — (device words; kad_route_pack zeroes them, so a caller running many batches folds them after each). Async on
 * stream. */
int kad_route_fold_flags(const uint32_t* ctr, uint32_t world, uint32_t* flags, int device, void* stream);

/* ---- native multi-GPU executor (csrc/kad_comm.hip) ----
 * The two multi-GPU steps issued from C++ over an RCCL communicator of the engine's own (RCCL is loaded at run time:
 * the librccl.so.1 already in the process, else /opt/rocm/lib's; KAD_ERR_UNSUPPORTED without one).
 * kad_comm_unique_id: a new communicator id (KAD_COMM_ID_BYTES bytes) on rank 0; the caller hands it to every rank.
 * kad_comm_create: this rank's communicator on `device` (collective: every rank calls it at once), plus a compute
 *   and a comm stream of its own for the pipelined forms. kad_comm_all_to_all: ncclAllToAll of bytes_per_rank bytes
 *   per rank on stream.
 * kad_route_run: owner routing (sharded.OwnerRoute; reference callers dht.cpp:3189-3217) over n_batches batches of
 *   q targets: kad_route_pack into `world` blocks of `cap` records, all_to_all of the blocks, the owner's query of
 *   every received record (packed != 0: the rows go back packed — count 8 on tables with short window lines through
 *   kad_rt_closest_batch_packed, else kad_rt_closest_batch + kad_route_compress —; packed = 0: rows and counts), the
 *   all_to_all back, the unpack of batch i into out_idx[i] / out_cnt[i] with its counters folded into flags and zeroed
 *   (kad_route_unpack_packed_fold; 4 device words: [0] a block overflowed — grow cap and run again —, [1] a row
 *   escaped packing — run again unpacked —, [2] a key-only query needed the target's low bits — run again with
 *   KAD_ROUTE_KEYS off —, [3] the largest block capacity a batch needed). Every set's ctr must be zero on entry (a new
 *   zeroed buffer, or a previous kad_route_run's) and is left zero. `packed` is a mask:
 *   KAD_ROUTE_PACKED (rows back packed), KAD_ROUTE_KEYS (with it, count 8 on tables with short window lines: the
 *   targets travel as 8-byte keys, kad_route_pack_keys + kad_rt_closest_keys_packed; send / recv then hold world *
 *   cap keys; a table without short lines sets flags[2]).
 *   n_sets = 1: every batch in order on `stream` (comm may be NULL at world 1: no collective, recv == send and
 *   back_* == the answer buffers allowed). n_sets >= 3 (comm required): pipelined on the communicator's streams —
 *   batch i+1's pack and batch i's query on the compute stream while batch i's targets and batch i-1's rows are on the
 *   links —, forked from and joined back to `stream`. Pointers in `targets`, `out_idx`, `out_cnt` (host arrays of
 *   n_batches device pointers) and in the sets are device pointers; a set's buffers: send / recv world * cap * 20
 *   bytes, slot q words, ctr KAD_ROUTE_CTR_WORDS(world) words, rows / back_rows world * cap * count words and cnt /
 *   back_cnt world * cap bytes (packed = 0), prow / back_prow world * cap * KAD_ROUTE_PACKED_WORDS(count) words.
 * kad_shard_run: the north-star step (global_shard.GlobalShard.step) over n_batches replicated batches:
 *   kad_rt_shard_step_home into the `world` home blocks of send[k], all_to_all into recv[k],
 *   kad_rt_home_finish_reset into out_idx[i] / out_cnt[i] (this rank's home range), set k = i % n_sets; the send
 *   counters must start zero (each finish zeroes its set's). n_sets = 1 serial on `stream`, >= 3 pipelined (batch
 *   i+1's all_to_all under batch i's finish and batch i+2's shard kernel). overflow: the sticky word of
 *   kad_rt_home_finish. */
#define KAD_COMM_ID_BYTES 128u
typedef struct kad_comm kad_comm;
typedef struct kad_route_set {
    uint8_t* send;
    uint8_t* recv;
    uint32_t* slot;
    uint32_t* ctr;
    uint32_t* rows;
    uint8_t* cnt;
    uint32_t* back_rows;
    uint8_t* back_cnt;
    uint32_t* prow;
    uint32_t* back_prow;
} kad_route_set;
int kad_comm_unique_id(uint8_t* out_id);
int kad_comm_create(kad_comm** out, int device, uint32_t world, uint32_t rank, const uint8_t* id);
int kad_comm_destroy(kad_comm* comm);
int kad_comm_info(const kad_comm* comm, uint32_t* world, uint32_t* rank, int* device);
int kad_comm_all_to_all(kad_comm* comm, const void* send, void* recv, uint64_t bytes_per_rank, void* stream);
int kad_route_run(kad_comm* comm, const kad_table* t, uint32_t n_batches, const uint8_t* const* targets, uint32_t q,
                  uint32_t count, uint32_t world, uint32_t shard_bits, uint32_t cap, uint32_t packed, uint32_t n_sets,
                  const kad_route_set* sets, uint32_t* const* out_idx, uint8_t* const* out_cnt, uint32_t* flags,
                  void* stream);
int kad_shard_run(kad_comm* comm, const kad_table* shard, const uint32_t* global_good_prefix, uint32_t global_buckets,
                  uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                  uint32_t reach_hi, uint32_t n_batches, const uint8_t* const* targets, uint32_t q, uint32_t count,
                  uint32_t row_cap, uint32_t part_cap, uint32_t n_sets, uint32_t* const* send, uint32_t* const* recv,
                  uint32_t* const* scratch, uint32_t* overflow, uint32_t* const* out_idx, uint8_t* const* out_cnt,
                  void* stream);

/* ---- wire step after the query ------------------------ */
#define KAD_SEND_NODES 8u           /* reference network_engine.cpp:59 SEND_NODES */
#define KAD_ADDR4_LEN 6u            /* sin_addr (4) + sin_port (2), bytes as stored in sockaddr_in */
#define KAD_ADDR6_LEN 18u           /* sin6_addr (16) + sin6_port (2) */
#define KAD_NODE4_INFO_LEN 26u      /* network_engine.h:464 NODE4_INFO_BUF_LEN */
#define KAD_NODE6_INFO_LEN 38u      /* network_engine.h:466 NODE6_INFO_BUF_LEN */
/* Attach node addresses to a table (one family): host array, n_nodes x addr_len bytes
 * (KAD_ADDR4_LEN or KAD_ADDR6_LEN). Synchronous. */
int kad_table_set_addrs(kad_table* t, uint32_t addr_len, const uint8_t* addrs);
/* Batched NetworkEngine::bufferNodes(af, id, nodes) (network_engine.cpp:942-974): for query i the
 * candidates idx[i*k .. i*k + cnt[i]) (node indices incl. index_base, e.g. a findClosestNodes or
 * getCachedNodes result; cnt may be NULL: entries up to the first KAD_NO_NODE), sorted by XOR
 * distance to targets[i], the first KAD_SEND_NODES packed as ID + address records into
 * out[i * KAD_SEND_NODES * (20 + addr_len)]; out_n[i] = records written. Device pointers. */
int kad_buffer_nodes_batch(const kad_table* t, const uint8_t* targets, uint32_t q, const uint32_t* idx,
                           const uint8_t* cnt, uint32_t k, uint8_t* out, uint8_t* out_n, void* stream);
/* NetworkEngine::deserializeNodes' filter (network_engine.cpp:788-828): for n records of rec_len
 * (KAD_NODE4_INFO_LEN / KAD_NODE6_INFO_LEN) bytes, keep[i] = 0 if the record's ID is myid (host,
 * 20 bytes) or its address is martian (NetworkEngine::isMartian, :308-339). Device pointers. */
int kad_parse_nodes_batch(const uint8_t* records, uint32_t n, uint32_t rec_len, const uint8_t* myid,
                          uint8_t* keep, int device, void* stream);

/* ---- config 5: simulated swarm, iterative lookups ----
 * BUILD-DEFINED model (kad_swarm.hip header): n peers with shape-K routing tables (Dht::onNewNode
 * policy, dht.cpp:867-936) built on the device; lookups run synchronous hops of
 * MAX_REQUESTED_SEARCH_NODES = 4 findClosestNodes(t, 8) answers merged by Search::insertNode
 * (dht.cpp:961-1047, with its bad-node accounting) into a list of SEARCH_NODES = 14 non-bad nodes, until
 * the first 8 non-bad nodes have answered. A share of the peers can be offline: queried, they do not answer
 * and become bad (expired) search nodes. */
#define KAD_SWARM_LEVELS 28u        /* bucket levels per peer table (depth <= 27) */
#define KAD_SEARCH_NODES_LEN 14u    /* dht.h:314 SEARCH_NODES */
#define KAD_SEARCH_LIST 32u         /* list capacity: SEARCH_NODES non-bad nodes + the bad ones kept among them */
typedef struct kad_swarm kad_swarm;
typedef struct kad_search kad_search;
/* sorted_ids: host, n x 20 bytes, strictly ascending; peer index = position. */
int kad_swarm_create(kad_swarm** out, int device, uint32_t n, const uint8_t* sorted_ids);
int kad_swarm_destroy(kad_swarm* s);
int kad_swarm_info(const kad_swarm* s, uint32_t* n_peers, uint64_t* device_bytes);
/* Peer `peer`'s table (host outputs): depth D, counts[KAD_SWARM_LEVELS] per level (level D = my
 * bucket), entries[KAD_SWARM_LEVELS][8] peer indices (KAD_NO_NODE padded). */
int kad_swarm_get_table(const kad_swarm* s, uint32_t peer, uint32_t* depth, uint8_t* counts,
                        uint32_t* entries);
/* RoutingTable::findClosestNodes(targets[i], count) on peer peers[i]'s table (device pointers,
 * count <= 16): out_idx q x count peer indices, out_cnt q. */
int kad_swarm_closest_batch(const kad_swarm* s, const uint32_t* peers, const uint8_t* targets, uint32_t q,
                            uint32_t count, uint32_t* out_idx, uint8_t* out_cnt, void* stream);
/* S lookups (src peer, target); src/targets host or device. The initial list is the source's
 * findClosestNodes(t, 14). offline_per_10k: share of the peers (by a hash of the index) that never answer,
 * per 10,000 (0: all online). Asynchronous on `stream`. */
int kad_search_create(kad_search** out, const kad_swarm* s, uint32_t S, const uint32_t* src,
                      const uint8_t* targets, uint32_t offline_per_10k, void* stream);
/* One synchronous hop for every running lookup; *n_active (if given) = lookups still running
 * after it (synchronises the stream). */
int kad_search_hop(kad_search* x, uint32_t* n_active);
/* Host outputs (any may be NULL): list S x KAD_SEARCH_LIST peer indices (KAD_NO_NODE padded), queried and
 * bad flags S x KAD_SEARCH_LIST, list length S, hops S, done S (0 running, 1 synced: the first 8 non-bad
 * nodes answered, 2 stalled, 3 expired: the first min(size, 25) nodes are bad), overflow (1 value: lists that
 * reached KAD_SEARCH_LIST entries). */
int kad_search_get(const kad_search* x, uint32_t* list, uint8_t* queried, uint8_t* bad, uint8_t* n, uint32_t* hops,
                   uint8_t* done, uint32_t* overflow);
int kad_search_destroy(kad_search* x);

/* ---- InfoHash primitives (infohash.h), batched, device pointers ---------- */
/* out[i] = targets[i].xorCmp(a[i], b[i]) in {-1,0,1}   (infohash.h:131-146) */
int kad_xor_cmp_batch(const uint8_t* targets, const uint8_t* a, const uint8_t* b, uint32_t n,
                      int8_t* out, void* stream);
/* out[i] = InfoHash::commonBits(a[i], b[i]) in [0,160] (infohash.h:106-128) */
int kad_common_bits_batch(const uint8_t* a, const uint8_t* b, uint32_t n, uint32_t* out, void* stream);
/* out[i] = a[i].lowbit(), 0xFFFFFFFF for the zero ID     (infohash.h:84-95)  */
int kad_lowbit_batch(const uint8_t* a, uint32_t n, uint32_t* out, void* stream);
/* out_ids[i] = InfoHash::get(key i) = SHA-1 of data[offsets[i] .. offsets[i+1]) (infohash.cpp:46-61,
 * HASH_LEN 20 -> SHA-1). Device pointers; offsets has n+1 entries. */
int kad_infohash_get_batch(const uint8_t* data, const uint64_t* offsets, uint32_t n, uint8_t* out_ids,
                           int device, void* stream);

/* ---- synthetic tables (host code; bench and tests) ----------------------- */
/* n distinct random IDs from std::mt19937_64(seed): ID i = big-endian bytes of
 * draws (3i, 3i+1) and the top 4 bytes of draw 3i+2; duplicates are rejected and
 * redrawn. */
int kad_synth_ids(uint64_t seed, uint32_t n, uint8_t* out_ids);
/* status mix from std::mt19937_64(seed): u = draw % 100; u < good_pct -> GOOD,
 * u < good_pct+expired_pct -> EXPIRED, else dubious (0). */
int kad_synth_status(uint64_t seed, uint32_t n, uint32_t good_pct, uint32_t expired_pct,
                     uint8_t* out_status);
/* Sort ids ascending (stable permutation out_perm, may be NULL) in place. */
int kad_sort_ids(uint32_t n, uint8_t* ids, uint32_t* out_perm);
/* Uniform-depth table U(depth) over ascending ids: bucket firsts = prefix << (160-depth)
 * for every prefix in [prefix_lo, prefix_hi) (all 2^depth if prefix_hi == 0), bucket
 * offsets by ID range. out_first: (prefix_hi-prefix_lo) x 20 bytes, out_offset: +1. */
int kad_uniform_buckets(uint32_t n, const uint8_t* sorted_ids, uint32_t depth,
                        uint64_t prefix_lo, uint64_t prefix_hi,
                        uint8_t* out_first, uint32_t* out_offset);
/* Split-policy table S (Dht::onNewNode, dht.cpp:903-934, without the my-bucket
 * restriction; RoutingTable::split, routing_table.cpp:137-163): insert ids in
 * order, split the found bucket while it holds >= bucket_cap nodes.
 * Outputs the node order grouped by bucket (out_perm: n indices into ids, list
 * order inside each bucket), bucket firsts and offsets; *out_n_buckets <= n+1. */
int kad_split_table(uint32_t n, const uint8_t* ids, uint32_t bucket_cap,
                    uint32_t* out_perm, uint8_t* out_first, uint32_t* out_offset,
                    uint32_t* out_n_buckets);
/* Counter-based uniform swarm shard: every bucket of U(depth) in
 * [prefix_lo, prefix_hi) gets Poisson(mean) nodes drawn from a hash of
 * (seed, prefix), so any bucket range is reproducible independently (shards and
 * their halos). First call with out_ids == NULL returns the node count in *out_n. */
int kad_synth_uniform_shard(uint64_t seed, uint32_t depth, uint64_t prefix_lo, uint64_t prefix_hi,
                            double mean_per_bucket, uint32_t good_pct, uint32_t expired_pct,
                            uint32_t* out_n, uint8_t* out_ids, uint8_t* out_status,
                            uint32_t* out_offset);
/* The SURVEY.md §8d recipe of a whole n-node table (kad_synth_ids(seed_ids, n) and
 * kad_synth_status(seed_status, n, ...)) restricted to the U(depth) buckets
 * [prefix_lo, prefix_hi): ids ascending, status, bucket offsets (+1), and in
 * *out_below the number of the table's IDs below the range (global index of the
 * range's first node). One sequential pass over the n draws; fails on a duplicate
 * ID instead of redrawing it (probability < 1e-30 at n = 1e8). With out_ids ==
 * NULL: counts only; out arrays hold cap nodes (more in the range: KAD_ERR_NOMEM,
 * the count in *out_n). */
int kad_synth_recipe_range(uint64_t seed_ids, uint64_t seed_status, uint64_t n, uint32_t depth,
                           uint64_t prefix_lo, uint64_t prefix_hi, uint32_t good_pct,
                           uint32_t expired_pct, uint64_t cap, uint32_t* out_n, uint64_t* out_below,
                           uint8_t* out_ids, uint8_t* out_status, uint32_t* out_offset);

#ifdef __cplusplus
}
#endif
#endif /* KADGPU_H */
