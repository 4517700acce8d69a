// kad_comm.hip — the native multi-GPU executor: an RCCL communicator of the engine's own and the two
// multi-GPU steps issued from C++, so that a step costs the device work plus a few microseconds of host issue
// instead of the ~100-160 us of Python / c10d issue per batch measured for the same steps driven from Python
// (profiles/r06/pipeline_issue.json).
//
//   kad_comm_*       one communicator per rank (ncclCommInitRank over an id that rank 0 makes and the caller
//                    distributes, e.g. over a gloo group), plus a compute and a comm stream of its own. RCCL is
//                    loaded at run time: the librccl.so.1 already in the process (torch's) when there is one, else
//                    the ROCm one, so that one process never holds two RCCL builds.
//   kad_route_run    owner routing (the headline form as a serving front end; sharded.OwnerRoute) over n batches:
//                    pack -> all_to_all of the target blocks -> the owner's query -> all_to_all of the rows ->
//                    unpack. One buffer set: every batch in order on the caller's stream. Three or more sets: the
//                    batches pipelined, batch i+1's pack and batch i's answer on the compute stream while batch
//                    i's targets and batch i-1's rows are on the links (comm stream), ordered by events.
//   kad_shard_run    the north-star step (global_shard.GlobalShard) over n batches: shard kernel -> all_to_all of
//                    the home blocks -> scatter + merge; pipelined the same way with three or more sets.
// The reference answers each request where it arrives (Dht::onFindNode / onGetValues, dht.cpp:3189-3217); these are
// the exchanges a node-wide front end over N shard GPUs adds, with every answer the whole table's
// RoutingTable::findClosestNodes (routing_table.cpp:67-111).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/kadgpu.h"

namespace kadgpu_internal {
int set_error(int code, const char* msg);
}  // namespace kadgpu_internal

using kadgpu_internal::set_error;

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclAllToAll) all_to_all = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool ok = false;
    std::string why;
};

Rccl& rccl() {
    static Rccl r = [] {
        Rccl x;
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);  // already loaded (torch's build)
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
        if (!h) {
            const char* e = dlerror();
            x.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return x;
        }
        x.get_unique_id = (decltype(x.get_unique_id))dlsym(h, "ncclGetUniqueId");
        x.init_rank = (decltype(x.init_rank))dlsym(h, "ncclCommInitRank");
        x.destroy = (decltype(x.destroy))dlsym(h, "ncclCommDestroy");
        x.all_to_all = (decltype(x.all_to_all))dlsym(h, "ncclAllToAll");
        x.error_string = (decltype(x.error_string))dlsym(h, "ncclGetErrorString");
        x.ok = x.get_unique_id && x.init_rank && x.destroy && x.all_to_all && x.error_string;
        if (!x.ok) x.why = "librccl.so.1 lacks ncclGetUniqueId / ncclCommInitRank / ncclAllToAll";
        return x;
    }();
    return r;
}

struct DevSwitch {
    int prev = -1;
    explicit DevSwitch(int device) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != device) (void)hipSetDevice(device);
    }
    ~DevSwitch() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int hip_err(hipError_t e) { return set_error(KAD_ERR_HIP, hipGetErrorString(e)); }

int nccl_err(ncclResult_t r) {
    std::string m = "RCCL: ";
    m += rccl().error_string ? rccl().error_string(r) : "error";
    return set_error(KAD_ERR_HIP, m.c_str());
}

}  // namespace

struct kad_comm {
    int device = 0;
    uint32_t world = 1, rank = 0;
    ncclComm_t comm = nullptr;
    hipStream_t cs = nullptr, xs = nullptr;  // compute, comm
    std::vector<hipEvent_t> ev;               // a ring of events for the orderings of one run
    size_t next = 0;
    hipEvent_t event() {
        hipEvent_t e = ev[next];
        next = (next + 1) % ev.size();
        return e;
    }
};

namespace {

// e on `from`, `to` waits for it
hipError_t order(kad_comm* c, hipStream_t from, hipStream_t to) {
    hipEvent_t e = c->event();
    hipError_t r = hipEventRecord(e, from);
    if (r == hipSuccess) r = hipStreamWaitEvent(to, e, 0);
    return r;
}

int a2a(kad_comm* c, const void* send, void* recv, uint64_t bytes_per_rank, hipStream_t s) {
    ncclResult_t r = rccl().all_to_all(send, recv, bytes_per_rank, ncclUint8, c->comm, s);
    return r == ncclSuccess ? KAD_OK : nccl_err(r);
}

#define KAD_TRY(x)                     \
    do {                               \
        const int rc_ = (x);           \
        if (rc_ != KAD_OK) return rc_; \
    } while (0)
#define KAD_TRY_HIP(x)                             \
    do {                                           \
        const hipError_t e_ = (x);                 \
        if (e_ != hipSuccess) return hip_err(e_);  \
    } while (0)

__global__ void fold_flags_kernel(const uint32_t* __restrict__ words, uint32_t* __restrict__ flags) {
    if (threadIdx.x < 3) flags[threadIdx.x] |= words[threadIdx.x];
}

}  // namespace

extern "C" {

int kad_comm_unique_id(uint8_t* out) {
    if (!out) return set_error(KAD_ERR_INVALID, "NULL buffer");
    static_assert(sizeof(ncclUniqueId) <= KAD_COMM_ID_BYTES, "ncclUniqueId larger than KAD_COMM_ID_BYTES");
    if (!rccl().ok) return set_error(KAD_ERR_UNSUPPORTED, rccl().why.c_str());
    ncclUniqueId id;
    const ncclResult_t r = rccl().get_unique_id(&id);
    if (r != ncclSuccess) return nccl_err(r);
    std::memset(out, 0, KAD_COMM_ID_BYTES);
    std::memcpy(out, &id, sizeof(id));
    return KAD_OK;
}

int kad_comm_create(kad_comm** out, int device, uint32_t world, uint32_t rank, const uint8_t* id) {
    if (!out || !id) return set_error(KAD_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (world == 0 || world > KAD_ROUTE_MAX_WORLD || rank >= world)
        return set_error(KAD_ERR_INVALID, "world must be 1..16 and rank < world");
    if (!rccl().ok) return set_error(KAD_ERR_UNSUPPORTED, rccl().why.c_str());
    DevSwitch g(device);
    kad_comm* c = new kad_comm;
    c->device = device;
    c->world = world;
    c->rank = rank;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclResult_t r = rccl().init_rank(&c->comm, (int)world, uid, (int)rank);
    if (r != ncclSuccess) {
        delete c;
        return nccl_err(r);
    }
    hipError_t e = hipStreamCreateWithFlags(&c->cs, hipStreamNonBlocking);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->xs, hipStreamNonBlocking);
    c->ev.resize(64, nullptr);
    for (auto& x : c->ev)
        if (e == hipSuccess) e = hipEventCreateWithFlags(&x, hipEventDisableTiming);
    if (e != hipSuccess) {
        kad_comm_destroy(c);
        return hip_err(e);
    }
    *out = c;
    return KAD_OK;
}

int kad_comm_destroy(kad_comm* c) {
    if (!c) return KAD_OK;
    DevSwitch g(c->device);
    if (c->cs) (void)hipStreamSynchronize(c->cs);
    if (c->xs) (void)hipStreamSynchronize(c->xs);
    for (auto x : c->ev)
        if (x) (void)hipEventDestroy(x);
    if (c->cs) (void)hipStreamDestroy(c->cs);
    if (c->xs) (void)hipStreamDestroy(c->xs);
    if (c->comm) (void)rccl().destroy(c->comm);
    delete c;
    return KAD_OK;
}

int kad_comm_info(const kad_comm* c, uint32_t* world, uint32_t* rank, int* device) {
    if (!c) return set_error(KAD_ERR_INVALID, "NULL communicator");
    if (world) *world = c->world;
    if (rank) *rank = c->rank;
    if (device) *device = c->device;
    return KAD_OK;
}

int kad_comm_all_to_all(kad_comm* c, const void* send, void* recv, uint64_t bytes_per_rank, void* stream) {
    if (!c) return set_error(KAD_ERR_INVALID, "NULL communicator");
    if (bytes_per_rank && (!send || !recv)) return set_error(KAD_ERR_INVALID, "NULL buffer");
    DevSwitch g(c->device);
    return a2a(c, send, recv, bytes_per_rank, (hipStream_t)stream);
}

int kad_route_fold_flags(const uint32_t* ctr, uint32_t world, uint32_t* flags, int device, void* stream) {
    if (!ctr || !flags) return set_error(KAD_ERR_INVALID, "NULL buffer");
    if (world == 0 || world > KAD_ROUTE_MAX_WORLD) return set_error(KAD_ERR_INVALID, "world must be 1..16");
    DevSwitch g(device);
    hipLaunchKernelGGL(fold_flags_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, ctr + KAD_ROUTE_OVERFLOW_WORD(world),
                       flags);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? KAD_OK : hip_err(e);
}

int kad_route_run(kad_comm* c, const kad_table* t, uint32_t n_batches, const uint8_t* const* targets, uint32_t q,
                  uint32_t count, uint32_t world, uint32_t shard_bits, uint32_t cap, uint32_t packed, uint32_t n_sets,
                  const kad_route_set* sets, uint32_t* const* out_idx, uint8_t* const* out_cnt, uint32_t* flags,
                  void* stream) {
    if (!t || !sets || !flags || (n_batches && (!targets || !out_idx || !out_cnt)))
        return set_error(KAD_ERR_INVALID, "NULL argument");
    if (n_sets == 0 || n_sets == 2) return set_error(KAD_ERR_INVALID, "n_sets must be 1 (serial) or >= 3 (pipelined)");
    if (c && c->world != world) return set_error(KAD_ERR_INVALID, "world differs from the communicator's");
    if (!c && world != 1) return set_error(KAD_ERR_INVALID, "world > 1 needs a communicator");
    if (n_sets >= 3 && !c) return set_error(KAD_ERR_INVALID, "the pipelined form needs a communicator");
    if (count == 0 || count > KAD_ROUTE_PACKED_MAX_COUNT) return set_error(KAD_ERR_INVALID, "count must be 1..32");
    if (packed & ~(KAD_ROUTE_PACKED | KAD_ROUTE_KEYS)) return set_error(KAD_ERR_INVALID, "unknown mode bits");
    const bool keys = packed & KAD_ROUTE_KEYS;
    if (keys && (count != 8 || !(packed & KAD_ROUTE_PACKED)))
        return set_error(KAD_ERR_INVALID, "KAD_ROUTE_KEYS needs count 8 and KAD_ROUTE_PACKED");
    packed &= KAD_ROUTE_PACKED;
    for (uint32_t k = 0; k < n_sets; k++) {
        const kad_route_set& S = sets[k];
        if (!S.send || !S.recv || !S.slot || !S.ctr) return set_error(KAD_ERR_INVALID, "NULL buffer in a set");
        if (packed ? (!S.prow || !S.back_prow) : (!S.rows || !S.cnt || !S.back_rows || !S.back_cnt))
            return set_error(KAD_ERR_INVALID, "NULL row buffer in a set");
        if (c && (S.send == S.recv || (packed ? S.prow == S.back_prow : S.rows == S.back_rows)))
            return set_error(KAD_ERR_INVALID, "with a communicator the receive buffers must be separate");
    }
    kad_table_info info;
    KAD_TRY(kad_table_get_info(t, &info));
    if (c && info.device != c->device) return set_error(KAD_ERR_INVALID, "the table is on another device");
    DevSwitch g(info.device);
    const hipStream_t caller = (hipStream_t)stream;
    const uint64_t n = (uint64_t)world * cap, pw = KAD_ROUTE_PACKED_WORDS(count);
    const bool pipe = n_sets >= 3;
    const hipStream_t cs = pipe ? c->cs : caller, xs = pipe ? c->xs : caller;
    // count 8 on tables with short window lines: the query kernel writes the packed rows itself
    bool fused = packed && count == 8;
    const uint64_t rec = keys ? 8 : 20;  // bytes per record on the links
    auto answer = [&](const kad_route_set& S) -> int {
        uint32_t* esc = S.ctr + KAD_ROUTE_OVERFLOW_WORD(world) + 1;
        if (keys) {  // the owner's table has no short lines: the tail word asks for the batch again, full targets
            const int rc = kad_rt_closest_keys_packed(t, reinterpret_cast<const uint64_t*>(S.recv), (uint32_t)n, count,
                                                      S.prow, esc, esc + 1, cs);
            if (rc != KAD_ERR_UNSUPPORTED) return rc;
            const hipError_t e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(esc + 1), 1, 1, cs);
            return e == hipSuccess ? KAD_OK : hip_err(e);
        }
        if (fused) {
            const int rc = kad_rt_closest_batch_packed(t, S.recv, (uint32_t)n, count, S.prow, esc, cs);
            if (rc != KAD_ERR_UNSUPPORTED) return rc;
            fused = false;
        }
        if (packed) {
            KAD_TRY(kad_rt_closest_batch(t, S.recv, (uint32_t)n, count, S.rows, S.cnt, cs));
            return kad_route_compress(S.rows, S.cnt, (uint32_t)n, count, S.prow, esc, info.device, cs);
        }
        return kad_rt_closest_batch(t, S.recv, (uint32_t)n, count, S.rows, S.cnt, cs);
    };
    auto back = [&](const kad_route_set& S) -> int {
        if (!c) return KAD_OK;
        if (packed) return a2a(c, S.prow, S.back_prow, 4ull * cap * pw, xs);
        KAD_TRY(a2a(c, S.rows, S.back_rows, 4ull * cap * count, xs));
        return a2a(c, S.cnt, S.back_cnt, cap, xs);
    };
    // the unpack folds the set's counters into flags and zeroes them, so that its next pack needs no memset
    auto unpack = [&](uint32_t i) -> int {
        const kad_route_set& S = sets[i % n_sets];
        if (packed)
            return kad_route_unpack_packed_fold(S.slot, q, count, S.back_prow, out_idx[i], out_cnt[i], S.ctr, world, flags,
                                                info.device, cs);
        KAD_TRY(kad_route_unpack(S.slot, q, count, S.back_rows, S.back_cnt, out_idx[i], out_cnt[i], info.device, cs));
        return kad_route_unpack_packed_fold(S.slot, 0, count, nullptr, nullptr, nullptr, S.ctr, world, flags, info.device,
                                            cs);
    };
    const uint32_t pmode = (keys ? KAD_ROUTE_KEYS : 0u) | KAD_ROUTE_ZEROED;
    if (!pipe) {  // one set: every batch in order on the caller's stream
        const kad_route_set& S = sets[0];
        for (uint32_t i = 0; i < n_batches; i++) {
            KAD_TRY(kad_route_pack_ex(targets[i], q, world, shard_bits, cap, S.send, S.slot, S.ctr, pmode, info.device,
                                      caller));
            if (c) KAD_TRY(a2a(c, S.send, S.recv, rec * cap, caller));
            KAD_TRY(answer(S));
            KAD_TRY(back(S));
            KAD_TRY(unpack(i));
        }
        return KAD_OK;
    }
    c->next = 0;
    KAD_TRY_HIP(order(c, caller, cs));
    KAD_TRY_HIP(order(c, caller, xs));
    auto pack = [&](uint32_t i) -> int {
        const kad_route_set& S = sets[i % n_sets];
        KAD_TRY(kad_route_pack_ex(targets[i], q, world, shard_bits, cap, S.send, S.slot, S.ctr, pmode, info.device, cs));
        KAD_TRY_HIP(order(c, cs, xs));
        return a2a(c, S.send, S.recv, rec * cap, xs);
    };
    // compute: pack(i+1), answer(i), unpack(i-1); comm: targets(i+1), rows(i). Set i % n_sets is packed again by
    // batch i + n_sets only after unpack(i) (issued earlier on the compute stream), which needs n_sets >= 3.
    hipEvent_t sent_next = nullptr, back_prev = nullptr;
    if (n_batches) {
        KAD_TRY(pack(0));
        sent_next = c->event();
        KAD_TRY_HIP(hipEventRecord(sent_next, xs));
    }
    for (uint32_t i = 0; i < n_batches; i++) {
        const hipEvent_t sent_i = sent_next;
        if (i + 1 < n_batches) {
            KAD_TRY(pack(i + 1));
            sent_next = c->event();
            KAD_TRY_HIP(hipEventRecord(sent_next, xs));
        }
        KAD_TRY_HIP(hipStreamWaitEvent(cs, sent_i, 0));
        KAD_TRY(answer(sets[i % n_sets]));
        KAD_TRY_HIP(order(c, cs, xs));
        KAD_TRY(back(sets[i % n_sets]));
        const hipEvent_t back_i = c->event();
        KAD_TRY_HIP(hipEventRecord(back_i, xs));
        if (i >= 1) {
            KAD_TRY_HIP(hipStreamWaitEvent(cs, back_prev, 0));
            KAD_TRY(unpack(i - 1));
        }
        back_prev = back_i;
    }
    if (n_batches) {
        KAD_TRY_HIP(hipStreamWaitEvent(cs, back_prev, 0));
        KAD_TRY(unpack(n_batches - 1));
    }
    KAD_TRY_HIP(order(c, cs, caller));
    KAD_TRY_HIP(order(c, xs, caller));
    return KAD_OK;
}

int kad_shard_run(kad_comm* c, const kad_table* shard, const uint32_t* global_good_prefix, uint32_t global_buckets,
                  uint64_t global_base_hi, uint32_t depth, uint32_t shard_first_bucket, uint32_t reach_lo,
                  uint32_t reach_hi, uint32_t n_batches, const uint8_t* const* targets, uint32_t q, uint32_t count,
                  uint32_t row_cap, uint32_t part_cap, uint32_t n_sets, uint32_t* const* send, uint32_t* const* recv,
                  uint32_t* const* scratch, uint32_t* overflow, uint32_t* const* out_idx, uint8_t* const* out_cnt,
                  void* stream) {
    if (!c || !shard || !send || !recv || !scratch || !overflow || (n_batches && (!targets || !out_idx || !out_cnt)))
        return set_error(KAD_ERR_INVALID, "NULL argument");
    if (n_sets == 0 || n_sets == 2) return set_error(KAD_ERR_INVALID, "n_sets must be 1 (serial) or >= 3 (pipelined)");
    for (uint32_t k = 0; k < n_sets; k++)
        if (!send[k] || !recv[k] || !scratch[k] || send[k] == recv[k])
            return set_error(KAD_ERR_INVALID, "each set needs its own send, receive and scratch buffers");
    kad_table_info info;
    KAD_TRY(kad_table_get_info(shard, &info));
    if (info.device != c->device) return set_error(KAD_ERR_INVALID, "the table is on another device");
    DevSwitch g(c->device);
    const hipStream_t caller = (hipStream_t)stream;
    const uint64_t block = KAD_SHARD_BLOCK_WORDS(count, row_cap, part_cap);
    const uint32_t world = c->world, rank = c->rank;
    const bool pipe = n_sets >= 3;
    const hipStream_t cs = pipe ? c->cs : caller, xs = pipe ? c->xs : caller;
    // the send counters start zero (a new layout) and every finish zeroes its set's for the next use
    auto shard_k = [&](uint32_t i) -> int {
        return kad_rt_shard_step_home(shard, global_good_prefix, global_buckets, global_base_hi, depth,
                                      shard_first_bucket, reach_lo, reach_hi, targets[i], q, count, world,
                                      send[i % n_sets], row_cap, part_cap, cs);
    };
    auto finish = [&](uint32_t i) -> int {
        const uint32_t k = i % n_sets;
        return kad_rt_home_finish_reset(recv[k], send[k], world, rank, row_cap, part_cap, q, count, scratch[k],
                                        out_idx[i], out_cnt[i], overflow, c->device, cs);
    };
    if (!pipe) {
        for (uint32_t i = 0; i < n_batches; i++) {
            KAD_TRY(shard_k(i));
            KAD_TRY(a2a(c, send[0], recv[0], 4ull * block, caller));
            KAD_TRY(finish(i));
        }
        return KAD_OK;
    }
    c->next = 0;
    KAD_TRY_HIP(order(c, caller, cs));
    KAD_TRY_HIP(order(c, caller, xs));
    // compute: shard(i+1), finish(i); comm: all_to_all(i+1) after shard(i+1). Set k is written again by batch
    // i + n_sets's shard kernel only after finish(i) (same compute stream), and its receive blocks by that batch's
    // all_to_all only after the shard kernel that follows finish(i).
    std::vector<hipEvent_t> sent(n_batches ? 2 : 0);
    auto issue = [&](uint32_t i) -> int {
        KAD_TRY(shard_k(i));
        KAD_TRY_HIP(order(c, cs, xs));
        KAD_TRY(a2a(c, send[i % n_sets], recv[i % n_sets], 4ull * block, xs));
        sent[i & 1] = c->event();
        KAD_TRY_HIP(hipEventRecord(sent[i & 1], xs));
        return KAD_OK;
    };
    if (n_batches) KAD_TRY(issue(0));
    for (uint32_t i = 0; i < n_batches; i++) {
        if (i + 1 < n_batches) KAD_TRY(issue(i + 1));
        KAD_TRY_HIP(hipStreamWaitEvent(cs, sent[i & 1], 0));
        KAD_TRY(finish(i));
    }
    KAD_TRY_HIP(order(c, cs, caller));
    KAD_TRY_HIP(order(c, xs, caller));
    return KAD_OK;
}

}  // extern "C"
