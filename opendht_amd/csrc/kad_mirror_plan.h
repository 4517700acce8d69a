// Host plan of the incremental device mirror (kad_table_apply): the ops of one
// batch replayed on the bucket directory only, giving the new layout as segments that a gather
// kernel turns into the new node arrays. Host-only C++ (no HIP), so that the CPU sanitizer build
// (tests/cpp/sanitize_host.cpp) runs it against the oracle's std::list table.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace kadplan {

// Handles: old node index, or MIRROR_NEW | slot for a node of the batch.
constexpr uint32_t MIRROR_NEW = 0x80000000u;

struct MirrorSeg {
    uint32_t start, src, len, kind;  // kind 0: old nodes src.., 1: handles list[src..]
};

struct MirrorPlan {
    std::vector<MirrorSeg> segs;   // covering [0, n1) in order
    std::vector<uint32_t> list;    // the handle lists of kind-1 segments
    std::vector<uint32_t> off1;    // new bucket offsets, B1 + 1
    std::vector<uint8_t> first1;   // new bucket firsts (20 B each), only when B1 != B0 (splits)
    uint32_t B1 = 0, n1 = 0;
    bool new_in_range = true;      // every new node inside its bucket's dyadic range (range check asked)
};

// IDs (20 B each) of old nodes [a, e), written to out.
using OldIds = std::function<int(uint32_t a, uint32_t e, uint8_t* out)>;

// off0 (B0 + 1), first0 (20 B per bucket): the directory at the batch start; n0 its node count.
// ops (n_ops rows of kind, a, b; kinds as KAD_OP_*), new_ids (20 B per slot, n_new slots).
// range_shift >= 0 asks new_in_range for a uniform table: bucket o holds IDs whose top 64 bits
// >> range_shift equal range_pre0 + o. Returns KAD_OK or a KAD_ERR_* with `err` set.
int mirror_plan(const std::vector<uint32_t>& off0, const uint8_t* first0, uint32_t n0, const uint32_t* ops,
                uint32_t n_ops, const uint8_t* new_ids, uint32_t n_new, int range_shift, uint64_t range_pre0,
                const OldIds& old_ids, MirrorPlan& out, std::string& err);

}  // namespace kadplan
