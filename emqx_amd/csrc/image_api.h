// image_api.h — the slot-indexed device edge table built on the device from per-node
// records (result_kernels.hip).  The host keeps no copy of the slot-indexed table: it holds
// its nodes (parent, word, bloom, info, list, slot) and which slots are taken, and a full
// publish ships one 24-byte record per node instead of 20 bytes per slot.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tmx {

struct NodeImage {
    uint32_t slot;    // the node's edge slot (its device id)
    uint32_t parent;  // the parent's slot (ROOT_ID for a child of the root)
    uint32_t word;    // literal word id or W_PLUS
    uint32_t bloom;   // bloom_bit() of every literal child word
    uint32_t info;    // I_* of the node
    uint32_t list;    // first key of the node's list (the slot_list entry)
};
static_assert(sizeof(NodeImage) == 24, "node image record is 24 B");

// etab[0..cap) = empty slots and slot_list[0..cap) = 0, then each record written to its
// slot (records name distinct slots).  buf_slots: the two buffers' real capacity in slots and
// bnd the bounds record (read by the TM_BOUNDS build only).
hipError_t launch_edge_image(uint4 *etab, uint32_t *slot_list, uint64_t cap, const NodeImage *nodes, uint64_t n,
                             hipStream_t s, uint64_t buf_slots = ~0ull, unsigned long long *bnd = nullptr);
// The same in slices: clear slots [lo, hi); place records nodes[0..n) (all below cap).
hipError_t launch_edge_clear_range(uint4 *etab, uint32_t *slot_list, uint64_t lo, uint64_t hi, hipStream_t s,
                                   uint64_t buf_slots = ~0ull, unsigned long long *bnd = nullptr);
hipError_t launch_edge_place_range(uint4 *etab, uint32_t *slot_list, uint64_t cap, const NodeImage *nodes, uint64_t n,
                                   hipStream_t s, uint64_t buf_slots = ~0ull, unsigned long long *bnd = nullptr);

}  // namespace tmx
