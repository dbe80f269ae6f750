// layout.h — the frozen index as it sits in HBM, shared by the host builder
// (engine.cpp) and the gfx950 kernels (match_kernels.hip).
//
// The reference keeps filters as ETS ordered_set keys {Words, {ID}} and walks
// them with emqx_trie_search's seek/next loop (apps/emqx/src/emqx_trie_search.erl:192-348).
// Here the same key set is frozen into a trie whose edges live in ONE global
// open-addressed hash table keyed by (parent node, level-word id):
//
//   word table  : level-word bytes  -> word id    (tokeniser, one probe per topic level)
//   edge table  : (parent, word id) -> child rec  (walk, one probe per frontier node/level)
//   list arena  : u32 key handles; a node's exact-terminal keys followed by its
//                 '#'-child keys ("filter/#" hangs off the node of "filter").
//
// '+' edges are ordinary edges with word id TM_W_PLUS.  '#' never becomes a
// node: keys of "P/#" are stored in the hash-list of P's node.  A filter whose
// '#' is not the last level can never match (emqx_topic.erl:99-101 only accepts
// a final '#'; emqx_trie_search.erl:282-290 likewise), so it is kept on the host
// only.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define TM_HD __host__ __device__ __forceinline__
#else
#define TM_HD inline
#endif

namespace tmx {

constexpr uint32_t NONE = 0xFFFFFFFFu;     // empty slot / missing node / unknown word
constexpr uint32_t W_PLUS = 0xFFFFFFFEu;   // '+' edge label
constexpr uint32_t ROOT = 0u;              // root node id

// EdgeSlot.flags (describe the CHILD node the slot leads to)
constexpr uint32_t F_PLUS = 1u;   // child has a '+' child
constexpr uint32_t F_LIT = 2u;    // child has at least one literal child
constexpr uint32_t F_KIDS = F_PLUS | F_LIT;

// 32-byte edge slot: the key (parent, word) and the full record of the child,
// so one probe both follows the edge and tells what the child emits.
struct alignas(32) EdgeSlot {
    uint32_t parent;    // NONE = empty
    uint32_t word;      // literal word id or W_PLUS
    uint32_t child;     // child node id
    uint32_t flags;     // F_* of the child
    uint32_t list_off;  // child's terminal list in the arena
    uint32_t term_cnt;  // keys whose filter ends exactly at child
    uint32_t hash_cnt;  // keys of "child-path/#" (follow the term keys)
    uint32_t _pad;
};
static_assert(sizeof(EdgeSlot) == 32, "edge slot is 32 B");

// Root record (the root has no incoming edge).
struct alignas(16) RootRec {
    uint32_t flags;
    uint32_t list_off;
    uint32_t term_cnt;   // always 0: no filter has zero levels
    uint32_t hash_cnt;   // keys of "#"
};

// 32-byte word slot.  Verification is by bytes, never by hash alone: words of
// up to 12 bytes are compared inline, longer ones against the word arena.
constexpr uint32_t WORD_INLINE = 12;
struct alignas(32) WordSlot {
    uint64_t hash;       // full 64-bit word hash
    uint32_t wid;        // NONE = empty
    uint32_t len;
    uint32_t arena_off;  // bytes in the word arena (all words are stored there)
    uint8_t inl[WORD_INLINE];
};
static_assert(sizeof(WordSlot) == 32, "word slot is 32 B");

// FNV-1a 64 over the level's bytes (empty level -> offset basis).
constexpr uint64_t FNV_OFF = 0xcbf29ce484222325ull;
constexpr uint64_t FNV_PRIME = 0x100000001b3ull;
TM_HD uint64_t fnv_step(uint64_t h, uint8_t b) { return (h ^ b) * FNV_PRIME; }

// splitmix64 finaliser: spreads keys over the table index.
TM_HD uint64_t mix64(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    x ^= x >> 31;
    return x;
}
TM_HD uint64_t word_slot_hash(uint64_t h, uint32_t len) { return mix64(h ^ ((uint64_t)len << 56)); }
TM_HD uint64_t edge_hash(uint32_t parent, uint32_t word) {
    return mix64(((uint64_t)parent << 32) | word);
}

}  // namespace tmx
