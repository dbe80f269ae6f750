// layout.h — the frozen index as it sits in HBM, shared by the host builder
// (engine.cpp) and the gfx950 kernels (match_kernels.hip).
//
// The reference keeps filters as ETS ordered_set keys {Words, {ID}} and walks
// them with emqx_trie_search's seek/next loop (apps/emqx/src/emqx_trie_search.erl:192-389).
// Here the same key set is frozen into a trie whose edges live in ONE global
// open-addressed hash table keyed by (parent node, level-word id):
//
//   word table  : level-word bytes  -> word id    (tokeniser, one probe per topic level)
//   edge table  : (parent, word id) -> slot       (walk, one probe per frontier node/level)
//   slot lists  : slot -> offset of the node's terminal list in the arena
//   list arena  : u32 key handles; per list a LIST_HDR-word header [min bin-term key,
//                 min word-term key, min '#' key, term_cnt, hash_cnt], then the
//                 exact-terminal keys, then the '#'-child keys ("filter/#" hangs off the
//                 node of "filter").
//
// A node IS the index of the edge slot that leads to it (the root is ROOT_ID), so a
// slot needs no child field.  Its 16 bytes carry the key (parent, word), a 32-bit
// bloom of the node's literal child words (a lookup the bloom rules out is never
// issued: it would only miss), and the node's expansion flags plus, when the node
// has one key, that key inline: most probes are one 16-B read with nothing
// dependent behind them.  '+' edges are ordinary edges with word id W_PLUS.  '#'
// never becomes a node.  A filter whose '#' is not the last level can never match
// (emqx_topic.erl:99-101 only accepts a final '#'; emqx_trie_search.erl:282-290
// likewise), so it is kept on the host only.
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
constexpr uint32_t ROOT = 0u;              // root node id (host numbering)
constexpr uint32_t ROOT_ID = 0xFFFFFFFDu;  // the root as a parent in device edge keys

// EdgeSlot.info: what the CHILD node the slot leads to does
constexpr uint32_t I_PLUS = 1u << 31;       // child has a '+' child
constexpr uint32_t I_LIT = 1u << 30;        // child has at least one literal child
constexpr uint32_t I_KIDS = I_PLUS | I_LIT;
constexpr uint32_t I_MODE_SHIFT = 28;       // emission mode (2 bits):
constexpr uint32_t M_NONE = 0;    //   no keys end here
constexpr uint32_t M_INLINE = 1;  //   exactly one key, its handle inline (bits 0-26)
constexpr uint32_t M_CNT = 2;     //   list counts inline (term 14 b | hash 14 b); the list
                                  //   offset is read from the node record only when the
                                  //   keys are copied out (off the walk's critical path)
constexpr uint32_t M_REC = 3;     //   counts too large: read the node record during the walk
constexpr uint32_t I_INL_HASH = 1u << 27;   // M_INLINE: the key is a '#' key (else exact)
constexpr uint32_t I_KEY_MASK = (1u << 27) - 1;  // M_INLINE: the key handle
constexpr uint32_t INLINE_KEY_LIMIT = 1u << 27;  // handles >= this never go inline
constexpr uint32_t CNT_BITS = 14, CNT_MAX = (1u << CNT_BITS) - 1;
// List header words before a list's first key (lo): lo-6 the list's collapse bits (below),
// lo-5 smallest-id {Binary,{ID}} term key, lo-4 smallest-id word-list term key, lo-3
// smallest-id '#' key (NONE if none), lo-2 term_cnt, lo-1 hash_cnt.
constexpr uint32_t LIST_HDR = 6;
// lo-6: the OR over the list's keys of their device_api.h KDD_* flags (bit 0: the key's id is
// carried by another live key, so [unique] may collapse it; bit 1: a shared-subscription dest,
// which aggre/1 may collapse).  Kept as a superset (a bit is never cleared before the list is
// rewritten): the [unique] / aggre walks count a list's keys as collapsible only when its bit is
// set, so a topic none of whose lists carries one is final without reading its keys again.
constexpr uint32_t HDR_DD = 6;

TM_HD uint32_t info_mode(uint32_t info) { return (info >> I_MODE_SHIFT) & 3u; }
TM_HD uint32_t info_term_cnt(uint32_t info) { return (info >> CNT_BITS) & CNT_MAX; }
TM_HD uint32_t info_hash_cnt(uint32_t info) { return info & CNT_MAX; }

struct alignas(16) EdgeSlot {
    uint32_t parent;  // the parent's slot index (ROOT_ID for the root); NONE = empty
    uint32_t word;    // literal word id or W_PLUS
    uint32_t bloom;   // bloom_bit() of every literal child word of this node
    uint32_t info;    // I_* of this node
};
static_assert(sizeof(EdgeSlot) == 16, "edge slot is 16 B");

// One bit of a node's 32-bit child-word bloom (k = 1).
TM_HD uint32_t bloom_bit(uint32_t word) { return 1u << ((word * 0x9E3779B1u) >> 27); }

// Root record (the root has no incoming edge; no filter ends at it).
struct alignas(16) RootRec {
    uint32_t info;      // I_PLUS | I_LIT
    uint32_t bloom;     // literal child words of the root
    uint32_t list_off;  // first key of the "#" list
    uint32_t hash_cnt;  // keys of "#"
};

// Host-side terminal list of a node (host node numbering).
struct NodeList {
    uint32_t list_off;  // first key (the LIST_HDR-word header sits just before it)
    uint32_t term_cnt;  // keys whose filter ends exactly at the node
    uint32_t hash_cnt;  // keys of "node-path/#" (follow the term keys)
};

// 16-byte word slot.  Words of up to 8 bytes are their own key (the bytes, zero
// padded, little endian) so a hit is exact by construction; longer words are keyed
// by a 64-bit hash and verified byte-for-byte against the word arena.
constexpr uint32_t W_LONG = 1u << 31;  // WordSlot.len flag: key is a hash
struct alignas(16) WordSlot {
    uint64_t key;
    uint32_t len;  // byte length | W_LONG for words longer than 8 bytes
    uint32_t wid;  // NONE = empty
};
static_assert(sizeof(WordSlot) == 16, "word slot is 16 B");

// FNV-1a 64 over the level's bytes (words longer than 8 bytes).
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
TM_HD uint64_t word_slot_hash(uint64_t key, uint32_t len) { return mix64(key ^ ((uint64_t)len << 40)); }
TM_HD uint64_t edge_hash(uint32_t parent, uint32_t word) {
    return mix64(((uint64_t)parent << 32) | word);
}
// Home slot of edge (parent, word), where its linear probe starts.  The table has emask + 1
// slots, any count up to MAX_EDGE_SLOTS (not only powers of two): the home slot is the top 32
// bits of the hash scaled to the slot count (one 32 x 32 -> 64 multiply), and a probe that
// runs off the end wraps to slot 0 (next_slot).  Round 6: a power-of-two table stopped at
// 2^31 slots (the next one would reach the NONE / ROOT_ID sentinels), which held config D at
// load 0.26; it now grows to MAX_EDGE_SLOTS.
// TM_PLUS_NEAR=1 starts a '+' edge right after its parent's own slot, so the '+' probe that
// follows the walk's read of that slot usually hits the same L2 line: it cuts the walk's L2
// misses by 8 % and its HBM fetch by 11 %, yet a same-process A/B (tools/sweep.py plusnear/
// plushash, profiles/r04_sweep_plus_aa.jsonl) times it 1 % slower -- the walk waits on round
// trips, not on misses, and the clustering adds probes.  So every edge starts at its hash
// (DESIGN.md §4).
#ifndef TM_PLUS_NEAR
#define TM_PLUS_NEAR 0
#endif
constexpr uint64_t MAX_EDGE_SLOTS = 0xF0000000ull;  // below the sentinels; a multiple of 64
TM_HD uint64_t next_slot(uint64_t s, uint64_t emask) { return s == emask ? 0 : s + 1; }
TM_HD uint64_t edge_home(uint32_t parent, uint32_t word, uint64_t emask) {
    if (TM_PLUS_NEAR && word == W_PLUS && parent != ROOT_ID) return next_slot(parent, emask);
    return ((uint64_t)(uint32_t)(edge_hash(parent, word) >> 32) * (uint32_t)(emask + 1)) >> 32;
}

}  // namespace tmx
