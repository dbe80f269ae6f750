// match_kernels.hip — gfx950 (CDNA4) kernels of the topic-matching engine.
//
// Replaces the per-publish seek/next loop of emqx_trie_search
// (apps/emqx/src/emqx_trie_search.erl:192-389) with a batched walk of the frozen trie
// (layout.h).  Semantics are those of emqx_topic:match/2 (apps/emqx/src/emqx_topic.erl:78-102):
//   * a topic is split on '/' into levels; empty levels are ordinary words;
//   * '+' matches exactly one level (including an empty one);
//   * "P/#" matches P itself and everything below it;
//   * a topic whose first level starts with '$' is not matched by a filter whose
//     first level is '+' or '#' (emqx_topic.erl:81-84, emqx_trie_search.erl:160-163);
//   * a topic with a level exactly "+" or "#" is badarg (emqx_trie_search.erl:374-375).
//
// Kernels
//   k_match_fast  one WAVEFRONT per 64 topics.  The wave's topic bytes are staged in
//                 LDS with 16-B loads; lane = topic for the pre-scan and for the
//                 per-depth tokenise + word lookup.  The walk is level-synchronous:
//                 the frontier (all 64 topics' live trie nodes at this depth) sits in
//                 LDS and is expanded 64 entries per round, so one topic's '+'
//                 fan-out spreads over the whole wave; each lane issues its literal
//                 and '+' probes together.  Emitted key segments and next-frontier
//                 pushes are compacted with wave prefix scans; both overflow LDS into
//                 global chunk pools.  At the end the wave reserves its output with
//                 ONE atomic and expands the segments with a load-balanced copy.
//   k_match_slow  spill path for topics whose wave ran out of pool chunks: one lane
//                 per topic, depth-first with the stack in global scratch (depth
//                 bounded by the level count), count pass + fill pass.
// No MFMA: this is a latency/gather-bound walk.
#include <hip/hip_runtime.h>

#define TM_BND_FILE 1  // device_api.h TM_BOUNDS records

#include "device_api.h"
#include "wave.h"

namespace tmx {

constexpr int WAVE = 64;
#ifndef TM_FCAP
#define TM_FCAP 384  // with a 2 KiB topic stage: 10,016 B of LDS per wave, 16 waves/CU (the VGPR limit too); 448 / 2.5 KiB (14 waves) was best before the DPP scans
#endif
constexpr int FCAP = TM_FCAP;    // frontier entries per wave per depth held in LDS
constexpr int FCH = FR_CHUNK;    // frontier entries per global overflow chunk
constexpr int MAXF = 32;         // overflow chunks per frontier buffer per wave
#ifndef TM_SCAP
#define TM_SCAP 128
#endif
#ifndef TM_TBCAP
#define TM_TBCAP 2048
#endif
#ifndef TM_MIN_WAVES
#define TM_MIN_WAVES 1
#endif
constexpr int SCAP = TM_SCAP;    // key segments staged in LDS (<= one global chunk)
constexpr int MAXCHUNK = SEG_MAXCHUNK;  // global segment chunks one wave may flush (list in HBM)
constexpr int TBCAP = TM_TBCAP;  // topic bytes of one wave staged in LDS (else read from HBM)
constexpr uint32_t SEG_INLINE = 1u << 8;    // segment.w flag: .x is the key itself
constexpr uint32_t SEG_NODE = 1u << 9;      // segment.w flag: .x is a node (slot); its list
                                            // offset is read from slot_list at copy-out
constexpr uint32_t SEG_SKIP_SHIFT = 11;     // with SEG_NODE: keys to skip (term_cnt for the
                                            // '#' part) in .w bits 11-31
constexpr uint32_t SEG_DD = 1u << 10;       // list segment (not SEG_NODE): its list's header has
                                            // the batch's collapse bit (MatchArgs.dd_bit)
constexpr uint32_t DO_PLUS = 0x80u, DO_LIT = 0x40u;  // frontier meta: probes this entry needs
#ifndef TM_RPL
#define TM_RPL 2
#endif
#ifndef TM_QCOPY
#define TM_QCOPY 8  // lanes per group copying one medium list (0: the whole wave copies each long list)
#endif
#ifndef TM_QMED
#define TM_QMED 2  // a "medium" list is at most TM_QMED group-iterations long
#endif
#ifndef TM_CP_UNROLL
#define TM_CP_UNROLL 8
#endif
#ifndef TM_NT_DEPTH
#define TM_NT_DEPTH 0  // 0: every edge probe is a normal load; d: probes at depth >= d are non-temporal
#endif
#ifndef TM_NT_KEYS
#define TM_NT_KEYS 1  // key copy-out with non-temporal stores: the output is never re-read here, so it
                      // should not evict trie lines from L2 (0.9255 -> 0.9122 ms at config C)
#endif
// a key handle to the output arena
__device__ __forceinline__ void put_key(uint32_t *p, uint32_t k) {
#if TM_NT_KEYS
    __builtin_nontemporal_store(k, p);
#else
    *p = k;
#endif
}
// what k_match_fast's copy-out writes per key (template parameter OUT)
constexpr int O_KEYS = 0, O_RUNS = 1, O_IDS32 = 2, O_IDS64 = 3;
__device__ __forceinline__ void put_id32(uint32_t *p, uint32_t v) {
#if TM_NT_KEYS
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
__device__ __forceinline__ void put_id64(uint64_t *p, uint64_t v) {
#if TM_NT_KEYS
    __builtin_nontemporal_store(v, p);
#else
    *p = v;
#endif
}
// keys loaded from the arena -> what the output holds: the handles, or (MODE_IDS*) their ids
// (all gathers of the unrolled group are issued before the first store)
template <int OUT, int U>
__device__ __forceinline__ void store_group(const MatchArgs &a, uint64_t dst0, uint32_t stride, const uint32_t (&key)[U],
                                            uint32_t nvalid) {
    if constexpr (OUT == O_KEYS) {
#pragma unroll
        for (int u = 0; u < U; u++)
            if ((uint32_t)u < nvalid) put_key(&a.keys[BI(dst0 + (uint64_t)u * stride, keys)], key[u]);
    } else {
        uint64_t id[U];
#pragma unroll
        for (int u = 0; u < U; u++)
            if ((uint32_t)u < nvalid) id[u] = a.key_rec[BI(2ull * key[u], key_rec)];
#pragma unroll
        for (int u = 0; u < U; u++)
            if ((uint32_t)u < nvalid) {
                if constexpr (OUT == O_IDS32) put_id32(&a.keys[BI(dst0 + (uint64_t)u * stride, keys)], (uint32_t)id[u]);
                else put_id64(reinterpret_cast<uint64_t *>(a.keys) + BI(dst0 + (uint64_t)u * stride, keys), id[u]);
            }
    }
}
constexpr int RPL = TM_RPL;                 // frontier entries per lane per round
constexpr int CP_UNROLL = TM_CP_UNROLL;     // arena loads in flight per lane, long lists
constexpr int CP_SHORT = 8;                 // lists up to this long are copied by one lane

// ---------------------------------------------------------------------------
// wave helpers
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (WAVE - 1); }

#ifndef TM_ALIVE_REG
#define TM_ALIVE_REG 1  // k_match_fast: topics alive at this / the next depth in registers (DPP OR) not LDS atomics
#endif
#ifndef TM_DPP_SCAN
#define TM_DPP_SCAN 1  // wave scans on DPP lane moves (wave.h) instead of ds_bpermute round trips
#endif
// exclusive prefix sum over the 64 lanes; *total gets the wave sum
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
#if TM_DPP_SCAN
    const uint32_t x = wave_incl_scan_dpp(v);
    *total = lane_value(x, WAVE - 1);
#else
    uint32_t x = v;
    const uint32_t lane = lane_id();
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        uint32_t y = __shfl_up(x, d, WAVE);
        if (lane >= (uint32_t)d) x += y;
    }
    *total = __shfl(x, WAVE - 1, WAVE);
#endif
    return x - v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, WAVE);
    return v;
}

// ---------------------------------------------------------------------------
// word table: (key, tag) -> word id.  key = the word's bytes (<= 8) or its FNV-1a
// hash (longer, then verified byte-for-byte against the arena: never trust a hash).
template <class ByteAt>
__device__ __forceinline__ uint32_t word_lookup(const MatchArgs &a, uint64_t key, uint32_t len, uint32_t st,
                                                ByteAt &&byte_at, uint32_t *probes) {
    const uint32_t tag = len > 8 ? (len | W_LONG) : len;
    uint64_t s = word_slot_hash(key, tag) & a.wmask;
    for (;;) {
        const uint4 x = *reinterpret_cast<const uint4 *>(a.wtab + BI(s, wtab));
        (*probes)++;
        if (x.w == NONE) return NONE;
        if (x.z == tag && x.x == (uint32_t)key && x.y == (uint32_t)(key >> 32)) {
            if (len <= 8) return x.w;
            const uint8_t *w = a.warena + BIN(a.word_off[BI(x.w, word_off)], len, warena);
            bool eq = true;
            for (uint32_t i = 0; i < len && eq; i++) eq = byte_at(st + i) == w[i];
            if (eq) return x.w;
        }
        s = (s + 1) & a.wmask;
    }
}

// Tokenise one level starting at byte *i (== e for an empty last level):
// returns the word key and advances *i to the '/' or the end.
template <class ByteAt>
__device__ __forceinline__ uint64_t level_key(uint32_t *i, uint32_t e, ByteAt &&byte_at) {
    uint64_t w8 = 0, h = FNV_OFF;
    uint32_t k = *i, n = 0;
    uint8_t c;
    while (k < e && (c = byte_at(k)) != '/') {
        if (n < 8) w8 |= (uint64_t)c << (8 * n);
        h = fnv_step(h, c);
        k++;
        n++;
    }
    *i = k;
    return n <= 8 ? w8 : h;
}

// edge table: (parent, word) -> 16-byte slot; the child node IS the slot index
struct Rec {
    uint32_t child, bloom, info;
};
__device__ __forceinline__ bool edge_probe(const MatchArgs &a, uint32_t parent, uint32_t word, Rec *r,
                                           uint32_t *probes) {
    uint64_t s = edge_home(parent, word, a.emask);
    for (;;) {
        const uint4 x = *reinterpret_cast<const uint4 *>(a.etab + BI(s, etab));
        (*probes)++;
        if (x.x == NONE) return false;
        if (x.x == parent && x.y == word) {
            *r = Rec{(uint32_t)s, x.z, x.w};
            return true;
        }
        s = next_slot(s, a.emask);
    }
}

// Which probes a node at depth d needs for the topic's level-d word w: the '+' child
// if it has one; the literal child only if the child-word bloom admits w.
__device__ __forceinline__ uint32_t probes_needed(uint32_t info, uint32_t bloom, uint32_t w) {
    uint32_t m = (info & I_PLUS) ? DO_PLUS : 0u;
    if ((info & I_LIT) && w != NONE && (bloom & bloom_bit(w))) m |= DO_LIT;
    return m;
}

#if TM_PRELOOK
// Pre-scan of one topic (lane = topic) with its first TM_PRELOOK levels tokenised and their
// word-table probes issued together: one round trip instead of one per level inside the
// walk, which then takes level d's word id from registers (deeper levels are tokenised as
// the walk reaches them, from byte pre_b).  Also counts the levels (nl) and finds badarg.
// In: a, b, e, byte_at.  Out: widr[TM_PRELOOK], nl, badarg, pre_b; PROBES counts slot reads.
// A macro, expanded in place in both wave kernels: as an inlined helper function the
// compiler gave k_match_fast 134 VGPRs instead of 115 (3 waves per SIMD instead of 4).
#define TM_PRESCAN_PRELOOK(PROBES)                                                                  \
    do {                                                                                            \
        uint64_t key[TM_PRELOOK], sl[TM_PRELOOK];                                                   \
        uint32_t tag[TM_PRELOOK], wst[TM_PRELOOK];                                                  \
        uint4 x[TM_PRELOOK];                                                                        \
        uint32_t i = b;                                                                             \
    _Pragma("unroll")                                                                               \
        for (int l = 0; l < TM_PRELOOK; l++) {                                                      \
            widr[l] = NONE;                                                                         \
            tag[l] = NONE;  /* no such level */                                                     \
            if (i <= e) {  /* level l exists and starts at byte i */                                \
                wst[l] = i;                                                                         \
                key[l] = level_key(&i, e, byte_at);                                                 \
                const uint32_t len = i - wst[l];                                                    \
                if (len == 1 && (key[l] == '+' || key[l] == '#') && !a.topic_words) badarg = true;                    \
                tag[l] = len > 8 ? (len | W_LONG) : len;                                            \
                sl[l] = word_slot_hash(key[l], tag[l]) & a.wmask;                                   \
                x[l] = *reinterpret_cast<const uint4 *>(a.wtab + BI(sl[l], wtab));                  \
                (PROBES)++;                                                                         \
                nl++;                                                                               \
                i++;                                                                                \
            }                                                                                       \
        }                                                                                           \
        pre_b = i;                                                                                  \
  /* resolve the probes (collision chains and long-word byte checks are rare) */                    \
    _Pragma("unroll")                                                                               \
        for (int l = 0; l < TM_PRELOOK; l++) {                                                      \
            if (tag[l] == NONE) continue;                                                           \
            uint4 y = x[l];                                                                         \
            for (;;) {                                                                              \
                if (y.w == NONE) break;                                                             \
                if (y.z == tag[l] && y.x == (uint32_t)key[l] && y.y == (uint32_t)(key[l] >> 32)) {  \
                    const uint32_t len = tag[l] & ~W_LONG;                                          \
                    if (len <= 8) {                                                                 \
                        widr[l] = y.w;                                                              \
                        break;                                                                      \
                    }                                                                               \
                    const uint8_t *w = a.warena + BIN(a.word_off[BI(y.w, word_off)], len, warena);  \
                    bool eq = true;                                                                 \
                    for (uint32_t k = 0; k < len && eq; k++) eq = byte_at(wst[l] + k) == w[k];      \
                    if (eq) {                                                                       \
                        widr[l] = y.w;                                                              \
                        break;                                                                      \
                    }                                                                               \
                }                                                                                   \
                sl[l] = (sl[l] + 1) & a.wmask;                                                      \
                y = *reinterpret_cast<const uint4 *>(a.wtab + BI(sl[l], wtab));                     \
                (PROBES)++;                                                                         \
            }                                                                                       \
        }                                                                                           \
        if (pre_b <= e) {  /* levels past TM_PRELOOK: count them and check for badarg */            \
            uint32_t st = pre_b;                                                                    \
            for (uint32_t i2 = pre_b;; ++i2) {                                                      \
                const bool end = i2 == e;                                                           \
                const uint8_t c = end ? (uint8_t)'/' : byte_at(i2);                                 \
                if (c == '/') {                                                                     \
                    if (i2 - st == 1 && (byte_at(st) == '+' || byte_at(st) == '#') && !a.topic_words) badarg = true;  \
                    nl++;                                                                           \
                    st = i2 + 1;                                                                    \
                    if (end) break;                                                                 \
                }                                                                                   \
            }                                                                                       \
        }                                                                                           \
                                                                                                    \
    } while (0)

// widr[lv] for a wave-uniform lv < TM_PRELOOK (static register indices, no scratch)
__device__ __forceinline__ uint32_t prelook_word(const uint32_t (&widr)[TM_PRELOOK], uint32_t lv) {
    uint32_t v = NONE;
#pragma unroll
    for (int l = 0; l < TM_PRELOOK; l++)
        if (lv == (uint32_t)l) v = widr[l];
    return v;
}
#endif

// ---------------------------------------------------------------------------
// fast kernel: one wavefront (= one 64-thread workgroup) per 64 topics
//
// LDS per wave (~10.5 KiB): the topic bytes, the two frontier buffers (FCAP
// entries each, extended by global overflow chunks), a segment staging buffer that
// is flushed to a global chunk pool when full, and per-topic cursors.  Levels are
// tokenised lazily (one level per depth) so there is no level cap; a topic only
// spills to k_match_slow when a pool is exhausted.
template <int TB>
struct WaveLdsT {
    uint8_t tb[TB];               // the wave's topic bytes (16-B aligned window; a stub with k_prescan)
    uint32_t fr_node[2][FCAP];
    uint8_t fr_meta[2][FCAP];     // topic lane | DO_PLUS / DO_LIT
    uint32_t fch[2][MAXF];        // global overflow chunks of each frontier buffer
    uint4 seg[SCAP];              // {src or key, cnt, rel, topic lane | SEG_INLINE}
    uint32_t seg_scan[SCAP + 1];
    uint32_t wid[2][WAVE]; // word id of level d (wid[d&1]) and of level d+1 (tokenised ahead)
    uint32_t nlev[WAVE];
    uint32_t cnt[WAVE];    // keys matched so far (allocates each segment's rel)
    uint32_t tbase[WAVE];  // output base of the topic
    unsigned long long spill;     // bit per topic lane: spill to k_match_slow
    unsigned long long alive[2];  // bit per topic lane: has frontier entries at this / the next depth
};
using WaveLds = WaveLdsT<TBCAP>;

// Expand L.seg[0..ns) into the output.  Short segments (<= CP_SHORT keys, most of them
// single inline keys) are copied by the lane that holds them; long ones (hot '#'
// filters with thousands of subscribers) are queued and copied by the whole wave, 64
// consecutive keys per instruction, CP_UNROLL instructions in flight.
template <int OUT, class Lds>
__device__ __forceinline__ void expand_segments(const MatchArgs &a, Lds &L, uint32_t ns) {
    const uint32_t lane = lane_id();
    uint32_t nlong = 0;  // wave-uniform; long segment indices are queued in L.seg_scan
    uint32_t nmed = 0;   // TM_QCOPY: medium lists, queued from the front (huge ones from the back)
    (void)nmed;
    for (uint32_t sb = 0; sb < ns; sb += WAVE) {
        const uint32_t j = sb + lane;
        uint4 g = make_uint4(0u, 0u, 0u, 0u);
        if (j < ns) {
            g = L.seg[j];
            bool dd_list = (g.w & SEG_DD) != 0;
            if (g.w & SEG_NODE) {  // M_CNT list: its offset is read now, off the walk
                const uint32_t lo = a.slot_list[BI(g.x, slot_list)];
                if constexpr (OUT == O_KEYS)
                    if (a.dd_bit) dd_list = (a.arena[BI(lo - HDR_DD, arena)] & a.dd_bit) != 0;
                g.x = lo + (g.w >> SEG_SKIP_SHIFT);
                g.w &= 0xFFu | SEG_INLINE;
                L.seg[j] = g;
            }
            if ((L.spill >> (g.w & 0x3Fu)) & 1ull) g.y = 0;  // spilled topic: the slow kernel owns it
            if constexpr (OUT == O_KEYS) {
                // [unique] / aggre/1: the topic's keys that may collapse (a list's whole count
                // when its header bit is set; an inline key by its own flag), L.nlev reused
                if (a.dd_bit && g.y) {
                    const uint32_t c = (g.w & SEG_INLINE) ? ((a.key_dd[BI(g.x, key_dd)] & a.dd_bit) ? 1u : 0u)
                                                          : (dd_list ? g.y : 0u);
                    if (c) atomicAdd(&L.nlev[g.w & 0x3Fu], c);
                }
            }
        }
        const bool is_long = g.y > (uint32_t)CP_SHORT;
        if (!is_long && g.y) {
            const uint32_t dst = L.tbase[g.w & 0xFFu] + g.z;
            if (g.w & SEG_INLINE) {
                if constexpr (OUT == O_KEYS) {
                    put_key(&a.keys[BI(dst, keys)], g.x);
                } else {
                    const uint32_t one[1] = {g.x};
                    store_group<OUT, 1>(a, dst, 1, one, 1);
                }
            } else {
                uint32_t key[CP_SHORT];
#pragma unroll
                for (int k = 0; k < CP_SHORT; k++)
                    if ((uint32_t)k < g.y) key[k] = a.arena[BI(g.x + k, arena)];
                if constexpr (OUT == O_KEYS) {
#pragma unroll
                    for (int k = 0; k < CP_SHORT; k++)
                        if ((uint32_t)k < g.y) put_key(&a.keys[BI(dst + k, keys)], key[k]);
                } else {
                    store_group<OUT, CP_SHORT>(a, dst, 1, key, g.y);
                }
            }
        }
#if TM_QCOPY
        // medium lists go to lane groups (several lists in flight), huge ones to the wave
        const bool is_med = is_long && g.y <= (uint32_t)(TM_QCOPY * CP_UNROLL * TM_QMED);
        uint32_t totm;
        const uint32_t qm = nmed + wave_excl_scan(is_med ? 1u : 0u, &totm);
        if (is_med) L.seg_scan[qm] = j;
        nmed += totm;
        const bool is_huge = is_long && !is_med;
        uint32_t tot;
        const uint32_t q = nlong + wave_excl_scan(is_huge ? 1u : 0u, &tot);
        if (is_huge) L.seg_scan[SCAP - q] = j;
        nlong += tot;
#else
        uint32_t tot;
        const uint32_t q = nlong + wave_excl_scan(is_long ? 1u : 0u, &tot);
        if (is_long) L.seg_scan[q] = j;
        nlong += tot;
#endif
    }
    __syncthreads();
#if TM_QCOPY
    {
        constexpr uint32_t GRP = TM_QCOPY, NG = WAVE / TM_QCOPY;
        const uint32_t grp = lane / GRP, gl = lane % GRP;
        for (uint32_t qb = 0; qb < nmed; qb += NG) {
            const uint32_t qi = qb + grp;
            if (qi < nmed) {
                const uint4 g = L.seg[L.seg_scan[qi]];
                const uint32_t dst = L.tbase[g.w & 0xFFu] + g.z;
                for (uint32_t k0 = gl; k0 < g.y; k0 += GRP * CP_UNROLL) {
                    uint32_t key[CP_UNROLL];
#pragma unroll
                    for (int u = 0; u < CP_UNROLL; u++) {
                        const uint32_t k = k0 + u * GRP;
                        if (k < g.y) key[u] = a.arena[BI(g.x + k, arena)];
                    }
                    if constexpr (OUT == O_KEYS) {
#pragma unroll
                        for (int u = 0; u < CP_UNROLL; u++) {
                            const uint32_t k = k0 + u * GRP;
                            if (k < g.y) put_key(&a.keys[BI(dst + k, keys)], key[u]);
                        }
                    } else {  // keys k0, k0 + GRP, ... are valid while below g.y
                        store_group<OUT, CP_UNROLL>(a, (uint64_t)dst + k0, GRP, key, (g.y - k0 + GRP - 1) / GRP);
                    }
                }
            }
        }
    }
#endif
    for (uint32_t qq = 0; qq < nlong; qq++) {
#if TM_QCOPY
        const uint32_t q = SCAP - qq;
#else
        const uint32_t q = qq;
#endif
        const uint4 g = L.seg[L.seg_scan[q]];
        const uint32_t dst = L.tbase[g.w & 0xFFu] + g.z;
        for (uint32_t k0 = lane; k0 < g.y; k0 += WAVE * CP_UNROLL) {
            uint32_t key[CP_UNROLL];
#pragma unroll
            for (int u = 0; u < CP_UNROLL; u++) {
                const uint32_t k = k0 + u * WAVE;
                if (k < g.y) key[u] = a.arena[BI(g.x + k, arena)];
            }
            if constexpr (OUT == O_KEYS) {
#pragma unroll
                for (int u = 0; u < CP_UNROLL; u++) {
                    const uint32_t k = k0 + u * WAVE;
                    if (k < g.y) put_key(&a.keys[BI(dst + k, keys)], key[u]);
                }
            } else {
                store_group<OUT, CP_UNROLL>(a, (uint64_t)dst + k0, WAVE, key, (g.y - k0 + WAVE - 1) / WAVE);
            }
        }
    }
    __syncthreads();
}

// MODE_RUNS copy-out: every segment of the wave becomes one host span of its topic (no key is
// read or written: the consumer reads the ids from the engine's host id arena).
template <class Lds>
__device__ __forceinline__ void emit_spans(const MatchArgs &a, const Lds &L, const uint4 *seg, uint32_t ns) {
    uint4 *spans = reinterpret_cast<uint4 *>(a.keys);
    for (uint32_t j = lane_id(); j < ns; j += WAVE) {
        const uint4 g = seg[j];
        if (!g.y || ((L.spill >> (g.w & 0x3Fu)) & 1ull)) continue;  // spilled: the slow kernel owns it
        uint64_t p;
        if (g.w & SEG_INLINE) {
            p = a.span_keys + (uint64_t)a.span_kstride * g.x;
        } else {
            const uint32_t src = (g.w & SEG_NODE) ? a.slot_list[BI(g.x, slot_list)] + (g.w >> SEG_SKIP_SHIFT) : g.x;
            p = a.span_arena + (uint64_t)a.span_w * src;
        }
        spans[BI(L.tbase[g.w & 0x3Fu] + g.z, keys)] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), g.y, 0u);
    }
}

#if TM_PRELOOK
// Pre-pass: one wave per 64 consecutive topics stages their bytes in LDS and runs the
// pre-scan of k_match_fast (TM_PRESCAN_PRELOOK) at this kernel's own occupancy (2 KiB of LDS
// per wave instead of the walk's 10), writing each topic's word ids and level count for
// k_match_fast<PRE> (MatchArgs.pre_wid / pre_meta).  The walk then holds neither the topic
// bytes nor the pre-scan's registers.
template <bool STATS>
__global__ __launch_bounds__(WAVE) void k_prescan(MatchArgs a) {
    __shared__ uint8_t tb[TBCAP];
    const uint32_t lane = lane_id();
    const uint32_t t0 = blockIdx.x * WAVE, t = t0 + lane;
    const bool active = t < a.n;
    const uint32_t wb0 = a.off[BI(t0, off)], wb1 = a.off[BI(min(t0 + WAVE, a.n), off)];
    const uint32_t tbase = wb0 & ~15u;
    const bool staged = ((reinterpret_cast<uintptr_t>(a.bytes) & 15u) == 0) && (wb1 - tbase <= (uint32_t)TBCAP);
    if (staged) {
        for (uint32_t j = lane * 16; tbase + j < wb1; j += WAVE * 16) {
            if (tbase + j + 16 <= wb1) {
                *reinterpret_cast<uint4 *>(&tb[j]) = *reinterpret_cast<const uint4 *>(a.bytes + BIN(tbase + j, 16, bytes));
            } else {
                for (uint32_t k = 0; tbase + j + k < wb1; k++) tb[j + k] = a.bytes[BI(tbase + j + k, bytes)];
            }
        }
        __syncthreads();
    }
    auto byte_at = [&](uint32_t i) -> uint8_t { return staged ? tb[i - tbase] : a.bytes[BI(i, bytes)]; };
    bool badarg = false, dollar = false;
    uint32_t nl = 0, b = 0, e = 0, pre_b = 0, probes = 0;
    uint32_t widr[TM_PRELOOK];
    if (active) {
        b = a.off[BI(t, off)];
        e = a.off[BI(t + 1, off)];
        dollar = (e > b) && byte_at(b) == '$';
        // TM_PRESCAN_PRELOOK's work, with its collision / long-word path moved out of the
        // unrolled loop (here the compiler would otherwise keep the per-level arrays in scratch)
        uint64_t key[TM_PRELOOK];
        uint32_t tag[TM_PRELOOK], wst[TM_PRELOOK];
        uint4 x[TM_PRELOOK];
        uint32_t i = b;
#pragma unroll
        for (int l = 0; l < TM_PRELOOK; l++) {
            widr[l] = NONE;
            tag[l] = NONE;  // no such level
            key[l] = 0;
            wst[l] = 0;
            if (i <= e) {  // level l exists and starts at byte i
                wst[l] = i;
                key[l] = level_key(&i, e, byte_at);
                const uint32_t len = i - wst[l];
                if (len == 1 && (key[l] == '+' || key[l] == '#') && !a.topic_words) badarg = true;
                tag[l] = len > 8 ? (len | W_LONG) : len;
                x[l] = *reinterpret_cast<const uint4 *>(a.wtab + BI(word_slot_hash(key[l], tag[l]) & a.wmask, wtab));
                probes++;
                nl++;
                i++;
            }
        }
        pre_b = i;
#pragma unroll
        for (int l = 0; l < TM_PRELOOK; l++) {
            if (tag[l] == NONE) continue;
            const uint32_t len = tag[l] & ~W_LONG;
            const uint4 y = x[l];
            if (y.w == NONE) continue;  // not in the dictionary
            if (len <= 8 && y.z == tag[l] && y.x == (uint32_t)key[l] && y.y == (uint32_t)(key[l] >> 32))
                widr[l] = y.w;
            else  // a collision chain or a long word (byte check): the whole lookup again (rare)
                widr[l] = word_lookup(a, key[l], len, wst[l], byte_at, &probes);
        }
        if (pre_b <= e) {  // levels past TM_PRELOOK: count them and check for badarg
            uint32_t st = pre_b;
            for (uint32_t i2 = pre_b;; ++i2) {
                const bool end = i2 == e;
                const uint8_t c = end ? (uint8_t)'/' : byte_at(i2);
                if (c == '/') {
                    if (i2 - st == 1 && (byte_at(st) == '+' || byte_at(st) == '#') && !a.topic_words) badarg = true;
                    nl++;
                    st = i2 + 1;
                    if (end) break;
                }
            }
        }
#pragma unroll
        for (int l = 0; l < TM_PRELOOK; l++) a.pre_wid[BI((uint64_t)l * a.pre_stride + t, pre_wid)] = widr[l];
        a.pre_meta[BI(t, pre_meta)] =
            make_uint2(min(nl, 0x3FFFFFFFu) | (badarg ? 1u << 30 : 0u) | (dollar ? 1u << 31 : 0u), pre_b);
    }
    if constexpr (STATS) {
        const uint64_t p = wave_sum64(probes);
        if (lane == 0 && a.stats) atomicAdd(&a.stats[2], (unsigned long long)p);
    }
}
#endif

template <bool STATS, int OUT, bool PRE>
__global__ __launch_bounds__(WAVE, TM_MIN_WAVES) void k_match_fast(MatchArgs a) {
    constexpr bool RUNS = OUT == O_RUNS;
#ifndef TM_PRE_PAD
#define TM_PRE_PAD 0  // experiment knob: 1 keeps the PRE walk's LDS at the fused kernel's size (16 waves/CU)
#endif
    __shared__ WaveLdsT<(PRE && !TM_PRE_PAD) ? 16 : TBCAP> L;
    uint32_t *const wchunks = a.wave_chunks + BIN((uint64_t)blockIdx.x * MAXCHUNK, MAXCHUNK, wave_chunks);  // this wave's flushed chunks
    const uint32_t lane = lane_id();
    const uint32_t t = blockIdx.x * a.tpw + lane;
    const bool active = lane < a.tpw && t < a.n;
    uint32_t st_visit = 0, st_probe = 0, st_wprobe = 0, st_seg = 0, st_flush = 0, st_frch = 0, st_rec = 0,
             st_inl = 0;
    // STATS build only: phase stamps (shares of wave time, not absolute kernel time)
    uint64_t ts0 = 0, ts1 = 0, ts2 = 0, ts3 = 0;
    if constexpr (STATS) ts0 = __builtin_amdgcn_s_memtime();
    if (blockIdx.x == 0 && threadIdx.x < CTL_BYTES / 8) a.ctl_next[threadIdx.x] = 0ull;  // next launch's counters

    // ---- 0. stage the wave's topic bytes in LDS with 16-B coalesced loads
    const uint32_t t0 = blockIdx.x * a.tpw;
    const uint32_t wb0 = a.off[BI(t0, off)], wb1 = a.off[BI(min(t0 + a.tpw, a.n), off)];
    const uint32_t tbase = wb0 & ~15u;
    // (PRE: k_prescan did the pre-scan; only levels past TM_PRELOOK read bytes, from HBM)
    const bool staged =
        !PRE && ((reinterpret_cast<uintptr_t>(a.bytes) & 15u) == 0) && (wb1 - tbase <= (uint32_t)TBCAP);
    if (staged) {
        for (uint32_t j = lane * 16; tbase + j < wb1; j += WAVE * 16) {
            if (tbase + j + 16 <= wb1) {
                *reinterpret_cast<uint4 *>(&L.tb[j]) = *reinterpret_cast<const uint4 *>(a.bytes + BIN(tbase + j, 16, bytes));
            } else {
                for (uint32_t k = 0; tbase + j + k < wb1; k++) L.tb[j + k] = a.bytes[BI(tbase + j + k, bytes)];
            }
        }
        __syncthreads();
    }
    auto byte_at = [&](uint32_t i) -> uint8_t { return staged ? L.tb[i - tbase] : a.bytes[BI(i, bytes)]; };

    // ---- 1. pre-scan (lane = topic): levels, badarg, '$'
    bool badarg = false, dollar = false;
    uint32_t nl = 0, b = 0, e = 0;
#if TM_PRELOOK
    uint32_t widr[TM_PRELOOK];  // word ids of the first TM_PRELOOK levels
    uint32_t pre_b = 0;         // byte where level TM_PRELOOK starts
    uint32_t pre_w0 = NONE;     // PRE: level 0's word id, loaded with the topic's meta
    if constexpr (PRE) {
        if (active) {
            b = a.off[BI(t, off)];
            e = a.off[BI(t + 1, off)];
            const uint2 m = a.pre_meta[BI(t, pre_meta)];
            pre_w0 = a.pre_wid[BI(t, pre_wid)];
            nl = m.x & 0x3FFFFFFFu;
            badarg = (m.x >> 30) & 1u;
            dollar = (m.x >> 31) != 0;
            pre_b = m.y;
        }
    } else if (active) {
        b = a.off[BI(t, off)];
        e = a.off[BI(t + 1, off)];
        dollar = (e > b) && byte_at(b) == '$';
        TM_PRESCAN_PRELOOK(st_wprobe);
    }
#else
    if (active) {
        b = a.off[BI(t, off)];
        e = a.off[BI(t + 1, off)];
        dollar = (e > b) && byte_at(b) == '$';
        uint32_t st = b;
        for (uint32_t i = b;; ++i) {
            const bool end = i == e;
            const uint8_t c = end ? (uint8_t)'/' : byte_at(i);
            if (c == '/') {
                if (i - st == 1 && (byte_at(st) == '+' || byte_at(st) == '#') && !a.topic_words) badarg = true;
                nl++;
                st = i + 1;
                if (end) break;
            }
        }
    }
#endif
    const bool spill0 = active && !badarg && a.force_slow;
    const bool walk = active && !badarg && !spill0;
#if TM_PRELOOK
    uint32_t cur_b = pre_b;  // byte offset where level TM_PRELOOK starts (tokenised in the walk)
#else
    uint32_t cur_b = b;  // byte offset where this lane's topic's next level starts
#endif
    L.nlev[lane] = nl;
    L.cnt[lane] = 0;
    if constexpr (RUNS) L.tbase[lane] = 0;  // RUNS: keys of the topic during the walk (cnt counts spans)
    {
        const unsigned long long sp0 = __ballot(spill0);
        if (lane == 0) {
            L.spill = sp0;
            L.alive[0] = 0;
            L.alive[1] = 0;
        }
    }

    // tokenise one level of this lane's topic (the cursor walks left to right)
    // level lv's word id into L.wid[slot] (lv is wave-uniform)
    auto level_word = [&](uint32_t slot, uint32_t lv) {
#if TM_PRELOOK
        if (lv < (uint32_t)TM_PRELOOK) {
            if constexpr (PRE)
                L.wid[slot][lane] = lv == 0 ? pre_w0 : a.pre_wid[BI((uint64_t)lv * a.pre_stride + t, pre_wid)];
            else
                L.wid[slot][lane] = prelook_word(widr, lv);
            return;
        }
#endif
        (void)lv;
        uint32_t i = cur_b;
        const uint32_t st = i;
        const uint64_t key = level_key(&i, e, byte_at);
        L.wid[slot][lane] = word_lookup(a, key, i - st, st, byte_at, &st_wprobe);
        cur_b = i + 1;
    };

    // ---- 2. root: emit "#" keys (not for '$' topics), seed the frontier
    const RootRec R = *a.root;
    if (walk) level_word(0, 0);  // level 0
    uint32_t nseg = 0, nchunk = 0;  // wave-uniform
#if TM_ALIVE_REG
    unsigned long long alive_c = 0;  // wave-uniform: topics with frontier entries at this depth
#endif
    uint32_t nfr;
    {
        const bool em = walk && !dollar && R.hash_cnt;
        uint32_t tot;
        const uint32_t pos = wave_excl_scan(em ? 1u : 0u, &tot);
        if (em) {
            const uint32_t fl = (OUT == O_KEYS && a.dd_bit && (a.arena[BI(R.list_off - HDR_DD, arena)] & a.dd_bit))
                                    ? SEG_DD : 0u;
            L.seg[pos] = make_uint4(R.list_off, R.hash_cnt, 0u, lane | fl);
            if constexpr (RUNS) {
                L.cnt[lane] = 1;
                L.tbase[lane] = R.hash_cnt;
            } else {
                L.cnt[lane] = R.hash_cnt;
            }
        }
        nseg = tot;
        st_seg += em;
        const uint32_t rinfo = dollar ? (R.info & I_LIT) : R.info;  // '$' topics: no root '+'
        const uint32_t m = walk ? probes_needed(rinfo, R.bloom, L.wid[0][lane]) : 0u;
        const unsigned long long al0 = __ballot(m != 0);
        if (lane == 0) L.alive[0] = al0;
#if TM_ALIVE_REG
        alive_c = al0;
#endif
        const uint32_t p2 = wave_excl_scan(m ? 1u : 0u, &tot);
        if (m) {
            L.fr_node[0][p2] = ROOT_ID;
            L.fr_meta[0][p2] = (uint8_t)(lane | m);
            st_visit++;
        }
        nfr = tot;
    }
    __syncthreads();

    // frontier = LDS entries [0, FCAP) + global overflow chunks beyond; a buffer keeps
    // its chunks from level to level (it is rewritten every other depth)
    uint32_t nfch[2] = {0, 0};  // overflow chunks held by each buffer (wave-uniform)
    auto fr_read = [&](uint32_t lvl, uint32_t i, uint32_t &node, uint32_t &meta) {
        if (i < (uint32_t)FCAP) {
            node = L.fr_node[lvl][i];
            meta = L.fr_meta[lvl][i];
        } else {
            const uint32_t k = i - FCAP;
            const uint2 v = a.fr_pool[BI((uint64_t)L.fch[lvl][k / FCH] * FCH + k % FCH, fr_pool)];
            node = v.x;
            meta = v.y;
        }
    };
    auto fr_write = [&](uint32_t lvl, uint32_t i, uint32_t node, uint32_t meta) {
        if (i < (uint32_t)FCAP) {
            L.fr_node[lvl][i] = node;
            L.fr_meta[lvl][i] = (uint8_t)meta;
        } else {
            const uint32_t k = i - FCAP;
            a.fr_pool[BI((uint64_t)L.fch[lvl][k / FCH] * FCH + k % FCH, fr_pool)] = make_uint2(node, meta);
        }
    };

    if constexpr (STATS) ts1 = __builtin_amdgcn_s_memtime();
    // ---- 3. level-synchronous walk
    for (uint32_t d = 0; nfr > 0; ++d) {
        const uint32_t cur = d & 1, nxt = cur ^ 1;
        // STATS build: per-depth edge probes, wave cycles, frontier entries and probe round
        // trips (wave-level iterations of the dependent probe loop), tm_debug_depth_stats
        uint32_t dp_probe = 0, dp_rt = 0;
        uint64_t dp_t0 = 0;
        if constexpr (STATS) dp_t0 = __builtin_amdgcn_s_memtime();
        // 3a. tokenise level d+1 ahead for topics that are still alive and go deeper:
        //     the children pushed at this depth are filtered with it (bloom)
#if TM_ALIVE_REG
        if (walk && ((alive_c >> lane) & 1ull) && d + 1 < nl) level_word(nxt, d + 1);
        unsigned long long alive_n = 0;  // wave-uniform
#else
        if (walk && ((L.alive[cur] >> lane) & 1ull) && d + 1 < nl) level_word(nxt, d + 1);
        if (lane == 0) L.alive[nxt] = 0;
#endif
        __syncthreads();
        // 3b. expand the frontier, WAVE * RPL entries per round (RPL per lane, so each
        //     lane has up to 2 * RPL independent probes in flight)
        uint32_t nnext = 0;
        for (uint32_t base = 0; base < nfr; base += WAVE * RPL) {
            uint32_t tl[RPL];
            bool last[RPL], f1[RPL], f2[RPL];
            Rec r1[RPL], r2[RPL];
            {
                uint32_t node[RPL], w[RPL];
                bool p1[RPL], p2[RPL];
                uint64_t s1[RPL], s2[RPL];
#pragma unroll
                for (int k = 0; k < RPL; k++) {
                    const uint32_t i = base + k * WAVE + lane;
                    const bool has = i < nfr;
                    uint32_t meta = 0;
                    node[k] = 0;
                    if (has) fr_read(cur, i, node[k], meta);
                    tl[k] = meta & 63u;
                    w[k] = has ? L.wid[cur][tl[k]] : NONE;
                    last[k] = has && (d + 1 == L.nlev[tl[k]]);
                    p1[k] = has && (meta & DO_LIT);
                    p2[k] = has && (meta & DO_PLUS);
                    s1[k] = edge_home(node[k], w[k], a.emask);
                    s2[k] = edge_home(node[k], W_PLUS, a.emask);
                    f1[k] = f2[k] = false;
                }
                // all 2*RPL probe chains advance together
                for (;;) {
                    bool any = false;
#pragma unroll
                    for (int k = 0; k < RPL; k++) any = any || p1[k] || p2[k];
                    if (!any) break;
                    uint4 x1[RPL], x2[RPL];
#pragma unroll
                    for (int k = 0; k < RPL; k++) {
#if TM_NT_DEPTH
                        // probes past depth TM_NT_DEPTH are random lines of a 16 GiB table that are
                        // rarely met again: non-temporal loads keep them from evicting the upper
                        // levels and the hot lists from L2 (experiment knob)
                        if (d >= (uint32_t)TM_NT_DEPTH) {
                            typedef unsigned v4u __attribute__((ext_vector_type(4)));
                            v4u y1 = {NONE, 0, 0, 0}, y2 = {NONE, 0, 0, 0};
                            if (p1[k]) y1 = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(a.etab + s1[k]));
                            if (p2[k]) y2 = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(a.etab + s2[k]));
                            x1[k] = make_uint4(y1.x, y1.y, y1.z, y1.w);
                            x2[k] = make_uint4(y2.x, y2.y, y2.z, y2.w);
                        } else
#endif
                        {
                        x1[k] = p1[k] ? *reinterpret_cast<const uint4 *>(a.etab + BI(s1[k], etab)) : make_uint4(NONE, 0, 0, 0);
                        x2[k] = p2[k] ? *reinterpret_cast<const uint4 *>(a.etab + BI(s2[k], etab)) : make_uint4(NONE, 0, 0, 0);
                        }
                        st_probe += (uint32_t)p1[k] + (uint32_t)p2[k];
                        if constexpr (STATS) dp_probe += (uint32_t)p1[k] + (uint32_t)p2[k];
                    }
                    if constexpr (STATS) dp_rt++;
#pragma unroll
                    for (int k = 0; k < RPL; k++) {
                        if (p1[k]) {
                            if (x1[k].x == NONE) p1[k] = false;
                            else if (x1[k].x == node[k] && x1[k].y == w[k]) {
                                r1[k] = Rec{(uint32_t)s1[k], x1[k].z, x1[k].w};
                                f1[k] = true;
                                p1[k] = false;
                            } else s1[k] = next_slot(s1[k], a.emask);
                        }
                        if (p2[k]) {
                            if (x2[k].x == NONE) p2[k] = false;
                            else if (x2[k].x == node[k] && x2[k].y == W_PLUS) {
                                r2[k] = Rec{(uint32_t)s2[k], x2[k].z, x2[k].w};
                                f2[k] = true;
                                p2[k] = false;
                            } else s2[k] = next_slot(s2[k], a.emask);
                        }
                    }
                }
            }
            // what each found child emits: its '#' keys always, its exact keys at the
            // topic's last level.  One key: inline.  Counts inline (M_CNT): a node
            // segment resolved at copy-out.  Huge lists (M_REC): read the header now.
            uint32_t ns = 0;
#pragma unroll
            for (int k = 0; k < RPL; k++) {
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    const bool f = c ? f2[k] : f1[k];
                    const uint32_t info = c ? r2[k].info : r1[k].info;
                    if (!f) continue;
                    const uint32_t m = info_mode(info);
                    if (m == M_INLINE) ns += ((info & I_INL_HASH) || last[k]);
                    else if (m == M_CNT) ns += (info_hash_cnt(info) != 0) + (last[k] && info_term_cnt(info) != 0);
                    else if (m == M_REC) ns += 2;  // upper bound; an unused one gets cnt 0
                }
            }
            uint32_t tot_s;
            uint32_t ps = wave_excl_scan(ns, &tot_s);
            if (tot_s && nseg && nseg + tot_s > (uint32_t)SCAP) {
                // flush the staged segments to one global chunk
                __syncthreads();
                uint32_t c = 0;
                if (lane == 0) c = (uint32_t)atomicAdd(a.seg_cursor, 1ull);
                c = __shfl(c, 0, WAVE);
                if (c < a.seg_chunks && nchunk < (uint32_t)MAXCHUNK) {
                    uint4 *dst = a.seg_pool + BIN((uint64_t)c * SCAP, SCAP, seg_pool);
                    for (uint32_t j = lane; j < (uint32_t)SCAP; j += WAVE)
                        dst[j] = j < nseg ? L.seg[j] : make_uint4(0u, 0u, 0u, 0u);
                    if (lane == 0) wchunks[nchunk] = c;
                    nchunk++;
                    st_flush++;
                } else {
                    // pool exhausted: those topics take the spill kernel instead
                    for (uint32_t j = lane; j < nseg; j += WAVE) atomicOr(&L.spill, 1ull << (L.seg[j].w & 0x3Fu));
                }
                nseg = 0;
                __syncthreads();
            }
            // a round that emits more than the staging buffer holds writes its segments
            // straight into freshly reserved global chunks (wave-uniform decision)
            const bool direct = tot_s > (uint32_t)SCAP;
            uint32_t dc0 = 0;
            bool dok = true;
            if (direct) {
                const uint32_t ndc = (tot_s + SCAP - 1) / SCAP;
                unsigned long long c0 = 0;
                if (lane == 0) c0 = atomicAdd(a.seg_cursor, (unsigned long long)ndc);
                c0 = __shfl(c0, 0, WAVE);
                dok = c0 + ndc <= a.seg_chunks && nchunk + ndc <= (uint32_t)MAXCHUNK;
                dc0 = (uint32_t)c0;
                if (dok) {
                    for (uint32_t j = lane; j < ndc; j += WAVE) wchunks[nchunk + j] = dc0 + j;
                    for (uint32_t j = tot_s + lane; j < ndc * SCAP; j += WAVE)  // pad the last chunk
                        a.seg_pool[BI((uint64_t)dc0 * SCAP + j, seg_pool)] = make_uint4(0u, 0u, 0u, 0u);
                    nchunk += ndc;
                    st_flush += ndc;
                }
            } else {
                ps += nseg;
            }
            if (ns) {
#pragma unroll
                for (int k = 0; k < RPL; k++) {
                    auto put = [&](uint32_t src, uint32_t cnt, uint32_t fl2) {
                        uint32_t rel = 0;
                        if (cnt) {
                            if constexpr (RUNS) {
                                atomicAdd(&L.tbase[tl[k]], cnt);
                                rel = atomicAdd(&L.cnt[tl[k]], 1u);
                            } else {
                                rel = atomicAdd(&L.cnt[tl[k]], cnt);
                            }
                        }
                        const uint4 g = make_uint4(src, cnt, rel, tl[k] | fl2);
                        if (!direct) L.seg[ps] = g;
                        else if (dok) a.seg_pool[BI((uint64_t)dc0 * SCAP + ps, seg_pool)] = g;
                        else atomicOr(&L.spill, 1ull << tl[k]);  // pool exhausted: topic spills
                        ps++;
                    };
#pragma unroll
                    for (int c = 0; c < 2; c++) {
                        const bool f = c ? f2[k] : f1[k];
                        const Rec r = c ? r2[k] : r1[k];
                        if (!f) continue;
                        const uint32_t m = info_mode(r.info);
                        if (m == M_INLINE) {
                            if ((r.info & I_INL_HASH) || last[k]) {
                                put(r.info & I_KEY_MASK, 1u, SEG_INLINE);
                                st_inl++;
                            }
                        } else if (m == M_CNT) {
                            const uint32_t tc = info_term_cnt(r.info), hc = info_hash_cnt(r.info);
                            if (last[k] && tc) put(r.child, tc, SEG_NODE);
                            if (hc) put(r.child, hc, SEG_NODE | (tc << SEG_SKIP_SHIFT));
                        } else if (m == M_REC) {
                            const uint32_t lo = a.slot_list[BI(r.child, slot_list)];
                            const uint32_t tc = a.arena[BI(lo - 2, arena)], hc = a.arena[BI(lo - 1, arena)];
                            const uint32_t ddf =
                                (OUT == O_KEYS && a.dd_bit && (a.arena[BI(lo - HDR_DD, arena)] & a.dd_bit)) ? SEG_DD : 0u;
                            st_rec++;
                            put(lo, last[k] ? tc : 0u, ddf);
                            put(lo + tc, hc, ddf);
                        }
                    }
                }
            }
            nseg = direct ? 0u : nseg + tot_s;
            st_seg += ns;
            // next frontier: children that still need a probe for level d+1
            uint32_t q1[RPL], q2[RPL];
            uint32_t np = 0;
#pragma unroll
            for (int k = 0; k < RPL; k++) {
                const uint32_t wn = last[k] ? NONE : L.wid[nxt][tl[k]];
                q1[k] = (f1[k] && !last[k]) ? probes_needed(r1[k].info, r1[k].bloom, wn) : 0u;
                q2[k] = (f2[k] && !last[k]) ? probes_needed(r2[k].info, r2[k].bloom, wn) : 0u;
                np += (uint32_t)(q1[k] != 0) + (uint32_t)(q2[k] != 0);
            }
            uint32_t tot_p;
            uint32_t pp = nnext + wave_excl_scan(np, &tot_p);
            // capacity of the next buffer: LDS + overflow chunks (grown on demand)
            uint32_t cap = FCAP + nfch[nxt] * FCH;
            if (nnext + tot_p > cap && nfch[nxt] < (uint32_t)MAXF) {
                const uint32_t want = min((nnext + tot_p - FCAP + FCH - 1) / FCH, (uint32_t)MAXF) - nfch[nxt];
                unsigned long long c0 = 0;
                if (lane == 0) c0 = atomicAdd(a.fr_cursor, (unsigned long long)want);
                c0 = __shfl(c0, 0, WAVE);
                const uint32_t got = c0 >= a.fr_chunks ? 0u : (uint32_t)min((unsigned long long)want, a.fr_chunks - c0);
                if (lane < got) L.fch[nxt][nfch[nxt] + lane] = (uint32_t)(c0 + lane);
                nfch[nxt] += got;
                cap = FCAP + nfch[nxt] * FCH;
                __syncthreads();
                st_frch += got;
            }
            // lanes write in scan order, so every lane before the first one that does not fit
            // wrote all its entries and every lane after it writes none: the buffer's valid
            // prefix ends at the first overflowing lane's position
            const bool ovf = np && pp + np > cap;
            const unsigned long long ovm = __ballot(ovf);
            if (np) {
                if (!ovf) {
#pragma unroll
                    for (int k = 0; k < RPL; k++) {
                        if (q1[k]) fr_write(nxt, pp++, r1[k].child, tl[k] | q1[k]);
                        if (q2[k]) fr_write(nxt, pp++, r2[k].child, tl[k] | q2[k]);
#if !TM_ALIVE_REG
                        if (q1[k] || q2[k]) atomicOr(&L.alive[nxt], 1ull << tl[k]);
#endif
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < RPL; k++)  // frontier overflow: those topics spill
                        if (q1[k] || q2[k]) atomicOr(&L.spill, 1ull << tl[k]);
                }
            }
            nnext = ovm ? __builtin_amdgcn_readlane(pp, __builtin_ctzll(ovm)) : nnext + tot_p;
#if TM_ALIVE_REG
            {
                unsigned long long my = 0;
                if (np && !ovf) {
#pragma unroll
                    for (int k = 0; k < RPL; k++)
                        if (q1[k] || q2[k]) my |= 1ull << tl[k];
                }
                alive_n |= wave_or64_dpp(my);
            }
#endif
#pragma unroll
            for (int k = 0; k < RPL; k++) st_visit += (uint32_t)f1[k] + (uint32_t)f2[k];
        }
        __syncthreads();
        if constexpr (STATS) {
            const uint32_t dd = d < 15u ? d : 15u;
            const uint64_t pv = wave_sum64(dp_probe);
            const uint64_t dt = __builtin_amdgcn_s_memtime() - dp_t0;
            if (lane == 0) {
                atomicAdd(&a.stats[32 + dd], (unsigned long long)pv);
                atomicAdd(&a.stats[48 + dd], (unsigned long long)dt);
                atomicAdd(&a.stats[64 + dd], (unsigned long long)nfr);
                atomicAdd(&a.stats[80 + dd], (unsigned long long)dp_rt);
            }
        }
        nfr = nnext;
#if TM_ALIVE_REG
        alive_c = alive_n;
#endif
    }

    if constexpr (STATS) ts2 = __builtin_amdgcn_s_memtime();
    // ---- 4. reserve this wave's output with one atomic; per-topic results
    const bool spill = active && !badarg && ((L.spill >> lane) & 1ull);
    const uint32_t my = (walk && !spill) ? L.cnt[lane] : 0u;
    uint32_t my_keys = 0;
    if constexpr (RUNS) my_keys = (walk && !spill) ? L.tbase[lane] : 0u;
    uint32_t total;
    const uint32_t excl = wave_excl_scan(my, &total);
    unsigned long long gb = 0;
    if (lane == 0 && total) gb = atomicAdd(a.cursor, (unsigned long long)total);
    gb = __shfl(gb, 0, WAVE);
    const bool overflow = gb + total > a.keys_cap;
    L.tbase[lane] = (uint32_t)(gb + excl);
    if (active) {
        a.status[BI(t, out)] = badarg ? 1 : 0;
        a.out_off[BI(t, out)] = spill ? 0u : (uint32_t)(gb + excl);
        a.out_cnt[BI(t, out)] = my;
        if constexpr (RUNS) a.out_kcnt[BI(t, out)] = my_keys;
    }
    if constexpr (OUT == O_IDS32 || OUT == O_IDS64) {
        const bool any_spill = __ballot(spill) != 0;
        if (lane == 0) a.wave_info[BI(blockIdx.x, wave_info)] = make_uint4((uint32_t)gb, total, any_spill ? 1u : 0u, 0u);
    }
    {
        uint32_t tot_sp;
        const uint32_t ps = wave_excl_scan(spill ? 1u : 0u, &tot_sp);
        uint32_t sb = 0;
        if (lane == 0 && tot_sp) sb = atomicAdd(a.slow_count, tot_sp);
        sb = __shfl(sb, 0, WAVE);
        if (spill) a.slow_list[BI(sb + ps, slow_list)] = t;
    }
    if constexpr (OUT == O_KEYS)
        if (a.dd_bit) L.nlev[lane] = 0;  // the walk is done with it: collapsible keys per topic
    __syncthreads();

    // ---- 5. load-balanced expansion: staged segments, then flushed chunks
    if constexpr (RUNS) {
        if (!overflow && total) {
            emit_spans(a, L, L.seg, nseg);
            for (uint32_t c = 0; c < nchunk; ++c)
                emit_spans(a, L, a.seg_pool + BIN((uint64_t)wchunks[c] * SCAP, SCAP, seg_pool), SCAP);
        }
    } else if (!overflow && total && (OUT != O_KEYS || a.mode == MODE_ALL)) {
        expand_segments<OUT>(a, L, nseg);
        for (uint32_t c = 0; c < nchunk; ++c) {
            const uint4 *src = a.seg_pool + BIN((uint64_t)wchunks[c] * SCAP, SCAP, seg_pool);
            for (uint32_t j = lane; j < (uint32_t)SCAP; j += WAVE) L.seg[j] = src[j];
            __syncthreads();
            expand_segments<OUT>(a, L, SCAP);
        }
    }
    if constexpr (OUT == O_KEYS) {
        // [unique] / aggre/1: a topic with fewer than two keys that may collapse is final as it
        // stands; the others go to k_dedupe's worklist (the walk's reads replace k_dd_pass's)
        if (a.dd_bit && !overflow && active && !spill) {
            const uint32_t pf = L.nlev[lane];
            if (walk && pf >= 2) a.wl[BI(atomicAdd(a.wl_n, 1u), out)] = make_uint2(t, pf);
            else a.ucnt[BI(t, out)] = my;
        }
    }

    if constexpr (STATS) {
        ts3 = __builtin_amdgcn_s_memtime();
        const uint64_t v0 = wave_sum64(st_visit), v1 = wave_sum64(st_probe), v2 = wave_sum64(st_wprobe),
                       v4 = wave_sum64(nl), v5 = wave_sum64(spill ? 1u : 0u), v6 = wave_sum64(st_seg),
                       v9 = wave_sum64(st_rec), v10 = wave_sum64(st_inl);
        if (lane == 0) {
            atomicAdd(&a.stats[0], (unsigned long long)v0);
            atomicAdd(&a.stats[1], (unsigned long long)v1);
            atomicAdd(&a.stats[2], (unsigned long long)v2);
            atomicAdd(&a.stats[3], (unsigned long long)total);
            atomicAdd(&a.stats[4], (unsigned long long)v4);
            atomicAdd(&a.stats[5], (unsigned long long)v5);
            atomicAdd(&a.stats[6], (unsigned long long)v6);
            atomicAdd(&a.stats[7], (unsigned long long)st_flush);
            atomicAdd(&a.stats[8], (unsigned long long)st_frch);
            atomicAdd(&a.stats[9], (unsigned long long)v9);
            atomicAdd(&a.stats[10], (unsigned long long)v10);
            atomicAdd(&a.stats[11], (unsigned long long)(ts1 - ts0));  // stage + pre-scan + root
            atomicAdd(&a.stats[12], (unsigned long long)(ts2 - ts1));  // walk
            atomicAdd(&a.stats[13], (unsigned long long)(ts3 - ts2));  // reserve + copy-out
        }
        // the same phases for waves holding a "hot" topic (> HOT_KEYS keys: under a hot '#'
        // prefix), and how many such waves there are
        constexpr uint32_t HOT_KEYS = 256;
        const bool hot_wave = __ballot(my > HOT_KEYS) != 0;
        if (lane == 0 && hot_wave) {
            atomicAdd(&a.stats[14], (unsigned long long)(ts1 - ts0));
            atomicAdd(&a.stats[15], (unsigned long long)(ts2 - ts1));
            atomicAdd(&a.stats[16], (unsigned long long)(ts3 - ts2));
            atomicAdd(&a.stats[17], 1ull);
        }
    }
}

// ---------------------------------------------------------------------------
// spill kernel: lane per topic, DFS with the stack in global scratch.
// Stack entry: slot index (40 bits; ROOT_MARK for the root) | depth (24 bits).
constexpr uint64_t ROOT_MARK = (1ull << 40) - 1;

// one key of a topic the spill kernel walks, output slot i: the key handle, (MODE_RUNS) a
// one-key span, or (MODE_IDS*) its route id
__device__ __forceinline__ void out_key(const MatchArgs &a, uint64_t i, uint32_t key) {
    if (a.mode == MODE_RUNS) {
        const uint64_t p = a.span_keys + (uint64_t)a.span_kstride * key;
        reinterpret_cast<uint4 *>(a.keys)[BI(i, keys)] = make_uint4((uint32_t)p, (uint32_t)(p >> 32), 1u, 0u);
    } else if (a.mode == MODE_IDS32) {
        a.keys[BI(i, keys)] = (uint32_t)a.key_rec[BI(2ull * key, key_rec)];
    } else if (a.mode == MODE_IDS64) {
        reinterpret_cast<uint64_t *>(a.keys)[BI(i, keys)] = a.key_rec[BI(2ull * key, key_rec)];
    } else {
        a.keys[BI(i, keys)] = key;
    }
}

template <bool WRITE>
__device__ uint32_t dfs_walk(const MatchArgs &a, const RootRec &R, const uint32_t *wid, uint64_t *stk, uint32_t nl,
                             bool dollar, uint64_t out, uint32_t *probes, uint32_t *visits, uint32_t stk_cap) {
    (void)stk_cap;  // the stack's entries (len + 2), checked by the TM_BOUNDS build
    uint32_t sp = 0, count = 0;
    stk[sp++] = ROOT_MARK << 24;
    while (sp) {
        const uint64_t ent = stk[--sp];
        const uint64_t slot = ent >> 24;
        const uint32_t d = (uint32_t)(ent & 0xFFFFFF);
        uint32_t node, info, bloom, lo = 0, tc = 0, hc = 0;
        if (slot == ROOT_MARK) {
            node = ROOT_ID;
            info = dollar ? (R.info & I_LIT) : R.info;
            bloom = R.bloom;
            lo = R.list_off;
            hc = dollar ? 0 : R.hash_cnt;
        } else {
            const uint4 x = *reinterpret_cast<const uint4 *>(a.etab + BI(slot, etab));
            node = (uint32_t)slot;
            bloom = x.z;
            info = x.w;
            const uint32_t m = info_mode(info);
            if (m == M_REC || m == M_CNT) {
                lo = a.slot_list[BI(node, slot_list)];
                tc = a.arena[BI(lo - 2, arena)];
                hc = a.arena[BI(lo - 1, arena)];
            } else if (m == M_INLINE && ((info & I_INL_HASH) || d == nl)) {
                // the node's only key, inline in the slot
                if (WRITE) out_key(a, out + count, info & I_KEY_MASK);
                count++;
            }
        }
        (*visits)++;
        // "P/#" keys match at P and below
        if (WRITE)
            for (uint32_t k = 0; k < hc; k++) out_key(a, out + count + k, a.arena[BI(lo + tc + k, arena)]);
        count += hc;
        if (d == nl) {
            if (WRITE)
                for (uint32_t k = 0; k < tc; k++) out_key(a, out + count + k, a.arena[BI(lo + k, arena)]);
            count += tc;
            continue;
        }
        const uint32_t need = probes_needed(info, bloom, wid[d]);
        Rec r;
        if ((need & DO_PLUS) && edge_probe(a, node, W_PLUS, &r, probes))
            stk[BIR(sp++, stk_cap, a.bnd)] = ((uint64_t)r.child << 24) | (d + 1);
        if ((need & DO_LIT) && edge_probe(a, node, wid[d], &r, probes))
            stk[BIR(sp++, stk_cap, a.bnd)] = ((uint64_t)r.child << 24) | (d + 1);
    }
    return count;
}

template <bool STATS>
__global__ __launch_bounds__(WAVE) void k_match_slow(MatchArgs a) {
    const uint32_t nslow = *a.slow_count;
    const RootRec R = *a.root;
    uint32_t st_visit = 0, st_probe = 0, st_wprobe = 0;
    uint64_t st_keys = 0;
    auto byte_at = [&](uint32_t i) -> uint8_t { return a.bytes[BI(i, bytes)]; };
    for (uint32_t idx = blockIdx.x * WAVE + lane_id(); idx < nslow; idx += gridDim.x * WAVE) {
        const uint32_t t = a.slow_list[BI(idx, slow_list)];
        const uint32_t b = a.off[BI(t, off)], e = a.off[BI(t + 1, off)];
        const uint32_t ns = e - b + 2;  // len+2 entries per topic
        const uint64_t sbase = BIN((uint64_t)(b - a.off[0]) + 2ull * t, ns, scratch);
        uint32_t *wid = a.scratch_w + sbase;
        uint64_t *stk = a.scratch_s + sbase;
        const bool dollar = (e > b) && byte_at(b) == '$';
        uint32_t nl = 0;
        for (uint32_t i = b;; ++i) {  // tokenise every level (the topic is not badarg)
            const uint32_t st = i;
            const uint64_t key = level_key(&i, e, byte_at);
            wid[BIR(nl++, ns, a.bnd)] = word_lookup(a, key, i - st, st, byte_at, &st_wprobe);
            if (i >= e) break;
        }
        uint32_t dummy_v = 0, dummy_p = 0;
        const uint32_t c = dfs_walk<false>(a, R, wid, stk, nl, dollar, 0, &dummy_p, &dummy_v, ns);
        const unsigned long long pos = atomicAdd(a.cursor, (unsigned long long)c);
        a.out_off[BI(t, out)] = (uint32_t)pos;
        a.out_cnt[BI(t, out)] = c;
        a.status[BI(t, out)] = 0;
        st_keys += c;
        if (a.mode == MODE_RUNS) a.out_kcnt[BI(t, out)] = c;
        if (a.mode != MODE_COUNT && pos + c <= a.keys_cap) {  // output slots: keys, spans or ids
            dfs_walk<true>(a, R, wid, stk, nl, dollar, pos, &st_probe, &st_visit, ns);
            if (a.dd_bit) {  // [unique] / aggre/1: the reducer decides (no per-list bits here)
                if (c >= 2) a.wl[BI(atomicAdd(a.wl_n, 1u), out)] = make_uint2(t, c);
                else a.ucnt[BI(t, out)] = c;
            }
        }
    }
    if constexpr (STATS) {
        // levels were already counted by the fast kernel's pre-scan
        atomicAdd(&a.stats[0], (unsigned long long)st_visit);
        atomicAdd(&a.stats[1], (unsigned long long)st_probe);
        atomicAdd(&a.stats[2], (unsigned long long)st_wprobe);
        atomicAdd(&a.stats[3], (unsigned long long)st_keys);
    }
}


// ---------------------------------------------------------------------------
// FIRST: emqx_topic_index:match/2 (return_first, emqx_trie_search.erl:171-178) — the FIRST
// matching key in ETS term order, per topic.
//
// Every key that matches topic T spells T's words at its literal levels, so two matching
// keys differ only in WHERE they have '+' / '#' / the end of the list.  Their Erlang term
// order is therefore the order of their shape codes (engine.cpp key_ord): per level END 0 <
// '#' 1 < '+' 2 < literal 3 (a shorter list sorts first; atoms '#' < '+' < any binary), two
// bits per level from bit 61 down; {Binary, {ID}} keys sort after every list (bit 62).  Equal
// codes are one filter, and the node's list header holds its smallest-id keys ({ID} tuples).
//
// k_match_first_wave (index without keys deeper than 31 levels): the level-synchronous wave
// walk of k_match_fast, with each frontier entry carrying its path's code prefix.  A
// candidate (a node's '#' keys; at the last level its word-list and binary terminal keys)
// has a code computed from that prefix alone; the wave keeps the smallest per topic (LDS
// atomicMin), then the lane holding it records where its handle lives.  A frontier entry
// whose prefix sorts after the best candidate cannot lead to a smaller key and is dropped,
// so a walk ends as soon as nothing smaller can exist.  No key lists are copied.
// k_first_dfs: lane per topic, depth-first in term order ('#' keys, then the '+' subtree,
// then the literal one), stack in global scratch: any key depth, and the spill path.
constexpr uint32_t FW_HANDLE = 0, FW_HASHLIST = 1, FW_ROOTHASH = 2;  // where the winner's handle lives
constexpr uint64_t ORD_BIN_D = 1ull << 62;

__device__ __forceinline__ uint32_t first_dfs_topic(const MatchArgs &a, const RootRec &R, uint32_t t) {
    uint32_t dummy = 0;
    auto byte_at = [&](uint32_t i) -> uint8_t { return a.bytes[i]; };
    const uint32_t b = a.off[t], e = a.off[t + 1];
    const uint64_t sbase = (uint64_t)(a.off[t] - a.off[0]) + 2ull * t;
    uint32_t *wid = a.scratch_w + sbase;
    uint64_t *stk = a.scratch_s + sbase;
    const bool dollar = (e > b) && a.bytes[b] == '$';
    uint32_t nl = 0;
    for (uint32_t i = b;; ++i) {
        const uint32_t st = i;
        const uint64_t key = level_key(&i, e, byte_at);
        wid[nl++] = word_lookup(a, key, i - st, st, byte_at, &dummy);
        if (i >= e) break;
    }
    uint32_t best = NONE, bbest = NONE;
    uint32_t sp = 0;
    stk[sp++] = ROOT_MARK << 24;
    while (sp) {
        const uint64_t ent = stk[--sp];
        const uint64_t slot = ent >> 24;
        const uint32_t d = (uint32_t)(ent & 0xFFFFFF);
        // the node's return_first candidates: its smallest-id {Binary,{ID}} term key,
        // word-list term key and '#' key (list header, or the inline key)
        uint32_t node, info, bloom, tb = NONE, tw = NONE, th = NONE;
        if (slot == ROOT_MARK) {
            node = ROOT_ID;
            info = dollar ? (R.info & I_LIT) : R.info;
            bloom = R.bloom;
            if (!dollar && R.hash_cnt) th = a.arena[R.list_off - 3];
        } else {
            const uint4 x = *reinterpret_cast<const uint4 *>(a.etab + BI(slot, etab));
            node = (uint32_t)slot;
            bloom = x.z;
            info = x.w;
            const uint32_t m = info_mode(info);
            if (m == M_REC || m == M_CNT) {
                const uint32_t lo = a.slot_list[node];
                tb = a.arena[lo - 5];
                tw = a.arena[lo - 4];
                th = a.arena[lo - 3];
            } else if (m == M_INLINE) {
                const uint32_t k = info & I_KEY_MASK;
                if (info & I_INL_HASH) th = k;
                else if (a.key_bin[k]) tb = k;
                else tw = k;
            }
        }
        if (d == nl) {  // P + end of list, then P + '#'; binaries only if no list matches
            if (tb != NONE) bbest = tb;  // only the all-literal path holds binary keys
            best = tw != NONE ? tw : th;
            if (best != NONE) break;
            continue;
        }
        if (th != NONE) {  // P + '#'
            best = th;
            break;
        }
        // children: the '+' subtree before the literal one (pushed last, popped first)
        const uint32_t need = probes_needed(info, bloom, wid[d]);
        Rec r;
        if ((need & DO_LIT) && edge_probe(a, node, wid[d], &r, &dummy)) stk[sp++] = ((uint64_t)r.child << 24) | (d + 1);
        if ((need & DO_PLUS) && edge_probe(a, node, W_PLUS, &r, &dummy)) stk[sp++] = ((uint64_t)r.child << 24) | (d + 1);
    }
    return best == NONE ? bbest : best;
}

__device__ __forceinline__ bool topic_badarg(const MatchArgs &a, uint32_t t) {
    const uint32_t b = a.off[t], e = a.off[t + 1];
    bool badarg = false;
    for (uint32_t i = b, st = b;; ++i) {
        const bool end = i == e;
        if (end || a.bytes[i] == '/') {
            if (i - st == 1 && (a.bytes[st] == '+' || a.bytes[st] == '#') && !a.topic_words) badarg = true;
            st = i + 1;
            if (end) break;
        }
    }
    return badarg;
}

// every topic, lane per topic (indexes holding keys deeper than the 31-level code)
__global__ __launch_bounds__(WAVE) void k_match_first(MatchArgs a) {
    const RootRec R = *a.root;
    if (blockIdx.x == 0 && threadIdx.x < CTL_BYTES / 8) a.ctl_next[threadIdx.x] = 0ull;  // next launch's counters
    for (uint32_t t = blockIdx.x * WAVE + lane_id(); t < a.n; t += gridDim.x * WAVE) {
        const bool badarg = topic_badarg(a, t);
        a.out_off[t] = t;
        a.status[t] = badarg ? 1 : 0;
        const uint32_t k = badarg ? NONE : first_dfs_topic(a, R, t);
        a.out_cnt[t] = k != NONE ? 1u : 0u;
        a.keys[t] = k;
    }
}

// the topics k_match_first_wave handed off (frontier pool exhausted, or the test aid)
__global__ __launch_bounds__(WAVE) void k_first_slow(MatchArgs a) {
    const uint32_t nslow = *a.slow_count;
    const RootRec R = *a.root;
    for (uint32_t idx = blockIdx.x * WAVE + lane_id(); idx < nslow; idx += gridDim.x * WAVE) {
        const uint32_t t = a.slow_list[idx];
        const uint32_t k = first_dfs_topic(a, R, t);
        a.out_cnt[t] = k != NONE ? 1u : 0u;
        a.keys[t] = k;
    }
}

#ifndef TM_FCAP_FIRST
#define TM_FCAP_FIRST 256  // k_match_first_wave's frontier entries per depth in LDS (13 B each: node, code, meta); 256: 10,776 B, 15 waves/CU (0.567 -> 0.509 ms vs 384)
#endif
constexpr int FCAP_F = TM_FCAP_FIRST;
struct FirstLds {
    uint8_t tb[TBCAP];
    uint32_t fr_node[2][FCAP_F];
    uint64_t fr_ord[2][FCAP_F];      // code prefix of the entry's path (levels < depth)
    uint8_t fr_meta[2][FCAP_F];      // topic lane | DO_PLUS / DO_LIT
    uint32_t fch[2][MAXF];         // overflow chunks (uint4 entries {node, meta, ord lo, ord hi})
    uint32_t wid[2][WAVE];
    uint32_t nlev[WAVE];
    unsigned long long best[WAVE];  // smallest candidate code so far (~0: none)
    unsigned long long win[WAVE];   // its handle, or where it lives: value | FW_* << 32
    unsigned long long spill;
    unsigned long long alive[2];
};
constexpr uint32_t FCH4 = FCH / 2;  // uint4 entries per overflow chunk (the pool is sized in uint2)

__global__ __launch_bounds__(WAVE) void k_match_first_wave(MatchArgs a) {
    __shared__ FirstLds L;
    const uint32_t lane = lane_id();
    const uint32_t t = blockIdx.x * a.tpw + lane;
    const bool active = lane < a.tpw && t < a.n;
    if (blockIdx.x == 0 && threadIdx.x < CTL_BYTES / 8) a.ctl_next[threadIdx.x] = 0ull;  // next launch's counters
    uint4 *const pool4 = reinterpret_cast<uint4 *>(a.fr_pool);

    // ---- stage the wave's topic bytes (as k_match_fast)
    const uint32_t t0 = blockIdx.x * a.tpw;
    const uint32_t wb0 = a.off[BI(t0, off)], wb1 = a.off[BI(min(t0 + a.tpw, a.n), off)];
    const uint32_t tbase = wb0 & ~15u;
    const bool staged = ((reinterpret_cast<uintptr_t>(a.bytes) & 15u) == 0) && (wb1 - tbase <= (uint32_t)TBCAP);
    if (staged) {
        for (uint32_t j = lane * 16; tbase + j < wb1; j += WAVE * 16) {
            if (tbase + j + 16 <= wb1) {
                *reinterpret_cast<uint4 *>(&L.tb[j]) = *reinterpret_cast<const uint4 *>(a.bytes + BIN(tbase + j, 16, bytes));
            } else {
                for (uint32_t k = 0; tbase + j + k < wb1; k++) L.tb[j + k] = a.bytes[BI(tbase + j + k, bytes)];
            }
        }
        __syncthreads();
    }
    auto byte_at = [&](uint32_t i) -> uint8_t { return staged ? L.tb[i - tbase] : a.bytes[BI(i, bytes)]; };

    bool badarg = false, dollar = false;
    uint32_t nl = 0, b = 0, e = 0;
    uint32_t dummy = 0;
#if TM_PRELOOK
    uint32_t widr[TM_PRELOOK];
    uint32_t pre_b = 0;
    if (active) {
        b = a.off[BI(t, off)];
        e = a.off[BI(t + 1, off)];
        dollar = (e > b) && byte_at(b) == '$';
        TM_PRESCAN_PRELOOK(dummy);
    }
    uint32_t cur_b = pre_b;
#else
    if (active) {
        b = a.off[BI(t, off)];
        e = a.off[BI(t + 1, off)];
        dollar = (e > b) && byte_at(b) == '$';
        uint32_t st = b;
        for (uint32_t i = b;; ++i) {
            const bool end = i == e;
            const uint8_t c = end ? (uint8_t)'/' : byte_at(i);
            if (c == '/') {
                if (i - st == 1 && (byte_at(st) == '+' || byte_at(st) == '#') && !a.topic_words) badarg = true;
                nl++;
                st = i + 1;
                if (end) break;
            }
        }
    }
    uint32_t cur_b = b;
#endif
    const bool spill0 = active && !badarg && a.force_slow;
    const bool walk = active && !badarg && !spill0;
    L.nlev[lane] = nl;
    L.best[lane] = ~0ull;
    L.win[lane] = 0;
    {
        const unsigned long long sp0 = __ballot(spill0);
        if (lane == 0) {
            L.spill = sp0;
            L.alive[0] = 0;
            L.alive[1] = 0;
        }
    }
    auto level_word = [&](uint32_t slot, uint32_t lv) {  // level lv's word id (lv wave-uniform)
#if TM_PRELOOK
        if (lv < (uint32_t)TM_PRELOOK) {
            L.wid[slot][lane] = prelook_word(widr, lv);
            return;
        }
#endif
        (void)lv;
        uint32_t i = cur_b;
        const uint32_t st = i;
        const uint64_t key = level_key(&i, e, byte_at);
        L.wid[slot][lane] = word_lookup(a, key, i - st, st, byte_at, &dummy);
        cur_b = i + 1;
    };

    // ---- root: a root '#' key (code '#' at level 0) is the smallest any topic can match
    const RootRec R = *a.root;
    if (walk) level_word(0, 0);
    uint32_t nfr;
#if TM_ALIVE_REG
    unsigned long long alive_c = 0;  // wave-uniform: topics with frontier entries at this depth
#endif
    {
        const bool rh = walk && !dollar && R.hash_cnt;
        if (rh) {
            L.best[lane] = 1ull << 60;
            L.win[lane] = (unsigned long long)FW_ROOTHASH << 32;
        }
        const uint32_t rinfo = dollar ? (R.info & I_LIT) : R.info;
        const uint32_t m = (walk && !rh) ? probes_needed(rinfo, R.bloom, L.wid[0][lane]) : 0u;
        const unsigned long long al0 = __ballot(m != 0);
        if (lane == 0) L.alive[0] = al0;
#if TM_ALIVE_REG
        alive_c = al0;
#endif
        uint32_t tot;
        const uint32_t p2 = wave_excl_scan(m ? 1u : 0u, &tot);
        if (m) {
            L.fr_node[0][p2] = ROOT_ID;
            L.fr_meta[0][p2] = (uint8_t)(lane | m);
            L.fr_ord[0][p2] = 0ull;
        }
        nfr = tot;
    }
    __syncthreads();

    uint32_t nfch[2] = {0, 0};
    auto fr_read = [&](uint32_t lvl, uint32_t i, uint32_t &node, uint32_t &meta, uint64_t &ord) {
        if (i < (uint32_t)FCAP_F) {
            node = L.fr_node[lvl][i];
            meta = L.fr_meta[lvl][i];
            ord = L.fr_ord[lvl][i];
        } else {
            const uint32_t k = i - FCAP_F;
            const uint4 v = pool4[(uint64_t)L.fch[lvl][k / FCH4] * FCH4 + k % FCH4];
            node = v.x;
            meta = v.y;
            ord = ((uint64_t)v.w << 32) | v.z;
        }
    };
    auto fr_write = [&](uint32_t lvl, uint32_t i, uint32_t node, uint32_t meta, uint64_t ord) {
        if (i < (uint32_t)FCAP_F) {
            L.fr_node[lvl][i] = node;
            L.fr_meta[lvl][i] = (uint8_t)meta;
            L.fr_ord[lvl][i] = ord;
        } else {
            const uint32_t k = i - FCAP_F;
            pool4[(uint64_t)L.fch[lvl][k / FCH4] * FCH4 + k % FCH4] =
                make_uint4(node, meta, (uint32_t)ord, (uint32_t)(ord >> 32));
        }
    };

    // Without word-list keys deeper than the code (31 levels; '#' keys 30), only {Binary, {ID}}
    // keys hang below depth 31, and only on the all-literal path: past depth 30 the walk
    // follows that path alone (code prefix ALL_LIT) and looks for binary terminal keys.
    constexpr uint64_t ALL_LIT = (1ull << 62) - 1;
    for (uint32_t d = 0; nfr > 0; ++d) {
        const uint32_t cur = d & 1, nxt = cur ^ 1;
#if TM_ALIVE_REG
        if (walk && ((alive_c >> lane) & 1ull) && d + 1 < nl) level_word(nxt, d + 1);
        unsigned long long alive_n = 0;  // wave-uniform
#else
        if (walk && ((L.alive[cur] >> lane) & 1ull) && d + 1 < nl) level_word(nxt, d + 1);
        if (lane == 0) L.alive[nxt] = 0;
#endif
        __syncthreads();
        uint32_t nnext = 0;
        // a child at depth d+1 adds its level-d symbol ('+' 2, literal 3) at bit sh; its '#'
        // keys have '#' (1) at level d+1, bit sh-2 (none when d == 30: no such keys)
        const bool deep = d > 30;
        const uint32_t sh = deep ? 0u : 60 - 2 * d;
        const uint64_t hbit = (!deep && sh >= 2) ? 1ull << (sh - 2) : 0ull;
        for (uint32_t base = 0; base < nfr; base += WAVE * RPL) {
            uint32_t tl[RPL];
            bool last[RPL], f1[RPL], f2[RPL];
            Rec r1[RPL], r2[RPL];
            uint64_t pre[RPL];
            {
                uint32_t node[RPL], w[RPL];
                bool p1[RPL], p2[RPL];
                uint64_t s1[RPL], s2[RPL];
#pragma unroll
                for (int k = 0; k < RPL; k++) {
                    const uint32_t i = base + k * WAVE + lane;
                    bool has = i < nfr;
                    uint32_t meta = 0;
                    node[k] = 0;
                    pre[k] = 0;
                    if (has) fr_read(cur, i, node[k], meta, pre[k]);
                    tl[k] = meta & 63u;
                    // nothing under this entry can sort before the topic's best candidate
                    if (has && (L.best[tl[k]] < pre[k] || (deep && pre[k] != ALL_LIT))) has = false;
                    w[k] = has ? L.wid[cur][tl[k]] : NONE;
                    last[k] = has && (d + 1 == L.nlev[tl[k]]);
                    p1[k] = has && (meta & DO_LIT);
                    p2[k] = has && !deep && (meta & DO_PLUS);
                    s1[k] = edge_home(node[k], w[k], a.emask);
                    s2[k] = edge_home(node[k], W_PLUS, a.emask);
                    f1[k] = f2[k] = false;
                }
                for (;;) {
                    bool any = false;
#pragma unroll
                    for (int k = 0; k < RPL; k++) any = any || p1[k] || p2[k];
                    if (!any) break;
                    uint4 x1[RPL], x2[RPL];
#pragma unroll
                    for (int k = 0; k < RPL; k++) {
                        x1[k] = p1[k] ? *reinterpret_cast<const uint4 *>(a.etab + BI(s1[k], etab)) : make_uint4(NONE, 0, 0, 0);
                        x2[k] = p2[k] ? *reinterpret_cast<const uint4 *>(a.etab + BI(s2[k], etab)) : make_uint4(NONE, 0, 0, 0);
                    }
#pragma unroll
                    for (int k = 0; k < RPL; k++) {
                        if (p1[k]) {
                            if (x1[k].x == NONE) p1[k] = false;
                            else if (x1[k].x == node[k] && x1[k].y == w[k]) {
                                r1[k] = Rec{(uint32_t)s1[k], x1[k].z, x1[k].w};
                                f1[k] = true;
                                p1[k] = false;
                            } else s1[k] = next_slot(s1[k], a.emask);
                        }
                        if (p2[k]) {
                            if (x2[k].x == NONE) p2[k] = false;
                            else if (x2[k].x == node[k] && x2[k].y == W_PLUS) {
                                r2[k] = Rec{(uint32_t)s2[k], x2[k].z, x2[k].w};
                                f2[k] = true;
                                p2[k] = false;
                            } else s2[k] = next_slot(s2[k], a.emask);
                        }
                    }
                }
            }
            // candidates of each found child (depth d+1): its '#' keys (code P'|'#' at level
            // d+1) and, at the topic's last level, its word-list terminal keys (code P') and
            // binary ones (after every list)
            uint64_t cord[RPL][2][2];  // [entry][child][0: '#', 1: terminal] code (~0: none)
            uint64_t cwin[RPL][2][2];
#pragma unroll
            for (int k = 0; k < RPL; k++) {
#pragma unroll
                for (int c = 0; c < 2; c++) {
                    cord[k][c][0] = cord[k][c][1] = ~0ull;
                    cwin[k][c][0] = cwin[k][c][1] = 0;
                    const bool f = c ? f2[k] : f1[k];
                    if (!f) continue;
                    const Rec r = c ? r2[k] : r1[k];
                    const uint64_t P = deep ? pre[k] : pre[k] | ((uint64_t)(c ? 2u : 3u) << sh);
                    const uint32_t m = info_mode(r.info);
                    uint32_t hc = 0, tcnt = 0, lo = 0;
                    if (m == M_INLINE) {
                        const uint32_t key = r.info & I_KEY_MASK;
                        if (r.info & I_INL_HASH) {
                            if (hbit) {
                                cord[k][c][0] = P | hbit;
                                cwin[k][c][0] = key;
                            }
                        } else if (last[k]) {
                            cord[k][c][1] = a.key_bin[key] ? ORD_BIN_D : P;
                            cwin[k][c][1] = key;
                        }
                    } else if (m == M_CNT) {
                        hc = info_hash_cnt(r.info);
                        tcnt = info_term_cnt(r.info);
                    } else if (m == M_REC) {
                        lo = a.slot_list[r.child];
                        tcnt = a.arena[lo - 2];
                        hc = a.arena[lo - 1];
                    }
                    if (hc && hbit) {
                        cord[k][c][0] = P | hbit;
                        cwin[k][c][0] = ((unsigned long long)FW_HASHLIST << 32) | r.child;
                    }
                    if (last[k] && tcnt) {  // which terminal kinds: the list header's min-id keys
                        if (m == M_CNT) lo = a.slot_list[r.child];
                        const uint32_t tw = a.arena[lo - 4], tb = a.arena[lo - 5];
                        if (tw != NONE) {
                            cord[k][c][1] = P;
                            cwin[k][c][1] = tw;
                        } else if (tb != NONE) {
                            cord[k][c][1] = ORD_BIN_D;
                            cwin[k][c][1] = tb;
                        }
                    }
#pragma unroll
                    for (int j = 0; j < 2; j++)
                        if (cord[k][c][j] != ~0ull) atomicMin(&L.best[tl[k]], (unsigned long long)cord[k][c][j]);
                }
            }
            __syncthreads();
            // the lane holding a topic's smallest code records its handle (codes are unique
            // per topic: the code and the topic's words determine the filter)
#pragma unroll
            for (int k = 0; k < RPL; k++)
#pragma unroll
                for (int c = 0; c < 2; c++)
#pragma unroll
                    for (int j = 0; j < 2; j++)
                        if (cord[k][c][j] != ~0ull && cord[k][c][j] == L.best[tl[k]]) L.win[tl[k]] = cwin[k][c][j];
            // next frontier: children still needing a probe whose prefix can still win
            uint32_t q1[RPL], q2[RPL];
            uint64_t P1[RPL], P2[RPL];
            uint32_t np = 0;
#pragma unroll
            for (int k = 0; k < RPL; k++) {
                const uint32_t wn = last[k] ? NONE : L.wid[nxt][tl[k]];
                P1[k] = deep ? pre[k] : pre[k] | (3ull << sh);
                P2[k] = deep ? pre[k] : pre[k] | (2ull << sh);
                const unsigned long long bt = L.best[tl[k]];
                // a child at depth d+1 > 30 matters only on the all-literal path (binary keys)
                const bool deeper = !last[k] && (d + 1 <= 30 || P1[k] == ALL_LIT);
                q1[k] = (f1[k] && deeper && !(bt < P1[k])) ? probes_needed(r1[k].info, r1[k].bloom, wn) : 0u;
                q2[k] = (f2[k] && deeper && d + 1 <= 30 && !(bt < P2[k])) ? probes_needed(r2[k].info, r2[k].bloom, wn) : 0u;
                np += (uint32_t)(q1[k] != 0) + (uint32_t)(q2[k] != 0);
            }
            uint32_t tot_p;
            uint32_t pp = nnext + wave_excl_scan(np, &tot_p);
            uint32_t cap = FCAP_F + nfch[nxt] * FCH4;
            if (nnext + tot_p > cap && nfch[nxt] < (uint32_t)MAXF) {
                const uint32_t want = min((nnext + tot_p - FCAP_F + FCH4 - 1) / FCH4, (uint32_t)MAXF) - nfch[nxt];
                unsigned long long c0 = 0;
                if (lane == 0) c0 = atomicAdd(a.fr_cursor, (unsigned long long)want);
                c0 = __shfl(c0, 0, WAVE);
                const uint32_t got = c0 >= a.fr_chunks ? 0u : (uint32_t)min((unsigned long long)want, a.fr_chunks - c0);
                if (lane < got) L.fch[nxt][nfch[nxt] + lane] = (uint32_t)(c0 + lane);
                nfch[nxt] += got;
                cap = FCAP_F + nfch[nxt] * FCH4;
                __syncthreads();
            }
            const bool ovf = np && pp + np > cap;
            const unsigned long long ovm = __ballot(ovf);
            if (np) {
                if (!ovf) {
#pragma unroll
                    for (int k = 0; k < RPL; k++) {
                        if (q1[k]) fr_write(nxt, pp++, r1[k].child, tl[k] | q1[k], P1[k]);
                        if (q2[k]) fr_write(nxt, pp++, r2[k].child, tl[k] | q2[k], P2[k]);
#if !TM_ALIVE_REG
                        if (q1[k] || q2[k]) atomicOr(&L.alive[nxt], 1ull << tl[k]);
#endif
                    }
                } else {
#pragma unroll
                    for (int k = 0; k < RPL; k++)  // frontier overflow: those topics take the DFS
                        if (q1[k] || q2[k]) atomicOr(&L.spill, 1ull << tl[k]);
                }
            }
            nnext = ovm ? __builtin_amdgcn_readlane(pp, __builtin_ctzll(ovm)) : nnext + tot_p;
#if TM_ALIVE_REG
            {
                unsigned long long my = 0;
                if (np && !ovf) {
#pragma unroll
                    for (int k = 0; k < RPL; k++)
                        if (q1[k] || q2[k]) my |= 1ull << tl[k];
                }
                alive_n |= wave_or64_dpp(my);
            }
#endif
            __syncthreads();
        }
        __syncthreads();
        nfr = nnext;
#if TM_ALIVE_REG
        alive_c = alive_n;
#endif
    }

    // ---- results: the winner's handle (one more read for a '#' list), or the DFS for spills
    const bool spill = active && !badarg && ((L.spill >> lane) & 1ull);
    if (active) {
        a.out_off[t] = t;
        a.status[t] = badarg ? 1 : 0;
        if (!spill) {
            uint32_t k = NONE;
            const unsigned long long wv = L.win[lane];
            if (walk && L.best[lane] != ~0ull) {
                const uint32_t kind = (uint32_t)(wv >> 32), v = (uint32_t)wv;
                k = kind == FW_HANDLE ? v : kind == FW_ROOTHASH ? a.arena[R.list_off - 3] : a.arena[a.slot_list[v] - 3];
            }
            a.out_cnt[t] = k != NONE ? 1u : 0u;
            a.keys[t] = k;
        }
    }
    {
        uint32_t tot_sp;
        const uint32_t ps = wave_excl_scan(spill ? 1u : 0u, &tot_sp);
        uint32_t sb = 0;
        if (lane == 0 && tot_sp) sb = atomicAdd(a.slow_count, tot_sp);
        sb = __shfl(sb, 0, WAVE);
        if (spill) a.slow_list[BI(sb + ps, slow_list)] = t;
    }
}

// ---------------------------------------------------------------------------
__global__ void k_scatter16(uint4 *dst, const uint64_t *idx, const uint4 *src, uint64_t n, uint64_t cap,
                            unsigned long long *bnd) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[BIR(idx[i], cap, bnd)] = src[i];
}

__global__ void k_scatter4(uint32_t *dst, const uint64_t *idx, const uint32_t *src, uint64_t n, uint64_t cap,
                           unsigned long long *bnd) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[BIR(idx[i], cap, bnd)] = src[i];
}

hipError_t launch_scatter16(uint4 *dst, const uint64_t *idx, const uint4 *src, uint64_t n, hipStream_t s,
                            uint64_t cap, unsigned long long *bnd) {
    if (!n) return hipSuccess;
    k_scatter16<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dst, idx, src, n, cap, bnd);
    return hipGetLastError();
}

hipError_t launch_scatter4(uint32_t *dst, const uint64_t *idx, const uint32_t *src, uint64_t n, hipStream_t s,
                           uint64_t cap, unsigned long long *bnd) {
    if (!n) return hipSuccess;
    k_scatter4<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dst, idx, src, n, cap, bnd);
    return hipGetLastError();
}

hipError_t launch_match(const MatchArgs &a, hipStream_t s) {
    hipError_t e;
    // this launch's counters were zeroed by the previous launch (or at allocation); it
    // zeroes the next launch's block itself — only an empty batch, which launches no
    // kernel, does that with a memset
    if (a.n == 0) return hipMemsetAsync(a.ctl_next, 0, CTL_BYTES, s);
    const unsigned grid = (unsigned)match_grid(a.n, a.tpw);
    if (a.mode == MODE_FIRST) {  // <= 1 key per topic at keys[t]; cursor stays 0
        if (a.ev_fast0 && (e = hipEventRecord(a.ev_fast0, s))) return e;
        if (a.first_dfs) {  // keys deeper than the 31-level code: lane-per-topic DFS
            k_match_first<<<grid < 4096u ? grid : 4096u, WAVE, 0, s>>>(a);
            if ((e = hipGetLastError())) return e;
            if (a.ev_fast1 && (e = hipEventRecord(a.ev_fast1, s))) return e;
            return hipSuccess;
        }
        k_match_first_wave<<<grid, WAVE, 0, s>>>(a);
        if ((e = hipGetLastError())) return e;
        if (a.ev_fast1 && (e = hipEventRecord(a.ev_fast1, s))) return e;
        k_first_slow<<<grid < 2048u ? grid : 2048u, WAVE, 0, s>>>(a);
        return hipGetLastError();
    }
    if (a.ev_fast0 && (e = hipEventRecord(a.ev_fast0, s))) return e;  // (the timed span includes k_prescan)
#if TM_PRELOOK
    // (not the ids copy-outs: at PRE's 5 waves per SIMD their id arrays went to scratch)
    if (a.pre_wid && a.mode != MODE_IDS32 && a.mode != MODE_IDS64) {
        const unsigned pgrid = (unsigned)(((uint64_t)a.n + WAVE - 1) / WAVE);
        if (a.stats) k_prescan<true><<<pgrid, WAVE, 0, s>>>(a);
        else k_prescan<false><<<pgrid, WAVE, 0, s>>>(a);
        if ((e = hipGetLastError())) return e;
        if (a.mode == MODE_RUNS) {
            if (a.stats) k_match_fast<true, O_RUNS, true><<<grid, WAVE, 0, s>>>(a);
            else k_match_fast<false, O_RUNS, true><<<grid, WAVE, 0, s>>>(a);
        } else {
            if (a.stats) k_match_fast<true, O_KEYS, true><<<grid, WAVE, 0, s>>>(a);
            else k_match_fast<false, O_KEYS, true><<<grid, WAVE, 0, s>>>(a);
        }
    } else
#endif
    if (a.mode == MODE_RUNS) {
        if (a.stats) k_match_fast<true, O_RUNS, false><<<grid, WAVE, 0, s>>>(a);
        else k_match_fast<false, O_RUNS, false><<<grid, WAVE, 0, s>>>(a);
    } else if (a.mode == MODE_IDS32) {
        k_match_fast<false, O_IDS32, false><<<grid, WAVE, 0, s>>>(a);
    } else if (a.mode == MODE_IDS64) {
        k_match_fast<false, O_IDS64, false><<<grid, WAVE, 0, s>>>(a);
    } else {
        if (a.stats) k_match_fast<true, O_KEYS, false><<<grid, WAVE, 0, s>>>(a);
        else k_match_fast<false, O_KEYS, false><<<grid, WAVE, 0, s>>>(a);
    }
    if ((e = hipGetLastError())) return e;
    if (a.ev_fast1 && (e = hipEventRecord(a.ev_fast1, s))) return e;
    // spill kernel: fixed grid, grid-stride over the device-side spill list
    const unsigned sgrid = grid < 2048u ? grid : 2048u;
    if (a.stats) k_match_slow<true><<<sgrid, WAVE, 0, s>>>(a);
    else k_match_slow<false><<<sgrid, WAVE, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace tmx
