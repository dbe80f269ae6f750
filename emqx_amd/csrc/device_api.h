// device_api.h — private interface between the host engine (engine.cpp) and
// the gfx950 kernels (match_kernels.hip).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "layout.h"

namespace tmx {

constexpr uint32_t MODE_ALL = 0, MODE_COUNT = 1, MODE_FIRST = 2;  // MatchArgs.mode
// MODE_RUNS: instead of copying keys, every key segment the walk found (a run of consecutive
// arena keys, or one inline key) is written as a host span {const uint64_t *ids, uint64_t n}
// (include/emqx_tm.h tm_span): keys points at uint4 spans, keys_cap counts spans, cursor
// counts spans, out_cnt[t] = topic t's spans, out_kcnt[t] = its keys.
constexpr uint32_t MODE_RUNS = 3;
// MODE_IDS32 / MODE_IDS64: the copy-out writes each key's route id (key_rec[2h], the id word of
// its {id, order code} record) instead of its handle, as u32 (every id < 2^32) or u64: keys
// points at the caller's id buffer, keys_cap counts ids (emqx_router:match_to_route/1,
// apps/emqx/src/emqx_router.erl:648-649, fused into the walk: no separate k_result_ids pass).
constexpr uint32_t MODE_IDS32 = 4, MODE_IDS64 = 5;
constexpr int SEG_CHUNK = 128;  // key segments per global chunk (16 B each)
constexpr int SEG_MAXCHUNK = 128;  // segment chunks one wave may flush (its list lives in HBM)
constexpr int FR_CHUNK = 256;   // frontier entries per global overflow chunk (8 B each)

// Counter block of one launch (byte offsets); the engine alternates two of them.
constexpr uint32_t CTL_BYTES = 32, CTL_CURSOR = 0, CTL_SLOW = 8, CTL_SEG = 16, CTL_FR = 24;

// ---------------------------------------------------------------------------
// TM_BOUNDS=1: the debug build (libemqx_tm_bounds.so).  Every index the match,
// upload and scatter kernels compute into an engine buffer goes through BI(i, cap): in the
// debug build an index at or past the buffer's real capacity is recorded in the engine's bounds
// record {count, source line, index, capacity} and replaced by 0, so the launch cannot fault and
// the host reports the first offending access (tm_debug_bounds).  In the product build BI(i, cap)
// is i.
#ifndef TM_BOUNDS
#define TM_BOUNDS 0
#endif
// the recorded source line's file: 1 match_kernels.hip, 2 result_kernels.hip, 3 filter_kernels.hip
#ifndef TM_BND_FILE
#define TM_BND_FILE 0
#endif
struct BndCaps {
    uint64_t bytes, off, wtab, warena, word_off, etab, slot_list, arena, key_bin, key_rec, key_dd;  // inputs, index
    uint64_t out, keys, slow_list, scratch, seg_pool, wave_chunks, fr_pool, wave_info;     // outputs, scratch
    uint64_t pre_wid, pre_meta;                                                              // k_prescan
};
#if TM_BOUNDS && defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ uint64_t tm_bchk(uint64_t i, uint64_t cap, uint32_t line, unsigned long long *rec) {
    if (i < cap) return i;
    if (rec && atomicAdd(&rec[0], 1ull) == 0) {
        atomicExch(&rec[1], (unsigned long long)line);
        atomicExch(&rec[2], (unsigned long long)i);
        atomicExch(&rec[3], (unsigned long long)cap);
    }
    return 0;
}
// n elements from i (a 16-B load of bytes, a chunk of a pool): i if they all fit, else 0
__device__ __forceinline__ uint64_t tm_bchk_n(uint64_t i, uint64_t n, uint64_t cap, uint32_t line,
                                              unsigned long long *rec) {
    if (i + n <= cap) return i;
    tm_bchk(i + n - 1, cap, line, rec);  // records the last element's index
    return 0;
}
#define TM_BND_WHERE ((uint32_t)(TM_BND_FILE << 24) | (uint32_t)__LINE__)
#define BIR(i, cap, rec) ::tmx::tm_bchk((uint64_t)(i), (cap), TM_BND_WHERE, (rec))
#define BIRN(i, n, cap, rec) ::tmx::tm_bchk_n((uint64_t)(i), (uint64_t)(n), (cap), TM_BND_WHERE, (rec))
#else
#define BIR(i, cap, rec) (i)
#define BIRN(i, n, cap, rec) (i)
#endif
#define BI(i, capfield) BIR(i, a.cap.capfield, a.bnd)
#define BIN(i, n, capfield) BIRN(i, n, a.cap.capfield, a.bnd)

// Everything one match launch needs.  Device pointers only.
struct MatchArgs {
    // topic batch: topic i is bytes[off[i] .. off[i+1])
    const uint8_t *bytes;
    const uint32_t *off;
    uint32_t n;
    uint32_t force_slow;  // 1: every topic takes the spill kernel (test aid)
    uint32_t mode;        // MODE_ALL: every key; MODE_COUNT: counts only; MODE_FIRST: k_match_first
    uint32_t tpw;         // topics per wave of k_match_fast (pick_tpw)
    uint32_t first_dfs;   // MODE_FIRST: 1 = lane-per-topic DFS (index holds keys deeper than the
                          // 31-level order code), 0 = k_match_first_wave + k_first_slow
    uint32_t topic_words; // 1: topics are '/'-joined word lists (matches/3's [word()] form): a
                          // "+" or "#" level is a literal word, not badarg (emqx_trie_search.erl:369-370)
    // frozen index
    const WordSlot *wtab;
    uint64_t wmask;
    const uint8_t *warena;
    const uint32_t *word_off;  // arena offset of each word (long-word verification)
    const EdgeSlot *etab;
    uint64_t emask;
    const uint32_t *slot_list; // node (= slot) -> first key of its list in the arena
    const RootRec *root;
    const uint32_t *arena;
    const uint32_t *key_bin;   // key handle -> 1 for {Binary, {ID}} keys (sort after word lists)
    const uint64_t *key_rec;   // MODE_IDS*: 2 u64 per key handle {id, order code}
    // results
    uint32_t *out_off;
    uint32_t *out_cnt;
    int32_t *status;
    uint32_t *keys;
    uint64_t keys_cap;
    // MODE_RUNS
    uint32_t *out_kcnt;
    uint64_t span_arena;  // host address of the id arena: an arena run at src spans span_arena + span_w * src
    uint64_t span_keys;   // host address of key handle 0's id: key h's id is at span_keys + span_kstride * h
    uint32_t span_w;       // 8: the u64 id arena; 4: the u32 one
    uint32_t span_kstride; // bytes between consecutive keys' ids (16: KeyRec.id; 4: key_id32)
    unsigned long long *cursor;  // keys requested so far (may exceed keys_cap)
    // the counters (cursor, slow_count, seg_cursor, fr_cursor) share one CTL_BYTES block;
    // the launch zeroes the block the next launch will use (no memsets before a batch)
    unsigned long long *ctl_next;
    // spill path
    uint32_t *slow_list;
    uint32_t *slow_count;
    uint32_t *scratch_w;  // (total bytes + 2n + 2) u32: word ids, at off[t]-off[0] + 2t
    uint64_t *scratch_s;  // (total bytes + 2n + 2) u64: DFS stack, same indexing
    // MODE_IDS*: per wave {output base, ids, 1 if a topic of the wave spilled, 0}: a wave's
    // topics are contiguous and in order in its output range, so the topic-major compaction
    // moves whole wave blocks (launch_compact_waves)
    uint4 *wave_info;
    // segment chunk pool (wave LDS overflow): seg_chunks chunks of SEG_CHUNK uint4
    uint4 *seg_pool;
    uint64_t seg_chunks;
    unsigned long long *seg_cursor;  // chunks requested (may exceed seg_chunks)
    uint32_t *wave_chunks;           // SEG_MAXCHUNK chunk indices per wave (grid * SEG_MAXCHUNK)
    // frontier overflow pool: fr_chunks chunks of FR_CHUNK uint2 {node, meta}
    uint2 *fr_pool;
    uint64_t fr_chunks;
    unsigned long long *fr_cursor;
    // optional walk statistics (nullptr = off): [0] node visits, [1] edge-slot
    // probes, [2] word-slot probes, [3] keys emitted, [4] topic levels,
    // [5] topics spilled, [6] key segments, [7] segment-chunk flushes,
    // [8] frontier overflow chunks, [9] node-record reads, [10] keys emitted inline
    // (fast kernel only for [5]-[10]); [32 + d], [48 + d], [64 + d], [80 + d]: per walk depth
    // d (15 = 15 and deeper) edge probes, wave cycles, frontier entries, probe round trips
    unsigned long long *stats;
    // optional: events recorded around k_match_fast on the launch stream
    hipEvent_t ev_fast0, ev_fast1;
    // [unique] / aggre/1 (round 5): dd_bit = KDD_MULTI or KDD_SHARED, else 0.  The walk also
    // counts, per topic, the keys of its lists whose header collapse bit (layout.h HDR_DD) has
    // dd_bit, inline keys by their own key_dd flag; a topic with fewer than two is final
    // (ucnt[t] = its count), the others go to the reducer's worklist wl {topic, that count}.
    uint32_t dd_bit;
    const uint8_t *key_dd;
    uint32_t *ucnt;
    uint2 *wl;
    uint32_t *wl_n;
    // Pre-pass (round 5): k_prescan tokenises every topic and looks up the word ids of its
    // first TM_PRELOOK levels in a launch of its own (pre_wid[l * pre_stride + t]; pre_meta[t]
    // = {levels | badarg << 30 | '$' << 31, byte where level TM_PRELOOK starts}), and
    // k_match_fast reads them instead of staging the topic bytes and scanning them itself.
    // Null pre_wid: k_match_fast does its own pre-scan.
    uint32_t *pre_wid;
    uint2 *pre_meta;
    uint32_t pre_stride;
    // Real capacities (elements) of the buffers above, and the bounds record: read only by the
    // TM_BOUNDS debug build, whose kernels check every index against them (BI() above).
    BndCaps cap;
    unsigned long long *bnd;
};

// Levels whose word ids the pre-scan looks up, all in flight together (k_match_fast's own
// pre-scan, or k_prescan)
#ifndef TM_PRELOOK
#define TM_PRELOOK 10
#endif

// Topics per wave of k_match_fast.  A wave's walk is a chain of dependent round trips
// whose length grows with its frontier, so a small batch is spread thin (down to 4
// topics per wave) to fill the chip with short waves; from 256 Ki topics on, 64 per wave.
inline uint32_t pick_tpw(uint32_t n, uint32_t fixed = 0) {
    if (fixed == 4 || fixed == 8 || fixed == 16 || fixed == 32 || fixed == 64) return fixed;
    uint32_t t = 4;
    while (t < 64 && (uint64_t)t * 2 * 4096 <= n) t *= 2;
    return t;
}
inline uint64_t match_grid(uint32_t n, uint32_t tpw) { return ((uint64_t)n + tpw - 1) / tpw; }

// Enqueue the whole match pipeline for one batch on `stream`:
// reset counters, fast wave-BFS kernel, spill kernel for topics the fast
// kernel handed off.  Asynchronous.
hipError_t launch_match(const MatchArgs &a, hipStream_t stream);

// Delta-epoch patches: dst[idx[i]] = src[i] (16-byte records / u32 entries).
// dst_cap: dst's real capacity in elements, bnd: the bounds record (both read by the TM_BOUNDS build only)
hipError_t launch_scatter16(uint4 *dst, const uint64_t *idx, const uint4 *src, uint64_t n, hipStream_t stream,
                            uint64_t dst_cap = ~0ull, unsigned long long *bnd = nullptr);
hipError_t launch_scatter4(uint32_t *dst, const uint64_t *idx, const uint32_t *src, uint64_t n, hipStream_t stream,
                           uint64_t dst_cap = ~0ull, unsigned long long *bnd = nullptr);

// result_kernels.hip --------------------------------------------------------
// Exclusive scan of n u32 values (in[i * in_stride]) into out[0..n]; out[n] = total.
// scratch: scan_scratch_words(n) u32.
uint64_t scan_scratch_words(uint32_t n);
hipError_t launch_excl_scan(const uint32_t *in, uint64_t in_stride, uint32_t n, uint32_t *out, uint32_t *scratch,
                            hipStream_t stream);
// ids[dst_off[t] + k] = key_rec[2 * keys[src_off[t] + k]] (the id word of the key's
// {id, order code} record) for k < cnt[t] (topics whose range
// would pass `cap`, or whose keys lie past the walk's arena `keys_cap`, are skipped).
// flags (may be null): one u32 := RES_* bits, computed on the device from the walk's
// cursor (requested keys) and dst_off[n].
constexpr uint32_t RES_KEYS_OVERFLOW = 1, RES_IDS_OVERFLOW = 2;
hipError_t launch_result_ids(const uint32_t *cnt, const uint32_t *src_off, const uint32_t *keys,
                             const uint64_t *key_rec, const uint32_t *dst_off, uint32_t n, uint64_t *ids,
                             uint64_t cap, uint64_t keys_cap, const unsigned long long *cursor, uint32_t *flags,
                             hipStream_t stream);
// the same with the ids narrowed to u32 (every live id < 2^32): half the bytes to move
hipError_t launch_result_ids32(const uint32_t *cnt, const uint32_t *src_off, const uint32_t *keys,
                               const uint64_t *key_rec, const uint32_t *dst_off, uint32_t n, uint32_t *ids,
                               uint64_t cap, uint64_t keys_cap, const unsigned long long *cursor, hipStream_t stream);
// The same copy without the gather: src already holds ids of id_bytes (4 or 8) each, laid
// out as the walk wrote them (MODE_IDS*); ids[dst_off[t] + k] = src[src_off[t] + k].
hipError_t launch_compact_ids(uint32_t id_bytes, const uint32_t *src_off, const void *src, const uint32_t *dst_off,
                              uint32_t n, void *ids, uint64_t cap, uint64_t src_cap, const unsigned long long *cursor,
                              uint32_t *flags, hipStream_t stream);
// MODE_IDS* compaction by wave blocks: wave w's ids src[info.x .. + info.y) go to
// dst[dst_off[w * tpw] ..) whole; a wave with a spilled topic copies topic by topic
// (src_off / cnt: the walk's per-topic arrays).  Nothing is written when the walk overflowed
// (cursor > src_cap); ids past cap are dropped (flags report both, as launch_compact_ids).
hipError_t launch_compact_waves(uint32_t id_bytes, const uint4 *wave_info, uint32_t nwaves, uint32_t tpw, uint32_t n,
                                const uint32_t *src_off, const uint32_t *cnt, const void *src, const uint32_t *dst_off,
                                void *dst, uint64_t cap, uint64_t src_cap, const unsigned long long *cursor,
                                uint32_t *flags, hipStream_t stream);
// Concatenate G shards' topic-major compacted ids per topic (tm_merge_shard_ids_device):
// roff G rows (stride roff_stride) of n+1 per-rank exclusive scans, rank r's ids (id_bytes
// each) at ids + base[r] elements; off: n+1 merged scan out; out: merged u64 ids.
constexpr uint32_t MERGE_MAX_G = 64;
// max_total bounds every rank's id count (its chunks are launched from it; surplus blocks exit).
hipError_t launch_merge_shard_ids(uint32_t G, uint32_t n, const uint32_t *roff, uint64_t roff_stride, const void *ids,
                                  uint32_t id_bytes, const uint64_t *base, uint32_t *off, uint64_t *out, uint64_t cap,
                                  uint32_t max_total, hipStream_t stream);
// Concatenate G shards' topic-major results per topic.  roff: G*(n+1) u32, tot: n u32,
// scratch: scan_scratch_words(n) u32 (work areas); off: n+1 u32 out; out: merged ids.
hipError_t launch_merge_shards(uint32_t G, uint32_t n, const uint32_t *counts, const uint64_t *ids, uint64_t stride,
                               uint32_t *roff, uint32_t *tot, uint32_t *scratch, uint32_t *off, uint64_t *out,
                               uint64_t cap, hipStream_t stream);
// Per-topic reducers over a TM_MATCH_ALL result (result_kernels.hip k_dd_pass + k_dedupe),
// in place: topic t's reduced keys overwrite keys[off[t] ..), their number goes to
// ucnt[t].  key_rec: 2 u64 per key handle {id, order code}; key_node: u32 per handle
// (device slot of the key's node); key_dd: u8 per handle, the KDD_* flags of the keys
// that can collapse at all.  scratch: keys_cap u32; wl: n uint2; wl_n: one u32.
constexpr uint32_t DD_UNIQUE = 0, DD_AGGRE = 1;
constexpr uint8_t KDD_MULTI = 1;   // UNIQUE: the key's id is carried by more than one live key
constexpr uint8_t KDD_SHARED = 2;  // AGGRE: the key's dest is a shared-subscription member
hipError_t launch_dedupe(uint32_t mode, const uint32_t *cnt, const uint32_t *off, uint32_t *keys, uint64_t keys_cap,
                         const uint64_t *key_rec, const uint32_t *key_node, const uint8_t *key_dd, uint32_t n,
                         uint32_t *ucnt, uint32_t *scratch, uint2 *wl, uint32_t *wl_n, hipStream_t stream);
// k_dedupe alone, over the worklist a walk with MatchArgs.dd_bit left (round 5: no k_dd_pass)
hipError_t launch_dedupe_wl(uint32_t mode, const uint32_t *cnt, const uint32_t *off, uint32_t *keys,
                            const uint64_t *key_rec, const uint32_t *key_node, const uint8_t *key_dd, uint32_t n,
                            uint32_t *ucnt, uint32_t *scratch, const uint2 *wl, const uint32_t *wl_n, hipStream_t stream);
hipError_t launch_scatter1(uint8_t *dst, const uint64_t *idx, const uint8_t *src, uint64_t n, hipStream_t stream,
                           uint64_t dst_cap = ~0ull, unsigned long long *bnd = nullptr);
hipError_t launch_scatter8(uint64_t *dst, const uint64_t *idx, const uint64_t *src, uint64_t n, hipStream_t stream,
                           uint64_t dst_cap = ~0ull, unsigned long long *bnd = nullptr);

}  // namespace tmx
