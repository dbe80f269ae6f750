// filter_api.h — private interface between the host engine (engine.cpp) and the
// matches_filter/3 and intersection/2 kernels (filter_kernels.hip).  Not part of the C-ABI.
// Kept apart from device_api.h so the match kernels' sources (and the hash that ties their
// PMC profiles to them, bench.py kernel_src_sha) do not change with these.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmx {

// filter_kernels.hip ---------------------------------------------------------
// matches_filter/3 over the term-ordered word-list keys (engine.cpp FilterIndex).
struct FilterArgs {
    const uint32_t *kw;    // order codes of every key's words, keys back to back
    const uint32_t *koff;  // K+1: key j's words are kw[koff[j] .. koff[j+1])
    const uint4 *krec;     // 2 per key: {length, words 0 .. FW_REC_WORDS-1 (0-padded)}
    const uint32_t *kend;  // FW_END_DEPTHS per key: kend[j * FW_END_DEPTHS + d] = the first key
                           // after j whose first d+1 words differ from key j's (its prefix
                           // group's end; key j shorter than d+1 words: j + 1)
    const uint32_t *kh;    // K: key handle of sorted key j
    uint32_t K;
    uint32_t n;            // queries
    const uint32_t *qw;    // order codes of the query words
    const uint32_t *qoff;  // n+1
    const uint8_t *qdollar;  // 1: the first query word starts with '$' (base_init/1)
    const int32_t *qstatus;  // 0: walk; else skipped (count 0)
    uint32_t first;          // return_first: stop at the first hit
    uint32_t *cnt;           // pass 0 out: n;  FW_ONEPASS out: n
    uint32_t *out_off;       // pass 1 in: n (exclusive scan of cnt);  FW_ONEPASS out: n
    uint32_t *out;           // pass 1 / FW_ONEPASS out: key handles, per query in walk order
    // FW_ONEPASS: the walk streams its matches as ranges {first sorted key, count} into linked
    // chunks of FW_CHUNK u32 words (entry 0's .x = next chunk) from `pool`, then reserves its
    // contiguous output range with one atomic and expands the ranges into it; ranges longer
    // than FW_BULK keys become jobs of k_filter_bulk (all CUs copy them)
    uint32_t *pool;
    uint64_t pool_chunks;
    uint64_t out_cap;
    unsigned long long *ctl;  // [0] output keys requested, [1] chunks requested (may pass the caps),
                              // [2] bulk jobs
    uint4 *jobs;              // FW_ONEPASS: {src sorted key, dst, count (<= FW_JOB), 0}
    uint64_t jobs_cap;
    // FW_RUNS: the walk's ranges themselves are the result: query q's rcnt[q] ranges {first
    // sorted key, count} at ((uint2 *)out)[out_off[q] ..], cnt[q] keys; ctl[0] counts ranges and
    // out_cap is in ranges
    uint32_t *rcnt;
    // FW_RUNS parts (round 5, engine.cpp plan_filter_parts): when items is set, wave i walks
    // item i = {query, start key, end key (NONE: none), 1 for the query's first part} from its
    // start until it stops or reaches its end, and cnt / rcnt / out_off / stop are per item
    // (stop[i] = 1 unless the part reached its end); null: item i is query i, whole
    const uint4 *items;
    uint32_t n_items;
    uint32_t *stop;
    // development (EMQX_TM_FILTER_WTIME=1, FW_RUNS): per wave, its duration in wall-clock ticks
    // (100 MHz); null in the product
    unsigned long long *wtime;
};
constexpr int FW_COUNT = 0, FW_EMIT = 1, FW_ONEPASS = 2, FW_RUNS = 3;
constexpr uint32_t FW_CHUNK = 256;   // u32 words per pool chunk (1 link entry + 127 ranges of 2 words)
constexpr uint32_t FW_BULK = 4096;   // ranges longer than this are copied by k_filter_bulk
constexpr uint32_t FW_JOB = 8192;    // keys per k_filter_bulk job (a long range is split)
constexpr uint32_t FW_REC_WORDS = 7; // key words held in the fixed-stride record
constexpr uint32_t FW_END_DEPTHS = 8; // prefix-group ends kept per key (prefixes of 1..8 words)
hipError_t launch_filter_walk(const FilterArgs &a, int pass, hipStream_t stream);
// FW_ONEPASS's bulk copies (after launch_filter_walk, same stream; reads the job count on device)
hipError_t launch_filter_bulk(const FilterArgs &a, hipStream_t stream);
// emqx_topic:intersection/2 per pair; out_len[i] = bytes, or one of:
constexpr int32_t INTERSECT_FALSE = -1, INTERSECT_BADHASH = -2;
hipError_t launch_intersect(const uint8_t *a, const uint32_t *a_off, const uint8_t *b, const uint32_t *b_off,
                            uint32_t n, uint8_t *out, int32_t *out_len, hipStream_t stream);


}  // namespace tmx
