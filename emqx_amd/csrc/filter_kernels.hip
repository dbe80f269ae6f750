// filter_kernels.hip — gfx950 kernels for matches_filter/3 (filter-vs-filter search).
//
// emqx_trie_search:matches_filter/3 (apps/emqx/src/emqx_trie_search.erl:186-189) runs the
// search_new/search_up seek walk (:230-258) with the filter-search clauses of compare/3
// (:260-348, :291-300) over the ETS ordered_set.  Its result is defined by that walk, not
// by a predicate (a seek can jump over a key the query would cover), so the device replays
// the walk itself over a term-ordered array of the word-list keys (engine.cpp builds it per
// epoch): key j's words are kw[koff[j] .. koff[j+1]) as order codes ('#' 0, '+' 1, the k-th
// dictionary word 2k+3, a query word outside the dictionary 2*lower_bound+2), keys sorted by
// (words, id).  `next({Prefix, {}})` is a lower bound; `next(Key)` is the following index.
//
// One wave per query: the lanes compare 64 consecutive keys per step (the walk only jumps at
// a seek) and search 64 probes wide.  Every step either stops or moves to a strictly greater
// index (a seek target is greater than the key it came from for queries with '#' only last;
// the host refuses the others, and wave_seek searches from the next key on), so a wave
// makes at most K steps.
#include <algorithm>

#include "filter_api.h"

namespace tmx {

namespace {

constexpr uint32_t C_HASH = 0, C_PLUS = 1;
constexpr uint32_t NONE_FW = 0xFFFFFFFFu;
constexpr int R_FULL = 0, R_PREFIX = 1, R_LOWER = 2, R_SEEK = 3;

// key j vs pre[0..np) ++ [w]: -1 / 0 / 1
__device__ inline int cmp_key_seek(const FilterArgs &a, uint32_t j, const uint32_t *pre, uint32_t np, uint32_t w) {
    const uint32_t b = a.koff[j], L = a.koff[j + 1] - b;
    const uint32_t *k = a.kw + b;
    for (uint32_t i = 0; i < np; i++) {
        if (i == L) return -1;
        const uint32_t x = k[i];
        if (x != pre[i]) return x < pre[i] ? -1 : 1;
    }
    if (np == L) return -1;
    const uint32_t x = k[np];
    if (x != w) return x < w ? -1 : 1;
    return L == np + 1 ? 0 : 1;
}

// next({pre ++ [w], {}}) among keys [lo, K): the first key >= the probe, found by the whole
// wave.  Gallop: lane L probes lo + 2^L - 1 (lane 32 lies past any K < 2^32), which
// brackets the answer; then 64-ary narrowing, each round probing 64 evenly spaced keys
// (a range of K keys takes about log64(K) rounds).  Wave-uniform result.
__device__ uint32_t wave_seek(const FilterArgs &a, uint32_t lo, const uint32_t *pre, uint32_t np, uint32_t w,
                              uint32_t lane) {
    const uint64_t K = a.K;
    if (lo >= K) return (uint32_t)K;
    const uint64_t p = lane < 33 ? (uint64_t)lo + ((1ull << lane) - 1) : ~0ull;
    const bool ge = p >= K || cmp_key_seek(a, (uint32_t)p, pre, np, w) >= 0;
    const uint32_t g = (uint32_t)__ffsll((long long)__ballot(ge)) - 1;  // lane 32 is always ge
    if (g == 0) return lo;
    // invariant: every key below l is < the probe; key h is >= it (or h == K)
    uint64_t l = (uint64_t)lo + (1ull << (g - 1)), h = std::min<uint64_t>((uint64_t)lo + (1ull << g) - 1, K);
    while (l < h) {
        const uint64_t step = (h - l + 63) / 64;
        const uint64_t x = l + lane * step;
        const bool xge = x >= h || cmp_key_seek(a, (uint32_t)x, pre, np, w) >= 0;
        const uint64_t m = __ballot(xge);
        if (!m) {
            l = l + 63 * step + 1;
            continue;
        }
        const uint32_t f = (uint32_t)__ffsll((long long)m) - 1;
        if (f == 0) return (uint32_t)l;
        const uint64_t hf = std::min<uint64_t>(l + f * step, h);
        l = l + (f - 1) * step + 1;
        h = hf;
    }
    return (uint32_t)l;
}

// One position of compare/3 with the filter-search clauses, in the reference's clause
// order; falls through to the next position.  A filter '+' facing a query word is the last
// backtrack point (lp, with its query word lpw); a query '+' passes the deeper result
// through unchanged.  F_ / W_ are evaluated only once the position exists.
#define CMP_STEP(POS, F_, W_)                                                                  \
    {                                                                                          \
        const uint32_t pos_ = (POS);                                                           \
        if (pos_ == FL) return pos_ == WL ? R_FULL : R_PREFIX; /* ([], [], _) / ([], _, _) */  \
        const uint32_t f_ = (F_);                                                              \
        if (FL - pos_ == 1 && f_ == C_HASH) return R_FULL; /* (['#'], _, _) */                 \
        if (pos_ == WL) { /* ([_|_], [], _): lower */                                         \
            if (lp >= 0) {                                                                     \
                spos = (uint32_t)lp;                                                           \
                sword = lpw;                                                                   \
                return R_SEEK;                                                                 \
            }                                                                                  \
            return R_LOWER;                                                                    \
        }                                                                                      \
        const uint32_t w_ = (W_);                                                              \
        if (WL - pos_ == 1 && w_ == C_HASH) return R_FULL; /* (_, ['#'], _) */                 \
        if (w_ != C_PLUS) { /* ([_|TF], ['+'|TW], Pos) continues */                            \
            if (f_ == C_PLUS) { /* (['+'|TF], [HW|TW], Pos) */                                 \
                lp = (int)pos_;                                                                \
                lpw = w_;                                                                      \
            } else if (f_ != w_) { /* ([HW|TF], [HW|TW], Pos) continues */                     \
                if (f_ > w_) { /* HF > HW: lower */                                            \
                    if (lp >= 0) {                                                             \
                        spos = (uint32_t)lp;                                                   \
                        sword = lpw;                                                           \
                        return R_SEEK;                                                         \
                    }                                                                          \
                    return R_LOWER;                                                            \
                }                                                                              \
                spos = pos_; /* {Pos, HW} */                                                   \
                sword = w_;                                                                    \
                return R_SEEK;                                                                 \
            }                                                                                  \
        }                                                                                      \
    }

// compare/3 for a filter search.  The first 8 words of the key (fr) and of the query (wr)
// come preloaded in registers and the first 8 positions are unrolled (static indices keep
// them in registers), so a compare is not a chain of dependent loads.
__device__ __attribute__((always_inline)) inline int cmp_filter(const uint32_t (&fr)[8], const uint32_t *F,
                                                                uint32_t FL, const uint32_t (&wr)[8],
                                                                const uint32_t *W, uint32_t WL, uint32_t &spos,
                                                                uint32_t &sword) {
    int lp = -1;
    uint32_t lpw = 0;
#pragma unroll
    for (uint32_t p = 0; p < 8; p++) CMP_STEP(p, fr[p], wr[p])
    for (uint32_t p = 8;; p++) CMP_STEP(p, F[p], W[p])
}
#undef CMP_STEP

// One wave per query.  The walk moves to the next key after match_full / match_prefix, so
// the 64 lanes compare keys idx .. idx+63 at once: up to the first key that compares
// `lower` or seeks, the sequential walk visits exactly those keys in order.  FULL keys
// before that point are emitted in order (ballot + prefix popcount); then the wave stops
// (lower / end of table), seeks (wave_seek), or moves on by 64.
// FW_COUNT: cnt[q] = keys the walk matches; FW_EMIT: write their handles at out_off[q].
// FW_ONEPASS: one walk; keys go to the wave's chunk chain as they are met, then to a
// contiguous range reserved at the end (out_off[q], cnt[q]).  A wave whose chunks or output
// range do not fit the pool / out_cap leaves its query unwritten; the host sees the demand
// in ctl and re-runs the batch (two-pass) after growing.
__global__ __launch_bounds__(256) void k_filter_walk(FilterArgs a, int pass) {
    const uint32_t q = blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (q >= a.n) return;  // wave-uniform
    const uint32_t qb = a.qoff[q], WL = a.qoff[q + 1] - qb;
    const uint32_t *W = a.qw + qb;
    const uint32_t K = a.K;
    uint32_t c = 0;  // wave-uniform
    // FW_ONEPASS chunk chain (wave-uniform): head, current chunk, keys in the current chunk
    constexpr uint32_t CK = FW_CHUNK - 1;
    uint32_t head = NONE_FW, curc = NONE_FW, fill = CK;
    bool short_pool = false;
    auto new_chunk = [&]() -> uint32_t {  // wave-uniform; NONE_FW when the pool is exhausted
        unsigned long long c0 = 0;
        if (lane == 0) c0 = atomicAdd(&a.ctl[1], 1ull);
        c0 = __shfl(c0, 0);
        if (c0 >= a.pool_chunks) return NONE_FW;
        if (lane == 0) a.pool[c0 * FW_CHUNK] = NONE_FW;
        return (uint32_t)c0;
    };
    if (WL && a.qstatus[q] == 0) {
        // base_init/1 (:160-163): a first word <<"$", _/bytes>> starts at next({[W0], {}})
        uint32_t idx = a.qdollar[q] ? wave_seek(a, 0, nullptr, 0, W[0], lane) : 0;
        uint32_t *out = pass == FW_EMIT ? a.out + a.out_off[q] : nullptr;
        const uint64_t below = (1ull << lane) - 1;
        uint32_t wr[8];  // the query's first 8 words (qw is padded by 8 words on the device)
#pragma unroll
        for (int i = 0; i < 8; i++) wr[i] = W[i];
        while (idx < K) {
            const uint32_t j = idx + lane;
            int r = R_LOWER;  // past the end of the table: the walk stops there
            uint32_t spos = 0, sword = 0;
            if (j < K && j >= idx) {
                const uint32_t b = a.koff[j];
                uint32_t fr[8];  // independent loads (kw is padded by 8 words on the device)
#pragma unroll
                for (int i = 0; i < 8; i++) fr[i] = a.kw[b + i];
                r = cmp_filter(fr, a.kw + b, a.koff[j + 1] - b, wr, W, WL, spos, sword);
            }
            const uint64_t stop = __ballot(r == R_LOWER || r == R_SEEK);
            const uint32_t fs = stop ? (uint32_t)__ffsll((long long)stop) - 1 : 64;
            const bool full = lane < fs && r == R_FULL;
            uint64_t fm = __ballot(full);
            if (a.first && fm) fm &= 0 - fm;  // return_first: the first key met only
            const uint32_t nf = __popcll(fm);
            if (pass == FW_ONEPASS && nf && !short_pool) {
                // room in the current chunk for `room` keys; the rest go to a fresh chunk
                const uint32_t room = CK - fill;
                uint32_t nc = NONE_FW;
                if (nf > room) {
                    nc = new_chunk();
                    if (nc == NONE_FW) short_pool = true;
                    else if (curc == NONE_FW) head = nc;
                    else if (lane == 0) a.pool[(uint64_t)curc * FW_CHUNK] = nc;  // link
                }
                if (!short_pool) {
                    if ((fm >> lane) & 1ull) {
                        const uint32_t rk = __popcll(fm & below);
                        const uint64_t at = rk < room ? (uint64_t)curc * FW_CHUNK + 1 + fill + rk
                                                      : (uint64_t)nc * FW_CHUNK + 1 + (rk - room);
                        a.pool[at] = a.kh[j];
                    }
                    if (nf > room) {
                        curc = nc;
                        fill = nf - room;
                    } else {
                        fill += nf;
                    }
                }
            } else if (pass == FW_EMIT && ((fm >> lane) & 1ull)) {
                out[c + __popcll(fm & below)] = a.kh[j];  // match_add/2, walk order
            }
            c += nf;
            if (a.first && nf) break;
            if (fs == 64) {                      // 64 x next(Cursor)
                idx += 64;
                continue;
            }
            const int rs = __shfl(r, fs);
            const uint32_t ks = idx + fs;
            if (rs == R_LOWER || ks >= K) break;  // lower, or '$end_of_table'
            // seek/3: next({first spos words of key ks ++ [sword], {}})
            const uint32_t sp = __shfl(spos, fs), sw = __shfl(sword, fs);
            idx = wave_seek(a, ks + 1, a.kw + a.koff[ks], sp, sw, lane);
        }
    }
    if (pass == FW_COUNT && lane == 0) a.cnt[q] = c;
    if (pass == FW_ONEPASS) {
        unsigned long long base = 0;
        if (lane == 0 && c) base = atomicAdd(&a.ctl[0], (unsigned long long)c);
        base = __shfl(base, 0);
        if (lane == 0) {
            a.cnt[q] = c;
            a.out_off[q] = (uint32_t)base;
        }
        if (short_pool || base + c > a.out_cap) return;  // the host re-runs the batch
        __threadfence_block();  // the chain's keys and links (other lanes' stores) before reading them
        // copy the chain into [base, base + c): 255 keys per chunk, 64 lanes at a time
        uint32_t ch = head;
        for (uint32_t done = 0; done < c; done += CK) {
            const uint32_t m = min(CK, c - done);
            const uint32_t *src = a.pool + (uint64_t)ch * FW_CHUNK + 1;
            for (uint32_t k = lane; k < m; k += 64) a.out[base + done + k] = src[k];
            ch = a.pool[(uint64_t)ch * FW_CHUNK];
        }
    }
}

}  // namespace

hipError_t launch_filter_walk(const FilterArgs &a, int pass, hipStream_t stream) {
    if (!a.n) return hipSuccess;
    const uint32_t blocks = (a.n + 3) / 4;  // 4 waves of 64 per block, one query per wave
    hipLaunchKernelGGL(k_filter_walk, dim3(blocks), dim3(256), 0, stream, a, pass);
    return hipGetLastError();
}


// ============================================================================
// emqx_topic:intersection/2 (apps/emqx/src/emqx_topic.erl:111-151), batched: pair i is
// (a_i, b_i); one lane per pair walks both word lists level by level with the clauses of
// intersect/2 in source order and writes join/1 of the result (:311-322) at
// out[(a_off[i]-a_off[0]) + (b_off[i]-b_off[0]) + i] -- a result level is a level of a or
// of b at the same position, so len(a) + len(b) + 1 bytes always suffice.
// out_len[i]: bytes, INTERSECT_FALSE, or INTERSECT_BADHASH when join/1 would raise
// error('topic_invalid_#') (a '#' before the last level; only for invalid inputs).
namespace {

struct Lvl {  // the remaining levels of one topic: the current level is [p, q), the topic ends at e
    const uint8_t *p, *q, *e;
    bool done;
};
__device__ inline void lvl_set(Lvl &l, const uint8_t *p) {
    l.p = p;
    l.done = p > l.e;
    const uint8_t *q = p;
    if (!l.done)
        while (q < l.e && *q != '/') q++;
    l.q = q;
}
__device__ inline void lvl_next(Lvl &l) { lvl_set(l, l.q + 1); }
__device__ inline bool lvl_single(const Lvl &l) { return !l.done && l.q == l.e; }
__device__ inline bool lvl_is(const Lvl &l, uint8_t c) { return !l.done && l.q - l.p == 1 && *l.p == c; }
__device__ inline bool lvl_wild(const Lvl &l) { return lvl_is(l, '+') || lvl_is(l, '#'); }
__device__ inline bool lvl_eq(const Lvl &x, const Lvl &y) {
    if (x.q - x.p != y.q - y.p) return false;
    for (const uint8_t *i = x.p, *j = y.p; i < x.q; i++, j++)
        if (*i != *j) return false;
    return true;
}

__global__ __launch_bounds__(256) void k_intersect(const uint8_t *a, const uint32_t *a_off, const uint8_t *b,
                                                   const uint32_t *b_off, uint32_t n, uint8_t *out, int32_t *out_len) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    Lvl x, y;
    x.e = a + a_off[i + 1];
    y.e = b + b_off[i + 1];
    lvl_set(x, a + a_off[i]);
    lvl_set(y, b + b_off[i]);
    uint8_t *o0 = out + (uint64_t)(a_off[i] - a_off[0]) + (b_off[i] - b_off[0]) + i, *o = o0;
    bool first = true;
    auto put = [&](const uint8_t *p, const uint8_t *q) {  // append one level (or a run of levels)
        if (!first) *o++ = '/';
        first = false;
        for (; p < q; p++) *o++ = *p;
    };
    // intersect_start/2: a '$' first word never meets a wildcard first word
    if ((x.q > x.p && *x.p == '$' && lvl_wild(y)) || (y.q > y.p && *y.p == '$' && lvl_wild(x))) {
        out_len[i] = INTERSECT_FALSE;
        return;
    }
    int32_t res = 0;
    for (;;) {
        if (lvl_single(y) && lvl_is(y, '#')) {          // intersect(Words1, ['#']) -> Words1
            if (!x.done) put(x.p, x.e);
            break;
        }
        if (lvl_single(x) && lvl_is(x, '#')) {          // intersect(['#'], Words2) -> Words2
            if (!y.done) put(y.p, y.e);
            break;
        }
        if (lvl_single(x) && lvl_single(y) && lvl_is(y, '+')) {  // intersect([W1], ['+']) -> [W1]
            put(x.p, x.q);
            break;
        }
        if (lvl_single(x) && lvl_is(x, '+') && lvl_single(y)) {  // intersect(['+'], [W2]) -> [W2]
            put(y.p, y.q);
            break;
        }
        if (x.done || y.done) {                          // intersect([], []) -> []; else false
            if (!(x.done && y.done)) res = INTERSECT_FALSE;
            break;
        }
        const bool wx = lvl_wild(x), wy = lvl_wild(y);
        if (wx && wy) {                                  // wildcard_intersection/2
            if (lvl_eq(x, y)) put(x.p, x.q);
            else {
                const uint8_t plus = '+';
                put(&plus, &plus + 1);
            }
        } else if (lvl_eq(x, y)) {
            put(x.p, x.q);
        } else if (wx) {
            put(y.p, y.q);
        } else if (wy) {
            put(x.p, x.q);
        } else {
            res = INTERSECT_FALSE;
            break;
        }
        lvl_next(x);
        lvl_next(y);
    }
    if (res == 0) {
        res = (int32_t)(o - o0);
        // join/1 raises error('topic_invalid_#') on a '#' level before the last one
        for (const uint8_t *p = o0; p < o; p++)
            if (*p == '#' && (p == o0 || p[-1] == '/') && p + 1 < o && p[1] == '/') res = INTERSECT_BADHASH;
    }
    out_len[i] = res;
}

}  // namespace

hipError_t launch_intersect(const uint8_t *a, const uint32_t *a_off, const uint8_t *b, const uint32_t *b_off,
                            uint32_t n, uint8_t *out, int32_t *out_len, hipStream_t stream) {
    if (!n) return hipSuccess;
    hipLaunchKernelGGL(k_intersect, dim3((n + 255) / 256), dim3(256), 0, stream, a, a_off, b, b_off, n, out, out_len);
    return hipGetLastError();
}

}  // namespace tmx
