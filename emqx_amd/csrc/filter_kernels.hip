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
// One lane per query: a walk is a chain of dependent probes whose length depends on the
// query, and queries are few (the reference has no caller on the publish path).  Every
// step either stops or moves to a strictly greater index (a seek target is greater than the
// key it came from for queries with '#' only last; the host refuses the others), so a lane
// makes at most K steps.
#include "device_api.h"

namespace tmx {

namespace {

constexpr uint32_t C_HASH = 0, C_PLUS = 1;
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

// next({pre ++ [w], {}}) among keys [lo, K): the first key >= the probe.  Galloping from lo
// (seeks mostly land near the key they start from), then a binary search.
__device__ uint32_t seek_from(const FilterArgs &a, uint32_t lo, const uint32_t *pre, uint32_t np, uint32_t w) {
    const uint32_t K = a.K;
    if (lo >= K || cmp_key_seek(a, lo, pre, np, w) >= 0) return lo;
    uint32_t below = lo, hi = K;
    for (uint64_t step = 1;; step <<= 1) {
        const uint64_t p = (uint64_t)below + step;
        if (p >= K) break;
        if (cmp_key_seek(a, (uint32_t)p, pre, np, w) >= 0) {
            hi = (uint32_t)p;
            break;
        }
        below = (uint32_t)p;
    }
    uint32_t l = below + 1, h = hi;
    while (l < h) {
        const uint32_t m = l + (h - l) / 2;
        if (cmp_key_seek(a, m, pre, np, w) < 0) l = m + 1;
        else h = m;
    }
    return l;
}

// compare/3 with the filter-search clauses, iteratively: clause order as in the reference;
// a filter '+' facing a query word is the last backtrack point, a query '+' passes the
// deeper result through unchanged.
__device__ inline int cmp_filter(const uint32_t *F, uint32_t FL, const uint32_t *W, uint32_t WL, uint32_t &spos,
                                 uint32_t &sword) {
    int last_plus = -1;
    for (uint32_t pos = 0;; pos++) {
        const bool fin = pos == FL, win = pos == WL;
        if (fin) return win ? R_FULL : R_PREFIX;                      // compare([], [], _) / ([], _, _)
        const uint32_t f = F[pos];
        if (FL - pos == 1 && f == C_HASH) return R_FULL;               // compare(['#'], _, _)
        if (win) {                                                     // compare([_|_], [], _): lower
            if (last_plus >= 0) {
                spos = (uint32_t)last_plus;
                sword = W[last_plus];
                return R_SEEK;
            }
            return R_LOWER;
        }
        const uint32_t w = W[pos];
        if (WL - pos == 1 && w == C_HASH) return R_FULL;               // compare(_, ['#'], _)
        if (w == C_PLUS) continue;                                     // compare([_|TF], ['+'|TW], Pos)
        if (f == C_PLUS) {                                             // compare(['+'|TF], [HW|TW], Pos)
            last_plus = (int)pos;
            continue;
        }
        if (f == w) continue;                                          // compare([HW|TF], [HW|TW], Pos)
        if (f > w) {                                                   // HF > HW: lower
            if (last_plus >= 0) {
                spos = (uint32_t)last_plus;
                sword = W[last_plus];
                return R_SEEK;
            }
            return R_LOWER;
        }
        spos = pos;                                                    // {Pos, HW}
        sword = w;
        return R_SEEK;
    }
}

// pass 0: cnt[q] = keys the walk of query q matches; pass 1: write their handles at out_off[q]
__global__ __launch_bounds__(256) void k_filter_walk(FilterArgs a, int pass) {
    const uint32_t q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.n) return;
    const uint32_t qb = a.qoff[q], WL = a.qoff[q + 1] - qb;
    const uint32_t *W = a.qw + qb;
    uint32_t c = 0;
    if (WL && a.qstatus[q] == 0) {
        // base_init/1 (:160-163): a first word <<"$", _/bytes>> starts at next({[W0], {}})
        uint32_t idx = a.qdollar[q] ? seek_from(a, 0, nullptr, 0, W[0]) : 0;
        uint32_t *out = pass ? a.out + a.out_off[q] : nullptr;
        while (idx < a.K) {
            const uint32_t b = a.koff[idx];
            uint32_t spos = 0, sword = 0;
            const int r = cmp_filter(a.kw + b, a.koff[idx + 1] - b, W, WL, spos, sword);
            if (r == R_FULL) {                   // match_add/2, then next(Cursor)
                if (pass) out[c] = a.kh[idx];
                c++;
                if (a.first) break;              // return_first
                idx++;
            } else if (r == R_PREFIX) {
                idx++;
            } else if (r == R_LOWER) {
                break;
            } else {                             // seek/3: next({first spos words ++ [sword], {}})
                idx = seek_from(a, idx + 1, a.kw + b, spos, sword);
            }
        }
    }
    if (!pass) a.cnt[q] = c;
}

}  // namespace

hipError_t launch_filter_walk(const FilterArgs &a, int pass, hipStream_t stream) {
    if (!a.n) return hipSuccess;
    const uint32_t blocks = (a.n + 255) / 256;
    hipLaunchKernelGGL(k_filter_walk, dim3(blocks), dim3(256), 0, stream, a, pass);
    return hipGetLastError();
}

}  // namespace tmx
