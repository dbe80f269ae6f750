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
#include "wave.h"

namespace tmx {

namespace {

constexpr uint32_t C_HASH = 0, C_PLUS = 1;
constexpr uint32_t NONE_FW = 0xFFFFFFFFu;
constexpr int R_FULL = 0, R_PREFIX = 1, R_LOWER = 2, R_SEEK = 3;

constexpr uint32_t RW = FW_REC_WORDS;

// key j's record: its length and first RW words (0-padded)
__device__ __forceinline__ uint32_t load_rec(const FilterArgs &a, uint32_t j, uint32_t (&kr)[RW]) {
    const uint4 r0 = a.krec[2 * (uint64_t)j], r1 = a.krec[2 * (uint64_t)j + 1];
    kr[0] = r0.y;
    kr[1] = r0.z;
    kr[2] = r0.w;
    kr[3] = r1.x;
    kr[4] = r1.y;
    kr[5] = r1.z;
    kr[6] = r1.w;
    return r0.x;
}

// The seek probe {first np words of key ks ++ [w], {}}: the first RW prefix words in registers
// (taken from key ks's record, which the wave already holds), the rest read from kw.
struct Probe {
    uint32_t pr[RW];
    uint32_t ks, np, w;
};

// key j (its record kr, length L already in registers) vs the probe: -1 / 0 / 1.  Memory
// is read only when the prefix is longer than the record.
__device__ inline int cmp_rec_probe(const FilterArgs &a, uint32_t j, const uint32_t (&kr)[RW], uint32_t L,
                                    const Probe &pb) {
    uint32_t xn = 0;  // the key's word at position np (when np < RW)
#pragma unroll
    for (int i = 0; i < (int)RW; i++) {
        if ((uint32_t)i < pb.np) {
            if ((uint32_t)i == L) return -1;
            if (kr[i] != pb.pr[i]) return kr[i] < pb.pr[i] ? -1 : 1;
        }
        if ((uint32_t)i == pb.np) xn = kr[i];
    }
    if (pb.np > RW) {
        const uint32_t *k = a.kw + a.koff[j], *pre = a.kw + a.koff[pb.ks];
        for (uint32_t i = RW; i < pb.np; i++) {
            if (i == L) return -1;
            if (k[i] != pre[i]) return k[i] < pre[i] ? -1 : 1;
        }
    }
    if (pb.np == L) return -1;
    const uint32_t x = pb.np < RW ? xn : a.kw[a.koff[j] + pb.np];
    if (x != pb.w) return x < pb.w ? -1 : 1;
    return L == pb.np + 1 ? 0 : 1;
}

// key j vs the probe: one record load (a round trip), then the compare in registers
__device__ inline int cmp_key_seek(const FilterArgs &a, uint32_t j, const Probe &pb) {
    uint32_t kr[RW];
    const uint32_t L = load_rec(a, j, kr);
    return cmp_rec_probe(a, j, kr, L, pb);
}

// next(probe) among keys [lo, hi): the first key >= the probe, found by the whole wave; hi
// itself when none is (the caller knows key hi is past the probe, or hi == K).  A far bound
// starts with a gallop (lane L probes lo + 2^L - 1; lanes past hi count as past the probe),
// which brackets the answer; then 64-ary narrowing, each round probing 64 evenly spaced keys
// (a range of R keys takes about log64(R) rounds).  A near bound (the probe's prefix group,
// kend) is narrowed directly.  Wave-uniform result.
__device__ uint32_t wave_seek(const FilterArgs &a, uint32_t lo, const Probe &pb, uint32_t lane, uint32_t hi) {
    if (lo >= hi) return hi;
    // invariant: every key below l is < the probe; key h is >= it (or h == hi)
    uint64_t l = lo, h = hi;
    if (hi - lo > 64u * 64u) {
        const uint64_t p = lane < 33 ? (uint64_t)lo + ((1ull << lane) - 1) : ~0ull;
        const bool ge = p >= hi || cmp_key_seek(a, (uint32_t)p, pb) >= 0;
        const uint32_t g = (uint32_t)__ffsll((long long)__ballot(ge)) - 1;  // lane 32 is always ge
        if (g == 0) return lo;
        l = (uint64_t)lo + (1ull << (g - 1));
        h = std::min<uint64_t>((uint64_t)lo + (1ull << g) - 1, hi);
    }
    while (l < h) {
        const uint64_t step = (h - l + 63) / 64;
        const uint64_t x = l + lane * step;
        const bool xge = x >= h || cmp_key_seek(a, (uint32_t)x, pb) >= 0;
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

// The end of key ks's group of keys sharing its first np words (1 <= np <= FW_END_DEPTHS), or
// K when np is out of that range: an upper bound of next({first np words of ks ++ [w], {}}).
__device__ __forceinline__ uint32_t prefix_end(const FilterArgs &a, uint32_t ks, uint32_t np) {
    if (np == 0 || np > FW_END_DEPTHS) return a.K;
    return a.kend[(uint64_t)ks * FW_END_DEPTHS + np - 1];  // wave-uniform address: one load
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
        if (WL - pos_ == 1 && w_ == C_HASH) { /* (_, ['#'], _) */                             \
            qh = pos_;                                                                         \
            return R_FULL;                                                                     \
        }                                                                                      \
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

// compare/3 for a filter search.  The key's record (fr: its first RW words) and the query's
// first 8 words (wr) come preloaded in registers and the first RW positions are unrolled
// (static indices keep them in registers), so a compare is one record load.  qh := the position
// when the result is match_full by the query's last-level '#' (else left unchanged).
__device__ __attribute__((always_inline)) inline int cmp_filter(const uint32_t (&fr)[RW], const FilterArgs &a,
                                                                uint32_t j, uint32_t FL, const uint32_t (&wr)[8],
                                                                const uint32_t *W, uint32_t WL, uint32_t &spos,
                                                                uint32_t &sword, uint32_t &qh) {
    int lp = -1;
    uint32_t lpw = 0;
#pragma unroll
    for (uint32_t p = 0; p < RW; p++) CMP_STEP(p, fr[p], wr[p])
    const uint32_t *F = a.kw + a.koff[j];  // past the record: the key's words in kw
    for (uint32_t p = RW;; p++) CMP_STEP(p, F[p], W[p])
}
#undef CMP_STEP

// src[0..m) -> dst[0..m) by the 64 lanes of a wave, 8 loads in flight per lane
__device__ void copy_keys(const uint32_t *src, uint32_t *dst, uint32_t m, uint32_t lane) {
    for (uint32_t k0 = lane; k0 < m; k0 += 64 * 8) {
        uint32_t v[8];
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (k0 + u * 64 < m) v[u] = src[k0 + u * 64];
#pragma unroll
        for (int u = 0; u < 8; u++)
            if (k0 + u * 64 < m) dst[k0 + u * 64] = v[u];
    }
}

// exclusive prefix sum over the 64 lanes; *total gets the wave sum
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total, uint32_t lane) {
    (void)lane;
    const uint32_t x = wave_incl_scan_dpp(v);
    *total = lane_value(x, 63);
    return x - v;
}

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
    const uint32_t it = blockIdx.x * 4 + (threadIdx.x >> 6);  // the item: a query, or a part of one
    const uint32_t lane = threadIdx.x & 63;
    if (it >= (a.items ? a.n_items : a.n)) return;  // wave-uniform
    const unsigned long long t_begin = a.wtime ? wall_clock64() : 0ull;
    const uint4 item = a.items ? a.items[it] : make_uint4(it, 0u, NONE_FW, 1u);
    const uint32_t q = item.x;
    const uint32_t qb = a.qoff[q], WL = a.qoff[q + 1] - qb;
    const uint32_t *W = a.qw + qb;
    const uint32_t K = a.K;
    // a part ends where the next one starts: keys at or past pend are not its own (they count
    // as a stop in a step), and reaching pend is not a stop of the query's walk
    const uint32_t pend = min(item.z, K);
    bool reached = false;  // wave-uniform
    uint32_t c = 0;  // wave-uniform
    // FW_ONEPASS chain of ranges (wave-uniform): head, current chunk, ranges in the current chunk
    constexpr uint32_t CE = FW_CHUNK / 2 - 1;  // ranges per chunk (entry 0 is the link)
    uint2 *const pool2 = reinterpret_cast<uint2 *>(a.pool);
    uint32_t head = NONE_FW, curc = NONE_FW, fill = CE, nent = 0;
    bool short_pool = false;
    auto new_chunk = [&]() -> uint32_t {  // wave-uniform; NONE_FW when the pool is exhausted
        unsigned long long c0 = 0;
        if (lane == 0) c0 = atomicAdd(&a.ctl[1], 1ull);
        c0 = __shfl(c0, 0);
        if (c0 >= a.pool_chunks) return NONE_FW;
        if (lane == 0) pool2[c0 * (FW_CHUNK / 2)] = make_uint2(NONE_FW, 0u);
        return (uint32_t)c0;
    };
    // append one range per lane in `em` (this lane's is {src, len}), in lane order
    auto chain_put = [&](uint64_t em, uint32_t src, uint32_t len) {
        const uint32_t ne = __popcll(em);
        if (!ne || short_pool) return;
        const uint32_t room = CE - fill;
        uint32_t nc = NONE_FW;
        if (ne > room) {
            nc = new_chunk();
            if (nc == NONE_FW) {
                short_pool = true;
                return;
            }
            if (curc == NONE_FW) head = nc;
            else if (lane == 0) pool2[(uint64_t)curc * (FW_CHUNK / 2)] = make_uint2(nc, 0u);  // link
        }
        if ((em >> lane) & 1ull) {
            const uint32_t rk = __popcll(em & ((1ull << lane) - 1));
            const uint64_t at = rk < room ? (uint64_t)curc * (FW_CHUNK / 2) + 1 + fill + rk
                                          : (uint64_t)nc * (FW_CHUNK / 2) + 1 + (rk - room);
            pool2[at] = make_uint2(src, len);
        }
        if (ne > room) {
            curc = nc;
            fill = ne - room;
        } else {
            fill += ne;
        }
        nent += ne;
    };
    if (WL && a.qstatus[q] == 0) {
        // base_init/1 (:160-163): a first word <<"$", _/bytes>> starts at next({[W0], {}})
        uint32_t idx = item.y;  // a later part starts at its child-group start
        if (item.w && a.qdollar[q]) {
            Probe pb{};
            pb.np = 0;
            pb.w = W[0];
            idx = wave_seek(a, 0, pb, lane, K);
        }
        uint32_t *out = pass == FW_EMIT ? a.out + a.out_off[q] : nullptr;
        const uint64_t below = (1ull << lane) - 1;
        uint32_t wr[8];  // the query's first 8 words (qw is padded by 8 words on the device)
#pragma unroll
        for (int i = 0; i < 8; i++) wr[i] = W[i];
        // The window: lanes [0, nv) hold the records of keys wbase + lane.  A seek whose
        // target lies inside it moves the window by shifting registers across lanes, not by
        // reloading: a walk under a query '+' visits many small prefix groups one after the
        // other, and most of its seeks land a few keys ahead.
        // The compare of a key depends on that key alone, so its result (r, spos, sword, qh)
        // travels with the record.
        uint32_t fr[RW] = {};
        uint32_t FL = 0, nv = 0, wbase = 0;
        int r = R_LOWER;  // past the end of the table (or not loaded yet): a stop
        uint32_t spos = 0, sword = 0, qh = NONE_FW;
        while (idx < pend) {
            const uint32_t j = idx + lane;
            const bool inr = j < pend;
            {  // keep what the previous window already holds
                const uint32_t o = idx - wbase;
                if (nv > o) {
                    const int src = (int)(lane + o) & 63;
#pragma unroll
                    for (int i = 0; i < (int)RW; i++) fr[i] = __shfl(fr[i], src);
                    FL = __shfl(FL, src);
                    r = __shfl(r, src);
                    spos = __shfl(spos, src);
                    sword = __shfl(sword, src);
                    qh = __shfl(qh, src);
                    nv -= o;
                } else {
                    nv = 0;
                }
                wbase = idx;
                if (!inr || lane >= nv) {
                    r = R_LOWER;
                    qh = NONE_FW;
                }
            }
            {
                // the step is decided by its first event (a stop, or a '#'-run start); when
                // that comes before the first key not held yet, nothing needs loading
                const bool known = lane < nv || !inr;
                const uint64_t ev = __ballot(known && (r == R_LOWER || r == R_SEEK || qh != NONE_FW));
                const uint64_t unk = __ballot(!known);
                const bool need = unk && (!ev || __ffsll((long long)unk) < __ffsll((long long)ev));
                if (need) {
                    if (inr && lane >= nv) {
                        FL = load_rec(a, j, fr);
                        r = cmp_filter(fr, a, j, FL, wr, W, WL, spos, sword, qh);
                        // A seek whose probe prefix (the key's first spos words) no other key
                        // shares lands on the next key: seek({Pos, W}) from key j returns a key
                        // in (j, end of j's spos-word group], and that end is j + 1.  Such a
                        // step is next(Cursor), like match_prefix.
                        if (r == R_SEEK && spos >= 1 && spos <= FW_END_DEPTHS &&
                            a.kend[(uint64_t)j * FW_END_DEPTHS + spos - 1] == j + 1)
                            r = R_PREFIX;
                    }
                    nv = 64;
                }
            }
            // next(probe) from key lo = idx + from + 1: the lanes past `from` already hold
            // their records, so a target inside this window costs no memory round trip;
            // past it, the wave searches from the first key not held (keys past K count as
            // the end)
            auto seek_from = [&](uint32_t from, const Probe &pb) -> uint32_t {
                const bool ge = lane > from && (!inr || (lane < nv && cmp_rec_probe(a, j, fr, FL, pb) >= 0));
                const uint64_t gm = __ballot(ge);
                if (gm && (nv == 64 || __ffsll((long long)gm) - 1 < (int)nv)) return min(idx + (uint32_t)__ffsll((long long)gm) - 1, K);
                const uint32_t lo = idx + nv;
                // past the window: the target lies in the probe's prefix group, whose end is
                // known per key (kend); a '#'-run's end (probe word +inf) IS that end
                // (never below lo, which the window just ruled out: the walk only moves on)
                const uint32_t hi = min(max(prefix_end(a, pb.ks, pb.np), lo), K);
                if (pb.w == NONE_FW && pb.np >= 1 && pb.np <= FW_END_DEPTHS) return hi;
                return wave_seek(a, lo, pb, lane, hi);
            };
            // the probe of a seek or run end from lane l: key idx+l's record words, no loads
            auto probe_from = [&](uint32_t l, uint32_t np, uint32_t w) {
                Probe pb;
#pragma unroll
                for (int i = 0; i < (int)RW; i++) pb.pr[i] = lane_value(fr[i], l);
                pb.ks = idx + l;
                pb.np = np;
                pb.w = w;
                return pb;
            };
            const uint64_t stop = __ballot(r == R_LOWER || r == R_SEEK);
            const uint32_t fs = stop ? (uint32_t)__ffsll((long long)stop) - 1 : 64;
            // A key that is match_full by the query's last-level '#' at position p starts a run:
            // every following key with the same first p words is match_full too (the compare
            // reads nothing else of them), and those keys are contiguous in term order.
            const uint64_t runm = __ballot(lane < fs && qh != NONE_FW);
            const uint32_t rl = runm ? (uint32_t)__ffsll((long long)runm) - 1 : 64;
            const uint32_t lim = min(fs, rl);
            const bool full = lane < lim && r == R_FULL;
            uint64_t fm = __ballot(full);
            if (a.first && fm) fm &= 0 - fm;  // return_first: the first key met only
            const uint32_t nf = __popcll(fm);
            if (pass == FW_ONEPASS || pass == FW_RUNS) {
                // consecutive FULL lanes form one range: {first key, run length}
                const bool st0 = ((fm >> lane) & 1ull) && (lane == 0 || !((fm >> (lane - 1)) & 1ull));
                const uint64_t sm = __ballot(st0);
                const uint64_t rest = ~(fm >> lane);  // 0 only at lane 0 with all 64 lanes FULL
                const uint32_t rlen = st0 ? (rest ? (uint32_t)__ffsll((long long)rest) - 1 : 64u) : 0u;
                chain_put(sm, j, rlen);
            } else if (pass == FW_EMIT && ((fm >> lane) & 1ull)) {
                out[c + __popcll(fm & below)] = a.kh[j];  // match_add/2, walk order
            }
            c += nf;
            if (a.first && nf) break;
            if (rl < fs) {
                // the run [rs, E): E = next({first p words of key rs ++ [+inf], {}})
                const uint32_t rs = idx + rl, p = lane_value(qh, rl);
                // (a run ends inside its child group: never past a part's end)
                const uint32_t E = a.first ? rs + 1 : min(seek_from(rl, probe_from(rl, p, NONE_FW)), pend);
                const uint32_t m = E - rs;
                if (pass == FW_EMIT) {
                    copy_keys(a.kh + rs, out + c, m, lane);
                } else if (pass == FW_ONEPASS || pass == FW_RUNS) {
                    chain_put(1ull, rs, m);
                }
                c += m;
                if (a.first) break;
                idx = E;
                continue;
            }
            if (fs == 64) {                      // 64 x next(Cursor)
                idx += 64;
                continue;
            }
            const int rs = (int)lane_value((uint32_t)r, fs);
            const uint32_t ks = idx + fs;
            if (ks >= pend) {  // the part's end (or '$end_of_table')
                idx = pend;
                break;
            }
            if (rs == R_LOWER) break;  // lower
            // seek/3: next({first spos words of key ks ++ [sword], {}})
            const uint32_t sp = lane_value(spos, fs), sw = lane_value(sword, fs);
            idx = seek_from(fs, probe_from(fs, sp, sw));
        }
        // a part that reached its end hands the walk to the next part (return_first: unless it
        // found its key); anything else is the walk's own stop
        reached = idx >= pend && pend < K && !(a.first && c);
    }
    if (pass == FW_COUNT && lane == 0) a.cnt[q] = c;
    if (pass == FW_RUNS) {
        // the chain's ranges, in walk order, to a contiguous range of the output: no key is
        // copied (tm_match_filter_batch_runs turns them into spans of the host's sorted ids)
        unsigned long long base = 0;
        if (lane == 0 && nent) base = atomicAdd(&a.ctl[0], (unsigned long long)nent);
        base = __shfl(base, 0);
        if (lane == 0) {
            a.cnt[it] = c;
            a.rcnt[it] = nent;
            a.out_off[it] = (uint32_t)base;
            if (a.stop) a.stop[it] = reached ? 0u : 1u;
        }
        if (a.wtime && lane == 0) a.wtime[it] = wall_clock64() - t_begin;  // before the range copy
        if (short_pool || base + nent > a.out_cap) return;  // the host grows and re-runs
        __threadfence_block();
        uint2 *out2 = reinterpret_cast<uint2 *>(a.out);
        uint32_t ch = head;
        for (uint32_t cb = 0; cb < nent; cb += CE) {
            const uint32_t m = min(CE, nent - cb);
            const uint2 *ent = pool2 + (uint64_t)ch * (FW_CHUNK / 2) + 1;
            for (uint32_t e = lane; e < m; e += 64) out2[base + cb + e] = ent[e];
            if (cb + CE < nent) ch = pool2[(uint64_t)ch * (FW_CHUNK / 2)].x;  // next chunk
        }
    }
    if (pass == FW_ONEPASS) {
        unsigned long long base = 0;
        if (lane == 0 && c) base = atomicAdd(&a.ctl[0], (unsigned long long)c);
        base = __shfl(base, 0);
        if (lane == 0) {
            a.cnt[q] = c;
            a.out_off[q] = (uint32_t)base;
        }
        if (short_pool || base + c > a.out_cap) return;  // the host re-runs the batch
        __threadfence_block();  // the chain's ranges and links (other lanes' stores) before reading them
        // expand the ranges into [base, base + c), chunk by chunk: ranges of up to 8 keys by
        // their lane, longer ones by the wave, longer than FW_BULK keys by k_filter_bulk
        uint32_t ch = head, pos = 0;
        for (uint32_t cb = 0; cb < nent; cb += CE) {
            const uint32_t m = min(CE, nent - cb);
            const uint2 *ent = pool2 + (uint64_t)ch * (FW_CHUNK / 2) + 1;
            for (uint32_t e0 = 0; e0 < m; e0 += 64) {
                uint2 r = e0 + lane < m ? ent[e0 + lane] : make_uint2(0u, 0u);
                uint32_t tot;
                const uint32_t d = (uint32_t)base + pos + wave_excl_scan(r.y, &tot, lane);
                pos += tot;
                if (d + (uint64_t)r.y > base + c) r.y = 0;  // never write past the range (a bad
                                                            // chain shows as a parity failure)
                if (r.y <= 8) {
                    for (uint32_t k = 0; k < r.y; k++) a.out[d + k] = a.kh[r.x + k];
                }
                bool queued = false;
                if (r.y > FW_BULK) {  // FW_JOB keys per job
                    const uint32_t nj = (r.y + FW_JOB - 1) / FW_JOB;
                    const unsigned long long jn = atomicAdd(&a.ctl[2], (unsigned long long)nj);
                    if (jn + nj <= a.jobs_cap) {
                        for (uint32_t u = 0; u < nj; u++)
                            a.jobs[jn + u] = make_uint4(r.x + u * FW_JOB, d + u * FW_JOB, min(FW_JOB, r.y - u * FW_JOB), 0u);
                        queued = true;
                    }
                }
                uint64_t wv = __ballot(r.y > 8 && !queued);  // the wave copies these one by one
                while (wv) {
                    const uint32_t l = (uint32_t)__ffsll((long long)wv) - 1;
                    wv &= wv - 1;
                    copy_keys(a.kh + lane_value(r.x, l), a.out + lane_value(d, l), lane_value(r.y, l), lane);
                }
            }
            if (cb + CE < nent) ch = pool2[(uint64_t)ch * (FW_CHUNK / 2)].x;  // next chunk
        }
    }
}

// FW_ONEPASS's long ranges, split into jobs of at most FW_JOB keys: a block per job
__global__ __launch_bounds__(256) void k_filter_bulk(FilterArgs a) {
    const unsigned long long nj = min(a.ctl[2], (unsigned long long)a.jobs_cap);
    for (unsigned long long jn = blockIdx.x; jn < nj; jn += gridDim.x) {
        uint4 jb = a.jobs[jn];
        if (jb.y + (uint64_t)jb.z > a.out_cap) jb.z = 0;  // never write past the output
        const uint32_t *src = a.kh + jb.x;
        uint32_t *dst = a.out + jb.y;
        for (uint32_t k0 = threadIdx.x; k0 < jb.z; k0 += 256 * 8) {
            uint32_t v[8];
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (k0 + u * 256 < jb.z) v[u] = src[k0 + u * 256];
#pragma unroll
            for (int u = 0; u < 8; u++)
                if (k0 + u * 256 < jb.z) dst[k0 + u * 256] = v[u];
        }
    }
}

}  // namespace

hipError_t launch_filter_bulk(const FilterArgs &a, hipStream_t stream) {
    if (!a.n || !a.jobs_cap) return hipSuccess;
    hipLaunchKernelGGL(k_filter_bulk, dim3(4096), dim3(256), 0, stream, a);
    return hipGetLastError();
}

hipError_t launch_filter_walk(const FilterArgs &a, int pass, hipStream_t stream) {
    if (!a.n) return hipSuccess;
    const uint32_t waves = a.items ? a.n_items : a.n;  // one query, or one part of one, per wave
    const uint32_t blocks = (waves + 3) / 4;           // 4 waves of 64 per block
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
