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
//   k_match_fast  one WAVEFRONT per 64 topics.  Lane = topic for tokenising; then a
//                 level-synchronous walk whose frontier (all 64 topics' live trie
//                 nodes at this depth) is staged in LDS and processed 64 entries at a
//                 time, so '+' fan-out of one topic spreads over the whole wave.
//                 Child probes, emitted key segments and next-frontier pushes are
//                 compacted with wave prefix scans.  At the end the wave reserves its
//                 output with ONE atomic and expands the segments with a
//                 load-balanced copy (every lane busy, contiguous stores).
//                 Levels are tokenised lazily, one per depth, so there is no level
//                 cap; segments overflow LDS into a global chunk pool.
//   k_match_slow  spill path for topics whose wave frontier overflows LDS (FCAP
//                 entries): one lane per topic, depth-first with the stack in global
//                 scratch (depth bounded by the level count), count pass + fill pass.
// No MFMA: this is a latency/gather-bound walk.
#include <hip/hip_runtime.h>

#include "device_api.h"

namespace tmx {

constexpr int WAVE = 64;
constexpr int FCAP = 256;      // frontier entries per wave per depth held in LDS
constexpr int FCH = FR_CHUNK;  // frontier entries per global overflow chunk
constexpr int MAXF = 64;       // overflow chunks per wave per depth
constexpr int SCAP = SEG_CHUNK;  // key segments staged in LDS = one global chunk (128)
constexpr int MAXCHUNK = 64;   // global segment chunks one wave may flush
constexpr int TBCAP = 3072;    // topic bytes of one wave staged in LDS (else read from HBM)

// ---------------------------------------------------------------------------
// wave helpers
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & (WAVE - 1); }

// exclusive prefix sum over the 64 lanes; *total gets the wave sum
__device__ __forceinline__ uint32_t wave_excl_scan(uint32_t v, uint32_t *total) {
    uint32_t x = v;
    const uint32_t lane = lane_id();
#pragma unroll
    for (int d = 1; d < WAVE; d <<= 1) {
        uint32_t y = __shfl_up(x, d, WAVE);
        if (lane >= (uint32_t)d) x += y;
    }
    *total = __shfl(x, WAVE - 1, WAVE);
    return x - v;
}

__device__ __forceinline__ uint64_t wave_sum64(uint64_t v) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, WAVE);
    return v;
}

// ---------------------------------------------------------------------------
// word table: bytes -> word id (byte-verified; never trusts the hash alone)
__device__ __forceinline__ uint32_t word_lookup(const MatchArgs &a, const uint8_t *p, uint32_t len, uint64_t h,
                                                uint32_t *probes) {
    uint64_t s = word_slot_hash(h, len) & a.wmask;
    for (;;) {
        const uint4 *q = reinterpret_cast<const uint4 *>(a.wtab + s);
        uint4 x = q[0];
        uint4 y = q[1];
        (*probes)++;
        uint64_t sh = (uint64_t)x.x | ((uint64_t)x.y << 32);
        uint32_t wid = x.z;
        if (wid == NONE) return NONE;
        if (sh == h && x.w == len) {
            // y = {arena_off, inl[0..3], inl[4..7], inl[8..11]}
            bool eq = true;
            uint32_t inl[3] = {y.y, y.z, y.w};
            uint32_t ni = len < WORD_INLINE ? len : WORD_INLINE;
            for (uint32_t i = 0; i < ni && eq; i++) eq = p[i] == (uint8_t)(inl[i >> 2] >> ((i & 3) * 8));
            for (uint32_t i = WORD_INLINE; i < len && eq; i++) eq = p[i] == a.warena[y.x + i];
            if (eq) return wid;
        }
        s = (s + 1) & a.wmask;
    }
}

// edge table: (parent, word) -> 32-byte slot; returns slot index or ~0
struct Rec {
    uint32_t child, flags, list_off, term_cnt, hash_cnt;
};
__device__ __forceinline__ uint64_t edge_probe(const MatchArgs &a, uint32_t parent, uint32_t word, Rec *r,
                                               uint32_t *probes) {
    uint64_t s = edge_hash(parent, word) & a.emask;
    for (;;) {
        const uint4 *q = reinterpret_cast<const uint4 *>(a.etab + s);
        uint4 x = q[0];
        uint4 y = q[1];
        (*probes)++;
        if (x.x == NONE) return ~0ull;
        if (x.x == parent && x.y == word) {
            r->child = x.z;
            r->flags = x.w;
            r->list_off = y.x;
            r->term_cnt = y.y;
            r->hash_cnt = y.z;
            return s;
        }
        s = (s + 1) & a.emask;
    }
}

// Probe (parent, word) and (parent, '+') together: both first loads are in flight
// before either result is consumed (the two are independent chains).
__device__ __forceinline__ void edge_probe2(const MatchArgs &a, uint32_t parent, bool want1, uint32_t word,
                                            bool want2, Rec *r1, bool *f1, Rec *r2, bool *f2, uint32_t *probes) {
    uint64_t s1 = edge_hash(parent, word) & a.emask;
    uint64_t s2 = edge_hash(parent, W_PLUS) & a.emask;
    bool p1 = want1, p2 = want2;
    *f1 = false;
    *f2 = false;
    while (p1 || p2) {
        uint4 x1 = make_uint4(NONE, 0, 0, 0), y1 = x1, x2 = x1, y2 = x1;
        if (p1) {
            const uint4 *q = reinterpret_cast<const uint4 *>(a.etab + s1);
            x1 = q[0];
            y1 = q[1];
        }
        if (p2) {
            const uint4 *q = reinterpret_cast<const uint4 *>(a.etab + s2);
            x2 = q[0];
            y2 = q[1];
        }
        *probes += (uint32_t)p1 + (uint32_t)p2;
        if (p1) {
            if (x1.x == NONE) {
                p1 = false;
            } else if (x1.x == parent && x1.y == word) {
                *r1 = Rec{x1.z, x1.w, y1.x, y1.y, y1.z};
                *f1 = true;
                p1 = false;
            } else {
                s1 = (s1 + 1) & a.emask;
            }
        }
        if (p2) {
            if (x2.x == NONE) {
                p2 = false;
            } else if (x2.x == parent && x2.y == W_PLUS) {
                *r2 = Rec{x2.z, x2.w, y2.x, y2.y, y2.z};
                *f2 = true;
                p2 = false;
            } else {
                s2 = (s2 + 1) & a.emask;
            }
        }
    }
}

// Tokenise topic t: calls f(level_index, word_id) per level; returns levels,
// sets *badarg when a level is exactly "+" or "#", *dollar when the first level
// starts with '$'.
template <class F>
__device__ __forceinline__ uint32_t tokenize(const MatchArgs &a, uint32_t t, bool *badarg, bool *dollar,
                                             uint32_t *wprobes, F &&f) {
    const uint32_t b = a.off[t], e = a.off[t + 1];
    *dollar = (e > b) && a.bytes[b] == '$';
    *badarg = false;
    uint32_t nl = 0, st = b;
    uint64_t h = FNV_OFF;
    for (uint32_t i = b;; ++i) {
        const bool end = (i == e);
        const uint8_t c = end ? (uint8_t)'/' : a.bytes[i];
        if (c == '/') {
            const uint32_t len = i - st;
            uint32_t wid = NONE;
            if (len == 1 && (a.bytes[st] == '+' || a.bytes[st] == '#')) *badarg = true;
            else wid = word_lookup(a, a.bytes + st, len, h, wprobes);
            f(nl, wid);
            nl++;
            h = FNV_OFF;
            st = i + 1;
            if (end) break;
        } else {
            h = fnv_step(h, c);
        }
    }
    return nl;
}

// ---------------------------------------------------------------------------
// fast kernel: one wavefront (= one 64-thread workgroup) per 64 topics
//
// LDS per wave (~10 KiB): the two frontier buffers (FCAP entries each, extended by
// global overflow chunks), a segment staging buffer that is flushed to a global
// chunk pool when full, and per-topic cursors.  Levels are tokenised lazily (one
// level per depth, lane = topic) so there is no level cap; a topic only spills to
// k_match_slow when a pool is exhausted.
struct WaveLds {
    uint8_t tb[TBCAP];            // the wave's topic bytes (16-B aligned window)
    uint32_t fr_node[2][FCAP];
    uint8_t fr_meta[2][FCAP];     // topic lane | node flags << 6
    uint32_t fch[2][MAXF];        // global overflow chunks of each frontier buffer
    uint4 seg[SCAP];  // {src, cnt, rel, topic lane}
    uint32_t seg_scan[SCAP + 1];
    uint32_t chunk[MAXCHUNK];
    uint32_t cur[WAVE];    // byte offset where the topic's next level starts
    uint32_t wid[WAVE];    // word id of the level being expanded
    uint32_t nlev[WAVE];
    uint32_t cnt[WAVE];    // keys matched so far (allocates each segment's rel)
    uint32_t tbase[WAVE];  // output base of the topic
    uint32_t lflags[WAVE]; // bit0: spill to k_match_slow
    uint32_t alive[2][WAVE];  // frontier entries per topic at this / the next depth
};

// Expand L.seg[0..ns) into the output (all lanes busy: element e of the flattened
// segment list is found by binary search over the segment prefix sums).
__device__ __forceinline__ void expand_segments(const MatchArgs &a, WaveLds &L, uint32_t ns) {
    const uint32_t lane = lane_id();
    uint32_t run = 0;
    for (uint32_t sb = 0; sb < ns; sb += WAVE) {
        const uint32_t j = sb + lane;
        uint32_t c = 0;
        if (j < ns) {
            const uint4 g = L.seg[j];
            if (!(L.lflags[g.w] & 1u)) c = g.y;
        }
        uint32_t tot;
        const uint32_t ex = wave_excl_scan(c, &tot);
        if (j < ns) L.seg_scan[j] = run + ex;
        run += tot;
    }
    if (lane == 0) L.seg_scan[ns] = run;
    __syncthreads();
    for (uint32_t e = lane; e < run; e += WAVE) {
        uint32_t lo = 0, hi = ns;  // seg_scan[lo] <= e < seg_scan[hi]
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (L.seg_scan[mid] <= e) lo = mid;
            else hi = mid;
        }
        const uint4 g = L.seg[lo];
        const uint32_t k = e - L.seg_scan[lo];
        a.keys[L.tbase[g.w] + g.z + k] = a.arena[g.x + k];
    }
    __syncthreads();
}

template <bool STATS>
__global__ __launch_bounds__(WAVE) void k_match_fast(MatchArgs a) {
    __shared__ WaveLds L;
    const uint32_t lane = lane_id();
    const uint32_t t = blockIdx.x * WAVE + lane;
    const bool active = t < a.n;
    uint32_t st_visit = 0, st_probe = 0, st_wprobe = 0, st_seg = 0, st_flush = 0, st_frch = 0;

    // ---- 0. stage the wave's topic bytes in LDS with 16-B coalesced loads
    const uint32_t t0 = blockIdx.x * WAVE;
    const uint32_t wb0 = a.off[t0], wb1 = a.off[min(t0 + WAVE, a.n)];
    const uint32_t tbase = wb0 & ~15u;
    const bool staged = ((reinterpret_cast<uintptr_t>(a.bytes) & 15u) == 0) && (wb1 - tbase <= (uint32_t)TBCAP);
    if (staged) {
        for (uint32_t j = lane * 16; tbase + j < wb1; j += WAVE * 16) {
            if (tbase + j + 16 <= wb1) {
                *reinterpret_cast<uint4 *>(&L.tb[j]) = *reinterpret_cast<const uint4 *>(a.bytes + tbase + j);
            } else {
                for (uint32_t k = 0; tbase + j + k < wb1; k++) L.tb[j + k] = a.bytes[tbase + j + k];
            }
        }
        __syncthreads();
    }
    auto byte_at = [&](uint32_t i) -> uint8_t { return staged ? L.tb[i - tbase] : a.bytes[i]; };

    // ---- 1. pre-scan (lane = topic): levels, badarg, '$'
    bool badarg = false, dollar = false;
    uint32_t nl = 0, b = 0, e = 0;
    if (active) {
        b = a.off[t];
        e = a.off[t + 1];
        dollar = (e > b) && byte_at(b) == '$';
        uint32_t st = b;
        for (uint32_t i = b;; ++i) {
            const bool end = i == e;
            const uint8_t c = end ? (uint8_t)'/' : byte_at(i);
            if (c == '/') {
                if (i - st == 1 && (byte_at(st) == '+' || byte_at(st) == '#')) badarg = true;
                nl++;
                st = i + 1;
                if (end) break;
            }
        }
    }
    const bool spill0 = active && !badarg && a.force_slow;
    const bool walk = active && !badarg && !spill0;
    L.cur[lane] = b;
    L.nlev[lane] = nl;
    L.cnt[lane] = 0;
    L.lflags[lane] = spill0 ? 1u : 0u;
    L.alive[0][lane] = 0;
    L.alive[1][lane] = 0;

    // ---- 2. root: emit "#" keys (not for '$' topics), seed the frontier
    const RootRec R = *a.root;
    uint32_t nseg = 0, nchunk = 0;  // wave-uniform
    uint32_t nfr;
    {
        const bool em = walk && !dollar && R.hash_cnt;
        uint32_t tot;
        const uint32_t pos = wave_excl_scan(em ? 1u : 0u, &tot);
        if (em) {
            L.seg[pos] = make_uint4(R.list_off + R.term_cnt, R.hash_cnt, 0u, lane);
            L.cnt[lane] = R.hash_cnt;
        }
        nseg = tot;
        st_seg += em;
        const uint32_t rf = dollar ? (R.flags & F_LIT) : (R.flags & F_KIDS);
        const bool push = walk && rf;
        const uint32_t p2 = wave_excl_scan(push ? 1u : 0u, &tot);
        if (push) {
            L.fr_node[0][p2] = ROOT;
            L.fr_meta[0][p2] = (uint8_t)(lane | (rf << 6));
            L.alive[0][lane] = 1;
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
            const uint2 v = a.fr_pool[(uint64_t)L.fch[lvl][k / FCH] * FCH + k % FCH];
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
            a.fr_pool[(uint64_t)L.fch[lvl][k / FCH] * FCH + k % FCH] = make_uint2(node, meta);
        }
    };

    // ---- 3. level-synchronous walk
    for (uint32_t d = 0; nfr > 0; ++d) {
        const uint32_t cur = d & 1, nxt = cur ^ 1;
        // 3a. tokenise level d of every topic that still has frontier entries
        if (walk && L.alive[cur][lane]) {
            uint32_t i = L.cur[lane];
            const uint32_t st = i;
            uint64_t h = FNV_OFF;
            uint8_t c;
            while (i < e && (c = byte_at(i)) != '/') {
                h = fnv_step(h, c);
                i++;
            }
            L.wid[lane] = staged ? word_lookup(a, &L.tb[st - tbase], i - st, h, &st_wprobe)
                                 : word_lookup(a, a.bytes + st, i - st, h, &st_wprobe);
            L.cur[lane] = i + 1;
        }
        L.alive[nxt][lane] = 0;
        __syncthreads();
        // 3b. expand the frontier, 64 entries per round
        uint32_t nnext = 0;
        for (uint32_t base = 0; base < nfr; base += WAVE) {
            const uint32_t i = base + lane;
            const bool has = i < nfr;
            uint32_t node = 0, tl = 0, fl = 0;
            if (has) {
                uint32_t meta;
                fr_read(cur, i, node, meta);
                tl = meta & 63u;
                fl = meta >> 6;
            }
            const uint32_t w = has ? L.wid[tl] : NONE;
            const bool last = has && (d + 1 == L.nlev[tl]);
            Rec r1{}, r2{};
            bool f1, f2;
            edge_probe2(a, node, has && (fl & F_LIT) && w != NONE, w, has && (fl & F_PLUS), &r1, &f1, &r2, &f2,
                        &st_probe);
            // segments: each found child's '#' list; its exact list at the topic's last level
            const bool s1h = f1 && r1.hash_cnt, s1t = f1 && last && r1.term_cnt;
            const bool s2h = f2 && r2.hash_cnt, s2t = f2 && last && r2.term_cnt;
            const uint32_t ns = (uint32_t)s1h + s1t + s2h + s2t;
            uint32_t tot_s;
            uint32_t ps = wave_excl_scan(ns, &tot_s);
            if (tot_s && nseg + tot_s > (uint32_t)SCAP) {
                // flush the staged segments to one global chunk
                __syncthreads();
                uint32_t c = 0;
                if (lane == 0) c = (uint32_t)atomicAdd(a.seg_cursor, 1ull);
                c = __shfl(c, 0, WAVE);
                if (c < a.seg_chunks && nchunk < (uint32_t)MAXCHUNK) {
                    uint4 *dst = a.seg_pool + (uint64_t)c * SCAP;
                    for (uint32_t j = lane; j < (uint32_t)SCAP; j += WAVE)
                        dst[j] = j < nseg ? L.seg[j] : make_uint4(0u, 0u, 0u, 0u);
                    if (lane == 0) L.chunk[nchunk] = c;
                    nchunk++;
                    st_flush++;
                } else {
                    // pool exhausted: those topics take the spill kernel instead
                    for (uint32_t j = lane; j < nseg; j += WAVE) atomicOr(&L.lflags[L.seg[j].w], 1u);
                }
                nseg = 0;
                __syncthreads();
            }
            ps += nseg;
            if (ns) {
                auto put = [&](uint32_t src, uint32_t c) {
                    L.seg[ps++] = make_uint4(src, c, atomicAdd(&L.cnt[tl], c), tl);
                };
                if (s1t) put(r1.list_off, r1.term_cnt);
                if (s1h) put(r1.list_off + r1.term_cnt, r1.hash_cnt);
                if (s2t) put(r2.list_off, r2.term_cnt);
                if (s2h) put(r2.list_off + r2.term_cnt, r2.hash_cnt);
            }
            nseg += tot_s;
            st_seg += ns;
            // next frontier: children that can still expand
            const bool p1 = f1 && !last && (r1.flags & F_KIDS);
            const bool p2b = f2 && !last && (r2.flags & F_KIDS);
            uint32_t tot_p;
            uint32_t pp = nnext + wave_excl_scan((uint32_t)p1 + p2b, &tot_p);
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
            if (p1 || p2b) {
                if (pp + (uint32_t)p1 + p2b <= cap) {
                    if (p1) fr_write(nxt, pp++, r1.child, tl | ((r1.flags & F_KIDS) << 6));
                    if (p2b) fr_write(nxt, pp, r2.child, tl | ((r2.flags & F_KIDS) << 6));
                    atomicAdd(&L.alive[nxt][tl], (uint32_t)p1 + p2b);
                } else {
                    atomicOr(&L.lflags[tl], 1u);  // frontier overflow: topic spills
                }
            }
            nnext = min(nnext + tot_p, cap);
            st_visit += (uint32_t)f1 + f2;
        }
        __syncthreads();
        nfr = nnext;
    }

    // ---- 4. reserve this wave's output with one atomic; per-topic results
    const bool spill = active && !badarg && (L.lflags[lane] & 1u);
    const uint32_t my = (walk && !spill) ? L.cnt[lane] : 0u;
    uint32_t total;
    const uint32_t excl = wave_excl_scan(my, &total);
    unsigned long long gb = 0;
    if (lane == 0 && total) gb = atomicAdd(a.cursor, (unsigned long long)total);
    gb = __shfl(gb, 0, WAVE);
    const bool overflow = gb + total > a.keys_cap;
    L.tbase[lane] = (uint32_t)(gb + excl);
    if (active) {
        a.status[t] = badarg ? 1 : 0;
        a.out_off[t] = spill ? 0u : (uint32_t)(gb + excl);
        a.out_cnt[t] = my;
    }
    {
        uint32_t tot_sp;
        const uint32_t ps = wave_excl_scan(spill ? 1u : 0u, &tot_sp);
        uint32_t sb = 0;
        if (lane == 0 && tot_sp) sb = atomicAdd(a.slow_count, tot_sp);
        sb = __shfl(sb, 0, WAVE);
        if (spill) a.slow_list[sb + ps] = t;
    }
    __syncthreads();

    // ---- 5. load-balanced expansion: staged segments, then flushed chunks
    if (!overflow && total) {
        expand_segments(a, L, nseg);
        for (uint32_t c = 0; c < nchunk; ++c) {
            const uint4 *src = a.seg_pool + (uint64_t)L.chunk[c] * SCAP;
            for (uint32_t j = lane; j < (uint32_t)SCAP; j += WAVE) L.seg[j] = src[j];
            __syncthreads();
            expand_segments(a, L, SCAP);
        }
    }

    if constexpr (STATS) {
        const uint64_t v0 = wave_sum64(st_visit), v1 = wave_sum64(st_probe), v2 = wave_sum64(st_wprobe),
                       v4 = wave_sum64(nl), v5 = wave_sum64(spill ? 1u : 0u), v6 = wave_sum64(st_seg);
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
        }
    }
}

// ---------------------------------------------------------------------------
// spill kernel: lane per topic, DFS with the stack in global scratch.
// Stack entry: slot index (40 bits; ROOT_MARK for the root) | depth (24 bits).
constexpr uint64_t ROOT_MARK = (1ull << 40) - 1;

template <bool WRITE>
__device__ uint32_t dfs_walk(const MatchArgs &a, const RootRec &R, const uint32_t *wid, uint64_t *stk, uint32_t nl,
                             bool dollar, uint32_t *out, uint32_t *probes, uint32_t *visits) {
    uint32_t sp = 0, count = 0;
    stk[sp++] = ROOT_MARK << 24;
    while (sp) {
        const uint64_t ent = stk[--sp];
        const uint64_t slot = ent >> 24;
        const uint32_t d = (uint32_t)(ent & 0xFFFFFF);
        const bool is_root = slot == ROOT_MARK;
        uint32_t node, flags, lo, tc, hc;
        if (is_root) {
            node = ROOT;
            flags = dollar ? (R.flags & F_LIT) : R.flags;
            lo = R.list_off;
            tc = R.term_cnt;
            hc = dollar ? 0 : R.hash_cnt;
        } else {
            const uint4 *q = reinterpret_cast<const uint4 *>(a.etab + slot);
            uint4 x = q[0], y = q[1];
            node = x.z;
            flags = x.w;
            lo = y.x;
            tc = y.y;
            hc = y.z;
        }
        (*visits)++;
        // "P/#" keys match at P and below
        if (WRITE)
            for (uint32_t k = 0; k < hc; k++) out[count + k] = a.arena[lo + tc + k];
        count += hc;
        if (d == nl) {
            if (WRITE)
                for (uint32_t k = 0; k < tc; k++) out[count + k] = a.arena[lo + k];
            count += tc;
            continue;
        }
        Rec r;
        if (flags & F_PLUS) {
            uint64_t s = edge_probe(a, node, W_PLUS, &r, probes);
            if (s != ~0ull) stk[sp++] = (s << 24) | (d + 1);
        }
        const uint32_t w = wid[d];
        if ((flags & F_LIT) && w != NONE) {
            uint64_t s = edge_probe(a, node, w, &r, probes);
            if (s != ~0ull) stk[sp++] = (s << 24) | (d + 1);
        }
    }
    return count;
}

template <bool STATS>
__global__ __launch_bounds__(WAVE) void k_match_slow(MatchArgs a) {
    const uint32_t nslow = *a.slow_count;
    const RootRec R = *a.root;
    uint32_t st_visit = 0, st_probe = 0, st_wprobe = 0;
    uint64_t st_keys = 0, st_lev = 0;
    for (uint32_t idx = blockIdx.x * WAVE + lane_id(); idx < nslow; idx += gridDim.x * WAVE) {
        const uint32_t t = a.slow_list[idx];
        const uint64_t sbase = (uint64_t)(a.off[t] - a.off[0]) + 2ull * t;  // len+2 entries per topic
        uint32_t *wid = a.scratch_w + sbase;
        uint64_t *stk = a.scratch_s + sbase;
        bool badarg, dollar;
        const uint32_t nl = tokenize(a, t, &badarg, &dollar, &st_wprobe, [&](uint32_t i, uint32_t w) { wid[i] = w; });
        st_lev += nl;
        uint32_t dummy_v = 0, dummy_p = 0;
        const uint32_t c = dfs_walk<false>(a, R, wid, stk, nl, dollar, nullptr, &dummy_p, &dummy_v);
        const unsigned long long pos = atomicAdd(a.cursor, (unsigned long long)c);
        a.out_off[t] = (uint32_t)pos;
        a.out_cnt[t] = c;
        a.status[t] = 0;
        st_keys += c;
        if (pos + c <= a.keys_cap) dfs_walk<true>(a, R, wid, stk, nl, dollar, a.keys + pos, &st_probe, &st_visit);
    }
    if constexpr (STATS) {
        // levels were already counted by the fast kernel's pre-scan
        atomicAdd(&a.stats[0], (unsigned long long)st_visit);
        atomicAdd(&a.stats[1], (unsigned long long)st_probe);
        atomicAdd(&a.stats[2], (unsigned long long)st_wprobe);
        atomicAdd(&a.stats[3], (unsigned long long)st_keys);
        (void)st_lev;
    }
}

// ---------------------------------------------------------------------------
template <class Slot>
__global__ void k_scatter(Slot *dst, const uint64_t *idx, const Slot *src, uint64_t n) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[idx[i]] = src[i];
}

hipError_t launch_scatter_edges(EdgeSlot *dst, const uint64_t *idx, const EdgeSlot *src, uint64_t n,
                                hipStream_t s) {
    if (!n) return hipSuccess;
    k_scatter<EdgeSlot><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dst, idx, src, n);
    return hipGetLastError();
}
hipError_t launch_scatter_words(WordSlot *dst, const uint64_t *idx, const WordSlot *src, uint64_t n,
                                hipStream_t s) {
    if (!n) return hipSuccess;
    k_scatter<WordSlot><<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dst, idx, src, n);
    return hipGetLastError();
}

hipError_t launch_match(const MatchArgs &a, hipStream_t s) {
    hipError_t e;
    if ((e = hipMemsetAsync(a.cursor, 0, sizeof(unsigned long long), s))) return e;
    if ((e = hipMemsetAsync(a.slow_count, 0, sizeof(uint32_t), s))) return e;
    if ((e = hipMemsetAsync(a.seg_cursor, 0, sizeof(unsigned long long), s))) return e;
    if ((e = hipMemsetAsync(a.fr_cursor, 0, sizeof(unsigned long long), s))) return e;
    if (a.n == 0) return hipSuccess;
    const unsigned grid = (a.n + WAVE - 1) / WAVE;
    if (a.ev_fast0 && (e = hipEventRecord(a.ev_fast0, s))) return e;
    if (a.stats) k_match_fast<true><<<grid, WAVE, 0, s>>>(a);
    else k_match_fast<false><<<grid, WAVE, 0, s>>>(a);
    if ((e = hipGetLastError())) return e;
    if (a.ev_fast1 && (e = hipEventRecord(a.ev_fast1, s))) return e;
    // spill kernel: fixed grid, grid-stride over the device-side spill list
    const unsigned sgrid = grid < 2048u ? grid : 2048u;
    if (a.stats) k_match_slow<true><<<sgrid, WAVE, 0, s>>>(a);
    else k_match_slow<false><<<sgrid, WAVE, 0, s>>>(a);
    return hipGetLastError();
}

}  // namespace tmx
