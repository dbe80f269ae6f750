// result_kernels.hip — gfx950 kernels that reshape match results after k_match_fast:
//
//   * key handles -> route ids, compacted topic-major (tm_result_ids_device).  The walk
//     writes each wave's keys wherever its one atomic reserved them; a consumer that
//     ships results off the GPU (the sharded mode's all-gather, a NIF copying to the
//     caller's heap like match_to_route/1, apps/emqx/src/emqx_router.erl:648-649) wants
//     them as ids in topic order.
//   * merge of per-shard results (tm_merge_shards_device): every rank of the filter-
//     sharded mode matched the same topics against a disjoint key shard;
//     after the all-gather, topic t's result is the concatenation of its slices from
//     rank 0..G-1 (shards are disjoint, so no dedupe).
//
//   * per-topic reducers (k_dedupe): matches/3 with [unique] and emqx_broker:aggre/1 on
//     the GPU, over the full result.
//
// All of it is byte movement: coalesced where the layout allows, HBM-bound.
#include <hip/hip_runtime.h>

#define TM_BND_FILE 2  // device_api.h TM_BOUNDS records

#include <algorithm>

#include "copy_api.h"
#include "device_api.h"
#include "image_api.h"
#include "wave.h"

namespace tmx {

constexpr int SCAN_T = 256;           // threads per scan block
constexpr int SCAN_V = 8;             // values per thread
constexpr int SCAN_B = SCAN_T * SCAN_V;  // values per scan block

// ---------------------------------------------------------------------------
// exclusive scan of u32 values into out[0..n] (out[n] = total), three passes.
// Values are counts whose total stays below 2^32 (a batch's key count).
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t *sh, uint32_t *total) {
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wid = tid >> 6;
    const uint32_t x = wave_incl_scan_dpp(v);
    if (lane == 63) sh[wid] = x;
    __syncthreads();
    uint32_t base = 0, tot = 0;
    for (uint32_t w = 0; w < SCAN_T / 64; w++) {
        if (w < wid) base += sh[w];
        tot += sh[w];
    }
    __syncthreads();
    *total = tot;
    return base + x - v;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_local(const uint32_t *in, uint64_t in_stride, uint32_t n,
                                                      uint32_t *out, uint32_t *block_sums) {
    __shared__ uint32_t sh[SCAN_T / 64];
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_V;
    uint32_t v[SCAN_V], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_V; k++) {
        v[k] = (b0 + k < n) ? in[(b0 + k) * in_stride] : 0u;
        s += v[k];
    }
    uint32_t tot;
    uint32_t run = block_excl_scan(s, sh, &tot);
#pragma unroll
    for (int k = 0; k < SCAN_V; k++) {
        if (b0 + k < n) out[b0 + k] = run;
        run += v[k];
    }
    if (threadIdx.x == 0) block_sums[blockIdx.x] = tot;
}

// one block: exclusive scan of the block sums in place; sums[nb] = total
__global__ __launch_bounds__(SCAN_T) void k_scan_sums(uint32_t *sums, uint32_t nb) {
    __shared__ uint32_t sh[SCAN_T / 64];
    uint32_t carry = 0;
    for (uint32_t base = 0; base < nb; base += SCAN_T) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < nb ? sums[i] : 0u;
        uint32_t tot;
        const uint32_t ex = block_excl_scan(v, sh, &tot);
        if (i < nb) sums[i] = carry + ex;
        carry += tot;
    }
    if (threadIdx.x == 0) sums[nb] = carry;
}

__global__ __launch_bounds__(SCAN_T) void k_scan_add(uint32_t *out, uint32_t n, const uint32_t *sums, uint32_t nb) {
    const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_B + (uint64_t)threadIdx.x * SCAN_V;
    const uint32_t add = sums[blockIdx.x];
#pragma unroll
    for (int k = 0; k < SCAN_V; k++)
        if (b0 + k < n) out[b0 + k] += add;
    if (blockIdx.x == 0 && threadIdx.x == 0) out[n] = sums[nb];
}

uint64_t scan_scratch_words(uint32_t n) { return (uint64_t)(n + SCAN_B - 1) / SCAN_B + 1; }

hipError_t launch_excl_scan(const uint32_t *in, uint64_t in_stride, uint32_t n, uint32_t *out, uint32_t *scratch,
                            hipStream_t s) {
    const uint32_t nb = (uint32_t)((n + SCAN_B - 1) / SCAN_B);
    if (nb == 0) return hipMemsetAsync(out, 0, sizeof(uint32_t), s);
    k_scan_local<<<nb, SCAN_T, 0, s>>>(in, in_stride, n, out, scratch);
    k_scan_sums<<<1, SCAN_T, 0, s>>>(scratch, nb);
    k_scan_add<<<nb, SCAN_T, 0, s>>>(out, n, scratch, nb);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// key handles -> ids, topic-major, flat over the OUTPUT: a block owns RI_BLK consecutive
// output positions (grid-stride over blocks of them), finds the topics that cover them
// (binary search of dst_off, narrowed to the block's first..last topic), and each thread
// maps its positions independently: ids[q] = id(keys[src_off[t] + q - dst_off[t]]).  Every
// thread has RI_PER independent gathers, whatever the mix of list lengths (one lane per
// topic left a 16 K-topic batch with a few hundred waves walking 2,000-key lists serially).
constexpr uint32_t RI_T = 256, RI_PER = 16, RI_BLK = RI_T * RI_PER;

__device__ __forceinline__ uint32_t topic_of(const uint32_t *dst_off, uint32_t lo, uint32_t hi, uint64_t q) {
    // the last t in [lo, hi] with dst_off[t] <= q (dst_off[lo] <= q holds)
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo + 1) / 2;
        if (dst_off[mid] <= q) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}

// GATHER: src holds key handles and ids[q] = key_rec[2 * handle]; otherwise src already holds
// the ids (the walk wrote them, MODE_IDS*) and this is a pure topic-major compaction copy.
template <class IdT, bool GATHER>
__global__ __launch_bounds__(RI_T) void k_result_ids(const uint32_t *src_off, const void *src,
                                                     const uint64_t *key_rec, const uint32_t *dst_off, uint32_t n,
                                                     IdT *ids, uint64_t cap, uint64_t keys_cap,
                                                     const unsigned long long *cursor) {
    // the walk's arena overflowed: waves past the cap skipped their copy-out, nothing to read
    if (cursor && *cursor > keys_cap) return;
    const uint64_t lim = min((uint64_t)dst_off[n], cap);  // topics past the caller's cap stay unwritten
    __shared__ uint32_t s_t0, s_t1;
    for (uint64_t q0 = (uint64_t)blockIdx.x * RI_BLK; q0 < lim; q0 += (uint64_t)gridDim.x * RI_BLK) {
        const uint64_t q1 = min(q0 + RI_BLK, lim);
        __syncthreads();  // the previous block-range is done with s_t0 / s_t1
        if (threadIdx.x == 0) {
            s_t0 = topic_of(dst_off, 0, n, q0);
            s_t1 = topic_of(dst_off, s_t0, n, q1 - 1);
        }
        __syncthreads();
        uint32_t t = s_t0;
        const uint32_t t1 = s_t1;
#pragma unroll 4
        for (uint32_t i = 0; i < RI_PER; i++) {
            const uint64_t q = q0 + (uint64_t)i * RI_T + threadIdx.x;
            if (q >= q1) break;
            t = topic_of(dst_off, t, t1, q);  // positions rise with i: start from the last topic
            const uint64_t j = (uint64_t)src_off[t] + (q - dst_off[t]);
            if (j < keys_cap) {
                if constexpr (GATHER) ids[q] = (IdT)key_rec[2ull * static_cast<const uint32_t *>(src)[j]];
                else ids[q] = static_cast<const IdT *>(src)[j];
            }
        }
    }
}

// flags[0] = RES_KEYS_OVERFLOW if the walk asked for more keys than its arena holds,
// | RES_IDS_OVERFLOW if the compacted ids passed the caller's buffer (dst_off[n] > cap).
__global__ void k_result_flags(const unsigned long long *cursor, uint64_t keys_cap, const uint32_t *dst_off,
                               uint32_t n, uint64_t cap, uint32_t *flags) {
    if (threadIdx.x == 0)
        flags[0] = (*cursor > keys_cap ? RES_KEYS_OVERFLOW : 0u) | ((uint64_t)dst_off[n] > cap ? RES_IDS_OVERFLOW : 0u);
}

template <class IdT, bool GATHER>
static hipError_t launch_result_ids_t(const uint32_t *src_off, const void *src, const uint64_t *key_rec,
                                      const uint32_t *dst_off, uint32_t n, IdT *ids, uint64_t cap, uint64_t keys_cap,
                                      const unsigned long long *cursor, uint32_t *flags, hipStream_t s) {
    if (n && cap) {
        // sized from the caller's cap (the result's size is on the device): surplus blocks exit
        const uint64_t blocks = std::min<uint64_t>((cap + RI_BLK - 1) / RI_BLK, 2048);
        k_result_ids<IdT, GATHER><<<(uint32_t)blocks, RI_T, 0, s>>>(src_off, src, key_rec, dst_off, n, ids, cap,
                                                                    keys_cap, cursor);
        hipError_t e = hipGetLastError();
        if (e) return e;
    }
    if (flags) {
        k_result_flags<<<1, 64, 0, s>>>(cursor, keys_cap, dst_off, n, cap, flags);
        return hipGetLastError();
    }
    return hipSuccess;
}

hipError_t launch_result_ids(const uint32_t *cnt, const uint32_t *src_off, const uint32_t *keys,
                             const uint64_t *key_rec, const uint32_t *dst_off, uint32_t n, uint64_t *ids,
                             uint64_t cap, uint64_t keys_cap, const unsigned long long *cursor, uint32_t *flags,
                             hipStream_t s) {
    (void)cnt;  // dst_off is its scan
    return launch_result_ids_t<uint64_t, true>(src_off, keys, key_rec, dst_off, n, ids, cap, keys_cap, cursor, flags, s);
}

hipError_t launch_result_ids32(const uint32_t *cnt, const uint32_t *src_off, const uint32_t *keys,
                               const uint64_t *key_rec, const uint32_t *dst_off, uint32_t n, uint32_t *ids,
                               uint64_t cap, uint64_t keys_cap, const unsigned long long *cursor, hipStream_t s) {
    (void)cnt;
    return launch_result_ids_t<uint32_t, true>(src_off, keys, key_rec, dst_off, n, ids, cap, keys_cap, cursor, nullptr,
                                               s);
}

// ---------------------------------------------------------------------------
// topic-major compaction of a MODE_IDS* walk by wave blocks (launch_compact_waves): one
// block per wave, a straight coalesced copy of the wave's whole output range (its topics are
// contiguous and in order there), CW_U loads in flight per thread.
constexpr uint32_t CW_T = 256, CW_U = 4;

template <class IdT>
__global__ __launch_bounds__(CW_T) void k_compact_waves(const uint4 *wave_info, uint32_t nwaves, uint32_t tpw, uint32_t n,
                                                        const uint32_t *src_off, const uint32_t *cnt, const IdT *src,
                                                        const uint32_t *dst_off, IdT *dst, uint64_t cap,
                                                        uint64_t src_cap, const unsigned long long *cursor) {
    if (*cursor > src_cap) return;  // the walk overflowed: its waves past the cap wrote nothing
    for (uint32_t w = blockIdx.x; w < nwaves; w += gridDim.x) {
        const uint4 wi = wave_info[w];
        const uint32_t t0 = w * tpw;
        if (!wi.z) {  // no spilled topic: the wave's range moves whole
            const uint64_t d0 = dst_off[t0];
            const uint64_t m = (uint64_t)wi.y;
            const uint64_t lim = d0 + m <= cap ? m : (cap > d0 ? cap - d0 : 0);
            for (uint64_t k0 = threadIdx.x; k0 < lim; k0 += CW_T * CW_U) {
                IdT v[CW_U];
#pragma unroll
                for (uint32_t u = 0; u < CW_U; u++)
                    if (k0 + u * CW_T < lim) v[u] = src[(uint64_t)wi.x + k0 + u * CW_T];
#pragma unroll
                for (uint32_t u = 0; u < CW_U; u++)
                    if (k0 + u * CW_T < lim) dst[d0 + k0 + u * CW_T] = v[u];
            }
        } else {  // topic by topic (a spilled topic's ids are where the spill kernel put them)
            const uint32_t t1 = min(t0 + tpw, n);
            for (uint32_t t = t0; t < t1; t++) {
                const uint64_t d0 = dst_off[t], s0 = src_off[t], c = cnt[t];
                if (d0 + c > cap) continue;
                for (uint64_t k = threadIdx.x; k < c; k += CW_T) dst[d0 + k] = src[s0 + k];
            }
        }
    }
}

// launch_copy_to_host: a grid-stride stream, 16-B loads and stores when source and
// destination share their alignment (the head up to a 16-B boundary word by word), else
// 4-B words; consecutive lanes write consecutive addresses, so each wave's stores leave the
// chip as whole 256-B runs.
__global__ __launch_bounds__(256) void k_copy_to_host(uint32_t *__restrict__ dst, const uint32_t *__restrict__ src,
                                                      uint64_t n) {
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, nt = (uint64_t)gridDim.x * blockDim.x;
    const uintptr_t da = reinterpret_cast<uintptr_t>(dst), sa = reinterpret_cast<uintptr_t>(src);
    if (((da ^ sa) & 15u) == 0) {
        const uint64_t head = std::min<uint64_t>(((16u - (da & 15u)) & 15u) / 4u, n);
        if (tid < head) dst[tid] = src[tid];
        const uint64_t nv = (n - head) / 4;
        const uint4 *s4 = reinterpret_cast<const uint4 *>(src + head);
        uint4 *d4 = reinterpret_cast<uint4 *>(dst + head);
        for (uint64_t i = tid; i < nv; i += nt) d4[i] = s4[i];
        const uint64_t t0 = head + nv * 4;
        if (tid < n - t0) dst[t0 + tid] = src[t0 + tid];
    } else {
        for (uint64_t i = tid; i < n; i += nt) dst[i] = src[i];
    }
}

hipError_t launch_copy_to_host(uint32_t *dst, const uint32_t *src, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint64_t want = (n / 4 + 255) / 256;
    const uint32_t blocks = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(want, 2048));
    k_copy_to_host<<<blocks, 256, 0, s>>>(dst, src, n);
    return hipGetLastError();
}

hipError_t launch_compact_waves(uint32_t id_bytes, const uint4 *wave_info, uint32_t nwaves, uint32_t tpw, uint32_t n,
                                const uint32_t *src_off, const uint32_t *cnt, const void *src, const uint32_t *dst_off,
                                void *dst, uint64_t cap, uint64_t src_cap, const unsigned long long *cursor,
                                uint32_t *flags, hipStream_t s) {
    if (n && cap && nwaves) {
        const uint32_t blocks = std::min<uint32_t>(nwaves, 8192);
        if (id_bytes == 4)
            k_compact_waves<uint32_t><<<blocks, CW_T, 0, s>>>(wave_info, nwaves, tpw, n, src_off, cnt,
                                                              (const uint32_t *)src, dst_off, (uint32_t *)dst, cap,
                                                              src_cap, cursor);
        else
            k_compact_waves<uint64_t><<<blocks, CW_T, 0, s>>>(wave_info, nwaves, tpw, n, src_off, cnt,
                                                              (const uint64_t *)src, dst_off, (uint64_t *)dst, cap,
                                                              src_cap, cursor);
        hipError_t e = hipGetLastError();
        if (e) return e;
    }
    if (flags) {
        k_result_flags<<<1, 64, 0, s>>>(cursor, src_cap, dst_off, n, cap, flags);
        return hipGetLastError();
    }
    return hipSuccess;
}

hipError_t launch_compact_ids(uint32_t id_bytes, const uint32_t *src_off, const void *src, const uint32_t *dst_off,
                              uint32_t n, void *ids, uint64_t cap, uint64_t src_cap, const unsigned long long *cursor,
                              uint32_t *flags, hipStream_t s) {
    if (id_bytes == 4)
        return launch_result_ids_t<uint32_t, false>(src_off, src, nullptr, dst_off, n, (uint32_t *)ids, cap, src_cap,
                                                    cursor, flags, s);
    return launch_result_ids_t<uint64_t, false>(src_off, src, nullptr, dst_off, n, (uint64_t *)ids, cap, src_cap, cursor,
                                                flags, s);
}

// ---------------------------------------------------------------------------
// shard merge.  counts: G rows of n; ids: G rows of `stride` (rank r's compacted,
// topic-major ids); roff: G rows of n+1 (per-rank exclusive scans of counts);
// off: merged exclusive scan (n+1).
__global__ void k_colsum(const uint32_t *counts, uint32_t G, uint32_t n, uint32_t *tot) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= n) return;
    uint32_t s = 0;
    for (uint32_t r = 0; r < G; r++) s += counts[(uint64_t)r * n + t];
    tot[t] = s;
}

__global__ __launch_bounds__(64) void k_merge(const uint32_t *counts, const uint64_t *ids, uint64_t stride,
                                              const uint32_t *roff, const uint32_t *off, uint32_t G, uint32_t n,
                                              uint64_t *out, uint64_t cap) {
    const uint32_t lane = threadIdx.x;
    const uint32_t t0 = blockIdx.x * 64;
    for (uint32_t i = 0; i < 64 && t0 + i < n; i++) {
        const uint32_t t = t0 + i;
        uint64_t dst = off[t];
        if (off[t + 1] > cap) return;  // caller's buffer too small (wave-uniform; it re-sizes from off[n])
        for (uint32_t r = 0; r < G; r++) {
            const uint32_t c = counts[(uint64_t)r * n + t];
            const uint32_t so = roff[(uint64_t)r * (n + 1) + t];
            const uint64_t src = (uint64_t)r * stride + so;
            if ((uint64_t)so + c <= stride)  // a shard's slice never leaves its row
                for (uint32_t k = lane; k < c; k += 64) out[dst + k] = ids[src + k];
            dst += c;
        }
    }
}

hipError_t launch_merge_shards(uint32_t G, uint32_t n, const uint32_t *counts, const uint64_t *ids, uint64_t stride,
                               uint32_t *roff, uint32_t *tot, uint32_t *scratch, uint32_t *off, uint64_t *out,
                               uint64_t cap, hipStream_t s) {
    hipError_t e;
    for (uint32_t r = 0; r < G; r++)
        if ((e = launch_excl_scan(counts + (uint64_t)r * n, 1, n, roff + (uint64_t)r * (n + 1), scratch, s))) return e;
    if (n) {
        k_colsum<<<(n + 255) / 256, 256, 0, s>>>(counts, G, n, tot);
        if ((e = hipGetLastError())) return e;
    }
    if ((e = launch_excl_scan(tot, 1, n, off, scratch, s))) return e;
    if (!n) return hipSuccess;
    k_merge<<<(n + 63) / 64, 64, 0, s>>>(counts, ids, stride, roff, off, G, n, out, cap);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// shard merge over topic-major compacted ids (tm_merge_shard_ids_device).  roff: G rows of
// n+1 (rank r's exclusive scan of its per-topic counts, i.e. its own d_off_out), rank r's ids
// at ids + base[r].  The merged exclusive scan is the column sum of the rows' scans, so no
// scan is launched: off[t] = sum_r roff_r[t].  Then one output-parallel pass: position q of
// topic t takes the k-th id of the topic's concatenation over ranks 0..G-1.
struct ShardBases {
    uint64_t b[MERGE_MAX_G];
};

__global__ void k_roff_colsum(const uint32_t *roff, uint64_t stride, uint32_t G, uint32_t n, uint32_t *off) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > n) return;
    uint32_t s = 0;
    for (uint32_t r = 0; r < G; r++) s += roff[(uint64_t)r * stride + t];
    off[t] = s;
}

// Rank-chunk parallel: block (r, c) moves rank r's ids [c * MG_CH, (c + 1) * MG_CH) (its
// topic-major array) to their merged positions.  The block marks in LDS where each of the
// chunk's topics starts (its local index k, with the topic's destination shift), a max-scan
// gives every element its topic, and each element lands at
//   off[t] + (ids of ranks < r in topic t) + (i - roff_r[t]).
// Reads and writes are contiguous runs (a topic's slice from one rank), no per-element search.
constexpr uint32_t MG_T = 256, MG_PER = 16, MG_CH = MG_T * MG_PER;

__device__ __forceinline__ uint32_t first_topic_ending_after(const uint32_t *ro, uint32_t n, uint64_t i) {
    // the first t in [0, n) with ro[t + 1] > i (ro is nondecreasing, ro[n] > i)
    uint32_t lo = 0, hi = n - 1;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        if ((uint64_t)ro[mid + 1] > i) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

template <class IdT>
__global__ __launch_bounds__(MG_T) void k_merge_ranks(const uint32_t *roff, uint64_t stride, uint32_t G, uint32_t n,
                                                      const IdT *ids, ShardBases base, const uint32_t *off,
                                                      uint64_t *out, uint64_t cap, uint32_t chunks_per_rank,
                                                      uint64_t max_total) {
    __shared__ uint32_t s_mark[MG_CH];  // 1 + the position where the topic covering it starts (0: none yet)
    __shared__ int64_t s_shift[MG_CH];  // at a topic's first position: its destination - source index
    __shared__ uint32_t s_part[MG_T];
    __shared__ uint32_t s_t0, s_t1;
    const uint32_t tid = threadIdx.x;
    for (uint64_t bc = blockIdx.x; bc < (uint64_t)G * chunks_per_rank; bc += gridDim.x) {
        const uint32_t r = (uint32_t)(bc / chunks_per_rank), c = (uint32_t)(bc % chunks_per_rank);
        const uint32_t *ro = roff + (uint64_t)r * stride;
        // a rank that outgrew its id buffer (TM_RES_IDS_OVERFLOW: ro[n] > what it holds) is read
        // only as far as the buffer goes; its step is flagged and the caller re-runs it
        const uint64_t total = min((uint64_t)ro[n], max_total);
        const uint64_t i0 = (uint64_t)c * MG_CH;
        if (i0 >= total) continue;  // block-uniform
        const uint64_t i1 = min(i0 + MG_CH, total);
        __syncthreads();
        if (tid == 0) {
            s_t0 = first_topic_ending_after(ro, n, i0);
            s_t1 = first_topic_ending_after(ro, n, i1 - 1);
        }
        for (uint32_t k = tid; k < MG_CH; k += MG_T) s_mark[k] = 0;
        __syncthreads();
        const uint32_t t0 = s_t0, t1 = s_t1;
        // mark each nonempty topic's first element in the chunk with its local index + 1
        for (uint32_t t = t0 + tid; t <= t1; t += MG_T) {
            const uint32_t a = ro[t], e = ro[t + 1];
            if (e == a) continue;
            uint64_t before = 0;  // ids of ranks < r in topic t
            for (uint32_t q = 0; q < r; q++)
                before += roff[(uint64_t)q * stride + t + 1] - roff[(uint64_t)q * stride + t];
            const uint64_t at = a > i0 ? a : i0;  // the topic's first position in the chunk
            s_shift[at - i0] = (int64_t)off[t] + (int64_t)before - (int64_t)a;
            s_mark[at - i0] = (uint32_t)(at - i0) + 1;
        }
        __syncthreads();
        // inclusive max-scan of the marks: thread-local over MG_PER, then over the threads
        uint32_t m = 0;
        for (uint32_t u = 0; u < MG_PER; u++) {
            const uint32_t v = s_mark[tid * MG_PER + u];
            m = v > m ? v : m;
            s_mark[tid * MG_PER + u] = m;
        }
        s_part[tid] = m;
        __syncthreads();
        for (uint32_t d = 1; d < MG_T; d <<= 1) {
            const uint32_t v = tid >= d ? s_part[tid - d] : 0u;
            __syncthreads();
            if (v > s_part[tid]) s_part[tid] = v;
            __syncthreads();
        }
        const uint32_t carry = tid ? s_part[tid - 1] : 0u;
        for (uint32_t u = 0; u < MG_PER; u++) {
            const uint32_t v = s_mark[tid * MG_PER + u];
            s_mark[tid * MG_PER + u] = v > carry ? v : carry;
        }
        __syncthreads();
        // every element: its topic's shift; coalesced reads of the rank's ids
        for (uint32_t u = 0; u < MG_PER; u++) {
            const uint32_t k = u * MG_T + tid;
            const uint64_t i = i0 + k;
            if (i >= i1) break;
            const uint32_t lt = s_mark[k];  // >= 1: position 0 carries the chunk's first topic
            const uint64_t d = (uint64_t)((int64_t)i + s_shift[lt - 1]);
            if (d < cap) out[d] = (uint64_t)ids[base.b[r] + i];
        }
    }
}

hipError_t launch_merge_shard_ids(uint32_t G, uint32_t n, const uint32_t *roff, uint64_t roff_stride, const void *ids,
                                  uint32_t id_bytes, const uint64_t *base, uint32_t *off, uint64_t *out, uint64_t cap,
                                  uint32_t max_total, hipStream_t s) {
    if (G == 0 || G > MERGE_MAX_G) return hipErrorInvalidValue;
    ShardBases b{};
    for (uint32_t r = 0; r < G; r++) b.b[r] = base[r];
    k_roff_colsum<<<(n + 1 + 255) / 256, 256, 0, s>>>(roff, roff_stride, G, n, off);
    hipError_t e = hipGetLastError();
    if (e || !n || !cap || !max_total) return e;
    // chunks per rank from the caller's bound on any rank's total (the totals are on the device)
    const uint32_t cpr = (uint32_t)(((uint64_t)max_total + MG_CH - 1) / MG_CH);
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((uint64_t)G * cpr, 16384);
    if (id_bytes == 4)
        k_merge_ranks<uint32_t><<<blocks, MG_T, 0, s>>>(roff, roff_stride, G, n, (const uint32_t *)ids, b, off, out, cap,
                                                        cpr, max_total);
    else
        k_merge_ranks<uint64_t><<<blocks, MG_T, 0, s>>>(roff, roff_stride, G, n, (const uint64_t *)ids, b, off, out, cap,
                                                        cpr, max_total);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// Per-topic reducers over a full (TM_MATCH_ALL) result, IN PLACE: topic t's reduced list
// overwrites the head of its full list (a reduced list is never longer), its length goes
// to ucnt[t]:
//
//   DD_UNIQUE  matches/3 with [unique]: the walk visits keys in ascending ETS term order
//              and match_add/2 does Acc#{ID => K} (emqx_trie_search.erl:349-351), so per
//              id the GREATEST matching key survives.  key_rec[2h+1] is the key's order
//              code (engine.cpp key_ord): among keys that match one topic it orders them
//              exactly as Erlang term order does.
//   DD_AGGRE   emqx_broker:aggre/1 (emqx_broker.erl:361-377): keys of shared dests
//              (TM_ID_SHARED) collapse per {Filter, Group}; a filter is (node slot, '#'
//              flag) among the keys of one topic; the largest handle represents the class.
//
// Only some keys can ever collapse, and the engine flags them per handle in key_dd:
//   KDD_MULTI   (UNIQUE) the key's id is carried by more than one live key of the index —
//               a key whose id is its own can meet no other key of that id;
//   KDD_SHARED  (AGGRE) the key's dest is a shared-subscription member.
// So the reduction is two launches:
//   k_dd_pass   one wave per 64 topics, read-only over the keys: streams the 64 lists
//               as one sequence (DDP_U keys per lane in flight) and gathers the handles'
//               1-byte flags.  A topic with fewer than two flagged keys is final as it
//               stands (ucnt = cnt); the others go to a worklist with their flagged-key
//               count.
//   k_dedupe    one wave per worklist topic: a per-wave LDS hash table {class, max value}
//               over the flagged keys only (unflagged keys are kept as they are).
//     * up to DD_REG keys (nearly all lists): ONE pass with every key held in registers,
//       all loads issued before the first is used;
//     * longer lists: ceil(flagged / DD_PASS) passes, pass p handling the classes whose
//       hash falls in p, so the table never runs past half full; every pass re-reads the
//       list, so it is first copied to a scratch array at the same offsets.
//     Insert = CAS on the class word, then a 64-bit LDS atomic max on the value; every
//     lane's probe loop ends on its own CAS result, so no lane waits on another.
constexpr int DD_TAB = 1024;   // slots per wave (16 KiB of LDS)
constexpr uint32_t DD_PASS = 512;
constexpr int DD_U = 8;        // keys per lane in the one-pass case
constexpr uint32_t DD_REG = 64u * DD_U;
constexpr uint64_t DD_EMPTY = ~0ull;
constexpr uint64_t ORD_HASH_FLAG = 1ull << 63;  // key_rec ord bit 63: a '#' key (not part of the order)
constexpr int DDP_U = 8;       // keys per lane per round in k_dd_pass

__device__ __forceinline__ uint8_t dd_bit(uint32_t mode) { return mode == DD_UNIQUE ? KDD_MULTI : KDD_SHARED; }

struct DdKey {
    uint64_t cls, val;
    bool dd;  // false: never deduplicated (kept as is)
};

// class and value of a FLAGGED key
__device__ __forceinline__ DdKey dd_class(uint32_t mode, uint32_t h, const uint64_t *key_rec,
                                          const uint32_t *key_node) {
    const ulonglong2 r = *reinterpret_cast<const ulonglong2 *>(key_rec + 2ull * h);  // {id, ord}
    if (mode == DD_UNIQUE) return DdKey{r.x, r.y & ~ORD_HASH_FLAG, true};
    if (!(r.x >> 63)) return DdKey{0, 0, false};  // plain node dest (a stale flag): always kept
    return DdKey{((uint64_t)key_node[h] << 32) | (((r.x >> 32) & 0x7FFFFFFFull) << 1) | (r.y >> 63), h, true};
}

__global__ __launch_bounds__(64) void k_dd_pass(uint32_t mode, const uint32_t *cnt, const uint32_t *off,
                                                const uint32_t *keys, uint64_t keys_cap, const uint8_t *key_dd,
                                                uint32_t n, uint32_t *ucnt, uint2 *wl, uint32_t *wl_n) {
    __shared__ uint32_t s_start[65];  // exclusive prefix of the 64 topics' counts
    __shared__ uint32_t s_off[64];
    __shared__ uint32_t s_nflag[64];
    const uint32_t lane = threadIdx.x;
    const uint32_t t = blockIdx.x * 64 + lane;
    uint32_t c = 0, o = 0;
    if (t < n) {
        c = cnt[t];
        o = off[t];
        if ((uint64_t)o + c > keys_cap) c = 0;  // overflowed batch: the caller re-runs it
    }
    const uint32_t x = wave_incl_scan_dpp(c);  // inclusive scan over the wave
    s_start[lane + 1] = x;
    if (lane == 0) s_start[0] = 0;
    s_off[lane] = o;
    s_nflag[lane] = 0;
    const uint32_t total = lane_value(x, 63);
    __syncthreads();
    const uint8_t bit = dd_bit(mode);
    // the 64 topics' lists as one sequence, 64 * DDP_U keys per round; a lane's key index
    // only grows, so its topic cursor only moves forward
    uint32_t ti = 0;
    for (uint32_t base = 0; base < total; base += 64 * DDP_U) {
        uint32_t hh[DDP_U], tt[DDP_U];
#pragma unroll
        for (int u = 0; u < DDP_U; u++) {
            const uint32_t j = base + u * 64 + lane;
            hh[u] = 0;
            tt[u] = 64;
            if (j < total) {
                while (s_start[ti + 1] <= j) ti++;
                hh[u] = keys[(uint64_t)s_off[ti] + (j - s_start[ti])];
                tt[u] = ti;
            }
        }
#pragma unroll
        for (int u = 0; u < DDP_U; u++)
            if (tt[u] < 64 && (key_dd[hh[u]] & bit)) atomicAdd(&s_nflag[tt[u]], 1u);
    }
    __syncthreads();
    if (t < n) {
        const uint32_t nf = s_nflag[lane];
        if (nf >= 2) wl[atomicAdd(wl_n, 1u)] = make_uint2(t, nf);
        else ucnt[t] = c;
    }
}

struct DdTable {
    unsigned long long *cls, *val, *ff;
    uint32_t mask;
    __device__ __forceinline__ void insert(const DdKey &k) const {
        if (k.cls == DD_EMPTY) {
            atomicMax(ff, (unsigned long long)k.val);
            return;
        }
        uint32_t s = (uint32_t)mix64(k.cls) & mask;
        for (;;) {
            const unsigned long long prev = atomicCAS(&cls[s], DD_EMPTY, (unsigned long long)k.cls);
            if (prev == DD_EMPTY || prev == k.cls) {
                atomicMax(&val[s], (unsigned long long)k.val);
                return;
            }
            s = (s + 1) & mask;
        }
    }
    __device__ __forceinline__ bool winner(const DdKey &k) const {
        if (k.cls == DD_EMPTY) return *ff == k.val;
        uint32_t s = (uint32_t)mix64(k.cls) & mask;
        while (cls[s] != k.cls) s = (s + 1) & mask;
        return val[s] == k.val;
    }
};

__global__ __launch_bounds__(64) void k_dedupe(uint32_t mode, const uint32_t *cnt, const uint32_t *off,
                                               uint32_t *keys, const uint64_t *key_rec, const uint32_t *key_node,
                                               const uint8_t *key_dd, const uint2 *wl, const uint32_t *wl_n,
                                               uint32_t *ucnt, uint32_t *scratch) {
    __shared__ unsigned long long t_cls[DD_TAB];
    __shared__ unsigned long long t_val[DD_TAB];
    __shared__ unsigned long long ff_val;  // the one class equal to DD_EMPTY (UNIQUE id ~0)
    const uint32_t lane = threadIdx.x;
    const uint8_t bit = dd_bit(mode);
    const uint32_t nwl = *wl_n;
    for (uint32_t w = blockIdx.x; w < nwl; w += gridDim.x) {
        const uint2 job = wl[w];
        const uint32_t t = job.x, nflag = job.y;
        const uint32_t c = cnt[t];  // k_dd_pass listed only topics inside keys_cap
        const uint64_t o = off[t];
        uint32_t S = 64;
        while (S < 2 * nflag && S < (uint32_t)DD_TAB) S <<= 1;
        const DdTable T{t_cls, t_val, &ff_val, S - 1};
        for (uint32_t j = lane; j < S; j += 64) {
            t_cls[j] = DD_EMPTY;
            t_val[j] = 0;
        }
        if (lane == 0) ff_val = 0;
        uint32_t base = 0;
        if (c <= DD_REG) {
            uint32_t hh[DD_U];
            DdKey kk[DD_U];
#pragma unroll
            for (int u = 0; u < DD_U; u++) {
                const uint32_t i = u * 64 + lane;
                hh[u] = i < c ? keys[o + i] : 0u;
            }
#pragma unroll
            for (int u = 0; u < DD_U; u++) {
                const uint32_t i = u * 64 + lane;
                kk[u] = (i < c && (key_dd[hh[u]] & bit)) ? dd_class(mode, hh[u], key_rec, key_node)
                                                         : DdKey{0, 0, false};
            }
            __syncthreads();  // table cleared
#pragma unroll
            for (int u = 0; u < DD_U; u++)
                if (kk[u].dd) T.insert(kk[u]);
            __syncthreads();
#pragma unroll
            for (int u = 0; u < DD_U; u++) {
                if (u * 64u >= c) break;  // wave-uniform
                const uint32_t i = u * 64 + lane;
                const bool keep = i < c && (!kk[u].dd || T.winner(kk[u]));
                const uint64_t m = __ballot(keep);
                if (keep) keys[o + base + __popcll(m & ((1ull << lane) - 1))] = hh[u];  // reads all done
                base += __popcll(m);
            }
            __syncthreads();  // the table is cleared again for the next topic
        } else {
            for (uint32_t i = lane; i < c; i += 64) scratch[o + i] = keys[o + i];
            const uint32_t *src = scratch;  // the passes read the copy and compact into keys
            const uint32_t P = (nflag + DD_PASS - 1) / DD_PASS;
            for (uint32_t p = 0; p < P; p++) {
                if (p) {
                    for (uint32_t j = lane; j < S; j += 64) {
                        t_cls[j] = DD_EMPTY;
                        t_val[j] = 0;
                    }
                    if (lane == 0) ff_val = 0;
                }
                __syncthreads();
                for (uint32_t i = lane; i < c; i += 64) {
                    const uint32_t h = src[o + i];
                    if (!(key_dd[h] & bit)) continue;
                    const DdKey k = dd_class(mode, h, key_rec, key_node);
                    if (k.dd && (uint32_t)(mix64(k.cls) >> 40) % P == p) T.insert(k);
                }
                __syncthreads();
                for (uint32_t i0 = 0; i0 < c; i0 += 64) {
                    const uint32_t i = i0 + lane;
                    bool keep = false;
                    uint32_t h = 0;
                    if (i < c) {
                        h = src[o + i];
                        const DdKey k = (key_dd[h] & bit) ? dd_class(mode, h, key_rec, key_node) : DdKey{0, 0, false};
                        if (!k.dd) keep = p == 0;  // never deduplicated: emitted once, in the first pass
                        else keep = (uint32_t)(mix64(k.cls) >> 40) % P == p && T.winner(k);
                    }
                    const uint64_t m = __ballot(keep);
                    if (keep) keys[o + base + __popcll(m & ((1ull << lane) - 1))] = h;
                    base += __popcll(m);
                }
                __syncthreads();
            }
        }
        if (lane == 0) ucnt[t] = base;
    }
}

hipError_t launch_dedupe_wl(uint32_t mode, const uint32_t *cnt, const uint32_t *off, uint32_t *keys,
                            const uint64_t *key_rec, const uint32_t *key_node, const uint8_t *key_dd, uint32_t n,
                            uint32_t *ucnt, uint32_t *scratch, const uint2 *wl, const uint32_t *wl_n, hipStream_t s) {
    if (!n) return hipSuccess;
    const uint32_t grid = n < 4096u ? n : 4096u;
    k_dedupe<<<grid, 64, 0, s>>>(mode, cnt, off, keys, key_rec, key_node, key_dd, wl, wl_n, ucnt, scratch);
    return hipGetLastError();
}

hipError_t launch_dedupe(uint32_t mode, const uint32_t *cnt, const uint32_t *off, uint32_t *keys, uint64_t keys_cap,
                         const uint64_t *key_rec, const uint32_t *key_node, const uint8_t *key_dd, uint32_t n,
                         uint32_t *ucnt, uint32_t *scratch, uint2 *wl, uint32_t *wl_n, hipStream_t s) {
    if (!n) return hipSuccess;
    hipError_t e = hipMemsetAsync(wl_n, 0, 4, s);
    if (e) return e;
    k_dd_pass<<<(n + 63) / 64, 64, 0, s>>>(mode, cnt, off, keys, keys_cap, key_dd, n, ucnt, wl, wl_n);
    if ((e = hipGetLastError())) return e;
    const uint32_t grid = n < 4096u ? n : 4096u;
    k_dedupe<<<grid, 64, 0, s>>>(mode, cnt, off, keys, key_rec, key_node, key_dd, wl, wl_n, ucnt, scratch);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
__global__ void k_scatter1(uint8_t *dst, const uint64_t *idx, const uint8_t *src, uint64_t n, uint64_t cap,
                           unsigned long long *bnd) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[BIR(idx[i], cap, bnd)] = src[i];
}

hipError_t launch_scatter1(uint8_t *dst, const uint64_t *idx, const uint8_t *src, uint64_t n, hipStream_t s,
                           uint64_t cap, unsigned long long *bnd) {
    if (!n) return hipSuccess;
    k_scatter1<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dst, idx, src, n, cap, bnd);
    return hipGetLastError();
}

__global__ void k_scatter8(uint64_t *dst, const uint64_t *idx, const uint64_t *src, uint64_t n, uint64_t cap,
                           unsigned long long *bnd) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[BIR(idx[i], cap, bnd)] = src[i];
}

hipError_t launch_scatter8(uint64_t *dst, const uint64_t *idx, const uint64_t *src, uint64_t n, hipStream_t s,
                           uint64_t cap, unsigned long long *bnd) {
    if (!n) return hipSuccess;
    k_scatter8<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dst, idx, src, n, cap, bnd);
    return hipGetLastError();
}

// ---------------------------------------------------------------------------
// The edge table image of a full publish: every slot empty, then each node's record in its
// slot.  HBM-bound writes (20 B per slot, then 20 B per node at random slots).
__global__ void k_edge_clear(uint4 *etab, uint32_t *slot_list, uint64_t lo, uint64_t hi, uint64_t buf_slots,
                             unsigned long long *bnd) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < hi; i += stride) {
        const uint64_t j = BIR(i, buf_slots, bnd);
        etab[j] = make_uint4(NONE, 0u, 0u, 0u);
        slot_list[j] = 0u;
    }
}

__global__ void k_edge_place(uint4 *etab, uint32_t *slot_list, const NodeImage *nodes, uint64_t n, uint64_t cap,
                             uint64_t buf_slots, unsigned long long *bnd) {
    const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
        const NodeImage r = nodes[i];
        // a record past the table the publish sized (cap) would be a host bug: the bounds build
        // reports it against the table's size, not the buffer's
        const uint64_t j = BIR(BIR(r.slot, cap, bnd), buf_slots, bnd);
        etab[j] = make_uint4(r.parent, r.word, r.bloom, r.info);
        slot_list[j] = r.list;
    }
}

// Both kernels run beside the matches of the image being replaced (a full publish into the
// standby): at most EDGE_IMAGE_BLOCKS workgroups each (grid-stride), so they hold two of a CU's
// wave slots instead of all of them; the matches' waves keep the rest (a match of 131,072
// publishes beside an uncapped build took 1-2.6 ms instead of 0.135).  The
// engine also launches them in slices (launch_edge_*_range), paced from the host, so a match
// shares the memory system with at most one slice.
constexpr uint64_t EDGE_IMAGE_BLOCKS = 512;

hipError_t launch_edge_clear_range(uint4 *etab, uint32_t *slot_list, uint64_t lo, uint64_t hi, hipStream_t s,
                                   uint64_t buf_slots, unsigned long long *bnd) {
    if (hi <= lo) return hipSuccess;
    const uint64_t want = (hi - lo + 255) / 256;
    k_edge_clear<<<(unsigned)std::min<uint64_t>(want, EDGE_IMAGE_BLOCKS), 256, 0, s>>>(etab, slot_list, lo, hi, buf_slots,
                                                                                       bnd);
    return hipGetLastError();
}

hipError_t launch_edge_place_range(uint4 *etab, uint32_t *slot_list, uint64_t cap, const NodeImage *nodes, uint64_t n,
                                   hipStream_t s, uint64_t buf_slots, unsigned long long *bnd) {
    if (!n) return hipSuccess;
    k_edge_place<<<(unsigned)std::min<uint64_t>((n + 255) / 256, EDGE_IMAGE_BLOCKS), 256, 0, s>>>(etab, slot_list, nodes, n,
                                                                                               cap, buf_slots, bnd);
    return hipGetLastError();
}

hipError_t launch_edge_image(uint4 *etab, uint32_t *slot_list, uint64_t cap, const NodeImage *nodes, uint64_t n,
                             hipStream_t s, uint64_t buf_slots, unsigned long long *bnd) {
    if (!cap) return hipSuccess;
    hipError_t e = launch_edge_clear_range(etab, slot_list, 0, cap, s, buf_slots, bnd);
    if (e) return e;
    return launch_edge_place_range(etab, slot_list, cap, nodes, n, s, buf_slots, bnd);
}

}  // namespace tmx
