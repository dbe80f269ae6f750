/*
 * emqx_tm.h — C-ABI of the MI355X batched topic-matching engine.
 *
 * This is the drop-in boundary for EMQX's routing hot path: the lookup that
 * emqx_router:match_routes/1 -> emqx_topic_index:matches/3 -> emqx_trie_search
 * performs for every PUBLISH.  Everything above this header (an Erlang NIF, the
 * Python mirror in emqx_amd/, bench.py) calls only these symbols; everything
 * below it (host trie builder, delta epochs, HIP kernels for gfx950) is private.
 *
 * Reference interfaces replaced (paths relative to the ivangsm/emqx tree):
 *   tm_create / tm_destroy      emqx_topic_index:new/0,1          apps/emqx/src/emqx_topic_index.erl:40-48
 *   tm_apply (TM_OP_ADD)        emqx_topic_index:insert/4         apps/emqx/src/emqx_topic_index.erl:53-56
 *                               emqx_router:do_add_route/2 (v2)   apps/emqx/src/emqx_router.erl:194-196,483-490
 *   tm_apply (TM_OP_DEL)        emqx_topic_index:delete/3         apps/emqx/src/emqx_topic_index.erl:60-62
 *                               emqx_router:do_delete_route/2     apps/emqx/src/emqx_router.erl:238-240,497-509
 *   tm_apply batch + commit     emqx_router:do_batch/1 (syncer)   apps/emqx/src/emqx_router.erl:255-257,
 *                                                                 apps/emqx/src/emqx_router_syncer.erl:381-401
 *   tm_match_batch (ALL)        emqx_topic_index:matches/3 ([])   apps/emqx/src/emqx_topic_index.erl:76-78
 *                               emqx_router:match_routes/1 (v2)   apps/emqx/src/emqx_router.erl:205-212,511-516
 *   tm_match_batch (UNIQUE)     emqx_topic_index:matches/3 ([unique])  apps/emqx/src/emqx_trie_search.erl:350-352
 *   tm_match_batch (FIRST)      emqx_topic_index:match/2 (return_first) apps/emqx/src/emqx_trie_search.erl:171-178
 *   tm_match_filter_batch(_runs) emqx_topic_index:matches_filter/3 apps/emqx/src/emqx_topic_index.erl:82-84,
 *                               emqx_trie_search:matches_filter/3 apps/emqx/src/emqx_trie_search.erl:186-189
 *   tm_intersect_batch          emqx_topic:intersection/2         apps/emqx/src/emqx_topic.erl:111-151
 *   tm_key_info                 emqx_topic_index:get_id/1, get_topic/1 apps/emqx/src/emqx_topic_index.erl:87-94
 *   tm_stats                    emqx_router:stats/1 (n_routes)    apps/emqx/src/emqx_router.erl:632-635
 *
 * Conventions
 *   - No exceptions cross this ABI.  Every call returns an int status (TM_OK = 0,
 *     negative on error); tm_last_error() gives a message for the last failure.
 *   - A "key" is the reference's index key {Filter, {ID}} (emqx_trie_search.erl:110):
 *     one (filter, id) pair.  Inserting the same pair twice is one key; deleting a
 *     missing key is not an error (emqx_topic_index.erl:58-62).  The engine names
 *     each live key by a stable u32 "key handle"; matches are reported as handles.
 *   - Topics whose levels include a level exactly equal to "+" or "#" get the
 *     per-topic status TM_BADARG, mirroring error(badarg) in
 *     emqx_trie_search:word/2 (emqx_trie_search.erl:374-375).
 *   - Ops are staged by tm_apply and become visible atomically at tm_commit_epoch
 *     (one delta epoch).  Within one epoch the LAST op per key wins, the rule of
 *     emqx_router_syncer:merge_route_op/2.  A match batch always sees exactly one
 *     committed epoch (stronger than ETS' per-key atomicity).  Staged ops are invisible to
 *     matches until their commit: a match never fails because writes are pending.
 *   - Failed commits (emqx_router_syncer.erl:269-277 keeps a failed batch's stash and
 *     retries it): a commit that would exceed a capacity (trie nodes, terminal-list arena;
 *     tm_config.max_nodes / max_list_words lower them) returns TM_ENOMEM BEFORE changing
 *     anything: its ops stay staged (in order, ahead of any staged since), matches keep
 *     serving the previous epoch, and the next tm_commit_epoch retries them
 *     (tm_discard_staged drops them instead).  A commit whose device upload fails after the
 *     host copy advanced returns TM_ENOMEM / TM_EDEVICE with the device still holding the
 *     previous epoch intact; the next commit uploads the whole index again.
 *   - Threading.  One engine drives one GPU (tm_config.device).  Every entry point may be
 *     called from any number of threads at once, in any mix (the reference index is a
 *     public, read_concurrency ETS table written by any process, emqx_topic_index.erl:41-42;
 *     emqx_router.erl:141-160).  Inside: staging never waits for matches or commits; a
 *     commit's host work (the trie, the lists, and a full rebuild's upload into a standby
 *     device image) runs beside the matches, which wait only while the commit publishes
 *     (a delta's in-place scatters, or the pointer swap of a standby image).  Host results
 *     (tm_result, tm_runs_result, tm_intersect_result) belong to the calling thread: valid
 *     until that thread's next call of the same kind.  Device results (tm_dev_result) belong
 *     to the engine: valid until the next tm_match_device* call from ANY thread, which the
 *     engine orders after everything already queued on the previous call's stream (keep
 *     that stream alive until then).  tm_last_error() is per thread.  Host-form calls
 *     (tm_match_batch, tm_match_batch_runs) of different threads run concurrently: each
 *     thread has its own device lane (batch buffers, streams, pinned staging), and a call
 *     holds the engine's device lock only while it queues work that reads the index
 *     (UNIQUE / AGGRE and word-list topics keep it for the whole call).  Give the process
 *     one HIP hardware queue per concurrent caller or more (GPU_MAX_HW_QUEUES).
 */
#ifndef EMQX_TM_H
#define EMQX_TM_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define TM_ABI_VERSION 10u

/* status codes */
#define TM_OK          0
#define TM_EINVAL     (-1)   /* bad argument */
#define TM_ENOMEM     (-2)   /* host or device allocation failed */
#define TM_EDEVICE    (-3)   /* HIP runtime error / no gfx950 device */
#define TM_ESTATE     (-4)   /* call not valid in this state */
#define TM_ENOTFOUND  (-5)   /* key handle not live */

/* per-topic status in tm_result.status */
#define TM_TOPIC_OK      0
#define TM_BADARG        1   /* a level is exactly "+" or "#" */

/* op kinds for tm_op.op */
#define TM_OP_ADD 1u
#define TM_OP_DEL 2u

/* tm_op.flags */
#define TM_KEY_WORDS 1u  /* key was given as a word list (emqx_trie_search:make_key/2 list
                            clause, :127-128).  For a filter WITHOUT wildcards this is a
                            different key from the binary form (:121-125); for a wildcard
                            filter both forms are the same key. */

/* match modes for tm_match_batch */
#define TM_MATCH_ALL    0u  /* every matching key (matches/3 with [])            */
#define TM_MATCH_UNIQUE 1u  /* one key per id (matches/3 with [unique])          */
#define TM_MATCH_FIRST  2u  /* the first key in ETS term order (match/2); on the GPU
                               (k_match_first): topic i's key, if any, is keys[off[i]]  */
#define TM_MATCH_COUNT  3u  /* counts only, no keys: has_any_route/1
                               (emqx_persistent_session_ds_router.erl:115-125) is cnt > 0 */
#define TM_MATCH_AGGRE  4u  /* emqx_broker:aggre/1 (emqx_broker.erl:361-377): keys whose id is a
                               shared-subscription dest (TM_ID_SHARED) collapse to one key per
                               {Filter, Group}; every other key is kept */
/* OR'd into tm_match_batch's mode: the topics are pre-split word lists, '/'-joined
 * (matches/3's `[word()]` form, emqx_trie_search.erl:182, topic_words/1 :369-370).  A "+" or "#"
 * level is then a plain word (no TM_BADARG), and keys given as binaries ({Binary, {ID}})
 * do not match (match_topics/4 compares the list itself, :380-389).  With ALL, UNIQUE, FIRST
 * and COUNT; not on replicas.  Words containing '/' have no joined form. */
#define TM_MATCH_TOPIC_WORDS 0x100u

/* Route-id convention for TM_MATCH_AGGRE: a $share/$queue dest {Group, Node}
 * (emqx_shared_sub.erl:444-456) gets an id with TM_ID_SHARED set and its group index in
 * bits 32..62; the low 32 bits tell the nodes of one group apart.  Ids without the flag
 * are plain node dests. */
#define TM_ID_SHARED        (1ull << 63)
#define TM_ID_GROUP(id)     (((id) >> 32) & 0x7FFFFFFFull)
#define TM_SHARED_ID(group, member) (TM_ID_SHARED | ((uint64_t)(group) << 32) | (uint32_t)(member))

/* tm_config.flags */
#define TM_CFG_FORCE_SLOW   1u  /* route every topic through the spill (slow) kernel: test aid */
#define TM_CFG_RECORD_PATCH 2u  /* master of a replicated index: every commit records the device
                                   changes it made as an epoch patch (tm_patch_export) */
#define TM_CFG_FAIL_HOST_CALLS 4u /* test aid: tm_match_batch_runs fails (TM_EDEVICE) after taking
                                     its read lease, to check a failed call leaves no lease held */
#define TM_CFG_FAIL_FLUSH_ONCE 8u /* test aid (ABI 10): the first delta commit that scatters fails
                                     in its upload, as an out-of-HBM staging buffer would */
#define TM_CFG_EDGE_EXACT 16u     /* (ABI 10) size the edge table at reserve_nodes x edge_load_inv
                                     slots rounded up to 64, not to a power of two (the table
                                     takes any slot count up to 0xF0000000; it still doubles when
                                     it fills, up to that cap) */

typedef struct tm_engine tm_engine;

typedef struct tm_config {
    int32_t  device;        /* HIP device ordinal                                  */
    uint32_t flags;         /* TM_CFG_*                                            */
    uint32_t reserve_keys;  /* capacity hints (0 = default); tables grow as needed */
    uint32_t reserve_nodes;
    uint32_t reserve_topics;      /* largest batch expected                    */
    uint32_t reserve_matches;     /* expected matches per batch (output arena) */
    uint32_t seg_chunks;          /* 0 = auto; else fixed size of the key-segment and
                                     frontier-overflow chunk pools (test aid: exhaustion
                                     routes topics to the spill kernel, results stay exact) */
    uint32_t edge_load_inv;       /* edge-table load <= 1/edge_load_inv (0 = default 16): a wave
                                     waits for its longest probe chain, so lower load shortens
                                     the walk at the price of HBM (16 B per slot) */
    uint32_t topics_per_wave;     /* 0 = by batch size (4..64); else 4, 8, 16, 32 or 64 */
    uint32_t max_nodes;           /* trie-node budget (0 = the edge table's limit, 0x78000000): a commit
                                     that would pass it fails with TM_ENOMEM, ops kept staged */
    uint32_t max_list_words;      /* terminal-list arena budget in u32 words (0 = 2^32 - 16) */
} tm_config;

typedef struct tm_op {
    uint32_t       op;          /* TM_OP_ADD | TM_OP_DEL          */
    uint32_t       flags;       /* TM_KEY_*                       */
    const uint8_t *filter;      /* filter bytes (not NUL-terminated) */
    uint32_t       filter_len;  /* <= 65535 (MQTT max topic length) */
    uint32_t       _pad;
    uint64_t       id;          /* caller's record id / route dest id */
} tm_op;

/* Result of one match batch.  Engine-owned host memory, valid until the next
 * tm_match_batch / tm_commit_epoch / tm_destroy on the same engine.
 * Topic i's matches are keys[off[i] .. off[i]+cnt[i]), in unspecified order
 * (the reference returns them in reverse ETS term order; callers must not rely
 * on order).  In TM_MATCH_FIRST mode cnt[i] is 0 or 1.  Lists need not be contiguous:
 * TM_MATCH_UNIQUE / TM_MATCH_AGGRE reduce each list in place of the full one. */
typedef struct tm_result {
    uint32_t        n;
    uint32_t        _pad;
    uint64_t        total;     /* sum of cnt[]                      */
    const uint32_t *off;       /* n entries                         */
    const uint32_t *cnt;       /* n entries                         */
    const uint32_t *keys;      /* key handles                       */
    const int32_t  *status;    /* n entries: TM_TOPIC_OK / TM_BADARG */
} tm_result;

/* Device-resident result (tm_match_device): device pointers, engine-owned. */
typedef struct tm_dev_result {
    uint32_t  n;
    uint32_t  _pad;
    uint32_t *d_off;      /* n entries: start of topic i's keys in d_keys   */
    uint32_t *d_cnt;      /* n entries                                      */
    uint32_t *d_keys;     /* capacity tm_dev_result.keys_cap                */
    int32_t  *d_status;   /* n entries                                      */
    uint64_t *d_total;    /* 1 entry: keys requested by the batch (device)  */
    uint64_t  keys_cap;
} tm_dev_result;

typedef struct tm_stats_t {
    uint64_t epoch;
    uint64_t n_keys;        /* live keys (emqx_router:stats(n_routes))      */
    uint64_t n_nodes;       /* trie nodes incl. root                        */
    uint64_t n_words;       /* interned level words                         */
    uint64_t edge_slots;    /* device edge-table capacity (slots)           */
    uint64_t word_slots;    /* device word-table capacity (slots)           */
    uint64_t list_words;    /* u32 words in the terminal-list arena (live+garbage) */
    uint64_t device_bytes;  /* HBM held by the frozen index (the standby image, standby_bytes,
                               is not included) */
    uint64_t n_full_rebuilds;
    uint64_t n_delta_commits;
    uint64_t n_slow_topics; /* topics routed to the spill kernel in the last batch */
    /* wall time of the last tm_commit_epoch by phase, microseconds (host clock):
     * staged ops folded into the host trie / lists rebuilt or appended / device upload */
    uint64_t commit_apply_us;
    uint64_t commit_lists_us;
    uint64_t commit_upload_us;
    uint64_t n_deep_keys;   /* live word-list keys deeper than the device order code (31 levels) */
    uint64_t n_filter_onepass;  /* tm_match_filter_batch batches walked once (keys chunked on device) */
    uint64_t n_filter_twopass;  /* ... that needed the count + emit passes (output sized from them) */
    uint64_t commit_stall_us;   /* last commit: how long matches were held back while it published
                                   (a delta's in-place scatters; a full rebuild's standby swap) */
    uint64_t n_commits_refused; /* commits refused for capacity, ops kept staged               */
    uint64_t n_staged;          /* ops staged now (not yet committed)                          */
    uint64_t standby_bytes;     /* (ABI 10) device bytes of the standby image a full publish
                                   uploads into (0: none kept; the next one allocates)         */
} tm_stats_t;

/* lifecycle --------------------------------------------------------------- */
uint32_t    tm_abi_version(void);
/* "src_sha=<sha256 of the library's sources> abi=<n> arch=gfx950": ties a built library to the
 * sources it was built from (emqx_amd/build.py src_sha). */
const char *tm_build_info(void);
int         tm_create(const tm_config *cfg, tm_engine **out);
void        tm_destroy(tm_engine *eng);
const char *tm_last_error(const tm_engine *eng);
/* Why the calling thread's last tm_create / tm_replica_create failed ("" after a success on
 * that thread, or before any call). */
const char *tm_create_last_error(void);

/* writes ------------------------------------------------------------------ */
int tm_apply(tm_engine *eng, const tm_op *ops, size_t n);
/* Bulk form of tm_apply for one op kind: filter i is bytes[off[i] .. off[i+1])
 * (off has n+1 entries), id ids[i], flags flags[i] (flags may be NULL). */
int tm_apply_packed(tm_engine *eng, uint32_t op, const uint8_t *bytes, const uint64_t *off,
                    const uint64_t *ids, const uint32_t *flags, size_t n);
int tm_commit_epoch(tm_engine *eng, uint64_t *epoch_out);
/* Drop every staged op (e.g. a batch a capacity error refused); *n_out = ops dropped. */
int tm_discard_staged(tm_engine *eng, uint64_t *n_out);
/* Free the calling thread's host result buffers (tm_result / tm_intersect_result / runs), its
 * device lane (the batch buffers and streams its host-form calls use) and end its runs lease;
 * results it still points to become invalid.  A thread that stops calling the engine calls it
 * (a NIF's dirty scheduler threads live as long as the VM and need not). */
int tm_result_release(tm_engine *eng);

/* reads ------------------------------------------------------------------- */
/* Host buffers in, host result out (H2D + kernels + D2H inside).
 * Topic i is bytes[off[i] .. off[i+1]); `off` has n+1 entries.  TM_MATCH_ALL batches of
 * 524,288 topics or more are pipelined: sub-batches of about 262,144 topics on two streams,
 * each one's staging, H2D and walk overlapping the previous one's D2H (PCIe is this path's
 * bound).  The device then holds sub-batch results, not the batch: tm_result_ids_device*
 * refuse (TM_ESTATE) until the next tm_match_device* call. */
int tm_match_batch(tm_engine *eng, const uint8_t *bytes, const uint32_t *off,
                   uint32_t n, uint32_t mode, tm_result *out);

/* Runs form of tm_match_batch (TM_MATCH_ALL), for callers that consume route ids on the host
 * (emqx_broker:do_publish/1 -> match_routes/1, emqx_broker.erl:285-290; emqx_router.erl:648-649
 * turns each key into a #route{}).  The walk already knows each topic's matches as a few runs
 * of consecutive keys of the terminal-list arena; only those runs cross PCIe (16 B each, vs
 * 4 B per key), and each run is a span of the engine's HOST id arena: topic i's ids are the
 * concatenation of spans[span_off[i] .. span_off[i] + span_cnt[i]), kcnt[i] ids in all, in
 * unspecified order (the same multiset tm_match_batch + tm_key_ids gives).  The GPU writes
 * the spans themselves (host addresses), so the host does no per-key or per-run work: a
 * consumer reads each id once, where it builds its reply.  Zero-copy: the spans point
 * into engine memory that the calling thread holds a READ LEASE on until its next
 * tm_match_batch_runs, tm_runs_release or tm_result_release; a commit's host phase waits for
 * every lease (release promptly; a thread's own commit first ends its own lease).  On a
 * replica (round 4) the spans point into the host id arena it keeps from its device copy,
 * rebuilt at tm_replica_load and updated by tm_replica_apply_patch, which wait for the
 * leases the same way; so the aggregator's runs transport works on replicas too. */
typedef struct tm_span {
    const uint64_t *ids;
    uint64_t        n;
} tm_span;
typedef struct tm_runs_result {
    uint32_t        n;
    uint32_t        _pad;
    uint64_t        epoch;        /* the committed epoch matched        */
    uint64_t        total_ids;    /* sum of kcnt[]                      */
    uint64_t        total_spans;
    const uint32_t *span_off;     /* n entries                          */
    const uint32_t *span_cnt;     /* n entries                          */
    const tm_span  *spans;
    const uint32_t *kcnt;         /* n entries: ids of topic i          */
    const int32_t  *status;       /* n entries: TM_TOPIC_OK / TM_BADARG */
} tm_runs_result;
int tm_match_batch_runs(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n,
                        tm_runs_result *out);
int tm_runs_release(tm_engine *eng);
/* Device buffers in, device result out, asynchronous on the engine's stream
 * (or on `stream` if non-NULL: a hipStream_t).  The engine's own stream is
 * non-blocking: work the caller queues on other streams (including the legacy
 * default stream) is NOT ordered after it; pass your stream, or tm_device_sync()
 * first.  `d_off` has n+1 entries and
 * total_bytes = d_off[n] - d_off[0] (it sizes the spill kernel's scratch).
 * Call tm_device_sync() before reading; if *d_total > keys_cap the batch
 * overflowed and must be re-run after tm_reserve_matches().
 * Batch limits: total topic bytes < 4 GiB, total matches < 4 Gi keys. */
int tm_match_device(tm_engine *eng, const uint8_t *d_bytes, const uint32_t *d_off,
                    uint32_t n, uint64_t total_bytes, void *stream, tm_dev_result *out);
/* Wait for the last tm_match_device batch; refresh tm_stats().n_slow_topics and size
 * the internal chunk pools to that batch's demand for the next one. */
int tm_device_sync(tm_engine *eng);
/* tm_match_device with a match mode: TM_MATCH_ALL (= tm_match_device), TM_MATCH_FIRST
 * (one key per topic, d_total not used), TM_MATCH_COUNT (d_cnt only), TM_MATCH_UNIQUE or
 * TM_MATCH_AGGRE (the full set is reduced on the GPU: topic i's keys are
 * d_keys[d_off[i] .. d_off[i]+d_cnt[i]); *d_total still counts the UNREDUCED keys and
 * decides overflow as for TM_MATCH_ALL).  TM_MATCH_UNIQUE returns TM_ESTATE while the index
 * holds a filter of more than 31 levels (its term order does not fit the device's 64-bit
 * order code); tm_match_batch then reduces on the host. */
int tm_match_device_mode(tm_engine *eng, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                         uint64_t total_bytes, uint32_t mode, void *stream, tm_dev_result *out);
/* Two device batches in flight (ABI 8).  tm_match_device_mode on direct buffer set `set`:
 * 0 is tm_match_device's own set, 1 a second one (2 a third, round 4) with its own scratch
 * and output, so a
 * caller alternating sets on two streams overlaps one batch's tail with the next batch's
 * start (a launch costs ~0.1 ms of ramp and tail at config C).  A set's
 * result stays valid until that set's next batch.  tm_device_sync_set(eng, set) is
 * tm_device_sync for that set; tm_reserve_matches grows both sets once set 1 is in use.
 * No reference counterpart: the broker-side caller decides how many batches it keeps
 * in flight (emqx_broker.erl:285-290 calls one publish at a time). */
int tm_match_device_set(tm_engine *eng, uint32_t set, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                        uint64_t total_bytes, uint32_t mode, void *stream, tm_dev_result *out);
int tm_device_sync_set(tm_engine *eng, uint32_t set);
int tm_reserve_matches(tm_engine *eng, uint64_t keys_cap, uint32_t topics_cap);

/* Route ids of the last tm_match_device* batch (all keys, TM_MATCH_ALL), compacted topic-major on
 * the device: topic i's ids are d_ids[d_off[i] .. d_off[i+1]); d_off has n+1 entries and
 * d_off[n] = *d_total.  This is get_id/1 (emqx_topic_index.erl:87-89) applied on the GPU to
 * every key, in the topic order a caller expects (emqx_router.erl:648-649 maps each key
 * to a #route{}).  Asynchronous on `stream` (NULL: the batch's stream).  Topics whose ids
 * would pass ids_cap are left unwritten: size d_ids from *d_total. */
int tm_result_ids_device(tm_engine *eng, uint64_t *d_ids, uint64_t ids_cap, uint32_t *d_off, void *stream);
/* tm_result_ids_device that also reports, ON THE DEVICE, whether the result is complete, so
 * a pipeline (the filter-sharded step, the batching aggregator) never waits on the host
 * between the walk and the next stage: d_flags[0] (one u32) := TM_RES_KEYS_OVERFLOW when the
 * walk asked for more keys than its output arena holds (*d_total > keys_cap: no ids are
 * written; re-run after tm_reserve_matches), | TM_RES_IDS_OVERFLOW when d_off[n] > ids_cap;
 * 0 when every id is in d_ids. */
#define TM_RES_KEYS_OVERFLOW 1u
#define TM_RES_IDS_OVERFLOW  2u
int tm_result_ids_device_ex(tm_engine *eng, uint64_t *d_ids, uint64_t ids_cap, uint32_t *d_off, uint32_t *d_flags,
                            void *stream);

/* The walk with the route ids written by the walk itself (the key -> id gather of
 * emqx_router:match_to_route/1, apps/emqx/src/emqx_router.erl:648-649, fused into the
 * copy-out; get_id/1, emqx_topic_index.erl:87-89, of every key), then compacted topic-major
 * on the device: topic i's ids are d_ids[d_off[i] .. d_off[i+1]) (d_off: n+1 entries,
 * d_off[n] = the batch's id count), ids of id_bytes each: 8 (u64), or 4 (u32: TM_ESTATE
 * unless every id the engine ever held is below 2^32).  d_flags (may be NULL): one u32 of
 * TM_RES_* bits written on the device (TM_RES_KEYS_OVERFLOW: the walk's own buffer was short,
 * call tm_reserve_matches and run again; TM_RES_IDS_OVERFLOW: d_off[n] > ids_cap).  Works on
 * replicas.  Asynchronous on `stream`; nothing waits on the host. */
int tm_match_ids_device(tm_engine *eng, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                        uint64_t total_bytes, uint32_t id_bytes, void *d_ids, uint64_t ids_cap, uint32_t *d_off_out,
                        uint32_t *d_flags, void *stream);

/* Filter-sharded merge over tm_match_ids_device results: rank r's d_off_out row (n+1 u32) at
 * d_roff + r * roff_stride, its ids (id_bytes each) at d_ids + base[r] elements (base: G
 * host values); max_rank_ids is what every rank's id buffer holds (e.g. the padded stride): a
 * rank whose row counts more (it raised TM_RES_IDS_OVERFLOW) is read only that far.  Writes
 * the merged result as u64: topic i's ids are the concatenation of its slices from shard
 * 0..G-1 at d_out_ids[d_out_off[i] .. d_out_off[i+1]) (n+1 offsets).  One column-sum launch
 * and one rank-chunk-parallel copy; ids past out_cap are left unwritten.  G <= 64. */
int tm_merge_shard_ids_device(tm_engine *eng, uint32_t G, uint32_t n, const uint32_t *d_roff, uint64_t roff_stride,
                              const void *d_ids, uint32_t id_bytes, const uint64_t *base, uint64_t max_rank_ids,
                              uint32_t *d_out_off, uint64_t *d_out_ids, uint64_t out_cap, void *stream);

/* Filter-sharded mode: G shards matched the same n topics against disjoint
 * key sets; shard r's compacted result (tm_result_ids_device) is counts[r*n .. r*n+n) and
 * ids[r*stride ..).  Writes the merged result: topic i's ids are the concatenation of its
 * slices from shard 0..G-1 at out_ids[out_off[i] .. out_off[i+1]) (shards are disjoint, so
 * nothing is deduplicated; the reference's own result is one unordered list per topic).
 * Device form: asynchronous on `stream`; topics past out_cap are left unwritten.
 * Host form: no device needed; TM_ENOMEM if out_cap is too small. */
int tm_merge_shards_device(tm_engine *eng, uint32_t G, uint32_t n, const uint32_t *d_counts, const uint64_t *d_ids,
                           uint64_t stride, uint32_t *d_out_off, uint64_t *d_out_ids, uint64_t out_cap,
                           void *stream);
int tm_merge_shards(uint32_t G, uint32_t n, const uint32_t *counts, const uint64_t *ids, uint64_t stride,
                    uint32_t *out_off, uint64_t *out_ids, uint64_t out_cap);

/* Replicated mode (DESIGN.md §6 mode 1).  The reference keeps one full route table per node,
 * replicated by mria (emqx_router.erl:133-162) and fed by one syncer per node
 * (emqx_router_syncer.erl:244-280).  Here ONE master engine per node holds the host master
 * copy and applies the route ops; every other GPU holds a READ REPLICA: the master's frozen
 * device index, copied device to device (RCCL broadcast over xGMI, or a peer copy), with no
 * host copy of its own.  Each commit's device changes travel as an epoch patch.
 *   tm_image_size / tm_image_export  the committed device index as one contiguous image
 *                                    (d_dst: device memory on the master's GPU; synchronous)
 *   tm_replica_create                a read-only engine on cfg->device from an image there
 *   tm_replica_load                  replace a replica's index with a newer image
 *   tm_patch_size / tm_patch_export  (master built with TM_CFG_RECORD_PATCH) the last commit's
 *                                    device changes as host bytes; *full = 1 when that commit
 *                                    re-uploaded everything: send an image instead
 *   tm_replica_apply_patch           replay a patch on a replica holding the epoch it was made
 *                                    from (TM_ESTATE otherwise: reload from an image)
 * A replica matches (tm_match_batch / tm_match_device*, tm_result_ids_device*) exactly like its
 * master at the same epoch; writes, tm_match_filter_batch and key introspection return
 * TM_ESTATE / TM_ENOTFOUND (route ids come back through tm_result_ids_device). */
int tm_image_size(const tm_engine *eng, uint64_t *bytes);
int tm_image_export(tm_engine *eng, void *d_dst, uint64_t cap, void *stream);
int tm_replica_create(const tm_config *cfg, const void *d_image, uint64_t bytes, void *stream, tm_engine **out);
int tm_replica_load(tm_engine *replica, const void *d_image, uint64_t bytes, void *stream);
int tm_patch_size(const tm_engine *master, uint64_t *bytes, int *full);
int tm_patch_export(const tm_engine *master, void *dst, uint64_t cap);
int tm_replica_apply_patch(tm_engine *replica, const void *patch, uint64_t bytes);

/* matches_filter/3: query i is a topic FILTER, bytes[off[i] .. off[i+1]).  Returns the keys
 * the reference's seek walk (emqx_trie_search.erl:192-258 with the filter-search clauses of
 * compare/3, :291-300) meets, as key handles in walk order (the reference's accumulator holds
 * the same keys reversed).  Only word-list keys can match ({Binary, {ID}} keys end the walk).
 * mode: TM_MATCH_ALL, TM_MATCH_UNIQUE (last key per id in walk order, listed by id) or
 * TM_MATCH_FIRST (the first key met).  A query with '#' before its last level gets per-query
 * status TM_BADARG: the reference's walk does not terminate on it.  The walk runs on the GPU
 * (filter_kernels.hip) over a term-ordered copy of the word-list keys that the first call
 * after each commit builds.  Result memory as for tm_match_batch, valid until the next
 * tm_match_filter_batch / tm_commit_epoch / tm_destroy. */
/* matches_filter/3 in runs form (ABI 9): the same walk, each query's keys as spans of the ids
 * of the term-ordered word-list keys, in walk order.  The walk's own output is ranges of that
 * order, so only the ranges cross PCIe (8 B each instead of 4 B per key).  mode: TM_MATCH_ALL or
 * TM_MATCH_FIRST.  Query i: spans[span_off[i] .. + span_cnt[i]), kcnt[i] ids, status[i].  The
 * spans point into a host copy of the ids made with the term-ordered index; it and the result
 * stay valid, across commits too, until this thread's next tm_match_filter_batch_runs on this
 * engine, its tm_result_release, or tm_destroy. */
int tm_match_filter_batch_runs(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode,
                               tm_runs_result *out);
int tm_match_filter_batch(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode,
                          tm_result *out);

/* emqx_topic:intersection/2 (apps/emqx/src/emqx_topic.erl:111-151), batched: pair i is
 * (a[a_off[i] .. a_off[i+1]), b[b_off[i] .. b_off[i+1])).  Pair i's result (join/1 of the
 * intersected words) is bytes[off[i] .. off[i]+len[i]) when len[i] >= 0; len[i] is
 * TM_INTERSECT_FALSE for `false`, TM_INTERSECT_BADHASH where join/1 raises
 * error('topic_invalid_#') (a '#' level before the last, only for invalid inputs).  No
 * index involved (engine = the GPU and stream to run on; kernel k_intersect).  Result memory
 * engine-owned until the next tm_intersect_batch / tm_destroy. */
#define TM_INTERSECT_FALSE   (-1)
#define TM_INTERSECT_BADHASH (-2)
typedef struct tm_intersect_result {
    uint32_t        n;
    uint32_t        _pad;
    const uint64_t *off;    /* n entries */
    const int32_t  *len;    /* n entries */
    const uint8_t  *bytes;
} tm_intersect_result;
int tm_intersect_batch(tm_engine *eng, const uint8_t *a, const uint32_t *a_off, const uint8_t *b,
                       const uint32_t *b_off, uint32_t n, tm_intersect_result *out);

/* key introspection (get_id/1, get_topic/1) */
int tm_key_info(const tm_engine *eng, uint32_t key, uint64_t *id, uint32_t *flags,
                uint8_t *filter_buf, uint32_t buf_cap, uint32_t *filter_len);
/* Bulk get_id/1: ids_out[i] = id of key handle keys[i] (TM_ENOTFOUND if any is not live). */
int tm_key_ids(const tm_engine *eng, const uint32_t *keys, size_t n, uint64_t *ids_out);
int tm_stats(const tm_engine *eng, tm_stats_t *out);

/* diagnostics: enable/disable device walk counters; when out18 != NULL, first
 * read the counters accumulated since the last call: {node visits, edge-slot
 * probes, word-slot probes, keys emitted, topic levels, topics spilled to the
 * slow kernel, key segments, segment-chunk flushes, frontier overflow chunks,
 * list-header reads, keys emitted inline from edge slots, the summed wave
 * cycles of the fast kernel's phases: stage+pre-scan, walk, copy-out; the same
 * three phases summed over the waves holding a topic with more than 256 keys
 * (under a hot '#' filter), and the number of such waves}. */
int tm_debug_stats(tm_engine *eng, int enable, uint64_t *out18);
/* diagnostics: the same counters by walk depth d (16 rows, the last = depth 15 and deeper),
 * read WITHOUT resetting (call before tm_debug_stats' read): out64[d] edge-slot probes,
 * out64[16 + d] summed wave cycles spent at depth d, out64[32 + d] frontier entries
 * expanded, out64[48 + d] dependent probe round trips (per wave). */
int tm_debug_depth_stats(tm_engine *eng, uint64_t *out64);
/* diagnostics: time the dominant kernel of the next match with HIP events on its
 * launch stream; enable=1 arms, then (after the match) enable=0 + ms_out reads. */
int tm_debug_timing(tm_engine *eng, int enable, float *ms_out);
/* test aid (ABI 9): the device index as delta commits left it vs a full publish of the same
 * host state, array by array; *diff_mask gets bit a for each differing array (0: identical;
 * the word table, word arena, word offsets, edge table, slot lists, list arena and root are
 * compared).  The full publish stays in place. */
int tm_debug_image_check(tm_engine *eng, uint32_t *diff_mask);
/* diagnostics (ABI 10): what the bounds-checked debug build (libemqx_tm_bounds.so, built with
 * TM_BOUNDS=1) found since the engine was created: *hits = device indices at or past a buffer's
 * real capacity (recorded and redirected by the kernels, so nothing faults) plus overwritten
 * canary tails plus host copies past a buffer's end; msg (cap bytes) the first findings.  The
 * product build returns TM_ENOTFOUND (it checks nothing). */
int tm_debug_bounds(tm_engine *eng, uint64_t *hits, char *msg, uint32_t cap);
/* diagnostics (ABI 10): steady-clock (CLOCK_MONOTONIC) microseconds of the last full publish's
 * steps, for attributing a match stall to one of them: out9[0..7] = start, node image
 * uploaded, edge table built, arrays staged, upload synced, swap begin, swap end, standby
 * kept (0: that step did not run); out9[8] = device buffers the publish (re)allocated. */
int tm_debug_commit_marks(const tm_engine *eng, uint64_t *out9);

#ifdef __cplusplus
}
#endif
#endif /* EMQX_TM_H */
