/* emqx_tm_batcher.h — publish batching aggregator over the topic-matching engine.
 *
 * The reference matches one publish per call: every emqx_broker:do_publish/1
 * (apps/emqx/src/emqx_broker.erl:285-290) runs emqx_router:match_routes/1
 * (apps/emqx/src/emqx_router.erl:205-212) synchronously in the publishing process.  A GPU
 * wants one call per WINDOW of publishes, so this aggregator sits between the many
 * concurrent publishers and tm_match_*: publishers submit single topics, a cutter thread
 * cuts the queue into windows, runs one engine batch per window and delivery threads hand
 * each publisher its own id list (SURVEY.md §8 (b) "Who calls it", §8 (f) f3).
 *
 *   window   a batch is dispatched when max_batch publishes are queued, or when the
 *            oldest queued publish has waited max_wait_us, or at tm_batcher_destroy
 *            (which drains the queue).  Six windows are in flight at once: the newest
 *            walk on the GPU (consecutive windows on two streams, each with its own engine
 *            buffer set, so their walks overlap) while earlier windows' ids cross PCIe and
 *            the oldest's publishers are called back; under load windows grow by themselves.
 *   result   per publish: TM_TOPIC_OK with the ids of its matched keys (route dests,
 *            emqx_topic_index:get_id/1 of every key, emqx_topic_index.erl:87-89), or
 *            TM_BADARG with no ids (a level exactly "+" or "#": emqx_trie_search.erl:374-375),
 *            or a negative TM_E* status when the batch failed as a whole.  COUNT mode
 *            gives the count and no ids.
 *   transport  TM_MATCH_ALL windows on a master engine travel as RUNS (tm_match_batch_runs):
 *            the walk's spans of the engine's host id arena cross PCIe, not the ids, and each
 *            publish's reply is read straight from the arena (one span: zero-copy; several:
 *            gathered by the delivery thread).  A window holds a read lease on the arena from
 *            its enqueue until its last callback returns; a commit waits for those leases, so
 *            every window sees exactly one committed epoch.  With EMQX_TM_RUNS_IDW=4 the spans
 *            are of the engine's u32 id arena while every id fits (a u32-span callback reads
 *            them in place, the others get them widened).  Other modes, and replicas, ship the
 *            ids (u32 while every id fits).
 *   writes   any thread may write the engine directly (tm_apply / tm_commit_epoch are safe
 *            beside the aggregator); tm_batcher_apply / tm_batcher_commit are the same calls.
 *            A delivery callback may stage (tm_apply) but not commit: tm_commit_epoch and
 *            tm_batcher_commit return TM_ESTATE on every delivery thread, whatever the
 *            transport.  A commit waits for the read leases of every runs window in flight,
 *            and only the delivery threads can finish those windows: a commit made from one of
 *            them could wait on a window queued behind its own (with one delivery thread it
 *            always would).  A callback's own tm_match_batch_runs call passes a waiting commit
 *            only when its window holds a lease (the arena cannot change meanwhile); a callback
 *            of a window without one (ids transport, other modes) waits for the commit.
 *
 * Erlang binding: a NIF calls tm_batcher_submit with a callback that
 * enif_send()s the id list to the publishing pid, which waits in `receive`; the callback
 * runs on a delivery thread (several run at once, each for different publishes) and must
 * not block.  Callbacks of different publishes may run in any order; a publisher with one
 * publish in flight (emqx_broker:publish/1 is synchronous) sees its results in order.
 */
#ifndef EMQX_TM_BATCHER_H
#define EMQX_TM_BATCHER_H

#include <stddef.h>
#include <stdint.h>

#include "emqx_tm.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct tm_batcher tm_batcher;

typedef struct tm_batcher_config {
    uint32_t max_batch;    /* publishes per engine batch (0 = 65536)              */
    uint32_t max_wait_us;  /* window bound from the oldest queued publish (0 = 200) */
    uint32_t mode;         /* TM_MATCH_ALL / UNIQUE / AGGRE / FIRST / COUNT        */
    uint32_t delivery_threads; /* threads calling publishers back (0 = 4); they take
                                  ranges of a window from one queue, so a thread that is
                                  slow (or descheduled) never holds the others */
    uint32_t transport;    /* TM_TRANSPORT_AUTO (runs for TM_MATCH_ALL on a master engine, ids
                              otherwise), TM_TRANSPORT_IDS, TM_TRANSPORT_RUNS (TM_ESTATE on a
                              replica) */
} tm_batcher_config;
#define TM_TRANSPORT_AUTO 0u
#define TM_TRANSPORT_IDS  1u
#define TM_TRANSPORT_RUNS 2u

/* One publish's result; `ids` is valid only during the call. */
typedef void (*tm_match_cb)(void *ctx, int32_t status, const uint64_t *ids, uint32_t n);
/* The same as spans (ids = the concatenation of spans[0 .. nspans), nids in all), valid only
 * during the call: a NIF builds its reply list straight from the engine's id arena. */
typedef void (*tm_spans_cb)(void *ctx, int32_t status, const tm_span *spans, uint32_t nspans, uint64_t nids);
/* (ABI 9) The same with u32 ids, for a consumer that builds small integers: spans of the
 * engine's u32 id arena when the aggregator runs its windows on it (EMQX_TM_RUNS_IDW=4), else
 * the reply narrowed into one span.  A reply with an id past 32 bits gets status TM_ESTATE
 * and no spans. */
typedef struct tm_span32 {
    const uint32_t *ids;
    uint64_t        n;
} tm_span32;
typedef void (*tm_spans32_cb)(void *ctx, int32_t status, const tm_span32 *spans, uint32_t nspans, uint64_t nids);

/* A batch matcher other than an engine (e.g. a filter-sharded index): match topics
 * bytes[off[i] .. off[i+1]) for i < n and fill `out` with memory the backend owns until
 * its next call.  Topic i's ids are ids[out->off[i] .. out->off[i] + out->cnt[i]).
 * Calls are never concurrent. */
typedef struct tm_batch_view {
    const uint32_t *off;
    const uint32_t *cnt;
    const uint64_t *ids;     /* NULL in COUNT mode */
    const int32_t  *status;
} tm_batch_view;
typedef int (*tm_batch_fn)(void *backend, const uint8_t *bytes, const uint32_t *off, uint32_t n,
                           uint32_t mode, tm_batch_view *out);

typedef struct tm_batcher_stats {
    uint64_t batches;
    uint64_t publishes;
    uint64_t max_batch_seen;
    uint64_t backend_us;        /* wall time inside the engine / backend, summed  */
    /* submit -> callback latency of EVERY publish delivered since the batcher started or the
     * last tm_batcher_stats_reset (a whole-run histogram, <= 1.6 % bucket error), microseconds */
    double   lat_p50_us, lat_p99_us, lat_max_us;
    /* per pipeline stage, microseconds summed over windows: cutting a window from the queue,
     * queueing its GPU part, waiting for the GPU part; then, averaged over the delivery
     * threads: waiting for ids still on PCIe, calling back */
    uint64_t cut_us, enqueue_us, gpu_wait_us, copy_us, deliver_us;
    /* (ABI 9) the same window: mean latency, publishes delivered (the percentiles' sample),
     * p99.9, and the window's length in seconds (steady clock) */
    double   lat_mean_us;
    uint64_t lat_count;
    double   lat_p999_us;
    double   window_s;
} tm_batcher_stats;

/* Over an engine: batches go through tm_match_device_mode on the engine's device and the
 * ids come back topic-major (tm_result_ids_device); UNIQUE over filters deeper than the
 * device order code goes through tm_match_batch.  The engine must outlive the batcher and
 * receive its writes through tm_batcher_apply / tm_batcher_commit while the batcher runs. */
int  tm_batcher_create(tm_engine *eng, const tm_batcher_config *cfg, tm_batcher **out);
int  tm_batcher_create_fn(tm_batch_fn fn, void *backend, const tm_batcher_config *cfg, tm_batcher **out);
/* Drains the queue (every submitted publish gets its callback), then stops the threads. */
void tm_batcher_destroy(tm_batcher *b);

/* Queue one publish (topic bytes are copied).  TM_ESTATE once destroy has begun. */
int tm_batcher_submit(tm_batcher *b, const uint8_t *topic, uint32_t len, tm_match_cb cb, void *ctx);
/* tm_batcher_submit with a span callback (no copy of the ids on the host at all). */
int tm_batcher_submit_spans(tm_batcher *b, const uint8_t *topic, uint32_t len, tm_spans_cb cb, void *ctx);
/* tm_batcher_submit with a u32-span callback (ABI 9; see tm_spans32_cb). */
int tm_batcher_submit_spans32(tm_batcher *b, const uint8_t *topic, uint32_t len, tm_spans32_cb cb, void *ctx);
/* Blocking form: waits for the publish's batch.  Copies up to `cap` ids, *n_out = the
 * full count (> cap means truncated), *status = the publish's status. */
int tm_batcher_match(tm_batcher *b, const uint8_t *topic, uint32_t len, uint64_t *ids, uint32_t cap,
                     uint32_t *n_out, int32_t *status);

/* Engine writes, serialised with the windows (engine batchers only: TM_ESTATE otherwise). */
int tm_batcher_apply(tm_batcher *b, const tm_op *ops, size_t n);
int tm_batcher_commit(tm_batcher *b, uint64_t *epoch_out);

int tm_batcher_stats_get(tm_batcher *b, tm_batcher_stats *out);
/* Starts a new latency window: the percentiles, mean and count cover publishes delivered from
 * here on (a load generator resets after its warm-up and reads the stats before its drain).
 * Stage times and batch counts are not reset. */
int tm_batcher_stats_reset(tm_batcher *b);

/* (ABI 10) Per-window stage stamps: where a window's time went, to attribute the latency tail to
 * a stage.  Nanoseconds on the aggregator's clock (the TSC scaled to ns).  The aggregator keeps
 * the last TM_BATCHER_WINDOWS windows completed since tm_batcher_stats_reset. */
#define TM_BATCHER_WINDOWS 16384
#define TM_WIN_RERUN 1u    /* the window's output was too small: grown and walked again */
#define TM_WIN_RUNS  2u    /* runs transport (spans of the host id arena) */
#define TM_WIN_FAILED 4u   /* the window failed as a whole (every publish got the status) */
typedef struct tm_batcher_window {
    uint32_t n;            /* publishes */
    uint32_t flags;        /* TM_WIN_* */
    uint64_t t_oldest;     /* submit stamp of the window's oldest publish */
    uint64_t t_cut;        /* the cutter starts taking the window from the queue */
    uint64_t t_queued;     /* its GPU part queued (bytes H2D, walk, result copies on the stream) */
    uint64_t t_gpu;        /* the GPU part observed done (including any re-run) */
    uint64_t t_ready;      /* results copied / D2H queued: handed to the delivery threads */
    uint64_t t_deliver;    /* the first delivery thread starts on it */
    uint64_t t_done;       /* its last callback returned */
    uint64_t epoch;        /* engine epoch when the window was queued (commits between windows) */
    /* CPU accounting (CPU time: CLOCK_THREAD_CPUTIME_ID; context switches: getrusage
     * RUSAGE_THREAD), to tell a stage that worked from one whose thread was off its CPU: */
    uint64_t t_slot;       /* the cutter starts waiting for a free slot (<= t_cut; the rest of
                              t_oldest..t_cut is the window filling / max_wait polling) */
    uint32_t cut_cpu_us;   /* the cutter's CPU time over t_cut..t_queued */
    uint16_t cut_ivcsw;    /* its involuntary context switches over t_cut..t_queued */
    uint16_t wait_ivcsw;   /* ... since it queued the previous window (over this one's wait) */
    uint32_t del_cpu_us;   /* the delivery threads' CPU time on this window's ranges, summed */
    uint32_t del_wall_us;  /* their wall time on those ranges, summed */
    uint32_t del_ivcsw;    /* their involuntary context switches inside those ranges */
    uint32_t reserved;
} tm_batcher_window;
/* Copies up to `cap` of the kept windows, oldest first; *n_out = how many. */
int tm_batcher_windows(tm_batcher *b, tm_batcher_window *out, uint32_t cap, uint32_t *n_out);

#ifdef __cplusplus
}
#endif

#endif /* EMQX_TM_BATCHER_H */
