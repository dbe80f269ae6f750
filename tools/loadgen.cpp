// loadgen.cpp — closed-loop publisher load for the batching aggregator (bench tooling, not
// product code).  `publishers` concurrent publishers each keep exactly one publish in
// flight, like broker processes that call emqx_broker:publish/1 back to back
// (apps/emqx/src/emqx_broker.erl:285-290): a publisher's next topic is submitted from the
// callback that delivers its previous result.  Runs until `seconds` have passed, then waits
// for the publishes in flight.  Every callback reads each id it is given once (a checksum),
// as a NIF building its reply list would; with `spans` it takes the span callback
// (tm_batcher_submit_spans) and reads the ids straight from the engine's id arena.
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <vector>

#include "../include/emqx_tm_batcher.h"

namespace {

struct Load;
// One publisher: one publish in flight, its own counters (its callbacks never run
// concurrently), so the load generator adds no shared write per publish.
struct alignas(64) Pub {
    Load *L;
    uint64_t k;  // next topic index
    uint64_t done, ids, errors, sum;
};

struct Load {
    tm_batcher *b;
    const uint8_t *bytes;
    const uint32_t *off;
    uint32_t n_topics;
    std::atomic<int64_t> deadline{INT64_MAX};  // steady_clock ticks; the main thread may move it
    std::atomic<uint32_t> live{0};
    std::mutex m;
    std::condition_variable cv;
    bool spans = false;
};

void on_result(void *ctx, int32_t status, const uint64_t *ids, uint32_t n);
void on_spans(void *ctx, int32_t status, const tm_span *sp, uint32_t ns, uint64_t nids);

bool submit_next(Pub *p) {
    Load *L = p->L;
    const uint64_t k = p->k++ % L->n_topics;
    if (L->spans)
        return tm_batcher_submit_spans(L->b, L->bytes + L->off[k], L->off[k + 1] - L->off[k], on_spans, p) == TM_OK;
    return tm_batcher_submit(L->b, L->bytes + L->off[k], L->off[k + 1] - L->off[k], on_result, p) == TM_OK;
}

void retire(Load *L) {  // under the lock: the waiter may destroy L as soon as it sees 0
    std::lock_guard<std::mutex> g(L->m);
    if (--L->live == 0) L->cv.notify_all();
}

void next_or_retire(Pub *p);

void on_result(void *ctx, int32_t status, const uint64_t *ids, uint32_t n) {
    Pub *p = static_cast<Pub *>(ctx);
    p->done++;
    p->ids += n;
    uint64_t s = 0;
    for (uint32_t i = 0; i < n; i++) s += ids[i];
    p->sum += s;
    if (status < 0) p->errors++;
    next_or_retire(p);
}

void on_spans(void *ctx, int32_t status, const tm_span *sp, uint32_t ns, uint64_t nids) {
    Pub *p = static_cast<Pub *>(ctx);
    p->done++;
    p->ids += nids;
    uint64_t s = 0;
    for (uint32_t j = 0; j < ns; j++)
        for (uint64_t i = 0; i < sp[j].n; i++) s += sp[j].ids[i];
    p->sum += s;
    if (status < 0) p->errors++;
    next_or_retire(p);
}

void next_or_retire(Pub *p) {
    // the deadline is looked at every 8th publish of a publisher (a clock read is not free)
    if (((p->done & 7) == 0 &&
         std::chrono::steady_clock::now().time_since_epoch().count() >= p->L->deadline.load(std::memory_order_relaxed)) ||
        !submit_next(p))
        retire(p->L);
}

}  // namespace

// Closed loop for warmup_s + seconds.  With `window` non-null: after warmup_s the batcher's
// latency window is reset (tm_batcher_stats_reset), and at the end of the measured `seconds`,
// BEFORE the publishers stop and the queue drains, its stats are read into *window: the
// latency of every publish delivered in the steady state, and how many there were.
extern "C" int loadgen_run3(tm_batcher *b, const uint8_t *bytes, const uint32_t *off, uint32_t n_topics,
                            uint32_t publishers, double warmup_s, double seconds, int spans, uint64_t *published,
                            uint64_t *ids_out, uint64_t *errors, uint64_t *checksum, double *elapsed_s,
                            tm_batcher_stats *window) {
    if (!b || !bytes || !off || !n_topics || !publishers) return TM_EINVAL;
    Load L;
    L.spans = spans != 0;
    L.b = b;
    L.bytes = bytes;
    L.off = off;
    L.n_topics = n_topics;
    std::vector<Pub> pubs(publishers);
    using clk = std::chrono::steady_clock;
    const auto t0 = clk::now();
    const auto dur = [](double s) { return std::chrono::duration_cast<clk::duration>(std::chrono::duration<double>(s)); };
    if (!window) L.deadline = (t0 + dur(warmup_s + seconds)).time_since_epoch().count();
    L.live = publishers;
    for (uint32_t p = 0; p < publishers; p++) {
        pubs[p] = Pub{&L, (uint64_t)p * 7919u, 0, 0, 0, 0};
        if (!submit_next(&pubs[p])) retire(&L);
    }
    if (window) {
        std::this_thread::sleep_until(t0 + dur(warmup_s));
        int rc = tm_batcher_stats_reset(b);
        std::this_thread::sleep_until(t0 + dur(warmup_s + seconds));
        if (!rc) rc = tm_batcher_stats_get(b, window);
        L.deadline = clk::now().time_since_epoch().count();  // now the publishers stop
        if (rc) window->lat_count = 0;
    }
    {
        std::unique_lock<std::mutex> lk(L.m);
        L.cv.wait(lk, [&] { return L.live.load() == 0; });
    }
    *elapsed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t d = 0, i = 0, e = 0, cs = 0;
    for (const Pub &p : pubs) {
        d += p.done;
        i += p.ids;
        e += p.errors;
        cs += p.sum;
    }
    *published = d;
    *ids_out = i;
    *errors = e;
    if (checksum) *checksum = cs;
    return TM_OK;
}

extern "C" int loadgen_run2(tm_batcher *b, const uint8_t *bytes, const uint32_t *off, uint32_t n_topics,
                            uint32_t publishers, double seconds, int spans, uint64_t *published, uint64_t *ids_out,
                            uint64_t *errors, uint64_t *checksum, double *elapsed_s) {
    return loadgen_run3(b, bytes, off, n_topics, publishers, 0.0, seconds, spans, published, ids_out, errors, checksum,
                        elapsed_s, nullptr);
}

extern "C" int loadgen_run(tm_batcher *b, const uint8_t *bytes, const uint32_t *off, uint32_t n_topics,
                           uint32_t publishers, double seconds, uint64_t *published, uint64_t *ids_out,
                           uint64_t *errors, double *elapsed_s) {
    return loadgen_run2(b, bytes, off, n_topics, publishers, seconds, 0, published, ids_out, errors, nullptr,
                        elapsed_s);
}

// Read every id a tm_match_batch_runs result covers (a checksum), on `threads` threads by
// topic range: what a consumer building replies from the spans does at least once per id.
extern "C" uint64_t spans_checksum(const tm_runs_result *r, uint32_t threads) {
    if (!r || !r->n) return 0;
    threads = threads ? threads : 1;
    std::vector<uint64_t> part(threads, 0);
    std::vector<std::thread> th;
    for (uint32_t t = 0; t < threads; t++)
        th.emplace_back([&, t] {
            const uint32_t lo = (uint32_t)((uint64_t)r->n * t / threads), hi = (uint32_t)((uint64_t)r->n * (t + 1) / threads);
            uint64_t s = 0;
            for (uint32_t i = lo; i < hi; i++)
                for (uint32_t j = r->span_off[i], e = r->span_off[i] + r->span_cnt[i]; j < e; j++)
                    for (uint64_t k = 0; k < r->spans[j].n; k++) s += r->spans[j].ids[k];
            part[t] = s;
        });
    uint64_t s = 0;
    for (uint32_t t = 0; t < threads; t++) {
        th[t].join();
        s += part[t];
    }
    return s;
}
