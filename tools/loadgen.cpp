// loadgen.cpp — closed-loop publisher load for the batching aggregator (bench tooling, not
// product code).  `publishers` concurrent publishers each keep exactly one publish in
// flight, like broker processes that call emqx_broker:publish/1 back to back
// (apps/emqx/src/emqx_broker.erl:285-290): a publisher's next topic is submitted from the
// callback that delivers its previous result.  Runs until `seconds` have passed, then waits
// for the publishes in flight.  Every callback reads each id it is given once (a checksum),
// as a NIF building its reply list would; with `spans` 1 it takes the span callback
// (tm_batcher_submit_spans), 3 the u32-span one (tm_batcher_submit_spans32), and reads the ids
// straight from the engine's id arena.
#include <cstring>
#include <cstdio>
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
    bool spans32 = false;  // spans == 3 (u32-span callback, tm_batcher_submit_spans32)
    bool no_read = false;  // spans == 2 / 4 (development): span / u32-span callbacks reading no id
};

void on_result(void *ctx, int32_t status, const uint64_t *ids, uint32_t n);
void on_spans(void *ctx, int32_t status, const tm_span *sp, uint32_t ns, uint64_t nids);
void on_spans32(void *ctx, int32_t status, const tm_span32 *sp, uint32_t ns, uint64_t nids);

bool submit_next(Pub *p) {
    Load *L = p->L;
    const uint64_t k = p->k++ % L->n_topics;
    if (L->spans32)
        return tm_batcher_submit_spans32(L->b, L->bytes + L->off[k], L->off[k + 1] - L->off[k], on_spans32, p) == TM_OK;
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
    if (!p->L->no_read)
        for (uint32_t j = 0; j < ns; j++)
            for (uint64_t i = 0; i < sp[j].n; i++) s += sp[j].ids[i];
    p->sum += s;
    if (status < 0) p->errors++;
    next_or_retire(p);
}

void on_spans32(void *ctx, int32_t status, const tm_span32 *sp, uint32_t ns, uint64_t nids) {
    Pub *p = static_cast<Pub *>(ctx);
    p->done++;
    p->ids += nids;
    uint64_t s = 0;
    if (!p->L->no_read)
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
// The cgroup's CPU accounting (cgroup v2 cpu.stat): usage, and how often / how long the CPU
// quota throttled this job -- a throttled period stops every thread of the process at once.
// out4: usage_usec, nr_periods, nr_throttled, throttled_usec (all 0 when there is no such file).
static void cpu_stat(uint64_t *out4) {
    out4[0] = out4[1] = out4[2] = out4[3] = 0;
    FILE *f = std::fopen("/sys/fs/cgroup/cpu.stat", "r");
    if (!f) return;
    char k[64];
    unsigned long long v;
    while (std::fscanf(f, "%63s %llu", k, &v) == 2) {
        if (!std::strcmp(k, "usage_usec")) out4[0] = v;
        else if (!std::strcmp(k, "nr_periods")) out4[1] = v;
        else if (!std::strcmp(k, "nr_throttled")) out4[2] = v;
        else if (!std::strcmp(k, "throttled_usec")) out4[3] = v;
    }
    std::fclose(f);
}

// loadgen_run3 + what the measured window saw besides latency: the aggregator's per-window stage
// stamps of the windows completed in it (tm_batcher_windows, read with the stats, before the
// drain) and the cgroup CPU accounting over it (cpu_stat deltas).
extern "C" int loadgen_run4(tm_batcher *b, const uint8_t *bytes, const uint32_t *off, uint32_t n_topics,
                            uint32_t publishers, double warmup_s, double seconds, int spans, uint64_t *published,
                            uint64_t *ids_out, uint64_t *errors, uint64_t *checksum, double *elapsed_s,
                            tm_batcher_stats *window, tm_batcher_window *wins, uint32_t wcap, uint32_t *wn,
                            uint64_t *cg4);

extern "C" int loadgen_run3(tm_batcher *b, const uint8_t *bytes, const uint32_t *off, uint32_t n_topics,
                            uint32_t publishers, double warmup_s, double seconds, int spans, uint64_t *published,
                            uint64_t *ids_out, uint64_t *errors, uint64_t *checksum, double *elapsed_s,
                            tm_batcher_stats *window) {
    return loadgen_run4(b, bytes, off, n_topics, publishers, warmup_s, seconds, spans, published, ids_out, errors,
                        checksum, elapsed_s, window, nullptr, 0, nullptr, nullptr);
}

extern "C" int loadgen_run4(tm_batcher *b, const uint8_t *bytes, const uint32_t *off, uint32_t n_topics,
                            uint32_t publishers, double warmup_s, double seconds, int spans, uint64_t *published,
                            uint64_t *ids_out, uint64_t *errors, uint64_t *checksum, double *elapsed_s,
                            tm_batcher_stats *window, tm_batcher_window *wins, uint32_t wcap, uint32_t *wn,
                            uint64_t *cg4) {
    if (!b || !bytes || !off || !n_topics || !publishers) return TM_EINVAL;
    Load L;
    L.spans = spans != 0;
    L.spans32 = spans == 3 || spans == 4;
    L.no_read = spans == 2 || spans == 4;
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
        uint64_t c0[4], c1[4];
        cpu_stat(c0);
        int rc = tm_batcher_stats_reset(b);
        std::this_thread::sleep_until(t0 + dur(warmup_s + seconds));
        if (!rc) rc = tm_batcher_stats_get(b, window);
        cpu_stat(c1);
        if (!rc && wins && wn) rc = tm_batcher_windows(b, wins, wcap, wn);
        L.deadline = clk::now().time_since_epoch().count();  // now the publishers stop
        if (rc) window->lat_count = 0;
        if (cg4)
            for (int k = 0; k < 4; k++) cg4[k] = c1[k] - c0[k];
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

// Host-form callers on `threads` native threads at once (tests/test_gpu_concurrency.py): thread k
// makes `reps` calls on its own batch (bytes[k], offs[k], ns[k] topics) per round, `rounds`
// rounds between barriers (the first ones warm each thread's engine lane, as a NIF's dirty
// schedulers keep theirs); *wall_s_out = the LAST round's wall time; then one untimed call per
// thread whose result is digested.  form 0: tm_match_batch_runs,
// 1: tm_match_batch (keys) + tm_key_ids.  digest_out[k]: over thread k's last result,
// sum over topics t of sum over its ids of mix(id + t * golden), and every status folded in:
// order-independent within a topic, tied to the topic.
#include <cstring>
namespace {
struct Gate {
    std::mutex m;
    std::condition_variable cv;
    uint32_t n, waiting = 0;
    uint64_t gen = 0;
    explicit Gate(uint32_t n_) : n(n_) {}
    void wait() {
        std::unique_lock<std::mutex> lk(m);
        const uint64_t g = gen;
        if (++waiting == n) {
            waiting = 0;
            gen++;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g; });
        }
    }
};
inline uint64_t mix64(uint64_t x) {
    x ^= x >> 30;
    x *= 0xBF58476D1CE4E5B9ull;
    x ^= x >> 27;
    x *= 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
}  // namespace

extern "C" int conc_calls2(tm_engine *eng, int form, const uint8_t *const *bytes, const uint32_t *const *offs,
                           const uint32_t *ns, uint32_t threads, uint32_t reps, uint32_t rounds, double *wall_s_out,
                           uint64_t *digest_out, double *call_s_out);
extern "C" int conc_calls(tm_engine *eng, int form, const uint8_t *const *bytes, const uint32_t *const *offs,
                          const uint32_t *ns, uint32_t threads, uint32_t reps, uint32_t rounds, double *wall_s_out,
                          uint64_t *digest_out) {
    return conc_calls2(eng, form, bytes, offs, ns, threads, reps, rounds, wall_s_out, digest_out, nullptr);
}
// call_s_out (optional): threads x reps, each call's duration in the last round
extern "C" int conc_calls2(tm_engine *eng, int form, const uint8_t *const *bytes, const uint32_t *const *offs,
                           const uint32_t *ns, uint32_t threads, uint32_t reps, uint32_t rounds, double *wall_s_out,
                           uint64_t *digest_out, double *call_s_out) {
    if (!eng || !threads || !reps || !rounds) return TM_EINVAL;
    Gate start(threads + 1), done(threads + 1);
    std::vector<int> rcs(threads, TM_OK);
    std::vector<std::thread> th;
    for (uint32_t k = 0; k < threads; k++)
        th.emplace_back([&, k] {
            std::vector<uint64_t> ids;
            // the timed rounds make plain calls; one more, untimed, computes the digests
            for (uint32_t r = 0; r <= rounds; r++) {
                start.wait();
                const uint32_t nrep = r == rounds ? 1 : reps;
                for (uint32_t q = 0; q < nrep && rcs[k] == TM_OK; q++) {
                    const bool last = r == rounds;
                    uint64_t dg = 0;
                    const auto c0 = std::chrono::steady_clock::now();
                    if (form == 0) {
                        tm_runs_result res;
                        rcs[k] = tm_match_batch_runs(eng, bytes[k], offs[k], ns[k], &res);
                        if (rcs[k] == TM_OK && last)
                            for (uint32_t t = 0; t < res.n; t++) {
                                dg += mix64((uint64_t)(uint32_t)res.status[t] + 0x51ull * t);
                                for (uint32_t j = res.span_off[t]; j < res.span_off[t] + res.span_cnt[t]; j++)
                                    for (uint64_t i = 0; i < res.spans[j].n; i++)
                                        dg += mix64(res.spans[j].ids[i] + 0x9E3779B97F4A7C15ull * t);
                            }
                    } else {
                        tm_result res;
                        rcs[k] = tm_match_batch(eng, bytes[k], offs[k], ns[k], TM_MATCH_ALL, &res);
                        if (rcs[k] == TM_OK && last) {
                            ids.resize(res.total + 1);
                            if (res.total) rcs[k] = tm_key_ids(eng, res.keys, res.total, ids.data());
                            for (uint32_t t = 0; t < res.n && rcs[k] == TM_OK; t++) {
                                dg += mix64((uint64_t)(uint32_t)res.status[t] + 0x51ull * t);
                                for (uint32_t i = 0; i < res.cnt[t]; i++)
                                    dg += mix64(ids[res.off[t] + i] + 0x9E3779B97F4A7C15ull * t);
                            }
                        }
                    }
                    if (last) digest_out[k] = dg;
                    if (call_s_out && r + 1 == rounds)  // the last timed round
                        call_s_out[(size_t)k * reps + q] =
                            std::chrono::duration<double>(std::chrono::steady_clock::now() - c0).count();
                }
                if (form == 0) tm_runs_release(eng);
                done.wait();
            }
            tm_result_release(eng);  // this thread's lane
        });
    double wall = 0;
    for (uint32_t r = 0; r <= rounds; r++) {
        start.wait();
        const auto t0 = std::chrono::steady_clock::now();
        done.wait();
        if (r < rounds) wall = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    for (auto &t : th) t.join();
    *wall_s_out = wall;
    for (int rc : rcs)
        if (rc != TM_OK) return rc;
    return TM_OK;
}

// A backend with no matching at all (development: the aggregator's own per-publish cost on a
// CPU-only host).  Every publish of a window gets the same `fake_ids` ids (one shared list,
// like a hot '#' list every topic matches).
namespace {
struct FakeBackend {
    std::vector<uint32_t> off, cnt;
    std::vector<int32_t> status;
    std::vector<uint64_t> ids;
};
}  // namespace

extern "C" void *fake_backend_new(uint32_t ids_per_publish) {
    FakeBackend *f = new FakeBackend();
    f->ids.resize(ids_per_publish ? ids_per_publish : 1);
    for (size_t i = 0; i < f->ids.size(); i++) f->ids[i] = i * 7 + 1;
    return f;
}
extern "C" void fake_backend_free(void *p) { delete static_cast<FakeBackend *>(p); }
extern "C" int fake_backend_fn(void *p, const uint8_t *, const uint32_t *, uint32_t n, uint32_t, tm_batch_view *out) {
    FakeBackend *f = static_cast<FakeBackend *>(p);
    if (f->off.size() < n + 1) {
        f->off.assign(n + 1, 0);
        f->cnt.assign(n, (uint32_t)f->ids.size());
        f->status.assign(n, TM_TOPIC_OK);
    }
    *out = tm_batch_view{f->off.data(), f->cnt.data(), f->ids.data(), f->status.data()};
    return TM_OK;
}
