// loadgen.cpp — closed-loop publisher load for the batching aggregator (bench tooling, not
// product code).  `publishers` concurrent publishers each keep exactly one publish in
// flight, like broker processes that call emqx_broker:publish/1 back to back
// (apps/emqx/src/emqx_broker.erl:285-290): a publisher's next topic is submitted from the
// callback that delivers its previous result.  Runs until `seconds` have passed, then waits
// for the publishes in flight.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <vector>

#include "../include/emqx_tm_batcher.h"

namespace {

struct Load;
// One publisher: one publish in flight, its own counters (its callbacks never run
// concurrently), so the load generator adds no shared write per publish.
struct alignas(64) Pub {
    Load *L;
    uint64_t k;  // next topic index
    uint64_t done, ids, errors;
};

struct Load {
    tm_batcher *b;
    const uint8_t *bytes;
    const uint32_t *off;
    uint32_t n_topics;
    std::chrono::steady_clock::time_point deadline;
    std::atomic<uint32_t> live{0};
    std::mutex m;
    std::condition_variable cv;
};

void on_result(void *ctx, int32_t status, const uint64_t *, uint32_t n);

bool submit_next(Pub *p) {
    Load *L = p->L;
    const uint64_t k = p->k++ % L->n_topics;
    return tm_batcher_submit(L->b, L->bytes + L->off[k], L->off[k + 1] - L->off[k], on_result, p) == TM_OK;
}

void retire(Load *L) {  // under the lock: the waiter may destroy L as soon as it sees 0
    std::lock_guard<std::mutex> g(L->m);
    if (--L->live == 0) L->cv.notify_all();
}

void on_result(void *ctx, int32_t status, const uint64_t *, uint32_t n) {
    Pub *p = static_cast<Pub *>(ctx);
    p->done++;
    p->ids += n;
    if (status < 0) p->errors++;
    // the deadline is looked at every 8th publish of a publisher (a clock read is not free)
    if (((p->done & 7) == 0 && std::chrono::steady_clock::now() >= p->L->deadline) || !submit_next(p)) retire(p->L);
}

}  // namespace

extern "C" int loadgen_run(tm_batcher *b, const uint8_t *bytes, const uint32_t *off, uint32_t n_topics,
                           uint32_t publishers, double seconds, uint64_t *published, uint64_t *ids_out,
                           uint64_t *errors, double *elapsed_s) {
    if (!b || !bytes || !off || !n_topics || !publishers) return TM_EINVAL;
    Load L;
    L.b = b;
    L.bytes = bytes;
    L.off = off;
    L.n_topics = n_topics;
    std::vector<Pub> pubs(publishers);
    const auto t0 = std::chrono::steady_clock::now();
    L.deadline = t0 + std::chrono::duration_cast<std::chrono::steady_clock::duration>(
                          std::chrono::duration<double>(seconds));
    L.live = publishers;
    for (uint32_t p = 0; p < publishers; p++) {
        pubs[p] = Pub{&L, (uint64_t)p * 7919u, 0, 0, 0};
        if (!submit_next(&pubs[p])) retire(&L);
    }
    {
        std::unique_lock<std::mutex> lk(L.m);
        L.cv.wait(lk, [&] { return L.live.load() == 0; });
    }
    *elapsed_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    uint64_t d = 0, i = 0, e = 0;
    for (const Pub &p : pubs) {
        d += p.done;
        i += p.ids;
        e += p.errors;
    }
    *published = d;
    *ids_out = i;
    *errors = e;
    return TM_OK;
}
