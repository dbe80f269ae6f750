// batcher.cpp — the publish batching aggregator (include/emqx_tm_batcher.h).
//
// Reference behaviour it stands in for: emqx_broker:do_publish/1 calls
// emqx_router:match_routes/1 once per publish, synchronously, in the publisher's own process
// (apps/emqx/src/emqx_broker.erl:285-290, apps/emqx/src/emqx_router.erl:205-212).  Here many
// publishers queue single topics; one worker thread cuts the queue into windows
// (max_batch publishes or max_wait_us since the oldest, whichever comes first), runs ONE
// engine batch per window and calls every publisher back with its own id list.  While it
// runs a window, the next one fills.
//
// The engine backend keeps the whole batch on the GPU until the ids are final:
// tm_match_device_mode (walk + optional reducer) -> tm_result_ids_device (key handles ->
// route ids, topic-major) -> one D2H of offsets, ids and statuses.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/emqx_tm.h"
#include "../../include/emqx_tm_batcher.h"

extern "C" int tmx_engine_device(const tm_engine *eng);  // engine.cpp, library-internal

namespace {

uint64_t now_ns() {
    return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

// grow-only device / pinned buffers
struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = std::max<size_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipMalloc(&p, c);
        if (e == hipSuccess) cap = c;
        return e;
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
};
struct HBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
        size_t c = std::max<size_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipHostMalloc(&p, c, hipHostMallocDefault);
        if (e == hipSuccess) cap = c;
        return e;
    }
    template <class T>
    T *as() const {
        return (T *)p;
    }
    ~HBuf() {
        if (p) (void)hipHostFree(p);
    }
};

#define BT_HIP(E)                              \
    do {                                       \
        if ((E) != hipSuccess) return TM_EDEVICE; \
    } while (0)

// tm_batch_fn over an engine.  Everything is queued on the backend's own stream and
// the batch waits on it twice: once for the offsets / statuses / demand, once for the ids.
// Host result buffers alternate between two slots, so a view stays valid until the
// second-next call.
struct EngineBackend {
    tm_engine *eng;
    int device;
    hipStream_t stream = nullptr;
    DBuf d_bytes, d_off, d_ids, d_off_out;
    HBuf h_bytes, h_off, h_total;
    struct Slot {
        HBuf h_off_out, h_ids, h_status, h_cnt;
        std::vector<uint32_t> cnt;
        std::vector<uint64_t> ids;  // host path only
    } slot[2];
    uint32_t turn = 0;

    ~EngineBackend() {
        if (stream) (void)hipStreamDestroy(stream);
    }

    int run(const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode, tm_batch_view *v) {
        Slot &S = slot[turn++ & 1];
        BT_HIP(hipSetDevice(device));
        if (!stream) BT_HIP(hipStreamCreateWithFlags(&stream, hipStreamNonBlocking));
        const uint64_t nbytes = (uint64_t)off[n] - off[0];
        S.cnt.resize(n);
        BT_HIP(S.h_status.ensure((size_t)n * 4 + 4));
        BT_HIP(S.h_off_out.ensure((size_t)n * 4 + 4));
        BT_HIP(S.h_cnt.ensure((size_t)n * 4 + 4));
        BT_HIP(h_total.ensure(8));
        BT_HIP(h_bytes.ensure(nbytes + 16));
        BT_HIP(h_off.ensure((size_t)n * 4 + 4));
        std::memcpy(h_bytes.p, bytes + off[0], nbytes);
        for (uint32_t i = 0; i <= n; i++) h_off.as<uint32_t>()[i] = off[i] - off[0];
        BT_HIP(d_bytes.ensure(nbytes + 16));
        BT_HIP(d_off.ensure((size_t)n * 4 + 4));
        BT_HIP(d_off_out.ensure((size_t)n * 4 + 4));
        BT_HIP(hipMemcpyAsync(d_bytes.p, h_bytes.p, nbytes + 1, hipMemcpyHostToDevice, stream));
        BT_HIP(hipMemcpyAsync(d_off.p, h_off.p, (size_t)n * 4 + 4, hipMemcpyHostToDevice, stream));
        const bool ids_mode = mode != TM_MATCH_COUNT;
        uint32_t *oo = S.h_off_out.as<uint32_t>();
        tm_dev_result r;
        int rc = 0;
        for (int attempt = 0;; attempt++) {
            rc = tm_match_device_mode(eng, (const uint8_t *)d_bytes.p, (const uint32_t *)d_off.p, n, nbytes, mode,
                                      stream, &r);
            if (rc == TM_ESTATE && mode == TM_MATCH_UNIQUE) return run_host(S, bytes, off, n, mode, v);
            if (rc) return rc;
            *h_total.as<uint64_t>() = 0;
            if (ids_mode) {
                // key handles -> ids, compacted topic-major; a batch past keys_cap is re-run
                const uint64_t cap = mode == TM_MATCH_FIRST ? n : r.keys_cap;
                BT_HIP(d_ids.ensure(cap * 8 + 8));
                if ((rc = tm_result_ids_device(eng, (uint64_t *)d_ids.p, cap, (uint32_t *)d_off_out.p, stream)))
                    return rc;
                BT_HIP(hipMemcpyAsync(oo, d_off_out.p, (size_t)n * 4 + 4, hipMemcpyDeviceToHost, stream));
                if (mode != TM_MATCH_FIRST)
                    BT_HIP(hipMemcpyAsync(h_total.p, r.d_total, 8, hipMemcpyDeviceToHost, stream));
            } else {
                BT_HIP(hipMemcpyAsync(S.h_cnt.p, r.d_cnt, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
            }
            BT_HIP(hipMemcpyAsync(S.h_status.p, r.d_status, (size_t)n * 4, hipMemcpyDeviceToHost, stream));
            if ((rc = tm_device_sync(eng))) return rc;  // waits on `stream`; sizes the engine's pools
            const uint64_t total = *h_total.as<uint64_t>();
            if (total <= r.keys_cap) break;
            if (attempt || (rc = tm_reserve_matches(eng, total + total / 8 + 1024, 0))) return rc ? rc : TM_EDEVICE;
        }
        v->status = S.h_status.as<int32_t>();
        if (!ids_mode) {
            std::memset(oo, 0, (size_t)n * 4);
            v->off = oo;
            v->cnt = S.h_cnt.as<uint32_t>();
            v->ids = nullptr;
            return TM_OK;
        }
        const uint64_t got = oo[n];
        BT_HIP(S.h_ids.ensure(got * 8 + 8));
        if (got) {
            BT_HIP(hipMemcpyAsync(S.h_ids.p, d_ids.p, got * 8, hipMemcpyDeviceToHost, stream));
            BT_HIP(hipStreamSynchronize(stream));
        }
        for (uint32_t i = 0; i < n; i++) S.cnt[i] = oo[i + 1] - oo[i];
        v->off = oo;
        v->cnt = S.cnt.data();
        v->ids = S.h_ids.as<uint64_t>();
        return TM_OK;
    }

    // UNIQUE over keys deeper than the device order code: tm_match_batch reduces on the host
    int run_host(Slot &S, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode, tm_batch_view *v) {
        tm_result res;
        int rc = tm_match_batch(eng, bytes, off, n, mode, &res);
        if (rc) return rc;
        std::vector<uint64_t> &ids = S.ids;
        std::vector<uint32_t> &cnt = S.cnt;
        ids.resize(res.total);
        uint32_t *oo = S.h_off_out.as<uint32_t>();
        uint64_t pos = 0;
        for (uint32_t i = 0; i < n; i++) {
            oo[i] = (uint32_t)pos;
            cnt[i] = res.cnt[i];
            if (res.cnt[i] && (rc = tm_key_ids(eng, res.keys + res.off[i], res.cnt[i], ids.data() + pos))) return rc;
            pos += res.cnt[i];
        }
        oo[n] = (uint32_t)pos;
        std::memcpy(S.h_status.p, res.status, (size_t)n * 4);
        v->off = oo;
        v->cnt = cnt.data();
        v->ids = ids.data();
        v->status = S.h_status.as<int32_t>();
        return TM_OK;
    }
};

int engine_batch(void *be, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode, tm_batch_view *out) {
    return static_cast<EngineBackend *>(be)->run(bytes, off, n, mode, out);
}

struct Pending {
    uint32_t off, len;  // the topic's bytes in the queue's byte buffer
    tm_match_cb cb;
    void *ctx;
    uint64_t t0;  // submit time (ns)
};

constexpr size_t LAT_RING = 65536;
constexpr size_t QUEUE_BYTES_MAX = 1ull << 31;

}  // namespace

struct tm_batcher {
    tm_batch_fn fn = nullptr;
    void *backend = nullptr;
    EngineBackend *eb = nullptr;  // owned when the batcher runs over an engine
    tm_batcher_config cfg{};

    std::mutex mu;  // queue, stats
    std::condition_variable cv;
    std::vector<uint8_t> qbytes;
    std::vector<Pending> q;
    bool stopping = false;

    std::mutex eng_mu;  // backend calls vs tm_batcher_apply / tm_batcher_commit

    std::thread worker;

    uint64_t n_batches = 0, n_pub = 0, max_seen = 0, backend_ns = 0;
    std::vector<uint32_t> lat_ns;  // ring of submit -> callback latencies (ns, saturating)
    size_t lat_pos = 0, lat_n = 0;

    // One thread cuts windows, runs the backend and calls the publishers back.  (A
    // separate delivery thread overlapping batch k's callbacks with batch k+1 was measured
    // slower under closed-loop load: the population splits into two half-size windows and
    // the fixed per-batch cost doubles)
    void loop() {
        std::vector<uint8_t> bbytes;
        std::vector<Pending> batch;
        std::vector<uint32_t> offs, lats;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            cv.wait(lk, [&] { return stopping || !q.empty(); });
            if (q.empty()) break;  // stopping and drained
            const uint64_t deadline = q.front().t0 + (uint64_t)cfg.max_wait_us * 1000;
            while (!stopping && q.size() < cfg.max_batch && qbytes.size() < QUEUE_BYTES_MAX / 2) {
                const uint64_t t = now_ns();
                if (t >= deadline) break;
                cv.wait_for(lk, std::chrono::nanoseconds(deadline - t));
            }
            batch.clear();
            bbytes.clear();
            batch.swap(q);
            bbytes.swap(qbytes);
            if (batch.size() > cfg.max_batch) {  // the tail waits for the next window
                for (size_t i = cfg.max_batch; i < batch.size(); i++) {
                    Pending p = batch[i];
                    const uint8_t *src = bbytes.data() + p.off;
                    p.off = (uint32_t)qbytes.size();
                    qbytes.insert(qbytes.end(), src, src + p.len);
                    q.push_back(p);
                }
                batch.resize(cfg.max_batch);
            }
            lk.unlock();

            const uint32_t n = (uint32_t)batch.size();
            offs.resize((size_t)n + 1);
            for (uint32_t i = 0; i < n; i++) offs[i] = batch[i].off;  // contiguous, in queue order
            offs[n] = batch[n - 1].off + batch[n - 1].len;
            tm_batch_view v{};
            const uint64_t tb = now_ns();
            int rc;
            {
                std::lock_guard<std::mutex> g(eng_mu);
                rc = fn(backend, bbytes.data(), offs.data(), n, cfg.mode, &v);
            }
            const uint64_t te = now_ns();
            lk.lock();  // counted before the callbacks: a caller woken by one sees its batch
            n_batches++;
            n_pub += n;
            max_seen = std::max<uint64_t>(max_seen, n);
            backend_ns += te - tb;
            lk.unlock();
            lats.resize(n);
            for (uint32_t i = 0; i < n; i++) {
                const Pending &p = batch[i];
                if (rc < 0) {
                    p.cb(p.ctx, rc, nullptr, 0);
                } else {
                    const int32_t st = v.status[i];
                    const uint32_t c = st == TM_TOPIC_OK ? v.cnt[i] : 0;
                    p.cb(p.ctx, st, (v.ids && c) ? v.ids + v.off[i] : nullptr, c);
                }
                const uint64_t d = now_ns() - p.t0;
                lats[i] = d > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)d;
            }
            lk.lock();
            for (uint32_t i = 0; i < n; i++) {
                lat_ns[lat_pos] = lats[i];
                lat_pos = (lat_pos + 1) % LAT_RING;
            }
            lat_n = std::min(LAT_RING, lat_n + n);
        }
    }

    int start(const tm_batcher_config *c) {
        if (c) cfg = *c;
        if (cfg.max_batch == 0) cfg.max_batch = 65536;
        if (cfg.max_wait_us == 0) cfg.max_wait_us = 200;
        if (cfg.mode > TM_MATCH_AGGRE) return TM_EINVAL;
        lat_ns.assign(LAT_RING, 0);
        try {
            worker = std::thread([this] { loop(); });
        } catch (...) {
            return TM_ENOMEM;
        }
        return TM_OK;
    }

    void stop() {
        {
            std::lock_guard<std::mutex> g(mu);
            stopping = true;
        }
        cv.notify_all();
        if (worker.joinable()) worker.join();
    }
};

extern "C" {

int tm_batcher_create_fn(tm_batch_fn fn, void *backend, const tm_batcher_config *cfg, tm_batcher **out) {
    if (!fn || !out) return TM_EINVAL;
    *out = nullptr;
    tm_batcher *b = new (std::nothrow) tm_batcher();
    if (!b) return TM_ENOMEM;
    b->fn = fn;
    b->backend = backend;
    int rc = b->start(cfg);
    if (rc) {
        delete b;
        return rc;
    }
    *out = b;
    return TM_OK;
}

int tm_batcher_create(tm_engine *eng, const tm_batcher_config *cfg, tm_batcher **out) {
    if (!eng || !out) return TM_EINVAL;
    EngineBackend *eb = new (std::nothrow) EngineBackend();
    if (!eb) return TM_ENOMEM;
    eb->eng = eng;
    eb->device = tmx_engine_device(eng);
    int rc = tm_batcher_create_fn(engine_batch, eb, cfg, out);
    if (rc) {
        delete eb;
        return rc;
    }
    (*out)->eb = eb;
    return TM_OK;
}

void tm_batcher_destroy(tm_batcher *b) {
    if (!b) return;
    b->stop();  // drains: every queued publish is matched and called back first
    delete b->eb;
    delete b;
}

int tm_batcher_submit(tm_batcher *b, const uint8_t *topic, uint32_t len, tm_match_cb cb, void *ctx) {
    if (!b || !cb || (len && !topic) || len > 65535) return TM_EINVAL;
    const uint64_t t0 = now_ns();
    bool wake;
    {
        std::lock_guard<std::mutex> g(b->mu);
        if (b->stopping) return TM_ESTATE;
        if (b->qbytes.size() + len > QUEUE_BYTES_MAX) return TM_ENOMEM;  // back-pressure
        b->q.push_back(Pending{(uint32_t)b->qbytes.size(), len, cb, ctx, t0});
        b->qbytes.insert(b->qbytes.end(), topic, topic + len);
        wake = b->q.size() == 1 || b->q.size() >= b->cfg.max_batch;
    }
    if (wake) b->cv.notify_one();
    return TM_OK;
}

namespace {
struct Waiter {
    std::mutex m;
    std::condition_variable cv;
    bool done = false;
    int32_t status = 0;
    uint32_t n = 0, cap = 0;
    uint64_t *ids = nullptr;
};
void waiter_cb(void *ctx, int32_t status, const uint64_t *ids, uint32_t n) {
    Waiter *w = static_cast<Waiter *>(ctx);
    if (ids && w->ids) std::memcpy(w->ids, ids, (size_t)std::min(n, w->cap) * 8);
    std::lock_guard<std::mutex> g(w->m);
    w->status = status;
    w->n = n;
    w->done = true;
    w->cv.notify_one();
}
}  // namespace

int tm_batcher_match(tm_batcher *b, const uint8_t *topic, uint32_t len, uint64_t *ids, uint32_t cap, uint32_t *n_out,
                     int32_t *status) {
    if (!n_out || !status || (cap && !ids)) return TM_EINVAL;
    Waiter w;
    w.ids = ids;
    w.cap = cap;
    int rc = tm_batcher_submit(b, topic, len, waiter_cb, &w);
    if (rc) return rc;
    std::unique_lock<std::mutex> lk(w.m);
    w.cv.wait(lk, [&] { return w.done; });
    *n_out = w.n;
    *status = w.status;
    return w.status < 0 ? w.status : TM_OK;
}

int tm_batcher_apply(tm_batcher *b, const tm_op *ops, size_t n) {
    if (!b) return TM_EINVAL;
    if (!b->eb) return TM_ESTATE;
    std::lock_guard<std::mutex> g(b->eng_mu);
    return tm_apply(b->eb->eng, ops, n);
}

int tm_batcher_commit(tm_batcher *b, uint64_t *epoch_out) {
    if (!b) return TM_EINVAL;
    if (!b->eb) return TM_ESTATE;
    std::lock_guard<std::mutex> g(b->eng_mu);
    return tm_commit_epoch(b->eb->eng, epoch_out);
}

int tm_batcher_stats_get(tm_batcher *b, tm_batcher_stats *out) {
    if (!b || !out) return TM_EINVAL;
    std::vector<uint32_t> lat;
    {
        std::lock_guard<std::mutex> g(b->mu);
        out->batches = b->n_batches;
        out->publishes = b->n_pub;
        out->max_batch_seen = b->max_seen;
        out->backend_us = b->backend_ns / 1000;
        lat.assign(b->lat_ns.begin(), b->lat_ns.begin() + (ptrdiff_t)b->lat_n);
    }
    out->lat_p50_us = out->lat_p99_us = out->lat_max_us = 0;
    if (!lat.empty()) {
        auto pct = [&](double q) {
            size_t k = std::min(lat.size() - 1, (size_t)(q * (double)(lat.size() - 1) + 0.5));
            std::nth_element(lat.begin(), lat.begin() + (ptrdiff_t)k, lat.end());
            return lat[k] / 1000.0;
        };
        out->lat_p50_us = pct(0.50);
        out->lat_p99_us = pct(0.99);
        out->lat_max_us = *std::max_element(lat.begin(), lat.end()) / 1000.0;
    }
    return TM_OK;
}

}  // extern "C"
