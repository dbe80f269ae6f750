// batcher.cpp — the publish batching aggregator (include/emqx_tm_batcher.h).
//
// Reference behaviour it stands in for: emqx_broker:do_publish/1 calls
// emqx_router:match_routes/1 once per publish, synchronously, in the publisher's own process
// (apps/emqx/src/emqx_broker.erl:285-290, apps/emqx/src/emqx_router.erl:205-212).  Here many
// publishers queue single topics and the aggregator answers each with its own id list, one
// engine batch per WINDOW (max_batch publishes or max_wait_us since the oldest).
//
// Pipeline (engine backend), three stages that overlap across consecutive windows:
//   1. the cutter thread takes a window from the submission shards straight into a pinned
//      staging slot and queues its whole GPU part on the compute stream: H2D of the topics,
//      the walk (tm_match_device_mode), ids compacted topic-major (tm_result_ids_device), and
//      D2H of the offsets, statuses and the batch's counter block;
//   2. the completion thread waits for that, then copies the ids back on a separate copy
//      stream (so window k's PCIe transfer overlaps window k+1's walk);
//   3. the delivery threads call the publishers back: the completion thread splits each
//      window into publish ranges (per PCIe chunk) on one work queue, and every delivery
//      thread takes the next range, waits for its chunk's copy if it has not landed, and
//      calls that range back.  No thread waits for another: a window's slot is freed by
//      whichever thread finishes its last range, and the next window's ranges are taken
//      while stragglers of this one still run.
// Six slots rotate: the newest window is cut and walks on the GPU while earlier windows' ids cross
// PCIe and window k's publishers are called back.
// Submissions go to one of SHARDS queue shards (by submitting thread), so publishers that
// resubmit from their callbacks do not all contend on one lock.
#include <hip/hip_runtime.h>
#include <execinfo.h>
#include <signal.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/emqx_tm.h"
#include "../../include/emqx_tm_batcher.h"

extern "C" int tmx_engine_device(const tm_engine *eng);  // engine.cpp, library-internal
extern "C" int tmx_engine_grow_pools(tm_engine *eng, uint32_t set, uint64_t seg_demand, uint64_t fr_demand);
extern "C" int tmx_engine_reserve_batch(tm_engine *eng, uint32_t set, uint32_t n, uint64_t bytes);
extern "C" void tmx_engine_forget_stream(tm_engine *eng, void *stream);
extern "C" void tmx_engine_pool_caps(const tm_engine *eng, uint32_t set, uint64_t *seg_chunks, uint64_t *fr_chunks);
extern "C" int tmx_result_ids32_device(tm_engine *eng, uint32_t set, uint32_t *d_ids, uint64_t ids_cap, uint32_t *d_off_out,
                                       void *stream);
extern "C" void tmx_engine_lock(tm_engine *eng);
extern "C" void tmx_engine_unlock(tm_engine *eng);
extern "C" int tmx_batch_match_device(tm_engine *eng, uint32_t set, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                                      uint64_t total_bytes, uint32_t mode, void *stream, tm_dev_result *out);
extern "C" int tmx_result_ids64_device(tm_engine *eng, uint32_t set, uint64_t *d_ids, uint64_t ids_cap, uint32_t *d_off_out,
                                       void *stream);
extern "C" int tmx_batch_match_ids(tm_engine *eng, uint32_t set, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                                   uint64_t total_bytes, uint32_t id_bytes, void *d_ids, uint64_t ids_cap,
                                   uint32_t *d_off_out, void *stream, tm_dev_result *out);
extern "C" int tmx_batch_match_runs(tm_engine *eng, uint32_t set, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                                    uint64_t total_bytes, void *stream, void *d_spans, uint64_t spans_cap,
                                    uint32_t *d_soff, uint32_t *d_scnt, uint32_t *d_kcnt, int32_t *d_status,
                                    unsigned long long *d_cursor, const void **d_ctl_out, uint32_t id_w);
extern "C" void tmx_lease_take(tm_engine *eng);
extern "C" int tmx_batch_reserve_matches(tm_engine *eng, uint32_t set, uint64_t keys_cap);
extern "C" void tmx_lease_drop(tm_engine *eng);
extern "C" int tmx_engine_is_replica(const tm_engine *eng);
extern "C" int tmx_engine_runs_ok(const tm_engine *eng);
extern "C" uint64_t tmx_engine_epoch(const tm_engine *eng);

namespace {
// set on the delivery threads: the engine refuses a commit from a callback (it would wait for
// the read lease of the very window being delivered) and lets a callback's own runs call take
// a lease past a waiting commit
thread_local int tl_delivering = 0;
// set while a delivery thread calls back a window that holds a read lease on the engine's host
// id arena (a runs window): only then may the callback's own runs call take a lease past a
// waiting commit -- the arena cannot change while that window's lease is held.  A window without
// one (ids transport, other modes) gives its callbacks no such guarantee, so their runs calls
// wait for a commit in progress like any other caller's (advisor, round 4).
thread_local int tl_window_leased = 0;
// On a delivery thread: the clock as deliver_range last read it (it reads it once per 16
// callbacks), the submit time of a publish re-submitted from a callback.  A clock read costs
// about as much as the rest of a submit; this stamp is at most 16 callbacks (a few
// microseconds) early, so such a publish's latency is overstated by that much, never hidden.
thread_local uint64_t tl_clock_ns = 0;
}  // namespace
extern "C" __attribute__((visibility("hidden"))) int tmx_in_delivery(void) { return tl_delivering; }
extern "C" __attribute__((visibility("hidden"))) int tmx_in_leased_delivery(void) { return tl_window_leased; }

namespace {

// A thread's own CPU time (CLOCK_THREAD_CPUTIME_ID: the scheduler's runtime, ns; rusage's
// times are tick-granular) and involuntary context switches (getrusage RUSAGE_THREAD): read a
// few times per window, to tell a stage that worked from one whose thread was preempted.
struct ThreadUse {
    uint64_t cpu_ns = 0, ivcsw = 0;
};
ThreadUse thread_use() {
    ThreadUse u;
    struct timespec ts;
    if (clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts) == 0) u.cpu_ns = (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
    struct rusage r;
    if (getrusage(RUSAGE_THREAD, &r) == 0) u.ivcsw = (uint64_t)r.ru_nivcsw;
    return u;
}

// The aggregator stamps every publish (submit -> callback latency), so its clock is on the
// per-publish path: the TSC (invariant on the hosts this runs on; Linux uses it as the
// clocksource there) read in ~7 ns, against ~18 ns for steady_clock's vDSO call, scaled to
// nanoseconds by a calibration against steady_clock the first time it is used.
struct TscClock {
    uint64_t tsc0 = 0;
    double ns_per_tick = 1.0;
    TscClock() {
        using clk = std::chrono::steady_clock;
        const auto c0 = clk::now();
        tsc0 = __builtin_ia32_rdtsc();
        std::this_thread::sleep_for(std::chrono::milliseconds(3));
        const auto c1 = clk::now();
        const uint64_t t1 = __builtin_ia32_rdtsc();
        const double ns = (double)std::chrono::duration_cast<std::chrono::nanoseconds>(c1 - c0).count();
        if (t1 > tsc0 && ns > 0) ns_per_tick = ns / (double)(t1 - tsc0);
    }
};
const TscClock &tsc_clock() {
    static const TscClock c;
    return c;
}
uint64_t now_ns() {
    const TscClock &c = tsc_clock();
    const uint64_t t = __builtin_ia32_rdtsc();
    return t > c.tsc0 ? (uint64_t)((double)(t - c.tsc0) * c.ns_per_tick) : 0;
}

// Submit -> callback latency of EVERY delivered publish since the last reset, as a log-linear
// histogram (64 buckets per power of two: <= 1.6 % relative error), one per delivery thread so
// a record is two plain stores; tm_batcher_stats_get sums them.  Round 3 kept the last 65,536
// latencies in a ring, which at 60 M publishes/s held only the final millisecond of a run.
constexpr uint32_t LAT_SUB = 6;
constexpr uint32_t LAT_NB = 44u << LAT_SUB;  // up to 2^43 ns (~2.4 h): the top bucket clamps
inline uint32_t lat_bucket(uint64_t ns) {
    if (ns < (1u << LAT_SUB)) return (uint32_t)ns;
    const uint32_t sh = (uint32_t)(63 - __builtin_clzll(ns)) - LAT_SUB;
    return std::min<uint32_t>(LAT_NB - 1, ((sh + 1) << LAT_SUB) + (uint32_t)((ns >> sh) & ((1u << LAT_SUB) - 1)));
}
inline double lat_bucket_mid(uint32_t b) {  // the bucket's midpoint, ns
    if (b < (1u << LAT_SUB)) return (double)b;
    const uint32_t sh = (b >> LAT_SUB) - 1, m = b & ((1u << LAT_SUB) - 1);
    return (double)(((uint64_t)(m + (1u << LAT_SUB)) << sh)) + (double)((1ull << sh) - 1) / 2.0;
}
struct alignas(64) LatHist {
    std::atomic<uint64_t> gen{0};  // the reset generation these counts belong to
    std::atomic<uint64_t> n{0}, sum_ns{0}, max_ns{0};
    std::atomic<uint64_t> b[LAT_NB];
    LatHist() {
        for (auto &x : b) x.store(0, std::memory_order_relaxed);
    }
    // single writer (the owning delivery thread): relaxed load + store, no locked instruction
    static void bump(std::atomic<uint64_t> &x, uint64_t d) {
        x.store(x.load(std::memory_order_relaxed) + d, std::memory_order_relaxed);
    }
    void sync_gen(uint64_t g) {  // the owner clears its counts when a reset happened
        if (gen.load(std::memory_order_relaxed) == g) return;
        for (auto &x : b) x.store(0, std::memory_order_relaxed);
        n.store(0, std::memory_order_relaxed);
        sum_ns.store(0, std::memory_order_relaxed);
        max_ns.store(0, std::memory_order_relaxed);
        gen.store(g, std::memory_order_release);
    }
    void add(uint64_t ns) {
        bump(b[lat_bucket(ns)], 1);
        bump(n, 1);
        bump(sum_ns, ns);
        if (ns > max_ns.load(std::memory_order_relaxed)) max_ns.store(ns, std::memory_order_relaxed);
    }
};

// grow-only device / pinned buffers
// Growth is a stall: hipFree waits for the whole device and hipHostMalloc takes milliseconds
// (the slowest windows of a steady run were exactly the ones that grew a buffer, their
// cutter busy 3-6 ms, round 5).  So a buffer grows once to its size for a max_batch window
// (`hint`, from the per-publish high-water marks), not to the demand of the window at hand.
struct DBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes, size_t hint = 0) {
        if (bytes <= cap) return hipSuccess;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        size_t c = std::max<size_t>(std::max<size_t>(bytes + bytes / 4, hint), 4096);
        hipError_t e = hipMalloc(&p, c);
        if (e != hipSuccess && c > bytes) {  // the hint did not fit: the window's own demand
            (void)hipGetLastError();
            c = std::max<size_t>(bytes, 4096);
            e = hipMalloc(&p, c);
        }
        if (e == hipSuccess) cap = c;
        else p = nullptr;
        return e;
    }
    ~DBuf() {
        if (p) (void)hipFree(p);
    }
};
// pinned host memory (engine backend: DMA-able), or plain memory for a custom backend
struct HBuf {
    void *p = nullptr;
    size_t cap = 0;
    bool pinned = true;
    void drop() {
        if (p) {
            if (pinned) (void)hipHostFree(p);
            else std::free(p);
        }
        p = nullptr;
        cap = 0;
    }
    hipError_t ensure(size_t bytes, size_t hint = 0) {
        if (bytes <= cap) return hipSuccess;
        drop();
        size_t c = std::max<size_t>(std::max<size_t>(bytes + bytes / 4, hint), 4096);
        if (!pinned) {
            p = std::malloc(c);
            if (!p) return hipErrorOutOfMemory;
            cap = c;
            return hipSuccess;
        }
        hipError_t e = hipHostMalloc(&p, c, hipHostMallocDefault);
        if (e != hipSuccess && c > bytes) {  // the hint did not fit: the window's own demand
            (void)hipGetLastError();
            c = std::max<size_t>(bytes, 4096);
            e = hipHostMalloc(&p, c, hipHostMallocDefault);
        }
        if (e == hipSuccess) cap = c;
        else p = nullptr;
        return e;
    }
    template <class T>
    T *as() const {
        return (T *)p;
    }
    ~HBuf() { drop(); }
};

// the HIP call that failed last on this thread (reported with the window's failure)
thread_local char bt_err[160];
#define BT_HIP(E)                                                                                  \
    do {                                                                                           \
        const hipError_t bt_e_ = (E);                                                              \
        if (bt_e_ != hipSuccess) {                                                                 \
            std::snprintf(bt_err, sizeof bt_err, "%s at batcher.cpp:%d", hipGetErrorString(bt_e_), \
                          __LINE__);                                                               \
            return TM_EDEVICE;                                                                     \
        }                                                                                          \
    } while (0)

struct Pending {
    uint32_t len;
    uint32_t kind;     // CB_IDS: id list, CB_SPANS: u64 spans, CB_SPANS32: u32 spans
    void (*fn)();      // the callback, of the type `kind` names
    void *ctx;
    uint64_t t0;  // submit time (ns)
};
enum : uint32_t { CB_IDS = 0, CB_SPANS = 1, CB_SPANS32 = 2 };

constexpr size_t QUEUE_BYTES_MAX = 1ull << 31;
constexpr uint32_t SHARDS = 16;
#ifndef TM_NSLOT
#define TM_NSLOT 6
#endif
// windows in flight: the newest cut / on the GPU, older ones on PCIe or waiting, the oldest being
// delivered.  Round 2: a fourth slot let the next window be cut while delivery still held one
// (65,536 closed-loop publishers: 39 -> 44 M publishes/s); round 3, span callbacks: 4 slots
// 42.7, 6 slots 48.7, 8 slots 40.7 M publishes/s (smaller windows: the cutter's share grows),
// profiles/r03_batcher_sweep.jsonl
constexpr uint32_t NSLOT = TM_NSLOT;
constexpr uint32_t NSLOT_MAX = 8;  // EMQX_TM_NSLOT (development knob) may raise it up to this
constexpr uint32_t CTL_BYTES = 32;
// the threads that wait on these sleep in the driver instead of spinning a CPU of the quota
constexpr unsigned EV_FLAGS = hipEventDisableTiming | hipEventBlockingSync;  // the engine's per-launch counter block {total, slow, seg, fr}

struct alignas(64) Shard {
    std::mutex m;
    std::vector<uint8_t> bytes;
    std::vector<Pending> q;
    std::atomic<uint32_t> n{0};  // q.size(), readable without the lock (the cutter's polls)
};

uint32_t shard_of_thread() {
    static std::atomic<uint32_t> next{0};
    thread_local uint32_t me = next.fetch_add(1) % SHARDS;
    return me;
}

// One window in flight: its publishers, its host/device buffers and its result view.
struct Slot {
    enum State { FREE, BUSY } state = FREE;
    std::vector<Pending> pubs;
    uint32_t n = 0;
    uint32_t mode = 0;
    int rc = 0;
    uint64_t t_enq = 0, t_done = 0;
    // stage stamps of this window (tm_batcher_window)
    uint64_t t_old = 0, t_cut = 0, t_queued = 0, t_gpu = 0;
    std::atomic<uint64_t> t_deliver{0};
    uint64_t t_slot = 0;
    uint32_t cut_cpu_us = 0, cut_ivcsw = 0, wait_ivcsw = 0;
    std::atomic<uint64_t> del_cpu_ns{0}, del_wall_ns{0};
    std::atomic<uint32_t> del_ivcsw{0};
    uint32_t wflags = 0;
    uint64_t epoch = 0;
    // engine backend
    HBuf h_bytes, h_off, h_off_out, h_status, h_cnt, h_ids, h_ctl;
    DBuf d_bytes, d_off, d_ids, d_off_out;
    uint64_t nbytes = 0, ids_cap = 0, keys_cap = 0;
    hipEvent_t ev = nullptr;
    // the ids cross PCIe in chunks (by publish range) and delivery starts on a chunk as soon
    // as its copy is done, so a window's copy and its callbacks overlap
    static constexpr uint32_t MAXCH = 8;
    uint32_t nchunk = 1;
    uint32_t chunk_lo[MAXCH + 1] = {};
    hipEvent_t cev[MAXCH] = {};
    std::atomic<uint8_t> chunk_ready[MAXCH] = {};  // cev[j] has been waited for by some thread
    std::atomic<uint32_t> parts_left{0};           // delivery ranges not yet called back
    bool cev_wait = false;              // chunk events to wait for before delivering
    bool narrow = false;                // ids crossed PCIe as u32 (every id < 2^32); widened at delivery
    bool host_done = false;             // the result was produced synchronously (custom / host path)
    std::vector<uint32_t> cnt;          // per-publish counts
    std::vector<uint64_t> ids_host;     // host-path ids
    tm_batch_view v{};
    // runs transport (TM_MATCH_ALL on a master engine): the walk's spans of the engine's host
    // id arena cross PCIe instead of the ids; the window holds a read lease until delivered
    bool runs = false, leased = false;
    uint32_t runs_w = 8;  // runs: id width of the window's spans (4: the engine's u32 id arena)
    DBuf d_spans, d_soff, d_scnt, d_kcnt, d_st, d_cur;
    HBuf h_spans, h_soff, h_scnt, h_kcnt;
    uint64_t spans_cap = 0;
    uint64_t spans_need = 0;  // a re-run's span demand (complete_runs), 0 otherwise
    const void *d_ctl = nullptr;
    uint32_t set = 0;  // the engine buffer set and compute stream of this slot (slot index & 1)
};

}  // namespace

struct tm_batcher {
    tm_batch_fn fn = nullptr;
    void *backend = nullptr;
    tm_engine *eng = nullptr;  // engine backend (else fn/backend)
    tm_batcher_config cfg{};
    uint32_t n_delivery = 4;

    Shard shards[SHARDS];
    std::mutex wake_mu;  // cutter sleep/wake
    std::condition_variable wake_cv;
    std::atomic<bool> stopping{false};
    std::atomic<uint32_t> cutter_idle{0};  // 1 while the cutter sleeps on an empty queue

    std::mutex eng_mu;  // the cutter's enqueue vs a re-run from the completion thread
    // runs transport: spans per publish of recent windows (sizes the next); written by the
    // completion thread, read by the cutter (found by ThreadSanitizer, round 4)
    std::atomic<double> spans_per_pub{4.0};
    // per-publish high-water marks: buffer sizes for a max_batch window (DBuf/HBuf::ensure).
    // Only windows of at least max_batch/8 publishes raise them: a lone high-fan-out publish
    // in a low-load window (one publish, 10 K route ids) would otherwise size every later
    // window's buffers at 1.25 x max_batch x 10 K ids.  Each hint is capped at HINT_MAX bytes;
    // past that a buffer grows to a window's own demand (DBuf/HBuf::ensure).
    std::atomic<double> hw_bytes{64.0}, hw_spans{4.0}, hw_ids{16.0};
    static constexpr size_t HINT_MAX = size_t(256) << 20;
    void raise_hw(std::atomic<double> &hw, double v, uint32_t n) {
        if ((uint64_t)n * 8 < cfg.max_batch) return;
        double c = hw.load(std::memory_order_relaxed);
        while (v > c && !hw.compare_exchange_weak(c, v, std::memory_order_relaxed)) {
        }
    }
    bool hints = true;  // EMQX_TM_BATCHER_HINTS=0 (development): grow to each window's demand only
    size_t hint_of(const std::atomic<double> &hw, size_t width) const {
        if (!hints) return 0;
        const double b = hw.load(std::memory_order_relaxed) * 1.25 * cfg.max_batch * (double)width + 64;
        return (size_t)std::min<double>(b, (double)HINT_MAX);
    }
    size_t hint_pub4() const { return hints ? ((size_t)cfg.max_batch + 1) * 4 : 0; }
    // pool growth for a max_batch window at this window's rate, from windows of at least
    // max_batch/8 publishes only (at most 8x their demand)
    double pool_scale(uint32_t n) const {
        if (!hints) return 1.0;
        return std::min(8.0, std::max(1.0, (double)cfg.max_batch / std::max<uint32_t>(n, 1)));
    }
    std::atomic<bool> reported{false};  // the first failed window is reported on stderr (once)
    void report(const char *stage, int rc) {
        if (rc >= 0 || reported.exchange(true)) return;
        std::fprintf(stderr, "tm_batcher: a window failed in %s: rc %d (%s%s%s)\n", stage, rc,
                     eng ? tm_last_error(eng) : "custom backend", bt_err[0] ? "; " : "", bt_err);
    }
    bool runs_ok = false;        // runs transport in use (TM_MATCH_ALL windows of a master engine)
    // delivery prefetch (runs transport): replies this many publishes ahead have their spans'
    // first line prefetched, or (pf_lines > 0) up to pf_lines lines of them (development knobs
    // EMQX_TM_PF_PUBS / EMQX_TM_PF_LINES)
    uint32_t pf_pubs = 6, pf_lines = 0;
    // delivery threads' nice value (EMQX_TM_DELIVERY_NICE; unprivileged processes may raise it)
    int deliver_nice = 0;
    // publish ranges per delivery thread and chunk (EMQX_TM_RANGES_PER_THREAD): with more, a
    // delivery thread preempted in mid-range holds back fewer publishes while the others take
    // the rest of the chunk
    uint32_t ranges_per_thread = 1;
    // runs windows: spans of the u64 id arena (zero-copy for id-list and u64-span callbacks), or
    // (EMQX_TM_RUNS_IDW=4) of the u32 one while every id fits.  Measured on the box at 65,536
    // closed-loop publishers: u32 windows made the id-list and u64-span callbacks
    // pay a widening copy per reply (64 -> 42 / 72 -> 37 M/s) and gave the u32-span callback
    // no gain over u64 spans, so u64 is the default.
    uint32_t runs_w = 8;
    // two compute streams, each with its own engine buffer set: consecutive windows alternate,
    // so one window's walk starts while the previous one's last waves finish
    hipStream_t s_comps[2] = {}, s_copy = nullptr;
    int device = 0;

    Slot slot[NSLOT_MAX];
    uint32_t nslot = NSLOT;
    std::mutex slot_mu;  // slot states + completion FIFO
    std::condition_variable slot_cv;
    std::deque<uint32_t> fifo;   // slots queued for completion, in window order
    bool cutter_done = false;    // under slot_mu

    std::thread cutter, completer;
    std::vector<std::thread> workers;  // delivery threads
    // delivery work: publish ranges of the windows, in window order
    struct Work {
        uint32_t slot, chunk, lo, hi;
    };
    std::mutex work_mu;
    std::condition_variable work_cv;
    std::deque<Work> work;
    std::atomic<uint32_t> work_n{0};     // work.size(), polled without the lock
    std::atomic<uint32_t> sleepers{0};   // delivery threads blocked on work_cv
    bool work_closed = false;            // under work_mu: no more ranges will come

    std::mutex st_mu;  // stats
    uint64_t n_batches = 0, n_pub = 0, max_seen = 0, backend_ns = 0;
    std::atomic<uint64_t> ns_cut{0}, ns_enq{0}, ns_gpu{0}, ns_copy{0}, ns_del{0};  // stage times
    std::unique_ptr<LatHist[]> lat;        // one per delivery thread
    std::atomic<uint64_t> lat_gen{1};      // tm_batcher_stats_reset bumps it
    std::chrono::steady_clock::time_point t_window;  // start of the stats window (under st_mu)

    // ------------------------------------------------------------------ submit side
    // No state shared by all submitters on this path: one shard lock (shards by submitting
    // thread) and a read of the cutter's idle flag.
    int submit(const uint8_t *topic, uint32_t len, uint32_t kind, void (*fn)(), void *ctx) {
        const uint64_t t0 = tl_clock_ns ? tl_clock_ns : now_ns();
        Shard &sh = shards[shard_of_thread()];
        {
            std::lock_guard<std::mutex> g(sh.m);
            // checked under the shard lock: the cutter's last pass over this shard comes after
            // `stopping` is set, so a publish either lands before that pass or is refused here
            if (stopping.load()) return TM_ESTATE;
            if (sh.bytes.size() + len > QUEUE_BYTES_MAX / SHARDS) return TM_ENOMEM;  // back-pressure
            sh.q.push_back(Pending{len, kind, fn, ctx, t0});
            sh.bytes.insert(sh.bytes.end(), topic, topic + len);
            sh.n.store((uint32_t)sh.q.size(), std::memory_order_relaxed);
        }
        if (cutter_idle.load()) {
            std::lock_guard<std::mutex> g(wake_mu);
            wake_cv.notify_one();
        }
        return TM_OK;
    }

    uint64_t queued_now() const {
        uint64_t n = 0;
        for (const Shard &sh : shards) n += sh.n.load(std::memory_order_relaxed);
        return n;
    }

    uint64_t oldest_t0() {
        uint64_t t = ~0ull;
        for (Shard &sh : shards) {
            std::lock_guard<std::mutex> g(sh.m);
            if (!sh.q.empty()) t = std::min(t, sh.q.front().t0);
        }
        return t;
    }

    // Move up to max_batch queued publishes into slot S (bytes into its pinned staging).
    int take_window(Slot &S) {
        S.pubs.clear();
        uint64_t nb = 0;
        // sizes first (the shards keep filling; we take what is there now)
        for (Shard &sh : shards) {
            std::lock_guard<std::mutex> g(sh.m);
            nb += sh.bytes.size();
        }
        S.n = 0;
        BT_HIP(S.h_bytes.ensure(nb + 64, hint_of(hw_bytes, 1)));
        BT_HIP(S.h_off.ensure(((size_t)cfg.max_batch + 1) * 4));
        uint8_t *dst = S.h_bytes.as<uint8_t>();
        uint64_t at = 0, taken_bytes = 0;
        static thread_local uint32_t rot = 0;
        rot++;
        for (uint32_t k = 0; k < SHARDS && S.pubs.size() < cfg.max_batch; k++) {
            Shard &sh = shards[(rot + k) % SHARDS];
            std::lock_guard<std::mutex> g(sh.m);
            if (sh.q.empty()) continue;
            size_t take = std::min<size_t>(sh.q.size(), cfg.max_batch - S.pubs.size());
            uint64_t tb = 0;
            for (size_t i = 0; i < take; i++) tb += sh.q[i].len;
            if (at + tb > nb + 64) {  // grew since sizing: take what fits
                take = 0;
                tb = 0;
                while (take < sh.q.size() && at + tb + sh.q[take].len <= nb + 64 && S.pubs.size() + take < cfg.max_batch)
                    tb += sh.q[take++].len;
            }
            std::memcpy(dst + at, sh.bytes.data(), tb);
            at += tb;
            S.pubs.insert(S.pubs.end(), sh.q.begin(), sh.q.begin() + (ptrdiff_t)take);
            sh.q.erase(sh.q.begin(), sh.q.begin() + (ptrdiff_t)take);
            sh.bytes.erase(sh.bytes.begin(), sh.bytes.begin() + (ptrdiff_t)tb);
            sh.n.store((uint32_t)sh.q.size(), std::memory_order_relaxed);
            taken_bytes += tb;
        }
        (void)taken_bytes;
        S.n = (uint32_t)S.pubs.size();
        // each shard is FIFO, so the window's oldest publish is the oldest of the shards' heads
        S.t_old = ~0ull;
        for (const Pending &p : S.pubs) S.t_old = std::min(S.t_old, p.t0);
        S.nbytes = at;
        if (S.n) raise_hw(hw_bytes, (double)at / S.n, S.n);
        uint32_t *o = S.h_off.as<uint32_t>();
        uint32_t pos = 0;
        for (uint32_t i = 0; i < S.n; i++) {
            o[i] = pos;
            pos += S.pubs[i].len;
        }
        o[S.n] = pos;
        return TM_OK;
    }

    // ------------------------------------------------------------------ engine backend
    // Queue window S's GPU part on the compute stream.  Caller holds eng_mu.  The engine's
    // device lock is held across the whole sequence, so no other caller's batch (a direct
    // tm_match_device on the same engine) lands between the walk and the reads of its result.
    int enqueue(Slot &S) {
        tmx_engine_lock(eng);
        const int rc = enqueue_locked(S);
        tmx_engine_unlock(eng);
        return rc;
    }
    int enqueue_locked(Slot &S) {
        const uint32_t n = S.n;
        S.host_done = false;
        if (S.runs) return enqueue_runs(S);
        hipStream_t s_comp = s_comps[S.set];
        BT_HIP(hipSetDevice(device));
        BT_HIP(S.d_bytes.ensure(S.nbytes + 16, hint_of(hw_bytes, 1)));
        BT_HIP(S.d_off.ensure((size_t)n * 4 + 4, hint_pub4()));
        BT_HIP(S.d_off_out.ensure((size_t)n * 4 + 4, hint_pub4()));
        BT_HIP(S.h_off_out.ensure((size_t)n * 4 + 4, hint_pub4()));
        BT_HIP(S.h_status.ensure((size_t)n * 4 + 4, hint_pub4()));
        BT_HIP(S.h_cnt.ensure((size_t)n * 4 + 4, hint_pub4()));
        BT_HIP(S.h_ctl.ensure(CTL_BYTES));
        if (!S.ev) BT_HIP(hipEventCreateWithFlags(&S.ev, EV_FLAGS));
        BT_HIP(hipMemcpyAsync(S.d_bytes.p, S.h_bytes.p, S.nbytes + 1, hipMemcpyHostToDevice, s_comp));
        BT_HIP(hipMemcpyAsync(S.d_off.p, S.h_off.p, (size_t)n * 4 + 4, hipMemcpyHostToDevice, s_comp));
        tm_dev_result r;
        if (S.mode == TM_MATCH_ALL) {
            // the walk writes the route ids itself (u32 while every id fits), compacted
            // topic-major: no key handles, no separate id pass (tm_match_ids_device)
            S.ids_cap = std::max<uint64_t>(S.ids_cap, std::max<uint64_t>(hint_of(hw_ids, 8) / 8, 1 << 16));
            BT_HIP(S.d_ids.ensure(S.ids_cap * 8 + 8));
            S.narrow = true;
            int rc = tmx_batch_match_ids(eng, S.set, (const uint8_t *)S.d_bytes.p, (const uint32_t *)S.d_off.p, n, S.nbytes, 4,
                                         S.d_ids.p, S.ids_cap, (uint32_t *)S.d_off_out.p, s_comp, &r);
            if (rc == TM_ESTATE) {
                S.narrow = false;
                rc = tmx_batch_match_ids(eng, S.set, (const uint8_t *)S.d_bytes.p, (const uint32_t *)S.d_off.p, n, S.nbytes, 8,
                                         S.d_ids.p, S.ids_cap, (uint32_t *)S.d_off_out.p, s_comp, &r);
            }
            if (rc) return rc;
            S.keys_cap = std::min(r.keys_cap, S.ids_cap);
            std::memset(S.h_ctl.p, 0, CTL_BYTES);
            BT_HIP(hipMemcpyAsync(S.h_ctl.p, r.d_total, CTL_BYTES, hipMemcpyDeviceToHost, s_comp));
            BT_HIP(hipMemcpyAsync(S.h_off_out.p, S.d_off_out.p, (size_t)n * 4 + 4, hipMemcpyDeviceToHost, s_comp));
            BT_HIP(hipMemcpyAsync(S.h_status.p, r.d_status, (size_t)n * 4, hipMemcpyDeviceToHost, s_comp));
            BT_HIP(hipEventRecord(S.ev, s_comp));
            return TM_OK;
        }
        int rc = tmx_batch_match_device(eng, S.set, (const uint8_t *)S.d_bytes.p, (const uint32_t *)S.d_off.p, n, S.nbytes,
                                        S.mode, s_comp, &r);
        if (rc) return rc;
        S.keys_cap = r.keys_cap;
        std::memset(S.h_ctl.p, 0, CTL_BYTES);
        // the batch's counter block (total, spills, pool demand): the next launch reuses it
        BT_HIP(hipMemcpyAsync(S.h_ctl.p, r.d_total, CTL_BYTES, hipMemcpyDeviceToHost, s_comp));
        if (S.mode == TM_MATCH_COUNT) {
            BT_HIP(hipMemcpyAsync(S.h_cnt.p, r.d_cnt, (size_t)n * 4, hipMemcpyDeviceToHost, s_comp));
        } else {
            S.ids_cap = S.mode == TM_MATCH_FIRST ? n : r.keys_cap;
            BT_HIP(S.d_ids.ensure(S.ids_cap * 8 + 8));
            // u32 ids while they fit: half the PCIe bytes, the bottleneck of this path
            rc = tmx_result_ids32_device(eng, S.set, (uint32_t *)S.d_ids.p, S.ids_cap, (uint32_t *)S.d_off_out.p, s_comp);
            S.narrow = rc == TM_OK;
            if (rc == TM_ESTATE)
                rc = tmx_result_ids64_device(eng, S.set, (uint64_t *)S.d_ids.p, S.ids_cap, (uint32_t *)S.d_off_out.p, s_comp);
            if (rc) return rc;
            BT_HIP(hipMemcpyAsync(S.h_off_out.p, S.d_off_out.p, (size_t)n * 4 + 4, hipMemcpyDeviceToHost, s_comp));
        }
        BT_HIP(hipMemcpyAsync(S.h_status.p, r.d_status, (size_t)n * 4, hipMemcpyDeviceToHost, s_comp));
        BT_HIP(hipEventRecord(S.ev, s_comp));
        return TM_OK;
    }

    // Runs transport: the walk writes the window's spans and per-publish arrays into the slot;
    // the counters (span cursor, pool demand) and the per-publish arrays come back on the
    // compute stream, the spans themselves on the copy stream once their count is known.
    int enqueue_runs(Slot &S) {
        const uint32_t n = S.n;
        hipStream_t s_comp = s_comps[S.set];
        BT_HIP(hipSetDevice(device));
        BT_HIP(S.d_bytes.ensure(S.nbytes + 16, hint_of(hw_bytes, 1)));
        BT_HIP(S.d_off.ensure((size_t)n * 4 + 4, hint_pub4()));
        for (DBuf *d : {&S.d_soff, &S.d_scnt, &S.d_kcnt, &S.d_st}) BT_HIP(d->ensure((size_t)n * 4 + 4, hint_pub4()));
        BT_HIP(S.d_cur.ensure(64));
        for (HBuf *h : {&S.h_soff, &S.h_scnt, &S.h_kcnt, &S.h_status}) BT_HIP(h->ensure((size_t)n * 4 + 4, hint_pub4()));
        BT_HIP(S.h_ctl.ensure(64));
        if (!S.ev) BT_HIP(hipEventCreateWithFlags(&S.ev, EV_FLAGS));
        const uint64_t want = std::max<uint64_t>(
            std::max<uint64_t>(4096, (uint64_t)(spans_per_pub.load(std::memory_order_relaxed) * 1.5 * n) + 1024),
            S.spans_need);
        if (S.spans_cap < want) {
            BT_HIP(S.d_spans.ensure(want * 16, hint_of(hw_spans, 16)));
            S.spans_cap = S.d_spans.cap / 16;
        }
        BT_HIP(hipMemcpyAsync(S.d_bytes.p, S.h_bytes.p, S.nbytes + 1, hipMemcpyHostToDevice, s_comp));
        BT_HIP(hipMemcpyAsync(S.d_off.p, S.h_off.p, (size_t)n * 4 + 4, hipMemcpyHostToDevice, s_comp));
        // spans of the u32 id arena while every id fits (half the lines a reply reads), else u64
        S.runs_w = runs_w;
        int rc = TM_ESTATE;
        for (int k = 0; k < 2 && rc == TM_ESTATE; k++) {
            rc = tmx_batch_match_runs(eng, S.set, (const uint8_t *)S.d_bytes.p, (const uint32_t *)S.d_off.p, n, S.nbytes,
                                      s_comp, S.d_spans.p, S.spans_cap, (uint32_t *)S.d_soff.p, (uint32_t *)S.d_scnt.p,
                                      (uint32_t *)S.d_kcnt.p, (int32_t *)S.d_st.p, (unsigned long long *)S.d_cur.p,
                                      &S.d_ctl, S.runs_w);
            if (rc == TM_ESTATE && S.runs_w == 4) S.runs_w = 8;
            else break;
        }
        if (rc) return rc;
        // h_ctl: [0] spans reserved, [1..4] the launch's counter block {-, slow, seg, fr}
        BT_HIP(hipMemcpyAsync(S.h_ctl.p, S.d_cur.p, 8, hipMemcpyDeviceToHost, s_comp));
        BT_HIP(hipMemcpyAsync(S.h_ctl.as<uint8_t>() + 8, S.d_ctl, CTL_BYTES, hipMemcpyDeviceToHost, s_comp));
        BT_HIP(hipMemcpyAsync(S.h_soff.p, S.d_soff.p, (size_t)n * 4, hipMemcpyDeviceToHost, s_comp));
        BT_HIP(hipMemcpyAsync(S.h_scnt.p, S.d_scnt.p, (size_t)n * 4, hipMemcpyDeviceToHost, s_comp));
        BT_HIP(hipMemcpyAsync(S.h_kcnt.p, S.d_kcnt.p, (size_t)n * 4, hipMemcpyDeviceToHost, s_comp));
        BT_HIP(hipMemcpyAsync(S.h_status.p, S.d_st.p, (size_t)n * 4, hipMemcpyDeviceToHost, s_comp));
        BT_HIP(hipEventRecord(S.ev, s_comp));
        return TM_OK;
    }

    int complete_runs(Slot &S) {
        const uint64_t tw0 = now_ns();
        BT_HIP(hipEventSynchronize(S.ev));
        S.t_gpu = now_ns();
        ns_gpu.fetch_add(S.t_gpu - tw0, std::memory_order_relaxed);
        const uint64_t *ctl = S.h_ctl.as<uint64_t>();
        uint64_t total = ctl[0];
        const uint64_t seg = ctl[3], fr = ctl[4];
        uint64_t seg_cap = 0, fr_cap = 0;
        tmx_engine_pool_caps(eng, S.set, &seg_cap, &fr_cap);
        const bool over = total > S.spans_cap;
        if (over || seg > seg_cap || fr > fr_cap) {
            std::lock_guard<std::mutex> g(eng_mu);
            BT_HIP(hipStreamSynchronize(s_comps[S.set]));
            // to a max_batch window's demand at this window's rate (growth stalls the device)
            const double sc = pool_scale(S.n);
            int rc = tmx_engine_grow_pools(eng, S.set, (uint64_t)(seg * sc), (uint64_t)(fr * sc));
            if (rc) return rc;
            if (over) {  // more spans than the window's buffer: grow to the demand, run again
                raise_hw(hw_spans, (double)total / std::max<uint32_t>(S.n, 1), S.n);
                if ((uint64_t)S.n * 8 >= cfg.max_batch)  // a small window sizes only its own re-run
                    spans_per_pub.store(std::max(spans_per_pub.load(std::memory_order_relaxed),
                                                 (double)total / std::max<uint32_t>(S.n, 1)),
                                        std::memory_order_relaxed);
                S.spans_need = total + total / 8 + 1024;
                S.wflags |= TM_WIN_RERUN;
                rc = enqueue(S);
                S.spans_need = 0;
                if (rc) return rc;
                BT_HIP(hipEventSynchronize(S.ev));
                S.t_gpu = now_ns();
                total = S.h_ctl.as<uint64_t>()[0];
                if (total > S.spans_cap) return TM_EDEVICE;
            }
        }
        {  // a moving average weighted by the window's size (small windows barely move it)
            const double a = 0.1 * std::min(1.0, 8.0 * S.n / std::max<uint32_t>(cfg.max_batch, 1));
            spans_per_pub.store((1 - a) * spans_per_pub.load(std::memory_order_relaxed) +
                                    a * ((double)total / std::max<uint32_t>(S.n, 1)),
                                std::memory_order_relaxed);
        }
        raise_hw(hw_spans, (double)total / std::max<uint32_t>(S.n, 1), S.n);
        BT_HIP(S.h_spans.ensure(total * 16 + 16, hint_of(hw_spans, 16)));
        S.nchunk = 1;
        S.chunk_lo[0] = 0;
        S.chunk_lo[1] = S.n;
        BT_HIP(hipStreamWaitEvent(s_copy, S.ev, 0));
        if (total) BT_HIP(hipMemcpyAsync(S.h_spans.p, S.d_spans.p, total * 16, hipMemcpyDeviceToHost, s_copy));
        BT_HIP(hipEventRecord(S.cev[0], s_copy));
        S.cev_wait = true;
        S.v.status = S.h_status.as<int32_t>();
        return TM_OK;
    }

    // UNIQUE over keys deeper than the device order code: tm_match_batch reduces on the host.
    // Synchronous; copies the result into the slot (engine memory is reused by the next call).
    int run_host(Slot &S) {
        S.narrow = false;
        for (hipStream_t sc : s_comps) BT_HIP(hipStreamSynchronize(sc));  // nothing of ours in flight on the engine
        tm_result res;
        int rc = tm_match_batch(eng, S.h_bytes.as<uint8_t>(), S.h_off.as<uint32_t>(), S.n, S.mode, &res);
        if (rc) return rc;
        S.ids_host.resize(res.total + 1);
        S.cnt.resize(S.n);
        BT_HIP(S.h_off_out.ensure((size_t)S.n * 4 + 4));
        BT_HIP(S.h_status.ensure((size_t)S.n * 4 + 4));
        uint32_t *oo = S.h_off_out.as<uint32_t>();
        uint64_t pos = 0;
        for (uint32_t i = 0; i < S.n; i++) {
            oo[i] = (uint32_t)pos;
            S.cnt[i] = res.cnt[i];
            if (res.cnt[i] && (rc = tm_key_ids(eng, res.keys + res.off[i], res.cnt[i], S.ids_host.data() + pos)))
                return rc;
            pos += res.cnt[i];
        }
        oo[S.n] = (uint32_t)pos;
        std::memcpy(S.h_status.p, res.status, (size_t)S.n * 4);
        S.v = tm_batch_view{oo, S.cnt.data(), S.ids_host.data(), S.h_status.as<int32_t>()};
        S.host_done = true;
        return TM_OK;
    }

    // Completion of an engine window: counter block back -> maybe re-run -> ids D2H -> view.
    int complete(Slot &S) {
        if (S.host_done) {
            S.nchunk = 1;
            S.chunk_lo[0] = 0;
            S.chunk_lo[1] = S.n;
            S.cev_wait = false;
            return TM_OK;
        }
        if (S.runs) return complete_runs(S);
        const uint64_t tw0 = now_ns();
        BT_HIP(hipEventSynchronize(S.ev));
        const uint64_t tw1 = now_ns();
        S.t_gpu = tw1;
        ns_gpu.fetch_add(tw1 - tw0, std::memory_order_relaxed);
        const uint64_t *ctl = S.h_ctl.as<uint64_t>();
        const uint64_t total = ctl[0], seg = ctl[2], fr = ctl[3];
        const bool over = (S.mode != TM_MATCH_COUNT && S.mode != TM_MATCH_FIRST) && total > S.keys_cap;
        uint64_t seg_cap = 0, fr_cap = 0;
        tmx_engine_pool_caps(eng, S.set, &seg_cap, &fr_cap);
        if (over || seg > seg_cap || fr > fr_cap) {
            // pools sized to the demand for later windows (only when short: the engine compares)
            std::lock_guard<std::mutex> g(eng_mu);
            BT_HIP(hipStreamSynchronize(s_comps[S.set]));
            // to a max_batch window's demand at this window's rate (growth stalls the device)
            const double sc = pool_scale(S.n);
            int rc = tmx_engine_grow_pools(eng, S.set, (uint64_t)(seg * sc), (uint64_t)(fr * sc));
            if (rc) return rc;
            if (over) {  // output arena too small: grow to the demand, run this window again
                raise_hw(hw_ids, (double)total / std::max<uint32_t>(S.n, 1), S.n);
                const uint64_t want = std::max<uint64_t>(total + total / 8 + 1024, hint_of(hw_ids, 8) / 8);
                // a TM_MATCH_ALL window's walk writes ids: u64 ones take two words of the arena
                const uint64_t words = S.mode == TM_MATCH_ALL && !S.narrow ? 2 * want : want;
                if ((rc = tmx_batch_reserve_matches(eng, S.set, words))) return rc;
                if (S.mode == TM_MATCH_ALL) S.ids_cap = std::max(S.ids_cap, want);
                S.wflags |= TM_WIN_RERUN;
                if ((rc = enqueue(S))) return rc;
                BT_HIP(hipEventSynchronize(S.ev));
                S.t_gpu = now_ns();
                if (S.h_ctl.as<uint64_t>()[0] > S.keys_cap) {
                    std::snprintf(bt_err, sizeof bt_err, "re-run still past its output (%llu > %llu ids)",
                                  (unsigned long long)S.h_ctl.as<uint64_t>()[0], (unsigned long long)S.keys_cap);
                    return TM_EDEVICE;
                }
            }
        }
        S.v.status = S.h_status.as<int32_t>();
        S.nchunk = 1;
        S.chunk_lo[0] = 0;
        S.chunk_lo[1] = S.n;
        if (S.mode == TM_MATCH_COUNT) {
            S.cev_wait = false;
            uint32_t *oo = S.h_off_out.as<uint32_t>();
            std::memset(oo, 0, (size_t)S.n * 4);
            S.v.off = oo;
            S.v.cnt = S.h_cnt.as<uint32_t>();
            S.v.ids = nullptr;
            return TM_OK;
        }
        const uint32_t *oo = S.h_off_out.as<uint32_t>();
        const uint64_t got = oo[S.n];
        const uint64_t w = S.narrow ? 4 : 8;
        raise_hw(hw_ids, (double)got / std::max<uint32_t>(S.n, 1), S.n);
        BT_HIP(S.h_ids.ensure(got * w + 8, hint_of(hw_ids, w)));
        // chunks of >= 2 MiB of ids, at most MAXCH, cut at publish boundaries
        uint32_t nch = (uint32_t)std::min<uint64_t>(Slot::MAXCH, std::max<uint64_t>(1, got * w >> 21));
        nch = std::max<uint32_t>(1, std::min<uint32_t>(nch, S.n));
        S.chunk_lo[0] = 0;
        for (uint32_t j = 1; j < nch; j++) {  // first publish whose ids start at or past j/nch
            const uint64_t want = got * j / nch;
            S.chunk_lo[j] = (uint32_t)(std::lower_bound(oo, oo + S.n, (uint32_t)want) - oo);
            S.chunk_lo[j] = std::max(S.chunk_lo[j], S.chunk_lo[j - 1]);
        }
        S.chunk_lo[nch] = S.n;
        S.nchunk = nch;
        for (uint32_t j = 0; j < nch; j++) {
            const uint64_t a = oo[S.chunk_lo[j]], b = oo[S.chunk_lo[j + 1]];
            if (b > a)
                // DMA, not launch_copy_to_host: a window's chunks are a few MB, and a copy kernel
                // here competes with the next windows' walks (ids transport 45 -> 37 M/s at
                // 65,536 publishers when it was tried)
                BT_HIP(hipMemcpyAsync(S.h_ids.as<uint8_t>() + a * w, (const uint8_t *)S.d_ids.p + a * w, (b - a) * w,
                                      hipMemcpyDeviceToHost, s_copy));
            BT_HIP(hipEventRecord(S.cev[j], s_copy));
        }
        S.cnt.resize(S.n);
        for (uint32_t i = 0; i < S.n; i++) S.cnt[i] = oo[i + 1] - oo[i];
        S.v.off = oo;
        S.v.cnt = S.cnt.data();
        S.v.ids = S.h_ids.as<uint64_t>();  // u32 words when narrow (deliver_range widens)
        S.cev_wait = true;
        return TM_OK;
    }

    // ------------------------------------------------------------------ delivery
    // one publish's reply: its own id list (gathered from its spans when it has several), or
    // the spans themselves for a span callback
    // one publish's reply from spans of u64 ids: its own id list (gathered when it has
    // several), the spans themselves for a span callback; a u32-span callback gets them only
    // narrowed from a window whose ids fit (else TM_ESTATE)
    static void reply(const Pending &p, int32_t st, const tm_span *sp, uint32_t ns, uint64_t nids) {
        thread_local std::vector<uint64_t> flat;
        if (p.kind == CB_SPANS) {
            reinterpret_cast<tm_spans_cb>(p.fn)(p.ctx, st, sp, ns, nids);
            return;
        }
        if (p.kind == CB_SPANS32) {  // a window of u64 ids: narrowed into one span while they fit
            thread_local std::vector<uint32_t> narrow;
            if (narrow.size() < nids) narrow.resize(nids);
            uint64_t at = 0, wide = 0;
            for (uint32_t j = 0; j < ns; j++) {
                const uint64_t *src = sp[j].ids;
                for (uint64_t k = 0; k < sp[j].n; k++) {
                    wide |= src[k];
                    narrow[at + k] = (uint32_t)src[k];
                }
                at += sp[j].n;
            }
            const tm_span32 one{narrow.data(), nids};
            if (wide >> 32) reinterpret_cast<tm_spans32_cb>(p.fn)(p.ctx, TM_ESTATE, nullptr, 0, 0);
            else reinterpret_cast<tm_spans32_cb>(p.fn)(p.ctx, st, nids ? &one : nullptr, nids ? 1u : 0u, nids);
            return;
        }
        const tm_match_cb cb = reinterpret_cast<tm_match_cb>(p.fn);
        if (ns == 1) {  // zero-copy: one run of the id arena
            cb(p.ctx, st, sp[0].ids, (uint32_t)nids);
            return;
        }
        if (flat.size() < nids) flat.resize(nids);
        uint64_t at = 0;
        for (uint32_t j = 0; j < ns; j++) {
            std::memcpy(flat.data() + at, sp[j].ids, sp[j].n * 8);
            at += sp[j].n;
        }
        cb(p.ctx, st, nids ? flat.data() : nullptr, (uint32_t)nids);
    }
    // the same from spans of u32 ids (the engine's u32 id arena): a u32-span callback reads
    // them in place; the others get them widened into one list (one span)
    static void reply32(const Pending &p, int32_t st, const tm_span32 *sp, uint32_t ns, uint64_t nids) {
        thread_local std::vector<uint64_t> flat;
        if (p.kind == CB_SPANS32) {
            reinterpret_cast<tm_spans32_cb>(p.fn)(p.ctx, st, sp, ns, nids);
            return;
        }
        if (flat.size() < nids) flat.resize(nids);
        uint64_t at = 0;
        for (uint32_t j = 0; j < ns; j++) {
            const uint32_t *src = sp[j].ids;
            uint64_t *dst = flat.data() + at;
            for (uint64_t k = 0; k < sp[j].n; k++) dst[k] = src[k];
            at += sp[j].n;
        }
        const uint64_t *ids = nids ? flat.data() : nullptr;
        if (p.kind == CB_SPANS) {
            const tm_span one{ids, nids};
            reinterpret_cast<tm_spans_cb>(p.fn)(p.ctx, st, nids ? &one : nullptr, nids ? 1u : 0u, nids);
        } else {
            reinterpret_cast<tm_match_cb>(p.fn)(p.ctx, st, ids, (uint32_t)nids);
        }
    }
    // a failed window, or a publish with no ids
    static void reply_none(const Pending &p, int32_t st) {
        if (p.kind == CB_SPANS) reinterpret_cast<tm_spans_cb>(p.fn)(p.ctx, st, nullptr, 0, 0);
        else if (p.kind == CB_SPANS32) reinterpret_cast<tm_spans32_cb>(p.fn)(p.ctx, st, nullptr, 0, 0);
        else reinterpret_cast<tm_match_cb>(p.fn)(p.ctx, st, nullptr, 0);
    }

    // Submit -> callback-return latency, with the clock read once per 16 callbacks, AFTER them:
    // each of the 16 is overstated by at most the callbacks that follow it in its group, never
    // understated (round 4 read the clock before the group and left the callbacks out: advisor).
    // The stamp taken as a group starts serves publishes its callbacks re-submit (tl_clock_ns):
    // early, so their latency is overstated too.
    struct LatGroup {
        uint64_t t0[16];
        uint32_t n = 0;
        template <class Clock>
        void start(const Clock &clock) {
            if (!n) tl_clock_ns = clock();
        }
        template <class Clock>
        void done(uint64_t t, bool last, LatHist &H, const Clock &clock) {
            t0[n++] = t;
            if (n < 16 && !last) return;
            const uint64_t now = clock();
            for (uint32_t k = 0; k < n; k++) H.add(now > t0[k] ? now - t0[k] : 0);
            n = 0;
        }
    };

    void deliver_range(Slot &S, uint32_t lo, uint32_t hi, int rc, LatHist &H) {
        H.sync_gen(lat_gen.load(std::memory_order_acquire));
        LatGroup G;
        auto clock = [] { return now_ns(); };
        if (S.runs && rc >= 0) {
            const tm_span *spans = S.h_spans.as<tm_span>();
            const uint32_t *so = S.h_soff.as<uint32_t>(), *sc = S.h_scnt.as<uint32_t>(), *kc = S.h_kcnt.as<uint32_t>();
            const int32_t *stv = S.h_status.as<int32_t>();
            // the id arena is read at random places (a span's start, an inline key's id): start
            // the loads of a few publishes ahead so the replies do not wait on each miss in turn
            const uint32_t PF = pf_pubs;
            auto prefetch = [&](uint32_t i) {
                const uint32_t b = so[i], e = b + std::min<uint32_t>(sc[i], 4);
                if (!pf_lines) {
                    for (uint32_t j = b; j < e; j++) __builtin_prefetch(spans[j].ids);
                    return;
                }
                // every line of the reply's first spans, up to pf_lines lines
                uint32_t left = pf_lines;
                for (uint32_t j = b; j < e && left; j++) {
                    const char *p = (const char *)spans[j].ids;
                    const char *end = p + spans[j].n * S.runs_w;
                    for (p = (const char *)((uintptr_t)p & ~(uintptr_t)63); p < end && left; p += 64, left--)
                        __builtin_prefetch(p);
                }
            };
            for (uint32_t i = lo; i < std::min(hi, lo + PF); i++) prefetch(i);
            for (uint32_t i = lo; i < hi; i++) {
                const Pending &p = S.pubs[i];
                if (i + 8 < hi) __builtin_prefetch(S.pubs[i + 8].ctx);
                if (i + PF < hi) prefetch(i + PF);
                G.start(clock);
                const uint64_t t0 = p.t0;
                const int32_t st = stv[i];
                if (st != TM_TOPIC_OK) reply_none(p, st);
                else if (S.runs_w == 4) reply32(p, st, reinterpret_cast<const tm_span32 *>(spans) + so[i], sc[i], kc[i]);
                else reply(p, st, spans + so[i], sc[i], kc[i]);
                G.done(t0, i + 1 == hi, H, clock);
            }
            tl_clock_ns = 0;
            return;
        }
        thread_local std::vector<uint64_t> wide;  // a narrowed window's ids, one publish at a time
        const uint32_t *ids32 = S.narrow ? reinterpret_cast<const uint32_t *>(S.v.ids) : nullptr;
        for (uint32_t i = lo; i < hi; i++) {
            const Pending &p = S.pubs[i];
            if (i + 8 < hi) __builtin_prefetch(S.pubs[i + 8].ctx);  // the caller's per-publish state
            G.start(clock);
            const uint64_t t0 = p.t0;
            if (rc < 0) {
                reply_none(p, rc);
            } else if (p.kind == CB_SPANS32) {  // u32 ids: in place when they crossed as u32
                const int32_t st = S.v.status[i];
                const uint32_t c = st == TM_TOPIC_OK ? S.v.cnt[i] : 0;
                const tm_spans32_cb cb = reinterpret_cast<tm_spans32_cb>(p.fn);
                if (!c) {
                    cb(p.ctx, st, nullptr, 0, 0);
                } else if (ids32) {
                    const tm_span32 one{ids32 + S.v.off[i], c};
                    cb(p.ctx, st, &one, 1, c);
                } else {
                    cb(p.ctx, TM_ESTATE, nullptr, 0, 0);  // u64 ids (some id needs 64 bits)
                }
            } else {
                const int32_t st = S.v.status[i];
                const uint32_t c = st == TM_TOPIC_OK ? S.v.cnt[i] : 0;
                const uint64_t *ids = nullptr;
                if (S.v.ids && c) {
                    if (ids32) {
                        if (wide.size() < c) wide.resize(c);
                        const uint32_t *src = ids32 + S.v.off[i];
                        for (uint32_t k = 0; k < c; k++) wide[k] = src[k];
                        ids = wide.data();
                    } else {
                        ids = S.v.ids + S.v.off[i];
                    }
                }
                if (p.kind == CB_SPANS) {
                    const tm_span one{ids, c};
                    reinterpret_cast<tm_spans_cb>(p.fn)(p.ctx, st, c ? &one : nullptr, c ? 1u : 0u, c);
                } else {
                    reinterpret_cast<tm_match_cb>(p.fn)(p.ctx, st, ids, c);
                }
            }
            G.done(t0, i + 1 == hi, H, clock);
        }
        tl_clock_ns = 0;
    }

    static constexpr int SPIN = 256;  // polls (a few microseconds) before sleeping: the CPUs are a quota
    static constexpr uint32_t MIN_RANGE = 256;  // publishes: smaller ranges are not worth a hand-off

    // Queue window S's delivery: each chunk cut into ranges, about one per delivery thread.
    void post_delivery(uint32_t si) {
        Slot &S = slot[si];
        const uint32_t nthreads = (uint32_t)workers.size();
        std::vector<Work> ws;
        for (uint32_t j = 0; j < S.nchunk; j++) {
            const uint32_t lo = S.chunk_lo[j], hi = S.chunk_lo[j + 1];
            S.chunk_ready[j].store(S.cev_wait ? 0 : 1, std::memory_order_relaxed);
            if (hi <= lo) continue;
            const uint32_t parts =
                std::max<uint32_t>(1, std::min<uint32_t>(nthreads * ranges_per_thread, (hi - lo) / MIN_RANGE));
            for (uint32_t k = 0; k < parts; k++)
                ws.push_back(Work{si, j, lo + (uint32_t)((uint64_t)(hi - lo) * k / parts),
                                  lo + (uint32_t)((uint64_t)(hi - lo) * (k + 1) / parts)});
        }
        if (ws.empty()) {
            free_slot(S);
            return;
        }
        S.parts_left.store((uint32_t)ws.size(), std::memory_order_release);
        {
            std::lock_guard<std::mutex> g(work_mu);
            work.insert(work.end(), ws.begin(), ws.end());
            work_n.store((uint32_t)work.size(), std::memory_order_release);
        }
        if (sleepers.load()) work_cv.notify_all();
    }

    // the last TM_BATCHER_WINDOWS windows' stage stamps (tm_batcher_windows)
    std::unique_ptr<tm_batcher_window[]> wins{new tm_batcher_window[TM_BATCHER_WINDOWS]};
    std::atomic<uint64_t> win_next{0}, win_first{0};  // ring positions; win_first: the reset's
    std::mutex win_mu;  // a record is written and copied whole (tm_batcher_windows reads no torn entry)
    void trace_window(Slot &S) {
        if (!S.n) return;
        std::lock_guard<std::mutex> g(win_mu);
        const uint64_t i = win_next.fetch_add(1, std::memory_order_relaxed);
        tm_batcher_window &w = wins[i % TM_BATCHER_WINDOWS];
        w.n = S.n;
        w.flags = S.wflags | (S.runs ? TM_WIN_RUNS : 0u) | (S.rc < 0 ? TM_WIN_FAILED : 0u);
        w.t_oldest = S.t_old;
        w.t_cut = S.t_cut;
        w.t_queued = S.t_queued;
        w.t_gpu = S.t_gpu ? S.t_gpu : S.t_queued;
        w.t_ready = S.t_done;
        w.t_deliver = S.t_deliver.load(std::memory_order_relaxed);
        w.t_done = now_ns();
        w.epoch = S.epoch;
        w.t_slot = S.t_slot;
        w.cut_cpu_us = S.cut_cpu_us;
        w.cut_ivcsw = (uint16_t)std::min<uint32_t>(S.cut_ivcsw, 0xFFFF);
        w.wait_ivcsw = (uint16_t)std::min<uint32_t>(S.wait_ivcsw, 0xFFFF);
        w.del_cpu_us = (uint32_t)(S.del_cpu_ns.load(std::memory_order_relaxed) / 1000);
        // rounded up: a window delivered in under 1 us still records its (nonzero) wall time
        w.del_wall_us = (uint32_t)((S.del_wall_ns.load(std::memory_order_relaxed) + 999) / 1000);
        w.del_ivcsw = S.del_ivcsw.load(std::memory_order_relaxed);
        w.reserved = 0;
    }
    void free_slot(Slot &S) {
        trace_window(S);
        if (S.leased) {  // the window's spans are delivered: a commit may change the id arena now
            S.leased = false;
            tmx_lease_drop(eng);
        }
        {
            std::lock_guard<std::mutex> g(slot_mu);
            S.state = Slot::FREE;
        }
        slot_cv.notify_all();
    }

    // the next range, or false once the queue is closed and empty
    bool next_work(Work &w) {
        for (int spins = 0; spins < SPIN && work_n.load(std::memory_order_acquire) == 0; spins++)
            __builtin_ia32_pause();
        std::unique_lock<std::mutex> lk(work_mu);
        if (work.empty()) {
            sleepers.fetch_add(1);
            work_cv.wait(lk, [&] { return !work.empty() || work_closed; });
            sleepers.fetch_sub(1);
            if (work.empty()) return false;
        }
        w = work.front();
        work.pop_front();
        work_n.store((uint32_t)work.size(), std::memory_order_release);
        return true;
    }

    void worker_loop(uint32_t me) {
        LatHist &H = lat[me];
        tl_delivering = 1;
        // below the cutter and the completer: on a full CPU share a woken cutter/completer
        // preempts a delivery thread instead of waiting out its time slice (the latency tail)
        if (deliver_nice > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), deliver_nice);
        Work w;
        while (next_work(w)) {
            Slot &S = slot[w.slot];
            int rc = S.rc;
            if (!S.chunk_ready[w.chunk].load(std::memory_order_acquire)) {
                // several threads may wait on one chunk's copy at once; each returns when it lands
                const uint64_t t0 = now_ns();
                if (hipEventSynchronize(S.cev[w.chunk]) != hipSuccess) rc = TM_EDEVICE;
                else S.chunk_ready[w.chunk].store(1, std::memory_order_release);
                ns_copy.fetch_add(now_ns() - t0, std::memory_order_relaxed);  // waited on PCIe
            }
            const ThreadUse u0 = thread_use();
            const uint64_t td0 = now_ns();
            uint64_t z = 0;
            S.t_deliver.compare_exchange_strong(z, td0, std::memory_order_relaxed);
            tl_window_leased = S.leased ? 1 : 0;
            deliver_range(S, w.lo, w.hi, rc, H);
            tl_window_leased = 0;
            const uint64_t td1 = now_ns();
            ns_del.fetch_add(td1 - td0, std::memory_order_relaxed);
            const ThreadUse u1 = thread_use();
            S.del_cpu_ns.fetch_add(u1.cpu_ns - u0.cpu_ns, std::memory_order_relaxed);
            S.del_wall_ns.fetch_add(td1 - td0, std::memory_order_relaxed);
            S.del_ivcsw.fetch_add((uint32_t)(u1.ivcsw - u0.ivcsw), std::memory_order_relaxed);
            if (S.parts_left.fetch_sub(1, std::memory_order_acq_rel) == 1) free_slot(S);
        }
    }

    // ------------------------------------------------------------------ threads
    void cutter_loop() {
        uint32_t next = 0;
        ThreadUse u_prev = thread_use();
        for (;;) {
            // a window: something queued, and (max_batch queued, or the oldest waited
            // max_wait_us, or stopping)
            uint64_t t_old;
            {
                std::unique_lock<std::mutex> lk(wake_mu);
                bool quit = false;
                for (;;) {
                    const bool stop = stopping.load();  // before looking at the shards
                    t_old = oldest_t0();
                    if (t_old != ~0ull) break;
                    if (stop) {
                        quit = true;
                        break;
                    }
                    // idle is published before the check above repeats under wake_mu, and a
                    // submitter notifies under wake_mu: no wakeup is lost
                    cutter_idle.store(1);
                    if (oldest_t0() == ~0ull && !stopping.load()) wake_cv.wait(lk);
                    cutter_idle.store(0);
                }
                if (quit) break;
            }
            const uint64_t deadline = t_old + (uint64_t)cfg.max_wait_us * 1000;
            for (;;) {
                if (stopping.load() || queued_now() >= cfg.max_batch) break;
                const uint64_t t = now_ns();
                if (t >= deadline) break;
                // polled: a submitter does not signal a filling window (that would put one
                // shared write on every publish); the wait is bounded by the deadline anyway
                const uint64_t nap = std::min<uint64_t>(deadline - t, 20000);
                std::this_thread::sleep_for(std::chrono::nanoseconds(nap));
            }
            // a free slot (slots complete in order, so the next one in turn)
            Slot &S = slot[next];
            const uint64_t t_slot = now_ns();
            {
                std::unique_lock<std::mutex> lk(slot_mu);
                slot_cv.wait(lk, [&] { return S.state == Slot::FREE; });
                S.state = Slot::BUSY;
            }
            const ThreadUse u0 = thread_use();
            const uint64_t tc0 = now_ns();
            S.t_slot = t_slot;
            S.wait_ivcsw = (uint32_t)(u0.ivcsw - u_prev.ivcsw);
            S.del_cpu_ns.store(0, std::memory_order_relaxed);
            S.del_wall_ns.store(0, std::memory_order_relaxed);
            S.del_ivcsw.store(0, std::memory_order_relaxed);
            S.runs = false;
            S.wflags = 0;
            S.t_gpu = 0;
            S.t_deliver.store(0, std::memory_order_relaxed);
            S.t_cut = tc0;
            S.rc = take_window(S);
            S.mode = cfg.mode;
            S.t_enq = now_ns();
            ns_cut.fetch_add(S.t_enq - tc0, std::memory_order_relaxed);
            if (S.rc == TM_OK && S.n) {
                if (eng) {
                    S.runs = runs_ok && S.mode == TM_MATCH_ALL;
                    if (S.runs) {  // leases come before any engine lock (include/emqx_tm.h)
                        tmx_lease_take(eng);
                        S.leased = true;
                    }
                    std::lock_guard<std::mutex> g(eng_mu);
                    S.rc = enqueue(S);
                    report("enqueue", S.rc);
                    if (S.rc == TM_ESTATE && S.mode == TM_MATCH_UNIQUE) S.rc = run_host(S);
                } else {
                    // custom backend: synchronous; its view lives until its next call, which
                    // the slot ordering below delays until this window is delivered
                    std::lock_guard<std::mutex> g(eng_mu);
                    S.rc = fn(backend, S.h_bytes.as<uint8_t>(), S.h_off.as<uint32_t>(), S.n, S.mode, &S.v);
                    S.host_done = true;
                    S.narrow = false;
                }
            }
            S.t_queued = now_ns();
            u_prev = thread_use();
            S.cut_cpu_us = (uint32_t)((u_prev.cpu_ns - u0.cpu_ns) / 1000);
            S.cut_ivcsw = (uint32_t)(u_prev.ivcsw - u0.ivcsw);
            S.epoch = eng ? tmx_engine_epoch(eng) : 0;
            ns_enq.fetch_add(S.t_queued - S.t_enq, std::memory_order_relaxed);
            {
                std::lock_guard<std::mutex> g(slot_mu);
                fifo.push_back(next);
            }
            slot_cv.notify_all();
            // a custom backend's view must be delivered before the next call: one slot at a time
            next = eng ? (next + 1) % nslot : next;
        }
        {
            std::lock_guard<std::mutex> g(slot_mu);
            cutter_done = true;
        }
        slot_cv.notify_all();
    }

    // stage 2: the GPU part is done -> ids over PCIe (copy stream) -> to the delivery stage
    void completer_loop() {
        for (;;) {
            uint32_t si;
            {
                std::unique_lock<std::mutex> lk(slot_mu);
                slot_cv.wait(lk, [&] { return !fifo.empty() || cutter_done; });
                if (fifo.empty()) break;
                si = fifo.front();
                fifo.pop_front();
            }
            Slot &S = slot[si];
            S.nchunk = 1;  // one chunk, nothing to wait for, unless complete() streams the ids
            S.chunk_lo[0] = 0;
            S.chunk_lo[1] = S.n;
            S.cev_wait = false;
            if (S.rc == TM_OK && S.n && eng) {
                S.rc = complete(S);
                report("completion", S.rc);
            }
            S.t_done = now_ns();
            if (S.n) {
                std::lock_guard<std::mutex> g(st_mu);  // counted before the callbacks
                n_batches++;
                n_pub += S.n;
                max_seen = std::max<uint64_t>(max_seen, S.n);
                backend_ns += S.t_done - S.t_enq;
            }
            post_delivery(si);
        }
        {
            std::lock_guard<std::mutex> g(work_mu);
            work_closed = true;
        }
        work_cv.notify_all();
    }

    int start(const tm_batcher_config *c) {
        if (c) cfg = *c;
        if (cfg.max_batch == 0) cfg.max_batch = 65536;
        if (cfg.max_wait_us == 0) cfg.max_wait_us = 200;
        if (cfg.mode > TM_MATCH_AGGRE) return TM_EINVAL;
        n_delivery = cfg.delivery_threads ? cfg.delivery_threads : 4;
        if (n_delivery > 64) return TM_EINVAL;
        lat.reset(new (std::nothrow) LatHist[n_delivery]);
        if (!lat) return TM_ENOMEM;
        t_window = std::chrono::steady_clock::now();
        (void)now_ns();  // calibrate the clock before the first publish is stamped
        if (const char *e = std::getenv("EMQX_TM_NSLOT")) nslot = std::max(2u, std::min(NSLOT_MAX, (uint32_t)std::atoi(e)));
        if (const char *e = std::getenv("EMQX_TM_PF_PUBS")) pf_pubs = std::max(1u, std::min(64u, (uint32_t)std::atoi(e)));
        if (const char *e = std::getenv("EMQX_TM_PF_LINES")) pf_lines = std::min(256u, (uint32_t)std::atoi(e));
        if (const char *e = std::getenv("EMQX_TM_RUNS_IDW")) runs_w = std::atoi(e) == 4 ? 4u : 8u;
        if (const char *e = std::getenv("EMQX_TM_DELIVERY_NICE")) deliver_nice = std::max(0, std::min(19, std::atoi(e)));
        if (const char *e = std::getenv("EMQX_TM_RANGES_PER_THREAD"))
            ranges_per_thread = (uint32_t)std::max(1, std::min(16, std::atoi(e)));
        if (const char *e = std::getenv("EMQX_TM_BATCHER_HINTS")) hints = std::atoi(e) != 0;
        if (!eng)
            for (Slot &S : slot)
                for (HBuf *h : {&S.h_bytes, &S.h_off, &S.h_off_out, &S.h_status, &S.h_cnt, &S.h_ids, &S.h_ctl})
                    h->pinned = false;
        if (eng) {
            runs_ok = cfg.transport != TM_TRANSPORT_IDS && tmx_engine_runs_ok(eng);
            if (cfg.transport == TM_TRANSPORT_RUNS && !runs_ok) return TM_ESTATE;
            device = tmx_engine_device(eng);
            if (hipSetDevice(device) != hipSuccess ||
                hipStreamCreateWithFlags(&s_comps[0], hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithFlags(&s_comps[1], hipStreamNonBlocking) != hipSuccess ||
                hipStreamCreateWithFlags(&s_copy, hipStreamNonBlocking) != hipSuccess)
                return TM_EDEVICE;
            // EMQX_TM_STREAMS=1: every window on one stream and one buffer set (A/B runs)
            const char *es = std::getenv("EMQX_TM_STREAMS");
            const uint32_t nstreams = es && std::atoi(es) == 1 ? 1u : 2u;
            // the engine's buffer sets sized for max_batch windows of up to 128 B per topic
            // now, not by the first window that outgrows them (later growth stays possible)
            const char *er = std::getenv("EMQX_TM_BATCHER_RESERVE");  // development: 0 skips it
            if (!er || std::atoi(er) != 0)
                for (uint32_t st = 0; st < nstreams; st++)
                    if (tmx_engine_reserve_batch(eng, st, cfg.max_batch, (uint64_t)cfg.max_batch * 128) != TM_OK) {
                        // not fatal: the buffers grow to the windows' demand instead
                        std::fprintf(stderr, "tm_batcher: reserving buffer set %u failed (%s); growing lazily\n", st,
                                     tm_last_error(eng));
                        (void)hipGetLastError();
                        break;
                    }
            for (uint32_t i = 0; i < NSLOT_MAX; i++) {
                slot[i].set = nstreams == 2 ? (i & 1u) : 0u;
                for (hipEvent_t &e : slot[i].cev)
                    if (hipEventCreateWithFlags(&e, EV_FLAGS) != hipSuccess) return TM_EDEVICE;
            }
        }
        try {
            for (uint32_t i = 0; i < n_delivery; i++) workers.emplace_back([this, i] { worker_loop(i); });
            completer = std::thread([this] { completer_loop(); });
            cutter = std::thread([this] { cutter_loop(); });
        } catch (...) {
            stop();
            return TM_ENOMEM;
        }
        return TM_OK;
    }

    void stop() {
        {
            std::lock_guard<std::mutex> g(wake_mu);
            stopping = true;
        }
        wake_cv.notify_all();
        if (cutter.joinable()) cutter.join();
        else {
            std::lock_guard<std::mutex> g(slot_mu);
            cutter_done = true;
        }
        slot_cv.notify_all();
        if (completer.joinable()) completer.join();
        {
            std::lock_guard<std::mutex> g(work_mu);
            work_closed = true;
        }
        work_cv.notify_all();
        for (std::thread &t : workers)  // they drain the queue before they see it closed
            if (t.joinable()) t.join();
        if (eng) {
            (void)hipSetDevice(device);
            for (Slot &S : slot) {
                if (S.ev) (void)hipEventDestroy(S.ev);
                S.ev = nullptr;
                for (hipEvent_t &e : S.cev)
                    if (e) {
                        (void)hipEventDestroy(e);
                        e = nullptr;
                    }
            }
            // the engine remembers the streams its batches ran on: make it forget ours first
            for (hipStream_t sc : s_comps)
                if (sc) tmx_engine_forget_stream(eng, sc);
            if (s_copy) tmx_engine_forget_stream(eng, s_copy);
            for (hipStream_t &sc : s_comps)
                if (sc) {
                    (void)hipStreamDestroy(sc);
                    sc = nullptr;
                }
            if (s_copy) (void)hipStreamDestroy(s_copy);
            s_copy = nullptr;
        }
    }
};

// development (EMQX_TM_SEGV_TRACE=1): a crash on any thread prints that thread's native
// backtrace to stderr (addresses map to source lines with addr2line on the same build)
static void segv_trace(int sig) {
    void *fr[64];
    const int n = backtrace(fr, 64);
    const char msg[] = "\n[emqx_tm] fatal signal, native backtrace:\n";
    (void)!write(2, msg, sizeof msg - 1);
    backtrace_symbols_fd(fr, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

extern "C" {

static int batcher_new(tm_engine *eng, tm_batch_fn fn, void *backend, const tm_batcher_config *cfg,
                       tm_batcher **out) {
    if (const char *e = std::getenv("EMQX_TM_SEGV_TRACE"))
        if (std::atoi(e)) {
            signal(SIGSEGV, segv_trace);
            signal(SIGBUS, segv_trace);
        }
    tm_batcher *b = new (std::nothrow) tm_batcher();
    if (!b) return TM_ENOMEM;
    b->eng = eng;
    b->fn = fn;
    b->backend = backend;
    int rc = b->start(cfg);
    if (rc) {
        b->stop();  // streams and events created before the failure (no thread runs yet)
        delete b;
        return rc;
    }
    *out = b;
    return TM_OK;
}

int tm_batcher_create_fn(tm_batch_fn fn, void *backend, const tm_batcher_config *cfg, tm_batcher **out) {
    if (!fn || !out) return TM_EINVAL;
    *out = nullptr;
    return batcher_new(nullptr, fn, backend, cfg, out);
}

int tm_batcher_create(tm_engine *eng, const tm_batcher_config *cfg, tm_batcher **out) {
    if (!eng || !out) return TM_EINVAL;
    *out = nullptr;
    return batcher_new(eng, nullptr, nullptr, cfg, out);
}

void tm_batcher_destroy(tm_batcher *b) {
    if (!b) return;
    b->stop();  // drains: every queued publish is matched and called back first
    delete b;
}

int tm_batcher_submit(tm_batcher *b, const uint8_t *topic, uint32_t len, tm_match_cb cb, void *ctx) {
    if (!b || !cb || (len && !topic) || len > 65535) return TM_EINVAL;
    return b->submit(topic, len, CB_IDS, reinterpret_cast<void (*)()>(cb), ctx);
}

int tm_batcher_submit_spans(tm_batcher *b, const uint8_t *topic, uint32_t len, tm_spans_cb cb, void *ctx) {
    if (!b || !cb || (len && !topic) || len > 65535) return TM_EINVAL;
    return b->submit(topic, len, CB_SPANS, reinterpret_cast<void (*)()>(cb), ctx);
}

int tm_batcher_submit_spans32(tm_batcher *b, const uint8_t *topic, uint32_t len, tm_spans32_cb cb, void *ctx) {
    if (!b || !cb || (len && !topic) || len > 65535) return TM_EINVAL;
    return b->submit(topic, len, CB_SPANS32, reinterpret_cast<void (*)()>(cb), ctx);
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

// The engine is safe under concurrent callers (include/emqx_tm.h "Threading"): writes go
// straight to it, and its commit publishes only between the windows' device work (the
// windows already queued finish on the old epoch; the next one sees the new).  These two are
// kept for callers that hold only the batcher.
int tm_batcher_apply(tm_batcher *b, const tm_op *ops, size_t n) {
    if (!b) return TM_EINVAL;
    if (!b->eng) return TM_ESTATE;
    return tm_apply(b->eng, ops, n);
}

int tm_batcher_commit(tm_batcher *b, uint64_t *epoch_out) {
    if (!b) return TM_EINVAL;
    if (!b->eng) return TM_ESTATE;
    return tm_commit_epoch(b->eng, epoch_out);
}

int tm_batcher_stats_get(tm_batcher *b, tm_batcher_stats *out) {
    if (!b || !out) return TM_EINVAL;
    {
        std::lock_guard<std::mutex> g(b->st_mu);
        out->batches = b->n_batches;
        out->publishes = b->n_pub;
        out->max_batch_seen = b->max_seen;
        out->backend_us = b->backend_ns / 1000;
        out->cut_us = b->ns_cut / 1000;
        out->enqueue_us = b->ns_enq / 1000;
        out->gpu_wait_us = b->ns_gpu / 1000;
        const uint64_t nt = std::max<size_t>(1, b->workers.size());  // per delivery thread
        out->copy_us = b->ns_copy / 1000 / nt;
        out->deliver_us = b->ns_del / 1000 / nt;
        out->window_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - b->t_window).count();
    }
    // every publish delivered since the last reset: the delivery threads' histograms of this
    // generation (a thread that has not delivered since the reset holds none of its publishes)
    const uint64_t g = b->lat_gen.load(std::memory_order_acquire);
    std::vector<uint64_t> hist(LAT_NB, 0);
    uint64_t n = 0, mx = 0;
    double sum = 0;
    for (uint32_t t = 0; t < b->n_delivery; t++) {
        const LatHist &H = b->lat[t];
        if (H.gen.load(std::memory_order_acquire) != g) continue;
        for (uint32_t k = 0; k < LAT_NB; k++) hist[k] += H.b[k].load(std::memory_order_relaxed);
        n += H.n.load(std::memory_order_relaxed);
        sum += (double)H.sum_ns.load(std::memory_order_relaxed);
        mx = std::max<uint64_t>(mx, H.max_ns.load(std::memory_order_relaxed));
    }
    uint64_t hn = 0;
    for (uint64_t x : hist) hn += x;  // read after n: a record in flight may be half counted
    out->lat_count = hn;
    out->lat_mean_us = n ? sum / (double)n / 1000.0 : 0;
    out->lat_max_us = mx / 1000.0;
    auto pct = [&](double q) {
        if (!hn) return 0.0;
        const uint64_t want = std::min<uint64_t>(hn - 1, (uint64_t)(q * (double)(hn - 1) + 0.5));
        uint64_t seen = 0;
        for (uint32_t k = 0; k < LAT_NB; k++) {
            seen += hist[k];
            if (seen > want) return lat_bucket_mid(k) / 1000.0;
        }
        return mx / 1000.0;
    };
    out->lat_p50_us = pct(0.50);
    out->lat_p99_us = pct(0.99);
    out->lat_p999_us = pct(0.999);
    return TM_OK;
}

int tm_batcher_stats_reset(tm_batcher *b) {
    if (!b) return TM_EINVAL;
    std::lock_guard<std::mutex> g(b->st_mu);
    b->lat_gen.fetch_add(1, std::memory_order_acq_rel);
    b->t_window = std::chrono::steady_clock::now();
    b->win_first.store(b->win_next.load(std::memory_order_relaxed), std::memory_order_relaxed);
    return TM_OK;
}

int tm_batcher_windows(tm_batcher *b, tm_batcher_window *out, uint32_t cap, uint32_t *n_out) {
    if (!b || !n_out || (cap && !out)) return TM_EINVAL;
    std::lock_guard<std::mutex> g(b->win_mu);
    const uint64_t hi = b->win_next.load(std::memory_order_acquire);
    uint64_t lo = std::max(b->win_first.load(std::memory_order_relaxed),
                           hi > TM_BATCHER_WINDOWS ? hi - TM_BATCHER_WINDOWS : 0);
    if (hi - lo > cap) lo = hi - cap;
    for (uint64_t i = lo; i < hi; i++) out[i - lo] = b->wins[i % TM_BATCHER_WINDOWS];
    *n_out = (uint32_t)(hi - lo);
    return TM_OK;
}

}  // extern "C"
