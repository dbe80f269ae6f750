// engine.cpp — host side of the MI355X topic-matching engine and the C-ABI
// declared in include/emqx_tm.h.
//
// What the reference does on this side of the path, and what replaces it:
//   * emqx_topic_index:insert/4 / delete/3 (apps/emqx/src/emqx_topic_index.erl:53-62) write one
//     {Words | Binary, {ID}} key into an ETS ordered_set (key shape from
//     emqx_trie_search:make_key/2, apps/emqx/src/emqx_trie_search.erl:115-128).
//     Here tm_apply stages the op and tm_commit_epoch folds a whole batch of ops into
//     the frozen trie (one delta epoch), like emqx_router_syncer batches route ops
//     (apps/emqx/src/emqx_router_syncer.erl:244-280,381-401).
//   * emqx_topic_index:matches/3 / emqx_router:match_routes/1 run the ETS seek walk per
//     topic (apps/emqx/src/emqx_trie_search.erl:192-389).  Here tm_match_batch ships a
//     whole batch of topics to the GPU kernels in match_kernels.hip.
//
// Host state is the source of truth; the device copy is a derived cache rebuilt
// from it (SURVEY.md §5 checkpoint/resume).
#include <hip/hip_runtime.h>

#include <sched.h>
#include <sys/mman.h>
#include <sys/resource.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <unordered_map>
#include <unordered_set>
#include <string>
#include <thread>
#include <vector>

#include "../../include/emqx_tm.h"
#include "copy_api.h"
#include "device_api.h"
#include "filter_api.h"
#include "image_api.h"
#include "layout.h"

using namespace tmx;

// batcher.cpp, library-internal: nonzero on an aggregator delivery thread (inside a callback),
// and while that callback's window holds a read lease on the host id arena
extern "C" int tmx_in_delivery(void);
extern "C" int tmx_in_leased_delivery(void);

namespace {

// key kinds (where the key hangs in the trie)
enum : uint8_t {
    K_FREE = 0,
    K_EXACT_BIN = 1,    // {Binary, {ID}}: filter without wildcards, binary form
    K_EXACT_WORDS = 2,  // {Words, {ID}}: same filter given as a word list
    K_WILD = 3,         // wildcard filter without a final '#': ends at the node
    K_HASH = 4,         // "P/#": lives in P's hash list
    K_DEAD = 5,         // '#' before the last level: can never match
};
inline bool is_term_kind(uint8_t k) { return k == K_EXACT_BIN || k == K_EXACT_WORDS || k == K_WILD; }

struct KeyRec {
    uint32_t node;  // terminal node (NONE for K_DEAD)
    uint8_t kind;
    uint8_t _p[3];  // _p[0]: KR_MULTI once another live key carries the same id
    uint64_t id;
};

struct Delta {
    uint32_t node;
    uint32_t key;
    uint8_t hash;  // 1: hash list, 0: term list
    uint8_t add;   // 1 add, 0 delete
};

struct StagedOp {
    uint32_t op, flags;
    uint64_t id;
    uint64_t off;  // filter bytes in tm_engine::stage_bytes
    uint32_t len;
};

// The host master copy's big tables (edge slots, node arrays, key records, key set, ids,
// arena) are read at random places by every commit: on 4-KiB pages nearly each such read also
// misses the TLB.  Allocations of 4 MiB or more are mapped 2-MiB aligned and advised as
// transparent huge pages (the hosts here run THP in "madvise" mode).
template <class T>
struct HugeAlloc {
    using value_type = T;
    static constexpr size_t HUGE = 2u << 20, MIN = 4u << 20;
    HugeAlloc() = default;
    template <class U>
    HugeAlloc(const HugeAlloc<U> &) {}
    static size_t span(size_t bytes) { return (bytes + HUGE - 1) & ~(HUGE - 1); }
    T *allocate(size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < MIN) return static_cast<T *>(::operator new(bytes));
        const size_t len = span(bytes);
        void *p = mmap(nullptr, len + HUGE, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        if (p == MAP_FAILED) throw std::bad_alloc();
        const uintptr_t a = ((uintptr_t)p + HUGE - 1) & ~(uintptr_t)(HUGE - 1);
        if (a > (uintptr_t)p) munmap(p, a - (uintptr_t)p);                 // unaligned head
        munmap((void *)(a + len), (uintptr_t)p + len + HUGE - (a + len));  // the rest of the tail
        (void)madvise((void *)a, len, MADV_HUGEPAGE);
        return reinterpret_cast<T *>(a);
    }
    void deallocate(T *p, size_t n) {
        const size_t bytes = n * sizeof(T);
        if (bytes < MIN) ::operator delete(p);
        else munmap(p, span(bytes));
    }
    template <class U>
    bool operator==(const HugeAlloc<U> &) const { return true; }
    template <class U>
    bool operator!=(const HugeAlloc<U> &) const { return false; }
};
template <class T>
using hvec = std::vector<T, HugeAlloc<T>>;

// TM_BOUNDS=1 (debug build, libemqx_tm_bounds.so): every device buffer carries
// a canary tail of BND_CANARY bytes past its capacity, and a registry of the live ones lets
// tm_engine::bounds_check() find any launch that wrote past a buffer's end; the kernels check
// their indices against the buffers' real capacities (device_api.h BI()).
#ifndef TM_BOUNDS
#define TM_BOUNDS 0
#endif
constexpr size_t BND_CANARY = TM_BOUNDS ? 4096 : 0;
[[maybe_unused]] constexpr uint8_t BND_FILL = 0xA5;
#if TM_BOUNDS
// One per process (every engine's buffers, every device's bounds record, what was found): a
// test runner checks the whole process after each test (tm_debug_bounds with a null engine).
struct BndRegistry {
    std::mutex m;
    std::unordered_map<void *, size_t> live;  // pointer -> capacity (the canary follows it)
    unsigned long long *rec[64] = {};         // per device: {count, file << 24 | line, index, capacity}
    uint64_t hits = 0;
    std::string msg;  // the first findings
};
static BndRegistry &bnd_registry() {
    static BndRegistry *r = new BndRegistry();  // never destroyed: buffers outlive static teardown
    return *r;
}
#endif

struct DevBuf {
    void *p = nullptr;
    size_t cap = 0;
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        release();
        size_t want = bytes ? bytes : 64;
        hipError_t e = hipMalloc(&p, want + BND_CANARY);
        if (e == hipSuccess) {
            cap = want;
            // EMQX_TM_POISON=1 (test aid): every new device buffer starts as 0xA7 bytes, so a read
            // of memory nothing wrote shows up as garbage, not as the zeros a fresh page holds
            static const bool poison = getenv("EMQX_TM_POISON") && atoi(getenv("EMQX_TM_POISON")) != 0;
            if (poison && (e = hipMemset(p, 0xA7, want)) == hipSuccess) e = hipStreamSynchronize(nullptr);
#if TM_BOUNDS
            e = hipMemset(static_cast<uint8_t *>(p) + want, BND_FILL, BND_CANARY);
            std::lock_guard<std::mutex> g(bnd_registry().m);
            bnd_registry().live[p] = want;
#endif
        } else {
            p = nullptr;
        }
        return e;
    }
    void release() {
#if TM_BOUNDS
        if (p) {  // freed under the lock: a canary scan never reads a buffer being freed
            std::lock_guard<std::mutex> g(bnd_registry().m);
            bnd_registry().live.erase(p);
            (void)hipFree(p);
            p = nullptr;
        }
#endif
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

struct PinBuf {
    void *p = nullptr;
    size_t cap = 0;
    void *dev = nullptr;  // the buffer's device address (kernels write results into it), or null
    hipError_t ensure(size_t bytes) {
        if (bytes <= cap && p) return hipSuccess;
        if (p) (void)hipHostFree(p);
        p = nullptr;
        dev = nullptr;
        cap = 0;
        size_t want = std::max<size_t>(bytes, 4096);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) {
            cap = want;
            if (hipHostGetDevicePointer(&dev, p, 0) != hipSuccess) {
                dev = nullptr;
                (void)hipGetLastError();  // not sticky: the DMA path is used instead
            }
        }
        return e;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        dev = nullptr;
        cap = 0;
    }
    template <class T> T *as() const { return static_cast<T *>(p); }
};

// n u32 words from device memory into a pinned buffer at word `at`.  Large copies are written
// by a kernel through the buffer's device address (launch_copy_to_host: ~45 GB/s where the
// DMA engine path ran at ~27 GB/s on repeated 570 MB copies), small ones by DMA.
constexpr uint64_t D2H_KERNEL_MIN_WORDS = 1u << 18;
static hipError_t d2h_words(const PinBuf &h, uint64_t at, const void *src, uint64_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    if (h.dev && n >= D2H_KERNEL_MIN_WORDS)
        return launch_copy_to_host(static_cast<uint32_t *>(h.dev) + at, static_cast<const uint32_t *>(src), n, s);
    return hipMemcpyAsync(h.as<uint32_t>() + at, src, n * 4, hipMemcpyDeviceToHost, s);
}

// One set of per-batch device buffers and the counters sized from its batches' demand.
struct BatchBufs {
    DevBuf d_bytes, d_off, d_outoff, d_outcnt, d_status, d_keys, d_slow_list, d_scr_w, d_scr_s, d_seg_pool, d_fr_pool,
        d_wave_chunks;
    DevBuf d_ukeys, d_ucnt;     // UNIQUE / AGGRE: reducer scratch at the result's offsets; reduced counts
    DevBuf d_dd_wl, d_dd_wl_n;  // k_dd_pass -> k_dedupe worklist
    DevBuf d_kcnt, d_rcur;      // runs: ids per topic; the batch's span cursor (shared by its sub-batches)
    DevBuf d_wave_info;         // ids modes: per wave {base, ids, spilled} (MatchArgs.wave_info)
    DevBuf d_pre;               // k_prescan's output: TM_PRELOOK word ids + {levels, byte} per topic
    DevBuf d_res_scan;          // scan scratch of the set's result passes (one per set: sets run concurrently)
    // A launch's counters live in one 32-B block {cursor u64, slow_count u32 (+pad),
    // seg_cursor u64, fr_cursor u64}.  Two blocks alternate: each launch zeroes the block
    // the NEXT launch will use, so no memset launches precede a batch.
    DevBuf d_ctl;
    uint8_t *p_ctl = nullptr;  // the last launch's block
    uint32_t ctl_cur = 0;
    uint64_t keys_cap = 0, seg_chunks = 0, fr_chunks = 0, ukeys_cap = 0;
    uint64_t seg_demand_last = 0, fr_demand_last = 0;
    uint32_t last_n = 0;     // topics of the last batch
    uint32_t last_mode = 0;  // TM_MATCH_* of the last batch
    bool dev_batch = true;   // the device holds the last batch whole (tm_result_ids_device*)
    hipStream_t last_stream = nullptr;  // stream of the last batch (the next one is ordered after it)
    void release() {
        for (DevBuf *b : {&d_bytes, &d_off, &d_outoff, &d_outcnt, &d_status, &d_keys, &d_slow_list, &d_scr_w, &d_scr_s,
                          &d_seg_pool, &d_fr_pool, &d_wave_chunks, &d_ukeys, &d_ucnt, &d_dd_wl, &d_dd_wl_n, &d_kcnt,
                          &d_rcur, &d_ctl, &d_wave_info, &d_pre, &d_res_scan})
            b->release();
        // the sizes recorded for the released buffers go with them (a later ensure_batch
        // allocates again instead of trusting a capacity nothing holds)
        p_ctl = nullptr;
        ctl_cur = 0;
        keys_cap = seg_chunks = fr_chunks = ukeys_cap = 0;
        seg_demand_last = fr_demand_last = 0;
        last_stream = nullptr;
    }
};

// Edge table load <= 1/EDGE_LOAD_INV.  A wave waits for the longest of its ~256
// concurrent probe chains, so short chains (low load) matter more than table size:
// 1/16 walks config C 3.4 % faster than 1/8 (0.912 -> 0.881 ms) for 16 GiB of HBM instead
// of 8; an MI355X has 288 GB.
constexpr uint64_t EDGE_LOAD_INV = 16;
// Largest edge table: node ids are u32 slot indices and must stay below the sentinels
// (NONE, W_PLUS, ROOT_ID); 2^31 slots = 32 GiB of HBM.
// Word table load <= 1/WORD_LOAD_INV (small: it sizes with the vocabulary, not the nodes).
constexpr uint64_t WORD_LOAD_INV = 4;

// Device arrays of the frozen index: what a device image holds and what an epoch patch
// touches (replicated mode, tm_image_export / tm_replica_*).
enum : uint32_t {
    A_WTAB, A_WARENA, A_WORD_OFF, A_ETAB, A_SLOT_LIST, A_ARENA, A_ROOT, A_KEY_REC, A_KEY_NODE, A_KEY_BIN, A_KEY_DD,
    A_N
};
constexpr uint32_t ARR_ELEM[A_N] = {16, 1, 4, 16, 4, 4, 16, 16, 4, 4, 1};

// Epoch patch: what one delta commit changed on the device, as records a replica replays.
enum : uint32_t { P_TAIL = 1, P_SCATTER = 2, P_WHOLE = 3 };
struct PatchRec {
    uint32_t kind, arr;
    uint64_t count;  // elements
    uint64_t a;      // P_TAIL: first element written; P_WHOLE: capacity (bytes) to allocate
    uint64_t bytes;  // payload bytes following this record (8-byte padded)
};
// "TMPATCH2" / "EXTMIMG2": the trailing digit is the layout version (2: LIST_HDR 6, the HDR_DD
// collapse word of round 5), so a replica of another build refuses the image or patch instead
// of reading every list header one word off
constexpr uint64_t PATCH_MAGIC = 0x3248435441504d54ull, IMAGE_MAGIC = 0x32474d494d545845ull;
constexpr size_t STATS_BYTES = 96 * 8;  // walk counters (device_api.h MatchArgs.stats)

struct PatchHdr {
    uint64_t magic;
    uint64_t epoch_from, epoch_to;
    uint64_t wmask, emask, n_deep, n_live, n_records;
    uint64_t full;   // the commit re-uploaded everything: replicas reload from an image
    uint64_t nonce;  // the master's identity: a replica applies patches of its own master only
    uint64_t max_id;
};
struct ImageHdr {
    uint64_t magic;
    uint64_t epoch, wmask, emask, n_deep, n_live, n_nodes, n_words;
    uint64_t nonce, max_id;
    uint64_t cap[A_N], used[A_N], off[A_N];
};
constexpr uint64_t IMAGE_ALIGN = 256;

struct PatchLog {
    bool on = false;   // tm_config.flags & TM_CFG_RECORD_PATCH
    bool full = false;
    uint64_t n = 0;
    std::vector<uint8_t> buf;
    void reset() {
        full = false;
        n = 0;
        buf.clear();
    }
    void add(uint32_t kind, uint32_t arr, uint64_t count, uint64_t a, const void *p1, size_t n1,
             const void *p2 = nullptr, size_t n2 = 0) {
        if (!on || full) return;
        const uint64_t pay = (n1 + n2 + 7) & ~7ull;
        PatchRec r{kind, arr, count, a, pay};
        const size_t at = buf.size();
        buf.resize(at + sizeof r + pay, 0);
        memcpy(&buf[at], &r, sizeof r);
        if (n1) memcpy(&buf[at + sizeof r], p1, n1);
        if (n2) memcpy(&buf[at + sizeof r + n1], p2, n2);
        n++;
    }
};

inline uint64_t next_pow2(uint64_t x) {
    uint64_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// tm_last_error(): the calling thread's last failure (several threads may call one engine at
// once, so one shared message would be overwritten by another thread's call).
std::string &tl_err() {
    thread_local std::string s;
    return s;
}
// tm_create_last_error(): why the calling thread's last tm_create / tm_replica_create failed
std::string &tl_create_err() {
    thread_local std::string s;
    return s;
}
struct ErrSlot {
    ErrSlot &operator=(std::string s) {
        tl_err() = std::move(s);
        return *this;
    }
    ErrSlot &operator=(const char *s) {
        tl_err() = s;
        return *this;
    }
    const char *c_str() const { return tl_err().c_str(); }
};

// Resident helpers for a commit's parallel phases (resolve, list builds, list placement, the
// delta upload's gathers): starting 15 threads costs ~0.3-0.5 ms, several times per commit,
// against phases of 1-2 ms.  run(nt, f) calls f(0..nt-1), f(0) on the caller, and returns when
// all are done.  One caller at a time (commits are serialised by mu_commit).
struct WorkPool {
    std::mutex m;
    std::condition_variable cv_go, cv_done;
    std::vector<std::thread> th;
    const std::function<void(unsigned)> *job = nullptr;
    unsigned want = 0, left = 0;
    uint64_t gen = 0;
    bool quit = false;
    void loop(unsigned id) {
        // A commit's helpers run below the threads that keep matching beside the commit: on a
        // process pinned to as many CPUs as it has threads, a matching thread woken by its GPU
        // event then preempts a helper at once instead of waiting out a helper's time slice
        // (10 ms matches during a full rebuild's apply/lists phases, profiles/r06_bench_b.json).
        // Raising one's own nice value needs no privilege.  EMQX_TM_HELPER_NICE overrides (0: off).
        static const int nice_v = [] {
            const char *e = getenv("EMQX_TM_HELPER_NICE");
            return e ? atoi(e) : 10;
        }();
        if (nice_v > 0) (void)setpriority(PRIO_PROCESS, (id_t)syscall(SYS_gettid), nice_v);
        uint64_t seen = 0;
        for (;;) {
            const std::function<void(unsigned)> *j;
            {
                std::unique_lock<std::mutex> lk(m);
                cv_go.wait(lk, [&] { return quit || gen != seen; });
                if (quit) return;
                seen = gen;
                if (id >= want) continue;
                j = job;
            }
            (*j)(id);
            std::lock_guard<std::mutex> g(m);
            if (--left == 0) cv_done.notify_one();
        }
    }
    void run(unsigned nt, const std::function<void(unsigned)> &f) {
        try {
            while (nt > 1 && th.size() < nt - 1) {
                const unsigned id = (unsigned)th.size() + 1;
                th.emplace_back([this, id] { loop(id); });
            }
        } catch (...) {  // fewer helpers than parts: the caller runs the parts left over
        }
        const unsigned helpers = std::min<unsigned>(nt ? nt - 1 : 0, (unsigned)th.size());
        if (helpers) {
            std::lock_guard<std::mutex> g(m);
            job = &f;
            want = helpers + 1;
            left = helpers;
            gen++;
        }
        if (helpers) cv_go.notify_all();
        f(0);
        for (unsigned k = helpers + 1; k < nt; k++) f(k);
        if (!helpers) return;
        std::unique_lock<std::mutex> lk(m);
        cv_done.wait(lk, [&] { return left == 0; });
    }
    ~WorkPool() {
        {
            std::lock_guard<std::mutex> g(m);
            quit = true;
        }
        cv_go.notify_all();
        for (std::thread &t : th) t.join();
    }
};
// Sort and deduplicate a commit's dirty list (node ids, key handles, arena words: all below
// 2^32): three 11-bit LSD radix passes for long lists (std::sort of 20 K random ids took ~2-3
// ms of a config-E commit).
static void sort_unique(std::vector<uint64_t> &v) {
    const size_t n = v.size();
    bool by_compare = n < 2048;
    for (size_t i = 0; !by_compare && i < n; i++) by_compare = v[i] >> 32;
    if (by_compare) {
        std::sort(v.begin(), v.end());
    } else {
        std::vector<uint64_t> t(n);
        uint32_t cnt[2048];
        for (int sh = 0; sh < 33; sh += 11) {
            std::fill(cnt, cnt + 2048, 0u);
            for (uint64_t x : v) cnt[(x >> sh) & 2047]++;
            uint32_t acc = 0;
            for (uint32_t &c : cnt) {
                const uint32_t k = c;
                c = acc;
                acc += k;
            }
            for (uint64_t x : v) t[cnt[(x >> sh) & 2047]++] = x;
            v.swap(t);
        }
    }
    v.erase(std::unique(v.begin(), v.end()), v.end());
}
// CPUs this process may keep busy at once: its affinity set, cut to the cgroup's CPU quota
// (cpu.max).  Past the quota a job's threads all stop until the period ends (the GPU boxes
// here grant 16 CPUs per 100 ms period while every CPU of the machine is in the affinity set),
// so parallel phases never use more helpers than this.
static unsigned usable_cpus() {
    static const unsigned n = [] {
        unsigned c = std::max(1u, std::thread::hardware_concurrency());
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof set, &set) == 0) c = std::min<unsigned>(c, (unsigned)CPU_COUNT(&set));
        if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
            char q[32] = {0};
            unsigned long long per = 0;
            if (fscanf(f, "%31s %llu", q, &per) == 2 && strcmp(q, "max") != 0 && per)
                c = std::min<unsigned>(c, (unsigned)std::max(1ull, strtoull(q, nullptr, 10) / per));
            fclose(f);
        }
        return std::max(1u, c);
    }();
    return n;
}
// Helpers of a commit's parallel phases: the usable CPUs less two, at most 16.  The two are left
// to the threads that keep matching meanwhile: on a process pinned to quota-many CPUs, as many
// helpers as CPUs leave a matching thread waiting for a time slice (EMQX_TM_COMMIT_THREADS
// overrides).
static unsigned commit_threads() {
    static const unsigned n = [] {
        if (const char *e = getenv("EMQX_TM_COMMIT_THREADS")) {
            const int v = atoi(e);
            if (v > 0) return (unsigned)v;
        }
        const unsigned u = usable_cpus();
        return std::max(1u, std::min(16u, u > 4 ? u - 2 : u));
    }();
    return n;
}

// A few resident threads that split large host copies (staging a pageable batch into pinned
// memory): thread start-up per copy would cost more than the copy of one sub-batch.
struct CopyPool {
    std::mutex m;
    std::condition_variable cv, done_cv;
    std::vector<std::thread> th;
    struct Job {
        uint8_t *dst;
        const uint8_t *src;
        size_t n;
    };
    std::vector<Job> q;
    size_t pending = 0;
    bool stop = false;
    void start(unsigned n) {
        for (unsigned k = 0; k < n; k++)
            th.emplace_back([this] {
                std::unique_lock<std::mutex> lk(m);
                for (;;) {
                    cv.wait(lk, [&] { return stop || !q.empty(); });
                    if (stop && q.empty()) return;
                    Job j = q.back();
                    q.pop_back();
                    lk.unlock();
                    memcpy(j.dst, j.src, j.n);
                    lk.lock();
                    if (--pending == 0) done_cv.notify_all();
                }
            });
    }
    void copy(void *dst, const void *src, size_t n) {
        // the pool only for large batches: several threads' calls may share it, and a small copy
        // is cheaper on the calling thread than a hand-off
        const size_t per = 4u << 20;
        const size_t parts = n < (8u << 20) ? 1 : std::min<size_t>(th.size() + 1, (n + per - 1) / per);
        if (parts <= 1 || th.empty()) {
            if (n) memcpy(dst, src, n);
            return;
        }
        {
            std::lock_guard<std::mutex> g(m);
            for (size_t k = 1; k < parts; k++) {
                const size_t a = n * k / parts, b = n * (k + 1) / parts;
                q.push_back(Job{(uint8_t *)dst + a, (const uint8_t *)src + a, b - a});
                pending++;
            }
        }
        cv.notify_all();
        memcpy(dst, src, n / parts);  // this thread takes the first part
        std::unique_lock<std::mutex> lk(m);
        done_cv.wait(lk, [&] { return pending == 0; });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(m);
            stop = true;
        }
        cv.notify_all();
        for (auto &t : th) t.join();
    }
};

// Host results of the calls that return host memory (tm_match_batch, tm_match_filter_batch,
// tm_intersect_batch, tm_match_batch_runs): one set per calling thread, so a result stays valid
// until the same thread's next such call however many threads share the engine.
struct HostOut {
    PinBuf h_outoff, h_outcnt, h_status, h_keys;
    std::vector<uint32_t> pp_off, pp_cnt, pp_keys;
    // matches_filter/3
    std::vector<uint32_t> f_off, f_cnt, f_ukeys;
    std::vector<int32_t> f_status;
    PinBuf f_keys;
    // tm_match_filter_batch_runs: per-query span counts, the walk's ranges, their spans, and the
    // sorted ids the spans point into (kept alive here across index rebuilds)
    std::vector<uint32_t> f_rcnt, fr_off, fr_cnt;  // fr_*: the runs result's (the keys form reuses f_*)
    std::vector<int32_t> fr_status;
    PinBuf f_rng;
    std::vector<tm_span> f_spans;
    std::shared_ptr<const std::vector<uint64_t>> f_ids;
    // intersection/2
    std::vector<uint64_t> ix_off;
    std::vector<int32_t> ix_len;
    std::vector<uint8_t> ix_bytes;
    // runs (tm_match_batch_runs)
    PinBuf r_off, r_cnt, r_kcnt, r_status, r_runs;
    std::vector<tm_span> spans;
    std::vector<uint32_t> span_off;
    uint64_t lease_epoch = 0;
    bool lease = false;  // holds a read lease on the host id arena (tm_match_batch_runs)
    // The device side of this thread's host-form calls (tm_match_batch ALL / FIRST / COUNT,
    // tm_match_batch_runs): its own batch buffers, streams, events and pinned staging, so the
    // calls of several threads overlap on the device.  A call holds the engine's device lock
    // only while it queues work that reads the index (and records that work, note_use, so a
    // commit orders its in-place writes and buffer swaps after it), not across the H2D, the
    // sync and the D2H of its own buffers (round 4; the reference index is read_concurrency,
    // emqx_topic_index.erl:41-42).
    BatchBufs bb;
    hipStream_t s_walk = nullptr, s_copy = nullptr, s_h2d = nullptr;
    hipEvent_t ev_pk[2] = {}, ev_pd[2] = {}, ev_h2d[16] = {};
    PinBuf h_bytes, h_off, h_ctl, h_rctl;
    double pipe_kpt = 0, runs_spt = 4.0;  // keys / spans per topic of this thread's last batch
    hipError_t lanes() {  // streams and events, once per thread (the device is already set)
        if (s_walk) return hipSuccess;
        hipError_t e;
        for (hipStream_t *st : {&s_walk, &s_copy, &s_h2d})
            if ((e = hipStreamCreateWithFlags(st, hipStreamNonBlocking))) return e;
        for (hipEvent_t *ev : {&ev_pk[0], &ev_pk[1], &ev_pd[0], &ev_pd[1]})
            if ((e = hipEventCreateWithFlags(ev, hipEventDisableTiming))) return e;
        for (hipEvent_t &ev : ev_h2d)
            if ((e = hipEventCreateWithFlags(&ev, hipEventDisableTiming))) return e;
        return hipSuccess;
    }
    void release() {
        for (hipStream_t st : {s_walk, s_copy, s_h2d})
            if (st) (void)hipStreamSynchronize(st);
        for (hipEvent_t ev : {ev_pk[0], ev_pk[1], ev_pd[0], ev_pd[1]})
            if (ev) (void)hipEventDestroy(ev);
        for (hipEvent_t &ev : ev_h2d)
            if (ev) (void)hipEventDestroy(ev);
        for (hipStream_t st : {s_walk, s_copy, s_h2d})
            if (st) (void)hipStreamDestroy(st);
        s_walk = s_copy = s_h2d = nullptr;
        ev_pk[0] = ev_pk[1] = ev_pd[0] = ev_pd[1] = nullptr;
        for (hipEvent_t &ev : ev_h2d) ev = nullptr;
        bb.release();
        for (PinBuf *b : {&h_bytes, &h_off, &h_ctl, &h_rctl}) b->release();
        for (PinBuf *b : {&h_outoff, &h_outcnt, &h_status, &h_keys, &f_keys, &f_rng, &r_off, &r_cnt, &r_kcnt, &r_status,
                          &r_runs})
            b->release();
        std::vector<uint32_t>().swap(f_rcnt);
        std::vector<uint32_t>().swap(fr_off);
        std::vector<uint32_t>().swap(fr_cnt);
        std::vector<int32_t>().swap(fr_status);
        std::vector<tm_span>().swap(f_spans);
        f_ids.reset();
        std::vector<uint32_t>().swap(pp_off);
        std::vector<uint32_t>().swap(pp_cnt);
        std::vector<uint32_t>().swap(pp_keys);
        std::vector<uint32_t>().swap(f_off);
        std::vector<uint32_t>().swap(f_cnt);
        std::vector<uint32_t>().swap(f_ukeys);
        std::vector<int32_t>().swap(f_status);
        std::vector<uint64_t>().swap(ix_off);
        std::vector<int32_t>().swap(ix_len);
        std::vector<uint8_t>().swap(ix_bytes);
        std::vector<tm_span>().swap(spans);
        std::vector<uint32_t>().swap(span_off);
    }
};

// What the match path reads of the index besides the device buffers: set only when a commit
// PUBLISHES (under mu_dev), so a match never sees a table mask of a host table that a commit
// running on another thread has already rehashed but not yet uploaded.
struct DevView {
    std::atomic<uint64_t> epoch{0};  // also read without the lock (the aggregator's window trace)
    uint64_t wmask = 0, emask = 0;
    uint64_t n_deep = 0;
    uint64_t max_id = 0;
    uint64_t n_live = 0, n_nodes = 0, n_words = 0;
};

}  // namespace

struct tm_engine {
    tm_config cfg{};
    ErrSlot err;
    uint64_t epoch = 0;  // host master epoch (== dv.epoch after every successful publish)

    // ---- locks (DESIGN.md §1 "Threading").  Order: mu_commit -> (leases) -> mu_host -> mu_dev
    // -> mu_stage / mu_out.
    //   mu_commit one commit at a time (only a commit changes the host copy, so its read-only
    //             pre-check needs no other lock)
    //   mu_stage  the staged op list (tm_apply never waits for a match or a commit)
    //   mu_host   the host master copy: commit's host phase, key introspection, the
    //             matches_filter index, host-side UNIQUE
    //   mu_dev    the device: index buffers, batch buffers, streams, DevView (every match)
    // A commit holds mu_host for its host phase and takes mu_dev only to publish: a delta's
    // scatters, or the pointer swap of a full rebuild built off to the side (standby image).
    std::mutex mu_commit, mu_stage, mu_host, mu_out;
    std::recursive_mutex mu_dev;
    DevView dv;
    // streams that ran work reading the index since the last publish, with an event recorded
    // after that work: a publish makes its own stream wait on them before writing in place
    std::vector<std::pair<hipStream_t, hipEvent_t>> uses;
    std::unordered_map<std::thread::id, std::unique_ptr<HostOut>> outs;
    // read leases on the host id arena (runs results): a commit's host phase waits for them
    std::mutex lease_mu;
    std::condition_variable lease_cv;
    uint64_t n_leases = 0;
    bool lease_block = false;

    // ---- words (interner + device word table mirror)
    std::vector<WordSlot> wtab;
    uint64_t wmask = 0;
    std::vector<uint8_t> warena;
    std::vector<uint32_t> word_off, word_len;  // by word id
    size_t warena_dev = 0;                      // bytes of warena already on device

    // ---- edges / nodes
    // The device edge table is slot-indexed (a node is its slot, at load <= 1/16: 16 GiB at
    // config C).  The host keeps no copy of it: per node its slot, bloom, info and device
    // list entry, a bitmap of the taken slots (where a new edge goes: the same linear probe
    // the device runs), and a node-sized map (parent node, word) -> child for its own walks.
    uint64_t emask = 0;  // device slots - 1
    uint64_t n_edges = 0;
    hvec<uint32_t> node_parent, node_word, node_slot;
    hvec<NodeList> node_list;  // terminal list of every node (host numbering)
    hvec<uint32_t> node_cap;   // keys the node's arena list has room for (>= its count)
    hvec<uint32_t> node_bloom, node_info;  // the node's EdgeSlot.bloom / .info on the device
    hvec<uint32_t> node_slist;             // the node's slot_list entry on the device
    hvec<uint64_t> eocc;                   // taken device slots, one bit each
    struct EMapEnt {
        uint32_t parent, word, child, pad;  // parent == NONE: empty
    };
    hvec<EMapEnt> emap;
    uint64_t emap_mask = 0;
    RootRec root{0, 0, 0, 0};

    // ---- terminal-list arena
    hvec<uint32_t> arena;
    uint64_t arena_garbage = 0;
    size_t arena_dev = 0;  // words already on device
    // Host id arena: arena_id[i] = id of the key handle arena[i] (key positions only), so a run
    // of the arena is a span of route ids (tm_match_batch_runs).  One fixed virtual reservation
    // (MAP_NORESERVE, touched as it fills), so spans stay valid while the arena grows.
    uint64_t *arena_id = nullptr;
    uint64_t arena_id_res = 0;  // entries reserved
    // The same as u32 (round 4), kept while every id ever added fits 32 bits (max_id < 2^32):
    // a span of it is half the cache lines for the consumer that reads it (the aggregator's
    // delivery threads: DESIGN.md §9).  Inline (single-key) spans point into key_id32.
    uint32_t *arena_id32 = nullptr;
    hvec<uint32_t> key_id32;  // by key handle
    bool ids32() const { return !replica && arena_id32 && max_id <= 0xFFFFFFFFull; }
    // A replica keeps the same host id arena (from its device copy: image loads and patches)
    // and the id of every key handle, so its windows and host calls can answer in runs form too.
    hvec<uint64_t> r_key_id;
    bool r_ids = false;  // arena_id / r_key_id follow the replica's device copy
    int replica_ids_full() {  // whole, from the device arrays (an image load, an array replaced)
        r_ids = false;
        if (!arena_id) return TM_OK;
        const uint64_t nk = dev_used[A_KEY_REC] / 16, nw = dev_used[A_ARENA] / 4;
        if (nw > arena_id_res) return TM_OK;  // past the reservation: runs stay off
        std::vector<uint64_t> rec(2 * nk + 2);
        std::vector<uint32_t> ar(nw + 1);
        if (nk && hipMemcpy(rec.data(), d_key_rec.p, nk * 16, hipMemcpyDeviceToHost) != hipSuccess) return TM_EDEVICE;
        if (nw && hipMemcpy(ar.data(), d_arena.p, nw * 4, hipMemcpyDeviceToHost) != hipSuccess) return TM_EDEVICE;
        r_key_id.resize(nk);
        for (uint64_t h = 0; h < nk; h++) r_key_id[h] = rec[2 * h];
        // list headers (counts, minima) get an id too: harmless, no span covers them
        par_for(nw, [&](size_t i) { arena_id[i] = ar[i] < nk ? r_key_id[ar[i]] : 0; });
        r_ids = true;
        return TM_OK;
    }
    // after a patch: the key records it wrote first, then the arena words it wrote
    int replica_ids_patch(const uint8_t *p0, uint64_t n_records) {
        if (!arena_id || !r_ids) return replica_ids_full();
        for (int pass = 0; pass < 2; pass++) {
            const uint8_t *p = p0;
            for (uint64_t i = 0; i < n_records; i++) {
                PatchRec r;
                memcpy(&r, p, sizeof r);
                const uint8_t *pay = p + sizeof r;
                p += sizeof r + r.bytes;
                if (r.arr != (pass ? A_ARENA : A_KEY_REC)) continue;
                if (r.kind == P_WHOLE) return replica_ids_full();
                const uint64_t el = ARR_ELEM[r.arr];
                const uint8_t *vals = r.kind == P_SCATTER ? pay + r.count * 8 : pay;
                for (uint64_t k = 0; k < r.count; k++) {
                    uint64_t at = r.a + k;
                    if (r.kind == P_SCATTER) memcpy(&at, pay + k * 8, 8);
                    if (pass == 0) {
                        uint64_t id;
                        memcpy(&id, vals + k * el, 8);
                        if (at >= r_key_id.size()) r_key_id.resize(at + 1, 0);
                        r_key_id[at] = id;
                    } else {
                        if (at >= arena_id_res) {
                            r_ids = false;  // past the reservation: runs stay off
                            return TM_OK;
                        }
                        uint32_t h;
                        memcpy(&h, vals + k * el, 4);
                        arena_id[at] = h < r_key_id.size() ? r_key_id[h] : 0;
                    }
                }
            }
        }
        return TM_OK;
    }
    void ids_of(uint64_t lo, uint64_t hi) {  // refresh arena_id over key positions [lo, hi)
        if (!arena_id) return;
        if (hi > arena_id_res) {  // past the reservation: only until the compaction this forces
            ids_stale = true;
            hi = arena_id_res;
        }
        for (uint64_t i = lo; i < hi; i++) arena_id[i] = keys[arena[i]].id;
        if (arena_id32)
            for (uint64_t i = lo; i < hi; i++) arena_id32[i] = (uint32_t)arena_id[i];
    }
    std::atomic<bool> ids_stale{false};  // set by list placements running in parallel
    bool reserve_ids() {  // a virtual reservation of the budget (halved until the OS grants it)
        uint64_t want = std::min<uint64_t>(std::max<uint64_t>(arena_budget() + 16, 1ull << 16), 1ull << 32);
        while (want >= (1ull << 12)) {
            void *p = mmap(nullptr, want * 8, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
            if (p != MAP_FAILED) {
                void *q = mmap(nullptr, want * 4, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
                (void)madvise(p, want * 8, MADV_HUGEPAGE);  // read at random places by every reply
                if (q != MAP_FAILED) (void)madvise(q, want * 4, MADV_HUGEPAGE);
                arena_id = (uint64_t *)p;
                arena_id32 = q != MAP_FAILED ? (uint32_t *)q : nullptr;  // without it: u64 runs only
                arena_id_res = want;
                return true;
            }
            want /= 2;
        }
        return false;
    }
    void release_ids() {
        if (arena_id) munmap(arena_id, arena_id_res * 8);
        if (arena_id32) munmap(arena_id32, arena_id_res * 4);
        arena_id = nullptr;
        arena_id32 = nullptr;
        arena_id_res = 0;
    }

    // ---- keys
    hvec<KeyRec> keys;
    std::vector<uint32_t> free_keys, free_pending;
    uint64_t n_live = 0;
    hvec<uint32_t> kset;  // open addressing over key handles
    uint64_t kmask = 0, kset_used = 0;
    std::map<std::pair<std::string, uint64_t>, uint32_t> dead_keys;

    // ---- live keys per id.  k_dedupe's UNIQUE table only needs the keys whose id some
    // other live key also carries (KR_MULTI, set once and kept: a stale flag only costs
    // a table insert).  Open addressing over ids; a slot with cnt == ID_EMPTY is free.
    struct IdUse {
        uint64_t id;
        uint32_t cnt;
        uint32_t solo;  // the one live key while cnt == 1 and it is not flagged yet
    };
    static constexpr uint32_t ID_EMPTY = 0xFFFFFFFFu;
    static constexpr uint8_t KR_MULTI = 1;
    hvec<IdUse> idtab;
    uint64_t idtab_used = 0;
    void id_rehash() {  // drops ids with no live key
        hvec<IdUse> old;
        old.swap(idtab);
        uint64_t live = 0;
        for (const IdUse &e : old) live += e.cnt != ID_EMPTY && e.cnt;
        uint64_t sz = 1024;
        while (sz < (live + 1) * 4) sz <<= 1;
        idtab.assign(sz, IdUse{0, ID_EMPTY, NONE});
        idtab_used = 0;
        for (const IdUse &e : old)
            if (e.cnt != ID_EMPTY && e.cnt) id_use(e.id) = e;
    }
    IdUse &id_use(uint64_t id) {
        if ((idtab_used + 1) * 2 > idtab.size()) id_rehash();
        const uint64_t m = idtab.size() - 1;
        uint64_t i = mix64(id) & m;
        while (idtab[i].cnt != ID_EMPTY && idtab[i].id != id) i = (i + 1) & m;
        if (idtab[i].cnt == ID_EMPTY) {
            idtab[i] = IdUse{id, 0, NONE};
            idtab_used++;
        }
        return idtab[i];
    }
    void id_add(uint32_t h) {
        IdUse &e = id_use(keys[h].id);
        if (e.cnt == 0) {
            e.solo = h;
        } else {
            if (e.solo != NONE) {  // the id's first key meets a second one: flag it too
                keys[e.solo]._p[0] |= KR_MULTI;
                dirty_kid.push_back(e.solo);
                dd_touch.push_back(e.solo);  // its list's header bit (lists_dd_touch)
                e.solo = NONE;
            }
            keys[h]._p[0] |= KR_MULTI;
        }
        e.cnt++;
    }
    void id_del(uint32_t h) {
        IdUse &e = id_use(keys[h].id);
        e.cnt--;
        e.solo = NONE;  // a key left behind was flagged when the count reached 2
    }
    std::vector<std::string> dead_filter;  // by key handle (only K_DEAD entries non-empty)
    // keys flagged KR_MULTI this epoch whose list may not be rewritten by it: their lists' header
    // collapse bits are OR'd in after the lists are placed (lists_dd_touch)
    std::vector<uint32_t> dd_touch;
    void lists_dd_touch() {
        for (uint32_t h : dd_touch) {
            const KeyRec &k = keys[h];
            if (k.kind == K_FREE || k.kind == K_DEAD) continue;
            const uint32_t lo = node_list[k.node].list_off;
            if (!lo || (arena[lo - HDR_DD] & KDD_MULTI)) continue;
            arena[lo - HDR_DD] |= KDD_MULTI;
            if (!need_full && lo - HDR_DD < arena_dev) dirty_arena.push_back(lo - HDR_DD);
        }
        dd_touch.clear();
    }

    // ---- staged ops and epoch deltas
    std::vector<StagedOp> staged;
    std::vector<uint8_t> stage_bytes;
    std::vector<std::pair<uint32_t, uint32_t>> lv_scratch;  // classify(): (start, len) per level
    std::vector<Delta> deltas;
    std::vector<uint64_t> dirty_wslots;
    std::vector<uint64_t> dirty_enodes, dirty_lnodes;  // nodes whose edge slot / slot_list entry changed
    std::vector<uint64_t> dirty_arena;  // arena words already on the device, rewritten in place
    uint64_t n_grows = 0;               // device arrays moved to a larger buffer by a delta commit
    bool root_dirty = true;
    bool need_full = true;  // full device upload at next commit
    bool words_full = false;  // word table rehashed: re-upload it whole at next commit

    // ---- device copy
    DevBuf d_wtab, d_warena, d_word_off, d_etab, d_slot_list, d_root, d_arena;
    size_t word_off_dev = 0;  // entries already on device
    DevBuf d_scatter_idx, d_scatter_src;
    DevBuf d_key_rec;                 // key handle -> {caller id, order code} (2 u64; key_ord)
    DevBuf d_key_node;                // key handle -> device slot of its node (u32; AGGRE classes)
    DevBuf d_key_bin;                 // key handle -> 1 for {Binary, {ID}} keys (u32; FIRST order)
    DevBuf d_key_dd;                  // key handle -> KDD_* flags (u8; which keys k_dedupe must table)
    std::vector<uint64_t> dirty_kid;  // handles (re)assigned since the last upload
    uint64_t n_deep = 0;              // live word-list keys too deep for the 64-bit order code
    DevBuf d_mrg_roff, d_mrg_tot;  // scratch of tm_merge_shards_device
    DevBuf d_stats;

    // Batch buffers: one set for the device-result calls (tm_match_device*, whose result the
    // engine keeps until the next such call) and one for the host-result calls (tm_match_batch*,
    // synchronous), so a host call from one thread never overwrites another thread's pending
    // device result.  `bb` is the set of the call in progress (under mu_dev).
    BatchBufs bb_dev, bb_batch;  // bb_batch: the batching aggregator's windows (batcher.cpp); host-form calls: HostOut::bb
    BatchBufs bb_dev2;  // tm_match_device_set(.., 1, ..): a second direct batch in flight
    BatchBufs bb_dev3;  // tm_match_device_set(.., 2, ..): a third
    BatchBufs bb_batch2;  // the aggregator's second window set (its windows alternate sets and streams)
    BatchBufs *batch_set(uint32_t set) { return set ? &bb_batch2 : &bb_batch; }
    BatchBufs *bb = &bb_dev;
    PinBuf h_cursor;           // tm_device_sync_set: the counter block of a direct batch
    hipStream_t stream = nullptr;
    hipStream_t s_build = nullptr;  // a full rebuild's standby upload (beside the matches)
    CopyPool copier;  // tm_match_batch_runs: staging a pageable batch into pinned memory
    mutable WorkPool pool;  // a commit's parallel phases (under mu_commit)
    // f(0..n-1) in contiguous chunks on the pool's threads (random reads: one helper per 1 K)
    template <class F>
    void par_for(size_t n, const F &f) const {
        const unsigned nt = n < 4096 ? 1u : (unsigned)std::min<size_t>(commit_threads(), n / 1024);
        pool.run(nt, [&](unsigned k) {
            for (size_t i = n * k / nt, e = n * (k + 1) / nt; i < e; i++) f(i);
        });
    }
    // The edge image of a full publish (clear every slot, then place every node) in slices of
    // about 0.1-0.2 ms each, every slice waited for and followed by a pause, so a match running
    // beside the rebuild shares the memory system with at most one slice.  Launched whole, the
    // two kernels (3 + 5 ms at config C: 20 GiB of writes, 64 M random record scatters) stretched
    // a 0.13 ms match to 3-5 ms (profiles/r06_rebuild_probe_nice.jsonl).  EMQX_TM_EDGE_PACE_US:
    // the pause (default 150; 0 launches each kernel whole, unpaced).
    hipError_t edge_image_paced(uint4 *etab, uint32_t *sl, uint64_t slots, const NodeImage *nodes, uint64_t n,
                                hipStream_t s, uint64_t buf_slots) {
        static const long pace_us = [] {
            const char *e = getenv("EMQX_TM_EDGE_PACE_US");
            return e ? atol(e) : 150L;
        }();
        constexpr uint64_t CLEAR_SLICE = 32ull << 20, PLACE_SLICE = 2ull << 20;  // slots / records
        if (pace_us <= 0) return launch_edge_image(etab, sl, slots, nodes, n, s, buf_slots, bnd_rec());
        hipError_t e = hipSuccess;
        auto pause = [&]() -> hipError_t {
            hipError_t r = hipStreamSynchronize(s);
            if (r == hipSuccess) std::this_thread::sleep_for(std::chrono::microseconds(pace_us));
            return r;
        };
        for (uint64_t lo = 0; lo < slots && !e; lo += CLEAR_SLICE) {
            e = launch_edge_clear_range(etab, sl, lo, std::min(slots, lo + CLEAR_SLICE), s, buf_slots, bnd_rec());
            if (!e && (lo + CLEAR_SLICE < slots || n)) e = pause();
        }
        for (uint64_t lo = 0; lo < n && !e; lo += PLACE_SLICE) {
            e = launch_edge_place_range(etab, sl, slots, nodes + lo, std::min(n - lo, PLACE_SLICE), s, buf_slots, bnd_rec());
            if (!e && lo + PLACE_SLICE < n) e = pause();
        }
        return e;
    }
    std::once_flag copier_once;
    hipEvent_t ev_chain = nullptr;  // orders a device match after the previous one's stream
    uint64_t n_full_rebuilds = 0, n_delta_commits = 0, n_slow_last = 0;
    uint64_t commit_us[3] = {0, 0, 0};  // last commit: apply / lists / upload (tm_stats)
    uint64_t commit_stall_us = 0;       // last commit: matches held back while it published
    uint64_t n_commits_refused = 0;     // commits refused for capacity (ops kept staged)
    uint64_t staged_count() {
        std::lock_guard<std::mutex> g(mu_stage);
        return staged.size();
    }
    bool stats_on = false;
    uint64_t max_id = 0;     // largest id ever added (ids fit u32 results while < 2^32)
    PatchLog patch;          // master: the last commit's device changes (TM_CFG_RECORD_PATCH)
    uint64_t patch_from = 0; // epoch the recorded patch applies to
    bool replica = false;    // built from a device image: no host master copy, read-only
    uint64_t master_nonce = 0;  // random per master engine; a replica holds its master's
    uint64_t dev_used[A_N] = {};  // bytes of each device array in use (image export)
    hipEvent_t ev_fast0 = nullptr, ev_fast1 = nullptr;  // around k_match_fast (tm_debug_timing)
    bool timing_on = false;
    bool topic_words = false;  // the batch being enqueued holds word-list topics (TM_MATCH_TOPIC_WORDS)
    uint32_t runs_w = 8;       // the MODE_RUNS batch being enqueued: id width of its spans (4: arena_id32)
    uint32_t dd_next = 0;      // the next enqueue_match counts collapsible keys for this KDD_* bit (under mu_dev)

    uint64_t edge_load_inv() const { return cfg.edge_load_inv ? cfg.edge_load_inv : EDGE_LOAD_INV; }
    uint64_t node_budget() const {  // trie nodes below the root
        const uint64_t hard = MAX_EDGE_SLOTS / 2;
        return cfg.max_nodes ? std::min<uint64_t>(cfg.max_nodes, hard) : hard;
    }
    uint64_t arena_budget() const {  // list offsets are u32; the host id arena's reservation
        const uint64_t hard = arena_id_res ? std::min<uint64_t>(0xFFFFFFF0ull, arena_id_res - 16) : 0xFFFFFFF0ull;
        return cfg.max_list_words ? std::min<uint64_t>(cfg.max_list_words, hard) : hard;
    }

    HostOut &out() {  // the calling thread's host results
        std::lock_guard<std::mutex> g(mu_out);
        std::unique_ptr<HostOut> &p = outs[std::this_thread::get_id()];
        if (!p) p.reset(new HostOut());
        return *p;
    }

    // ---- ordering of device work (under mu_dev)
    // index-reading work was queued on s: remember it (a publish waits for it)
    hipError_t note_use(hipStream_t s) {
        for (auto &u : uses)
            if (u.first == s) return hipEventRecord(u.second, s);
        hipEvent_t ev;
        hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
        if (e) return e;
        uses.push_back({s, ev});
        return hipEventRecord(ev, s);
    }
    // make `s` wait (on the device) for every recorded use
    hipError_t wait_uses(hipStream_t s) {
        for (auto &u : uses)
            if (u.first != s) {
                hipError_t e = hipStreamWaitEvent(s, u.second, 0);
                if (e) return e;
            }
        return hipSuccess;
    }
    // the host waits for every recorded use and the engine stream (before buffers are freed)
    hipError_t quiesce() {
        for (auto &u : uses) {
            hipError_t e = hipEventSynchronize(u.second);
            if (e) return e;
        }
        return stream ? hipStreamSynchronize(stream) : hipSuccess;
    }
    // A device match about to run on s reuses the batch buffers of the previous one (which ran
    // on last_stream): order s after everything queued on last_stream so far, which includes
    // the previous caller's reads of its result.
    hipError_t chain_after_last(hipStream_t s) {
        if (!bb->last_stream || bb->last_stream == s) return hipSuccess;
        hipError_t e;
        if (!ev_chain && (e = hipEventCreateWithFlags(&ev_chain, hipEventDisableTiming))) return e;
        if ((e = hipEventRecord(ev_chain, bb->last_stream))) return e;
        return hipStreamWaitEvent(s, ev_chain, 0);
    }

    // ---- TM_BOUNDS debug build
    // elements of `elem` bytes from p to the end of the live engine buffer holding p (~0: p is
    // not in one, e.g. a caller's tensor)
    static uint64_t bnd_cap_of(const void *p, size_t elem) {
#if TM_BOUNDS
        if (!p) return 0;
        std::lock_guard<std::mutex> g(bnd_registry().m);
        const uint8_t *q = static_cast<const uint8_t *>(p);
        for (const auto &kv : bnd_registry().live) {
            const uint8_t *b = static_cast<const uint8_t *>(kv.first);
            if (q >= b && q < b + kv.second) return (uint64_t)(b + kv.second - q) / elem;
        }
#else
        (void)p;
        (void)elem;
#endif
        return ~0ull;
    }
    // the real capacities behind a match launch's pointers (read by the bounds build's kernels)
    void fill_caps(MatchArgs &a) const {
        BndCaps &c = a.cap;
        if (!TM_BOUNDS) {
            memset(&c, 0xFF, sizeof c);
            a.bnd = nullptr;
            return;
        }
        const size_t kel = a.mode == MODE_RUNS ? 16 : a.mode == MODE_IDS64 ? 8 : 4;
        c.bytes = bnd_cap_of(a.bytes, 1);
        c.off = bnd_cap_of(a.off, 4);
        c.wtab = d_wtab.cap / 16;
        c.warena = d_warena.cap;
        c.word_off = d_word_off.cap / 4;
        c.etab = d_etab.cap / 16;
        c.slot_list = d_slot_list.cap / 4;
        c.arena = d_arena.cap / 4;
        c.key_bin = d_key_bin.cap / 4;
        c.key_rec = d_key_rec.cap / 8;
        c.key_dd = d_key_dd.cap;
        c.out = std::min(std::min(bnd_cap_of(a.out_off, 4), bnd_cap_of(a.out_cnt, 4)), bnd_cap_of(a.status, 4));
        if (a.mode == MODE_RUNS) c.out = std::min(c.out, bnd_cap_of(a.out_kcnt, 4));
        c.keys = bnd_cap_of(a.keys, kel);
        c.slow_list = bnd_cap_of(a.slow_list, 4);
        c.scratch = std::min(bnd_cap_of(a.scratch_w, 4), bnd_cap_of(a.scratch_s, 8));
        c.seg_pool = bnd_cap_of(a.seg_pool, 16);
        c.wave_chunks = bnd_cap_of(a.wave_chunks, 4);
        c.fr_pool = bnd_cap_of(a.fr_pool, 8);
        c.wave_info = a.wave_info ? bnd_cap_of(a.wave_info, 16) : 0;
        c.pre_wid = a.pre_wid ? bnd_cap_of(a.pre_wid, 4) : 0;
        c.pre_meta = a.pre_meta ? bnd_cap_of(a.pre_meta, 8) : 0;
        // self-test of the bounds build (tests/test_gpu_bounds.py): pretend the edge table has
        // one slot, so every probe past slot 0 must be recorded (and redirected to slot 0)
        static const bool selftest = getenv("EMQX_TM_BOUNDS_SELFTEST") != nullptr;
        if (selftest) c.etab = 1;
        a.bnd = bnd_rec();
    }
    unsigned long long *bnd_rec() const {
#if TM_BOUNDS
        return cfg.device >= 0 && cfg.device < 64 ? bnd_registry().rec[cfg.device] : nullptr;
#else
        return nullptr;
#endif
    }
    // the bounds build: this device's record (once per process; never freed)
    static bool bnd_init(int device) {
#if TM_BOUNDS
        std::lock_guard<std::mutex> g(bnd_registry().m);
        if (device < 0 || device >= 64) return false;
        unsigned long long *&r = bnd_registry().rec[device];
        if (r) return true;
        if (hipMalloc(&r, 64) != hipSuccess || hipMemset(r, 0, 64) != hipSuccess) {
            r = nullptr;
            return false;
        }
#else
        (void)device;
#endif
        return true;
    }
    const char *buf_name(const void *p) {
        struct N {
            const char *n;
            const DevBuf *b;
        };
        const N main[] = {{"wtab", &d_wtab},         {"warena", &d_warena},     {"word_off", &d_word_off},
                          {"etab", &d_etab},         {"slot_list", &d_slot_list}, {"root", &d_root},
                          {"arena", &d_arena},       {"key_rec", &d_key_rec},   {"key_node", &d_key_node},
                          {"key_bin", &d_key_bin},   {"key_dd", &d_key_dd},     {"sblob", &d_sblob},
                          {"scatter_idx", &d_scatter_idx}, {"scatter_src", &d_scatter_src}, {"stats", &d_stats}};
        for (const N &x : main)
            if (x.b->p == p) return x.n;
        const BatchBufs *sets[] = {&bb_dev, &bb_dev2, &bb_dev3, &bb_batch, &bb_batch2};
        for (const BatchBufs *B : sets) {
            const N bn[] = {{"batch.bytes", &B->d_bytes},     {"batch.off", &B->d_off},       {"batch.outoff", &B->d_outoff},
                            {"batch.outcnt", &B->d_outcnt},   {"batch.status", &B->d_status}, {"batch.keys", &B->d_keys},
                            {"batch.slow_list", &B->d_slow_list}, {"batch.scr_w", &B->d_scr_w}, {"batch.scr_s", &B->d_scr_s},
                            {"batch.seg_pool", &B->d_seg_pool}, {"batch.fr_pool", &B->d_fr_pool},
                            {"batch.wave_chunks", &B->d_wave_chunks}, {"batch.ctl", &B->d_ctl}};
            for (const N &x : bn)
                if (x.b->p == p) return x.n;
        }
        return "(other)";
    }
    // a host-side check of the bounds build that failed (a copy past a buffer's end)
    void bnd_host(const char *what, const void *p, uint64_t n, uint64_t cap) {
        char b[256];
        snprintf(b, sizeof b, "%s: %llu bytes into buffer %s with %llu left; ", what, (unsigned long long)n, buf_name(p),
                 (unsigned long long)cap);
        bnd_note(b, 1);
    }
    static void bnd_note(const std::string &m, uint64_t hits) {
#if TM_BOUNDS
        fprintf(stderr, "tm bounds: %s\n", m.c_str());
        std::lock_guard<std::mutex> g(bnd_registry().m);
        if (bnd_registry().msg.size() < 1500) bnd_registry().msg += m;
        bnd_registry().hits += hits;
#else
        (void)m;
        (void)hits;
#endif
    }
    // After work queued on s (a match, an upload, a scatter): in the bounds build, wait for it,
    // read the kernels' bounds record and every live buffer's canary tail; what they show is
    // kept for tm_debug_bounds and the record and canaries are reset.  No-op in the product.
    hipError_t bnd_after(hipStream_t s, const char *what) {
#if TM_BOUNDS
        const hipError_t e = s ? hipStreamSynchronize(s) : hipDeviceSynchronize();
        return e ? e : bnd_scan(cfg.device, what, this);
#else
        (void)s;
        (void)what;
        return hipSuccess;
#endif
    }
    // the bounds build: device `dev`'s record and every live buffer's canary (names from `eng`)
    static hipError_t bnd_scan(int dev, const char *what, tm_engine *eng) {
#if TM_BOUNDS
        hipError_t e;
        std::string msg;
        uint64_t hits = 0;
        unsigned long long rec[4] = {0, 0, 0, 0};
        unsigned long long *d_rec = dev >= 0 && dev < 64 ? bnd_registry().rec[dev] : nullptr;
        if (d_rec && (e = hipMemcpy(rec, d_rec, sizeof rec, hipMemcpyDeviceToHost))) return e;
        if (rec[0]) {
            static const char *files[] = {"?", "match_kernels.hip", "result_kernels.hip", "filter_kernels.hip"};
            char b[256];
            snprintf(b, sizeof b, "%s: %llu out-of-bounds indices, first at %s:%llu index %llu >= capacity %llu; ", what,
                     rec[0], files[(rec[1] >> 24) & 3], rec[1] & 0xFFFFFF, rec[2], rec[3]);
            msg += b;
            hits += rec[0];
            if ((e = hipMemset(d_rec, 0, sizeof rec))) return e;
        }
        {
            // under the registry lock: no buffer is freed while its canary is read
            std::lock_guard<std::mutex> g(bnd_registry().m);
            std::vector<uint8_t> tail(BND_CANARY);
            for (const auto &kv : bnd_registry().live) {
                uint8_t *t = static_cast<uint8_t *>(kv.first) + kv.second;
                if ((e = hipMemcpy(tail.data(), t, BND_CANARY, hipMemcpyDeviceToHost))) return e;
                for (size_t k = 0; k < BND_CANARY; k++)
                    if (tail[k] != BND_FILL) {
                        char b[256];
                        snprintf(b, sizeof b, "%s: canary of buffer %s (%zu bytes) overwritten at +%zu; ", what,
                                 eng ? eng->buf_name(kv.first) : "(buffer)", kv.second, k);
                        msg += b;
                        hits++;
                        if ((e = hipMemset(t, BND_FILL, BND_CANARY))) return e;
                        break;
                    }
            }
        }
        if (hits) bnd_note(msg, hits);
#else
        (void)dev;
        (void)what;
        (void)eng;
#endif
        return hipSuccess;
    }

    // a batch buffer that must grow: in-flight work may still use it, so drain first
    hipError_t grow_buf(DevBuf &b, size_t bytes) {
        if (bytes <= b.cap && b.p) return hipSuccess;
        hipError_t e = quiesce();
        return e ? e : b.ensure(bytes);
    }

    // ---- read leases on the host id arena (tm_match_batch_runs)
    void lease_take_raw() {
        std::unique_lock<std::mutex> lk(lease_mu);
        // writer preference, except on an aggregator delivery thread whose window holds a lease:
        // a waiting commit needs that lease dropped, so waiting there would never end (and the
        // arena cannot change under it while the lease is held).  A callback of a window without
        // a lease waits like any caller: a commit may be changing the arena (advisor, round 4).
        if (!tmx_in_leased_delivery()) lease_cv.wait(lk, [&] { return !lease_block; });
        n_leases++;
    }
    void lease_drop_raw() {
        {
            std::lock_guard<std::mutex> g(lease_mu);
            n_leases--;
        }
        lease_cv.notify_all();
    }
    void lease_take(HostOut &o) {
        if (o.lease) return;
        lease_take_raw();
        o.lease = true;
    }
    void lease_drop(HostOut &o) {
        if (!o.lease) return;
        o.lease = false;
        lease_drop_raw();
    }
    // a commit's host phase: no new leases, wait for the held ones (writer preference)
    void leases_block() {
        std::unique_lock<std::mutex> lk(lease_mu);
        lease_block = true;
        lease_cv.wait(lk, [&] { return n_leases == 0; });
    }
    void leases_unblock() {
        {
            std::lock_guard<std::mutex> g(lease_mu);
            lease_block = false;
        }
        lease_cv.notify_all();
    }

    DevBuf *arr_buf(uint32_t a) {
        DevBuf *b[A_N] = {&d_wtab, &d_warena, &d_word_off, &d_etab, &d_slot_list, &d_arena,
                          &d_root, &d_key_rec, &d_key_node, &d_key_bin, &d_key_dd};
        return a < A_N ? b[a] : nullptr;
    }
    uint32_t arr_of(const DevBuf *d) {
        for (uint32_t a = 0; a < A_N; a++)
            if (arr_buf(a) == d) return a;
        return A_N;
    }

    // =====================================================================
    // words: a word of <= 8 bytes is its own key (zero-padded LE bytes); longer
    // words are keyed by FNV-1a 64 and verified against the arena
    static uint64_t word_key(const uint8_t *p, uint32_t len) {
        if (len <= 8) {
            uint64_t k = 0;
            for (uint32_t i = 0; i < len; i++) k |= (uint64_t)p[i] << (8 * i);
            return k;
        }
        uint64_t h = FNV_OFF;
        for (uint32_t i = 0; i < len; i++) h = fnv_step(h, p[i]);
        return h;
    }
    static uint32_t word_tag(uint32_t len) { return len > 8 ? (len | W_LONG) : len; }
    uint32_t word_lookup(const uint8_t *p, uint32_t len) const {
        const uint64_t key = word_key(p, len);
        const uint32_t tag = word_tag(len);
        uint64_t s = word_slot_hash(key, tag) & wmask;
        for (;;) {
            const WordSlot &w = wtab[s];
            if (w.wid == NONE) return NONE;
            if (w.key == key && w.len == tag && (len <= 8 || memcmp(&warena[word_off[w.wid]], p, len) == 0))
                return w.wid;
            s = (s + 1) & wmask;
        }
    }
    void word_rehash(uint64_t cap) {
        std::vector<WordSlot> old;
        old.swap(wtab);
        wtab.assign(cap, WordSlot{0, 0, NONE});
        wmask = cap - 1;
        for (const WordSlot &w : old)
            if (w.wid != NONE) {
                uint64_t s = word_slot_hash(w.key, w.len) & wmask;
                while (wtab[s].wid != NONE) s = (s + 1) & wmask;
                wtab[s] = w;
            }
        words_full = true;  // only the word table is re-uploaded (word ids do not change)
    }
    uint32_t word_intern(const uint8_t *p, uint32_t len) {
        uint32_t wid = word_lookup(p, len);
        if (wid != NONE) return wid;
        if ((word_off.size() + 1) * WORD_LOAD_INV > wtab.size()) word_rehash(wtab.size() * 2);
        WordSlot w{word_key(p, len), word_tag(len), (uint32_t)word_off.size()};
        word_off.push_back((uint32_t)warena.size());
        word_len.push_back(len);
        warena.insert(warena.end(), p, p + len);
        uint64_t s = word_slot_hash(w.key, w.len) & wmask;
        while (wtab[s].wid != NONE) s = (s + 1) & wmask;
        wtab[s] = w;
        dirty_wslots.push_back(s);
        return w.wid;
    }

    // =====================================================================
    // edges.  Host nodes are numbered in creation order (a parent before its
    // children); on the device a node is the index of its edge slot.
    uint32_t dev_id(uint32_t node) const { return node == ROOT ? ROOT_ID : node_slot[node]; }
    uint64_t edge_slots() const { return emask + 1; }
    static uint64_t emap_hash(uint32_t parent, uint32_t word) { return mix64(((uint64_t)parent << 32) | word); }
    // the child of host node `parent` by `word`, or NONE
    uint32_t child_of(uint32_t parent, uint32_t word) const {
        for (uint64_t i = emap_hash(parent, word) & emap_mask;; i = (i + 1) & emap_mask) {
            const EMapEnt &e = emap[i];
            if (e.parent == NONE) return NONE;
            if (e.parent == parent && e.word == word) return e.child;
        }
    }
    void emap_put(uint32_t parent, uint32_t word, uint32_t child) {
        uint64_t i = emap_hash(parent, word) & emap_mask;
        while (emap[i].parent != NONE) i = (i + 1) & emap_mask;
        emap[i] = EMapEnt{parent, word, child, 0};
    }
    void emap_rehash(uint64_t cap) {  // load <= 1/2
        emap.assign(cap, EMapEnt{NONE, 0, 0, 0});
        emap_mask = cap - 1;
        for (size_t v = 1; v < node_parent.size(); v++) emap_put(node_parent[v], node_word[v], (uint32_t)v);
    }
    bool slot_taken(uint64_t s) const { return (eocc[s >> 6] >> (s & 63)) & 1u; }
    // where the device's linear probe for (parent slot, word) ends: the first free slot
    uint64_t edge_place(uint32_t parent_dev, uint32_t word) const {
        uint64_t s = edge_home(parent_dev, word, emask);
        while (slot_taken(s)) s = next_slot(s, emask);
        return s;
    }
    // Re-place every node: slot positions hash the parent's slot, so nodes go in in
    // creation order (parents first).  Node ids on the device change: full upload.
    bool edge_full = false;  // the edge table hit MAX_EDGE_SLOTS at load 1/2: commit fails
    void edge_rehash(uint64_t cap) {
        eocc.assign(std::max<uint64_t>(cap / 64, 1), 0);
        emask = cap - 1;
        for (size_t v = 1; v < node_parent.size(); v++) {
            const uint64_t ns = edge_place(dev_id(node_parent[v]), node_word[v]);
            eocc[ns >> 6] |= 1ull << (ns & 63);
            node_slot[v] = (uint32_t)ns;
        }
        need_full = true;
    }
    // the device EdgeSlot of node v
    EdgeSlot edge_rec(uint32_t v) const { return EdgeSlot{dev_id(node_parent[v]), node_word[v], node_bloom[v], node_info[v]}; }
    void node_set_flag(uint32_t node, uint32_t f, uint32_t bloom) {
        if (node == ROOT) {
            if ((root.info & f) != f || (root.bloom & bloom) != bloom) {
                root.info |= f;
                root.bloom |= bloom;
                root_dirty = true;
            }
            return;
        }
        if ((node_info[node] & f) != f || (node_bloom[node] & bloom) != bloom) {
            node_info[node] |= f;
            node_bloom[node] |= bloom;
            dirty_enodes.push_back(node);
        }
    }
    uint32_t edge_child(uint32_t parent, uint32_t word) {
        const uint32_t c = child_of(parent, word);
        if (c != NONE) return c;
        if ((n_edges + 1) * edge_load_inv() > edge_slots()) {
            // a node is its slot index (u32, below the NONE/ROOT_ID sentinels): at the
            // size cap the table fills up to half instead of growing
            if (edge_slots() < MAX_EDGE_SLOTS) edge_rehash(std::min<uint64_t>(edge_slots() * 2, MAX_EDGE_SLOTS));
            else if ((n_edges + 1) * 2 > edge_slots()) {
                edge_full = true;
                return ROOT;  // dropped; commit() reports TM_ENOMEM
            }
        }
        const uint32_t child = (uint32_t)node_parent.size();
        node_parent.push_back(parent);
        node_word.push_back(word);
        node_slot.push_back(NONE);
        node_list.push_back(NodeList{0, 0, 0});
        node_cap.push_back(0);
        node_bloom.push_back(0);
        node_info.push_back(0);
        node_slist.push_back(0);
        const uint64_t s = edge_place(dev_id(parent), word);
        eocc[s >> 6] |= 1ull << (s & 63);
        node_slot[child] = (uint32_t)s;
        if ((n_edges + 2) * 2 > emap.size()) emap_rehash(std::max<uint64_t>(emap.size() * 2, 1024));
        else emap_put(parent, word, child);
        n_edges++;
        dirty_enodes.push_back(child);
        node_set_flag(parent, word == W_PLUS ? I_PLUS : I_LIT, word == W_PLUS ? 0u : bloom_bit(word));
        return child;
    }

    // =====================================================================
    // key set (linear probing over handles, backward-shift delete)
    static uint64_t key_hash(uint32_t node, uint8_t kind, uint64_t id) {
        return mix64(mix64(((uint64_t)node << 8) | kind) ^ id);
    }
    void kset_rehash(uint64_t cap) {
        hvec<uint32_t> old;
        old.swap(kset);
        kset.assign(cap, NONE);
        kmask = cap - 1;
        for (uint32_t h : old)
            if (h != NONE) {
                const KeyRec &k = keys[h];
                uint64_t s = key_hash(k.node, k.kind, k.id) & kmask;
                while (kset[s] != NONE) s = (s + 1) & kmask;
                kset[s] = h;
            }
    }
    uint32_t kset_find(uint32_t node, uint8_t kind, uint64_t id, uint64_t *slot_out) const {
        uint64_t s = key_hash(node, kind, id) & kmask;
        for (;;) {
            uint32_t h = kset[s];
            if (h == NONE) {
                if (slot_out) *slot_out = s;
                return NONE;
            }
            const KeyRec &k = keys[h];
            if (k.node == node && k.kind == kind && k.id == id) {
                if (slot_out) *slot_out = s;
                return h;
            }
            s = (s + 1) & kmask;
        }
    }
    void kset_erase_slot(uint64_t i) {
        // backward-shift deletion for linear probing
        uint64_t j = i;
        for (;;) {
            j = (j + 1) & kmask;
            uint32_t h = kset[j];
            if (h == NONE) break;
            const KeyRec &k = keys[h];
            uint64_t home = key_hash(k.node, k.kind, k.id) & kmask;
            // can the entry at j move to i?
            bool move = (i <= j) ? (home <= i || home > j) : (home <= i && home > j);
            if (move) {
                kset[i] = h;
                i = j;
            }
        }
        kset[i] = NONE;
        kset_used--;
    }
    uint32_t alloc_key() {
        if (!free_keys.empty()) {
            uint32_t h = free_keys.back();
            free_keys.pop_back();
            return h;
        }
        keys.push_back(KeyRec{NONE, K_FREE, {0, 0, 0}, 0});
        key_id32.push_back(0);
        dead_filter.emplace_back();
        return (uint32_t)(keys.size() - 1);
    }

    // =====================================================================
    // filter parsing: emqx_trie_search:filter/1 + make_key/2 (emqx_trie_search.erl:115-140,358-366)
    // Returns kind and the terminal node (creating the path when `create`).
    // Returns kind and the terminal node (creating the path when `create`); *depth_out =
    // the node's level count.  The walk may start below the root at a node known to lie
    // on the filter's path (hint_node at level hint_depth: resolve_all()).
    bool classify(const uint8_t *f, uint32_t flen, uint32_t flags, bool create, uint8_t *kind_out,
                  uint32_t *node_out, uint32_t *depth_out = nullptr, uint32_t hint_node = ROOT,
                  uint32_t hint_depth = 0) {
        // split on '/': tokens (emqx_topic.erl:276-278)
        std::vector<std::pair<uint32_t, uint32_t>> &lv = lv_scratch;  // (start, len)
        lv.clear();
        uint32_t st = 0;
        for (uint32_t i = 0; i <= flen; i++) {
            if (i == flen || f[i] == '/') {
                lv.push_back({st, i - st});
                st = i + 1;
            }
        }
        bool wild = false;
        int hash_pos = -1;
        for (size_t i = 0; i < lv.size(); i++) {
            const uint8_t *p = f + lv[i].first;
            if (lv[i].second == 1 && (*p == '+' || *p == '#')) wild = true;
            if (lv[i].second == 1 && *p == '#' && hash_pos < 0) hash_pos = (int)i;
        }
        if (hash_pos >= 0 && hash_pos != (int)lv.size() - 1) {
            *kind_out = K_DEAD;
            *node_out = NONE;
            return true;
        }
        uint8_t kind = !wild ? ((flags & TM_KEY_WORDS) ? K_EXACT_WORDS : K_EXACT_BIN)
                             : (hash_pos >= 0 ? K_HASH : K_WILD);
        size_t nwalk = (kind == K_HASH) ? lv.size() - 1 : lv.size();
        if (depth_out) *depth_out = (uint32_t)nwalk;
        uint32_t node = hint_depth <= nwalk ? hint_node : ROOT;
        for (size_t i = hint_depth <= nwalk ? hint_depth : 0; i < nwalk; i++) {
            const uint8_t *p = f + lv[i].first;
            uint32_t len = lv[i].second;
            uint32_t w;
            if (len == 1 && *p == '+') {
                w = W_PLUS;
            } else if (create) {
                w = word_intern(p, len);
            } else {
                w = word_lookup(p, len);
                if (w == NONE) return false;
            }
            if (create) {
                node = edge_child(node, w);
            } else {
                node = child_of(node, w);
                if (node == NONE) return false;
            }
        }
        *kind_out = kind;
        *node_out = node;
        return true;
    }

    // Deepest existing node on a filter's path (resolve_all), read-only (safe to run in
    // parallel before an epoch's ops are applied: nodes are never removed while ops apply).
    // The walk runs in slot space: a node's device id IS its edge slot (node_slot[v] == the
    // slot edge_find returns for v), so each level costs one edge-table probe, and the host
    // node id is looked up once, at the end.
    static void split_levels(const uint8_t *f, uint32_t flen, std::vector<std::pair<uint32_t, uint32_t>> &lv) {
        lv.clear();
        uint32_t st = 0;
        for (uint32_t i = 0; i <= flen; i++)
            if (i == flen || f[i] == '/') {
                lv.push_back({st, i - st});
                st = i + 1;
            }
    }
    // level d's word id for the prefix walk, or NONE to stop there ('#', unknown word)
    uint32_t prefix_word(const uint8_t *f, const std::pair<uint32_t, uint32_t> &l) const {
        const uint8_t *p = f + l.first;
        if (l.second == 1 && *p == '#') return NONE;
        return (l.second == 1 && *p == '+') ? W_PLUS : word_lookup(p, l.second);
    }
    // the shape test of key_ord() from the level count alone (no parent-chain walk)
    static bool deep_shape(uint8_t kind, uint32_t depth) {
        if (kind == K_HASH) return depth > 30;
        return (kind == K_EXACT_WORDS || kind == K_WILD) && depth > 31;
    }

    // known_kind: the op's key kind when its whole path existed before the epoch (resolve_all's
    // pkind): the key then hangs at hint_node, hint_depth levels down, and the filter need not
    // be parsed again (nodes are never removed while an epoch applies)
    void apply_one(const StagedOp &op, const uint8_t *ob, uint32_t hint_node = ROOT, uint32_t hint_depth = 0,
                   uint8_t known_kind = PK_NONE) {
        uint8_t kind;
        uint32_t node, depth = 0;
        const uint8_t *fp = ob + op.off;
        const bool known = known_kind != PK_NONE;
        if (known) {
            kind = known_kind;
            node = hint_node;
            depth = hint_depth;
        }
        if (op.op == TM_OP_ADD) {
            if (!known) classify(fp, op.len, op.flags, true, &kind, &node, &depth, hint_node, hint_depth);
            if (kind == K_DEAD) {
                auto key = std::make_pair(std::string((const char *)fp, op.len), op.id);
                if (dead_keys.count(key)) return;
                uint32_t h = alloc_key();
                keys[h] = KeyRec{NONE, K_DEAD, {0, 0, 0}, op.id};
                dead_filter[h] = key.first;
                dead_keys[key] = h;
                n_live++;
                return;
            }
            if ((kset_used + 1) * 2 > kset.size()) kset_rehash(kset.size() * 2);
            uint64_t slot;
            if (kset_find(node, kind, op.id, &slot) != NONE) return;  // set semantics
            uint32_t h = alloc_key();
            if (free_keys.size() > 8) {  // the handle the 8th ADD from now reuses (random, cold)
                const uint32_t nx = free_keys[free_keys.size() - 8];
                __builtin_prefetch(&keys[nx]);
                __builtin_prefetch(&key_id32[nx]);
            }
            keys[h] = KeyRec{node, kind, {0, 0, 0}, op.id};
            key_id32[h] = (uint32_t)op.id;
            if (deep_shape(kind, depth)) n_deep++;
            id_add(h);
            max_id = std::max(max_id, op.id);
            dirty_kid.push_back(h);
            kset[slot] = h;
            kset_used++;
            n_live++;
            deltas.push_back(Delta{node, h, (uint8_t)(kind == K_HASH), 1});
        } else if (op.op == TM_OP_DEL) {
            if (!known && !classify(fp, op.len, op.flags, false, &kind, &node, &depth, hint_node, hint_depth))
                return;  // idempotent
            if (kind == K_DEAD) {
                auto it = dead_keys.find(std::make_pair(std::string((const char *)fp, op.len), op.id));
                if (it == dead_keys.end()) return;
                uint32_t h = it->second;
                keys[h] = KeyRec{NONE, K_FREE, {0, 0, 0}, 0};
                dead_filter[h].clear();
                dead_keys.erase(it);
                free_pending.push_back(h);
                n_live--;
                return;
            }
            uint64_t slot;
            uint32_t h = kset_find(node, kind, op.id, &slot);
            if (h == NONE) return;
            kset_erase_slot(slot);
            deltas.push_back(Delta{node, h, (uint8_t)(kind == K_HASH), 0});
            if (deep_shape(kind, depth)) n_deep--;
            id_del(h);
            keys[h].kind = K_FREE;
            free_pending.push_back(h);
            n_live--;
        }
    }

    // An epoch's ops in order.  Their filter paths are first resolved against the trie as
    // it stands, in parallel (read-only, memory-latency bound: one dependent hash probe
    // per level); the ops then apply in order, each walk starting at its resolved prefix.
    // A prefix stays valid while ops apply (nodes are only ever added), and an op whose
    // path appears only during this epoch resumes from where resolution stopped.
    // nwalk[i]: levels of the trie path an ADD creates or reuses (0: no path).
    // pkind[i]: the key kind when the op's whole path already exists (its key would hang at
    // hnode[i]), else PK_NONE: the apply loop prefetches the key-set slot of such ops ahead.
    static constexpr uint8_t PK_NONE = 0xFF;
    // okind[i]: the op's key kind whether or not its path exists (PK_NONE: a dead key).
    void resolve_all(const std::vector<StagedOp> &ops, const uint8_t *ob, std::vector<uint32_t> &hnode,
                     std::vector<uint32_t> &hdepth, std::vector<uint32_t> &nwalk, std::vector<uint8_t> &pkind,
                     std::vector<uint8_t> &okind) const {
        const size_t n = ops.size();
        // ops in groups of GRP, their walks advanced one level at a time, so the map probes of
        // the group are in flight together (one dependent miss per level each)
        constexpr size_t GRP = 8;
        auto walk_group = [&](size_t i0, size_t i1, std::vector<std::pair<uint32_t, uint32_t>> (&lvs)[GRP]) {
            uint32_t cur[GRP], d[GRP], wnext[GRP];
            uint64_t nxt[GRP];
            bool live[GRP];
            const size_t m = i1 - i0;
            for (size_t k = 0; k < m; k++) {
                split_levels(ob + ops[i0 + k].off, ops[i0 + k].len, lvs[k]);
                cur[k] = ROOT;
                d[k] = 0;
                live[k] = true;
            }
            for (;;) {
                bool any = false;
                for (size_t k = 0; k < m; k++) {  // this level's word and first probe slot
                    if (!live[k]) continue;
                    const uint8_t *f = ob + ops[i0 + k].off;
                    if (d[k] >= lvs[k].size() || (wnext[k] = prefix_word(f, lvs[k][d[k]])) == NONE) {
                        live[k] = false;
                        continue;
                    }
                    nxt[k] = emap_hash(cur[k], wnext[k]) & emap_mask;
                    __builtin_prefetch(&emap[nxt[k]]);
                    any = true;
                }
                if (!any) break;
                for (size_t k = 0; k < m; k++) {  // the probes (their lines requested above)
                    if (!live[k]) continue;
                    uint32_t c = NONE;
                    for (uint64_t i = nxt[k];; i = (i + 1) & emap_mask) {
                        const EMapEnt &e = emap[i];
                        if (e.parent == NONE) break;
                        if (e.parent == cur[k] && e.word == wnext[k]) {
                            c = e.child;
                            break;
                        }
                    }
                    if (c == NONE) {
                        live[k] = false;
                        continue;
                    }
                    cur[k] = c;
                    d[k]++;
                }
            }
            for (size_t k = 0; k < m; k++) {
                hnode[i0 + k] = cur[k];
                hdepth[i0 + k] = d[k];
            }
        };
        auto one = [&](size_t i, std::vector<std::pair<uint32_t, uint32_t>> &lv) {
            const uint8_t *f = ob + ops[i].off;  // lv: its levels, hnode / hdepth: its walk (walk_group)
            // a '#' before the last level: a dead key, no path; a final '#': the path stops above it
            int hash_pos = -1;
            bool wild = false;
            for (size_t k = 0; k < lv.size(); k++)
                if (lv[k].second == 1 && (f[lv[k].first] == '#' || f[lv[k].first] == '+')) {
                    wild = true;
                    if (f[lv[k].first] == '#' && hash_pos < 0) hash_pos = (int)k;
                }
            const bool dead = hash_pos >= 0 && hash_pos != (int)lv.size() - 1;
            const uint32_t levels = (uint32_t)(hash_pos >= 0 ? lv.size() - 1 : lv.size());
            okind[i] = dead ? PK_NONE
                            : !wild ? ((ops[i].flags & TM_KEY_WORDS) ? K_EXACT_WORDS : K_EXACT_BIN)
                                    : (hash_pos >= 0 ? K_HASH : K_WILD);
            pkind[i] = hdepth[i] == levels ? okind[i] : PK_NONE;
            if (ops[i].op != TM_OP_ADD) return;
            nwalk[i] = dead ? 0 : levels;
        };
        // memory-latency bound (a dependent miss per level): up to 16 threads from 2 K ops on
        const unsigned nt = n < 2048 ? 1u : (unsigned)std::min<size_t>(commit_threads(), n / 128);
        auto range = [&](unsigned k, unsigned nthreads) {  // a contiguous range of ops per thread
            std::vector<std::pair<uint32_t, uint32_t>> lvs[GRP];
            const size_t hi = n * (k + 1) / nthreads;
            for (size_t g = n * k / nthreads; g < hi; g += GRP) {
                const size_t e = std::min(hi, g + GRP);
                walk_group(g, e, lvs);
                for (size_t i = g; i < e; i++) one(i, lvs[i - g]);
            }
        };
        pool.run(nt, [&](unsigned k) { range(k, nt); });
    }

    // Recompute a node's emission bits from its list (and keep its I_PLUS/I_LIT):
    // a single key goes inline into the slot; otherwise the counts go inline and the
    // list offset stays in slot_list (M_CNT), or, for huge lists, the walk reads the
    // counts from the list header (M_REC).
    void refresh_info(uint32_t node) { refresh_info_to(node, dirty_enodes, dirty_lnodes); }
    // the same, recording the nodes whose device records change in the given vectors (several
    // threads at once on different nodes below the root: apply_deltas)
    void refresh_info_to(uint32_t node, std::vector<uint64_t> &d_enodes, std::vector<uint64_t> &d_lnodes) {
        const NodeList &r = node_list[node];
        if (node == ROOT) {
            root.list_off = r.list_off;
            root.hash_cnt = r.hash_cnt;
            root_dirty = true;
            return;
        }
        uint32_t info = node_info[node] & I_KIDS;
        const uint32_t n = r.term_cnt + r.hash_cnt;
        if (n == 1 && arena[r.list_off] < INLINE_KEY_LIMIT)
            info |= (M_INLINE << I_MODE_SHIFT) | (r.hash_cnt ? I_INL_HASH : 0u) | arena[r.list_off];
        else if (n && r.term_cnt <= CNT_MAX && r.hash_cnt <= CNT_MAX)
            info |= (M_CNT << I_MODE_SHIFT) | (r.term_cnt << CNT_BITS) | r.hash_cnt;
        else if (n)
            info |= M_REC << I_MODE_SHIFT;
        if (info != node_info[node]) {
            node_info[node] = info;
            if (!need_full) d_enodes.push_back(node);
        }
        if (node_slist[node] != r.list_off) {
            node_slist[node] = r.list_off;
            if (!need_full) d_lnodes.push_back(node);
        }
    }

    // The list header (layout.h LIST_HDR words before the first key):
    //   [min bin-term key, min word-term key, min '#' key, term_cnt, hash_cnt]
    // where "min" = the key with the smallest id of that kind (NONE if none).  A node's keys
    // all spell the same filter per kind, so these are the return_first candidates
    // (k_match_first) without scanning the list.
    // the KDD_* flags a key carries on the device (key_dev_rec), OR'd into its list's header
    uint32_t key_dd_bits(uint32_t h) const {
        const KeyRec &k = keys[h];
        return ((k._p[0] & KR_MULTI) ? KDD_MULTI : 0u) | ((k.id & TM_ID_SHARED) ? KDD_SHARED : 0u);
    }
    void write_header(uint32_t pos, const uint32_t *terms, uint32_t tc, const uint32_t *hashes, uint32_t hc) {
        uint32_t mb = NONE, mw = NONE, mh = NONE, dd = 0;
        auto take = [&](uint32_t &m, uint32_t h) {
            if (m == NONE || keys[h].id < keys[m].id) m = h;
            dd |= key_dd_bits(h);
        };
        for (uint32_t i = 0; i < tc; i++) take(keys[terms[i]].kind == K_EXACT_BIN ? mb : mw, terms[i]);
        for (uint32_t i = 0; i < hc; i++) take(mh, hashes[i]);
        arena[pos - HDR_DD] = dd;
        arena[pos - 5] = mb;
        arena[pos - 4] = mw;
        arena[pos - 3] = mh;
        arena[pos - 2] = tc;
        arena[pos - 1] = hc;
    }

    // Append one list (header, term keys, hash keys) to the arena.
    // cap >= tc + hc keys are reserved (the slack lets later epochs edit the list in place).
    NodeList append_list(const uint32_t *terms, uint32_t tc, const uint32_t *hashes, uint32_t hc, uint32_t cap = 0) {
        if (tc + hc == 0) return NodeList{0, 0, 0};
        arena.resize(arena.size() + LIST_HDR);
        const uint32_t off = (uint32_t)arena.size();
        arena.insert(arena.end(), terms, terms + tc);
        arena.insert(arena.end(), hashes, hashes + hc);
        if (cap > tc + hc) arena.resize(arena.size() + (cap - tc - hc), 0u);
        write_header(off, terms, tc, hashes, hc);
        ids_of(off, (uint64_t)off + tc + hc);
        return NodeList{off, tc, hc};
    }

    // Rebuild the whole arena from the key table (counting sort by node).
    void rebuild_arena() {
        need_full = true;  // everything is re-uploaded: no dirty tracking
        ids_stale = false;
        size_t nn = node_parent.size();
        std::vector<uint32_t> tcnt(nn, 0), hcnt(nn, 0);
        for (size_t h = 0; h < keys.size(); h++) {
            const KeyRec &k = keys[h];
            if (k.kind == K_FREE || k.kind == K_DEAD) continue;
            if (k.kind == K_HASH) hcnt[k.node]++;
            else tcnt[k.node]++;
        }
        std::vector<uint32_t> pos(nn);
        uint64_t total = 0;
        for (size_t v = 0; v < nn; v++) {
            const uint32_t n = tcnt[v] + hcnt[v];
            pos[v] = n ? (uint32_t)(total + LIST_HDR) : 0u;
            total += n ? n + LIST_HDR : 0;
        }
        arena.assign(total, 0);
        std::vector<uint32_t> tfill(pos), hfill(nn);
        for (size_t v = 0; v < nn; v++) hfill[v] = pos[v] + tcnt[v];
        for (size_t h = 0; h < keys.size(); h++) {
            const KeyRec &k = keys[h];
            if (k.kind == K_FREE || k.kind == K_DEAD) continue;
            if (k.kind == K_HASH) arena[hfill[k.node]++] = (uint32_t)h;
            else arena[tfill[k.node]++] = (uint32_t)h;
        }
        node_cap.assign(nn, 0);
        // per node: disjoint arena ranges and node records, so in parallel (random reads of the
        // key records for the headers and ids); the root's record apart
        std::vector<uint64_t> none_e, none_l;  // need_full: refresh_info_to records nothing
        par_for(nn, [&](size_t v) {
            node_list[v] = NodeList{pos[v], tcnt[v], hcnt[v]};
            node_cap[v] = tcnt[v] + hcnt[v];
            if (pos[v]) {
                write_header(pos[v], &arena[pos[v]], tcnt[v], &arena[pos[v] + tcnt[v]], hcnt[v]);
                ids_of(pos[v], (uint64_t)pos[v] + tcnt[v] + hcnt[v]);
            }
            if (v != ROOT) refresh_info_to((uint32_t)v, none_e, none_l);
        });
        refresh_info(ROOT);
        arena_garbage = 0;
        need_full = true;
    }

    // Fold this epoch's deltas into the arena.  Per dirty node, in parallel (read-only on the
    // host copy): its new key list, the list header's minima and the ids of its keys, i.e.
    // every random read of the key records a list needs.  Then in node order, sequentially:
    // the list is rewritten in place when it fits its room, else appended (the arena grows).
    struct NewList {
        std::vector<uint32_t> keys;  // term keys, then '#' keys
        std::vector<uint64_t> ids;   // their ids (the host id arena's words)
        uint32_t tc = 0, hc = 0, mb = NONE, mw = NONE, mh = NONE, dd = 0;
    };
    void build_list(size_t i, size_t j, NewList &L) const {
        const uint32_t node = deltas[i].node;
        const NodeList r = node_list[node];
        std::vector<uint32_t> terms(arena.begin() + r.list_off, arena.begin() + r.list_off + r.term_cnt);
        std::vector<uint32_t> hashes(arena.begin() + r.list_off + r.term_cnt,
                                     arena.begin() + r.list_off + r.term_cnt + r.hash_cnt);
        for (size_t k = i; k < j; k++) {
            std::vector<uint32_t> &Lst = deltas[k].hash ? hashes : terms;
            if (deltas[k].add) {
                Lst.push_back(deltas[k].key);
            } else {
                auto it = std::find(Lst.begin(), Lst.end(), deltas[k].key);
                if (it != Lst.end()) Lst.erase(it);
            }
        }
        L.tc = (uint32_t)terms.size();
        L.hc = (uint32_t)hashes.size();
        L.keys = std::move(terms);
        L.keys.insert(L.keys.end(), hashes.begin(), hashes.end());
        L.ids.resize(L.keys.size());
        auto take = [&](uint32_t &m, uint32_t h) {
            if (m == NONE || keys[h].id < keys[m].id) m = h;
        };
        for (uint32_t q = 0; q < L.tc + L.hc; q++) {
            const uint32_t h = L.keys[q];
            L.ids[q] = keys[h].id;
            L.dd |= key_dd_bits(h);
            if (q < L.tc) take(keys[h].kind == K_EXACT_BIN ? L.mb : L.mw, h);
            else take(L.mh, h);
        }
    }
    void place_header(uint32_t pos, const NewList &L) {
        arena[pos - HDR_DD] = L.dd;
        arena[pos - 5] = L.mb;
        arena[pos - 4] = L.mw;
        arena[pos - 3] = L.mh;
        arena[pos - 2] = L.tc;
        arena[pos - 1] = L.hc;
    }
    // returns false when the list ran past the id arena's reservation (ids_stale: the commit
    // compacts); several threads may place different lists at once
    bool place_ids(uint64_t pos, const NewList &L) {
        if (!arena_id) return true;
        uint64_t n = L.ids.size();
        bool ok = true;
        if (pos + n > arena_id_res) {  // past the reservation: only until the compaction this forces
            ok = false;
            n = pos < arena_id_res ? arena_id_res - pos : 0;
        }
        if (n) memcpy(arena_id + pos, L.ids.data(), n * 8);
        if (arena_id32)
            for (uint64_t i = 0; i < n; i++) arena_id32[pos + i] = (uint32_t)L.ids[i];
        return ok;
    }
    uint64_t ad_us[3] = {};  // the last apply_deltas: sort + list builds, in-place rewrites, moves
    size_t ad_groups = 0, ad_inplace = 0;
    void apply_deltas() {
        uint64_t ta = now_us();
        // grouped by node, in op order within a node (the last op on a key wins): a stable
        // LSD radix sort on the node id (std::stable_sort of 20 K deltas: ~1 ms)
        if (deltas.size() < 2048) {
            std::stable_sort(deltas.begin(), deltas.end(), [](const Delta &a, const Delta &b) { return a.node < b.node; });
        } else {
            std::vector<Delta> t(deltas.size());
            uint32_t cnt[2048];
            for (int sh = 0; sh < 33; sh += 11) {
                std::fill(cnt, cnt + 2048, 0u);
                for (const Delta &d : deltas) cnt[(d.node >> sh) & 2047]++;
                uint32_t acc = 0;
                for (uint32_t &c : cnt) {
                    const uint32_t k = c;
                    c = acc;
                    acc += k;
                }
                for (const Delta &d : deltas) t[cnt[(d.node >> sh) & 2047]++] = d;
                deltas.swap(t);
            }
        }
        std::vector<size_t> gs;  // group g: deltas [gs[g], gs[g + 1]) of one node
        for (size_t i = 0; i < deltas.size(); i++)
            if (i == 0 || deltas[i].node != deltas[i - 1].node) gs.push_back(i);
        gs.push_back(deltas.size());
        const size_t G = gs.size() - 1;
        std::vector<NewList> nl(G);
        // several dependent misses per node (its list, the key records): helpers from 512 nodes
        const unsigned nt = G < 512 ? 1u : (unsigned)std::min<size_t>(commit_threads(), G / 128);
        pool.run(nt, [&](unsigned k) {  // contiguous ranges: neighbouring nodes share lines
            for (size_t g = G * k / nt, e = G * (k + 1) / nt; g < e; g++) build_list(gs[g], gs[g + 1], nl[g]);
        });
        ad_us[0] = now_us() - ta;
        ta = now_us();
        // Where each list goes: lists that fit their room are rewritten in place; the others
        // move to the arena's tail, their offsets handed out here in node order (the root's
        // list always stays on this thread).  Then every list is written in parallel: disjoint
        // arena ranges, nodes and slots (the dirty records per thread, merged after).
        std::vector<uint8_t> inplace(G, 0);
        std::vector<uint32_t> dst(G, 0), room(G, 0);
        size_t n_in = 0;
        uint64_t tail = arena.size();
        for (size_t g = 0; g < G; g++) {
            const uint32_t node = deltas[gs[g]].node;
            const NodeList &r = node_list[node];
            const uint32_t k = nl[g].tc + nl[g].hc, cap = node_cap[node];
            if (node == ROOT) continue;
            if (r.list_off && k && k <= cap) {
                inplace[g] = 1;
                n_in++;
                dst[g] = r.list_off;
                room[g] = cap;
                continue;
            }
            arena_garbage += cap + (r.list_off ? LIST_HDR : 0);
            // lists of 16 keys or more get a quarter more room when they move
            room[g] = k >= 16 ? k + k / 4 : k;
            if (k) {
                dst[g] = (uint32_t)(tail + LIST_HDR);
                tail += LIST_HDR + room[g];
            }
        }
        arena.resize(tail, 0u);  // the moved lists' room (zero past their keys)
        auto place = [&](size_t g, std::vector<uint64_t> &da, std::vector<uint64_t> &de,
                         std::vector<uint64_t> &dl) -> bool {
            const uint32_t node = deltas[gs[g]].node;
            NewList &L = nl[g];
            const uint32_t tc = L.tc, hc = L.hc, off = dst[g];
            bool ok = true;
            if (tc + hc) {
                std::copy(L.keys.begin(), L.keys.end(), arena.begin() + off);
                place_header(off, L);
                ok = place_ids(off, L);
                if (inplace[g])  // words already on the device, rewritten in place
                    for (uint64_t w = off - LIST_HDR; w < (uint64_t)off + tc + hc; w++)
                        if (w < arena_dev) da.push_back(w);
                node_list[node] = NodeList{off, tc, hc};
            } else {
                node_list[node] = NodeList{0, 0, 0};
            }
            node_cap[node] = tc + hc ? room[g] : 0;
            refresh_info_to(node, de, dl);
            return ok;
        };
        const unsigned nt2 = G < 1024 ? 1u : (unsigned)std::min<size_t>(commit_threads(), G / 256);
        std::vector<std::vector<uint64_t>> da(nt2), de(nt2), dl(nt2);
        std::vector<uint8_t> stale(nt2, 0);
        pool.run(nt2, [&](unsigned k) {  // contiguous ranges: neighbouring nodes share lines
            for (size_t g = G * k / nt2, e = G * (k + 1) / nt2; g < e; g++)
                if (deltas[gs[g]].node != ROOT && !place(g, da[k], de[k], dl[k])) stale[k] = 1;
        });
        for (unsigned k = 0; k < nt2; k++) {
            dirty_arena.insert(dirty_arena.end(), da[k].begin(), da[k].end());
            dirty_enodes.insert(dirty_enodes.end(), de[k].begin(), de[k].end());
            dirty_lnodes.insert(dirty_lnodes.end(), dl[k].begin(), dl[k].end());
            if (stale[k]) ids_stale = true;
        }
        ad_us[1] = now_us() - ta;
        ta = now_us();
        for (size_t g = 0; g < G; g++) {  // the root's list (its record lives apart from the slots)
            const uint32_t node = deltas[gs[g]].node;
            if (node != ROOT) continue;
            const NodeList r = node_list[node];
            NewList &L = nl[g];
            const uint32_t tc = L.tc, hc = L.hc, cap = node_cap[node];
            if (r.list_off && tc + hc && tc + hc <= cap) {
                std::copy(L.keys.begin(), L.keys.end(), arena.begin() + r.list_off);
                place_header(r.list_off, L);
                if (!place_ids(r.list_off, L)) ids_stale = true;
                for (uint64_t w = r.list_off - LIST_HDR; w < (uint64_t)r.list_off + tc + hc; w++)
                    if (w < arena_dev) dirty_arena.push_back(w);
                node_list[node] = NodeList{r.list_off, tc, hc};
            } else {
                arena_garbage += cap + (r.list_off ? LIST_HDR : 0);
                const uint32_t rm = tc + hc >= 16 ? tc + hc + (tc + hc) / 4 : tc + hc;
                if (tc + hc == 0) {
                    node_list[node] = NodeList{0, 0, 0};
                } else {
                    arena.resize(arena.size() + LIST_HDR);
                    const uint32_t off = (uint32_t)arena.size();
                    arena.insert(arena.end(), L.keys.begin(), L.keys.end());
                    if (rm > tc + hc) arena.resize(arena.size() + (rm - tc - hc), 0u);
                    place_header(off, L);
                    if (!place_ids(off, L)) ids_stale = true;
                    node_list[node] = NodeList{off, tc, hc};
                }
                node_cap[node] = tc + hc ? rm : 0;
            }
            refresh_info(node);
        }
        ad_us[2] = now_us() - ta;
        ad_groups = G;
        ad_inplace = n_in;
    }

    // ---- device upload.  Every allocation of a publish comes before its first in-place
    // write, and a replaced buffer is allocated before the old one is freed, so a publish that
    // fails (out of HBM) leaves the device holding the previous epoch intact.

    // Replace array a's device buffer with one holding h (headroom num/den), allocated first.
    template <class V, class T = typename V::value_type>
    hipError_t replace_whole(DevBuf &d, uint32_t a, const V &h, size_t num = 3, size_t den = 2) {
        const size_t bytes = h.size() * sizeof(T);
        DevBuf nb;
        hipError_t e = nb.ensure(std::max<size_t>(bytes * num / den, 4096));
        if (e) return e;
        if (bytes && (e = upload(nb.p, h.data(), bytes, stream))) {
            nb.release();
            return e;
        }
        if ((e = hipStreamSynchronize(stream))) {
            nb.release();
            return e;
        }
        std::swap(d.p, nb.p);
        std::swap(d.cap, nb.cap);
        nb.release();
        dev_used[a] = bytes;
        patch.add(P_WHOLE, a, bytes / ARR_ELEM[a], d.cap, h.data(), bytes);
        return hipSuccess;
    }
    // the host array's new tail, staged with the epoch's scatters (one pinned H2D, then a
    // device-side copy into place): a pageable H2D per array cost ~0.2-0.5 ms of a delta commit
    template <class V, class T = typename V::value_type>
    hipError_t put_tail(DevBuf &d, const V &h, size_t &dev_n) {
        if (h.size() <= dev_n) return hipSuccess;
        const size_t bytes = (h.size() - dev_n) * sizeof(T);
        sjobs.push_back(SJob{0, d.as<T>() + dev_n, bytes, 0, stage_bytes_add(h.data() + dev_n, bytes)});
        const hipError_t e = hipSuccess;
        const uint32_t a = arr_of(&d);
        if (a < A_N) {
            patch.add(P_TAIL, a, (h.size() - dev_n) * sizeof(T) / ARR_ELEM[a], dev_n * sizeof(T) / ARR_ELEM[a],
                      h.data() + dev_n, (h.size() - dev_n) * sizeof(T));
            dev_used[a] = h.size() * sizeof(T);
        }
        dev_n = h.size();
        return e;
    }

    // key handle -> {id, order code}, device node slot, binary flag
    void key_dev_rec(uint32_t h, uint64_t *rec, uint32_t *node, uint32_t *bin, uint8_t *dd) const {
        const KeyRec &k = keys[h];
        rec[0] = k.id;
        (void)key_ord(h, &rec[1]);
        const bool live = k.kind != K_FREE && k.kind != K_DEAD;
        *node = live ? dev_id(k.node) : NONE;
        *bin = k.kind == K_EXACT_BIN ? 1u : 0u;
        *dd = (uint8_t)(((k._p[0] & KR_MULTI) ? KDD_MULTI : 0) | ((k.id & TM_ID_SHARED) ? KDD_SHARED : 0));
    }
    struct KeyArrays {
        std::vector<uint64_t> rec;
        std::vector<uint32_t> node, bin;
        std::vector<uint8_t> dd;
    };
    KeyArrays h_ka;  // kept between full publishes, as h_nim
    void key_arrays(KeyArrays &k) const {
        k.rec.resize(keys.size() * 2);
        k.node.resize(keys.size());
        k.bin.resize(keys.size());
        k.dd.resize(keys.size());
        par_for(keys.size(), [&](size_t h) { key_dev_rec((uint32_t)h, &k.rec[2 * h], &k.node[h], &k.bin[h], &k.dd[h]); });
    }

    // Full publish into a STANDBY image: every array is uploaded into fresh buffers on s_build
    // while matches keep running on the current image (mu_dev is not held); then, under
    // mu_dev, the in-flight matches drain and the buffers swap.  At config C that is ~20 GiB
    // uploaded beside the match path; the match path stalls only for the swap.
    // Full-publish uploads go through this pinned ring, never straight from pageable host
    // memory: the HIP runtime pins a large pageable source on the fly (a driver mapping of the
    // host range), and unmapping that range again (the runtime's unpin, or the free of the host
    // vector at the end of the commit) makes the driver invalidate the process's GPU mappings
    // beside the matches.  Two chunks, each filled by the commit's helper threads while the
    // other one's DMA runs.
    static constexpr size_t UP_CHUNK = size_t(32) << 20;
    PinBuf up_pin[2];
    hipEvent_t up_ev[2] = {};
    uint32_t up_next = 0;
    hipError_t upload(void *dst, const void *src, size_t bytes, hipStream_t s) {
        for (size_t at = 0; at < bytes; at += UP_CHUNK) {
            const size_t n = std::min(UP_CHUNK, bytes - at);
            const uint32_t k = up_next++ & 1u;
            hipError_t e;
            if (!up_ev[k]) {
                if ((e = hipEventCreateWithFlags(&up_ev[k], hipEventDisableTiming))) return e;
            } else if ((e = hipEventSynchronize(up_ev[k]))) {  // the chunk's previous DMA is done
                return e;
            }
            if ((e = up_pin[k].ensure(UP_CHUNK))) return e;
            uint8_t *pin = up_pin[k].as<uint8_t>();
            const uint8_t *from = static_cast<const uint8_t *>(src) + at;
            const unsigned nt = n < (size_t(4) << 20) ? 1u : std::min(8u, commit_threads());
            pool.run(nt, [&](unsigned j) {
                const size_t a = n * j / nt, b = n * (j + 1) / nt;
                std::memcpy(pin + a, from + a, b - a);
            });
            if ((e = hipMemcpyAsync(static_cast<uint8_t *>(dst) + at, pin, n, hipMemcpyHostToDevice, s))) return e;
            if ((e = hipEventRecord(up_ev[k], s))) return e;
        }
        return hipSuccess;
    }
    void upload_release() {
        for (uint32_t k = 0; k < 2; k++) {
            if (up_ev[k]) {
                (void)hipEventSynchronize(up_ev[k]);
                (void)hipEventDestroy(up_ev[k]);
                up_ev[k] = nullptr;
            }
            up_pin[k].release();
        }
    }
    // Full publish into a STANDBY image: every array is uploaded into fresh buffers on s_build
    // while matches keep running on the current image (mu_dev is not held); then, under
    // mu_dev, the in-flight matches drain and the buffers swap.  At config C that is ~20 GiB
    // uploaded beside the match path; the match path stalls only for the swap.
    uint32_t pub_reallocs = 0;  // device buffers (re)allocated by the last full publish
    template <class V, class T = typename V::value_type>
    hipError_t stage_to(DevBuf &d, const V &h, hipStream_t s, uint64_t *used, size_t num = 3, size_t den = 2) {
        const size_t bytes = h.size() * sizeof(T);
        // a standby buffer that holds the array is reused as it is (no allocation beside the
        // matches); a new one gets headroom for the delta commits that follow
        hipError_t e = hipSuccess;
        if (!(d.p && bytes <= d.cap)) {
            e = d.ensure(std::max<size_t>(bytes * num / den, 4096));
            pub_reallocs++;
        }
        if (e) return e;
        if (bytes && (e = upload(d.p, h.data(), bytes, s))) return e;
        *used = bytes;
        return hipSuccess;
    }
    // steady-clock microseconds of the last full publish's steps (tm_debug_commit_marks):
    // start, node image uploaded, edge table built, arrays staged, upload synced, swap begin,
    // swap end, standby kept
    uint64_t pub_marks[8] = {};
    DevBuf d_nim;  // the node image the edge table is built from (kept between full publishes)
    // The host arrays a full publish fills, kept between publishes (≈ 1.8 GB at config C): a
    // fresh 1.5 GB node image per rebuild was first-touched by 14 helper threads, and those page
    // faults held the process's address-space lock against everything else mapping memory
    // beside them (a 10 ms match in the rebuild probe, profiles/r06_rebuild_probe_rb1.jsonl)
    hvec<NodeImage> h_nim;
    uint64_t last_swap_us = 0;  // mu_dev held by the last full publish's swap (tm_stats)
    // The standby image (round 5).  A full publish used to allocate ~20 GiB of fresh buffers
    // (config C) beside the matches and hipFree the previous image after the swap; both stall
    // the match path (hipFree synchronises the device: a 25 ms match on the driver's box).  Now
    // the previous image's buffers are kept and the next full publish uploads into them; the
    // first full publish of a sizable index also sets up a standby of the same capacities (at
    // build time, not during a later rebuild).  Kept only while the device has room for it.
    DevBuf standby[A_N];
    uint64_t standby_bytes() const {
        uint64_t b = 0;
        for (const DevBuf &d : standby) b += d.cap;
        return b;
    }
    static bool standby_wanted() {
        static const bool on = [] {
            const char *e = getenv("EMQX_TM_STANDBY");
            return !(e && *e == '0');
        }();
        return on;
    }
    // room for `extra` more bytes of standby while leaving a quarter of the device free
    static bool standby_room(uint64_t extra) {
        size_t fr = 0, tot = 0;
        if (hipMemGetInfo(&fr, &tot) != hipSuccess) return false;
        return extra + tot / 4 <= fr;
    }
    void standby_release() {
        for (DevBuf &d : standby) d.release();
        d_nim.release();
    }
    // after a swap: the previous image (sb) becomes the standby, grown to the live image's
    // capacities when the device has room (else dropped: the next full publish allocates)
    void standby_keep(DevBuf (&sb)[A_N]) {
        for (uint32_t a = 0; a < A_N; a++) {
            std::swap(standby[a].p, sb[a].p);
            std::swap(standby[a].cap, sb[a].cap);
        }
        for (DevBuf &d : sb) d.release();  // only non-empty if standby was not empty (never)
        if (!standby_wanted()) {
            standby_release();
            return;
        }
        uint64_t grow = 0;
        for (uint32_t a = 0; a < A_N; a++) {
            const DevBuf *live = arr_buf(a);
            if (standby[a].cap < live->cap) grow += live->cap;
        }
        if (!grow) return;
        if (!standby_room(grow)) {
            standby_release();
            return;
        }
        for (uint32_t a = 0; a < A_N; a++) {
            const DevBuf *live = arr_buf(a);
            if (standby[a].cap < live->cap && standby[a].ensure(live->cap) != hipSuccess) {
                (void)hipGetLastError();
                standby_release();
                return;
            }
        }
    }
    hipError_t publish_full() {
        drop_scatters();  // nothing a failed delta staged may replay into the buffers this frees
        patch.reset();
        patch.full = true;  // replicas reload from an image
        DevBuf sb[A_N];
        for (uint64_t &m : pub_marks) m = 0;
        pub_marks[0] = now_us();
        pub_reallocs = 0;
        for (uint32_t a = 0; a < A_N; a++) {  // upload into the standby image's buffers
            std::swap(sb[a].p, standby[a].p);
            std::swap(sb[a].cap, standby[a].cap);
        }
        uint64_t used[A_N] = {};
        KeyArrays &ka = h_ka;
        key_arrays(ka);
        hipStream_t s = s_build;
        hipError_t e;
        auto fail = [&](hipError_t err) {
            (void)hipStreamSynchronize(s);
            for (DevBuf &b : sb) b.release();
            return err;
        };
        // the edge table and slot lists: reused when the standby holds them (ensure keeps a
        // buffer at least as large)
        // the edge table: built on the device from one record per node
        hvec<NodeImage> &nim = h_nim;
        nim.resize(node_parent.size() - 1);
        par_for(nim.size(), [&](size_t i) {
            const uint32_t v = (uint32_t)i + 1;
            const EdgeSlot r = edge_rec(v);
            nim[i] = NodeImage{node_slot[v], r.parent, r.word, r.bloom, r.info, node_slist[v]};
        });
        const uint64_t slots = edge_slots();
        const size_t nim_bytes = std::max<size_t>(nim.size() * sizeof(NodeImage), 4096);
        const bool grow_nim = d_nim.cap < nim_bytes, grow_etab = sb[A_ETAB].cap < slots * sizeof(EdgeSlot) || !sb[A_ETAB].p,
                   grow_sl = sb[A_SLOT_LIST].cap < slots * 4 || !sb[A_SLOT_LIST].p;
        pub_reallocs += grow_nim + grow_etab + grow_sl;
        if ((e = sb[A_ETAB].ensure(slots * sizeof(EdgeSlot))) || (e = sb[A_SLOT_LIST].ensure(slots * 4)) ||
            (e = d_nim.ensure(grow_nim ? nim_bytes + nim_bytes / 4 : nim_bytes)) ||
            (nim.size() && (e = upload(d_nim.p, nim.data(), nim.size() * sizeof(NodeImage), s))))
            return fail(e);
        pub_marks[1] = now_us();
        if ((e = edge_image_paced(sb[A_ETAB].as<uint4>(), sb[A_SLOT_LIST].as<uint32_t>(), slots, d_nim.as<NodeImage>(),
                                  nim.size(), s, std::min(sb[A_ETAB].cap / 16, sb[A_SLOT_LIST].cap / 4))) ||
            (e = bnd_after(s, "edge image")) || (e = hipStreamSynchronize(s)))
            return fail(e);
        pub_marks[2] = now_us();
        used[A_ETAB] = slots * sizeof(EdgeSlot);
        used[A_SLOT_LIST] = slots * 4;
        if ((e = stage_to(sb[A_WTAB], wtab, s, &used[A_WTAB], 1, 1)) || (e = stage_to(sb[A_WARENA], warena, s, &used[A_WARENA])) ||
            (e = stage_to(sb[A_WORD_OFF], word_off, s, &used[A_WORD_OFF])) ||
            (e = stage_to(sb[A_ARENA], arena, s, &used[A_ARENA])) || (e = stage_to(sb[A_KEY_REC], ka.rec, s, &used[A_KEY_REC])) ||
            (e = stage_to(sb[A_KEY_NODE], ka.node, s, &used[A_KEY_NODE])) ||
            (e = stage_to(sb[A_KEY_BIN], ka.bin, s, &used[A_KEY_BIN])) ||
            (e = stage_to(sb[A_KEY_DD], ka.dd, s, &used[A_KEY_DD])) || (e = sb[A_ROOT].ensure(sizeof(RootRec))) ||
            (e = hipMemcpyAsync(sb[A_ROOT].p, &root, sizeof(RootRec), hipMemcpyHostToDevice, s)))
            return fail(e);
        used[A_ROOT] = sizeof(RootRec);
        pub_marks[3] = now_us();
        if ((e = hipStreamSynchronize(s))) return fail(e);
        pub_marks[4] = now_us();
        {
            std::lock_guard<std::recursive_mutex> g(mu_dev);
            const uint64_t t0 = now_us();
            pub_marks[5] = t0;
            if ((e = quiesce())) return fail(e);  // matches in flight finish on the old image
            for (uint32_t a = 0; a < A_N; a++) {
                DevBuf *d = arr_buf(a);
                std::swap(d->p, sb[a].p);
                std::swap(d->cap, sb[a].cap);
                dev_used[a] = used[a];
            }
            warena_dev = warena.size();
            word_off_dev = word_off.size();
            arena_dev = arena.size();
            dirty_kid.clear();
            set_view();
            pub_marks[6] = now_us();
            last_swap_us = pub_marks[6] - t0;
        }
        standby_keep(sb);  // the previous image (nothing in flight reads it) is the next standby
        pub_marks[7] = now_us();
        return hipSuccess;
    }

    hipError_t upload_key_ids_delta() {
        if (dirty_kid.empty()) return hipSuccess;
        sort_unique(dirty_kid);
        const size_t n = dirty_kid.size();
        std::vector<uint64_t> idx(n), rec(2 * n);
        std::vector<uint32_t> node(n), bin(n);
        std::vector<uint8_t> dd(n);
        par_for(n, [&](size_t i) {
            idx[i] = dirty_kid[i];
            key_dev_rec((uint32_t)dirty_kid[i], &rec[2 * i], &node[i], &bin[i], &dd[i]);
        });
        dirty_kid.clear();
        patch.add(P_SCATTER, A_KEY_REC, n, 0, idx.data(), n * 8, rec.data(), n * 16);
        patch.add(P_SCATTER, A_KEY_BIN, n, 0, idx.data(), n * 8, bin.data(), n * 4);
        patch.add(P_SCATTER, A_KEY_NODE, n, 0, idx.data(), n * 8, node.data(), n * 4);
        patch.add(P_SCATTER, A_KEY_DD, n, 0, idx.data(), n * 8, dd.data(), n);
        // handles past the arrays' used part (inside their capacity) extend it
        const uint64_t top = idx[n - 1] + 1;
        for (uint32_t a : {A_KEY_REC, A_KEY_BIN, A_KEY_NODE, A_KEY_DD})
            dev_used[a] = std::max<uint64_t>(dev_used[a], top * ARR_ELEM[a]);
        const size_t io = stage_bytes_add(idx.data(), n * 8);
        sjobs.push_back(SJob{16, d_key_rec.p, n, io, stage_bytes_add(rec.data(), n * 16)});
        sjobs.push_back(SJob{4, d_key_bin.p, n, io, stage_bytes_add(bin.data(), n * 4)});
        sjobs.push_back(SJob{4, d_key_node.p, n, io, stage_bytes_add(node.data(), n * 4)});
        sjobs.push_back(SJob{1, d_key_dd.p, n, io, stage_bytes_add(dd.data(), n)});
        return hipSuccess;
    }

    // A delta commit's scatters are staged into one blob (indices and values of every array),
    // which crosses PCIe as ONE pinned copy; then one scatter kernel per array and one sync
    // (round 3 made two pageable copies, a kernel and a sync per array: ~3.6 ms at config E).
    struct SJob {
        uint32_t width;  // bytes per element: 16, 4 or 1; 0: a contiguous copy of n bytes to dst
        void *dst;
        size_t n, idx_off, src_off;  // offsets into the staged blob
    };
    std::vector<SJob> sjobs;
    std::vector<uint8_t> sblob;
    bool fail_flush_done = false;  // TM_CFG_FAIL_FLUSH_ONCE (test aid)
    PinBuf h_sblob;
    DevBuf d_sblob;
    size_t stage_bytes_add(const void *p, size_t bytes) {
        const size_t at = (sblob.size() + 15) & ~size_t(15);
        sblob.resize(at + bytes);
        if (bytes) memcpy(sblob.data() + at, p, bytes);
        return at;
    }
    void drop_scatters() {
        sjobs.clear();
        sblob.clear();
    }
    hipError_t flush_scatters() {
        if (sjobs.empty()) return hipSuccess;
        struct Drop {  // whatever happens below, no job outlives this flush
            tm_engine *e;
            ~Drop() { e->drop_scatters(); }
        } drop{this};
        if ((cfg.flags & TM_CFG_FAIL_FLUSH_ONCE) && !fail_flush_done) {
            fail_flush_done = true;
            return hipErrorOutOfMemory;
        }
        hipError_t e;
        const size_t bytes = sblob.size();
        if ((e = h_sblob.ensure(bytes))) return e;
        if (bytes > d_sblob.cap && (e = d_sblob.ensure(bytes + bytes / 2))) return e;
        memcpy(h_sblob.p, sblob.data(), bytes);
        if ((e = hipMemcpyAsync(d_sblob.p, h_sblob.p, bytes, hipMemcpyHostToDevice, stream))) return e;
        const uint8_t *base = d_sblob.as<uint8_t>();
        for (const SJob &j : sjobs) {
            const uint64_t *idx = reinterpret_cast<const uint64_t *>(base + j.idx_off);
            const uint64_t cap = bnd_cap_of(j.dst, j.width ? j.width : 1);  // ~0 in the product build
            if (j.width == 0) {
                if (TM_BOUNDS && j.n > cap) bnd_host("delta tail copy", j.dst, j.n, cap);
                e = hipMemcpyAsync(j.dst, base + j.src_off, j.n, hipMemcpyDeviceToDevice, stream);
            } else if (j.width == 16) {
                e = launch_scatter16((uint4 *)j.dst, idx, reinterpret_cast<const uint4 *>(base + j.src_off), j.n, stream, cap, bnd_rec());
            } else if (j.width == 4) {
                e = launch_scatter4((uint32_t *)j.dst, idx, reinterpret_cast<const uint32_t *>(base + j.src_off), j.n, stream, cap, bnd_rec());
            } else {
                e = launch_scatter1((uint8_t *)j.dst, idx, base + j.src_off, j.n, stream, cap, bnd_rec());
            }
            if (e) {
                (void)hipStreamSynchronize(stream);  // the pinned blob may still be read by the copy
                return e;
            }
        }
        if ((e = bnd_after(stream, "delta scatters"))) return e;
        return hipStreamSynchronize(stream);  // the pinned blob is reused by the next commit
    }

    // dst[idx[i]] = src[i] for 16-byte records (edge slots, word slots, node records): staged
    template <class V, class Rec16 = typename V::value_type>
    hipError_t scatter16(std::vector<uint64_t> &dirty, const V &tab, DevBuf &dbuf) {
        static_assert(sizeof(Rec16) == 16, "16-byte records");
        if (dirty.empty()) return hipSuccess;
        sort_unique(dirty);
        size_t n = dirty.size();
        std::vector<Rec16> src(n);
        for (size_t i = 0; i < n; i++) src[i] = tab[dirty[i]];
        patch.add(P_SCATTER, arr_of(&dbuf), n, 0, dirty.data(), n * 8, src.data(), n * 16);
        const size_t io = stage_bytes_add(dirty.data(), n * 8);
        sjobs.push_back(SJob{16, dbuf.p, n, io, stage_bytes_add(src.data(), n * 16)});
        return hipSuccess;
    }

    // the device records of nodes (host ids): their edge slots (width 16) or slot_list
    // entries (width 4), each at the node's slot: staged
    hipError_t scatter_nodes(std::vector<uint64_t> &dirty, uint32_t width) {
        if (dirty.empty()) return hipSuccess;
        sort_unique(dirty);
        const size_t n = dirty.size();
        std::vector<uint64_t> idx(n);
        DevBuf &dbuf = width == 16 ? d_etab : d_slot_list;
        size_t so;
        if (width == 16) {
            std::vector<EdgeSlot> src(n);
            par_for(n, [&](size_t i) {
                idx[i] = node_slot[dirty[i]];
                src[i] = edge_rec((uint32_t)dirty[i]);
            });
            patch.add(P_SCATTER, A_ETAB, n, 0, idx.data(), n * 8, src.data(), n * 16);
            so = stage_bytes_add(src.data(), n * 16);
        } else {
            std::vector<uint32_t> src(n);
            par_for(n, [&](size_t i) {
                idx[i] = node_slot[dirty[i]];
                src[i] = node_slist[dirty[i]];
            });
            patch.add(P_SCATTER, A_SLOT_LIST, n, 0, idx.data(), n * 8, src.data(), n * 4);
            so = stage_bytes_add(src.data(), n * 4);
        }
        const size_t io = stage_bytes_add(idx.data(), n * 8);
        sjobs.push_back(SJob{width, dbuf.p, n, io, so});
        return hipSuccess;
    }

    // dst[idx[i]] = src[i] for u32 entries (arena words): staged
    template <class V>
    hipError_t scatter4(std::vector<uint64_t> &dirty, const V &tab, DevBuf &dbuf) {
        if (dirty.empty()) return hipSuccess;
        sort_unique(dirty);
        size_t n = dirty.size();
        std::vector<uint32_t> src(n);
        for (size_t i = 0; i < n; i++) src[i] = tab[dirty[i]];
        patch.add(P_SCATTER, arr_of(&dbuf), n, 0, dirty.data(), n * 8, src.data(), n * 4);
        const size_t io = stage_bytes_add(dirty.data(), n * 8);
        sjobs.push_back(SJob{4, dbuf.p, n, io, stage_bytes_add(src.data(), n * 4)});
        return hipSuccess;
    }

    // A grow-only array that outgrew its device buffer moves to one 1.5x its size: its device
    // contents are copied on the device and only the tail then crosses PCIe (round 1
    // re-uploaded the whole index, edge table included: a 70 ms commit at config E).  Replicas
    // get the array whole (P_WHOLE with the new capacity) ahead of the tail.
    template <class V, class T = typename V::value_type>
    hipError_t grow(DevBuf &d, const V &h, size_t dev_n) {
        if (h.size() * sizeof(T) <= d.cap) return hipSuccess;
        DevBuf nb;
        hipError_t e = nb.ensure(std::max<size_t>(h.size() * sizeof(T) * 3 / 2, 4096));
        if (e) return e;
        if (dev_n && (e = hipMemcpyAsync(nb.p, d.p, dev_n * sizeof(T), hipMemcpyDeviceToDevice, stream))) {
            nb.release();
            return e;
        }
        if ((e = hipStreamSynchronize(stream))) {
            nb.release();
            return e;
        }
        d.release();
        d.p = nb.p;
        d.cap = nb.cap;
        nb.p = nullptr;
        const uint32_t a = arr_of(&d);
        if (a < A_N) patch.add(P_WHOLE, a, dev_n * sizeof(T) / ARR_ELEM[a], d.cap, h.data(), dev_n * sizeof(T));
        n_grows++;
        return hipSuccess;
    }

    // Delta publish, under mu_dev after quiesce().  Phase 1 allocates (moves of grown arrays,
    // key arrays that outgrew their buffers, the word table after a rehash, the scatter
    // staging); phase 2 writes in place.  A failure in phase 1 leaves the previous epoch whole.
    uint64_t pub_us[4] = {};
    size_t n_dirty_arena = 0;  // the last delta publish: quiesce, allocations, staging, H2D + scatter kernels
    hipError_t upload_delta() {
        hipError_t e;
        uint64_t tp = now_us();
        // jobs a failed publish left queued point into buffers a full publish may since have
        // freed: a delta starts from an empty queue (advisor, round 4)
        drop_scatters();
        // phase 1
        if ((e = grow(d_warena, warena, warena_dev))) return e;
        if ((e = grow(d_word_off, word_off, word_off_dev))) return e;
        if ((e = grow(d_arena, arena, arena_dev))) return e;
        if (keys.size() * 16 > d_key_rec.cap || keys.size() * sizeof(uint32_t) > d_key_bin.cap ||
            keys.size() * sizeof(uint32_t) > d_key_node.cap || keys.size() > d_key_dd.cap) {
            KeyArrays ka;
            key_arrays(ka);
            if ((e = replace_whole(d_key_rec, A_KEY_REC, ka.rec)) || (e = replace_whole(d_key_node, A_KEY_NODE, ka.node)) ||
                (e = replace_whole(d_key_bin, A_KEY_BIN, ka.bin)) || (e = replace_whole(d_key_dd, A_KEY_DD, ka.dd)))
                return e;
            dirty_kid.clear();
        }
        if (words_full) {
            if ((e = replace_whole(d_wtab, A_WTAB, wtab, 1, 1))) return e;
            dirty_wslots.clear();
        }
        size_t mx = 0;
        for (const std::vector<uint64_t> *v : {&dirty_arena, &dirty_wslots, &dirty_enodes, &dirty_lnodes, &dirty_kid})
            mx = std::max(mx, v->size());
        if ((e = d_scatter_idx.ensure(std::max<size_t>(mx, 1) * sizeof(uint64_t)))) return e;
        if ((e = d_scatter_src.ensure(std::max<size_t>(mx, 1) * 16))) return e;
        pub_us[1] = now_us() - tp;
        tp = now_us();
        // phase 2
        if ((e = put_tail(d_warena, warena, warena_dev))) return e;
        if ((e = put_tail(d_word_off, word_off, word_off_dev))) return e;
        if ((e = put_tail(d_arena, arena, arena_dev))) return e;
        n_dirty_arena = dirty_arena.size();
        if ((e = scatter4(dirty_arena, arena, d_arena))) return e;  // lists rewritten in place
        if ((e = scatter16(dirty_wslots, wtab, d_wtab))) return e;
        if ((e = scatter_nodes(dirty_enodes, 16))) return e;
        if ((e = scatter_nodes(dirty_lnodes, 4))) return e;
        if ((e = upload_key_ids_delta())) return e;
        pub_us[2] = now_us() - tp;
        tp = now_us();
        if ((e = flush_scatters())) return e;
        if (root_dirty) {
            if ((e = hipMemcpyAsync(d_root.p, &root, sizeof(RootRec), hipMemcpyHostToDevice, stream))) return e;
            patch.add(P_WHOLE, A_ROOT, 1, d_root.cap, &root, sizeof(RootRec));
        }
        e = hipStreamSynchronize(stream);
        pub_us[3] = now_us() - tp;
        return e;
    }

    static uint64_t now_us() {
        return (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                   std::chrono::steady_clock::now().time_since_epoch())
            .count();
    }

    // ---------------------------------------------------------------------
    // Capacity check of an epoch's ops BEFORE anything changes (a refused commit keeps its ops
    // staged and the engine serving the previous epoch: emqx_router_syncer.erl:269-277).
    // hnode/hdepth: the deepest existing node on each op's path; nwalk: the levels its key
    // hangs at (0 for ops that create no node: deletes, dead filters).
    int capacity_check(const std::vector<StagedOp> &ops, const uint8_t *ob, const std::vector<uint32_t> &hdepth,
                       const std::vector<uint32_t> &nwalk) {
        uint64_t upper = 0, adds = 0;
        for (size_t i = 0; i < ops.size(); i++)
            if (ops[i].op == TM_OP_ADD) {
                adds++;
                if (nwalk[i] > hdepth[i]) upper += nwalk[i] - hdepth[i];
            }
        // the arena after a compaction: every live key once, one header per node with keys
        const uint64_t keys_after = n_live + adds;
        auto arena_need = [&](uint64_t nn) { return keys_after + LIST_HDR * std::min(keys_after, n_edges + 1 + nn); };
        uint64_t new_nodes = upper;
        if (n_edges + upper > node_budget() || arena_need(upper) > arena_budget()) {
            // exact: a new node is named by its filter's byte prefix (its words)
            std::unordered_set<std::string> fresh;
            std::vector<std::pair<uint32_t, uint32_t>> lv;
            for (size_t i = 0; i < ops.size(); i++) {
                if (ops[i].op != TM_OP_ADD || nwalk[i] <= hdepth[i]) continue;
                const uint8_t *f = ob + ops[i].off;
                lv.clear();
                uint32_t st = 0;
                for (uint32_t j = 0; j <= ops[i].len; j++)
                    if (j == ops[i].len || f[j] == '/') {
                        lv.push_back({st, j - st});
                        st = j + 1;
                    }
                for (uint32_t k = hdepth[i]; k < nwalk[i]; k++)
                    fresh.emplace((const char *)f, lv[k].first + lv[k].second);
            }
            new_nodes = fresh.size();
        }
        if (n_edges + new_nodes > node_budget()) {
            err = "commit refused: " + std::to_string(n_edges + new_nodes) + " trie nodes > budget " +
                  std::to_string(node_budget()) +
                  " (ops kept staged; the previous epoch keeps serving; shard the filters or raise max_nodes)";
            return TM_ENOMEM;
        }
        if (arena_need(new_nodes) > arena_budget()) {
            err = "commit refused: the terminal-list arena would pass its budget of " + std::to_string(arena_budget()) +
                  " words (ops kept staged; the previous epoch keeps serving)";
            return TM_ENOMEM;
        }
        return TM_OK;
    }

    // Ops whose commit failed go back to the front of the staged list (ahead of ops staged
    // by other threads meanwhile), so a retry applies everything in the original order.
    void restage(std::vector<StagedOp> &ops, std::vector<uint8_t> &ob) {
        std::lock_guard<std::mutex> g(mu_stage);
        const uint64_t base = ob.size();
        for (StagedOp &o : staged) o.off += base;
        ob.insert(ob.end(), stage_bytes.begin(), stage_bytes.end());
        ops.insert(ops.end(), staged.begin(), staged.end());
        staged.swap(ops);
        stage_bytes.swap(ob);
    }

    // Publish the host copy's changes to the device.  Delta: scatter in place under mu_dev,
    // after every use already queued.  Full: upload into a standby image on s_build while
    // matches keep running on the current one, then swap under mu_dev.
    hipError_t publish(bool full) {
        if (full) {
            hipError_t e = publish_full();
            if (!e) commit_stall_us = last_swap_us;
            return e;
        }
        std::lock_guard<std::recursive_mutex> g(mu_dev);
        const uint64_t t0 = now_us();
        hipError_t e = quiesce();  // in-flight matches read what this writes in place
        pub_us[0] = now_us() - t0;
        if (!e) e = upload_delta();
        if (!e) set_view();
        commit_stall_us = now_us() - t0;
        return e;
    }
    void set_view() {  // under mu_dev
        dv.epoch = epoch;
        dv.wmask = wmask;
        dv.emask = emask;
        dv.n_deep = n_deep;
        dv.max_id = max_id;
        dv.n_live = n_live;
        dv.n_nodes = node_parent.size();
        dv.n_words = word_off.size();
    }

    int commit(HostOut *me) {  // caller holds mu_commit
        std::vector<StagedOp> ops;
        std::vector<uint8_t> ob;
        {
            std::lock_guard<std::mutex> g(mu_stage);
            ops.swap(staged);
            ob.swap(stage_bytes);
        }
        const uint64_t t0 = now_us();
        // EMQX_TM_COMMIT_TRACE=1 (development): each commit's sub-phases on stderr
        static const bool trace = getenv("EMQX_TM_COMMIT_TRACE") != nullptr;
        uint64_t tr_last = t0;
        std::string tr;
        auto tick = [&](const char *what) {
            if (!trace) return;
            const uint64_t t = now_us();
            tr += std::string(" ") + what + "=" + std::to_string(t - tr_last);
            tr_last = t;
        };
        const size_t n = ops.size();
        std::vector<uint32_t> hnode(n, ROOT), hdepth(n, 0), nwalk(n, 0);
        std::vector<uint8_t> pkind(n, PK_NONE);
        std::vector<uint8_t> okind(n, PK_NONE);
        resolve_all(ops, ob.data(), hnode, hdepth, nwalk, pkind, okind);
        tick("resolve");
        int rc = capacity_check(ops, ob.data(), hdepth, nwalk);
        tick("capacity");
        if (rc) {
            restage(ops, ob);
            n_commits_refused++;
            return rc;
        }
        // host phase: runs results read the host id arena and key table, so none may be held
        if (me) lease_drop(*me);
        leases_block();  // before mu_host: a lease holder may still read the host copy meanwhile
        struct Unblock {
            tm_engine *e;
            ~Unblock() { e->leases_unblock(); }
        } unblock{this};
        std::lock_guard<std::mutex> gh(mu_host);
        tick("leases+host_lock");
        // Ops apply in order (last op per key wins), each a few dependent random reads of host
        // tables far larger than the caches (key set, key records, ids).  Their addresses are
        // known ahead for ops whose path exists: a two-stage prefetch (the key-set slot 16 ops
        // ahead, then the key record and id slot it leads to 8 ops ahead) overlaps those misses.
        // An ADD whose path is new creates nodes below its deepest existing node.  The word of
        // its first new edge is interned here, in op order (the op itself would intern it before
        // any later op could look it up, and a DEL before it finds no edge either way), so the
        // loop knows ahead what that ADD touches: the parent's records, the node-map entry and
        // the slot-bitmap word of the new edge, and the key-set slot of the new key at the node
        // id it will most likely get (nodes are numbered in creation order).
        std::vector<uint32_t> mword(n, NONE), pnode(n, NONE);
        {
            uint64_t nid = node_parent.size();
            for (size_t i = 0; i < n; i++) {
                if (ops[i].op != TM_OP_ADD || okind[i] == PK_NONE || pkind[i] != PK_NONE || hdepth[i] >= nwalk[i])
                    continue;
                const uint8_t *f = ob.data() + ops[i].off;
                uint32_t a = 0, lvl = 0;
                while (lvl < hdepth[i]) {  // level hdepth[i]'s bytes
                    while (a < ops[i].len && f[a] != '/') a++;
                    a++;
                    lvl++;
                }
                uint32_t e = a;
                while (e < ops[i].len && f[e] != '/') e++;
                mword[i] = (e - a == 1 && f[a] == '+') ? W_PLUS : word_intern(f + a, e - a);
                nid += nwalk[i] - hdepth[i];
                pnode[i] = (uint32_t)std::min<uint64_t>(nid - 1, NONE - 1);
            }
        }
        auto pf_slot = [&](size_t i) {
            if (pkind[i] != PK_NONE) {
                __builtin_prefetch(&kset[key_hash(hnode[i], pkind[i], ops[i].id) & kmask]);
            } else if (mword[i] != NONE) {
                if (hnode[i] != ROOT) {
                    __builtin_prefetch(&node_info[hnode[i]]);
                    __builtin_prefetch(&node_bloom[hnode[i]]);
                    __builtin_prefetch(&node_slot[hnode[i]]);
                }
                __builtin_prefetch(&emap[emap_hash(hnode[i], mword[i]) & emap_mask]);
            }
        };
        auto pf_key = [&](size_t i) {
            if (!idtab.empty()) __builtin_prefetch(&idtab[mix64(ops[i].id) & (idtab.size() - 1)]);
            if (pkind[i] != PK_NONE) {
                const uint32_t h = kset[key_hash(hnode[i], pkind[i], ops[i].id) & kmask];
                if (h != NONE) __builtin_prefetch(&keys[h]);
            } else if (mword[i] != NONE) {
                const uint64_t es = edge_home(dev_id(hnode[i]), mword[i], emask);
                __builtin_prefetch(&eocc[es >> 6]);
                __builtin_prefetch(&kset[key_hash(pnode[i], okind[i], ops[i].id) & kmask]);
            }
        };
        uint64_t tsc_kind[3] = {}, n_kind[3] = {};  // trace: ADD with the path present, ADD with a new path, DEL
        for (size_t i = 0; i < n; i++) {
            if (i + 16 < n) pf_slot(i + 16);
            if (i + 8 < n) pf_key(i + 8);
            if (trace) {
                const int k = ops[i].op != TM_OP_ADD ? 2 : pkind[i] != PK_NONE ? 0 : 1;
                const uint64_t c0 = __builtin_ia32_rdtsc();
                apply_one(ops[i], ob.data(), hnode[i], hdepth[i], pkind[i]);
                tsc_kind[k] += __builtin_ia32_rdtsc() - c0;
                n_kind[k]++;
            } else {
                apply_one(ops[i], ob.data(), hnode[i], hdepth[i], pkind[i]);
            }
        }
        tick("apply_ops");
        if (trace) {
            const uint64_t tot = std::max<uint64_t>(1, tsc_kind[0] + tsc_kind[1] + tsc_kind[2]);
            tr += " [add_path=" + std::to_string(n_kind[0]) + ":" + std::to_string(100 * tsc_kind[0] / tot) + "% add_new=" +
                  std::to_string(n_kind[1]) + ":" + std::to_string(100 * tsc_kind[1] / tot) + "% del=" +
                  std::to_string(n_kind[2]) + ":" + std::to_string(100 * tsc_kind[2] / tot) + "% nodes=" +
                  std::to_string(node_parent.size()) + "]";
        }
        if (edge_full) {  // cannot happen after capacity_check; never serve a half-applied trie
            err = "internal: edge table overflow past the capacity check";
            return TM_EDEVICE;
        }
        const uint64_t t1 = now_us();
        bool full = need_full || deltas.size() > std::max<uint64_t>(n_live / 8, 1u << 16);
        if (full) {
            rebuild_arena();
        } else if (!deltas.empty()) {
            apply_deltas();
            if (arena_garbage > std::max<uint64_t>(arena.size() / 2, 1u << 20) || arena.size() > arena_budget() ||
                ids_stale)
                rebuild_arena();
        }
        lists_dd_touch();  // (a full rebuild wrote every header from the key flags already)
        tick(full ? "rebuild_arena" : "apply_deltas");
        if (trace && !full)
            tr += " [lists=" + std::to_string(ad_us[0]) + " inplace=" + std::to_string(ad_us[1]) + " moved=" +
                  std::to_string(ad_us[2]) + " nodes=" + std::to_string(ad_groups) + " inplace_nodes=" +
                  std::to_string(ad_inplace) + " deltas=" + std::to_string(deltas.size()) + "]";
        deltas.clear();
        const uint64_t t2 = now_us();
        patch.reset();
        patch_from = epoch;
        const bool was_full = need_full;
        epoch++;
        hipError_t e = publish(need_full);
        if (e == hipErrorOutOfMemory && standby_bytes() && !(cfg.flags & TM_CFG_FAIL_FLUSH_ONCE)) {
            // the standby image (a second copy of the index, unused until the next full
            // publish) gives its HBM back, and the publish runs once more
            (void)hipGetLastError();
            drop_scatters();
            standby_release();
            patch.reset();  // the failed attempt's records go; the retry records the epoch again
            e = publish(need_full);
        }
        if (e != hipSuccess) {
            // the device still holds the previous epoch, intact (allocations come before any
            // in-place write); the host copy has advanced: the next commit re-uploads it whole
            drop_scatters();
            epoch--;
            need_full = true;
            patch.reset();
            patch.full = true;
            err = std::string("device upload failed (the previous epoch keeps serving; the next commit "
                              "uploads the index again): ") + hipGetErrorString(e);
            return e == hipErrorOutOfMemory ? TM_ENOMEM : TM_EDEVICE;
        }
        tick(was_full ? "publish_full" : "publish_delta");
        if (trace && !was_full)
            tr += " [quiesce=" + std::to_string(pub_us[0]) + " alloc=" + std::to_string(pub_us[1]) +
                  " stage=" + std::to_string(pub_us[2]) + " h2d+scatter=" + std::to_string(pub_us[3]) +
                  " arena_words=" + std::to_string(n_dirty_arena) + "]";
        if (trace)
            fprintf(stderr, "tm commit epoch %llu: %zu ops, %s:%s\n", (unsigned long long)epoch, n,
                    was_full ? "full" : "delta", tr.c_str());
        commit_us[0] = t1 - t0;
        commit_us[1] = t2 - t1;
        commit_us[2] = now_us() - t2;
        if (was_full) n_full_rebuilds++;
        else n_delta_commits++;
        need_full = false;
        words_full = false;
        root_dirty = false;
        dirty_enodes.clear();
        dirty_wslots.clear();
        dirty_lnodes.clear();
        dirty_arena.clear();
        for (uint32_t h : free_pending) free_keys.push_back(h);
        free_pending.clear();
        return TM_OK;
    }

    // =====================================================================
    // key -> filter bytes (emqx_topic_index:get_topic/1 = emqx_topic:join(Words))
    std::string key_filter(uint32_t h) const {
        const KeyRec &k = keys[h];
        if (k.kind == K_DEAD) return dead_filter[h];
        std::vector<uint32_t> path;
        for (uint32_t v = k.node; v != ROOT; v = node_parent[v]) path.push_back(node_word[v]);
        std::string s;
        for (size_t i = path.size(); i-- > 0;) {
            uint32_t w = path[i];
            if (w == W_PLUS) s += '+';
            else s.append((const char *)warena.data() + word_off[w], word_len[w]);
            if (i) s += '/';
        }
        if (k.kind == K_HASH) s += path.empty() ? "#" : "/#";
        return s;
    }

    // Order code of a key among the keys that match ONE topic.  Such keys agree on every
    // literal level (each equals the topic's word), so Erlang term order between them is
    // decided by the shape alone: per level END < '#' < '+' < literal ('#' < '+' as atoms,
    // atoms < binaries, a list that ends first sorts first), and every {Binary, {ID}} key
    // sorts after every word list.  Code: bit 62 = binary key; levels 0..30 as 2-bit
    // symbols from bit 61 down (END 0, '#' 1, '+' 2, literal 3); bit 63 flags a '#' key and
    // is not part of the order.  Returns false when the shape needs more than 31 levels.
    static constexpr uint64_t ORD_HASH = 1ull << 63, ORD_BIN = 1ull << 62;
    bool key_ord(uint32_t h, uint64_t *ord) const {
        const KeyRec &k = keys[h];
        *ord = 0;
        if (k.kind == K_EXACT_BIN) {
            *ord = ORD_BIN;
            return true;
        }
        if (k.kind != K_EXACT_WORDS && k.kind != K_WILD && k.kind != K_HASH) return true;
        uint32_t n = 0;
        for (uint32_t v = k.node; v != ROOT; v = node_parent[v]) n++;
        uint64_t o = 0;
        uint32_t i = n;
        for (uint32_t v = k.node; v != ROOT; v = node_parent[v]) {
            i--;
            if (i < 31) o |= (uint64_t)(node_word[v] == W_PLUS ? 2u : 3u) << (60 - 2 * i);
        }
        bool deep = n > 31;
        if (k.kind == K_HASH) {
            if (n < 31) o |= 1ull << (60 - 2 * n);
            o |= ORD_HASH;
            deep = n > 30;
        }
        *ord = o;
        return !deep;
    }

    // ETS term order of two keys (emqx_trie_search.erl:109-111 key shapes; Erlang term
    // order: lists < binaries; atoms '#' < '+' < binaries; binaries bytewise; then {ID}).
    // Used to reproduce return_first (the first key the ordered walk meets) and unique
    // (last write wins in walk order) on top of an unordered match set.
    void key_words(uint32_t h, std::vector<uint32_t> &out) const {
        out.clear();
        const KeyRec &k = keys[h];
        for (uint32_t v = k.node; v != ROOT; v = node_parent[v]) out.push_back(node_word[v]);
        std::reverse(out.begin(), out.end());
        if (k.kind == K_HASH) out.push_back(NONE - 2);  // '#'
    }
    int cmp_word(uint32_t a, uint32_t b) const {
        const uint32_t HASHW = NONE - 2;
        auto cls = [&](uint32_t w) { return w == HASHW ? 0 : (w == W_PLUS ? 1 : 2); };
        int ca = cls(a), cb = cls(b);
        if (ca != cb) return ca < cb ? -1 : 1;
        if (ca != 2 || a == b) return 0;
        uint32_t la = word_len[a], lb = word_len[b];
        int c = memcmp(&warena[word_off[a]], &warena[word_off[b]], std::min(la, lb));
        if (c) return c < 0 ? -1 : 1;
        return la < lb ? -1 : (la > lb ? 1 : 0);
    }
    int cmp_keys(uint32_t a, uint32_t b) const {
        const KeyRec &ka = keys[a], &kb = keys[b];
        bool ba = ka.kind == K_EXACT_BIN, bb = kb.kind == K_EXACT_BIN;
        if (ba != bb) return ba ? 1 : -1;  // lists sort before binaries
        int c;
        if (ba) {
            std::string fa = key_filter(a), fb = key_filter(b);
            c = fa.compare(fb);  // bytewise (std::string compares as unsigned char)
            c = c < 0 ? -1 : (c > 0 ? 1 : 0);
        } else {
            std::vector<uint32_t> wa, wb;
            key_words(a, wa);
            key_words(b, wb);
            c = 0;
            size_t n = std::min(wa.size(), wb.size());
            for (size_t i = 0; i < n && !c; i++) c = cmp_word(wa[i], wb[i]);
            if (!c && wa.size() != wb.size()) c = wa.size() < wb.size() ? -1 : 1;
        }
        if (c) return c;
        return ka.id < kb.id ? -1 : (ka.id > kb.id ? 1 : 0);
    }

    // =====================================================================
    // matches_filter/3 index (filter_kernels.hip): every word-list key ({Words, {ID}}:
    // exact word-form, wildcard, 'P/#' and dead keys -- the keys a filter search can
    // meet; {Binary, {ID}} keys compare `lower` and end it) as order codes, sorted in
    // ETS term order.  Built on first use after a commit; the match path never pays it.
    struct FilterIndex {
        uint64_t epoch = UINT64_MAX;     // epoch the device copy was built for
        std::vector<std::string> dict;   // sorted distinct literal words of the keys
        uint32_t K = 0;
        DevBuf d_kw, d_koff, d_kh;
        DevBuf d_qw, d_qoff, d_qdollar, d_qstatus, d_cnt, d_off, d_out, d_scan, d_pool, d_ctl, d_jobs, d_krec, d_kend;
        DevBuf d_rcnt;                                  // FW_RUNS: ranges per query
        uint64_t out_want = 1 << 16, pool_want = 1024;  // one-pass sizes (from the demand seen)
        uint64_t rng_want = 1 << 16;                    // FW_RUNS output (ranges)
        std::shared_ptr<const std::vector<uint64_t>> ids;  // id of sorted key j (the runs form's spans)
        std::vector<uint32_t> qw, qoff;
        std::vector<uint32_t> wcode;     // interned word id -> order code (NONE: not cached yet)
        std::vector<uint32_t> h_kw, h_koff, h_kend;  // host copies of the order (plan_filter_parts)
        DevBuf d_items, d_stop;          // FW_RUNS parts: {query, start, end, first}; per part: stopped
        DevBuf d_wtime;                  // development: per wave duration (EMQX_TM_FILTER_WTIME)
        std::vector<uint4> items;
        std::vector<uint32_t> i_cnt, i_rcnt, i_off, i_stop;
        std::vector<uint8_t> qdollar;
        uint64_t n_onepass = 0, n_twopass = 0;  // batches by path (tests / bench)
    } fx;
    // intersection/2 batches (filter_kernels.hip k_intersect)
    DevBuf d_ia, d_iaoff, d_ib, d_iboff, d_iout, d_ilen;

    static void split_words(const uint8_t *p, size_t n, std::vector<std::pair<size_t, size_t>> &out) {
        out.clear();
        size_t st = 0;
        for (size_t i = 0; i <= n; i++)
            if (i == n || p[i] == '/') {
                out.emplace_back(st, i - st);
                st = i + 1;
            }
    }
    // order code of a literal word: 2k+3 for the k-th dictionary word, 2k+2 for a word
    // that is not in the dictionary and sorts just below its k-th entry
    uint32_t fx_code(const char *p, size_t n) const {
        const std::string w(p, n);
        size_t k = std::lower_bound(fx.dict.begin(), fx.dict.end(), w) - fx.dict.begin();
        return (uint32_t)(k < fx.dict.size() && fx.dict[k] == w ? 2 * k + 3 : 2 * k + 2);
    }
    static uint32_t fx_level(const char *p, size_t n) {  // '#' 0, '+' 1, else not a wildcard
        if (n == 1 && p[0] == '#') return 0;
        if (n == 1 && p[0] == '+') return 1;
        return NONE;
    }

    int build_filter_index() {
        const uint32_t HASHW = NONE - 2;
        std::vector<uint32_t> lk;  // word-list key handles
        std::vector<uint8_t> used(word_off.size(), 0);
        std::vector<std::string> words;
        std::vector<std::pair<size_t, size_t>> lv;
        for (uint32_t h = 0; h < keys.size(); h++) {
            const KeyRec &k = keys[h];
            if (k.kind == K_EXACT_WORDS || k.kind == K_WILD || k.kind == K_HASH) {
                lk.push_back(h);
                for (uint32_t v = k.node; v != ROOT; v = node_parent[v])
                    if (node_word[v] != W_PLUS) used[node_word[v]] = 1;
            } else if (k.kind == K_DEAD) {
                lk.push_back(h);
                const std::string &f = dead_filter[h];
                split_words((const uint8_t *)f.data(), f.size(), lv);
                for (auto &x : lv)
                    if (fx_level(f.data() + x.first, x.second) == NONE) words.emplace_back(f, x.first, x.second);
            }
        }
        for (uint32_t w = 0; w < used.size(); w++)
            if (used[w]) words.emplace_back((const char *)warena.data() + word_off[w], word_len[w]);
        std::sort(words.begin(), words.end());
        words.erase(std::unique(words.begin(), words.end()), words.end());
        fx.dict.swap(words);
        std::vector<uint32_t> wcode(word_off.size(), NONE);
        for (uint32_t w = 0; w < used.size(); w++)
            if (used[w]) wcode[w] = fx_code((const char *)warena.data() + word_off[w], word_len[w]);
        // codes of every key, unsorted
        std::vector<uint64_t> off(lk.size() + 1, 0);
        std::vector<uint32_t> code, path;
        for (size_t i = 0; i < lk.size(); i++) {
            const uint32_t h = lk[i];
            if (keys[h].kind == K_DEAD) {
                const std::string &f = dead_filter[h];
                split_words((const uint8_t *)f.data(), f.size(), lv);
                for (auto &x : lv) {
                    uint32_t c = fx_level(f.data() + x.first, x.second);
                    code.push_back(c != NONE ? c : fx_code(f.data() + x.first, x.second));
                }
            } else {
                key_words(h, path);
                for (uint32_t w : path) code.push_back(w == HASHW ? 0u : w == W_PLUS ? 1u : wcode[w]);
            }
            off[i + 1] = code.size();
        }
        if (code.size() + 8 >= 0xFFFFFFFFull || lk.size() >= 0xFFFFFF00ull) {
            err = "matches_filter index: more than 4 Gi key words or keys";
            return TM_ENOMEM;
        }
        // ETS term order: words (codes) lexicographically, a prefix first; then the id
        std::vector<uint32_t> perm(lk.size());
        for (uint32_t i = 0; i < perm.size(); i++) perm[i] = i;
        std::sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) {
            const uint32_t *pa = &code[off[a]], *pb = &code[off[b]];
            const uint64_t na = off[a + 1] - off[a], nb = off[b + 1] - off[b];
            for (uint64_t i = 0; i < std::min(na, nb); i++)
                if (pa[i] != pb[i]) return pa[i] < pb[i];
            if (na != nb) return na < nb;
            return keys[lk[a]].id < keys[lk[b]].id;
        });
        std::vector<uint32_t> kw, koff(lk.size() + 1, 0), kh(lk.size());
        kw.reserve(code.size() + 8);
        for (size_t j = 0; j < perm.size(); j++) {
            const uint32_t i = perm[j];
            kw.insert(kw.end(), code.begin() + off[i], code.begin() + off[i + 1]);
            koff[j + 1] = (uint32_t)kw.size();
            kh[j] = lk[i];
        }
        kw.insert(kw.end(), 8, 0u);  // k_filter_walk preloads 8 words of a key unconditionally
        {
            auto ids = std::make_shared<std::vector<uint64_t>>(kh.size());
            for (size_t j = 0; j < kh.size(); j++) (*ids)[j] = keys[kh[j]].id;
            fx.ids = std::move(ids);
        }
        // fixed-stride records {length, first FW_REC_WORDS codes}: a compare reads one 32-B
        // record instead of koff and then the words (one round trip instead of two)
        std::vector<uint32_t> krec(std::max<size_t>(lk.size(), 1) * 8, 0u);
        for (size_t j = 0; j < lk.size(); j++) {
            const uint32_t b = koff[j], L = koff[j + 1] - b;
            krec[j * 8] = L;
            for (uint32_t i = 0; i < std::min<uint32_t>(L, FW_REC_WORDS); i++) krec[j * 8 + 1 + i] = kw[b + i];
        }
        // prefix-group ends: kend[j][d] = the first key after j whose first d+1 words differ
        // from key j's.  A seek's probe {first np words of key ks ++ [w]} lands inside
        // [ks, kend[ks][np-1]] (every key in between shares those np words, the key at the end
        // is past them), so the walk searches that range instead of galloping from the cursor;
        // a '#'-run's end IS kend[rs][p-1].  One backward pass over the common prefixes of
        // neighbours.
        const size_t K = lk.size();
        std::vector<uint32_t> kend(std::max<size_t>(K, 1) * FW_END_DEPTHS, 0u);
        for (size_t j = K; j-- > 0;) {
            uint32_t lcp = 0;
            if (j + 1 < K) {
                const uint32_t *x = &kw[koff[j]], *y = &kw[koff[j + 1]];
                const uint32_t lx = koff[j + 1] - koff[j], ly = koff[j + 2] - koff[j + 1];
                while (lcp < lx && lcp < ly && lcp < FW_END_DEPTHS && x[lcp] == y[lcp]) lcp++;
            }
            for (uint32_t d = 0; d < FW_END_DEPTHS; d++)
                kend[j * FW_END_DEPTHS + d] = (j + 1 < K && lcp >= d + 1) ? kend[(j + 1) * FW_END_DEPTHS + d]
                                                                          : (uint32_t)(j + 1);
        }
        fx.K = (uint32_t)lk.size();
        hipError_t e;
        if ((e = fx.d_kend.ensure(kend.size() * 4)) != hipSuccess ||
            (e = fx.d_krec.ensure(krec.size() * 4)) != hipSuccess ||
            (e = fx.d_kw.ensure(std::max<size_t>(kw.size(), 1) * 4)) != hipSuccess ||
            (e = fx.d_koff.ensure(koff.size() * 4)) != hipSuccess ||
            (e = fx.d_kh.ensure(std::max<size_t>(kh.size(), 1) * 4)) != hipSuccess) {
            err = std::string("matches_filter index alloc: ") + hipGetErrorString(e);
            return TM_ENOMEM;
        }
        if ((e = hipMemcpy(fx.d_kend.p, kend.data(), kend.size() * 4, hipMemcpyHostToDevice)) ||
            (e = hipMemcpy(fx.d_krec.p, krec.data(), krec.size() * 4, hipMemcpyHostToDevice)) ||
            (!kw.empty() && (e = hipMemcpy(fx.d_kw.p, kw.data(), kw.size() * 4, hipMemcpyHostToDevice))) ||
            (e = hipMemcpy(fx.d_koff.p, koff.data(), koff.size() * 4, hipMemcpyHostToDevice)) ||
            (!kh.empty() && (e = hipMemcpy(fx.d_kh.p, kh.data(), kh.size() * 4, hipMemcpyHostToDevice))) ||
            // a copy from pageable memory may return before its DMA lands, and only the null
            // stream is ordered after it: wait before the walks on the engine's streams read it
            (e = hipStreamSynchronize(nullptr))) {
            err = std::string("matches_filter index upload: ") + hipGetErrorString(e);
            return TM_EDEVICE;
        }
        fx.wcode.swap(wcode);
        fx.wcode.resize(word_off.size(), NONE);
        // the runs form splits long '+' queries at child-group boundaries (plan_filter_parts):
        // it reads the order on the host
        fx.h_kw.swap(kw);
        fx.h_koff.swap(koff);
        fx.h_kend.swap(kend);
        fx.epoch = epoch;
        return TM_OK;
    }

    // matches_filter/3's walk over a query with '+' at level p (its levels before p literal)
    // spends its time inside G, the keys whose first p words are the query's: it enters every
    // child group of level p (a distinct word there) at its first key, since a seek inside G
    // lands in the child group it came from or at the next one's first key (its probe holds
    // the level-p word); and the keys before G cannot seek past G's first key.  So the walk
    // can be cut at child-group starts c_1 < c_2 < ... inside G: part k walks [c_k, c_{k+1})
    // from c_k as if it had arrived there (part 0 from the query's own start), and the query's
    // result is its parts' results in order up to the first part that stopped.
    // Only G: the keys that cover a literal level with '+' (R(W0, +) and the like) can seek
    // OUT of their region to the literal branch (compare's backtrack to the last '+', {Pos,
    // W[Pos]}), so the walk does not enter all their child groups; cutting there was tried and
    // returned keys the walk never reaches (round 5, tests/test_gpu_filter_runs.py).
    // Items {query, start, end (NONE: none), first part?}, queries in order, parts in order.
    // EMQX_TM_FILTER_SPLIT=min_keys:part_keys (0 or unset: no split, the default).
    void plan_filter_parts(uint32_t n, std::vector<uint4> &items) {
        items.clear();
        // off by default: every setting measured made the batches slower
        uint32_t min_keys = 0, part_keys = 4096;  // read per call: tests change it
        if (const char *e = getenv("EMQX_TM_FILTER_SPLIT")) {
            min_keys = (uint32_t)strtoul(e, nullptr, 10);
            if (const char *c = strchr(e, ':')) part_keys = std::max(1u, (uint32_t)strtoul(c + 1, nullptr, 10));
        }
        const uint32_t K = fx.K;
        bool any = false;
        std::vector<uint32_t> cuts;
        for (uint32_t q = 0; q < n; q++) {
            cuts.clear();
            const uint32_t *W = fx.qw.data() + fx.qoff[q];
            const uint32_t WL = fx.qoff[q + 1] - fx.qoff[q];
            uint32_t p = 0;
            while (p < WL && W[p] >= 2 && (W[p] & 1u)) p++;  // literal dictionary words
            if (min_keys && K && !fx.qdollar[q] && p >= 1 && p < WL && W[p] == 1u && p + 1 <= FW_END_DEPTHS) {
                // G = [g0, g1): the first key whose first p words are >= W's, if it has them
                auto less_prefix = [&](uint32_t j) {  // key j's words < W[0..p) (a shorter prefix is less)
                    const uint32_t *k = fx.h_kw.data() + fx.h_koff[j], L = fx.h_koff[j + 1] - fx.h_koff[j];
                    for (uint32_t i = 0; i < p; i++) {
                        if (i == L) return true;
                        if (k[i] != W[i]) return k[i] < W[i];
                    }
                    return false;
                };
                uint32_t lo = 0, hi = K;
                while (lo < hi) {
                    const uint32_t mid = lo + (hi - lo) / 2;
                    if (less_prefix(mid)) lo = mid + 1;
                    else hi = mid;
                }
                const uint32_t g0 = lo;
                bool has = g0 < K && fx.h_koff[g0 + 1] - fx.h_koff[g0] >= p;
                for (uint32_t i = 0; has && i < p; i++) has = fx.h_kw[fx.h_koff[g0] + i] == W[i];
                if (has) {
                    const uint32_t g1 = fx.h_kend[(uint64_t)g0 * FW_END_DEPTHS + p - 1];
                    if (g1 - g0 >= min_keys)
                        for (uint64_t x = (uint64_t)g0 + part_keys; x < g1; x += part_keys) {
                            // the next child-group start at or after x (x's group's end, unless
                            // x starts one itself)
                            const uint32_t xs = (uint32_t)x;
                            const bool starts = xs == g0 || fx.h_kend[(uint64_t)(xs - 1) * FW_END_DEPTHS + p] == xs;
                            const uint32_t c = starts ? xs : fx.h_kend[(uint64_t)xs * FW_END_DEPTHS + p];
                            // (a key of p words, the group of G's own prefix, never starts a part)
                            if (c < g1 && (cuts.empty() || c > cuts.back()) && fx.h_koff[c + 1] - fx.h_koff[c] > p)
                                cuts.push_back(c);
                        }
                }
            }
            any = any || !cuts.empty();
            uint32_t st = 0;
            for (size_t k = 0; k <= cuts.size(); k++) {
                const uint32_t en = k < cuts.size() ? cuts[k] : NONE;
                items.push_back(make_uint4(q, st, en, k == 0 ? 1u : 0u));
                st = en;
            }
        }
        if (!any) items.clear();  // nothing to split: one wave per query, as before
    }
};

// ============================================================================
// C-ABI
// ============================================================================

#define TM_TRY_HIP(E, CODE, MSG)                                                     \
    do {                                                                              \
        hipError_t _e = (E);                                                          \
        if (_e != hipSuccess) {                                                       \
            eng->err = std::string(MSG) + ": " + hipGetErrorString(_e);              \
            return CODE;                                                              \
        }                                                                             \
    } while (0)

extern "C" {

uint32_t tm_abi_version(void) { return TM_ABI_VERSION; }

#ifndef TM_SRC_SHA
#define TM_SRC_SHA "unknown"
#endif
const char *tm_build_info(void) {
    static const std::string info =
        std::string("src_sha=") + TM_SRC_SHA + " abi=" + std::to_string(TM_ABI_VERSION) + " arch=gfx950";
    return info.c_str();
}

int tm_create(const tm_config *cfg, tm_engine **out) {
    if (!out) return TM_EINVAL;
    *out = nullptr;
    tm_engine *eng = new (std::nothrow) tm_engine();
    if (!eng) return TM_ENOMEM;
    if (cfg) eng->cfg = *cfg;
    eng->patch.on = (eng->cfg.flags & TM_CFG_RECORD_PATCH) != 0;
    eng->master_nonce = mix64((uint64_t)std::chrono::steady_clock::now().time_since_epoch().count() ^
                              (uint64_t)(uintptr_t)eng) | 1ull;
    int ndev = 0;
    tl_create_err().clear();
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= eng->cfg.device || eng->cfg.device < 0) {
        tl_create_err() = "tm_create: no such HIP device";
        delete eng;
        return TM_EDEVICE;
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, eng->cfg.device) != hipSuccess ||
        std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
        tl_create_err() = "tm_create: the device is not a gfx950";
        delete eng;
        return TM_EDEVICE;  // kernels are built for gfx950 only
    }
    // a full publish's standby build runs at the device's lowest stream priority: the matches
    // beside it (on the engine's and the callers' streams) are dispatched first
    int prio_least = 0, prio_greatest = 0;
    if (hipSetDevice(eng->cfg.device) != hipSuccess ||
        hipStreamCreateWithFlags(&eng->stream, hipStreamNonBlocking) != hipSuccess ||
        hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess ||
        hipStreamCreateWithPriority(&eng->s_build, hipStreamNonBlocking, prio_least) != hipSuccess) {
        tl_create_err() = std::string("tm_create: stream creation failed: ") + hipGetErrorString(hipGetLastError());
        tm_destroy(eng);
        return TM_EDEVICE;
    }
    if (!eng->reserve_ids()) {
        tl_create_err() = "tm_create: no address space for the id arena reservation";
        tm_destroy(eng);
        return TM_ENOMEM;
    }
    if (!tm_engine::bnd_init(eng->cfg.device)) {
        tl_create_err() = "tm_create: bounds-build init failed";
        tm_destroy(eng);
        return TM_EDEVICE;
    }
    uint64_t rk = eng->cfg.reserve_keys ? eng->cfg.reserve_keys : 1024;
    uint64_t rn = eng->cfg.reserve_nodes ? eng->cfg.reserve_nodes : rk * 4;
    eng->word_rehash(1024);  // grows with the vocabulary (load <= 1/4), not with nodes
    eng->node_parent.reserve(rn);
    eng->node_word.reserve(rn);
    eng->node_slot.reserve(rn);
    eng->node_parent.push_back(NONE);  // root
    eng->node_word.push_back(NONE);
    eng->node_slot.push_back(NONE);
    eng->node_list.reserve(rn);
    eng->node_list.push_back(NodeList{0, 0, 0});
    eng->node_cap.push_back(0);
    for (hvec<uint32_t> *v : {&eng->node_bloom, &eng->node_info, &eng->node_slist}) {
        v->reserve(rn);
        v->push_back(0);
    }
    eng->emap_rehash(next_pow2(std::max<uint64_t>(rn * 2, 1024)));
    {
        const uint64_t want = std::max<uint64_t>(rn * eng->edge_load_inv(), 1024);
        eng->edge_rehash(std::min<uint64_t>((eng->cfg.flags & TM_CFG_EDGE_EXACT) ? (want + 63) & ~63ull : next_pow2(want),
                                            MAX_EDGE_SLOTS));
    }
    eng->kset_rehash(next_pow2(std::max<uint64_t>(rk * 2, 1024)));
    eng->keys.reserve(rk);
    eng->need_full = true;
    int rc;
    {
        std::lock_guard<std::mutex> g(eng->mu_commit);
        rc = eng->commit(nullptr);  // empty epoch 1: device tables exist from the start
    }
    if (rc != TM_OK) {
        tl_create_err() = std::string("tm_create: the first (empty) publish failed: ") + tl_err();
        tm_destroy(eng);
        return rc;
    }
    *out = eng;
    return TM_OK;
}

void tm_destroy(tm_engine *eng) {
    if (!eng) return;
    (void)hipSetDevice(eng->cfg.device);
    (void)eng->quiesce();
    if (eng->s_build) (void)hipStreamSynchronize(eng->s_build);
    for (auto &u : eng->uses) (void)hipEventDestroy(u.second);
    eng->uses.clear();
    if (eng->ev_chain) (void)hipEventDestroy(eng->ev_chain);
    for (auto &o : eng->outs) o.second->release();
    eng->outs.clear();
    eng->release_ids();
    eng->bb_dev.release();
    eng->bb_batch.release();
    eng->bb_batch2.release();
    eng->bb_dev2.release();
    eng->bb_dev3.release();
    for (DevBuf *b : {&eng->d_key_rec, &eng->d_key_node, &eng->d_key_bin, &eng->d_key_dd, &eng->d_mrg_roff, &eng->d_mrg_tot, &eng->fx.d_kw, &eng->fx.d_koff,
                      &eng->fx.d_kh, &eng->fx.d_qw, &eng->fx.d_qoff, &eng->fx.d_qdollar, &eng->fx.d_qstatus,
                      &eng->fx.d_cnt, &eng->fx.d_off, &eng->fx.d_out, &eng->fx.d_scan, &eng->fx.d_pool,
                      &eng->fx.d_ctl, &eng->fx.d_jobs, &eng->fx.d_krec, &eng->fx.d_kend, &eng->fx.d_rcnt, &eng->fx.d_items, &eng->fx.d_stop, &eng->fx.d_wtime, &eng->d_ia, &eng->d_iaoff,
                      &eng->d_ib, &eng->d_iboff, &eng->d_iout, &eng->d_ilen})
        b->release();
    for (DevBuf *b : {&eng->d_wtab, &eng->d_warena, &eng->d_word_off, &eng->d_etab, &eng->d_slot_list, &eng->d_root,
                      &eng->d_arena, &eng->d_scatter_idx, &eng->d_scatter_src, &eng->d_stats, &eng->d_sblob})
        b->release();
    eng->standby_release();
    eng->d_nim.release();
    eng->upload_release();
    eng->h_cursor.release();
    eng->h_sblob.release();
    if (eng->ev_fast0) (void)hipEventDestroy(eng->ev_fast0);
    if (eng->ev_fast1) (void)hipEventDestroy(eng->ev_fast1);
    if (eng->s_build) (void)hipStreamDestroy(eng->s_build);
    if (eng->stream) (void)hipStreamDestroy(eng->stream);
    delete eng;
}

// library-internal (batcher.cpp), not part of the C-ABI
__attribute__((visibility("hidden"))) int tmx_engine_device(const tm_engine *eng) { return eng->cfg.device; }
static int grow_pools(tm_engine *eng);
// library-internal (batcher.cpp): size the chunk pools to a batch's demand (the counter
// block the batcher copied back); no kernel of this engine may be in flight
__attribute__((visibility("hidden"))) void tmx_engine_pool_caps(const tm_engine *eng, uint32_t set, uint64_t *seg_chunks,
                                                               uint64_t *fr_chunks) {
    std::lock_guard<std::recursive_mutex> g(const_cast<tm_engine *>(eng)->mu_dev);
    const_cast<tm_engine *>(eng)->bb = const_cast<tm_engine *>(eng)->batch_set(set);
    *seg_chunks = eng->cfg.seg_chunks ? ~0ull : eng->bb->seg_chunks;  // fixed pools (test aid) never grow
    *fr_chunks = eng->cfg.seg_chunks ? ~0ull : eng->bb->fr_chunks;
}
__attribute__((visibility("hidden"))) int tmx_engine_grow_pools(tm_engine *eng, uint32_t set, uint64_t seg_demand,
                                                                uint64_t fr_demand) {
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    eng->bb = eng->batch_set(set);
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    eng->bb->seg_demand_last = seg_demand;
    eng->bb->fr_demand_last = fr_demand;
    return grow_pools(eng);
}

// library-internal (batcher.cpp): hold the engine's device lock across a window's whole
// enqueue (walk, id compaction, the D2H of its results), so no other caller's batch lands
// between them
__attribute__((visibility("hidden"))) void tmx_engine_lock(tm_engine *eng) { eng->mu_dev.lock(); }
__attribute__((visibility("hidden"))) void tmx_engine_unlock(tm_engine *eng) { eng->mu_dev.unlock(); }

const char *tm_last_error(const tm_engine *eng) { return eng ? eng->err.c_str() : "null engine"; }
const char *tm_create_last_error(void) { return tl_create_err().c_str(); }

static int replica_refuses(tm_engine *eng, const char *what) {
    eng->err = std::string(what) + ": a replica is read-only and keeps no host copy of the keys (use the master)";
    return TM_ESTATE;
}

int tm_apply(tm_engine *eng, const tm_op *ops, size_t n) {
    if (!eng || (n && !ops)) return TM_EINVAL;
    if (eng->replica) return replica_refuses(eng, "tm_apply");
    for (size_t i = 0; i < n; i++) {
        const tm_op &o = ops[i];
        if ((o.op != TM_OP_ADD && o.op != TM_OP_DEL) || o.filter_len > 65535u || (o.filter_len && !o.filter)) {
            eng->err = "tm_apply: bad op";
            return TM_EINVAL;
        }
    }
    std::lock_guard<std::mutex> g(eng->mu_stage);
    eng->staged.reserve(eng->staged.size() + n);
    for (size_t i = 0; i < n; i++) {
        const tm_op &o = ops[i];
        eng->staged.push_back(StagedOp{o.op, o.flags, o.id, eng->stage_bytes.size(), o.filter_len});
        eng->stage_bytes.insert(eng->stage_bytes.end(), o.filter, o.filter + o.filter_len);
    }
    return TM_OK;
}

int tm_apply_packed(tm_engine *eng, uint32_t op, const uint8_t *bytes, const uint64_t *off, const uint64_t *ids,
                    const uint32_t *flags, size_t n) {
    if (!eng || (n && (!off || !ids || (!bytes && off[n] > off[0])))) return TM_EINVAL;
    if (op != TM_OP_ADD && op != TM_OP_DEL) return TM_EINVAL;
    if (eng->replica) return replica_refuses(eng, "tm_apply_packed");
    for (size_t i = 0; i < n; i++)
        if (off[i + 1] < off[i] || off[i + 1] - off[i] > 65535u) {
            eng->err = "tm_apply_packed: bad filter offsets";
            return TM_EINVAL;
        }
    std::lock_guard<std::mutex> g(eng->mu_stage);
    eng->staged.reserve(eng->staged.size() + n);
    uint64_t base = eng->stage_bytes.size();
    if (n) eng->stage_bytes.insert(eng->stage_bytes.end(), bytes + off[0], bytes + off[n]);
    for (size_t i = 0; i < n; i++)
        eng->staged.push_back(StagedOp{op, flags ? flags[i] : 0u, ids[i], base + (off[i] - off[0]),
                                       (uint32_t)(off[i + 1] - off[i])});
    return TM_OK;
}

int tm_commit_epoch(tm_engine *eng, uint64_t *epoch_out) {
    if (!eng) return TM_EINVAL;
    if (eng->replica) return replica_refuses(eng, "tm_commit_epoch");
    if (tmx_in_delivery()) {
        // a commit waits for every runs window's read lease: the one whose callback this is, or
        // one queued behind it that only the delivery threads can finish -- it might never
        // return, whatever this window's transport (include/emqx_tm_batcher.h "writes").  Stage
        // with tm_apply here, commit from another thread.
        eng->err = "tm_commit_epoch from an aggregator delivery callback (it could wait for a lease only a delivery thread drops)";
        return TM_ESTATE;
    }
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::mutex> g(eng->mu_commit);
    HostOut *me = nullptr;
    {
        std::lock_guard<std::mutex> go(eng->mu_out);
        auto it = eng->outs.find(std::this_thread::get_id());
        if (it != eng->outs.end()) me = it->second.get();
    }
    int rc = eng->commit(me);
    if (epoch_out) *epoch_out = eng->epoch;
    return rc;
}

int tm_discard_staged(tm_engine *eng, uint64_t *n_out) {
    if (!eng) return TM_EINVAL;
    std::lock_guard<std::mutex> g(eng->mu_stage);
    if (n_out) *n_out = eng->staged.size();
    eng->staged.clear();
    eng->stage_bytes.clear();
    return TM_OK;
}

int tm_result_release(tm_engine *eng) {
    if (!eng) return TM_EINVAL;
    std::unique_ptr<HostOut> mine;
    {
        std::lock_guard<std::mutex> g(eng->mu_out);
        auto it = eng->outs.find(std::this_thread::get_id());
        if (it == eng->outs.end()) return TM_OK;
        mine = std::move(it->second);
        eng->outs.erase(it);
    }
    eng->lease_drop(*mine);
    {  // its streams leave the set a commit orders its writes after
        std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
        for (size_t i = 0; i < eng->uses.size();) {
            hipStream_t us = eng->uses[i].first;
            if (us && (us == mine->s_walk || us == mine->s_copy || us == mine->s_h2d)) {
                (void)hipEventSynchronize(eng->uses[i].second);
                (void)hipEventDestroy(eng->uses[i].second);
                eng->uses.erase(eng->uses.begin() + (ptrdiff_t)i);
            } else {
                i++;
            }
        }
    }
    mine->release();
    return TM_OK;
}

// Size the batch buffers for n topics / `bytes` topic bytes.
static int ensure_batch(tm_engine *eng, uint32_t n, uint64_t bytes) {
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_outoff, (size_t)n * 4 + 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_outcnt, (size_t)n * 4 + 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_status, (size_t)n * 4 + 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_slow_list, (size_t)n * 4 + 4), TM_ENOMEM, "alloc");
    if (!eng->bb->d_ctl.p) {
        TM_TRY_HIP(eng->grow_buf(eng->bb->d_ctl, 2 * CTL_BYTES), TM_ENOMEM, "alloc");
        // both blocks start at 0, and are 0 before any stream's launch reads them (hipMemset runs
        // on the null stream, which the engine's non-blocking streams do not wait for)
        TM_TRY_HIP(hipMemset(eng->bb->d_ctl.p, 0, 2 * CTL_BYTES), TM_EDEVICE, "memset");
        TM_TRY_HIP(hipStreamSynchronize(nullptr), TM_EDEVICE, "memset sync");
    }
    TM_TRY_HIP(eng->grow_buf(eng->d_stats, STATS_BYTES), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_scr_w, (bytes + 2ull * n + 2) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_scr_s, (bytes + 2ull * n + 2) * 8), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_wave_chunks, match_grid(n, pick_tpw(n, eng->cfg.topics_per_wave)) * SEG_MAXCHUNK * 4 + 4),
               TM_ENOMEM, "alloc");
    {
        // chunk pool for waves whose staged key segments overflow LDS
        uint64_t want = eng->cfg.seg_chunks ? eng->cfg.seg_chunks : std::max<uint64_t>(1024, ((uint64_t)n + 63) / 64 * 8);
        if (want > eng->bb->seg_chunks) {
            TM_TRY_HIP(eng->grow_buf(eng->bb->d_seg_pool, want * SEG_CHUNK * sizeof(uint4)), TM_ENOMEM, "alloc seg pool");
            eng->bb->seg_chunks = want;
        }
    }
    {
        // frontier overflow pool (waves whose per-depth frontier exceeds LDS)
        uint64_t want = eng->cfg.seg_chunks ? eng->cfg.seg_chunks : std::max<uint64_t>(1024, ((uint64_t)n + 63) / 64 * 4);
        if (want > eng->bb->fr_chunks) {
            TM_TRY_HIP(eng->grow_buf(eng->bb->d_fr_pool, want * FR_CHUNK * sizeof(uint2)), TM_ENOMEM, "alloc frontier pool");
            eng->bb->fr_chunks = want;
        }
    }
    if (eng->bb->keys_cap == 0) {
        uint64_t want = eng->cfg.reserve_matches ? eng->cfg.reserve_matches : std::max<uint64_t>(n * 8ull, 1 << 16);
        if (eng->bb == &eng->bb_dev2 || eng->bb == &eng->bb_dev3)
            want = std::max(want, eng->bb_dev.keys_cap);  // starts at set 0's reservation
        TM_TRY_HIP(eng->grow_buf(eng->bb->d_keys, want * 4), TM_ENOMEM, "alloc");
        eng->bb->keys_cap = want;
    }
    return TM_OK;
}

// After a batch: pools that ran short sent some topics to the spill kernel (results
// stay exact); size them to the observed demand for the next batch.
static int grow_pools(tm_engine *eng) {
    if (eng->cfg.seg_chunks) return TM_OK;  // fixed by the caller (test aid)
    if (eng->bb->seg_demand_last > eng->bb->seg_chunks) {
        uint64_t want = eng->bb->seg_demand_last + eng->bb->seg_demand_last / 4 + 64;
        TM_TRY_HIP(eng->grow_buf(eng->bb->d_seg_pool, want * SEG_CHUNK * sizeof(uint4)), TM_ENOMEM,
                   "alloc seg pool (" + std::to_string(want * SEG_CHUNK * sizeof(uint4)) + " B for a demand of " +
                       std::to_string(eng->bb->seg_demand_last) + " chunks)");
        eng->bb->seg_chunks = want;
    }
    if (eng->bb->fr_demand_last > eng->bb->fr_chunks) {
        uint64_t want = eng->bb->fr_demand_last + eng->bb->fr_demand_last / 4 + 64;
        TM_TRY_HIP(eng->grow_buf(eng->bb->d_fr_pool, want * FR_CHUNK * sizeof(uint2)), TM_ENOMEM, "alloc frontier pool");
        eng->bb->fr_chunks = want;
    }
    return TM_OK;
}

// `obase`: the batch's per-topic results go to d_outoff/d_outcnt/d_status + obase; `keys`,
// `keys_cap`: its key output (default: the whole arena)
// per-topic outputs of a batch in buffers the caller owns (the aggregator's windows)
struct TopicOut {
    uint32_t *off, *cnt, *kcnt;
    int32_t *status;
};
#ifndef TM_PREPASS
#define TM_PREPASS 0
#endif
// k_prescan ahead of k_match_fast<PRE>: off by default, measured 4 % slower
// (0.7185 vs 0.6923 ms per batch, profiles/r05_sweep_pre.jsonl) although it lifts the walk
// to 20 waves per CU; EMQX_TM_PREPASS=0 / 1 overrides the build's default per launch
static bool prepass_on() {
    const char *e = getenv("EMQX_TM_PREPASS");
    return e ? atoi(e) != 0 : TM_PREPASS != 0;
}

static hipError_t enqueue_match(tm_engine *eng, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                                hipStream_t s, uint32_t mode = MODE_ALL, uint32_t obase = 0, uint32_t *keys = nullptr,
                                uint64_t keys_cap = 0, unsigned long long *cursor = nullptr,
                                const TopicOut *to = nullptr, uint32_t tpw = 0) {
    MatchArgs a{};
    a.mode = mode;
    // [unique] / aggre/1 (set by the caller for this launch only): the walk counts each topic's
    // collapsible keys and leaves k_dedupe its worklist
    const uint32_t dd = eng->dd_next;
    eng->dd_next = 0;
    if (dd && mode == MODE_ALL && !to) {
        hipError_t e;
        if ((e = eng->grow_buf(eng->bb->d_ucnt, (uint64_t)(obase + n) * 4 + 4)) ||
            (e = eng->grow_buf(eng->bb->d_dd_wl, (uint64_t)n * 8 + 8)) || (e = eng->grow_buf(eng->bb->d_dd_wl_n, 4)) ||
            (e = hipMemsetAsync(eng->bb->d_dd_wl_n.p, 0, 4, s)))
            return e;
        a.dd_bit = dd;
        a.key_dd = eng->d_key_dd.as<uint8_t>();
        a.ucnt = eng->bb->d_ucnt.as<uint32_t>() + obase;
        a.wl = eng->bb->d_dd_wl.as<uint2>();
        a.wl_n = eng->bb->d_dd_wl_n.as<uint32_t>();
    }
    a.tpw = pick_tpw(n, tpw ? tpw : eng->cfg.topics_per_wave);
    a.first_dfs = eng->dv.n_deep ? 1u : 0u;
    a.key_bin = eng->d_key_bin.as<uint32_t>();
    a.key_rec = eng->d_key_rec.as<uint64_t>();
    a.topic_words = eng->topic_words ? 1u : 0u;
    a.bytes = d_bytes;
    a.off = d_off;
    a.n = n;
    a.force_slow = (eng->cfg.flags & TM_CFG_FORCE_SLOW) ? 1u : 0u;
    a.wtab = eng->d_wtab.as<WordSlot>();
    a.wmask = eng->dv.wmask;
    a.warena = eng->d_warena.as<uint8_t>();
    a.word_off = eng->d_word_off.as<uint32_t>();
    a.etab = eng->d_etab.as<EdgeSlot>();
    a.slot_list = eng->d_slot_list.as<uint32_t>();
    a.emask = eng->dv.emask;
    a.root = eng->d_root.as<RootRec>();
    a.arena = eng->d_arena.as<uint32_t>();
    a.out_off = eng->bb->d_outoff.as<uint32_t>() + obase;
    a.out_cnt = eng->bb->d_outcnt.as<uint32_t>() + obase;
    a.status = eng->bb->d_status.as<int32_t>() + obase;
    a.keys = keys ? keys : eng->bb->d_keys.as<uint32_t>();
    a.keys_cap = keys ? keys_cap : eng->bb->keys_cap;
    eng->bb->ctl_cur ^= 1u;
    eng->bb->p_ctl = eng->bb->d_ctl.as<uint8_t>() + eng->bb->ctl_cur * CTL_BYTES;
    a.cursor = cursor ? cursor : (unsigned long long *)(eng->bb->p_ctl + CTL_CURSOR);
    if (mode == MODE_RUNS) {
        a.out_kcnt = eng->bb->d_kcnt.as<uint32_t>() + obase;
        if (eng->runs_w == 4) {  // spans of the u32 id arena (the caller checked ids32())
            a.span_arena = (uint64_t)(uintptr_t)eng->arena_id32;
            a.span_keys = eng->key_id32.empty() ? 0 : (uint64_t)(uintptr_t)&eng->key_id32[0];
            a.span_w = 4;
            a.span_kstride = 4;
        } else if (eng->replica) {  // the replica's host copies (replica_ids_*)
            a.span_arena = (uint64_t)(uintptr_t)eng->arena_id;
            a.span_keys = eng->r_key_id.empty() ? 0 : (uint64_t)(uintptr_t)&eng->r_key_id[0];
            a.span_w = 8;
            a.span_kstride = 8;
        } else {
            a.span_arena = (uint64_t)(uintptr_t)eng->arena_id;
            a.span_keys = eng->keys.empty() ? 0 : (uint64_t)(uintptr_t)&eng->keys[0].id;
            a.span_w = 8;
            a.span_kstride = sizeof(KeyRec);
        }
    }
    if (to) {
        a.out_off = to->off;
        a.out_cnt = to->cnt;
        a.out_kcnt = to->kcnt;
        a.status = to->status;
    }
    a.ctl_next = (unsigned long long *)(eng->bb->d_ctl.as<uint8_t>() + (eng->bb->ctl_cur ^ 1u) * CTL_BYTES);
    a.slow_list = eng->bb->d_slow_list.as<uint32_t>();
    a.slow_count = (uint32_t *)(eng->bb->p_ctl + CTL_SLOW);
    a.scratch_w = eng->bb->d_scr_w.as<uint32_t>();
    a.scratch_s = eng->bb->d_scr_s.as<uint64_t>();
    a.seg_pool = eng->bb->d_seg_pool.as<uint4>();
    a.seg_chunks = eng->bb->seg_chunks;
    a.seg_cursor = (unsigned long long *)(eng->bb->p_ctl + CTL_SEG);
    a.wave_chunks = eng->bb->d_wave_chunks.as<uint32_t>();
    a.wave_info = eng->bb->d_wave_info.as<uint4>();
    a.fr_pool = eng->bb->d_fr_pool.as<uint2>();
    a.fr_chunks = eng->bb->fr_chunks;
    a.fr_cursor = (unsigned long long *)(eng->bb->p_ctl + CTL_FR);
    if (mode != MODE_FIRST && prepass_on() && TM_PRELOOK > 0) {
        // k_prescan's output, SoA: level l's word ids at [l * stride, ..), then the topics' meta
        const uint64_t stride = ((uint64_t)n + 63) & ~63ull;
        const uint64_t want = stride * TM_PRELOOK * 4 + stride * 8;
        if (eng->bb->d_pre.cap < want) {
            const hipError_t e = eng->grow_buf(eng->bb->d_pre, want + want / 4);
            if (e) return e;
        }
        a.pre_wid = eng->bb->d_pre.as<uint32_t>();
        a.pre_meta = reinterpret_cast<uint2 *>(eng->bb->d_pre.as<uint8_t>() + stride * TM_PRELOOK * 4);
        a.pre_stride = (uint32_t)stride;
    }
    a.stats = eng->stats_on ? eng->d_stats.as<unsigned long long>() : nullptr;
    a.ev_fast0 = eng->timing_on ? eng->ev_fast0 : nullptr;
    a.ev_fast1 = eng->timing_on ? eng->ev_fast1 : nullptr;
    eng->fill_caps(a);
    const hipError_t e = launch_match(a, s);
    return e ? e : eng->bnd_after(s, "match");
}

// UNIQUE / AGGRE on the GPU: k_dedupe reduces the full result of the batch just enqueued
// in place in d_keys, the reduced counts in d_ucnt.
static bool reduced_mode(uint32_t mode) { return mode == TM_MATCH_UNIQUE || mode == TM_MATCH_AGGRE; }
static uint32_t dd_bit_of(uint32_t mode) { return mode == TM_MATCH_UNIQUE ? KDD_MULTI : KDD_SHARED; }

// The walk just enqueued (with dd_next set) wrote the final count of every topic that cannot
// collapse and listed the others; k_dedupe reduces those in place (round 5: k_dd_pass, a second
// read of every key and a gather of every key's flag, is gone).
static int enqueue_reduce(tm_engine *eng, uint32_t mode, uint32_t n, hipStream_t s) {
    if (eng->bb->ukeys_cap < eng->bb->keys_cap) {
        TM_TRY_HIP(eng->grow_buf(eng->bb->d_ukeys, eng->bb->keys_cap * 4), TM_ENOMEM, "alloc reduced keys");
        eng->bb->ukeys_cap = eng->bb->keys_cap;
    }
    TM_TRY_HIP(launch_dedupe_wl(mode == TM_MATCH_UNIQUE ? DD_UNIQUE : DD_AGGRE, eng->bb->d_outcnt.as<uint32_t>(),
                                eng->bb->d_outoff.as<uint32_t>(), eng->bb->d_keys.as<uint32_t>(),
                                eng->d_key_rec.as<uint64_t>(), eng->d_key_node.as<uint32_t>(), eng->d_key_dd.as<uint8_t>(),
                                n, eng->bb->d_ucnt.as<uint32_t>(), eng->bb->d_ukeys.as<uint32_t>(),
                                eng->bb->d_dd_wl.as<uint2>(), eng->bb->d_dd_wl_n.as<uint32_t>(), s),
               TM_EDEVICE, "dedupe");
    return TM_OK;
}


// Host batches of TM_MATCH_ALL with at least 2 * PIPE_SUB topics run as sub-batches of
// about PIPE_SUB topics on two streams: sub-batch j+1 is staged, copied in and walked while
// sub-batch j's keys cross PCIe.  The keys D2H (PCIe) is the bound of this path, so the
// walk, the staging and the H2D hide behind it.
constexpr uint32_t PIPE_SUB = 262144;
constexpr uint32_t PIPE_MAXSUB = 8;

static int match_batch_pipelined(tm_engine *eng, HostOut &o, const uint8_t *bytes, const uint32_t *off, uint32_t n,
                                 tm_result *out) {
    // called without the device lock: it is taken only around the walks and the buffer sizing
    const uint32_t base = off[0];
    const uint64_t nbytes = (uint64_t)off[n] - base;
    const uint32_t S = std::max<uint32_t>(2, std::min<uint32_t>(PIPE_MAXSUB, n / PIPE_SUB));
    uint32_t b[PIPE_MAXSUB + 1];
    for (uint32_t j = 0; j <= S; j++) b[j] = (uint32_t)((uint64_t)n * j / S);
    BatchBufs &B = o.bb;
    // each half of the key arena holds one sub-batch; sized from this thread's last pipelined batch
    const uint64_t est_sub = (uint64_t)(o.pipe_kpt * (double)(n / S + 1) * 1.15) + 4096;
    {
        std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
        eng->bb = &B;
        int rc = ensure_batch(eng, n, nbytes);
        if (rc) return rc;
        TM_TRY_HIP(eng->grow_buf(B.d_bytes, nbytes + 16), TM_ENOMEM, "alloc");
        TM_TRY_HIP(eng->grow_buf(B.d_off, ((size_t)n + 1) * 4), TM_ENOMEM, "alloc");
        if (B.keys_cap < 2 * est_sub) {
            TM_TRY_HIP(eng->grow_buf(B.d_keys, 2 * est_sub * 4), TM_ENOMEM, "alloc keys");
            B.keys_cap = 2 * est_sub;
        }
    }
    TM_TRY_HIP(o.h_bytes.ensure(nbytes + 16), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_off.ensure(((size_t)n + 1) * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_outoff.ensure((size_t)n * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_outcnt.ensure((size_t)n * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_status.ensure((size_t)n * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_ctl.ensure(2 * CTL_BYTES), TM_ENOMEM, "pinned alloc");
    uint64_t hc = B.keys_cap / 2;
    TM_TRY_HIP(o.h_keys.ensure((size_t)(o.pipe_kpt * (double)n * 1.1) * 4 + 4), TM_ENOMEM, "pinned alloc");
    hipStream_t s = o.s_walk, c = o.s_copy;
    uint8_t *hb8 = o.h_bytes.as<uint8_t>(), *hctl = o.h_ctl.as<uint8_t>();
    uint32_t *ho = o.h_off.as<uint32_t>();
    uint64_t hb[PIPE_MAXSUB] = {}, hbase = 0, seg_d = 0, fr_d = 0, slow = 0;

    auto stage = [&](uint32_t j) -> int {  // sub-batch j's topics into pinned memory, then H2D
        const uint32_t lo = b[j], hi = b[j + 1];
        const uint64_t blo = off[lo] - base, bhi = off[hi] - base;
        if (bhi > blo) memcpy(hb8 + blo, bytes + base + blo, bhi - blo);
        for (uint32_t i = lo; i <= hi; i++) ho[i] = off[i] - base;
        if (bhi > blo)
            TM_TRY_HIP(hipMemcpyAsync(B.d_bytes.as<uint8_t>() + blo, hb8 + blo, bhi - blo, hipMemcpyHostToDevice, s),
                       TM_EDEVICE, "H2D");
        TM_TRY_HIP(hipMemcpyAsync(B.d_off.as<uint32_t>() + lo, ho + lo, ((size_t)hi - lo + 1) * 4, hipMemcpyHostToDevice, s),
                   TM_EDEVICE, "H2D");
        return TM_OK;
    };
    auto walk = [&](uint32_t j) -> int {  // sub-batch j walks into key half j % 2
        const uint32_t lo = b[j], hi = b[j + 1], h = j & 1;
        if (j >= 2) TM_TRY_HIP(hipStreamWaitEvent(s, o.ev_pd[h], 0), TM_EDEVICE, "wait");  // half's last D2H
        const uint8_t *pctl;
        {
            std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
            eng->bb = &B;
            B.last_n = hi - lo;
            TM_TRY_HIP(enqueue_match(eng, B.d_bytes.as<uint8_t>(), B.d_off.as<uint32_t>() + lo, hi - lo, s, MODE_ALL, lo,
                                     B.d_keys.as<uint32_t>() + h * hc, hc),
                       TM_EDEVICE, "kernel launch");
            TM_TRY_HIP(eng->note_use(s), TM_EDEVICE, "event");
            pctl = B.p_ctl;
        }
        TM_TRY_HIP(hipMemcpyAsync(hctl + h * CTL_BYTES, pctl, CTL_BYTES, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
        TM_TRY_HIP(hipEventRecord(o.ev_pk[h], s), TM_EDEVICE, "event");
        return TM_OK;
    };
    // sub-batch j's walk is done: its keys and per-topic results D2H on the copy stream
    // (1: its key half was too small)
    auto finish = [&](uint32_t j) -> int {
        const uint32_t lo = b[j], hi = b[j + 1], h = j & 1;
        TM_TRY_HIP(hipEventSynchronize(o.ev_pk[h]), TM_EDEVICE, "match kernels");
        const uint8_t *ctl = hctl + h * CTL_BYTES;
        const uint64_t total = *(const uint64_t *)ctl;
        if (total > hc) return 1;
        slow += *(const uint32_t *)(ctl + 8);
        seg_d = std::max(seg_d, *(const uint64_t *)(ctl + 16));
        fr_d = std::max(fr_d, *(const uint64_t *)(ctl + 24));
        if ((hbase + total) * 4 + 4 > o.h_keys.cap) {  // more keys than estimated: grow, keeping what landed
            TM_TRY_HIP(hipStreamSynchronize(c), TM_EDEVICE, "D2H");
            PinBuf nb;
            TM_TRY_HIP(nb.ensure((hbase + total) * 8 + 4), TM_ENOMEM, "pinned alloc");
            if (hbase) memcpy(nb.p, o.h_keys.p, hbase * 4);
            std::swap(nb.p, o.h_keys.p);
            std::swap(nb.cap, o.h_keys.cap);
            std::swap(nb.dev, o.h_keys.dev);
            nb.release();
        }
        TM_TRY_HIP(hipStreamWaitEvent(c, o.ev_pk[h], 0), TM_EDEVICE, "wait");
        TM_TRY_HIP(d2h_words(o.h_keys, hbase, B.d_keys.as<uint32_t>() + h * hc, total, c), TM_EDEVICE, "D2H");
        for (std::pair<PinBuf *, DevBuf *> pr : {std::make_pair(&o.h_outoff, &B.d_outoff), std::make_pair(&o.h_outcnt, &B.d_outcnt),
                                                 std::make_pair(&o.h_status, &B.d_status)})
            TM_TRY_HIP(hipMemcpyAsync(pr.first->as<uint32_t>() + lo, pr.second->as<uint32_t>() + lo, ((size_t)hi - lo) * 4,
                                      hipMemcpyDeviceToHost, c),
                       TM_EDEVICE, "D2H");
        TM_TRY_HIP(hipEventRecord(o.ev_pd[h], c), TM_EDEVICE, "event");
        hb[j] = hbase;
        hbase += total;
        return TM_OK;
    };

    int rc;
    if ((rc = stage(0)) || (rc = walk(0))) return rc;
    for (uint32_t j = 0; j < S; j++) {
        if (j + 1 < S && ((rc = stage(j + 1)) || (rc = walk(j + 1)))) return rc;
        rc = finish(j);
        if (rc == 1) {
            // the half was short: drain, grow both halves past this sub-batch's demand, walk
            // it (and the one queued behind it, whose output the move discards) again
            const uint64_t need = *(const uint64_t *)(hctl + (j & 1) * CTL_BYTES);
            TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "sync");
            TM_TRY_HIP(hipStreamSynchronize(c), TM_EDEVICE, "sync");
            const uint64_t want = 2 * (need + need / 8 + 1024);
            {
                std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
                TM_TRY_HIP(eng->grow_buf(B.d_keys, want * 4), TM_ENOMEM, "alloc keys");
                B.keys_cap = want;
            }
            hc = want / 2;
            if ((rc = walk(j)) || (j + 1 < S && (rc = walk(j + 1)))) return rc;
            rc = finish(j);
            if (rc == 1) return TM_EDEVICE;  // cannot happen: the half now holds the demand
        }
        if (rc) return rc;
    }
    TM_TRY_HIP(hipStreamSynchronize(c), TM_EDEVICE, "D2H");
    // sub-batch offsets are relative to its own keys: rebase onto the joined array
    uint32_t *oo = o.h_outoff.as<uint32_t>();
    for (uint32_t j = 1; j < S; j++)
        for (uint32_t i = b[j]; i < b[j + 1]; i++) oo[i] += (uint32_t)hb[j];
    {
        std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
        eng->bb = &B;
        eng->n_slow_last = slow;
        B.seg_demand_last = seg_d;
        B.fr_demand_last = fr_d;
        if ((rc = grow_pools(eng))) return rc;
    }
    o.pipe_kpt = (double)hbase / n;
    B.dev_batch = false;  // the device holds sub-batches, not this batch
    B.last_n = 0;
    out->total = hbase;
    out->off = oo;
    out->cnt = o.h_outcnt.as<uint32_t>();
    out->keys = o.h_keys.as<uint32_t>();
    out->status = o.h_status.as<int32_t>();
    return TM_OK;
}

// Host-form batch (tm_match_batch).  ALL / FIRST / COUNT run concurrently across threads: each
// thread has its own buffers and streams (HostOut::bb), and the device lock is held only while
// the walk is queued.  UNIQUE / AGGRE keep the lock across the call: their reducer reads key
// records the walk's result must match, so walk and reducer see one epoch.
static int match_batch_impl(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode,
                            tm_result *out) {
    if (!eng || !out || (n && (!off || (!bytes && off[n] > off[0])))) return TM_EINVAL;
    if (mode > TM_MATCH_AGGRE) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    // UNIQUE may reduce on the host (keys deeper than the device order code): term order of
    // keys needs the host copy, so that mode also holds mu_host (taken before mu_dev)
    std::unique_lock<std::mutex> gh(eng->mu_host, std::defer_lock);
    if (mode == TM_MATCH_UNIQUE && !eng->replica) gh.lock();
    HostOut &o = eng->out();
    memset(out, 0, sizeof(*out));
    out->n = n;
    TM_TRY_HIP(o.lanes(), TM_EDEVICE, "stream");
    BatchBufs &B = o.bb;
    std::unique_lock<std::recursive_mutex> gd(eng->mu_dev);
    eng->bb = &B;
    // UNIQUE is reduced on the GPU unless a key is too deep for the device order code
    const bool dev_reduce = reduced_mode(mode) && (mode == TM_MATCH_AGGRE || eng->dv.n_deep == 0);
    if (reduced_mode(mode) && !dev_reduce && eng->replica) return replica_refuses(eng, "tm_match_batch (host UNIQUE)");
    B.last_mode = (reduced_mode(mode) && !dev_reduce) ? TM_MATCH_ALL : mode;  // what the device holds
    if (n == 0) return TM_OK;
    if (mode == TM_MATCH_ALL && n >= 2 * PIPE_SUB) {
        gd.unlock();
        return match_batch_pipelined(eng, o, bytes, off, n, out);
    }
    const bool hold = reduced_mode(mode);  // keep the device lock across the whole call
    B.dev_batch = true;
    // rebase offsets to 0
    uint32_t base = off[0];
    uint64_t nbytes = (uint64_t)off[n] - base;
    int rc = ensure_batch(eng, n, nbytes);
    if (rc) return rc;
    TM_TRY_HIP(eng->grow_buf(B.d_bytes, nbytes + 16), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(B.d_off, ((size_t)n + 1) * 4), TM_ENOMEM, "alloc");
    // FIRST runs k_match_first (<= 1 key per topic); COUNT skips the key copy-out
    const uint32_t kmode = mode == TM_MATCH_FIRST ? MODE_FIRST : (mode == TM_MATCH_COUNT ? MODE_COUNT : MODE_ALL);
    if (kmode == MODE_FIRST && B.keys_cap < n) {
        TM_TRY_HIP(eng->grow_buf(B.d_keys, (uint64_t)n * 4), TM_ENOMEM, "alloc keys");
        B.keys_cap = n;
    }
    if (!hold) gd.unlock();
    TM_TRY_HIP(o.h_bytes.ensure(nbytes + 16), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_off.ensure(((size_t)n + 1) * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_ctl.ensure(64), TM_ENOMEM, "pinned alloc");
    if (nbytes) memcpy(o.h_bytes.p, bytes + base, nbytes);
    uint32_t *ho = o.h_off.as<uint32_t>();
    for (uint32_t i = 0; i <= n; i++) ho[i] = off[i] - base;
    hipStream_t s = o.s_walk;
    TM_TRY_HIP(hipMemcpyAsync(B.d_bytes.p, o.h_bytes.p, nbytes + 1, hipMemcpyHostToDevice, s), TM_EDEVICE, "H2D");
    TM_TRY_HIP(hipMemcpyAsync(B.d_off.p, ho, ((size_t)n + 1) * 4, hipMemcpyHostToDevice, s), TM_EDEVICE, "H2D");
    const uint64_t *ctl = o.h_ctl.as<uint64_t>();
    uint64_t total = 0;
    for (int attempt = 0; attempt < 2; attempt++) {
        {
            std::unique_lock<std::recursive_mutex> ga(eng->mu_dev, std::defer_lock);
            if (!hold) ga.lock();
            eng->bb = &B;
            if (attempt) {
                // output arena too small: grow to the demand and run again (once suffices:
                // the cursor counts every key the batch asked for)
                const uint64_t want = total + total / 8 + 1024;
                TM_TRY_HIP(eng->grow_buf(B.d_keys, want * 4), TM_ENOMEM, "alloc keys");
                B.keys_cap = want;
            }
            B.last_n = n;
            if (dev_reduce) eng->dd_next = dd_bit_of(mode);  // the walk counts collapsible keys
            TM_TRY_HIP(enqueue_match(eng, B.d_bytes.as<uint8_t>(), B.d_off.as<uint32_t>(), n, s, kmode), TM_EDEVICE,
                       "kernel launch");
            TM_TRY_HIP(eng->note_use(s), TM_EDEVICE, "event");
            // the counter block has the host layout: cursor @0, slow_count @8, seg @16, fr @24
            TM_TRY_HIP(hipMemcpyAsync(o.h_ctl.p, B.p_ctl, CTL_BYTES, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
        }
        TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "match kernels");
        total = ctl[0];
        B.seg_demand_last = ctl[2];
        B.fr_demand_last = ctl[3];
        if (kmode != MODE_ALL || total <= B.keys_cap) break;
    }
    const uint32_t n_slow = (uint32_t)ctl[1];
    total = kmode == MODE_ALL ? total : (kmode == MODE_FIRST ? n : 0);
    if (dev_reduce && (rc = enqueue_reduce(eng, mode, n, s))) return rc;  // (hold: under the lock)
    TM_TRY_HIP(o.h_outoff.ensure((size_t)n * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_outcnt.ensure((size_t)n * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_status.ensure((size_t)n * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_keys.ensure(total * 4 + 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(hipMemcpyAsync(o.h_outoff.p, B.d_outoff.p, (size_t)n * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
    TM_TRY_HIP(hipMemcpyAsync(o.h_outcnt.p, (dev_reduce ? B.d_ucnt : B.d_outcnt).p, (size_t)n * 4, hipMemcpyDeviceToHost, s),
               TM_EDEVICE, "D2H");
    TM_TRY_HIP(hipMemcpyAsync(o.h_status.p, B.d_status.p, (size_t)n * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
    TM_TRY_HIP(d2h_words(o.h_keys, 0, B.d_keys.p, total, s), TM_EDEVICE, "D2H");
    TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "D2H");
    {
        std::unique_lock<std::recursive_mutex> ga(eng->mu_dev, std::defer_lock);
        if (!hold) ga.lock();
        eng->bb = &B;
        eng->n_slow_last = n_slow;
        if ((rc = grow_pools(eng))) return rc;
    }
    if (gd.owns_lock()) gd.unlock();
    out->total = total;
    out->off = o.h_outoff.as<uint32_t>();
    out->cnt = o.h_outcnt.as<uint32_t>();
    out->keys = o.h_keys.as<uint32_t>();
    out->status = o.h_status.as<int32_t>();
    if (mode == TM_MATCH_ALL) return TM_OK;
    if (dev_reduce) {  // reduced lists sit at the full result's offsets, with gaps
        uint64_t t = 0;
        for (uint32_t i = 0; i < n; i++) t += out->cnt[i];
        out->total = t;
        return TM_OK;
    }
    if (mode == TM_MATCH_COUNT) {  // counts only: no keys
        o.pp_off.assign(n, 0);
        out->off = o.pp_off.data();
        out->keys = nullptr;
        out->total = 0;
        return TM_OK;
    }
    if (mode == TM_MATCH_FIRST) {  // k_match_first wrote topic i's key (if any) at keys[i]: compact
        o.pp_off.resize(n);
        o.pp_keys.clear();
        for (uint32_t i = 0; i < n; i++) {
            o.pp_off[i] = (uint32_t)o.pp_keys.size();
            if (out->cnt[i]) o.pp_keys.push_back(out->keys[i]);
        }
        out->off = o.pp_off.data();
        out->keys = o.pp_keys.data();
        out->total = o.pp_keys.size();
        return TM_OK;
    }

    // UNIQUE with a key deeper than the device order code: reduce each topic's set under
    // ETS term order here.
    o.pp_off.resize(n);
    o.pp_cnt.resize(n);
    o.pp_keys.clear();
    std::vector<uint32_t> tmp;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t *ks = out->keys + out->off[i];
        uint32_t c = out->cnt[i];
        o.pp_off[i] = (uint32_t)o.pp_keys.size();
        if (c == 0) {
            o.pp_cnt[i] = 0;
            continue;
        }
        tmp.assign(ks, ks + c);
        std::sort(tmp.begin(), tmp.end(), [&](uint32_t a, uint32_t b) { return eng->cmp_keys(a, b) < 0; });
        // maps:put in ascending walk order: the last (greatest) key per id wins,
        // maps:values/1 returns them ordered by id (small maps are sorted).
        std::vector<std::pair<uint64_t, uint32_t>> best;
        std::unordered_map<uint64_t, size_t> at;  // id -> index in best
        at.reserve(tmp.size() * 2);
        for (uint32_t k : tmp) {
            const uint64_t id = eng->keys[k].id;
            auto ins = at.emplace(id, best.size());
            if (ins.second) best.push_back({id, k});
            else best[ins.first->second].second = k;
        }
        std::sort(best.begin(), best.end());
        for (auto &p : best) o.pp_keys.push_back(p.second);
        o.pp_cnt[i] = (uint32_t)best.size();
    }
    out->off = o.pp_off.data();
    out->cnt = o.pp_cnt.data();
    out->keys = o.pp_keys.data();
    out->total = o.pp_keys.size();
    return TM_OK;
}

// matches/3 with a pre-split topic `[word()]` (emqx_trie_search.erl:182, topic_words/1 :369-370):
// the words come '/'-joined.  The walk is the same as for a binary topic except that a "+" or
// "#" level is a plain word (no badarg: topic_words/1 checks nothing for a list), and the
// final match_topics/4 step (:380-389) compares the LIST with the keys, so a key given as a
// binary ({Binary, {ID}}, K_EXACT_BIN) never matches: those are dropped here, on the host,
// which knows every key's form.  FIRST needs no filtering beyond that (binary keys sort after
// every list: a binary first key means no list key matched); COUNT and UNIQUE are taken from
// the filtered full result.
static int match_words_batch(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode,
                             tm_result *out) {
    if (mode > TM_MATCH_COUNT) {
        eng->err = "tm_match_batch: TM_MATCH_TOPIC_WORDS supports ALL, UNIQUE, FIRST and COUNT";
        return TM_EINVAL;
    }
    if (eng->replica) return replica_refuses(eng, "tm_match_batch (word-list topics)");
    std::lock_guard<std::mutex> gh(eng->mu_host);  // key kinds and term order: the host copy
    std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
    struct Flag {
        tm_engine *e;
        ~Flag() { e->topic_words = false; }
    } reset{eng};
    eng->topic_words = true;
    const uint32_t inner = mode == TM_MATCH_FIRST ? TM_MATCH_FIRST : TM_MATCH_ALL;
    int rc = match_batch_impl(eng, bytes, off, n, inner, out);
    if (rc || n == 0) return rc;
    HostOut &o = eng->out();
    std::vector<uint32_t> noff(n), ncnt(n), nkeys;
    nkeys.reserve(out->total);
    std::vector<uint32_t> tmp;
    for (uint32_t i = 0; i < n; i++) {
        const uint32_t *ks = out->keys ? out->keys + out->off[i] : nullptr;
        const uint32_t c = out->status[i] == TM_TOPIC_OK ? out->cnt[i] : 0;
        noff[i] = (uint32_t)nkeys.size();
        tmp.clear();
        for (uint32_t k = 0; k < c; k++)
            if (eng->keys[ks[k]].kind != K_EXACT_BIN) tmp.push_back(ks[k]);
        if (mode == TM_MATCH_UNIQUE && tmp.size() > 1) {
            // matches/3 [unique]: per id the greatest key in term order (match_add/2 overwrites)
            std::sort(tmp.begin(), tmp.end(), [&](uint32_t a, uint32_t b) { return eng->cmp_keys(a, b) < 0; });
            std::vector<std::pair<uint64_t, uint32_t>> best;
            std::unordered_map<uint64_t, size_t> at;
            for (uint32_t k : tmp) {
                auto ins = at.emplace(eng->keys[k].id, best.size());
                if (ins.second) best.push_back({eng->keys[k].id, k});
                else best[ins.first->second].second = k;
            }
            std::sort(best.begin(), best.end());
            tmp.clear();
            for (auto &p : best) tmp.push_back(p.second);
        }
        ncnt[i] = (uint32_t)tmp.size();
        if (mode != TM_MATCH_COUNT) nkeys.insert(nkeys.end(), tmp.begin(), tmp.end());
    }
    o.pp_off.swap(noff);
    o.pp_cnt.swap(ncnt);
    o.pp_keys.swap(nkeys);
    out->off = o.pp_off.data();
    out->cnt = o.pp_cnt.data();
    out->keys = mode == TM_MATCH_COUNT ? nullptr : o.pp_keys.data();
    out->total = o.pp_keys.size();
    if (mode == TM_MATCH_COUNT) {
        std::fill(o.pp_off.begin(), o.pp_off.end(), 0u);
        out->total = 0;
    }
    return TM_OK;
}

int tm_match_batch(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode,
                   tm_result *out) {
    if (!eng) return TM_EINVAL;
    if (mode & TM_MATCH_TOPIC_WORDS) {
        if (!out || (n && (!off || (!bytes && off[n] > off[0])))) return TM_EINVAL;
        return match_words_batch(eng, bytes, off, n, mode & ~TM_MATCH_TOPIC_WORDS, out);
    }
    return match_batch_impl(eng, bytes, off, n, mode, out);
}

int tm_reserve_matches(tm_engine *eng, uint64_t keys_cap, uint32_t topics_cap) {
    if (!eng) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    // the tm_match_device* path (host calls size their own output); the second direct set
    // once it is in use
    for (BatchBufs *b : {&eng->bb_dev, &eng->bb_dev2, &eng->bb_dev3}) {
        if (b != &eng->bb_dev && !b->keys_cap) continue;
        eng->bb = b;
        if (keys_cap > eng->bb->keys_cap) {
            TM_TRY_HIP(eng->grow_buf(eng->bb->d_keys, keys_cap * 4), TM_ENOMEM, "alloc keys");
            eng->bb->keys_cap = keys_cap;
        }
    }
    eng->bb = &eng->bb_dev;
    (void)topics_cap;
    return TM_OK;
}

int tm_match_device(tm_engine *eng, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                    uint64_t total_bytes, void *stream, tm_dev_result *out) {
    return tm_match_device_mode(eng, d_bytes, d_off, n, total_bytes, TM_MATCH_ALL, stream, out);
}

static int match_device_impl(tm_engine *eng, BatchBufs *set, const uint8_t *d_bytes, const uint32_t *d_off,
                             uint32_t n, uint64_t total_bytes, uint32_t mode, void *stream, tm_dev_result *out) {
    if (mode > TM_MATCH_AGGRE) return TM_EINVAL;
    if (!eng || !out || !d_off || (n && !d_bytes)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    eng->bb = set;
    if (mode == TM_MATCH_UNIQUE && eng->dv.n_deep) {
        eng->err = "tm_match_device_mode: UNIQUE with filters deeper than 31 levels is host-only (tm_match_batch)";
        return TM_ESTATE;
    }
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    // the batch buffers are reused: after everything queued behind the previous batch
    TM_TRY_HIP(eng->chain_after_last(s), TM_EDEVICE, "stream order");
    // total_bytes = d_off[n] - d_off[0] sizes the spill kernel's scratch
    int rc = ensure_batch(eng, n, total_bytes);
    if (rc) return rc;
    eng->bb->last_stream = s;
    eng->bb->last_n = n;
    const uint32_t kmode = mode == TM_MATCH_FIRST ? MODE_FIRST : (mode == TM_MATCH_COUNT ? MODE_COUNT : MODE_ALL);
    if (kmode == MODE_FIRST && eng->bb->keys_cap < n) {
        TM_TRY_HIP(eng->grow_buf(eng->bb->d_keys, (uint64_t)n * 4), TM_ENOMEM, "alloc keys");
        eng->bb->keys_cap = n;
    }
    if (reduced_mode(mode)) eng->dd_next = dd_bit_of(mode);  // the walk counts collapsible keys
    TM_TRY_HIP(enqueue_match(eng, d_bytes, d_off, n, s, kmode), TM_EDEVICE, "kernel launch");
    eng->bb->last_mode = mode;
    eng->bb->dev_batch = true;
    if (reduced_mode(mode) && (rc = enqueue_reduce(eng, mode, n, s))) return rc;
    TM_TRY_HIP(eng->note_use(s), TM_EDEVICE, "event");
    out->n = n;
    out->d_off = eng->bb->d_outoff.as<uint32_t>();
    out->d_cnt = (reduced_mode(mode) ? eng->bb->d_ucnt : eng->bb->d_outcnt).as<uint32_t>();
    out->d_keys = eng->bb->d_keys.as<uint32_t>();  // reduced modes compact in place
    out->d_status = eng->bb->d_status.as<int32_t>();
    out->d_total = (uint64_t *)(eng->bb->p_ctl + CTL_CURSOR);
    out->keys_cap = eng->bb->keys_cap;
    return TM_OK;
}

int tm_match_device_mode(tm_engine *eng, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                         uint64_t total_bytes, uint32_t mode, void *stream, tm_dev_result *out) {
    return eng ? match_device_impl(eng, &eng->bb_dev, d_bytes, d_off, n, total_bytes, mode, stream, out) : TM_EINVAL;
}
static BatchBufs *direct_set(tm_engine *eng, uint32_t set) {
    return !eng ? nullptr : set == 0 ? &eng->bb_dev : set == 1 ? &eng->bb_dev2 : set == 2 ? &eng->bb_dev3 : nullptr;
}
int tm_match_device_set(tm_engine *eng, uint32_t set, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                        uint64_t total_bytes, uint32_t mode, void *stream, tm_dev_result *out) {
    BatchBufs *b = direct_set(eng, set);
    return b ? match_device_impl(eng, b, d_bytes, d_off, n, total_bytes, mode, stream, out) : TM_EINVAL;
}
// library-internal (batcher.cpp): the same on the aggregator's own buffer set, so its windows
// never disturb a direct tm_match_device caller's pending result
__attribute__((visibility("hidden"))) int tmx_batch_match_device(tm_engine *eng, uint32_t set, const uint8_t *d_bytes,
                                                                 const uint32_t *d_off, uint32_t n, uint64_t total_bytes,
                                                                 uint32_t mode, void *stream, tm_dev_result *out) {
    return match_device_impl(eng, eng->batch_set(set), d_bytes, d_off, n, total_bytes, mode, stream, out);
}

int tm_device_sync(tm_engine *eng) { return tm_device_sync_set(eng, 0); }

int tm_device_sync_set(tm_engine *eng, uint32_t set) {
    BatchBufs *b = direct_set(eng, set);
    if (!b) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    eng->bb = b;
    hipStream_t s = eng->bb->last_stream ? eng->bb->last_stream : eng->stream;
    TM_TRY_HIP(eng->h_cursor.ensure(64), TM_ENOMEM, "pinned alloc");
    uint8_t *h = (uint8_t *)eng->h_cursor.p;
    if (eng->bb->p_ctl)
        TM_TRY_HIP(hipMemcpyAsync(h, eng->bb->p_ctl, CTL_BYTES, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
    TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "sync");
    if (eng->bb->p_ctl) {
        eng->n_slow_last = *(uint32_t *)(h + 8);
        eng->bb->seg_demand_last = *(uint64_t *)(h + 16);
        eng->bb->fr_demand_last = *(uint64_t *)(h + 24);
        if (eng->bb->seg_demand_last >> 31 || eng->bb->fr_demand_last >> 31) {
            // a counter block no launch could have produced (a wave takes at most SEG_MAXCHUNK
            // chunks): report it instead of sizing a pool from it
            char m[256];
            snprintf(m, sizeof m, "tm_device_sync: impossible counter block (block %u of %p: cursor %llx seg %llx fr %llx)",
                     eng->bb->ctl_cur, (void *)eng->bb->d_ctl.p, (unsigned long long)*(uint64_t *)h,
                     (unsigned long long)eng->bb->seg_demand_last, (unsigned long long)eng->bb->fr_demand_last);
            eng->err = m;
            eng->bb->seg_demand_last = eng->bb->fr_demand_last = 0;
            return TM_EDEVICE;
        }
        return grow_pools(eng);
    }
    return TM_OK;
}

int tm_result_ids_device(tm_engine *eng, uint64_t *d_ids, uint64_t ids_cap, uint32_t *d_off_out, void *stream) {
    return tm_result_ids_device_ex(eng, d_ids, ids_cap, d_off_out, nullptr, stream);
}

static int result_ids_impl(tm_engine *eng, BatchBufs *set, uint64_t *d_ids, uint64_t ids_cap, uint32_t *d_off_out,
                           uint32_t *d_flags, void *stream) {
    if (!eng || !d_off_out || (ids_cap && !d_ids)) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    eng->bb = set;
    if (!eng->bb->p_ctl || !eng->bb->dev_batch) {
        eng->err = "tm_result_ids_device: no tm_match_device batch since the last (pipelined) tm_match_batch";
        return TM_ESTATE;
    }
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    hipStream_t s = stream ? (hipStream_t)stream : (eng->bb->last_stream ? eng->bb->last_stream : eng->stream);
    const uint32_t n = eng->bb->last_n;
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_res_scan, scan_scratch_words(n) * 4), TM_ENOMEM, "alloc");
    const bool red = reduced_mode(eng->bb->last_mode);
    const uint32_t *cnt = (red ? eng->bb->d_ucnt : eng->bb->d_outcnt).as<uint32_t>();
    TM_TRY_HIP(launch_excl_scan(cnt, 1, n, d_off_out, eng->bb->d_res_scan.as<uint32_t>(), s), TM_EDEVICE, "scan");
    TM_TRY_HIP(launch_result_ids(cnt, eng->bb->d_outoff.as<uint32_t>(), eng->bb->d_keys.as<uint32_t>(),
                                 eng->d_key_rec.as<uint64_t>(), d_off_out, n, d_ids, ids_cap, eng->bb->keys_cap,
                                 (const unsigned long long *)(eng->bb->p_ctl + CTL_CURSOR), d_flags, s),
               TM_EDEVICE, "result ids");
    TM_TRY_HIP(eng->note_use(s), TM_EDEVICE, "event");
    return TM_OK;
}

int tm_result_ids_device_ex(tm_engine *eng, uint64_t *d_ids, uint64_t ids_cap, uint32_t *d_off_out, uint32_t *d_flags,
                            void *stream) {
    return eng ? result_ids_impl(eng, &eng->bb_dev, d_ids, ids_cap, d_off_out, d_flags, stream) : TM_EINVAL;
}
__attribute__((visibility("hidden"))) int tmx_result_ids64_device(tm_engine *eng, uint32_t set, uint64_t *d_ids,
                                                                  uint64_t ids_cap, uint32_t *d_off_out, void *stream) {
    return result_ids_impl(eng, eng->batch_set(set), d_ids, ids_cap, d_off_out, nullptr, stream);
}

// library-internal (batcher.cpp): tm_result_ids_device with u32 ids, when every id ever
// added is below 2^32 (TM_ESTATE otherwise)
__attribute__((visibility("hidden"))) int tmx_result_ids32_device(tm_engine *eng, uint32_t set, uint32_t *d_ids,
                                                                  uint64_t ids_cap, uint32_t *d_off_out, void *stream) {
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    eng->bb = eng->batch_set(set);
    if (eng->dv.max_id > 0xFFFFFFFFull || eng->replica || !eng->bb->dev_batch) return TM_ESTATE;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    hipStream_t s = stream ? (hipStream_t)stream : (eng->bb->last_stream ? eng->bb->last_stream : eng->stream);
    const uint32_t n = eng->bb->last_n;
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_res_scan, scan_scratch_words(n) * 4), TM_ENOMEM, "alloc");
    const uint32_t *cnt = (reduced_mode(eng->bb->last_mode) ? eng->bb->d_ucnt : eng->bb->d_outcnt).as<uint32_t>();
    TM_TRY_HIP(launch_excl_scan(cnt, 1, n, d_off_out, eng->bb->d_res_scan.as<uint32_t>(), s), TM_EDEVICE, "scan");
    TM_TRY_HIP(launch_result_ids32(cnt, eng->bb->d_outoff.as<uint32_t>(), eng->bb->d_keys.as<uint32_t>(),
                                   eng->d_key_rec.as<uint64_t>(), d_off_out, n, d_ids, ids_cap, eng->bb->keys_cap,
                                   (const unsigned long long *)(eng->bb->p_ctl + CTL_CURSOR), s),
               TM_EDEVICE, "result ids");
    TM_TRY_HIP(eng->note_use(s), TM_EDEVICE, "event");
    return TM_OK;
}

static int match_ids_impl(tm_engine *eng, BatchBufs *set, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                          uint64_t total_bytes, uint32_t id_bytes, void *d_ids, uint64_t ids_cap, uint32_t *d_off_out,
                          uint32_t *d_flags, void *stream, tm_dev_result *out) {
    if (!eng || !d_off || (n && !d_bytes) || !d_off_out || (ids_cap && !d_ids) || (id_bytes != 4 && id_bytes != 8))
        return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    eng->bb = set;
    if (id_bytes == 4 && eng->dv.max_id > 0xFFFFFFFFull) {
        eng->err = "tm_match_ids_device: an id of this index does not fit 32 bits";
        return TM_ESTATE;
    }
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    TM_TRY_HIP(eng->chain_after_last(s), TM_EDEVICE, "stream order");
    int rc = ensure_batch(eng, n, total_bytes);
    if (rc) return rc;
    eng->bb->last_stream = s;
    eng->bb->last_n = n;
    // the walk writes its ids wave-ordered into the batch's key buffer (as many u32 words per
    // id as id_bytes needs), then one pass copies them topic-major into the caller's buffer
    const uint64_t cap = eng->bb->keys_cap / (id_bytes / 4);
    const uint32_t kmode = id_bytes == 4 ? MODE_IDS32 : MODE_IDS64;
    const uint32_t tpw = pick_tpw(n, eng->cfg.topics_per_wave);
    const uint32_t nwaves = (uint32_t)match_grid(n, tpw);
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_wave_info, (uint64_t)nwaves * 16 + 16), TM_ENOMEM, "alloc");
    TM_TRY_HIP(enqueue_match(eng, d_bytes, d_off, n, s, kmode, 0, eng->bb->d_keys.as<uint32_t>(), cap),
               TM_EDEVICE, "kernel launch");
    eng->bb->last_mode = TM_MATCH_ALL;
    eng->bb->dev_batch = false;  // the key buffer holds ids now: no tm_result_ids_device on it
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_res_scan, scan_scratch_words(n) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(launch_excl_scan(eng->bb->d_outcnt.as<uint32_t>(), 1, n, d_off_out, eng->bb->d_res_scan.as<uint32_t>(), s),
               TM_EDEVICE, "scan");
    TM_TRY_HIP(launch_compact_waves(id_bytes, eng->bb->d_wave_info.as<uint4>(), nwaves, tpw, n,
                                    eng->bb->d_outoff.as<uint32_t>(), eng->bb->d_outcnt.as<uint32_t>(), eng->bb->d_keys.p,
                                    d_off_out, d_ids, ids_cap, cap,
                                    (const unsigned long long *)(eng->bb->p_ctl + CTL_CURSOR), d_flags, s),
               TM_EDEVICE, "compact ids");
    TM_TRY_HIP(eng->note_use(s), TM_EDEVICE, "event");
    if (out) {  // the walk's own per-topic arrays and counter block (library-internal callers)
        out->n = n;
        out->d_off = eng->bb->d_outoff.as<uint32_t>();
        out->d_cnt = eng->bb->d_outcnt.as<uint32_t>();
        out->d_keys = nullptr;
        out->d_status = eng->bb->d_status.as<int32_t>();
        out->d_total = (uint64_t *)(eng->bb->p_ctl + CTL_CURSOR);
        out->keys_cap = cap;
    }
    return TM_OK;
}

int tm_match_ids_device(tm_engine *eng, const uint8_t *d_bytes, const uint32_t *d_off, uint32_t n,
                        uint64_t total_bytes, uint32_t id_bytes, void *d_ids, uint64_t ids_cap, uint32_t *d_off_out,
                        uint32_t *d_flags, void *stream) {
    return eng ? match_ids_impl(eng, &eng->bb_dev, d_bytes, d_off, n, total_bytes, id_bytes, d_ids, ids_cap, d_off_out,
                                d_flags, stream, nullptr)
               : TM_EINVAL;
}
// library-internal (batcher.cpp): the same on the aggregator's own buffer set
__attribute__((visibility("hidden"))) int tmx_batch_match_ids(tm_engine *eng, uint32_t set, const uint8_t *d_bytes,
                                                              const uint32_t *d_off, uint32_t n, uint64_t total_bytes,
                                                              uint32_t id_bytes, void *d_ids, uint64_t ids_cap,
                                                              uint32_t *d_off_out, void *stream, tm_dev_result *out) {
    return match_ids_impl(eng, eng->batch_set(set), d_bytes, d_off, n, total_bytes, id_bytes, d_ids, ids_cap, d_off_out,
                          nullptr, stream, out);
}

int tm_merge_shard_ids_device(tm_engine *eng, uint32_t G, uint32_t n, const uint32_t *d_roff, uint64_t roff_stride,
                              const void *d_ids, uint32_t id_bytes, const uint64_t *base, uint64_t max_rank_ids,
                              uint32_t *d_out_off, uint64_t *d_out_ids, uint64_t out_cap, void *stream) {
    if (!eng || G == 0 || G > MERGE_MAX_G || !d_roff || !base || !d_out_off || roff_stride < (uint64_t)n + 1 ||
        (id_bytes != 4 && id_bytes != 8) || (out_cap && (!d_out_ids || !d_ids)) || max_rank_ids > 0xFFFFFFFFull)
        return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    TM_TRY_HIP(launch_merge_shard_ids(G, n, d_roff, roff_stride, d_ids, id_bytes, base, d_out_off, d_out_ids, out_cap,
                                      (uint32_t)max_rank_ids, s),
               TM_EDEVICE, "merge");
    return TM_OK;
}

int tm_merge_shards_device(tm_engine *eng, uint32_t G, uint32_t n, const uint32_t *d_counts, const uint64_t *d_ids,
                           uint64_t stride, uint32_t *d_off_out, uint64_t *d_ids_out, uint64_t out_cap, void *stream) {
    if (!eng || G == 0 || !d_off_out || (n && (!d_counts || !d_ids)) || (out_cap && !d_ids_out)) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    eng->bb = &eng->bb_dev;  // the device path's set (the sharded step's walk ran on it)
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_res_scan, scan_scratch_words(n) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->d_mrg_roff, (uint64_t)G * (n + 1) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->d_mrg_tot, (uint64_t)n * 4 + 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(launch_merge_shards(G, n, d_counts, d_ids, stride, eng->d_mrg_roff.as<uint32_t>(),
                                   eng->d_mrg_tot.as<uint32_t>(), eng->bb->d_res_scan.as<uint32_t>(), d_off_out, d_ids_out,
                                   out_cap, s),
               TM_EDEVICE, "merge");
    return TM_OK;
}

int tm_merge_shards(uint32_t G, uint32_t n, const uint32_t *counts, const uint64_t *ids, uint64_t stride,
                    uint32_t *off_out, uint64_t *ids_out, uint64_t out_cap) {
    if (G == 0 || !off_out || (n && (!counts || !ids))) return TM_EINVAL;
    std::vector<uint64_t> roff(G, 0);  // running source offset of each shard
    uint64_t total = 0;
    for (uint32_t t = 0; t < n; t++)
        for (uint32_t r = 0; r < G; r++) total += counts[(uint64_t)r * n + t];
    if (total > 0xFFFFFFFFull) return TM_EINVAL;
    if (total > out_cap || (total && !ids_out)) return TM_ENOMEM;
    uint64_t dst = 0;
    for (uint32_t t = 0; t < n; t++) {
        off_out[t] = (uint32_t)dst;
        for (uint32_t r = 0; r < G; r++) {
            const uint32_t c = counts[(uint64_t)r * n + t];
            if (roff[r] + c > stride) return TM_EINVAL;
            memcpy(ids_out + dst, ids + (uint64_t)r * stride + roff[r], (size_t)c * sizeof(uint64_t));
            roff[r] += c;
            dst += c;
        }
    }
    off_out[n] = (uint32_t)dst;
    return TM_OK;
}

int tm_key_info(const tm_engine *eng, uint32_t key, uint64_t *id, uint32_t *flags, uint8_t *buf, uint32_t cap,
                uint32_t *len) {
    if (!eng) return TM_EINVAL;
    std::lock_guard<std::mutex> g(const_cast<tm_engine *>(eng)->mu_host);
    if (key >= eng->keys.size() || eng->keys[key].kind == K_FREE) return TM_ENOTFOUND;
    const KeyRec &k = eng->keys[key];
    if (id) *id = k.id;
    if (flags) *flags = (k.kind == K_EXACT_WORDS) ? TM_KEY_WORDS : 0u;
    std::string f = eng->key_filter(key);
    if (len) *len = (uint32_t)f.size();
    if (buf && cap) memcpy(buf, f.data(), std::min<size_t>(cap, f.size()));
    return TM_OK;
}

int tm_key_ids(const tm_engine *eng, const uint32_t *keys, size_t n, uint64_t *ids_out) {
    if (!eng || (n && (!keys || !ids_out))) return TM_EINVAL;
    std::lock_guard<std::mutex> g(const_cast<tm_engine *>(eng)->mu_host);
    for (size_t i = 0; i < n; i++) {
        uint32_t k = keys[i];
        if (k >= eng->keys.size() || eng->keys[k].kind == K_FREE) return TM_ENOTFOUND;
        ids_out[i] = eng->keys[k].id;
    }
    return TM_OK;
}

// The queries of a matches_filter batch on the device and the walk's arguments (both forms):
// filter_words/1 as order codes, base_init/1's flag, per-query status.  Under mu_host + mu_dev.
static int filter_prepare(tm_engine *eng, HostOut &o, const uint8_t *bytes, const uint32_t *off, uint32_t n,
                          uint32_t mode, FilterArgs &a) {
    auto &fx = eng->fx;
    int rc;
    if (fx.epoch != eng->epoch && (rc = eng->build_filter_index())) return rc;
    // filter_words/1 (emqx_trie_search.erl:356-366) as order codes; base_init/1 flag
    fx.qw.clear();
    fx.qoff.assign(1, 0);
    fx.qdollar.assign(n, 0);
    o.f_status.assign(n, TM_TOPIC_OK);
    std::vector<std::pair<size_t, size_t>> lv;
    for (uint32_t i = 0; i < n; i++) {
        const char *t = (const char *)bytes + off[i];
        const size_t tl = off[i + 1] - off[i];
        tm_engine::split_words((const uint8_t *)t, tl, lv);
        for (size_t j = 0; j < lv.size(); j++) {
            uint32_t c = tm_engine::fx_level(t + lv[j].first, lv[j].second);
            if (c == 0 && j + 1 < lv.size()) o.f_status[i] = TM_BADARG;  // '#' before the last level
            if (c == NONE) {  // a literal: through the interner's hash table when it knows the word
                const uint8_t *wp = (const uint8_t *)t + lv[j].first;
                const uint32_t wl = (uint32_t)lv[j].second, wid = eng->word_lookup(wp, wl);
                if (wid == NONE || wid >= fx.wcode.size()) {
                    c = eng->fx_code((const char *)wp, wl);
                } else {
                    if (fx.wcode[wid] == NONE) fx.wcode[wid] = eng->fx_code((const char *)wp, wl);
                    c = fx.wcode[wid];
                }
            }
            fx.qw.push_back(c);
        }
        if (fx.qw.size() >= 0xFFFFFFFFull) return TM_EINVAL;
        fx.qoff.push_back((uint32_t)fx.qw.size());
        fx.qdollar[i] = tl && t[0] == '$';
    }
    hipStream_t s = eng->stream;
    fx.qw.insert(fx.qw.end(), 8, 0u);  // k_filter_walk preloads 8 words of a query unconditionally
    const size_t nq = fx.qw.size();
    TM_TRY_HIP(fx.d_qw.ensure(std::max<size_t>(nq, 1) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(fx.d_qoff.ensure(((size_t)n + 1) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(fx.d_qdollar.ensure(n), TM_ENOMEM, "alloc");
    TM_TRY_HIP(fx.d_qstatus.ensure((size_t)n * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(fx.d_cnt.ensure((size_t)n * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(fx.d_off.ensure(((size_t)n + 1) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(fx.d_scan.ensure(scan_scratch_words(n) * 4), TM_ENOMEM, "alloc");
    if (nq) TM_TRY_HIP(hipMemcpyAsync(fx.d_qw.p, fx.qw.data(), nq * 4, hipMemcpyHostToDevice, s), TM_EDEVICE, "H2D");
    TM_TRY_HIP(hipMemcpyAsync(fx.d_qoff.p, fx.qoff.data(), ((size_t)n + 1) * 4, hipMemcpyHostToDevice, s), TM_EDEVICE,
               "H2D");
    TM_TRY_HIP(hipMemcpyAsync(fx.d_qdollar.p, fx.qdollar.data(), n, hipMemcpyHostToDevice, s), TM_EDEVICE, "H2D");
    TM_TRY_HIP(hipMemcpyAsync(fx.d_qstatus.p, o.f_status.data(), (size_t)n * 4, hipMemcpyHostToDevice, s), TM_EDEVICE,
               "H2D");
    a.kw = fx.d_kw.as<uint32_t>();
    a.krec = fx.d_krec.as<uint4>();
    a.kend = fx.d_kend.as<uint32_t>();
    a.koff = fx.d_koff.as<uint32_t>();
    a.kh = fx.d_kh.as<uint32_t>();
    a.K = fx.K;
    a.n = n;
    a.qw = fx.d_qw.as<uint32_t>();
    a.qoff = fx.d_qoff.as<uint32_t>();
    a.qdollar = fx.d_qdollar.as<uint8_t>();
    a.qstatus = fx.d_qstatus.as<int32_t>();
    a.first = mode == TM_MATCH_FIRST;
    a.cnt = fx.d_cnt.as<uint32_t>();
    a.out_off = fx.d_off.as<uint32_t>();
    o.f_off.resize((size_t)n + 1);
    o.f_cnt.resize(n);
    return TM_OK;
}

int tm_match_filter_batch(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode,
                          tm_result *out) {
    if (!eng || !out || (n && (!off || (!bytes && off[n] > off[0])))) return TM_EINVAL;
    if (mode != TM_MATCH_ALL && mode != TM_MATCH_UNIQUE && mode != TM_MATCH_FIRST) return TM_EINVAL;
    if (eng->replica) return replica_refuses(eng, "tm_match_filter_batch");
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    // the walk's key index is built from the host copy (mu_host); it runs on the engine stream
    std::lock_guard<std::mutex> gh(eng->mu_host);
    std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
    HostOut &o = eng->out();
    memset(out, 0, sizeof(*out));
    out->n = n;
    if (n == 0) return TM_OK;
    auto &fx = eng->fx;
    FilterArgs a{};
    int rc = filter_prepare(eng, o, bytes, off, n, mode, a);
    if (rc) return rc;
    hipStream_t s = eng->stream;
    uint64_t total = 0;
    // One pass: the walk streams its keys into pooled chunks and copies them to a contiguous
    // range reserved at its end.  Sized from the demand of earlier batches; a batch that does
    // not fit takes the two-pass path below (count, scan, emit) and sizes the next one.
    bool done = false;
    {
        const uint64_t pool = std::max<uint64_t>(fx.pool_want, (uint64_t)n + 1024);
        const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>(fx.out_want, 1 << 16), 0xFFFFFFF0ull);
        TM_TRY_HIP(fx.d_pool.ensure(pool * FW_CHUNK * 4), TM_ENOMEM, "alloc filter pool");
        TM_TRY_HIP(fx.d_out.ensure(cap * 4), TM_ENOMEM, "alloc");
        TM_TRY_HIP(fx.d_ctl.ensure(24), TM_ENOMEM, "alloc");
        TM_TRY_HIP(hipMemsetAsync(fx.d_ctl.p, 0, 24, s), TM_EDEVICE, "memset");
        // bulk copy jobs: ranges of more than FW_BULK keys, all inside the output
        const uint64_t jobs = cap / FW_BULK + 64;
        TM_TRY_HIP(fx.d_jobs.ensure(jobs * sizeof(uint4)), TM_ENOMEM, "alloc filter jobs");
        a.pool = fx.d_pool.as<uint32_t>();
        a.pool_chunks = fx.d_pool.cap / (FW_CHUNK * 4);
        a.out = fx.d_out.as<uint32_t>();
        a.out_cap = fx.d_out.cap / 4;
        a.ctl = fx.d_ctl.as<unsigned long long>();
        a.jobs = fx.d_jobs.as<uint4>();
        a.jobs_cap = fx.d_jobs.cap / sizeof(uint4);
        uint64_t ctl[3] = {0, 0, 0};
        TM_TRY_HIP(launch_filter_walk(a, FW_ONEPASS, s), TM_EDEVICE, "k_filter_walk");
        TM_TRY_HIP(launch_filter_bulk(a, s), TM_EDEVICE, "k_filter_bulk");
        TM_TRY_HIP(hipMemcpyAsync(ctl, fx.d_ctl.p, 24, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
        TM_TRY_HIP(hipMemcpyAsync(o.f_off.data(), fx.d_off.p, (size_t)n * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE,
                   "D2H");
        TM_TRY_HIP(hipMemcpyAsync(o.f_cnt.data(), fx.d_cnt.p, (size_t)n * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE,
                   "D2H");
        TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "k_filter_walk");
        total = ctl[0];
        if (total <= a.out_cap && ctl[1] <= a.pool_chunks) {
            TM_TRY_HIP(o.f_keys.ensure(std::max<uint64_t>(total, 1) * 4), TM_ENOMEM, "pinned alloc");
            if (total) {
                TM_TRY_HIP(d2h_words(o.f_keys, 0, fx.d_out.p, total, s), TM_EDEVICE, "D2H");
                TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "k_filter_walk");
            }
            done = true;
        }
        fx.n_onepass += done;
    }
    if (!done) {
        fx.n_twopass++;
        TM_TRY_HIP(launch_filter_walk(a, FW_COUNT, s), TM_EDEVICE, "k_filter_walk count");
        TM_TRY_HIP(launch_excl_scan(a.cnt, 1, n, fx.d_off.as<uint32_t>(), fx.d_scan.as<uint32_t>(), s), TM_EDEVICE,
                   "scan");
        TM_TRY_HIP(hipMemcpyAsync(o.f_off.data(), fx.d_off.p, ((size_t)n + 1) * 4, hipMemcpyDeviceToHost, s),
                   TM_EDEVICE, "D2H");
        TM_TRY_HIP(hipMemcpyAsync(o.f_cnt.data(), fx.d_cnt.p, (size_t)n * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE,
                   "D2H");
        TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "k_filter_walk count");
        // the device scan is u32: a batch whose walks return 4 Gi keys or more is refused
        // before the emit pass could write past its offsets
        total = 0;
        for (uint32_t i = 0; i < n; i++) total += o.f_cnt[i];
        if (total >= 0xFFFFFFFFull) {
            eng->err = "tm_match_filter_batch: the batch returns 4 Gi keys or more; split it";
            return TM_ENOMEM;
        }
        // the next batch's one-pass sizes: this demand with headroom (a query wastes at most
        // one partly filled chunk; a chunk holds FW_CHUNK / 2 - 1 ranges)
        fx.out_want = total + total / 4 + 1024;
        fx.pool_want = (total / (FW_CHUNK / 2 - 1) + n) + (total / (FW_CHUNK / 2 - 1) + n) / 4 + 64;
        TM_TRY_HIP(o.f_keys.ensure(std::max<uint64_t>(total, 1) * 4), TM_ENOMEM, "pinned alloc");
        if (total) {
            TM_TRY_HIP(fx.d_out.ensure(total * 4), TM_ENOMEM, "alloc");
            a.out = fx.d_out.as<uint32_t>();
            TM_TRY_HIP(launch_filter_walk(a, FW_EMIT, s), TM_EDEVICE, "k_filter_walk emit");
            TM_TRY_HIP(d2h_words(o.f_keys, 0, fx.d_out.p, total, s), TM_EDEVICE, "D2H");
            TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "k_filter_walk emit");
        }
    }
    out->total = total;
    out->off = o.f_off.data();
    out->cnt = o.f_cnt.data();
    out->keys = o.f_keys.as<uint32_t>();
    out->status = o.f_status.data();
    if (mode == TM_MATCH_UNIQUE) {
        // match_add/2 into a map (:350-352): the last key per id in walk order wins;
        // maps:values/1 lists them by id
        o.f_ukeys.clear();
        std::vector<std::pair<uint64_t, uint32_t>> best;
        std::unordered_map<uint64_t, size_t> at;
        for (uint32_t i = 0; i < n; i++) {
            best.clear();
            at.clear();
            for (uint32_t k = o.f_off[i]; k < o.f_off[i] + o.f_cnt[i]; k++) {
                const uint32_t h = o.f_keys.as<uint32_t>()[k];
                const uint64_t id = eng->keys[h].id;
                auto it = at.find(id);
                if (it == at.end()) {
                    at.emplace(id, best.size());
                    best.emplace_back(id, h);
                } else {
                    best[it->second].second = h;
                }
            }
            std::sort(best.begin(), best.end());
            o.f_off[i] = (uint32_t)o.f_ukeys.size();
            o.f_cnt[i] = (uint32_t)best.size();
            for (auto &b : best) o.f_ukeys.push_back(b.second);
        }
        out->total = o.f_ukeys.size();
        out->keys = o.f_ukeys.data();
    }
    return TM_OK;
}

int tm_match_filter_batch_runs(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n, uint32_t mode,
                               tm_runs_result *out) {
    if (!eng || !out || (n && (!off || (!bytes && off[n] > off[0])))) return TM_EINVAL;
    if (mode != TM_MATCH_ALL && mode != TM_MATCH_FIRST) return TM_EINVAL;
    if (eng->replica) return replica_refuses(eng, "tm_match_filter_batch_runs");
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::mutex> gh(eng->mu_host);
    std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
    HostOut &o = eng->out();
    memset(out, 0, sizeof(*out));
    out->n = n;
    out->epoch = eng->epoch;
    if (n == 0) return TM_OK;
    auto &fx = eng->fx;
    FilterArgs a{};
    int rc = filter_prepare(eng, o, bytes, off, n, mode, a);
    if (rc) return rc;
    hipStream_t s = eng->stream;
    // long '+' queries walked as several parts, one wave each (plan_filter_parts)
    eng->plan_filter_parts(n, fx.items);
    const bool parts = !fx.items.empty();
    const uint32_t ni = parts ? (uint32_t)fx.items.size() : n;  // per-item outputs
    TM_TRY_HIP(fx.d_rcnt.ensure((size_t)ni * 4), TM_ENOMEM, "alloc");
    a.rcnt = fx.d_rcnt.as<uint32_t>();
    o.f_rcnt.resize(n);
    if (parts) {
        TM_TRY_HIP(fx.d_items.ensure((size_t)ni * sizeof(uint4)), TM_ENOMEM, "alloc");
        TM_TRY_HIP(fx.d_stop.ensure((size_t)ni * 4), TM_ENOMEM, "alloc");
        TM_TRY_HIP(fx.d_cnt.ensure((size_t)ni * 4), TM_ENOMEM, "alloc");
        TM_TRY_HIP(fx.d_off.ensure(((size_t)ni + 1) * 4), TM_ENOMEM, "alloc");
        TM_TRY_HIP(hipMemcpyAsync(fx.d_items.p, fx.items.data(), (size_t)ni * sizeof(uint4), hipMemcpyHostToDevice, s),
                   TM_EDEVICE, "H2D");
        a.items = fx.d_items.as<uint4>();
        a.n_items = ni;
        a.stop = fx.d_stop.as<uint32_t>();
        a.cnt = fx.d_cnt.as<uint32_t>();
        a.out_off = fx.d_off.as<uint32_t>();
        fx.i_off.resize(ni);
        fx.i_cnt.resize(ni);
        fx.i_rcnt.resize(ni);
        fx.i_stop.resize(ni);
    }
    // development: per-wave durations, the slowest reported on stderr (what sets a batch's time)
    static const bool wtime = getenv("EMQX_TM_FILTER_WTIME") != nullptr;
    if (wtime) {
        TM_TRY_HIP(fx.d_wtime.ensure((size_t)ni * 8), TM_ENOMEM, "alloc");
        a.wtime = fx.d_wtime.as<unsigned long long>();
    }
    uint32_t *h_off = parts ? fx.i_off.data() : o.f_off.data(), *h_cnt = parts ? fx.i_cnt.data() : o.f_cnt.data(),
             *h_rcnt = parts ? fx.i_rcnt.data() : o.f_rcnt.data();
    uint64_t ranges = 0;
    bool done = false;
    for (int attempt = 0; attempt < 3 && !done; attempt++) {
        // sized from the demand of earlier batches; a batch past them grows and runs again
        const uint64_t pool = std::max<uint64_t>(fx.pool_want, (uint64_t)n + 1024);
        const uint64_t cap = std::min<uint64_t>(std::max<uint64_t>(fx.rng_want, 1 << 16), 0xFFFFFFF0ull);
        TM_TRY_HIP(fx.d_pool.ensure(pool * FW_CHUNK * 4), TM_ENOMEM, "alloc filter pool");
        TM_TRY_HIP(fx.d_out.ensure(cap * 8), TM_ENOMEM, "alloc");
        TM_TRY_HIP(fx.d_ctl.ensure(24), TM_ENOMEM, "alloc");
        TM_TRY_HIP(hipMemsetAsync(fx.d_ctl.p, 0, 24, s), TM_EDEVICE, "memset");
        a.pool = fx.d_pool.as<uint32_t>();
        a.pool_chunks = fx.d_pool.cap / (FW_CHUNK * 4);
        a.out = fx.d_out.as<uint32_t>();
        a.out_cap = fx.d_out.cap / 8;
        a.ctl = fx.d_ctl.as<unsigned long long>();
        a.jobs = nullptr;
        a.jobs_cap = 0;
        uint64_t ctl[3] = {0, 0, 0};
        TM_TRY_HIP(launch_filter_walk(a, FW_RUNS, s), TM_EDEVICE, "k_filter_walk runs");
        TM_TRY_HIP(hipMemcpyAsync(ctl, fx.d_ctl.p, 24, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
        TM_TRY_HIP(hipMemcpyAsync(h_off, fx.d_off.p, (size_t)ni * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
        TM_TRY_HIP(hipMemcpyAsync(h_cnt, fx.d_cnt.p, (size_t)ni * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
        TM_TRY_HIP(hipMemcpyAsync(h_rcnt, fx.d_rcnt.p, (size_t)ni * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
        if (parts)
            TM_TRY_HIP(hipMemcpyAsync(fx.i_stop.data(), fx.d_stop.p, (size_t)ni * 4, hipMemcpyDeviceToHost, s),
                       TM_EDEVICE, "D2H");
        TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "k_filter_walk runs");
        ranges = ctl[0];
        if (ranges <= a.out_cap && ctl[1] <= a.pool_chunks) {
            TM_TRY_HIP(o.f_rng.ensure(std::max<uint64_t>(ranges, 1) * 8), TM_ENOMEM, "pinned alloc");
            if (ranges) {
                TM_TRY_HIP(d2h_words(o.f_rng, 0, fx.d_out.p, ranges * 2, s), TM_EDEVICE, "D2H");
                TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "k_filter_walk runs");
            }
            done = true;
        } else {
            fx.rng_want = std::max(fx.rng_want, ranges + ranges / 4 + 1024);
            fx.pool_want = std::max(fx.pool_want, ctl[1] + ctl[1] / 4 + 64);
        }
    }
    if (!done) {
        eng->err = "tm_match_filter_batch_runs: output still short after resizing";
        return TM_EDEVICE;
    }
    if (wtime) {
        std::vector<unsigned long long> wt(ni);
        TM_TRY_HIP(hipMemcpy(wt.data(), fx.d_wtime.p, (size_t)ni * 8, hipMemcpyDeviceToHost), TM_EDEVICE, "D2H");
        std::vector<uint32_t> ord(ni);
        for (uint32_t i = 0; i < ni; i++) ord[i] = i;
        std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return wt[x] > wt[y]; });
        unsigned long long sum = 0;
        for (auto v : wt) sum += v;
        fprintf(stderr, "[filter wtime] waves %u, sum %.1f us, max %.1f us, p50 %.1f us; slowest:", ni, sum / 100.0,
                wt[ord[0]] / 100.0, wt[ord[ni / 2]] / 100.0);
        for (uint32_t k = 0; k < std::min<uint32_t>(ni, 8); k++) {
            const uint32_t i = ord[k];
            const uint32_t q = parts ? fx.items[i].x : i;
            std::string qs;
            for (uint32_t j = fx.qoff[q]; j < fx.qoff[q + 1]; j++) qs += (fx.qw[j] == 1 ? "+" : fx.qw[j] == 0 ? "#" : "w") + std::string(j + 1 < fx.qoff[q + 1] ? "/" : "");
            fprintf(stderr, " [q %u %s part %u..%u keys %u %.1f us]", q, qs.c_str(), parts ? fx.items[i].y : 0u,
                    parts ? fx.items[i].z : NONE, h_cnt[i], wt[i] / 100.0);
        }
        fprintf(stderr, "\n");
    }
    // ranges of the sorted keys -> spans of their ids (this lane keeps the ids alive)
    o.f_ids = fx.ids;
    const uint64_t *ids = o.f_ids->data();
    const uint2 *rg = o.f_rng.as<uint2>();
    uint64_t tot = 0;
    if (!parts) {
        o.f_spans.resize(ranges);
        for (uint64_t r = 0; r < ranges; r++) o.f_spans[r] = tm_span{ids + rg[r].x, rg[r].y};
    } else {
        // a query's parts in order, up to the first one that stopped (its walk ends there)
        o.f_spans.clear();
        size_t i = 0;
        for (uint32_t q = 0; q < n; q++) {
            o.f_off[q] = (uint32_t)o.f_spans.size();
            uint32_t kc = 0;
            bool on = true;
            for (; i < ni && fx.items[i].x == q; i++) {
                if (!on) continue;
                for (uint32_t r = 0; r < fx.i_rcnt[i]; r++) {
                    const uint2 g = rg[(uint64_t)fx.i_off[i] + r];
                    o.f_spans.push_back(tm_span{ids + g.x, g.y});
                }
                kc += fx.i_cnt[i];
                on = !fx.i_stop[i];
            }
            o.f_cnt[q] = kc;
            o.f_rcnt[q] = (uint32_t)(o.f_spans.size() - o.f_off[q]);
        }
        ranges = o.f_spans.size();
    }
    for (uint32_t i = 0; i < n; i++) tot += o.f_cnt[i];
    o.fr_off.swap(o.f_off);  // the runs result's own arrays: a keys-form call does not touch them
    o.fr_cnt.swap(o.f_cnt);
    o.fr_status.swap(o.f_status);
    out->total_ids = tot;
    out->total_spans = ranges;
    out->span_off = o.fr_off.data();
    out->span_cnt = o.f_rcnt.data();
    out->spans = o.f_spans.data();
    out->kcnt = o.fr_cnt.data();
    out->status = o.fr_status.data();
    return TM_OK;
}

int tm_intersect_batch(tm_engine *eng, const uint8_t *a, const uint32_t *a_off, const uint8_t *b,
                       const uint32_t *b_off, uint32_t n, tm_intersect_result *out) {
    if (!eng || !out || (n && (!a_off || !b_off || (!a && a_off[n] > a_off[0]) || (!b && b_off[n] > b_off[0]))))
        return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    HostOut &o = eng->out();
    memset(out, 0, sizeof(*out));
    out->n = n;
    if (n == 0) return TM_OK;
    const uint64_t na = (uint64_t)a_off[n] - a_off[0], nb = (uint64_t)b_off[n] - b_off[0];
    const uint64_t cap = na + nb + n;
    if (cap >= 0xFFFFFFFFull) return TM_EINVAL;  // out offsets are u32 on the device
    hipStream_t s = eng->stream;
    TM_TRY_HIP(eng->d_ia.ensure(na + 1), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->d_ib.ensure(nb + 1), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->d_iaoff.ensure(((size_t)n + 1) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->d_iboff.ensure(((size_t)n + 1) * 4), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->d_iout.ensure(cap + 1), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->d_ilen.ensure((size_t)n * 4), TM_ENOMEM, "alloc");
    // offsets rebased to 0 (the kernel indexes the copies)
    std::vector<uint32_t> ao(a_off, a_off + n + 1), bo(b_off, b_off + n + 1);
    for (auto &v : ao) v -= a_off[0];
    for (auto &v : bo) v -= b_off[0];
    if (na) TM_TRY_HIP(hipMemcpyAsync(eng->d_ia.p, a + a_off[0], na, hipMemcpyHostToDevice, s), TM_EDEVICE, "H2D");
    if (nb) TM_TRY_HIP(hipMemcpyAsync(eng->d_ib.p, b + b_off[0], nb, hipMemcpyHostToDevice, s), TM_EDEVICE, "H2D");
    TM_TRY_HIP(hipMemcpyAsync(eng->d_iaoff.p, ao.data(), ao.size() * 4, hipMemcpyHostToDevice, s), TM_EDEVICE, "H2D");
    TM_TRY_HIP(hipMemcpyAsync(eng->d_iboff.p, bo.data(), bo.size() * 4, hipMemcpyHostToDevice, s), TM_EDEVICE, "H2D");
    TM_TRY_HIP(launch_intersect(eng->d_ia.as<uint8_t>(), eng->d_iaoff.as<uint32_t>(), eng->d_ib.as<uint8_t>(),
                                eng->d_iboff.as<uint32_t>(), n, eng->d_iout.as<uint8_t>(), eng->d_ilen.as<int32_t>(), s),
               TM_EDEVICE, "k_intersect");
    o.ix_len.resize(n);
    o.ix_bytes.resize(cap + 1);
    TM_TRY_HIP(hipMemcpyAsync(o.ix_len.data(), eng->d_ilen.p, (size_t)n * 4, hipMemcpyDeviceToHost, s), TM_EDEVICE,
               "D2H");
    TM_TRY_HIP(hipMemcpyAsync(o.ix_bytes.data(), eng->d_iout.p, cap, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
    TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "k_intersect");
    o.ix_off.resize(n);
    for (uint32_t i = 0; i < n; i++) o.ix_off[i] = (uint64_t)ao[i] + bo[i] + i;
    out->off = o.ix_off.data();
    out->len = o.ix_len.data();
    out->bytes = o.ix_bytes.data();
    return TM_OK;
}

int tm_stats(const tm_engine *eng, tm_stats_t *out) {
    if (!eng || !out) return TM_EINVAL;
    std::lock_guard<std::mutex> gh(const_cast<tm_engine *>(eng)->mu_host);
    std::lock_guard<std::recursive_mutex> gd(const_cast<tm_engine *>(eng)->mu_dev);
    memset(out, 0, sizeof(*out));
    out->epoch = eng->dv.epoch;
    out->n_keys = eng->replica ? eng->dv.n_live : eng->n_live;
    out->n_nodes = eng->replica ? eng->dv.n_nodes : eng->node_parent.size();
    out->n_words = eng->replica ? eng->dv.n_words : eng->word_off.size();
    out->edge_slots = eng->emask + 1;
    out->word_slots = eng->replica ? eng->wmask + 1 : eng->wtab.size();
    out->list_words = eng->replica ? eng->dev_used[A_ARENA] / 4 : eng->arena.size();
    out->device_bytes = eng->d_wtab.cap + eng->d_warena.cap + eng->d_word_off.cap + eng->d_etab.cap +
                        eng->d_slot_list.cap + eng->d_arena.cap + eng->d_root.cap;
    out->n_full_rebuilds = eng->n_full_rebuilds;
    out->n_delta_commits = eng->n_delta_commits;
    out->n_slow_topics = eng->n_slow_last;
    out->commit_apply_us = eng->commit_us[0];
    out->commit_lists_us = eng->commit_us[1];
    out->commit_upload_us = eng->commit_us[2];
    out->n_deep_keys = eng->n_deep;
    out->n_filter_onepass = eng->fx.n_onepass;
    out->n_filter_twopass = eng->fx.n_twopass;
    out->commit_stall_us = eng->commit_stall_us;
    out->n_commits_refused = eng->n_commits_refused;
    out->n_staged = const_cast<tm_engine *>(eng)->staged_count();
    out->standby_bytes = eng->standby_bytes();
    return TM_OK;
}

// ---- diagnostics (not part of the reference surface): walk counters -------
// Enable per-batch walk statistics (node visits, edge probes, word probes, keys,
// levels, spilled topics, segments, chunk flushes), accumulated on the device
// across batches until read.
int tm_debug_stats(tm_engine *eng, int enable, uint64_t *out18) {
    if (!eng) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    TM_TRY_HIP(eng->d_stats.ensure(STATS_BYTES), TM_ENOMEM, "alloc");
    if (out18) {
        TM_TRY_HIP(hipDeviceSynchronize(), TM_EDEVICE, "sync");
        TM_TRY_HIP(hipMemcpy(out18, eng->d_stats.p, 18 * 8, hipMemcpyDeviceToHost), TM_EDEVICE, "D2H");
    }
    TM_TRY_HIP(hipMemset(eng->d_stats.p, 0, STATS_BYTES), TM_EDEVICE, "memset");
    TM_TRY_HIP(hipStreamSynchronize(nullptr), TM_EDEVICE, "memset sync");  // before any stream's launch counts
    eng->stats_on = enable != 0;
    return TM_OK;
}

int tm_debug_depth_stats(tm_engine *eng, uint64_t *out64) {
    if (!eng || !out64) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    TM_TRY_HIP(eng->d_stats.ensure(STATS_BYTES), TM_ENOMEM, "alloc");
    TM_TRY_HIP(hipDeviceSynchronize(), TM_EDEVICE, "sync");
    TM_TRY_HIP(hipMemcpy(out64, (const uint8_t *)eng->d_stats.p + 32 * 8, 64 * 8, hipMemcpyDeviceToHost), TM_EDEVICE,
               "D2H");
    return TM_OK;
}

// The device index as delta commits left it, array by array, against a full publish of the
// same host state (the edge table then built on the device from one record per node, every
// other array uploaded whole): bit a of *diff_mask set for each array whose bytes differ.
// Words, edges, slot lists, the list arena and the root are compared; the key arrays are not
// (a freed handle's device record stays as it was after a delta, by design: nothing refers to
// it).  The full publish stays in place.  Test aid: commits wait meanwhile.
int tm_debug_bounds(tm_engine *eng, uint64_t *hits, char *msg, uint32_t cap) {
    if (!hits) return TM_EINVAL;
#if TM_BOUNDS
    {  // the engine's device (null: device 0): wait for it, then its record and every canary
        const int dev = eng ? eng->cfg.device : 0;
        if (hipSetDevice(dev) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
            tm_engine::bnd_scan(dev, "tm_debug_bounds", eng) != hipSuccess)
            return TM_EDEVICE;
    }
    std::lock_guard<std::mutex> g(bnd_registry().m);
    *hits = bnd_registry().hits;
    if (msg && cap) snprintf(msg, cap, "%s", bnd_registry().msg.c_str());
    return TM_OK;
#else
    (void)eng;
    (void)msg;
    (void)cap;
    return TM_ENOTFOUND;
#endif
}

int tm_debug_image_check(tm_engine *eng, uint32_t *diff_mask) {
    if (!eng || !diff_mask || eng->replica) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::mutex> gc(eng->mu_commit);
    static const uint32_t arrs[] = {A_WTAB, A_WARENA, A_WORD_OFF, A_ETAB, A_SLOT_LIST, A_ARENA, A_ROOT};
    std::vector<uint8_t> before[A_N];
    auto grab = [&](uint32_t a, std::vector<uint8_t> &v) -> hipError_t {
        v.resize(eng->dev_used[a]);
        return v.empty() ? hipSuccess : hipMemcpy(v.data(), eng->arr_buf(a)->p, v.size(), hipMemcpyDeviceToHost);
    };
    {
        std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
        TM_TRY_HIP(eng->quiesce(), TM_EDEVICE, "sync");
        for (uint32_t a : arrs) TM_TRY_HIP(grab(a, before[a]), TM_EDEVICE, "D2H");
    }
    {
        std::lock_guard<std::mutex> gh(eng->mu_host);
        TM_TRY_HIP(eng->publish_full(), TM_EDEVICE, "full publish");
    }
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    uint32_t mask = 0;
    for (uint32_t a : arrs) {
        std::vector<uint8_t> after;
        TM_TRY_HIP(grab(a, after), TM_EDEVICE, "D2H");
        if (after != before[a]) mask |= 1u << a;
    }
    *diff_mask = mask;
    return TM_OK;
}

// Time the dominant kernel (k_match_fast) of the NEXT match call with HIP events
// recorded on the stream it is launched on.  tm_debug_timing(eng, 1, NULL) arms;
// after the match and a sync, tm_debug_timing(eng, 0, &ms) returns its duration.
int tm_debug_timing(tm_engine *eng, int enable, float *ms_out) {
    if (!eng) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    if (!eng->ev_fast0) {
        TM_TRY_HIP(hipEventCreate(&eng->ev_fast0), TM_EDEVICE, "event");
        TM_TRY_HIP(hipEventCreate(&eng->ev_fast1), TM_EDEVICE, "event");
    }
    if (ms_out) {
        TM_TRY_HIP(hipEventSynchronize(eng->ev_fast1), TM_EDEVICE, "event sync");
        TM_TRY_HIP(hipEventElapsedTime(ms_out, eng->ev_fast0, eng->ev_fast1), TM_EDEVICE, "elapsed");
    }
    eng->timing_on = enable != 0;
    return TM_OK;
}

int tm_debug_commit_marks(const tm_engine *eng, uint64_t *out9) {
    if (!eng || !out9) return TM_EINVAL;
    std::lock_guard<std::mutex> g(const_cast<tm_engine *>(eng)->mu_commit);
    for (int k = 0; k < 8; k++) out9[k] = eng->pub_marks[k];
    out9[8] = eng->pub_reallocs;
    return TM_OK;
}

// ---- replicated mode: device image + epoch patches (DESIGN.md §6 mode 1) ----------
// Every array's used bytes come from dev_used (kept by each upload and scatter), and the
// counts from the published view: the image is the epoch the device serves (mu_dev).
static void image_layout(const tm_engine *eng, ImageHdr *h) {
    memset(h, 0, sizeof *h);
    h->magic = IMAGE_MAGIC;
    h->epoch = eng->dv.epoch;
    h->wmask = eng->dv.wmask;
    h->emask = eng->dv.emask;
    h->n_deep = eng->dv.n_deep;
    h->n_live = eng->dv.n_live;
    h->n_nodes = eng->dv.n_nodes;
    h->n_words = eng->dv.n_words;
    h->nonce = eng->master_nonce;
    h->max_id = eng->dv.max_id;
    uint64_t at = (sizeof(ImageHdr) + IMAGE_ALIGN - 1) / IMAGE_ALIGN * IMAGE_ALIGN;
    for (uint32_t a = 0; a < A_N; a++) {
        const DevBuf *b = const_cast<tm_engine *>(eng)->arr_buf(a);
        h->cap[a] = b->cap;
        h->used[a] = std::min<uint64_t>(eng->dev_used[a], b->cap);
        h->off[a] = at;
        at += (h->used[a] + IMAGE_ALIGN - 1) / IMAGE_ALIGN * IMAGE_ALIGN;
    }
}

static uint64_t image_bytes(const ImageHdr &h) {
    uint64_t end = (sizeof(ImageHdr) + IMAGE_ALIGN - 1) / IMAGE_ALIGN * IMAGE_ALIGN;
    for (uint32_t a = 0; a < A_N; a++) end = std::max(end, h.off[a] + (h.used[a] + IMAGE_ALIGN - 1) / IMAGE_ALIGN * IMAGE_ALIGN);
    return end;
}

int tm_image_size(const tm_engine *eng, uint64_t *bytes) {
    if (!eng || !bytes) return TM_EINVAL;
    std::lock_guard<std::recursive_mutex> g(const_cast<tm_engine *>(eng)->mu_dev);
    ImageHdr h;
    image_layout(eng, &h);
    *bytes = image_bytes(h);
    return TM_OK;
}

int tm_image_export(tm_engine *eng, void *d_dst, uint64_t cap, void *stream) {
    if (!eng || !d_dst) return TM_EINVAL;
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    ImageHdr h;
    image_layout(eng, &h);
    if (image_bytes(h) > cap) return TM_ENOMEM;
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    if (s != eng->stream) TM_TRY_HIP(eng->wait_uses(s), TM_EDEVICE, "stream order");
    uint8_t *dst = (uint8_t *)d_dst;
    for (uint32_t a = 0; a < A_N; a++)
        if (h.used[a])
            TM_TRY_HIP(hipMemcpyAsync(dst + h.off[a], eng->arr_buf(a)->p, h.used[a], hipMemcpyDeviceToDevice, s),
                       TM_EDEVICE, "image D2D");
    TM_TRY_HIP(hipMemcpyAsync(dst, &h, sizeof h, hipMemcpyHostToDevice, s), TM_EDEVICE, "image header");
    TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "image sync");  // h is on this stack frame
    return TM_OK;
}

int tm_replica_load(tm_engine *eng, const void *d_image, uint64_t bytes, void *stream) {
    if (!eng || !d_image || bytes < sizeof(ImageHdr)) return TM_EINVAL;
    if (!eng->replica) {
        eng->err = "tm_replica_load: not a replica";
        return TM_ESTATE;
    }
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    // runs results read the host id arena: no lease may be held while it is rewritten (leases
    // come before any engine lock)
    eng->leases_block();
    struct Unblock {
        tm_engine *e;
        ~Unblock() { e->leases_unblock(); }
    } unblock{eng};
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    ImageHdr h;
    TM_TRY_HIP(hipMemcpyAsync(&h, d_image, sizeof h, hipMemcpyDeviceToHost, s), TM_EDEVICE, "image header");
    TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "image sync");
    if (h.magic != IMAGE_MAGIC || image_bytes(h) > bytes) {
        eng->err = "tm_replica_load: not an engine image (or truncated)";
        return TM_EINVAL;
    }
    for (uint32_t a = 0; a < A_N; a++)
        if (h.used[a] > h.cap[a]) return TM_EINVAL;
    // the new image goes into fresh buffers first: a failed load keeps the old one serving
    DevBuf nb[A_N];
    const uint8_t *src = (const uint8_t *)d_image;
    for (uint32_t a = 0; a < A_N; a++) {
        hipError_t e = nb[a].ensure(std::max<uint64_t>(h.cap[a], 64));
        if (!e && h.used[a]) e = hipMemcpyAsync(nb[a].p, src + h.off[a], h.used[a], hipMemcpyDeviceToDevice, s);
        if (e) {
            (void)hipStreamSynchronize(s);
            for (DevBuf &b : nb) b.release();
            eng->err = std::string("tm_replica_load: ") + hipGetErrorString(e);
            return e == hipErrorOutOfMemory ? TM_ENOMEM : TM_EDEVICE;
        }
    }
    TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "image sync");
    TM_TRY_HIP(eng->quiesce(), TM_EDEVICE, "drain");  // matches in flight finish on the old image
    for (uint32_t a = 0; a < A_N; a++) {
        DevBuf *b = eng->arr_buf(a);
        std::swap(b->p, nb[a].p);
        std::swap(b->cap, nb[a].cap);
        nb[a].release();
        eng->dev_used[a] = h.used[a];
    }
    eng->epoch = h.epoch;
    eng->wmask = h.wmask;
    eng->emask = h.emask;
    eng->n_deep = h.n_deep;
    eng->master_nonce = h.nonce;
    eng->dv.epoch = h.epoch;
    eng->dv.wmask = h.wmask;
    eng->dv.emask = h.emask;
    eng->dv.n_deep = h.n_deep;
    eng->dv.max_id = h.max_id;
    eng->dv.n_live = h.n_live;
    eng->dv.n_nodes = h.n_nodes;
    eng->dv.n_words = h.n_words;
    return eng->replica_ids_full();
}

int tm_replica_create(const tm_config *cfg, const void *d_image, uint64_t bytes, void *stream, tm_engine **out) {
    if (!out || !d_image) return TM_EINVAL;
    *out = nullptr;
    tm_config c = cfg ? *cfg : tm_config{};
    c.flags &= ~TM_CFG_RECORD_PATCH;
    c.reserve_keys = 1;
    c.reserve_nodes = 1;
    tm_engine *eng = nullptr;
    int rc = tm_create(&c, &eng);
    if (rc != TM_OK) return rc;
    eng->replica = true;
    // the replica keeps no host master copy
    std::vector<WordSlot>().swap(eng->wtab);
    hvec<uint64_t>().swap(eng->eocc);
    decltype(eng->emap)().swap(eng->emap);
    hvec<uint32_t>().swap(eng->kset);
    // the host id arena stays: the replica fills it from its device copy (runs form)
    if ((rc = tm_replica_load(eng, d_image, bytes, stream)) != TM_OK) {
        tl_create_err() = std::string("tm_replica_create: loading the image failed: ") + tl_err();
        tm_destroy(eng);
        return rc;
    }
    *out = eng;
    return TM_OK;
}

int tm_patch_size(const tm_engine *eng, uint64_t *bytes, int *full) {
    if (!eng || !bytes) return TM_EINVAL;
    if (!(eng->cfg.flags & TM_CFG_RECORD_PATCH)) return TM_ESTATE;
    std::lock_guard<std::mutex> g(const_cast<tm_engine *>(eng)->mu_host);
    *bytes = sizeof(PatchHdr) + (eng->patch.full ? 0 : eng->patch.buf.size());
    if (full) *full = eng->patch.full ? 1 : 0;
    return TM_OK;
}

int tm_patch_export(const tm_engine *eng, void *dst, uint64_t cap) {
    if (!eng || !dst) return TM_EINVAL;
    if (!(eng->cfg.flags & TM_CFG_RECORD_PATCH)) return TM_ESTATE;
    std::lock_guard<std::mutex> g(const_cast<tm_engine *>(eng)->mu_host);
    const uint64_t body = eng->patch.full ? 0 : eng->patch.buf.size();
    if (cap < sizeof(PatchHdr) + body) return TM_ENOMEM;
    PatchHdr h{PATCH_MAGIC, eng->patch_from, eng->epoch, eng->wmask, eng->emask, eng->n_deep, eng->n_live,
               eng->patch.full ? 0 : eng->patch.n, eng->patch.full ? 1ull : 0ull, eng->master_nonce, eng->max_id};
    memcpy(dst, &h, sizeof h);
    if (body) memcpy((uint8_t *)dst + sizeof h, eng->patch.buf.data(), body);
    return TM_OK;
}

int tm_replica_apply_patch(tm_engine *eng, const void *patch, uint64_t bytes) {
    if (!eng || !patch || bytes < sizeof(PatchHdr)) return TM_EINVAL;
    if (!eng->replica) {
        eng->err = "tm_replica_apply_patch: not a replica";
        return TM_ESTATE;
    }
    eng->leases_block();  // as tm_replica_load
    struct Unblock {
        tm_engine *e;
        ~Unblock() { e->leases_unblock(); }
    } unblock{eng};
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    PatchHdr h;
    memcpy(&h, patch, sizeof h);
    if (h.magic != PATCH_MAGIC) return TM_EINVAL;
    if (h.nonce != eng->master_nonce) {
        eng->err = "tm_replica_apply_patch: the patch comes from another master than the replica's image";
        return TM_ESTATE;
    }
    if (h.full) {
        eng->err = "tm_replica_apply_patch: the master re-uploaded its whole index; reload from tm_image_export";
        return TM_ESTATE;
    }
    if (h.epoch_from != eng->epoch) {
        eng->err = "tm_replica_apply_patch: patch is for epoch " + std::to_string(h.epoch_from) + ", replica holds " +
                   std::to_string(eng->epoch);
        return TM_ESTATE;
    }
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    hipStream_t s = eng->stream;
    // validate every record before touching the device: a replica never half-applies, and no
    // record may write past the buffer it targets (capacities as they will be at that record)
    uint64_t cap_at[A_N];
    for (uint32_t a = 0; a < A_N; a++) cap_at[a] = eng->arr_buf(a)->cap;
    const uint8_t *p = (const uint8_t *)patch + sizeof h, *end = (const uint8_t *)patch + bytes;
    for (uint64_t i = 0; i < h.n_records; i++) {
        if (p + sizeof(PatchRec) > end) return TM_EINVAL;
        PatchRec r;
        memcpy(&r, p, sizeof r);
        const uint64_t el = r.arr < A_N ? ARR_ELEM[r.arr] : 0;
        if (!el || r.bytes > (uint64_t)(end - p) - sizeof r) return TM_EINVAL;
        if (r.kind != P_TAIL && r.kind != P_SCATTER && r.kind != P_WHOLE) return TM_EINVAL;
        if (r.count > (1ull << 40)) return TM_EINVAL;
        const uint64_t need = r.kind == P_SCATTER ? r.count * (8 + el) : r.count * el;
        if (need > r.bytes) return TM_EINVAL;
        if (r.kind == P_TAIL && (r.a + r.count) * el > cap_at[r.arr]) return TM_EINVAL;
        if (r.kind == P_WHOLE) {
            if (r.count * el > r.a) return TM_EINVAL;
            cap_at[r.arr] = std::max(cap_at[r.arr], r.a);
        }
        if (r.kind == P_SCATTER) {
            const uint8_t *ix = p + sizeof r;
            for (uint64_t k = 0; k < r.count; k++) {
                uint64_t idx;
                memcpy(&idx, ix + k * 8, 8);
                if ((idx + 1) * el > cap_at[r.arr]) return TM_EINVAL;
            }
        }
        p += sizeof r + r.bytes;
    }
    TM_TRY_HIP(eng->quiesce(), TM_EDEVICE, "drain");  // replica matches in flight read these arrays
    p = (const uint8_t *)patch + sizeof h;
    for (uint64_t i = 0; i < h.n_records; i++) {
        PatchRec r;
        memcpy(&r, p, sizeof r);
        const uint8_t *pay = p + sizeof r;
        const uint64_t el = ARR_ELEM[r.arr];
        DevBuf *b = eng->arr_buf(r.arr);
        if (r.kind == P_TAIL) {
            if (r.count)
                TM_TRY_HIP(hipMemcpyAsync(b->as<uint8_t>() + r.a * el, pay, r.count * el, hipMemcpyHostToDevice, s),
                           TM_EDEVICE, "patch H2D");
            eng->dev_used[r.arr] = std::max<uint64_t>(eng->dev_used[r.arr], (r.a + r.count) * el);
        } else if (r.kind == P_WHOLE) {
            if (b->cap < r.a) {
                TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "patch sync");
                b->release();
                TM_TRY_HIP(b->ensure(r.a), TM_ENOMEM, "replica alloc");
            }
            if (r.count)
                TM_TRY_HIP(hipMemcpyAsync(b->p, pay, r.count * el, hipMemcpyHostToDevice, s), TM_EDEVICE, "patch H2D");
            eng->dev_used[r.arr] = r.count * el;
        } else if (r.count) {
            uint64_t top = 0;
            for (uint64_t k = 0; k < r.count; k++) {
                uint64_t idx;
                memcpy(&idx, pay + k * 8, 8);
                top = std::max(top, idx + 1);
            }
            TM_TRY_HIP(eng->d_scatter_idx.ensure(r.count * 8), TM_ENOMEM, "alloc");
            TM_TRY_HIP(eng->d_scatter_src.ensure(r.count * el), TM_ENOMEM, "alloc");
            TM_TRY_HIP(hipMemcpyAsync(eng->d_scatter_idx.p, pay, r.count * 8, hipMemcpyHostToDevice, s), TM_EDEVICE,
                       "patch H2D");
            TM_TRY_HIP(hipMemcpyAsync(eng->d_scatter_src.p, pay + r.count * 8, r.count * el, hipMemcpyHostToDevice, s),
                       TM_EDEVICE, "patch H2D");
            const uint64_t *ix = eng->d_scatter_idx.as<uint64_t>();
            const uint64_t cap = b->cap / el;
            hipError_t e = el == 16  ? launch_scatter16(b->as<uint4>(), ix, eng->d_scatter_src.as<uint4>(), r.count, s, cap, eng->bnd_rec())
                           : el == 4 ? launch_scatter4(b->as<uint32_t>(), ix, eng->d_scatter_src.as<uint32_t>(), r.count, s, cap, eng->bnd_rec())
                                     : launch_scatter1(b->as<uint8_t>(), ix, eng->d_scatter_src.as<uint8_t>(), r.count, s, cap, eng->bnd_rec());
            TM_TRY_HIP(e, TM_EDEVICE, "patch scatter");
            TM_TRY_HIP(eng->bnd_after(s, "patch scatter"), TM_EDEVICE, "patch scatter");
            // a scatter past the used part (new key handles inside the capacity) extends it, so
            // an image exported from this replica carries them
            eng->dev_used[r.arr] = std::max<uint64_t>(eng->dev_used[r.arr], top * el);
            TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "patch sync");  // scratch is reused by the next record
        }
        p += sizeof r + r.bytes;
    }
    TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "patch sync");
    eng->epoch = h.epoch_to;
    eng->wmask = h.wmask;
    eng->emask = h.emask;
    eng->n_deep = h.n_deep;
    eng->dv.epoch = h.epoch_to;
    eng->dv.wmask = h.wmask;
    eng->dv.emask = h.emask;
    eng->dv.n_deep = h.n_deep;
    eng->dv.max_id = h.max_id;
    eng->dv.n_live = h.n_live;
    return eng->replica_ids_patch((const uint8_t *)patch + sizeof h, h.n_records);
}

// Is p host memory the device can DMA from directly (pinned / registered)?
static bool host_pinned(const void *p) {
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// memcpy of a large range on several threads (staging a batch into pinned memory)
static void par_memcpy(void *dst, const void *src, size_t n) {
    const size_t per = 8u << 20;
    const unsigned nt = (unsigned)std::min<size_t>(8, (n + per - 1) / per);
    if (nt <= 1) {
        if (n) memcpy(dst, src, n);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned k = 0; k < nt; k++)
        th.emplace_back([=] {
            const size_t a = n * k / nt, b = n * (k + 1) / nt;
            memcpy((uint8_t *)dst + a, (const uint8_t *)src + a, b - a);
        });
    for (auto &t : th) t.join();
}

// tm_match_batch_runs: sub-batches of about RUNS_SUB topics walk in MODE_RUNS on the engine
// stream, one after the other, reserving spans from one cursor (so each sub-batch's spans are
// one contiguous range); while sub-batch j+1 is staged and walked, sub-batch j's spans and
// per-topic arrays cross PCIe on the copy stream.
constexpr uint32_t RUNS_SUB = 262144;
constexpr uint32_t RUNS_MAXSUB = 16;
// development knobs (tools/prof_runs.py sweeps): sub-batch size and topics per wave
static uint32_t env_u32(const char *name, uint32_t dflt) {
    const char *v = getenv(name);
    return v && *v ? (uint32_t)strtoul(v, nullptr, 10) : dflt;
}

static int match_runs_impl(tm_engine *eng, HostOut &o, const uint8_t *bytes, const uint32_t *off, uint32_t n,
                           tm_runs_result *out);

int tm_match_batch_runs(tm_engine *eng, const uint8_t *bytes, const uint32_t *off, uint32_t n, tm_runs_result *out) {
    if (!eng || !out || (n && (!off || (!bytes && off[n] > off[0])))) return TM_EINVAL;
    if (eng->replica && !eng->r_ids)
        return replica_refuses(eng, "tm_match_batch_runs (the replica's host id arena is off)");
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    HostOut &o = eng->out();
    eng->lease_drop(o);  // the previous result of this thread ends here
    eng->lease_take(o);  // waits while a commit changes the host copy
    const int rc = match_runs_impl(eng, o, bytes, off, n, out);
    // a failed call hands back no spans, so its caller has no reason to release them: the
    // lease ends here (else every commit would wait for this thread's next runs call)
    if (rc != TM_OK) eng->lease_drop(o);
    return rc;
}

static int match_runs_impl(tm_engine *eng, HostOut &o, const uint8_t *bytes, const uint32_t *off, uint32_t n,
                           tm_runs_result *out) {
    if (eng->cfg.flags & TM_CFG_FAIL_HOST_CALLS) {
        eng->err = "tm_match_batch_runs: failure injected (TM_CFG_FAIL_HOST_CALLS)";
        return TM_EDEVICE;
    }
    // this thread's own buffers and streams (HostOut::bb); the device lock is held only while
    // the buffers are sized and while each sub-batch's walk is queued
    TM_TRY_HIP(o.lanes(), TM_EDEVICE, "stream");
    BatchBufs &B = o.bb;
    memset(out, 0, sizeof(*out));
    out->n = n;
    {
        std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
        out->epoch = eng->dv.epoch;
    }
    if (n == 0) return TM_OK;
    const uint32_t base = off[0];
    const uint64_t nbytes = (uint64_t)off[n] - base;
    const uint32_t runs_sub = std::max<uint32_t>(4096, env_u32("EMQX_TM_RUNS_SUB", RUNS_SUB));
    // 64 topics per wave from 131,072-topic sub-batches on (262,144: 1.845 vs 1.904 ms per 1 M at config C)
    const uint32_t runs_tpw_knob = env_u32("EMQX_TM_RUNS_TPW", 0);
    auto runs_tpw_of = [&](uint32_t sub) -> uint32_t { return runs_tpw_knob ? runs_tpw_knob : (sub >= 131072 ? 64u : 0u); };
    const uint32_t S = std::max<uint32_t>(1, std::min<uint32_t>(RUNS_MAXSUB, n / runs_sub));
    uint32_t b[RUNS_MAXSUB + 1];
    for (uint32_t j = 0; j <= S; j++) b[j] = (uint32_t)((uint64_t)n * j / S);
    {
        std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
        eng->bb = &B;
        int rc = ensure_batch(eng, n, nbytes);
        if (rc) return rc;
        // every sub-batch's grid must fit the per-wave chunk lists (sized for the whole batch above)
        uint64_t g = 0;
        for (uint32_t j = 0; j < S; j++) {
            const uint32_t sub = b[j + 1] - b[j], t = runs_tpw_of(sub);
            g = std::max<uint64_t>(g, match_grid(sub, pick_tpw(sub, t ? t : eng->cfg.topics_per_wave)));
        }
        TM_TRY_HIP(eng->grow_buf(B.d_wave_chunks, g * SEG_MAXCHUNK * 4 + 4), TM_ENOMEM, "alloc");
        TM_TRY_HIP(eng->grow_buf(B.d_bytes, nbytes + 16), TM_ENOMEM, "alloc");
        TM_TRY_HIP(eng->grow_buf(B.d_off, ((size_t)n + 1) * 4), TM_ENOMEM, "alloc");
        TM_TRY_HIP(eng->grow_buf(B.d_kcnt, (size_t)n * 4 + 4), TM_ENOMEM, "alloc");
        TM_TRY_HIP(eng->grow_buf(B.d_rcur, 64), TM_ENOMEM, "alloc");
    }
    TM_TRY_HIP(o.h_off.ensure(((size_t)n + 1) * 4), TM_ENOMEM, "pinned alloc");
    TM_TRY_HIP(o.h_rctl.ensure((size_t)RUNS_MAXSUB * 64), TM_ENOMEM, "pinned alloc");
    for (PinBuf *pb : {&o.r_off, &o.r_cnt, &o.r_kcnt, &o.r_status})
        TM_TRY_HIP(pb->ensure((size_t)n * 4 + 4), TM_ENOMEM, "pinned alloc");
    const bool direct = host_pinned(bytes + base);  // DMA straight from the caller's batch
    if (!direct) TM_TRY_HIP(o.h_bytes.ensure(nbytes + 16), TM_ENOMEM, "pinned alloc");
    if (!direct) std::call_once(eng->copier_once, [eng] { eng->copier.start(3); });
    // one sub-batch: everything in order on the thread's walk stream (no cross-stream waits, and
    // one hardware queue per calling thread); several: H2D, walks and D2H on three streams
    hipStream_t s = o.s_walk, c = S > 1 ? o.s_copy : o.s_walk, hq = S > 1 ? o.s_h2d : o.s_walk;
    B.last_n = 0;
    B.dev_batch = false;  // the device result is in span form, not keys
    uint32_t *ho = o.h_off.as<uint32_t>();
    uint8_t *hb = direct ? nullptr : o.h_bytes.as<uint8_t>();
    uint64_t *rctl = o.h_rctl.as<uint64_t>();  // per sub-batch: [0] span cursor, [1..4] counter block
    int rc;

    for (int attempt = 0; attempt < 2; attempt++) {
        const uint64_t cap = std::max<uint64_t>(65536, (uint64_t)(o.runs_spt * 1.3 * n) + 4096);
        if (B.d_keys.cap < cap * 16) {
            std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
            TM_TRY_HIP(eng->grow_buf(B.d_keys, cap * 16), TM_ENOMEM, "alloc spans");
            B.keys_cap = B.d_keys.cap / 4;
        }
        const uint64_t span_cap = B.d_keys.cap / 16;
        TM_TRY_HIP(o.r_runs.ensure(span_cap * 16), TM_ENOMEM, "pinned alloc");
        TM_TRY_HIP(hipMemsetAsync(B.d_rcur.p, 0, 8, s), TM_EDEVICE, "memset");
        unsigned long long *cur = B.d_rcur.as<unsigned long long>();
        auto stage = [&](uint32_t j) -> int {
            const uint32_t lo = b[j], hi = b[j + 1];
            const uint64_t blo = off[lo] - base, bhi = off[hi] - base;
            for (uint32_t i = lo; i <= hi; i++) ho[i] = off[i] - base;
            const uint8_t *src = bytes + base + blo;
            if (!direct) {
                eng->copier.copy(hb + blo, src, bhi - blo);
                src = hb + blo;
            }
            // on their own stream: sub-batch j+1's topics cross PCIe while sub-batch j walks
            if (bhi > blo)
                TM_TRY_HIP(hipMemcpyAsync(B.d_bytes.as<uint8_t>() + blo, src, bhi - blo, hipMemcpyHostToDevice, hq),
                           TM_EDEVICE, "H2D");
            TM_TRY_HIP(hipMemcpyAsync(B.d_off.as<uint32_t>() + lo, ho + lo, ((size_t)hi - lo + 1) * 4,
                                      hipMemcpyHostToDevice, hq),
                       TM_EDEVICE, "H2D");
            TM_TRY_HIP(hipEventRecord(o.ev_h2d[j], hq), TM_EDEVICE, "event");
            return TM_OK;
        };
        auto walk = [&](uint32_t j) -> int {
            const uint32_t lo = b[j], hi = b[j + 1], h = j & 1;
            TM_TRY_HIP(hipStreamWaitEvent(s, o.ev_h2d[j], 0), TM_EDEVICE, "wait");
            const uint8_t *pctl;
            {
                std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
                eng->bb = &B;
                TM_TRY_HIP(enqueue_match(eng, B.d_bytes.as<uint8_t>(), B.d_off.as<uint32_t>() + lo, hi - lo, s, MODE_RUNS,
                                         lo, B.d_keys.as<uint32_t>(), span_cap, cur, nullptr, runs_tpw_of(hi - lo)),
                           TM_EDEVICE, "kernel launch");
                TM_TRY_HIP(eng->note_use(s), TM_EDEVICE, "event");
                pctl = B.p_ctl;
            }
            TM_TRY_HIP(hipMemcpyAsync(rctl + 8 * j, cur, 8, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
            TM_TRY_HIP(hipMemcpyAsync(rctl + 8 * j + 1, pctl, CTL_BYTES, hipMemcpyDeviceToHost, s), TM_EDEVICE, "D2H");
            TM_TRY_HIP(hipEventRecord(o.ev_pk[h], s), TM_EDEVICE, "event");
            return TM_OK;
        };
        uint64_t prev = 0, slow = 0, seg_d = 0, fr_d = 0;
        bool over = false;
        auto finish = [&](uint32_t j) -> int {  // sub-batch j walked: its results cross PCIe
            const uint32_t lo = b[j], hi = b[j + 1], h = j & 1;
            TM_TRY_HIP(hipEventSynchronize(o.ev_pk[h]), TM_EDEVICE, "match kernels");
            const uint64_t c_j = rctl[8 * j];
            slow += (uint32_t)rctl[8 * j + 2];
            seg_d = std::max(seg_d, rctl[8 * j + 3]);
            fr_d = std::max(fr_d, rctl[8 * j + 4]);
            if (c_j > span_cap) {
                over = true;
                prev = c_j;
                return TM_OK;
            }
            TM_TRY_HIP(hipStreamWaitEvent(c, o.ev_pk[h], 0), TM_EDEVICE, "wait");
            if (c_j > prev)  // DMA: a copy kernel here competes with the next sub-batch's walk
                TM_TRY_HIP(hipMemcpyAsync(o.r_runs.as<uint8_t>() + prev * 16, B.d_keys.as<uint8_t>() + prev * 16,
                                          (c_j - prev) * 16, hipMemcpyDeviceToHost, c),
                           TM_EDEVICE, "D2H");
            for (std::pair<PinBuf *, DevBuf *> pr :
                 {std::make_pair(&o.r_off, &B.d_outoff), std::make_pair(&o.r_cnt, &B.d_outcnt),
                  std::make_pair(&o.r_kcnt, &B.d_kcnt), std::make_pair(&o.r_status, &B.d_status)})
                TM_TRY_HIP(hipMemcpyAsync(pr.first->as<uint32_t>() + lo, pr.second->as<uint32_t>() + lo,
                                          ((size_t)hi - lo) * 4, hipMemcpyDeviceToHost, c),
                           TM_EDEVICE, "D2H");
            prev = c_j;
            return TM_OK;
        };
        if ((rc = stage(0)) || (rc = walk(0))) return rc;
        for (uint32_t j = 0; j < S; j++) {
            if (j + 1 < S && ((rc = stage(j + 1)) || (rc = walk(j + 1)))) return rc;
            if ((rc = finish(j))) return rc;
            if (over) break;
        }
        TM_TRY_HIP(hipStreamSynchronize(hq), TM_EDEVICE, "sync");
        TM_TRY_HIP(hipStreamSynchronize(s), TM_EDEVICE, "sync");
        TM_TRY_HIP(hipStreamSynchronize(c), TM_EDEVICE, "D2H");
        {
            std::lock_guard<std::recursive_mutex> gd(eng->mu_dev);
            eng->bb = &B;
            eng->n_slow_last = slow;
            B.seg_demand_last = seg_d;
            B.fr_demand_last = fr_d;
            if ((rc = grow_pools(eng))) return rc;
        }
        if (over) {  // more spans than estimated: size from the demand seen so far, run again
            uint32_t done = 0;
            for (uint32_t j = 0; j < S; j++)
                if (rctl[8 * j] >= prev) {
                    done = b[j + 1];
                    break;
                }
            o.runs_spt = std::max(o.runs_spt * 2, (double)prev / std::max<uint32_t>(done, 1));
            continue;
        }
        o.runs_spt = (double)prev / n;
        uint64_t tot = 0;
        const uint32_t *kc = o.r_kcnt.as<uint32_t>();
        for (uint32_t i = 0; i < n; i++) tot += kc[i];
        out->total_ids = tot;
        out->total_spans = prev;
        out->span_off = o.r_off.as<uint32_t>();
        out->span_cnt = o.r_cnt.as<uint32_t>();
        out->spans = o.r_runs.as<tm_span>();
        out->kcnt = kc;
        out->status = o.r_status.as<int32_t>();
        return TM_OK;
    }
    eng->err = "tm_match_batch_runs: span output still short after resizing";
    return TM_EDEVICE;
}

// library-internal (batcher.cpp): a window in runs form, every output in the window's own
// buffers: spans (uint4 = tm_span) at d_spans, reserved from *d_cursor (zeroed here);
// per-topic span offset / span count / id count / status.  *d_ctl_out: the launch's counter
// block (pool demand).  The caller holds a lease (tmx_lease_take) until the spans are used.
__attribute__((visibility("hidden"))) int tmx_batch_match_runs(tm_engine *eng, uint32_t set, const uint8_t *d_bytes,
                                                               const uint32_t *d_off, uint32_t n, uint64_t total_bytes,
                                                               void *stream, void *d_spans, uint64_t spans_cap,
                                                               uint32_t *d_soff, uint32_t *d_scnt, uint32_t *d_kcnt,
                                                               int32_t *d_status, unsigned long long *d_cursor,
                                                               const void **d_ctl_out, uint32_t id_w) {
    if (eng->replica && !eng->r_ids) return TM_ESTATE;
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    // id_w 4: spans of the u32 id arena, while every id fits (the caller holds a lease: no
    // commit can add a wider id before the spans are used)
    if (id_w != 4 && id_w != 8) return TM_EINVAL;
    if (id_w == 4 && !eng->ids32()) return TM_ESTATE;
    struct W {
        tm_engine *e;
        ~W() { e->runs_w = 8; }
    } reset_w{eng};
    eng->runs_w = id_w;
    eng->bb = eng->batch_set(set);
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    hipStream_t s = stream ? (hipStream_t)stream : eng->stream;
    TM_TRY_HIP(eng->chain_after_last(s), TM_EDEVICE, "stream order");
    int rc = ensure_batch(eng, n, total_bytes);
    if (rc) return rc;
    eng->bb->last_stream = s;
    eng->bb->last_n = n;
    eng->bb->dev_batch = false;  // no key-form result in this set
    TM_TRY_HIP(hipMemsetAsync(d_cursor, 0, 8, s), TM_EDEVICE, "memset");
    const TopicOut to{d_soff, d_scnt, d_kcnt, d_status};
    TM_TRY_HIP(enqueue_match(eng, d_bytes, d_off, n, s, MODE_RUNS, 0, (uint32_t *)d_spans, spans_cap, d_cursor, &to),
               TM_EDEVICE, "kernel launch");
    TM_TRY_HIP(eng->note_use(s), TM_EDEVICE, "event");
    *d_ctl_out = eng->bb->p_ctl;
    return TM_OK;
}
// library-internal (batcher.cpp): the caller is about to destroy stream s.  The engine keeps
// stream handles beside the index (`uses`: streams whose reads a publish waits for; each batch
// set's `last_stream`, which the next batch on the set is ordered after): forget s in both, so
// no later call records an event on a destroyed stream (round 5: an aggregator closed, the next
// one's first window ordered itself after the old stream -- a use-after-free inside HIP).
__attribute__((visibility("hidden"))) void tmx_engine_forget_stream(tm_engine *eng, void *stream) {
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    hipStream_t s = (hipStream_t)stream;
    if (!s) return;
    (void)hipSetDevice(eng->cfg.device);
    (void)hipStreamSynchronize(s);
    for (size_t i = 0; i < eng->uses.size();) {
        if (eng->uses[i].first == s) {
            (void)hipEventDestroy(eng->uses[i].second);
            eng->uses.erase(eng->uses.begin() + (ptrdiff_t)i);
        } else {
            i++;
        }
    }
    for (BatchBufs *B : {&eng->bb_dev, &eng->bb_dev2, &eng->bb_dev3, &eng->bb_batch, &eng->bb_batch2})
        if (B->last_stream == s) B->last_stream = nullptr;
}
// library-internal (batcher.cpp): size buffer set `set` for batches of up to n topics and
// `bytes` topic bytes before the first window, so no window grows them (a growth waits for
// the whole device: the aggregator's slowest windows, round 5)
__attribute__((visibility("hidden"))) int tmx_engine_reserve_batch(tm_engine *eng, uint32_t set, uint32_t n,
                                                                   uint64_t bytes) {
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    eng->bb = eng->batch_set(set);
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    int rc = ensure_batch(eng, n, bytes);
    if (rc) return rc;
    // what a window of n topics grows besides (ids transport: per-wave info, scan scratch),
    // and the chunk pools at 4x / 4x the first batch's default (config C's 12 K-publish windows
    // asked for ~2x of it): the growth the round-5 window traces showed as 13-20 ms stalls
    const uint64_t nwaves = match_grid(n, pick_tpw(n, eng->cfg.topics_per_wave));
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_wave_info, nwaves * 16 + 16), TM_ENOMEM, "alloc");
    TM_TRY_HIP(eng->grow_buf(eng->bb->d_res_scan, scan_scratch_words(n) * 4), TM_ENOMEM, "alloc");
    eng->bb->seg_demand_last = std::max<uint64_t>(eng->bb->seg_demand_last, ((uint64_t)n + 63) / 64 * 32);
    eng->bb->fr_demand_last = std::max<uint64_t>(eng->bb->fr_demand_last, ((uint64_t)n + 63) / 64 * 16);
    return grow_pools(eng);
}
// library-internal (batcher.cpp): tm_reserve_matches for the aggregator's buffer set
__attribute__((visibility("hidden"))) int tmx_batch_reserve_matches(tm_engine *eng, uint32_t set, uint64_t keys_cap) {
    std::lock_guard<std::recursive_mutex> g(eng->mu_dev);
    eng->bb = eng->batch_set(set);
    if (hipSetDevice(eng->cfg.device) != hipSuccess) return TM_EDEVICE;
    if (keys_cap > eng->bb->keys_cap) {
        TM_TRY_HIP(eng->grow_buf(eng->bb->d_keys, keys_cap * 4), TM_ENOMEM, "alloc keys");
        eng->bb->keys_cap = keys_cap;
    }
    return TM_OK;
}
__attribute__((visibility("hidden"))) void tmx_lease_take(tm_engine *eng) { eng->lease_take_raw(); }
__attribute__((visibility("hidden"))) void tmx_lease_drop(tm_engine *eng) { eng->lease_drop_raw(); }
__attribute__((visibility("hidden"))) int tmx_engine_is_replica(const tm_engine *eng) { return eng->replica ? 1 : 0; }
// the epoch the device serves (a stamp for the aggregator's window trace: read without the lock)
__attribute__((visibility("hidden"))) uint64_t tmx_engine_epoch(const tm_engine *eng) {
    return eng->dv.epoch.load(std::memory_order_relaxed);
}
// the runs form on this engine: a master, or a replica that keeps its host id arena
__attribute__((visibility("hidden"))) int tmx_engine_runs_ok(const tm_engine *eng) {
    return !eng->replica || eng->r_ids ? 1 : 0;
}

int tm_runs_release(tm_engine *eng) {
    if (!eng) return TM_EINVAL;
    HostOut &o = eng->out();
    eng->lease_drop(o);
    return TM_OK;
}

}  // extern "C"
