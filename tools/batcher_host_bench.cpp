// batcher_host_bench.cpp — the batching aggregator's HOST overhead alone (bench tooling):
// a closed loop of P publishers (tools/loadgen.cpp) over a backend that answers every
// publish with K fixed ids and no device work, so what is measured is submit, window
// cutting, delivery threads and resubmission.  Usage: batcher_host_bench P K seconds threads
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../include/emqx_tm_batcher.h"

extern "C" int loadgen_run(tm_batcher *b, const uint8_t *bytes, const uint32_t *off, uint32_t n_topics,
                           uint32_t publishers, double seconds, uint64_t *published, uint64_t *ids_out,
                           uint64_t *errors, double *elapsed_s);

struct Fixed {
    uint32_t k;
    std::vector<uint32_t> off, cnt;
    std::vector<uint64_t> ids;
    std::vector<int32_t> st;
};

static int fixed_batch(void *be, const uint8_t *, const uint32_t *, uint32_t n, uint32_t, tm_batch_view *v) {
    Fixed *f = (Fixed *)be;
    if (f->off.size() < n) {
        f->off.assign(n, 0);  // every publish gets the same K ids
        f->cnt.assign(n, f->k);
        f->st.assign(n, 0);
    }
    v->off = f->off.data();
    v->cnt = f->cnt.data();
    v->ids = f->ids.data();
    v->status = f->st.data();
    return 0;
}

int main(int argc, char **argv) {
    const uint32_t P = argc > 1 ? atoi(argv[1]) : 65536, K = argc > 2 ? atoi(argv[2]) : 142;
    const double secs = argc > 3 ? atof(argv[3]) : 2.0;
    const uint32_t threads = argc > 4 ? atoi(argv[4]) : 4;
    Fixed f;
    f.k = K;
    f.ids.assign(K + 1, 7);
    std::vector<uint8_t> bytes;
    std::vector<uint32_t> off{0};
    for (int i = 0; i < 1000; i++) {
        char t[64];
        int n = snprintf(t, sizeof t, "tenant%d/region%d/dev%d/x/y", i % 32, i % 64, i);
        bytes.insert(bytes.end(), t, t + n);
        off.push_back((uint32_t)bytes.size());
    }
    tm_batcher_config cfg{65536, 200, TM_MATCH_ALL, threads};
    tm_batcher *b = nullptr;
    if (tm_batcher_create_fn(fixed_batch, &f, &cfg, &b)) return 1;
    uint64_t got = 0, ids = 0, errs = 0;
    double el = 0;
    loadgen_run(b, bytes.data(), off.data(), 1000, P, secs, &got, &ids, &errs, &el);
    tm_batcher_stats st{};
    tm_batcher_stats_get(b, &st);
    tm_batcher_destroy(b);
    // delivery cost per publish: the delivery threads' busy time (deliver_us is per thread)
    const double del_ns = (double)st.deliver_us * 1e3 * threads / (double)(got ? got : 1);
    printf("{\"publishers\": %u, \"ids_per_publish\": %u, \"threads\": %u, \"publishes_per_s\": %.0f, "
           "\"mean_batch\": %.1f, \"p50_ms\": %.3f, \"p99_ms\": %.3f, \"errors\": %lu, \"deliver_ns_per_publish\": %.1f, "
           "\"cut_ns_per_publish\": %.1f}\n",
           P, K, threads, got / el, st.batches ? (double)st.publishes / st.batches : 0.0, st.lat_p50_us / 1e3,
           st.lat_p99_us / 1e3, (unsigned long)errs, del_ns, (double)st.cut_us * 1e3 / (double)(got ? got : 1));
    return 0;
}
