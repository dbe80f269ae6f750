// cpu_costs.cpp — per-operation host costs on the GPU box's CPUs (bench tooling): the pieces
// a batching-aggregator delivery is made of, one thread each.  Usage: cpu_costs
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <ctime>
#include <mutex>
#include <random>
#include <vector>

static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
    const int N = 2'000'000;
    volatile uint64_t sink = 0;
    uint64_t s = 0;
    std::vector<uint64_t> ids(142 * 1024);
    for (auto &x : ids) x = (uint64_t)rand();
    double t = now();
    for (int i = 0; i < N; i++) {
        const uint64_t *p = &ids[(i & 1023) * 142];
        for (int k = 0; k < 142; k++) s += p[k];
    }
    sink = s;
    std::printf("{\"sum142_ns\": %.1f, ", (now() - t) / N * 1e9);
    std::vector<uint8_t> tb(60u << 20);
    std::vector<uint32_t> off(1000001);
    for (int i = 0; i <= 1000000; i++) off[i] = i * 60;
    std::mt19937 r(1);
    std::vector<uint32_t> ks(N);
    for (auto &k : ks) k = r() % 1000000;
    uint8_t buf[64];
    t = now();
    for (int i = 0; i < N; i++) {
        const uint32_t k = ks[i];
        std::memcpy(buf, &tb[off[k]], off[k + 1] - off[k]);
        s += buf[3];
    }
    sink = s;
    std::printf("\"random_topic_fetch_ns\": %.1f, ", (now() - t) / N * 1e9);
    std::mutex m;
    std::vector<uint64_t> q;
    q.reserve(N);
    t = now();
    for (int i = 0; i < N; i++) {
        std::lock_guard<std::mutex> g(m);
        q.push_back(i);
    }
    std::printf("\"mutex_push_ns\": %.1f, ", (now() - t) / N * 1e9);
    t = now();
    for (int i = 0; i < N; i++) s += (uint64_t)std::chrono::steady_clock::now().time_since_epoch().count();
    sink = s;
    std::printf("\"steady_clock_ns\": %.1f, ", (now() - t) / N * 1e9);
    t = now();
    for (int i = 0; i < N; i++) s += __builtin_ia32_rdtsc();
    sink = s;
    std::printf("\"rdtsc_ns\": %.1f, ", (now() - t) / N * 1e9);
    t = now();
    for (int i = 0; i < N; i++) {
        timespec ts;
        clock_gettime(CLOCK_MONOTONIC_COARSE, &ts);
        s += (uint64_t)ts.tv_nsec;
    }
    sink = s;
    std::printf("\"coarse_clock_ns\": %.1f}\n", (now() - t) / N * 1e9);
    (void)sink;
    return 0;
}
