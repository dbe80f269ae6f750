// tools/gather_roof.hip — the random-gather ceiling of one MI355X, for the walk's roofline.
//
// k_match_fast's probes are independent random 16-B loads into a table of GiBs (the edge
// table).  Their ceiling is not the streaming HBM bandwidth but the rate at which the
// memory system serves random 16-B requests that miss the caches.  This measures it with
// no dependence between loads: every lane keeps U loads in flight, tables of 2 MiB (L2-
// resident) to 32 GiB (round 3: the config-C edge table is 16 GiB at load 1/16), 16 waves
// per CU.
//
// `gather_roof contig [GiB]` allocates the table with hipExtMallocWithFlags(..,
// hipDeviceMallocContiguous) instead of hipMalloc (round 4: does physically contiguous VRAM,
// which lets the page tables use large fragments, relieve the address translation that the
// walk's PMC passes show busy?).  Every line then carries "alloc": "contig".
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/gather_roof.hip -o tools/gather_roof
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

static const char *g_alloc = "default";

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

template <int U>
__global__ __launch_bounds__(256) void k_gather(const uint4 *tab, unsigned long long mask16, unsigned iters,
                                                unsigned seed, unsigned *out) {
    const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (unsigned it = 0; it < iters; it++) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = tab[mix((g * iters + it) * U + u + seed) & mask16];
#pragma unroll
        for (int u = 0; u < U; u++) acc += v[u].x ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// The same loads, but the 64 lanes of a wave's load instruction fall into 64 / G distinct
// 2 MiB regions (G lanes per region, random 16-B slots inside it): how much of the ceiling is
// address translation, which lanes sharing a region share.
template <int U>
__global__ __launch_bounds__(256) void k_gather_grp(const uint4 *tab, unsigned long long nreg, unsigned g_shift,
                                                    unsigned iters, unsigned seed, unsigned *out) {
    const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    const unsigned long long wv = g >> 6, lane = g & 63;
    unsigned acc = 0;
    for (unsigned it = 0; it < iters; it++) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const unsigned long long k = (wv * iters + it) * U + u + seed;
            const unsigned long long reg = mix(k * 64 + (lane >> g_shift)) % nreg;
            const unsigned long long off = mix(k * 64 + lane + (1ull << 40)) & ((2ull << 20) / 16 - 1);
            v[u] = tab[reg * ((2ull << 20) / 16) + off];
        }
#pragma unroll
        for (int u = 0; u < U; u++) acc += v[u].x ^ v[u].w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

template <int U>
static void run_grp(const uint4 *tab, unsigned long long bytes, unsigned g_shift, unsigned *out) {
    const unsigned blocks = 256 * 4, threads = 256;
    const unsigned iters = 64 / U * 4;
    const unsigned long long loads = (unsigned long long)blocks * threads * iters * U, nreg = bytes >> 21;
    k_gather_grp<U><<<blocks, threads>>>(tab, nreg, g_shift, iters, 1, out);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    k_gather_grp<U><<<blocks, threads>>>(tab, nreg, g_shift, iters, 7, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("{\"alloc\": \"%s\", \"table_MiB\": %llu, \"lanes_per_2MiB_region\": %u, \"inflight_per_lane\": %d, "
           "\"loads\": %llu, \"ms\": %.4f, \"G_loads_per_s\": %.2f}\n",
           g_alloc, bytes >> 20, 1u << g_shift, U, loads, ms, loads / (ms * 1e6));
    fflush(stdout);
}

template <int U>
static void run(const uint4 *tab, unsigned long long bytes, unsigned *out) {
    const unsigned blocks = 256 * 4, threads = 256;  // 16 waves per CU
    const unsigned iters = 64 / U * 4;
    const unsigned long long loads = (unsigned long long)blocks * threads * iters * U;
    k_gather<U><<<blocks, threads>>>(tab, bytes / 16 - 1, iters, 1, out);
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k_gather<U><<<blocks, threads>>>(tab, bytes / 16 - 1, iters, 7, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("{\"alloc\": \"%s\", \"table_MiB\": %llu, \"inflight_per_lane\": %d, \"loads\": %llu, \"ms\": %.4f, "
           "\"G_loads_per_s\": %.2f, \"GBps_at_64B\": %.0f}\n",
           g_alloc, bytes >> 20, U, loads, ms, loads / (ms * 1e6), loads * 64.0 / (ms * 1e6));
    fflush(stdout);
}

int main(int argc, char **argv) {
    // `gather_roof regions [GiB]`: only the region-grouped loads, at the given table size
    const bool regions = argc > 1 && !strcmp(argv[1], "regions");
    const bool contig = argc > 1 && !strcmp(argv[1], "contig");
    const unsigned long long maxb = (argc > 2 ? strtoull(argv[2], nullptr, 10) : 32ull) << 30;
    uint4 *tab;
    unsigned *out;
    if (contig) {
        g_alloc = "contig";
        if (hipExtMallocWithFlags((void **)&tab, maxb, hipDeviceMallocContiguous) != hipSuccess) return 2;
    } else if (hipMalloc(&tab, maxb) != hipSuccess) {
        return 1;
    }
    if (hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(tab, 1, maxb);
    if (regions) {
        for (unsigned gs = 0; gs <= 6; gs++) {
            run_grp<1>(tab, maxb, gs, out);
            run_grp<4>(tab, maxb, gs, out);
        }
        (void)hipFree(tab);
        (void)hipFree(out);
        return 0;
    }
    for (unsigned long long b : {2ull << 20, 16ull << 20, 64ull << 20, 256ull << 20, 1ull << 30, 4ull << 30, 8ull << 30,
                                 16ull << 30, 32ull << 30}) {
        if (b > maxb) break;
        run<1>(tab, b, out);
        run<4>(tab, b, out);
        run<8>(tab, b, out);
        run<16>(tab, b, out);
    }
    hipFree(tab);
    hipFree(out);
    return 0;
}
