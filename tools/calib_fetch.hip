// tools/calib_fetch.hip — calibrate rocprofv3 FETCH_SIZE on gfx950 for the access
// pattern of k_match_fast (independent random 16-B loads), and for a wide coalesced
// stream.  MI355X_MICROARCH.md §HBM: "Other access widths are uncalibrated: calibrate
// on a known byte count in your own access pattern before trusting an absolute."
//
// Build: hipcc --offload-arch=gfx950 -O3 tools/calib_fetch.hip -o tools/calib_fetch
// Run:   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -- ./tools/calib_fetch
// Prints the known line/byte counts of each kernel; compare with FETCH_SIZE per dispatch.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__device__ __forceinline__ unsigned long long mix(unsigned long long x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

// Each lane loads `per` random 16-B records, each in its own 128-B line (the line
// index is a hash of the global load number; the table is 16 GiB so reuse is rare).
__global__ void k_random16(const uint4 *tab, unsigned long long lines, unsigned per, unsigned *out) {
    const unsigned long long g = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (unsigned k = 0; k < per; k++) {
        const unsigned long long line = mix(g * per + k + 1) % lines;
        const uint4 v = tab[line * 8 + (mix(line) & 7)];  // one 16-B record of the 128-B line
        acc += v.x ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

// Wide coalesced stream: 16 B per lane, contiguous.
__global__ void k_stream16(const uint4 *tab, unsigned long long n16, unsigned *out) {
    unsigned acc = 0;
    for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
         i += (unsigned long long)gridDim.x * blockDim.x) {
        const uint4 v = tab[i];
        acc += v.y;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const unsigned long long bytes = 16ull << 30;  // 16 GiB table
    uint4 *tab;
    unsigned *out;
    if (hipMalloc(&tab, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
        fprintf(stderr, "alloc failed\n");
        return 1;
    }
    hipMemset(tab, 1, bytes);
    const unsigned long long lines = bytes / 128;
    const unsigned blocks = 4096, threads = 256, per = 16;
    const unsigned long long loads = (unsigned long long)blocks * threads * per;
    k_random16<<<blocks, threads>>>(tab, lines, per, out);  // warm (TLB)
    hipDeviceSynchronize();
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    k_random16<<<blocks, threads>>>(tab, lines, per, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("k_random16: %llu random 16-B loads, each in a distinct 128-B line (~%llu lines, %.3f GB of lines), %.3f ms,"
           " %.1f G loads/s\n",
           loads, loads, loads * 128.0 / 1e9, ms, loads / (ms * 1e6));
    const unsigned long long n16 = (4ull << 30) / 16;  // stream 4 GiB
    hipEventRecord(e0);
    k_stream16<<<2048, 256>>>(tab, n16, out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    hipEventElapsedTime(&ms, e0, e1);
    printf("k_stream16: %llu bytes streamed, %.3f ms, %.1f GB/s\n", n16 * 16, ms, n16 * 16 / (ms * 1e6));
    hipFree(tab);
    hipFree(out);
    return 0;
}
