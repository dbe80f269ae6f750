// copy_api.h — device -> pinned host copies written by a kernel (result_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace tmx {

// n u32 words from device memory into pinned host memory (dst: its device address), written
// by a kernel over PCIe instead of a DMA engine.  Large D2H copies of match output take this
// path: on the pool's boxes the SDMA path of hipMemcpyAsync into pinned memory ran at ~27 GB/s
// after the first call, the kernel path at the link's ~45 GB/s.
hipError_t launch_copy_to_host(uint32_t *dst, const uint32_t *src, uint64_t n, hipStream_t s);

}  // namespace tmx
