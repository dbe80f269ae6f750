// wave.h — wave64 lane primitives shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace tmx {

// Inclusive prefix sum over the 64 lanes of a wave on DPP lane moves (VALU ops, no LDS):
// within each row of 16 lanes (row_shr 1, 2, 4, 8; lanes shifted in from outside the row
// read 0), then the row totals (row_bcast 15 into rows 1 and 3, row_bcast 31 into rows 2
// and 3).  ds_bpermute-based __shfl_up scans cost six LDS round trips per scan.
__device__ __forceinline__ uint32_t wave_incl_scan_dpp(uint32_t x) {
    x += __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);
    x += __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);
    return x;
}

// OR of x over the 64 lanes (the same DPP moves; the result is read from lane 63)
__device__ __forceinline__ uint32_t wave_or_dpp(uint32_t x) {
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x111, 0xf, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x112, 0xf, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x114, 0xf, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x118, 0xf, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x142, 0xa, 0xf, false);
    x |= __builtin_amdgcn_update_dpp(0u, x, 0x143, 0xc, 0xf, false);
    return __builtin_amdgcn_readlane(x, 63);
}
__device__ __forceinline__ uint64_t wave_or64_dpp(uint64_t x) {
    return ((uint64_t)wave_or_dpp((uint32_t)(x >> 32)) << 32) | wave_or_dpp((uint32_t)x);
}

// value of x in lane l (l wave-uniform): v_readlane, no LDS
__device__ __forceinline__ uint32_t lane_value(uint32_t x, uint32_t l) { return __builtin_amdgcn_readlane(x, l); }

}  // namespace tmx
