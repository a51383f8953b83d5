// Wave-level cross-lane helpers for gfx950 (wave64), shared by the kernels and tools/dpp_check.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zbpe {

// Cross-lane moves as DPP, one VALU op each (CDNA's wave-wide shifts and row broadcasts), where __shfl is an
// LDS-crossbar ds_bpermute plus its lane arithmetic. Whole-wave only (every lane active): a lane whose source
// lies outside the wave gets `fill`.
// lane i <- x of lane i - 1 (lane 0 <- fill) / of lane i + 1 (lane 63 <- fill)
__device__ __attribute__((always_inline)) inline uint32_t wave_shr1(uint32_t x, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)x, 0x138, 0xF, 0xF, false);
}
__device__ __attribute__((always_inline)) inline uint32_t wave_shl1(uint32_t x, uint32_t fill) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)fill, (int)x, 0x130, 0xF, 0xF, false);
}
// a DPP move inside rows (quad_perm, mirrors: every source lane valid)
template <int CTRL>
__device__ __attribute__((always_inline)) inline uint32_t dpp_mov(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
// all-reduces (every lane active), wave-uniform results: a butterfly inside each 16-lane row (quad_perm [1,0,3,2]
// and [2,3,0,1], half-row mirror, row mirror: each step joins two disjoint halves), then the four rows by readlane
__device__ __attribute__((always_inline)) inline uint32_t wave_max_u32(uint32_t x) {
    x = max(x, dpp_mov<0xB1>(x));
    x = max(x, dpp_mov<0x4E>(x));
    x = max(x, dpp_mov<0x141>(x));
    x = max(x, dpp_mov<0x140>(x));
    return max(max((uint32_t)__builtin_amdgcn_readlane((int)x, 0), (uint32_t)__builtin_amdgcn_readlane((int)x, 16)),
               max((uint32_t)__builtin_amdgcn_readlane((int)x, 32), (uint32_t)__builtin_amdgcn_readlane((int)x, 48)));
}
__device__ __attribute__((always_inline)) inline uint32_t wave_sum_u32(uint32_t x) {
    x += dpp_mov<0xB1>(x);
    x += dpp_mov<0x4E>(x);
    x += dpp_mov<0x141>(x);
    x += dpp_mov<0x140>(x);
    return (uint32_t)__builtin_amdgcn_readlane((int)x, 0) + (uint32_t)__builtin_amdgcn_readlane((int)x, 16) +
           (uint32_t)__builtin_amdgcn_readlane((int)x, 32) + (uint32_t)__builtin_amdgcn_readlane((int)x, 48);
}
// lane l's x, as a scalar
__device__ __attribute__((always_inline)) inline uint32_t lane_bcast(uint32_t x, int l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)x, l);
}
// inclusive prefix sum over the wave: shifts 1, 2, 4, 8 inside each 16-lane row, then row 0's total into row 1
// and row 2's into row 3 (row_bcast:15), rows 0-1's into rows 2 and 3 (row_bcast:31); lanes a step does not
// write add the 0 they start from
__device__ __attribute__((always_inline)) inline uint32_t wave_incl_scan_dpp(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
}

}  // namespace zbpe
