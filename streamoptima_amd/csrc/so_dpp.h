// so_dpp.h — wavefront reductions with DPP (register-to-register VALU, no LDS round trip)
// shared by the ME kernels.
#pragma once
#include "so_common.h"

namespace so {

// Cross-lane reductions with DPP (register-to-register VALU; no ds_bpermute round trips):
// quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror, row_mirror leave every lane with its
// 16-lane row's result; row_bcast15 (rows 1, 3) and row_bcast31 (rows 2, 3) carry it into
// lane 63, which v_readlane broadcasts.  DPP lanes without a source keep `old`.
constexpr int kDppQuad1032 = 0xB1, kDppQuad2301 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;
constexpr int kDppBcast15 = 0x142, kDppBcast31 = 0x143;

// (old = ~0u, the identity of min: the compiler folds each step into one v_min_u32_dpp)
SO_DEV uint32_t row_min_u32(uint32_t v) {
    v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, kDppQuad1032, 0xF, 0xF, false));
    v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, kDppQuad2301, 0xF, 0xF, false));
    v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, kDppHalfMirror, 0xF, 0xF, false));
    v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, kDppMirror, 0xF, 0xF, false));
    return v;
}

// wave-uniform minimum (SGPR)
SO_DEV uint32_t wave_min_u32(uint32_t v) {
    v = row_min_u32(v);
    v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, kDppBcast15, 0xA, 0xF, false));
    v = __builtin_elementwise_min(v, (uint32_t)__builtin_amdgcn_update_dpp(~0u, v, kDppBcast31, 0xC, 0xF, false));
    return __builtin_amdgcn_readlane(v, 63);
}

// sum over each 16-lane row, in every lane of the row
SO_DEV uint32_t row_sum_u32(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, kDppQuad1032, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, kDppQuad2301, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, kDppHalfMirror, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, kDppMirror, 0xF, 0xF, false);
    return v;
}

// wave-uniform sum (SGPR)
SO_DEV uint32_t wave_sum_u32(uint32_t v) {
    v = row_sum_u32(v);
    v += __builtin_amdgcn_update_dpp(0u, v, kDppBcast15, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, kDppBcast31, 0xC, 0xF, false);
    return __builtin_amdgcn_readlane(v, 63);
}

template <int CTRL, int RMASK>
SO_DEV uint64_t dpp_min_step(uint64_t v) {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    const uint32_t olo = __builtin_amdgcn_update_dpp(lo, lo, CTRL, RMASK, 0xF, false);
    const uint32_t ohi = __builtin_amdgcn_update_dpp(hi, hi, CTRL, RMASK, 0xF, false);
    const uint64_t o = ((uint64_t)ohi << 32) | olo;
    return o < v ? o : v;
}

// wave-uniform 64-bit minimum: the minimum high word, then the minimum low word among the
// lanes holding it (two folded 32-bit DPP reductions instead of six 64-bit compare steps)
SO_DEV uint64_t wave_min_u64_dpp(uint64_t v) {
    const uint32_t hi = wave_min_u32((uint32_t)(v >> 32));
    const uint32_t lo = wave_min_u32((uint32_t)(v >> 32) == hi ? (uint32_t)v : ~0u);
    return ((uint64_t)hi << 32) | lo;
}

SO_DEV uint64_t wave_min_u64(uint64_t v) { return wave_min_u64_dpp(v); }

// inclusive prefix sum over the wave (lane i: v_0 + ... + v_i): row_shr 1, 2, 4, 8 inside each
// 16-lane row, then row_bcast15 / row_bcast31 carry the row totals into the rows above
SO_DEV uint32_t wave_incl_scan_u32(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, kDppBcast15, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, kDppBcast31, 0xC, 0xF, false);
    return v;
}

SO_DEV uint32_t lane_prefix(uint64_t mask) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0u));
}

// sum over each aligned 4-lane quad, in every lane of the quad
SO_DEV uint32_t quad_sum_u32(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, kDppQuad1032, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, kDppQuad2301, 0xF, 0xF, false);
    return v;
}

}  // namespace so
