// so_blockops.hip — batched per-block transforms for the reference's per-block public
// methods (the drop-in surface): apply_2d_dct (Encoder.py:779-784),
// quantize_TC (:787-789), len(entropy_encoder_block) (:1086-1131) as calculate_RD_cost uses
// them (:1133-1158), and apply_2d_idct (:810-817) as reconstruct_block uses it (:824-827).
//
// The reference calls these one block at a time; here one launch transforms n blocks.  The
// arithmetic is the frame kernels' own: the pocketfft DCT-II / DCT-III replica in FP64
// (so_dct.h, no FMA contraction), np.round = rint (half to even), quantisation by 2^k with
// the Q-matrix exponents, the register-only token count (so_block.h).  Input blocks are
// doubles (the reference passes float64 residuals), so any integer- or float-valued block
// goes through exactly pocketfft's operation sequence.
//
// Layout: N lanes per block (lane l owns row l), 256-thread workgroups = 256/N blocks, an
// N x (N+1) FP64 LDS transpose tile per block.  Memory-bound and tiny next to the frame
// path; its job is parity of the per-block API, not throughput.
#include "so_common.h"
#include "so_dct.h"
#include "so_block.h"

namespace so {

template <int N>
__global__ void __launch_bounds__(256) block_xform_kernel(const double* __restrict__ in, int n, int inverse, int qp,
                                                          int32_t* __restrict__ out_tc, int32_t* __restrict__ out_q,
                                                          int32_t* __restrict__ out_tokens) {
    constexpr int G = 256 / N, P = N + 1;
    __shared__ double lds[G * N * P];
    const int g = threadIdx.x / N, l = threadIdx.x % N;
    const long b = (long)blockIdx.x * G + g;
    const bool live = b < n;   // every lane of the group still takes part in the transposes
    double row[N], out[N];
#pragma unroll
    for (int c = 0; c < N; ++c) row[c] = live ? in[(b * N + l) * N + c] : 0.0;
    double* s = lds + g * N * P;
    if (inverse)
        xform2d_rows<N, true>(s, l, row, out);
    else
        xform2d_rows<N, false>(s, l, row, out);
    int tc[N];
#pragma unroll
    for (int c = 0; c < N; ++c) tc[c] = (int)__builtin_rint(out[c]);   // np.round(...).astype(int)
    if (live && out_tc) {
#pragma unroll
        for (int c = 0; c < N; ++c) out_tc[(b * N + l) * N + c] = tc[c];
    }
    if (qp < 0 || inverse) return;   // uniform
    int q[N];
    quant_row_i<N>(tc, l, qp, q);     // np.round(TC / Q) (quantize_TC)
    if (live && out_q) {
#pragma unroll
        for (int c = 0; c < N; ++c) out_q[(b * N + l) * N + c] = q[c];
    }
    const int tok = block_tokens<N>(nullptr, l, q);
    if (live && out_tokens && l == 0) out_tokens[b] = tok;
}

int block_xform_launch(const double* in, int n, int N, int inverse, int qp, int32_t* out_tc, int32_t* out_q,
                       int32_t* out_tokens, hipStream_t st) {
    if (n <= 0) return SO_OK;
    if (N == 16) {
        hipLaunchKernelGGL(block_xform_kernel<16>, dim3((n + 15) / 16), dim3(256), 0, st, in, n, inverse, qp, out_tc,
                           out_q, out_tokens);
    } else {
        hipLaunchKernelGGL(block_xform_kernel<8>, dim3((n + 31) / 32), dim3(256), 0, st, in, n, inverse, qp, out_tc,
                           out_q, out_tokens);
    }
    return check_launch("block_xform_kernel");
}

}  // namespace so

extern "C" int so_block_xform(const double* in, int n, int N, int inverse, int qp, int32_t* out_tc, int32_t* out_q,
                              int32_t* out_tokens, void* stream) {
    if (n < 0 || !(N == 16 || N == 8) || (n > 0 && in == nullptr) || qp > 30) {
        so::set_error("so_block_xform: bad arguments (n=%d N=%d qp=%d)", n, N, qp);
        return SO_E_INVALID;
    }
    if (inverse && (out_q || out_tokens)) {
        so::set_error("so_block_xform: the inverse transform has no quantised output or tokens");
        return SO_E_INVALID;
    }
    return so::block_xform_launch(in, n, N, inverse, qp, out_tc, out_q, out_tokens, (hipStream_t)stream);
}
