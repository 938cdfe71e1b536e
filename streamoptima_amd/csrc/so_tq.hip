// so_tq.hip — P-frame transform / quantisation / RD / reconstruction, and the decoder's
// inter reconstruction, for gfx950.
//
// inter_tq_kernel replaces, for every block of a P-frame at once:
//   calculate_inter_frame_residual (Encoder.py:432-460, handle_boundary_conditions :750),
//   apply_2d_dct (:779) -> quantize_TC (:787) -> len(entropy_encoder_block) (:1086),
//   the VBS decision calculate_RD_cost(1,1,..) vs (1,0,..) (:564-578, :1133-1158),
//   the per-row-QP requantisation of complete_inter_flow (:1665-1697) and
//   reconstruct_frame / reconstruct_block (:824-932): rescale, IDCT, + pred, uint8 wrap.
// 16 lanes of one wavefront own one 16x16 block (8 lanes for 8x8 blocks); a 256-thread
// workgroup carries 16 blocks.  Everything between the HBM reads (cur, pred, ME result)
// and the HBM writes (QTC, recon, symbols) stays in VGPRs / LDS.
#include "so_block.h"

namespace so {

// Two-pass pass 2 with the QP map derived in the kernel (QPM; so_encode_p_run_2pass): the
// pass-1 token counts t1 (stripe-local, one per block), the ROI offsets and the clamp of
// qp_map_kernel (so_capi.hip), whose per-block QP this reproduces; the map is also written out.
struct QpmArgs {
    const int32_t* t1;
    const int32_t* roi;
    int qp_lo, qp_hi;
    int32_t* out_qpmap;
};

template <int BS, bool VBS, bool FME, bool QPM = false>
__global__ void __launch_bounds__(256)
inter_tq_kernel(const uint8_t* __restrict__ cur, RefSet refs, const uint8_t* __restrict__ planes, size_t pstride,
                int H, int W, int by0, int nrows,
                const int32_t* __restrict__ best, const int32_t* __restrict__ sub, int qp_rd,
                const int32_t* __restrict__ qp_row, const int32_t* __restrict__ qp_map, double lam,
                uint8_t* __restrict__ out_split,
                int16_t* __restrict__ out_mv, int16_t* __restrict__ out_qtc,
                int32_t* __restrict__ out_tokens, int32_t* __restrict__ out_mae,
                uint8_t* __restrict__ out_recon, int32_t* __restrict__ out_sse, const QpmArgs qa) {
    constexpr int G = BS, BPW = 256 / G, SB = BS / 2;
    constexpr int LDS_D = VBS ? 288 : BS * (BS + 1);
    __shared__ double ldsd[BPW * LDS_D];
    __shared__ uint8_t ldsf[BPW * BS * BS];
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    const int nbx = W / BS, nb = nbx * nrows;
    const int b = blockIdx.x * BPW + g;   // block index inside the stripe [by0, by0 + nrows)
    // QPM: the pass-1 token sum m of each block row this workgroup's blocks lie in (at most 3:
    // nbx >= 8), by the whole workgroup before any lane group leaves -- measured faster than
    // each block's 16 lanes summing its row themselves (configs[4] per-frame sequence 2.797 vs
    // 2.856 ms per GOP, and 2.937 with those loads unrolled)
    long long m_row = 0;
    if constexpr (QPM) {
        __shared__ long long s_m[3][4];
        const int b0 = blockIdx.x * BPW, bl = (b0 + BPW < nb ? b0 + BPW : nb) - 1;
        const int rA = b0 / nbx, nr = bl / nbx - rA + 1;
        for (int k = 0; k < nr; ++k) {   // uniform
            const int32_t* t = qa.t1 + (size_t)(rA + k) * nbx;
            long long m = 0;
            for (int i = tid; i < nbx; i += 256) m += t[i];
#pragma unroll
            for (int s = 32; s >= 1; s >>= 1) m += __shfl_xor(m, s, 64);
            if ((tid & 63) == 0) s_m[k][tid >> 6] = m;
        }
        __syncthreads();
        if (b < nb) {
            const int k = b / nbx - rA;
            m_row = s_m[k][0] + s_m[k][1] + s_m[k][2] + s_m[k][3];
        }
    }
    if (b >= nb) return;  // whole lane group leaves; only wave-scope exchange below
    double* dl = ldsd + g * LDS_D;
    uint8_t* fl = ldsf + g * BS * BS;
    const int bx = b % nbx, by = by0 + b / nbx, x = bx * BS, y = by * BS;
    // per-block QP map (ROI / two-pass RC) > per-row RC QP > the frame QP
    int qpr = qp_map ? qp_map[(size_t)by * nbx + bx] : (qp_row ? qp_row[by] : qp_rd);
    if constexpr (QPM) {   // qp_map_kernel's rule (delta from t n against 2m, 4m, m/2, m/4)
        const long long tn = (long long)qa.t1[b] * nbx;
        const int d = (tn >= 2 * m_row) + (tn >= 4 * m_row) - (2 * tn < m_row) - (4 * tn < m_row);
        int q = (qp_row ? qp_row[by] : qp_rd) + d + (qa.roi ? qa.roi[(size_t)by * nbx + bx] : 0);
        q = q < qa.qp_lo ? qa.qp_lo : (q > qa.qp_hi ? qa.qp_hi : q);
        qpr = q;
        if (l == 0) qa.out_qpmap[(size_t)by * nbx + bx] = q;
    }

    const int32_t* bb = best + (size_t)b * 4;
    const int dx = bb[0], dy = bb[1], rf = bb[2], sad = bb[3];
    int pred[BS], crow[BS], res[BS];
    if constexpr (FME) {
        fetch_row_fme<BS>(planes + (size_t)rf * 4 * pstride, pstride, W, H, 2 * x + dx, 2 * y + dy, l, 2 * BS, BS, pred);
    } else {
        const bool fast = (0 <= x + dx) && (x + dx < W - BS) && (0 <= y + dy) && (y + dy < H - BS);
        fetch_row<BS>(refs.p[rf], W, H, x + dx, y + dy + l, fast, pred);
    }
    load_cur_row<BS>(cur, W, x, y + l, crow);
#pragma unroll
    for (int c = 0; c < BS; ++c) res[c] = crow[c] - pred[c];
    double tcr[BS];
    xform2d_rows<BS, false>(dl, l, res, tcr);
#pragma unroll
    for (int c = 0; c < BS; ++c) tcr[c] = __builtin_rint(tcr[c]);
    // Without VBS the RD QP is never used: quantise once at the block's final QP, FP64
    // carriers throughout.  With VBS the state survives the RD decision as int32.
    double qd[BS];
    int q[BS], tc[BS];
    if constexpr (VBS) {
#pragma unroll
        for (int c = 0; c < BS; ++c) tc[c] = (int)tcr[c];
        quant_row_i<BS>(tc, l, qp_rd, q);
    } else {
        quant_row_d<BS>(tcr, l, qpr, qd, q);
    }

    bool split = false;
    int mae_num = sad;
    // sub-block state (VBS)
    const int j = l >> 2, r0 = l & 3;
    int sdx = 0, sdy = 0, sref = 0, xs = 0, ys = 0;
    int spred[2][8], stc[2][8], qs[2][8];
    if constexpr (VBS) {
        if (x != 0 && y != 0) {
            const int32_t* sj = sub + ((size_t)b * 4 + j) * 4;
            sdx = sj[0]; sdy = sj[1]; sref = sj[2];
            xs = x + (j & 1) * SB; ys = y + (j >> 1) * SB;
            const bool sfast = (0 <= xs + sdx) && (xs + sdx < W - SB) && (0 <= ys + sdy) && (ys + sdy < H - SB);
            int sres[2][8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int row = r0 + 4 * h;
                int scur[8];
                if constexpr (FME)
                    fetch_row_fme<8>(planes + (size_t)sref * 4 * pstride, pstride, W, H, 2 * xs + sdx, 2 * ys + sdy,
                                     row, 16, 8, spred[h]);
                else
                    fetch_row<8>(refs.p[sref], W, H, xs + sdx, ys + sdy + row, sfast, spred[h]);
                load_cur_row<8>(cur, W, xs, ys + row, scur);
#pragma unroll
                for (int c = 0; c < 8; ++c) sres[h][c] = scur[c] - spred[h][c];
            }
            double std_[2][8];
            xform2d_sub<false>(dl, l, sres, std_);
            const int qpm1_rd = qp_rd > 0 ? qp_rd - 1 : qp_rd;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int c = 0; c < 8; ++c) stc[h][c] = (int)__builtin_rint(std_[h][c]);
                quant_row_i<8>(stc[h], r0 + 4 * h, qpm1_rd, qs[h]);
            }
            const int tok_b = block_tokens<BS>(fl, l, q);
            const int tok_v = sub_tokens(fl, l, qs);
            int ssum = 0;
            bool vinf = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const int s = sub[((size_t)b * 4 + k) * 4 + 3];
                vinf |= s < 0;
                ssum += s;
            }
            const double mae_b = sad < 0 ? __builtin_inf() : (double)sad / 256.0;
            const double mae_v = vinf ? __builtin_inf() : (double)ssum / 256.0;
            const double c_v = rd_cost(lam, 64 + 8 * tok_v, mae_v);
            const double c_b = rd_cost(lam, 16 + 8 * tok_b, mae_b);
            split = !(c_b < c_v);
            mae_num = vinf ? -1 : ssum;
        }
    }

    int tok, sse = 0;
    if (!split) {
        if (VBS && qpr != qp_rd) quant_row_i<BS>(tc, l, qpr, q);
        tok = block_tokens<BS>(fl, l, q);
        store_row_i16<BS>(out_qtc + (size_t)b * BS * BS + l * BS, q);
        int rec[BS];
        int dq[BS];
        double rd[BS];
        dequant_row_int<BS>(q, l, qpr, dq);
        xform2d_rows<BS, true>(dl, l, dq, rd);
#pragma unroll
        for (int c = 0; c < BS; ++c) rec[c] = pred[c] + (int)__builtin_rint(rd[c]);
        store_row_u8<BS>(out_recon, W, x, y + l, rec);
        sse = 0;
#pragma unroll
        for (int c = 0; c < BS; ++c) {
            const int d = crow[c] - (rec[c] & 255);
            sse += d * d;
        }
        for (int k = l; k < 12; k += G) out_mv[(size_t)b * 12 + k] = (int16_t)(k == 0 ? dx : k == 1 ? dy : k == 2 ? rf : 0);
    } else {
        if constexpr (VBS) {
            const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
            const int qpm1_rd = qp_rd > 0 ? qp_rd - 1 : qp_rd;
            if (qpm1 != qpm1_rd)
#pragma unroll
                for (int h = 0; h < 2; ++h) quant_row_i<8>(stc[h], r0 + 4 * h, qpm1, qs[h]);
            tok = sub_tokens(fl, l, qs);
            int sdq[2][8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                store_row_i16<8>(out_qtc + (size_t)b * BS * BS + j * 64 + (r0 + 4 * h) * 8, qs[h]);
                dequant_row_int<8>(qs[h], r0 + 4 * h, qpm1, sdq[h]);
            }
            double srd[2][8];
            xform2d_sub<true>(dl, l, sdq, srd);
            if constexpr (FME) {
                // the split recon predicts with the FULL block's FME bound (Encoder.py:908-909),
                // stricter than the sub-block search: those sub-blocks reconstruct on 128
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    fetch_row_fme<8>(planes + (size_t)sref * 4 * pstride, pstride, W, H, 2 * xs + sdx, 2 * ys + sdy,
                                     r0 + 4 * h, BS, BS, spred[h]);
            }
            sse = 0;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int rec[8], scur[8];
#pragma unroll
                for (int c = 0; c < 8; ++c) rec[c] = spred[h][c] + (int)__builtin_rint(srd[h][c]);
                store_row_u8<8>(out_recon, W, xs, ys + r0 + 4 * h, rec);
                load_cur_row<8>(cur, W, xs, ys + r0 + 4 * h, scur);
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    const int d = scur[c] - (rec[c] & 255);
                    sse += d * d;
                }
            }
            if (r0 < 3) out_mv[(size_t)b * 12 + 3 * j + r0] = (int16_t)(r0 == 0 ? sdx : r0 == 1 ? sdy : sref);
        } else {
            tok = 0;
        }
    }
    if (out_sse) sse = group_sum<G>(sse);
    if (l == 0) {
        out_split[b] = (uint8_t)split;
        out_tokens[b] = tok;
        out_mae[b] = mae_num;
        if (out_sse) out_sse[b] = sse;
    }
}

// Decoder: reconstruct a P-frame from (split, mv, qtc) — decoder.py:97-211, which is the
// same arithmetic as reconstruct_frame (Encoder.py:831-932).
template <int BS, bool VBS, bool FME>
__global__ void __launch_bounds__(256)
inter_recon_kernel(RefSet refs, const uint8_t* __restrict__ planes, size_t pstride, int H, int W, int qp,
                   const int32_t* __restrict__ qp_row, const int32_t* __restrict__ qp_map,
                   const uint8_t* __restrict__ split, const int16_t* __restrict__ mv,
                   const int16_t* __restrict__ qtc, uint8_t* __restrict__ out_recon) {
    constexpr int G = BS, BPW = 256 / G, SB = BS / 2;
    constexpr int LDS_D = VBS ? 288 : BS * (BS + 1);
    __shared__ double ldsd[BPW * LDS_D];
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    const int nbx = W / BS, nb = nbx * (H / BS);
    const int b = blockIdx.x * BPW + g;
    if (b >= nb) return;
    double* dl = ldsd + g * LDS_D;
    const int bx = b % nbx, by = b / nbx, x = bx * BS, y = by * BS;
    const int qpr = qp_map ? qp_map[b] : (qp_row ? qp_row[by] : qp);
    const int16_t* m = mv + (size_t)b * 12;
    if (!VBS || !split[b]) {
        const int dx = m[0], dy = m[1], rf = m[2];
        int pred[BS], q[BS], dq[BS], rec[BS];
        if constexpr (FME) {
            fetch_row_fme<BS>(planes + (size_t)rf * 4 * pstride, pstride, W, H, 2 * x + dx, 2 * y + dy, l, 2 * BS, BS,
                              pred);
        } else {
            const bool fast = (0 <= x + dx) && (x + dx < W - BS) && (0 <= y + dy) && (y + dy < H - BS);
            fetch_row<BS>(refs.p[rf], W, H, x + dx, y + dy + l, fast, pred);
        }
        load_row_i16<BS>(qtc + (size_t)b * BS * BS + l * BS, q);
        dequant_row<BS>(q, l, qpr, dq);
        double rd[BS];
        xform2d_rows<BS, true>(dl, l, dq, rd);
#pragma unroll
        for (int c = 0; c < BS; ++c) rec[c] = pred[c] + (int)__builtin_rint(rd[c]);
        store_row_u8<BS>(out_recon, W, x, y + l, rec);
    } else if constexpr (VBS) {
        const int j = l >> 2, r0 = l & 3;
        const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
        const int sdx = m[3 * j], sdy = m[3 * j + 1], sref = m[3 * j + 2];
        const int xs = x + (j & 1) * SB, ys = y + (j >> 1) * SB;
        const bool sfast = (0 <= xs + sdx) && (xs + sdx < W - SB) && (0 <= ys + sdy) && (ys + sdy < H - SB);
        int spred[2][8], sdq[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int qv[8];
            if constexpr (FME)
                fetch_row_fme<8>(planes + (size_t)sref * 4 * pstride, pstride, W, H, 2 * xs + sdx, 2 * ys + sdy,
                                 r0 + 4 * h, BS, BS, spred[h]);
            else
                fetch_row<8>(refs.p[sref], W, H, xs + sdx, ys + sdy + r0 + 4 * h, sfast, spred[h]);
            load_row_i16<8>(qtc + (size_t)b * BS * BS + j * 64 + (r0 + 4 * h) * 8, qv);
            dequant_row<8>(qv, r0 + 4 * h, qpm1, sdq[h]);
        }
        double srd[2][8];
        xform2d_sub<true>(dl, l, sdq, srd);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int rec[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) rec[c] = spred[h][c] + (int)__builtin_rint(srd[h][c]);
            store_row_u8<8>(out_recon, W, xs, ys + r0 + 4 * h, rec);
        }
    }
}

int inter_tq_launch(const uint8_t* cur, const RefSet& refs, const uint8_t* planes, size_t pstride, int H, int W,
                    int bs, int by0, int by1, const int32_t* best, const int32_t* sub, int qp_rd, const int32_t* qp_row,
                    const int32_t* qp_map, int vbs, double lam, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens,
                    int32_t* out_mae, uint8_t* out_recon, int32_t* out_sse, hipStream_t st) {
    const int nrows = by1 - by0;
    if (nrows <= 0) return SO_OK;
    const int nb = (W / bs) * nrows;
    const int bpw = 256 / bs;
    dim3 grid((nb + bpw - 1) / bpw), blk(256);
#define SO_TQ(B, V, F)                                                                                             \
    hipLaunchKernelGGL((inter_tq_kernel<B, V, F>), grid, blk, 0, st, cur, refs, planes, pstride, H, W, by0, nrows,   \
                       best, sub, qp_rd, qp_row, qp_map, lam, out_split, out_mv, out_qtc, out_tokens, out_mae,       \
                       out_recon, out_sse, QpmArgs{})
    const bool fme = planes != nullptr;
    if (bs == 16 && vbs) { if (fme) SO_TQ(16, true, true); else SO_TQ(16, true, false); }
    else if (bs == 16) { if (fme) SO_TQ(16, false, true); else SO_TQ(16, false, false); }
    else { if (fme) SO_TQ(8, false, true); else SO_TQ(8, false, false); }
#undef SO_TQ
    return check_launch("inter_tq_kernel");
}

// Two-pass pass 2 (so_encode_p_run_2pass): inter_tq_kernel<16, false, false> with the QP map
// of the pass-1 token counts t1 computed in the kernel (one launch less per frame than
// qp_map_kernel + inter_tq_kernel; the same QPs, which it also stores into out_qpmap)
int inter_tq_2pass_launch(const uint8_t* cur, const RefSet& refs, int H, int W, const int32_t* best, const int32_t* t1,
                          int qp_rd, const int32_t* qp_row, const int32_t* roi, int qp_lo, int qp_hi,
                          int32_t* out_qpmap, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc,
                          int32_t* out_tokens, int32_t* out_mae, uint8_t* out_recon, int32_t* out_sse,
                          hipStream_t st) {
    const int nbx = W / 16, nrows = H / 16, nb = nbx * nrows;
    if (nbx < 8) {   // a workgroup's 16 blocks then span at most 3 block rows
        set_error("inter_tq_2pass_launch: W %d below 128", W);
        return SO_E_UNSUPPORTED;
    }
    hipLaunchKernelGGL((inter_tq_kernel<16, false, false, true>), dim3((nb + 15) / 16), dim3(256), 0, st, cur, refs,
                       nullptr, (size_t)0, H, W, 0, nrows, best, nullptr, qp_rd, qp_row, nullptr, 0.0, out_split,
                       out_mv, out_qtc, out_tokens, out_mae, out_recon, out_sse,
                       QpmArgs{t1, roi, qp_lo, qp_hi, out_qpmap});
    return check_launch("inter_tq_kernel");
}

int inter_recon_launch(const RefSet& refs, const uint8_t* planes, size_t pstride, int H, int W, int bs, int qp,
                       const int32_t* qp_row, const int32_t* qp_map, const uint8_t* split, const int16_t* mv, const int16_t* qtc,
                       uint8_t* out_recon, hipStream_t st) {
    const int nb = (W / bs) * (H / bs);
    const int bpw = 256 / bs;
    dim3 grid((nb + bpw - 1) / bpw), blk(256);
#define SO_REC(B, V, F)                                                                                          \
    hipLaunchKernelGGL((inter_recon_kernel<B, V, F>), grid, blk, 0, st, refs, planes, pstride, H, W, qp, qp_row, \
                       qp_map, split, mv, qtc, out_recon)
    const bool fme = planes != nullptr;
    if (bs == 16) { if (fme) SO_REC(16, true, true); else SO_REC(16, true, false); }
    else { if (fme) SO_REC(8, false, true); else SO_REC(8, false, false); }
#undef SO_REC
    return check_launch("inter_recon_kernel");
}

}  // namespace so
