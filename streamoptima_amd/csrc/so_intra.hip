// so_intra.hip — I-frame path (intra_mode 0) for gfx950.
//
// The reference's intra_prediction (Encoder.py:1238-1347) searches horizontally
// (intra_find_best_match_horizontal, :1010-1045) on an in-loop canvas into which every
// processed block writes pred + UNQUANTISED residual == the original pixels.  So, for a
// block at column x, the canvas holds the original frame left of x and 128 from x on
// (also for the four VBS sub-blocks, which are searched before the block is written):
// the search is data-parallel over all blocks.  Tie rule: mae == best and |dx| <= |best|
// replaces => the LAST-found minimum of (SAD, |dx|).  Blocks at x == 0 predict 128 with
// mv -1.  The hard-coded 288x352 canvas (:1248) is generalised to the frame size.
//
// reconstruct_frame_intra (:1350-1417) is sequential along each block row (a block copies
// from the reconstructed canvas left of it, unclipped float, final astype(uint8) wrap) but
// the rows are independent: intra_recon_rows runs one wavefront per block row over
// int32 values, the dequant/IDCT having been done for all blocks in parallel.
#include "so_block.h"

namespace so {

constexpr int kIntraMaxSr = 64;

SO_DEV uint32_t intra_key(int sad, int dx, int scan_rev) {
    return ((uint32_t)sad << 15) | ((uint32_t)(dx < 0 ? -dx : dx) << 8) | (uint32_t)scan_rev;
}

// canvas value at column col of frame row yy for a block whose column is x0
SO_DEV int canvas_at(const uint8_t* left /* LDS row: cols x0-sr .. x0-1 */, int sr, int col, int x0) {
    return col < x0 ? (int)left[col - (x0 - sr)] : 128;
}

template <int BS, bool VBS>
__global__ void __launch_bounds__(256)
intra_tq_kernel(const uint8_t* __restrict__ cur, int H, int W, int sr, int qp_rd,
                const int32_t* __restrict__ qp_row, double lam, uint8_t* __restrict__ out_split,
                int16_t* __restrict__ out_mv, int16_t* __restrict__ out_qtc,
                int32_t* __restrict__ out_tokens, int32_t* __restrict__ out_mae,
                int32_t* __restrict__ idres) {
    constexpr int G = BS, BPW = 256 / G, SB = BS / 2;
    constexpr int LDS_D = VBS ? 288 : BS * (BS + 1);
    __shared__ double ldsd[BPW * LDS_D];
    __shared__ uint8_t ldsf[BPW * BS * BS];
    __shared__ uint8_t ldsl[BPW * BS * kIntraMaxSr];
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    const int nbx = W / BS, nb = nbx * (H / BS);
    const int b = blockIdx.x * BPW + g;
    if (b >= nb) return;
    double* dl = ldsd + g * LDS_D;
    uint8_t* fl = ldsf + g * BS * BS;
    uint8_t* left = ldsl + g * BS * kIntraMaxSr;
    const int bx = b % nbx, by = b / nbx, x = bx * BS, y = by * BS;
    const int qpr = qp_row ? qp_row[by] : qp_rd;

    // stage the original pixels left of the block (cols x-sr .. x-1, 0 where < 0)
    uint8_t* lrow = left + l * kIntraMaxSr;
    for (int k = 0; k < sr; ++k) {
        const int col = x - sr + k;
        lrow[k] = col >= 0 ? cur[(size_t)(y + l) * W + col] : 0;
    }
    int crow[BS];
    load_cur_row<BS>(cur, W, x, y + l, crow);
    wave_sync();

    // ---- full-block search ----
    int mv, sad;
    if (x == 0) {
        int s = 0;
#pragma unroll
        for (int c = 0; c < BS; ++c) s += abs(crow[c] - 128);
        sad = group_sum<G>(s);
        mv = -1;
    } else {
        uint32_t bestk = 0xFFFFFFFFu;
        for (int dxi = 0; dxi <= 2 * sr; ++dxi) {
            const int dx = dxi - sr;
            if (!(x + dx >= 0 && x + dx + BS <= W)) continue;
            int s = 0;
#pragma unroll
            for (int c = 0; c < BS; ++c) s += abs(crow[c] - canvas_at(lrow, sr, x + dx + c, x));
            s = group_sum<G>(s);
            const uint32_t k = intra_key(s, dx, 2 * sr - dxi);
            bestk = k < bestk ? k : bestk;
        }
        sad = (int)(bestk >> 15);
        mv = 2 * sr - (int)(bestk & 0xFF) - sr;
    }
    int res[BS];
#pragma unroll
    for (int c = 0; c < BS; ++c) res[c] = crow[c] - (x == 0 ? 128 : canvas_at(lrow, sr, x + mv + c, x));
    double tcd[BS];
    xform2d_rows<BS, false>(dl, l, res, tcd);
    int tc[BS], q[BS];
#pragma unroll
    for (int c = 0; c < BS; ++c) tc[c] = (int)__builtin_rint(tcd[c]);
    quant_row<BS>(tc, l, qp_rd, q);

    bool split = false;
    int mae_num = sad;
    const int j = l >> 2, r0 = l & 3;
    int smv = 0, stc[2][8], qs[2][8];
    if constexpr (VBS) {
        if (x != 0 && y != 0) {
            const int xs = x + (j & 1) * SB, oy = (j >> 1) * SB;
            int scur[2][8];
#pragma unroll
            for (int h = 0; h < 2; ++h) load_cur_row<8>(cur, W, xs, y + oy + r0 + 4 * h, scur[h]);
            uint32_t bestk = 0xFFFFFFFFu;
            for (int dxi = 0; dxi <= 2 * sr; ++dxi) {
                const int dx = dxi - sr;
                if (!(xs + dx >= 0 && xs + dx + SB <= W)) continue;
                int s = 0;
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint8_t* lr = left + (oy + r0 + 4 * h) * kIntraMaxSr;
#pragma unroll
                    for (int c = 0; c < 8; ++c) s += abs(scur[h][c] - canvas_at(lr, sr, xs + dx + c, x));
                }
                s += __shfl_xor(s, 1, 64);
                s += __shfl_xor(s, 2, 64);
                const uint32_t k = intra_key(s, dx, 2 * sr - dxi);
                bestk = k < bestk ? k : bestk;
            }
            const int ssad = (int)(bestk >> 15);
            smv = 2 * sr - (int)(bestk & 0xFF) - sr;
            int sres[2][8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint8_t* lr = left + (oy + r0 + 4 * h) * kIntraMaxSr;
#pragma unroll
                for (int c = 0; c < 8; ++c) sres[h][c] = scur[h][c] - canvas_at(lr, sr, xs + smv + c, x);
            }
            double std_[2][8];
            xform2d_sub<false>(dl, l, sres, std_);
            const int qpm1_rd = qp_rd > 0 ? qp_rd - 1 : qp_rd;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
#pragma unroll
                for (int c = 0; c < 8; ++c) stc[h][c] = (int)__builtin_rint(std_[h][c]);
                quant_row<8>(stc[h], r0 + 4 * h, qpm1_rd, qs[h]);
            }
            const int tok_b = block_tokens<BS>(fl, l, q);
            const int tok_v = sub_tokens(fl, l, qs);
            // sum of the 4 sub-block SADs: one value per 4-lane sub group
            int ssum = (r0 == 0) ? ssad : 0;
            ssum = group_sum<16>(ssum);
            const double mae_b = (double)sad / 256.0;
            const double mae_v = (double)ssum / 256.0;
            const double c_v = rd_cost(lam, 32 + 8 * tok_v, mae_v);
            const double c_b = rd_cost(lam, 8 + 8 * tok_b, mae_b);
            split = !(c_b < c_v);
            mae_num = ssum;
        }
    }

    int tok;
    int32_t* rb = idres + (size_t)b * BS * BS;
    if (!split) {
        if (qpr != qp_rd) quant_row<BS>(tc, l, qpr, q);
        tok = block_tokens<BS>(fl, l, q);
        store_row_i16<BS>(out_qtc + (size_t)b * BS * BS + l * BS, q);
        int dq[BS];
        dequant_row<BS>(q, l, qpr, dq);
        double rd[BS];
        xform2d_rows<BS, true>(dl, l, dq, rd);
#pragma unroll
        for (int c = 0; c < BS; ++c) rb[l * BS + c] = (int)__builtin_rint(rd[c]);
        for (int k = l; k < 4; k += G) out_mv[(size_t)b * 4 + k] = (int16_t)(k == 0 ? mv : 0);
    } else {
        if constexpr (VBS) {
            const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
            const int qpm1_rd = qp_rd > 0 ? qp_rd - 1 : qp_rd;
            if (qpm1 != qpm1_rd)
#pragma unroll
                for (int h = 0; h < 2; ++h) quant_row<8>(stc[h], r0 + 4 * h, qpm1, qs[h]);
            tok = sub_tokens(fl, l, qs);
            int sdq[2][8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                store_row_i16<8>(out_qtc + (size_t)b * BS * BS + j * 64 + (r0 + 4 * h) * 8, qs[h]);
                dequant_row<8>(qs[h], r0 + 4 * h, qpm1, sdq[h]);
            }
            double srd[2][8];
            xform2d_sub<true>(dl, l, sdq, srd);
            // idres is row-major bs x bs for every block (intra_recon_rows indexes pixels)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
                for (int c = 0; c < 8; ++c)
                    rb[((j >> 1) * SB + r0 + 4 * h) * BS + (j & 1) * SB + c] = (int)__builtin_rint(srd[h][c]);
            if (r0 == 0) out_mv[(size_t)b * 4 + j] = (int16_t)smv;
        } else {
            tok = 0;
        }
    }
    if (l == 0) {
        out_split[b] = (uint8_t)split;
        out_tokens[b] = tok;
        out_mae[b] = mae_num;
    }
}

// rescale_QTC + apply_2d_idct of every block (decoder.py:347-365 / Encoder.py:1358-1376)
template <int BS, bool VBS>
__global__ void __launch_bounds__(256)
dequant_idct_kernel(int H, int W, int qp, const int32_t* __restrict__ qp_row,
                    const uint8_t* __restrict__ split, const int16_t* __restrict__ qtc,
                    int32_t* __restrict__ idres) {
    constexpr int G = BS, BPW = 256 / G;
    constexpr int LDS_D = VBS ? 288 : BS * (BS + 1);
    __shared__ double ldsd[BPW * LDS_D];
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    const int nbx = W / BS, nb = nbx * (H / BS);
    const int b = blockIdx.x * BPW + g;
    if (b >= nb) return;
    double* dl = ldsd + g * LDS_D;
    const int by = b / nbx;
    const int qpr = qp_row ? qp_row[by] : qp;
    int32_t* rb = idres + (size_t)b * BS * BS;
    if (!VBS || !split[b]) {
        int q[BS], dq[BS];
        load_row_i16<BS>(qtc + (size_t)b * BS * BS + l * BS, q);
        dequant_row<BS>(q, l, qpr, dq);
        double rd[BS];
        xform2d_rows<BS, true>(dl, l, dq, rd);
#pragma unroll
        for (int c = 0; c < BS; ++c) rb[l * BS + c] = (int)__builtin_rint(rd[c]);
    } else if constexpr (VBS) {
        const int j = l >> 2, r0 = l & 3;
        const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
        int sdq[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            int qv[8];
            load_row_i16<8>(qtc + (size_t)b * BS * BS + j * 64 + (r0 + 4 * h) * 8, qv);
            dequant_row<8>(qv, r0 + 4 * h, qpm1, sdq[h]);
        }
        double srd[2][8];
        xform2d_sub<true>(dl, l, sdq, srd);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int c = 0; c < 8; ++c)
                rb[((j >> 1) * 8 + r0 + 4 * h) * BS + (j & 1) * 8 + c] = (int)__builtin_rint(srd[h][c]);
    }
}

// Row-sequential intra reconstruction: one wavefront per block row.  Lane t owns
// PPL = bs*bs/64 pixels of the current block.  The canvas left of the block is kept as
// int32 (unclipped, like the reference's float canvas) in an LDS ring of the previous
// NR blocks; columns at or right of the block read 128.
template <int BS>
__global__ void __launch_bounds__(64)
intra_recon_rows_kernel(int H, int W, int sr, const uint8_t* __restrict__ split,
                        const int16_t* __restrict__ mv, const int32_t* __restrict__ idres,
                        uint8_t* __restrict__ out_recon) {
    constexpr int PPL = BS * BS / 64, SB = BS / 2;
    constexpr int NR = kIntraMaxSr / BS + 1;
    __shared__ int ring[NR][BS * BS];
    const int t = threadIdx.x;
    const int nbx = W / BS;
    const int by = blockIdx.x;
    const int y = by * BS;
    const int nring = (sr + BS - 1) / BS + 1;
    int res_next[PPL];
    {
        const int32_t* rb = idres + (size_t)(by * nbx) * BS * BS;
#pragma unroll
        for (int p = 0; p < PPL; ++p) res_next[p] = rb[t * PPL + p];
    }
    for (int bx = 0; bx < nbx; ++bx) {
        const int b = by * nbx + bx, x = bx * BS;
        int res[PPL];
#pragma unroll
        for (int p = 0; p < PPL; ++p) res[p] = res_next[p];
        if (bx + 1 < nbx) {
            const int32_t* rb = idres + (size_t)(b + 1) * BS * BS;
#pragma unroll
            for (int p = 0; p < PPL; ++p) res_next[p] = rb[t * PPL + p];
        }
        const bool sp = split[b] != 0;
        int v[PPL];
#pragma unroll
        for (int p = 0; p < PPL; ++p) {
            const int pix = t * PPL + p, i = pix / BS, c = pix % BS;
            if (x == 0) {
                v[p] = 128 + res[p];
            } else {
                const int jj = sp ? ((i >= SB) * 2 + (c >= SB)) : 0;
                const int src = x + c + mv[(size_t)b * 4 + jj];
                int base = 128;
                if (src < x) {
                    const int sbx = src / BS;
                    base = ring[sbx % nring][i * BS + (src - sbx * BS)];
                }
                v[p] = base + res[p];
            }
        }
        wave_sync();
#pragma unroll
        for (int p = 0; p < PPL; ++p) ring[bx % nring][t * PPL + p] = v[p];
        wave_sync();
        if constexpr (PPL == 4) {
            const int pix = t * 4, i = pix / BS, c = pix % BS;
            const uint32_t w = (uint32_t)(v[0] & 255) | ((uint32_t)(v[1] & 255) << 8) |
                               ((uint32_t)(v[2] & 255) << 16) | ((uint32_t)(v[3] & 255) << 24);
            *reinterpret_cast<uint32_t*>(out_recon + (size_t)(y + i) * W + x + c) = w;
        } else {
            const int pix = t, i = pix / BS, c = pix % BS;
            out_recon[(size_t)(y + i) * W + x + c] = (uint8_t)(v[0] & 255);
        }
    }
}

int intra_encode_launch(const uint8_t* cur, int H, int W, int bs, int sr, int qp_rd, const int32_t* qp_row,
                        int vbs, double lam, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc,
                        int32_t* out_tokens, int32_t* out_mae, uint8_t* out_recon, int32_t* idres,
                        hipStream_t st) {
    const int nb = (W / bs) * (H / bs);
    const int bpw = 256 / bs;
    dim3 grid((nb + bpw - 1) / bpw), blk(256);
    if (bs == 16 && vbs)
        hipLaunchKernelGGL((intra_tq_kernel<16, true>), grid, blk, 0, st, cur, H, W, sr, qp_rd, qp_row, lam,
                           out_split, out_mv, out_qtc, out_tokens, out_mae, idres);
    else if (bs == 16)
        hipLaunchKernelGGL((intra_tq_kernel<16, false>), grid, blk, 0, st, cur, H, W, sr, qp_rd, qp_row, lam,
                           out_split, out_mv, out_qtc, out_tokens, out_mae, idres);
    else
        hipLaunchKernelGGL((intra_tq_kernel<8, false>), grid, blk, 0, st, cur, H, W, sr, qp_rd, qp_row, lam,
                           out_split, out_mv, out_qtc, out_tokens, out_mae, idres);
    int rc = check_launch("intra_tq_kernel");
    if (rc) return rc;
    if (bs == 16)
        hipLaunchKernelGGL((intra_recon_rows_kernel<16>), dim3(H / bs), dim3(64), 0, st, H, W, sr, out_split,
                           out_mv, idres, out_recon);
    else
        hipLaunchKernelGGL((intra_recon_rows_kernel<8>), dim3(H / bs), dim3(64), 0, st, H, W, sr, out_split,
                           out_mv, idres, out_recon);
    return check_launch("intra_recon_rows_kernel");
}

int intra_recon_launch(int H, int W, int bs, int sr, int qp, const int32_t* qp_row, const uint8_t* split,
                       const int16_t* mv, const int16_t* qtc, uint8_t* out_recon, int32_t* idres,
                       hipStream_t st) {
    const int nb = (W / bs) * (H / bs);
    const int bpw = 256 / bs;
    dim3 grid((nb + bpw - 1) / bpw), blk(256);
    if (bs == 16)
        hipLaunchKernelGGL((dequant_idct_kernel<16, true>), grid, blk, 0, st, H, W, qp, qp_row, split, qtc, idres);
    else
        hipLaunchKernelGGL((dequant_idct_kernel<8, false>), grid, blk, 0, st, H, W, qp, qp_row, split, qtc, idres);
    int rc = check_launch("dequant_idct_kernel");
    if (rc) return rc;
    if (bs == 16)
        hipLaunchKernelGGL((intra_recon_rows_kernel<16>), dim3(H / bs), dim3(64), 0, st, H, W, sr, split, mv,
                           idres, out_recon);
    else
        hipLaunchKernelGGL((intra_recon_rows_kernel<8>), dim3(H / bs), dim3(64), 0, st, H, W, sr, split, mv,
                           idres, out_recon);
    return check_launch("intra_recon_rows_kernel");
}

}  // namespace so
