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
// from the reconstructed canvas left of it, unclipped float, final astype(uint8) wrap);
// intra_recon_kernel resolves those copy chains in parallel (pointer jumping), the
// dequant/IDCT having been done for all blocks in parallel.
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

// SRM: the search range the left-pixel LDS rows are sized for (16 for the default sr 16:
// 4 KB instead of 16 KB, three workgroups per CU instead of two)
template <int BS, bool VBS, int SRM = kIntraMaxSr>
__global__ void __launch_bounds__(256)
intra_tq_kernel(const uint8_t* __restrict__ cur, int H, int W, int by0, int nrows, int sr, int qp_rd,
                const int32_t* __restrict__ qp_row, const int32_t* __restrict__ qp_map, double lam,
                uint8_t* __restrict__ out_split,
                int16_t* __restrict__ out_mv, int16_t* __restrict__ out_qtc,
                int32_t* __restrict__ out_tokens, int32_t* __restrict__ out_mae,
                uint8_t* __restrict__ idres) {
    constexpr int G = BS, BPW = 256 / G, SB = BS / 2;
    constexpr int LDS_D = VBS ? 288 : BS * (BS + 1);
    __shared__ double ldsd[BPW * LDS_D];
    __shared__ uint8_t ldsf[VBS ? BPW * BS * BS : 1];   // sub_tokens' flags (block_tokens: registers only)
    __shared__ uint8_t ldsl[BPW * BS * SRM];
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    const int nbx = W / BS, nb = nbx * nrows;
    const int b = blockIdx.x * BPW + g;   // block index inside the stripe [by0, by0 + nrows)
    if (b >= nb) return;
    double* dl = ldsd + g * LDS_D;
    uint8_t* fl = ldsf + g * BS * BS;
    uint8_t* left = ldsl + g * BS * SRM;
    const int bx = b % nbx, by = by0 + b / nbx, x = bx * BS, y = by * BS;
    const int qpr = qp_map ? qp_map[(size_t)by * nbx + bx] : (qp_row ? qp_row[by] : qp_rd);

    // stage the original pixels left of the block (cols x-sr .. x-1, 0 where < 0)
    uint8_t* lrow = left + l * SRM;
    if (BS == 16 && sr == 16 && x != 0) {
        // x >= 16: one aligned 16-byte row load and one ds_write_b128
        *reinterpret_cast<uint4*>(lrow) = *reinterpret_cast<const uint4*>(cur + (size_t)(y + l) * W + x - 16);
    } else {
        for (int k = 0; k < sr; ++k) {
            const int col = x - sr + k;
            lrow[k] = col >= 0 ? cur[(size_t)(y + l) * W + col] : 0;
        }
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
    } else if (BS == 16 && sr == 16) {
        // Fast path.  A candidate dx > 0 reads only 128s (the canvas from x on), so its
        // SAD equals dx = 0's and the |dx| tie rule always prefers dx = 0: only
        // dx in [-16, 0] can win, and there (SAD, |dx|) is unique.  Canvas row bytes
        // [x-16, x+16) = 4 original words + 4 words of 0x80; candidate words are funnel
        // shifts of that array at compile-time offsets; v_sad_u8 per word.
        const uint8_t* rp = cur + (size_t)(y + l) * W + x;
        const uint4 lv = *reinterpret_cast<const uint4*>(rp - 16), cv = *reinterpret_cast<const uint4*>(rp);
        const uint32_t Z[9] = {lv.x, lv.y, lv.z, lv.w, 0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u,
                               0x80808080u};
        const uint32_t C[4] = {cv.x, cv.y, cv.z, cv.w};
        uint32_t bestk = 0xFFFFFFFFu;
#pragma unroll
        for (int dx = -16; dx <= 0; ++dx) {
            const int off = 16 + dx, d = off >> 2, sh = off & 3;
            uint32_t srow = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k)
                srow = __builtin_amdgcn_sad_u8(C[k], __builtin_amdgcn_alignbyte(Z[d + k + 1], Z[d + k], sh), srow);
            const int sfull = group_sum<G>((int)srow);
            const uint32_t key = ((uint32_t)sfull << 8) | (uint32_t)(-dx);
            bestk = key < bestk ? key : bestk;
        }
        sad = (int)(bestk >> 8);
        mv = -(int)(bestk & 0xFF);
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
    quant_row_i<BS>(tc, l, qp_rd, q);   // FP64 carriers, branch-free (so_block.h)

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
            int ssad;
            if (sr == 16) {
                // fast path, as for the full block: only dx in [-16, 0] can win
                uint32_t Zs[2][9], Cs[2][2];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const uint8_t* rp = cur + (size_t)(y + oy + r0 + 4 * h) * W + x;
                    const uint4 lv = *reinterpret_cast<const uint4*>(rp - 16);
                    const uint2 cv = *reinterpret_cast<const uint2*>(rp + (j & 1) * 8);
                    Zs[h][0] = lv.x; Zs[h][1] = lv.y; Zs[h][2] = lv.z; Zs[h][3] = lv.w;
                    Zs[h][4] = Zs[h][5] = Zs[h][6] = Zs[h][7] = Zs[h][8] = 0x80808080u;
                    Cs[h][0] = cv.x; Cs[h][1] = cv.y;
                }
                const int base = 16 + (j & 1) * 8;   // canvas byte of column xs relative to x-16
                uint32_t bestk = 0xFFFFFFFFu;
#pragma unroll
                for (int dx = -16; dx <= 0; ++dx) {
                    const int off = base + dx;        // 0 .. 24, depends on j (wave-divergent)
                    const int d = off >> 2, sh = off & 3;
                    uint32_t srow = 0;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        // runtime word index (j differs across lanes): select from registers
                        uint32_t w0 = Zs[h][0], w1 = Zs[h][1], w2 = Zs[h][2];
#pragma unroll
                        for (int q = 1; q <= 6; ++q)
                            if (d == q) { w0 = Zs[h][q]; w1 = Zs[h][q + 1]; w2 = Zs[h][q + 2]; }
                        srow = __builtin_amdgcn_sad_u8(Cs[h][0], __builtin_amdgcn_alignbyte(w1, w0, sh), srow);
                        srow = __builtin_amdgcn_sad_u8(Cs[h][1], __builtin_amdgcn_alignbyte(w2, w1, sh), srow);
                    }
                    int s4 = (int)srow;
                    s4 += __shfl_xor(s4, 1, 64);
                    s4 += __shfl_xor(s4, 2, 64);
                    const uint32_t key = ((uint32_t)s4 << 8) | (uint32_t)(-dx);
                    bestk = key < bestk ? key : bestk;
                }
                ssad = (int)(bestk >> 8);
                smv = -(int)(bestk & 0xFF);
            } else {
                uint32_t bestk = 0xFFFFFFFFu;
                for (int dxi = 0; dxi <= 2 * sr; ++dxi) {
                    const int dx = dxi - sr;
                    if (!(xs + dx >= 0 && xs + dx + SB <= W)) continue;
                    int s = 0;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const uint8_t* lr = left + (oy + r0 + 4 * h) * SRM;
#pragma unroll
                        for (int c = 0; c < 8; ++c) s += abs(scur[h][c] - canvas_at(lr, sr, xs + dx + c, x));
                    }
                    s += __shfl_xor(s, 1, 64);
                    s += __shfl_xor(s, 2, 64);
                    const uint32_t k = intra_key(s, dx, 2 * sr - dxi);
                    bestk = k < bestk ? k : bestk;
                }
                ssad = (int)(bestk >> 15);
                smv = 2 * sr - (int)(bestk & 0xFF) - sr;
            }
            int sres[2][8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const uint8_t* lr = left + (oy + r0 + 4 * h) * SRM;
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
    uint8_t* rb = idres + (size_t)b * BS * BS;
    if (!split) {
        if (qpr != qp_rd) quant_row_i<BS>(tc, l, qpr, q);
        tok = block_tokens<BS>(fl, l, q);
        store_row_i16<BS>(out_qtc + (size_t)b * BS * BS + l * BS, q);
        int dq[BS];
        dequant_row_int<BS>(q, l, qpr, dq);
        double rd[BS];
        xform2d_rows<BS, true>(dl, l, dq, rd);
        // residuals mod 256 (the reconstruction wraps to uint8: only the low byte matters)
        int rr[BS];
#pragma unroll
        for (int c = 0; c < BS; ++c) rr[c] = (int)__builtin_rint(rd[c]);
        store_row_u8<BS>(rb, BS, 0, l, rr);
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
            // idres is row-major bs x bs for every block (intra_recon_kernel indexes pixels)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int rr[SB];
#pragma unroll
                for (int c = 0; c < SB; ++c) rr[c] = (int)__builtin_rint(srd[h][c]);
                store_row_u8<SB>(rb, BS, (j & 1) * SB, (j >> 1) * SB + r0 + 4 * h, rr);
            }
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
dequant_idct_kernel(int H, int W, int qp, const int32_t* __restrict__ qp_row, const int32_t* __restrict__ qp_map,
                    const uint8_t* __restrict__ split, const int16_t* __restrict__ qtc,
                    uint8_t* __restrict__ idres) {
    constexpr int G = BS, BPW = 256 / G;
    constexpr int LDS_D = VBS ? 288 : BS * (BS + 1);
    __shared__ double ldsd[BPW * LDS_D];
    const int tid = threadIdx.x, g = tid / G, l = tid % G;
    const int nbx = W / BS, nb = nbx * (H / BS);
    const int b = blockIdx.x * BPW + g;
    if (b >= nb) return;
    double* dl = ldsd + g * LDS_D;
    const int by = b / nbx;
    const int qpr = qp_map ? qp_map[b] : (qp_row ? qp_row[by] : qp);
    uint8_t* rb = idres + (size_t)b * BS * BS;
    if (!VBS || !split[b]) {
        int q[BS], dq[BS];
        load_row_i16<BS>(qtc + (size_t)b * BS * BS + l * BS, q);
        dequant_row<BS>(q, l, qpr, dq);
        double rd[BS];
        xform2d_rows<BS, true>(dl, l, dq, rd);
        int rr[BS];   // mod 256, as intra_tq_kernel
#pragma unroll
        for (int c = 0; c < BS; ++c) rr[c] = (int)__builtin_rint(rd[c]);
        store_row_u8<BS>(rb, BS, 0, l, rr);
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
        for (int h = 0; h < 2; ++h) {
            int rr[8];
#pragma unroll
            for (int c = 0; c < 8; ++c) rr[c] = (int)__builtin_rint(srd[h][c]);
            store_row_u8<8>(rb, BS, (j & 1) * 8, (j >> 1) * 8 + r0 + 4 * h, rr);
        }
    }
}

// Intra reconstruction (reconstruct_frame_intra, Encoder.py:1350-1417 / decoder.py:367-432):
// every pixel of a block copies the canvas at column src = x + c + mv (same pixel row)
// and adds its IDCT residual; the canvas is the reconstruction where src < x and 128
// where src >= x; blocks at x == 0 use 128.  So pixel p's value is
//     128 + res[p] + res[src(p)] + res[src(src(p))] + ...   (until a source is >= its x)
// a chain that only moves left inside one pixel row.  One workgroup per pixel row
// resolves all chains by pointer jumping (log2(#blocks) rounds) in LDS: the sequential
// block-by-block dependency of the reference costs no serial latency here.
template <int BS>
__global__ void __launch_bounds__(256)
intra_recon_kernel(int H, int W, int by0, const uint8_t* __restrict__ split, const int16_t* __restrict__ mv,
                   const uint8_t* __restrict__ idres, const uint8_t* __restrict__ cur,
                   uint8_t* __restrict__ out_recon, int32_t* __restrict__ out_sse) {
    constexpr int SB = BS / 2, NT = 256;
    extern __shared__ __attribute__((aligned(16))) unsigned char dyn[];   // 12 * W bytes
    int* sval[2] = {reinterpret_cast<int*>(dyn), reinterpret_cast<int*>(dyn) + W};
    short* snxt[2] = {reinterpret_cast<short*>(dyn + 8 * (size_t)W), reinterpret_cast<short*>(dyn + 8 * (size_t)W) + W};
    __shared__ int ssum[NT / 64];
    // pixel row yl of the stripe starting at block row by0; symbols are stripe-local
    const int yl = blockIdx.x, yy = by0 * BS + yl, tid = threadIdx.x;
    const int byl = yl / BS, i = yl - byl * BS, nbx = W / BS;
    for (int p = tid; p < W; p += NT) {
        const int bx = p / BS, c = p - bx * BS, x = bx * BS, b = byl * nbx + bx;
        const int res = idres[(size_t)b * BS * BS + i * BS + c];
        int nx = -1;
        if (x != 0) {
            const int jj = split[b] ? ((i >= SB) * 2 + (c >= SB)) : 0;
            const int src = x + c + mv[(size_t)b * 4 + jj];
            nx = src < x ? src : -1;
        }
        sval[0][p] = res;
        snxt[0][p] = (short)nx;
    }
    __syncthreads();
    int cb = 0;
    // chain length <= number of blocks in the row; every hop moves >= 1 block left
    for (int span = 1; span < nbx; span <<= 1) {
        for (int p = tid; p < W; p += NT) {
            const int nx = snxt[cb][p];
            int v = sval[cb][p], n2 = nx;
            if (nx >= 0) {
                v += sval[cb][nx];
                n2 = snxt[cb][nx];
            }
            sval[cb ^ 1][p] = v;
            snxt[cb ^ 1][p] = (short)n2;
        }
        __syncthreads();
        cb ^= 1;
    }
    int sse = 0;
    for (int p = tid; p < W; p += NT) {
        const int v = (128 + sval[cb][p]) & 255;
        out_recon[(size_t)yy * W + p] = (uint8_t)v;
        if (out_sse) {
            const int d = (int)cur[(size_t)yy * W + p] - v;
            sse += d * d;
        }
    }
    if (out_sse) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) sse += __shfl_xor(sse, m, 64);
        if ((tid & 63) == 0) ssum[tid >> 6] = sse;
        __syncthreads();
        if (tid == 0) out_sse[yl] = ssum[0] + ssum[1] + ssum[2] + ssum[3];
    }
}

// Sequential form of the same recurrence (default): value(p) = res(p) + (src(p) < x ?
// value(src(p)) : 128), and src(p) >= x - sr, so walking a pixel row block by block left to
// right needs only the last sr pixels.  BS lanes own one row (lane = column c of the
// current block), a wave walks 64/BS rows side by side; a 128-entry LDS ring per row holds
// the values already produced (sr <= 64, so x - src <= 64 + BS - 1 < 128 never aliases the
// block being written).  nbx dependent steps of one LDS round trip each, instead of the
// pointer-jumping kernel's log2(nbx) passes over the whole row with a barrier each.
template <int BS, bool NEAR>
__global__ void __launch_bounds__(256)
intra_recon_seq_kernel(int W, int nrows_px, int by0, const uint8_t* __restrict__ split, const int16_t* __restrict__ mv,
                       const uint8_t* __restrict__ idres, const uint8_t* __restrict__ cur,
                       uint8_t* __restrict__ out_recon, int32_t* __restrict__ out_sse) {
    constexpr int SB = BS / 2, RPW = 64 / BS, RING = 128;
    __shared__ int ring[4 * RPW][RING];
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int g = lane / BS, c = lane - g * BS;            // row group, column within the block
    const int yl = (blockIdx.x * (blockDim.x >> 6) + wv) * RPW + g;   // stripe-local pixel row
    const bool act = yl < nrows_px;
    const int ylc = act ? yl : nrows_px - 1;
    const int yy = by0 * BS + ylc, byl = ylc / BS, i = ylc - byl * BS, nbx = W / BS;
    int* rg = ring[wv * RPW + g];
    const bool right = c >= SB, lower = i >= SB;
    int sse = 0;
    const uint8_t* crow = cur ? cur + (size_t)yy * W : nullptr;
    uint8_t* orow = out_recon + (size_t)yy * W;
    // the residuals and motion vectors of the next CH blocks are loaded while the current
    // CH blocks walk the chain (their loads do not depend on it)
#ifndef SO_IRS_CH   // blocks whose inputs are loaded one group ahead: the load latency is
#define SO_IRS_CH 32   // hidden behind 32 chain steps (4K I-frame 102 -> 95 us vs 8, tools/intra_ab.py)
#endif
    constexpr int CH = SO_IRS_CH;
    int resn[CH], dxn[CH], curn[CH];
    auto fetch = [&](int bx0, int (&rs)[CH], int (&dv)[CH], int (&cv)[CH]) {
#pragma unroll
        for (int s = 0; s < CH; ++s) {
            const int bx = bx0 + s < nbx ? bx0 + s : nbx - 1;
            const int b = byl * nbx + bx;
            rs[s] = idres[(size_t)b * BS * BS + i * BS + c];
            cv[s] = crow ? (int)crow[bx * BS + c] : 0;
            const uint2 m4 = *reinterpret_cast<const uint2*>(mv + (size_t)b * 4);
            const int jj = split[b] ? (lower * 2 + right) : 0;
            const uint32_t w = jj < 2 ? m4.x : m4.y;
            dv[s] = (int)(int16_t)((jj & 1) ? (w >> 16) : (w & 0xFFFF));
        }
    };
    fetch(0, resn, dxn, curn);
    volatile int* vr = rg;   // one wave: LDS ops retire in order; volatile keeps their order
    int pv = 0;              // NEAR: this lane's value in the previous block
    (void)vr;
    for (int bx0 = 0; bx0 < nbx; bx0 += CH) {
        int resc[CH], dxc[CH], curc[CH];
#pragma unroll
        for (int s = 0; s < CH; ++s) { resc[s] = resn[s]; dxc[s] = dxn[s]; curc[s] = curn[s]; }
        if (bx0 + CH < nbx) fetch(bx0 + CH, resn, dxn, curn);
        if constexpr (NEAR) {
            // sr <= BS: every source is in the previous block, whose values the group's lanes
            // still hold.  Only the ds_bpermute and two adds stay on the serial chain: the
            // permute address (bit 0 = "no left source": 128 instead) and res + 128 are set up
            // for the whole group first, the stores and the SSE come after it.
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                const int x = (bx0 + s) * BS, rel = c + dxc[s];
                const bool use = x != 0 && rel < 0;
                dxc[s] = (((lane & ~(BS - 1)) + ((rel + BS) & (BS - 1))) << 2) | (use ? 0 : 1);
                resc[s] += use ? 0 : 128;
            }
#pragma unroll
            for (int s = 0; s < CH; ++s) {   // past nbx: clamped inputs, values never stored
                const int pvv = __builtin_amdgcn_ds_bpermute(dxc[s], pv);
                pv = (pvv & ((dxc[s] & 1) - 1)) + resc[s];
                resc[s] = pv;
            }
#pragma unroll
            for (int s = 0; s < CH; ++s) {
                const int x = (bx0 + s) * BS;
                if (bx0 + s < nbx && act) {
                    const int o = resc[s] & 255;
                    orow[x + c] = (uint8_t)o;
                    const int d = curc[s] - o;
                    sse += d * d;
                }
            }
            continue;
        }
#pragma unroll
        for (int s = 0; s < CH; ++s) {
            const int bx = bx0 + s;
            if (bx < nbx) {                                    // wave-uniform
                const int x = bx * BS;
                int v = resc[s] + 128;
                const int src = x + c + dxc[s];
                if (x != 0 && src < x) v = resc[s] + vr[src & (RING - 1)];
                vr[(x + c) & (RING - 1)] = v;
                const int o = v & 255;
                if (act) {
                    orow[x + c] = (uint8_t)o;
                    const int d = curc[s] - o;
                    sse += d * d;
                }
            }
        }
    }
    if (out_sse) {
#pragma unroll
        for (int m = BS / 2; m >= 1; m >>= 1) sse += __shfl_xor(sse, m, 64);
        if (act && c == 0) out_sse[yl] = sse;
    }
}

// The same recurrence for sr <= BS as a chunked scan: WPR waves per pixel row, the row's nbx
// blocks in K = 64 WPR / BS chunks of L blocks, chunk k on threads [k BS, (k + 1) BS).  Block j
// maps the previous block's values to its own, v_j[c] = res_j[c] + (use_j[c] ?
// v_{j-1}[src_j(c)] : 128), and such maps compose: over a chunk, v[c] = A[c] + (S[c] ?
// e[S[c] - 1] : 0) with e the values entering the chunk (A mod 256 in bits 0-7, S in bits 8-12
// of a 16-bit word).
//   0. thread = block (64 WPR blocks per pass, one row load of each): every pixel's
//      (res, use, src) packed into the LDS slot of (block, column);
//   1. each chunk composes its blocks' maps left to right, one ds_bpermute per block, and
//      leaves the prefix map after every block in its slot;
//   2. the chunk maps composed over each wave's chunks (GPW - 1 ds_bpermute steps), then the
//      waves' end values in order through LDS (WPR - 1 barriers): the values leaving every chunk;
//   3. every block applies its prefix map to the values entering its chunk (independent),
//      into an LDS copy of the pixel row;
//   4. the row out in 16-byte stores, its SSE from 16-byte loads of the current row.
// L + GPW + WPR dependent steps instead of nbx (4K, WPR 2: 30 + 4 + 2 instead of 240);
// arithmetic mod 256 as above.
template <int BS, int WPR>
__global__ void __launch_bounds__(64 * WPR)
intra_recon_scan_kernel(int W, int nrows_px, int by0, const uint8_t* __restrict__ split, const int16_t* __restrict__ mv,
                        const uint8_t* __restrict__ idres, const uint8_t* __restrict__ cur,
                        uint8_t* __restrict__ out_recon, int32_t* __restrict__ out_sse) {
    constexpr int NT = 64 * WPR, K = NT / BS, GPW = 64 / BS, SB = BS / 2, ND = BS / 4, TU = 4, U3 = 4;
    extern __shared__ __attribute__((aligned(16))) uint16_t slot[];   // [L][NT], ev[NT], the pixel row
    __shared__ int ssum[WPR];
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const int k = tid / BS, c = tid - k * BS, g = k - wv * GPW;
    // workgroup -> pixel row so that the BS rows of a block row share an XCD (workgroups are
    // dealt round-robin over the 8 XCDs): each row reads BS bytes of every block's residual,
    // and its neighbours' reads of the same lines then hit that XCD's L2 (one row per XCD in
    // turn read every block's lines from memory 8 times over: 85 MB per 4K I-frame vs ~25)
    const int xcd = blockIdx.x & 7, kx = blockIdx.x >> 3;
    const int yl = (((kx / BS) << 3) + xcd) * BS + kx % BS;
    if (yl >= nrows_px) return;   // uniform: the grid is rounded up to 8 block rows
    const int yy = by0 * BS + yl, byl = yl / BS, i = yl - byl * BS, nbx = W / BS;
    const int L = (nbx + K - 1) / K, j0 = k * L;
    const bool lower = i >= SB;
    uint32_t* const ev = reinterpret_cast<uint32_t*>(slot + (size_t)L * NT);
    uint8_t* const rowb = reinterpret_cast<uint8_t*>(ev + NT);
    // ---- 0. inputs, a block per thread ------------------------------------------------------
    for (int t0 = 0; t0 * NT < nbx; t0 += TU) {
        uint32_t rw[TU][ND], mw[TU][2], sp[TU];
#pragma unroll
        for (int t = 0; t < TU; ++t) {
            int jb = (t0 + t) * NT + tid;
            jb = jb < nbx ? jb : nbx - 1;
            const size_t b = (size_t)byl * nbx + jb;
            const uint32_t* rp = reinterpret_cast<const uint32_t*>(idres + b * BS * BS + i * BS);
#pragma unroll
            for (int d = 0; d < ND; ++d) rw[t][d] = rp[d];
            const uint2 m4 = *reinterpret_cast<const uint2*>(mv + b * 4);
            mw[t][0] = m4.x;
            mw[t][1] = m4.y;
            sp[t] = split[b];
        }
#pragma unroll
        for (int t = 0; t < TU; ++t) {
            const int jb = (t0 + t) * NT + tid;
            if (jb < nbx) {
                // dx of the left / right half of this pixel row (the block's, or its sub-blocks')
                const uint32_t wlr = (sp[t] && lower) ? mw[t][1] : mw[t][0];
                const int dxl = (int)(int16_t)(wlr & 0xFFFF);
                const int dxr = sp[t] ? (int)(int16_t)(wlr >> 16) : dxl;
                const int kq = jb / L, s = jb - kq * L;
                uint32_t pk[BS / 2];
#pragma unroll
                for (int cc = 0; cc < BS; ++cc) {
                    const int rel = cc + (cc >= SB ? dxr : dxl);
                    const bool use = jb != 0 && rel < 0;
                    const uint32_t v = ((rw[t][cc >> 2] >> (8 * (cc & 3))) & 255u) | (use ? 256u : 0u) |
                                       ((uint32_t)((rel + BS) & (BS - 1)) << 9);
                    pk[cc >> 1] = (cc & 1) ? (pk[cc >> 1] | (v << 16)) : v;
                }
                uint4* dst = reinterpret_cast<uint4*>(slot + (size_t)s * NT + kq * BS);
#pragma unroll
                for (int q = 0; q < BS / 8; ++q) dst[q] = make_uint4(pk[4 * q], pk[4 * q + 1], pk[4 * q + 2], pk[4 * q + 3]);
            }
        }
    }
    __syncthreads();
    // ---- 1. prefix maps per chunk ------------------------------------------------------------
    const int gbase = lane & ~(BS - 1);
    const int nvalid = nbx - j0 < L ? (nbx - j0 > 0 ? nbx - j0 : 0) : L;
    uint32_t w = (uint32_t)(c + 1) << 8;   // identity: A = 0, S = c + 1
    uint32_t in = slot[tid];
    for (int s = 0; s < nvalid; ++s) {
        const uint32_t cin = in;
        if (s + 1 < nvalid) in = slot[(s + 1) * NT + tid];
        const uint32_t gv = (uint32_t)__builtin_amdgcn_ds_bpermute((gbase + (int)(cin >> 9)) << 2, (int)w);
        const bool use = (cin & 256u) != 0u;
        w = ((cin + (use ? gv : 128u)) & 255u) | (use ? (gv & 0x1F00u) : 0u);
        slot[s * NT + tid] = (uint16_t)w;
    }
    // ---- 2. values leaving each chunk ----------------------------------------------------------
    // the chunk maps composed over the wave's groups: P maps the values entering the wave's
    // first chunk to those leaving this one
    uint32_t P = w;
#pragma unroll
    for (int gg = 1; gg < GPW; ++gg) {
        const uint32_t si = (w >> 8) & 31u;
        const uint32_t pg = (uint32_t)__builtin_amdgcn_ds_bpermute(((gg - 1) * BS + (int)(si ? si - 1 : 0)) << 2, (int)P);
        if (g == gg) P = ((w + (si ? pg : 0u)) & 255u) | (si ? (pg & 0x1F00u) : 0u);
    }
    // wave 0 starts at block 0, where nothing has a source: its P are constants; wave ww takes
    // the values leaving wave ww-1's last chunk
#pragma unroll
    for (int ww = 0; ww < WPR; ++ww) {
        if (wv == ww) {
            const uint32_t si = (P >> 8) & 31u;
            const uint32_t e = (ww > 0 && si) ? ev[(ww * GPW - 1) * BS + si - 1] : 0u;
            ev[tid] = (P + e) & 255u;
        }
        __syncthreads();
    }
    // ---- 3. every pixel, into the LDS row ------------------------------------------------------
    const uint32_t* const ein = ev + (k > 0 ? k - 1 : 0) * BS - 1;
    for (int s0 = 0; s0 < nvalid; s0 += U3) {
        uint32_t m[U3];
#pragma unroll
        for (int u = 0; u < U3; ++u) m[u] = s0 + u < nvalid ? slot[(s0 + u) * NT + tid] : 0u;
#pragma unroll
        for (int u = 0; u < U3; ++u) {
            const uint32_t si = (m[u] >> 8) & 31u;
            const uint32_t e = si ? ein[si] : 0u;
            if (s0 + u < nvalid) rowb[(j0 + s0 + u) * BS + c] = (uint8_t)((m[u] + e) & 255u);
        }
    }
    __syncthreads();
    // ---- 4. the row out, its SSE ----------------------------------------------------------------
    const uint8_t* crow = cur ? cur + (size_t)yy * W : nullptr;
    uint8_t* orow = out_recon + (size_t)yy * W;
    int sse = 0;
    for (int x0 = tid * 16; x0 < W; x0 += NT * 16) {
        const uint4 r = *reinterpret_cast<const uint4*>(rowb + x0);
        *reinterpret_cast<uint4*>(orow + x0) = r;
        if (crow) {
            const uint4 q = *reinterpret_cast<const uint4*>(crow + x0);
            const uint32_t rr[4] = {r.x, r.y, r.z, r.w}, qq[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
            for (int d = 0; d < 4; ++d)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int df = (int)((qq[d] >> (8 * e)) & 255u) - (int)((rr[d] >> (8 * e)) & 255u);
                    sse += df * df;
                }
        }
    }
    if (out_sse) {
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) sse += __shfl_xor(sse, m, 64);
        if (lane == 0) ssum[wv] = sse;
        __syncthreads();
        if (tid == 0) {
            int t = 0;
#pragma unroll
            for (int ww = 0; ww < WPR; ++ww) t += ssum[ww];
            out_sse[yl] = t;
        }
    }
}

// rows [0, nrows_px) of the stripe starting at block row by0: sequential kernel for sr <= 64
static int intra_recon_rows(int W, int bs, int sr, int by0, int nrows_px, const uint8_t* split, const int16_t* mv,
                            const uint8_t* idres, const uint8_t* cur, uint8_t* out_recon, int32_t* out_sse, int H,
                            hipStream_t st) {
    if (nrows_px <= 0) return SO_OK;
#ifndef SO_IRS_SEQ   // A/B builds: the sequential walk for sr <= bs too
    // 16-byte row loads / stores of cur and out_recon: W % 16 == 0 and 16-byte aligned planes
    // (the C-ABI takes any plane pointer; a misaligned one takes the sequential walk)
    const bool a16 = ((reinterpret_cast<uintptr_t>(cur) | reinterpret_cast<uintptr_t>(out_recon)) & 15) == 0;
    if (sr <= bs && W % 16 == 0 && a16) {
#ifndef SO_IRS_WPR   // waves per pixel row of the scan
#define SO_IRS_WPR 4
#endif
        constexpr int WPR = SO_IRS_WPR, NT = 64 * WPR;
        const int k = NT / bs, nbx = W / bs, L = (nbx + k - 1) / k;
        const size_t lds = (size_t)L * NT * sizeof(uint16_t) + NT * sizeof(uint32_t) + (size_t)W;
        const int nbr = (nrows_px + bs - 1) / bs, grid = (nbr + 7) / 8 * 8 * bs;   // whole groups of 8 block rows
        if (bs == 16)
            hipLaunchKernelGGL((intra_recon_scan_kernel<16, WPR>), dim3(grid), dim3(NT), lds, st, W, nrows_px, by0,
                               split, mv, idres, cur, out_recon, out_sse);
        else
            hipLaunchKernelGGL((intra_recon_scan_kernel<8, WPR>), dim3(grid), dim3(NT), lds, st, W, nrows_px, by0,
                               split, mv, idres, cur, out_recon, out_sse);
        return check_launch("intra_recon_scan_kernel");
    }
#endif
    if (sr <= 64) {
        // SO_IRS_WPB waves per workgroup (the kernel is a latency chain per wave; 1 spreads
        // the 4K I-frame's 540 waves over all 256 CUs instead of 135)
#ifndef SO_IRS_WPB
#define SO_IRS_WPB 1
#endif
        const int rows_per_blk = SO_IRS_WPB * (64 / bs);
        const dim3 grid((nrows_px + rows_per_blk - 1) / rows_per_blk);
#define SO_IRS(B, N)                                                                                              \
    hipLaunchKernelGGL((intra_recon_seq_kernel<B, N>), grid, dim3(64 * SO_IRS_WPB), 0, st, W, nrows_px, by0, split, \
                       mv, idres, cur, out_recon, out_sse)
        if (bs == 16) { if (sr <= 16) SO_IRS(16, true); else SO_IRS(16, false); }
        else { if (sr <= 8) SO_IRS(8, true); else SO_IRS(8, false); }
#undef SO_IRS
        return check_launch("intra_recon_seq_kernel");
    }
    if (bs == 16)
        hipLaunchKernelGGL((intra_recon_kernel<16>), dim3(nrows_px), dim3(256), 12 * (size_t)W, st, H, W, by0, split,
                           mv, idres, cur, out_recon, out_sse);
    else
        hipLaunchKernelGGL((intra_recon_kernel<8>), dim3(nrows_px), dim3(256), 12 * (size_t)W, st, H, W, by0, split,
                           mv, idres, cur, out_recon, out_sse);
    return check_launch("intra_recon_kernel");
}

int intra_encode_launch(const uint8_t* cur, int H, int W, int bs, int sr, int by0, int by1, int qp_rd,
                        const int32_t* qp_row, const int32_t* qp_map, int vbs, double lam, uint8_t* out_split, int16_t* out_mv,
                        int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae, uint8_t* out_recon,
                        int32_t* out_sse, uint8_t* idres, hipStream_t st) {
    const int nrows = by1 - by0;
    if (nrows <= 0) return SO_OK;
    const int nb = (W / bs) * nrows;
    const int bpw = 256 / bs;
    dim3 grid((nb + bpw - 1) / bpw), blk(256);
    if (bs == 16 && vbs)
        hipLaunchKernelGGL((intra_tq_kernel<16, true>), grid, blk, 0, st, cur, H, W, by0, nrows, sr, qp_rd, qp_row, qp_map,
                           lam,
                           out_split, out_mv, out_qtc, out_tokens, out_mae, idres);
    else if (bs == 16 && sr <= 16)
        hipLaunchKernelGGL((intra_tq_kernel<16, false, 16>), grid, blk, 0, st, cur, H, W, by0, nrows, sr, qp_rd, qp_row,
                           qp_map, lam, out_split, out_mv, out_qtc, out_tokens, out_mae, idres);
    else if (bs == 16)
        hipLaunchKernelGGL((intra_tq_kernel<16, false>), grid, blk, 0, st, cur, H, W, by0, nrows, sr, qp_rd, qp_row, qp_map,
                           lam,
                           out_split, out_mv, out_qtc, out_tokens, out_mae, idres);
    else
        hipLaunchKernelGGL((intra_tq_kernel<8, false>), grid, blk, 0, st, cur, H, W, by0, nrows, sr, qp_rd, qp_row, qp_map,
                           lam,
                           out_split, out_mv, out_qtc, out_tokens, out_mae, idres);
    int rc = check_launch("intra_tq_kernel");
    if (rc) return rc;
    return intra_recon_rows(W, bs, sr, by0, nrows * bs, out_split, out_mv, idres, cur, out_recon, out_sse, H, st);
}

int intra_recon_launch(int H, int W, int bs, int sr, int qp, const int32_t* qp_row, const int32_t* qp_map,
                       const uint8_t* split,
                       const int16_t* mv, const int16_t* qtc, uint8_t* out_recon, uint8_t* idres,
                       hipStream_t st) {
    const int nb = (W / bs) * (H / bs);
    const int bpw = 256 / bs;
    dim3 grid((nb + bpw - 1) / bpw), blk(256);
    if (bs == 16)
        hipLaunchKernelGGL((dequant_idct_kernel<16, true>), grid, blk, 0, st, H, W, qp, qp_row, qp_map, split, qtc,
                           idres);
    else
        hipLaunchKernelGGL((dequant_idct_kernel<8, false>), grid, blk, 0, st, H, W, qp, qp_row, qp_map, split, qtc,
                           idres);
    int rc = check_launch("dequant_idct_kernel");
    if (rc) return rc;
    return intra_recon_rows(W, bs, sr, 0, H, split, mv, idres, nullptr, out_recon, nullptr, H, st);
}

}  // namespace so
