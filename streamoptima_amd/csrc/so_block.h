// so_block.h — per-block transform pipeline shared by the P-frame, I-frame and decoder
// kernels.  One block is owned by a group of G lanes inside one wavefront (G = 16 for
// 16x16 blocks, 8 for 8x8), so all cross-lane exchange stays inside the wave: LDS
// transposes ordered by wavefront-scope fences, reductions by __shfl_xor.
//
// Lane l of a 16x16 group owns block row l:   residual row -> LDS -> column l -> DCT-II
// -> LDS -> row l -> DCT-II -> rint (apply_2d_dct, Encoder.py:779-784) -> quantise
// (quantize_TC :787) -> token count (entropy_encoder_block :1086 length) ...
// For VBS the same 16 lanes run the four 8x8 sub-blocks: lane l owns sub-block
// j = l >> 2, rows/cols (l & 3) and (l & 3) + 4.
#pragma once
#include "so_common.h"
#include "so_dct.h"

namespace so {

SO_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// scan position of (i, j) in the anti-diagonal order of entropy_encoder_block
SO_DEV int scan_index(int n, int i, int j) {
    const int k = i + j;
    const int before = (k < n) ? (k * (k + 1)) / 2 : n * n - ((2 * n - 1 - k) * (2 * n - k)) / 2;
    const int first_i = (k < n) ? 0 : k - n + 1;
    return before + (i - first_i);
}

template <int G>
SO_DEV int group_sum(int v) {
#pragma unroll
    for (int m = G / 2; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    return v;
}

// ---- byte row fetch ----------------------------------------------------------------------
// NB bytes of frame row `py` starting at column px.  `fast` == the reference's strict
// in-bounds test held (0 <= px < W-bs, 0 <= py0 < H-bs), so the 4-byte-aligned words
// read below stay inside the frame buffer; otherwise handle_boundary_conditions
// (Encoder.py:750-768): zero-filled partial copy.
template <int NB>
SO_DEV void fetch_row(const uint8_t* __restrict__ f, int W, int H, int px, int py, bool fast, int* out) {
    if (fast) {
        const uint8_t* p = f + (size_t)py * W + px;
        const uintptr_t a = reinterpret_cast<uintptr_t>(p);
        const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
        const uint32_t sh = (uint32_t)(a & 3);
        uint32_t w[NB / 4 + 1];
#pragma unroll
        for (int k = 0; k <= NB / 4; ++k) w[k] = q[k];
#pragma unroll
        for (int k = 0; k < NB / 4; ++k) {
            uint32_t v = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
            out[4 * k + 0] = v & 255;
            out[4 * k + 1] = (v >> 8) & 255;
            out[4 * k + 2] = (v >> 16) & 255;
            out[4 * k + 3] = v >> 24;
        }
    } else {
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int xx = px + k;
            out[k] = (py >= 0 && py < H && xx >= 0 && xx < W) ? f[(size_t)py * W + xx] : 0;
        }
    }
}

// FME prediction row `row` of an NB x NB block at frac-frame position (px, py) -- the
// FMEEnable branches of calculate_inter_frame_residual (Encoder.py:444-456) and
// reconstruct_frame (:862-873, :907-919), on the reference's four phase planes
// P_ab[i][j] = F[2i+a][2j+b] (`planes`, pstride bytes apart; so_me.hip FmePhase):
//   0 <= px < W2-NB (and y)  and  0 <= px+ext < W2-lim (and y)  -> stride-2 sample of F,
//                                                                = a row of P_ab;
//   only the first                                              -> all 128;
//   neither (handle_boundary_conditions :750-768)               -> F's contiguous bytes,
//                                                                zero outside F.
// (ext, lim) = (2 NB, NB) for the residual and the unsplit recon; a split sub-block's
// recon uses the full block's (BS, BS).
template <int NB>
SO_DEV void fetch_row_fme(const uint8_t* __restrict__ planes, size_t pstride, int W, int H, int px, int py, int row,
                          int ext, int lim, int* out) {
    const int W2 = 2 * W - 1, H2 = 2 * H - 1;
    if (0 <= px && px < W2 - NB && 0 <= py && py < H2 - NB) {
        if (0 <= px + ext && px + ext < W2 - lim && 0 <= py + ext && py + ext < H2 - lim) {
            const uint8_t* pl = planes + (size_t)(2 * (py & 1) + (px & 1)) * pstride;
            fetch_row<NB>(pl, W, H, px >> 1, (py >> 1) + row, true, out);
        } else {
#pragma unroll
            for (int k = 0; k < NB; ++k) out[k] = 128;
        }
    } else {
        const int Y = py + row;
#pragma unroll
        for (int k = 0; k < NB; ++k) {
            const int X = px + k;
            out[k] = (Y >= 0 && Y < H2 && X >= 0 && X < W2)
                         ? planes[(size_t)(2 * (Y & 1) + (X & 1)) * pstride + (size_t)(Y >> 1) * W + (X >> 1)]
                         : 0;
        }
    }
}

// aligned row of the current frame (x multiple of NB, W multiple of NB)
template <int NB>
SO_DEV void load_cur_row(const uint8_t* __restrict__ f, int W, int x, int y, int* out) {
    const uint8_t* p = f + (size_t)y * W + x;
    if constexpr (NB == 16) {
        uint4 v = *reinterpret_cast<const uint4*>(p);
        uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) out[k] = (w[k >> 2] >> (8 * (k & 3))) & 255;
    } else {
        uint2 v = *reinterpret_cast<const uint2*>(p);
        uint32_t w[2] = {v.x, v.y};
#pragma unroll
        for (int k = 0; k < 8; ++k) out[k] = (w[k >> 2] >> (8 * (k & 3))) & 255;
    }
}

template <int NB>
SO_DEV void store_row_u8(uint8_t* __restrict__ f, int W, int x, int y, const int* v) {
    uint32_t w[NB / 4];
#pragma unroll
    for (int k = 0; k < NB / 4; ++k)
        w[k] = (uint32_t)(v[4 * k] & 255) | ((uint32_t)(v[4 * k + 1] & 255) << 8) |
               ((uint32_t)(v[4 * k + 2] & 255) << 16) | ((uint32_t)(v[4 * k + 3] & 255) << 24);
    uint8_t* p = f + (size_t)y * W + x;
    if constexpr (NB == 16) *reinterpret_cast<uint4*>(p) = make_uint4(w[0], w[1], w[2], w[3]);
    else *reinterpret_cast<uint2*>(p) = make_uint2(w[0], w[1]);
}

template <int NB>
SO_DEV void store_row_i16(int16_t* __restrict__ p, const int* v) {
    uint32_t w[NB / 2];
#pragma unroll
    for (int k = 0; k < NB / 2; ++k) w[k] = (uint32_t)(uint16_t)v[2 * k] | ((uint32_t)(uint16_t)v[2 * k + 1] << 16);
    if constexpr (NB == 16) {
        reinterpret_cast<uint4*>(p)[0] = make_uint4(w[0], w[1], w[2], w[3]);
        reinterpret_cast<uint4*>(p)[1] = make_uint4(w[4], w[5], w[6], w[7]);
    } else {
        reinterpret_cast<uint4*>(p)[0] = make_uint4(w[0], w[1], w[2], w[3]);
    }
}

template <int NB>
SO_DEV void load_row_i16(const int16_t* __restrict__ p, int* v) {
    uint32_t w[NB / 2];
    if constexpr (NB == 16) {
        uint4 a = reinterpret_cast<const uint4*>(p)[0], b = reinterpret_cast<const uint4*>(p)[1];
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y; w[6] = b.z; w[7] = b.w;
    } else {
        uint4 a = reinterpret_cast<const uint4*>(p)[0];
        w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w;
    }
#pragma unroll
    for (int k = 0; k < NB / 2; ++k) {
        v[2 * k] = (int)(int16_t)(w[k] & 0xFFFF);
        v[2 * k + 1] = (int)(int16_t)(w[k] >> 16);
    }
}

// ---- 2-D transforms through LDS --------------------------------------------------------------
// N x N transform of one block by N lanes (lane l owns row l on input and output).
// lds: N rows of pitch N+1 doubles owned by this lane group.
// Integer rows (T = int, N = 16: residuals forward, dequantised coefficients inverse) go through
// the scratch as int32 and take dct2_16_i / dct3_16_i on axis 0: half the first transpose's
// LDS bytes and the exact integer steps on the 2-cycle pipe.
template <int N, bool INVERSE, class T, class TWt = typename dct::Rfft<N>::TW>
SO_DEV void xform2d_rows(double* lds, int l, const T* in_row, double* out_row, const TWt& tw = TWt{}) {
    constexpr int P = N + 1;
    double v[N];
    if constexpr (N == 16 && __is_same(T, int)) {
        int* const li = reinterpret_cast<int*>(lds);
#pragma unroll
        for (int c = 0; c < N; ++c) li[l * P + c] = in_row[c];
        wave_sync();
        int x[N];
#pragma unroll
        for (int r = 0; r < N; ++r) x[r] = li[r * P + l];
        wave_sync();   // every lane's int reads before the doubles below overwrite them
        if constexpr (INVERSE) dct::dct3_16_i(x, v, tw); else dct::dct2_16_i(x, v, tw);   // axis 0 (columns)
    } else {
#pragma unroll
        for (int c = 0; c < N; ++c) lds[l * P + c] = (double)in_row[c];
        wave_sync();
#pragma unroll
        for (int r = 0; r < N; ++r) v[r] = lds[r * P + l];
        if constexpr (INVERSE) dct::dct3<N>(v, tw); else dct::dct2<N>(v, tw);   // axis 0 (columns)
    }
#pragma unroll
    for (int r = 0; r < N; ++r) lds[r * P + l] = v[r];
    wave_sync();
#pragma unroll
    for (int c = 0; c < N; ++c) v[c] = lds[l * P + c];
    if constexpr (INVERSE) dct::dct3<N>(v, tw); else dct::dct2<N>(v, tw);   // axis 1 (rows)
#pragma unroll
    for (int c = 0; c < N; ++c) out_row[c] = v[c];
    wave_sync();   // lds free for reuse
}

// The forward xform2d_rows<16, false> of integer rows through half its LDS (16 x 9 doubles): the
// int32 transpose fits the scratch whole (16 x 17 words), the FP64 one goes back to rows in two
// halves (as xform2d_rows_half).  The same operations as xform2d_rows bit for bit (the column
// pass dct2_16_i on the int32 columns, the row pass dct2 on the doubles).
template <class TWt>
SO_DEV void xform2d_fwd_i_half(double* lds, int l, const int* in_row, double* out_row, const TWt& tw) {
    constexpr int N = 16, PI = N + 1, P = 9;
    const int hl = l >> 3, cl = l & 7;
    double v[N];
    {
        int* const li = reinterpret_cast<int*>(lds);
#pragma unroll
        for (int c = 0; c < N; ++c) li[l * PI + c] = in_row[c];
        wave_sync();
        int x[N];
#pragma unroll
        for (int r = 0; r < N; ++r) x[r] = li[r * PI + l];
        wave_sync();   // every lane's int reads before the doubles below overwrite them
        dct::dct2_16_i(x, v, tw);   // axis 0 (columns)
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // columns -> rows
        if (hl == h) {
#pragma unroll
            for (int r = 0; r < N; ++r) lds[r * P + cl] = v[r];
        }
        wave_sync();
#pragma unroll
        for (int c = 0; c < 8; ++c) out_row[8 * h + c] = lds[l * P + c];
        wave_sync();
    }
    dct::dct2<N>(out_row, tw);   // axis 1 (rows)
}

// xform2d_rows<16> with half the LDS (16 x 9 doubles): each transpose goes through the buffer in
// two halves -- rows' columns 0-7 then 8-15 (lanes l < 8 take their column from the first, the
// others from the second), and back.  The same arithmetic bit for bit; 50 % more LDS
// instructions for half the scratch (the persistent kernel's LDS per workgroup, SO_TQ_HALF).
template <bool INVERSE, class T>
SO_DEV void xform2d_rows_half(double* lds, int l, const T* in_row, double* out_row) {
    constexpr int N = 16, P = 9;
    const int hl = l >> 3, cl = l & 7;
    double v[N];
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // rows -> columns
#pragma unroll
        for (int c = 0; c < 8; ++c) lds[l * P + c] = (double)in_row[8 * h + c];
        wave_sync();
        if (hl == h) {
#pragma unroll
            for (int r = 0; r < N; ++r) v[r] = lds[r * P + cl];
        }
        wave_sync();
    }
    if constexpr (INVERSE) dct::dct3<N>(v); else dct::dct2<N>(v);   // axis 0 (columns)
#pragma unroll
    for (int h = 0; h < 2; ++h) {   // columns -> rows
        if (hl == h) {
#pragma unroll
            for (int r = 0; r < N; ++r) lds[r * P + cl] = v[r];
        }
        wave_sync();
#pragma unroll
        for (int c = 0; c < 8; ++c) out_row[8 * h + c] = lds[l * P + c];
        wave_sync();
    }
    if constexpr (INVERSE) dct::dct3<N>(out_row); else dct::dct2<N>(out_row);   // axis 1 (rows)
}

// Four 8x8 sub-blocks by 16 lanes: lane l owns sub-block j = l >> 2 and rows
// (l & 3), (l & 3) + 4 on input and output.  lds: 4 x 8 x 9 doubles.
// Integer rows (T = int) go through the scratch as int32 and take dct2_8_i / dct3_8_i on the
// column pass, as xform2d_rows<16> does.
template <bool INVERSE, class T, class TWt = dct::TW8>
SO_DEV void xform2d_sub(double* lds, int l, const T (&in)[2][8], double (&out)[2][8], const TWt& tw = TWt{}) {
    const int j = l >> 2, r0 = l & 3;
    double* s = lds + j * 72;
    if constexpr (__is_same(T, int)) {
        int* const si = reinterpret_cast<int*>(s);
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int c = 0; c < 8; ++c) si[(r0 + 4 * h) * 9 + c] = in[h][c];
        wave_sync();
        int x[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int r = 0; r < 8; ++r) x[h][r] = si[r * 9 + r0 + 4 * h];
        wave_sync();   // every lane's int reads before the doubles below overwrite them
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            double v[8];
            if constexpr (INVERSE) dct::dct3_8_i(x[h], v, tw); else dct::dct2_8_i(x[h], v, tw);
#pragma unroll
            for (int r = 0; r < 8; ++r) s[r * 9 + r0 + 4 * h] = v[r];
        }
    } else {
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int c = 0; c < 8; ++c) s[(r0 + 4 * h) * 9 + c] = (double)in[h][c];
        wave_sync();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            double v[8];
            const int col = r0 + 4 * h;
#pragma unroll
            for (int r = 0; r < 8; ++r) v[r] = s[r * 9 + col];
            if constexpr (INVERSE) dct::dct3<8>(v, tw); else dct::dct2<8>(v, tw);
#pragma unroll
            for (int r = 0; r < 8; ++r) s[r * 9 + col] = v[r];
        }
    }
    wave_sync();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        double v[8];
        const int row = r0 + 4 * h;
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = s[row * 9 + c];
        if constexpr (INVERSE) dct::dct3<8>(v, tw); else dct::dct2<8>(v, tw);
#pragma unroll
        for (int c = 0; c < 8; ++c) out[h][c] = v[c];
    }
    wave_sync();
}

// ---- quantisation + tokens ------------------------------------------------------------------
// quantise row `row` of an n x n block: q = round_half_even(tc / 2^q_exp)
template <int N>
SO_DEV void quant_row(const int* tc, int row, int qp, int* q) {
#pragma unroll
    for (int c = 0; c < N; ++c) q[c] = quant_rne(tc[c], q_exp(row, c, N, qp));
}

template <int N>
SO_DEV void dequant_row(const int* q, int row, int qp, int* d) {
#pragma unroll
    for (int c = 0; c < N; ++c) d[c] = q[c] * (1 << q_exp(row, c, N, qp));
}

// The same two steps on FP64 carriers, branch-free.  tcr = rint(DCT) (an integer-valued
// double); ldexp by -k is exact and rint rounds half to even, so
//   qd = rint(ldexp(tcr, -k)) == np.round(TC / 2^k)      (quantize_TC, Encoder.py:787-789)
//   dq = ldexp(qd, k)          == QTC * Q                 (rescale_QTC, :820-821)
// exactly, with k = qp + e(row + c) (generate_Q_matrix, :938-945) and
// e(s) = med3(s - (N - 2), 0, 2): 0 above the anti-diagonal, 1 on it, 2 below.
template <int N>
SO_DEV int q_exp_fast(int row, int c, int qp) {
    const int s = row + c - (N - 2);
    return qp + (s < 0 ? 0 : (s > 2 ? 2 : s));
}

template <int N>
SO_DEV void quant_row_d(const double* tcr, int row, int qp, double* qd, int* q) {
#pragma unroll
    for (int c = 0; c < N; ++c) {
        qd[c] = __builtin_rint(__builtin_amdgcn_ldexp(tcr[c], -q_exp_fast<N>(row, c, qp)));
        q[c] = (int)qd[c];
    }
}

template <int N>
SO_DEV void dequant_row_d(const double* qd, int row, int qp, double* dq) {
#pragma unroll
    for (int c = 0; c < N; ++c) dq[c] = __builtin_amdgcn_ldexp(qd[c], q_exp_fast<N>(row, c, qp));
}

// Integer-carrier forms (fewer live VGPRs where the state must survive the RD decision):
// tc / q are exact int32 images of the integer-valued doubles.
template <int N>
SO_DEV void quant_row_i(const int* tc, int row, int qp, int* q) {
#pragma unroll
    for (int c = 0; c < N; ++c)
        q[c] = (int)__builtin_rint(__builtin_amdgcn_ldexp((double)tc[c], -q_exp_fast<N>(row, c, qp)));
}

template <int N>
SO_DEV void dequant_row_i(const int* q, int row, int qp, double* dq) {
#pragma unroll
    for (int c = 0; c < N; ++c) dq[c] = __builtin_amdgcn_ldexp((double)q[c], q_exp_fast<N>(row, c, qp));
}

// quantize_TC on integer TC (Encoder.py:787-789): np.round(TC / 2^k) half to even, branch-free in
// int32 (2-cycle VALU).  With TC = q0 2^k + r (floor, 0 <= r < 2^k), h = 2^(k-1) and b = q0 & 1,
// floor((TC + h - 1 + b) / 2^k) = q0 + [r > h or (r == h and b)] for k >= 1; k = 0 is TC.
SO_DEV int quant_rne_i(int tc, int k) {
    const int bias = k > 0 ? ((1 << k) >> 1) - 1 + ((tc >> k) & 1) : 0;
    return (tc + bias) >> k;
}
template <int N>
SO_DEV void quant_row_int(const int* tc, int row, int qp, int* q) {
#pragma unroll
    for (int c = 0; c < N; ++c) q[c] = quant_rne_i(tc[c], q_exp_fast<N>(row, c, qp));
}

// QTC * Q as int32 (xform2d_rows' integer inverse path): |q| 2^k <= |TC| + 2^(k-1)
template <int N>
SO_DEV void dequant_row_int(const int* q, int row, int qp, int* dq) {
#pragma unroll
    for (int c = 0; c < N; ++c) dq[c] = (int)((uint32_t)q[c] << q_exp_fast<N>(row, c, qp));
}

// Token count of an N x N block (N lanes, lane l owns row l) = nnz + number of maximal
// runs in anti-diagonal scan order (entropy_encoder_block emits one token per zero run,
// one count token per non-zero run, and one token per non-zero value), i.e.
// nnz + 1 + (number of consecutive scan pairs whose zero/non-zero flags differ).
// With M_i = the row-i non-zero bitmask, the 255 consecutive pairs are
//   inside diagonals:  (i, j) -> (i+1, j-1), j >= 1, i <= N-2  -> M_i bits 1..N-1 against
//                      M_{i+1} << 1, one XOR + popcount per lane (M_{i+1} by DPP row_shl:1);
//   across diagonals:  end (k, 0) -> start (0, k+1) for k <= N-2 (lane k: M_k bit 0 vs
//                      M_0 bit k+1) and end (N-1, k-N+1) -> start (k-N+2, N-1) for k >= N-1
//                      (lane m = k-N+2 >= 1: M_{N-1} bit m-1 vs M_m bit N-1).
// Registers only: no LDS, no barrier.  `flags` is unused (kept for the call sites).
template <int N>
SO_DEV int block_tokens(uint8_t* flags, int l, const int* q) {
    (void)flags;
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < N; ++c) m |= (q[c] != 0 ? 1u : 0u) << c;
    // M_{l+1}: DPP row_shl:1 (lane i reads lane i+1 of its 16-lane row; the value from
    // the next group at the group's last lane is never used: i = N-1 has no pair)
    const uint32_t mn = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x101, 0xF, 0xF, false);
    uint32_t m0, mlast;
    if constexpr (N == 16) {
        // M_0 and M_15 of the lane's 16-lane row: DPP row_newbcast (gfx90a+), no LDS round
        // trip and no lane index (which the persistent run hoisted and spilled)
        m0 = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x150, 0xF, 0xF, false);
        mlast = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)m, 0x150 + N - 1, 0xF, 0xF, false);
    } else {
        const int base = (threadIdx.x & 63) & ~(N - 1);
        m0 = (uint32_t)__shfl((int)m, base, 64);
        mlast = (uint32_t)__shfl((int)m, base + N - 1, 64);
    }
    constexpr uint32_t kInner = ((1u << N) - 1) & ~1u;
    int tr = 0;
    if (l <= N - 2) {
        tr += __builtin_popcount((m ^ (mn << 1)) & kInner);
        tr += (int)((m & 1u) ^ ((m0 >> (l + 1)) & 1u));
    }
    if (l >= 1) tr += (int)(((mlast >> (l - 1)) & 1u) ^ ((m >> (N - 1)) & 1u));
    return group_sum<N>(__builtin_popcount(m) + tr) + 1;
}

// Token counts of the four 8x8 sub-blocks (16 lanes, lane l owns sub j = l>>2, rows
// (l&3), (l&3)+4).  Returns the sum over the 4 sub-blocks (RD bits and residual_size).
SO_DEV int sub_tokens(uint8_t* flags, int l, const int (&q)[2][8]) {
    const int j = l >> 2, r0 = l & 3;
    uint8_t* s = flags + j * 64;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
        for (int c = 0; c < 8; ++c) s[scan_index(8, r0 + 4 * h, c)] = q[h][c] != 0;
    wave_sync();
    int nnz = 0, tr = 0;
    const int base = r0 * 16;
    int prev = s[base == 0 ? 0 : base - 1];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int f = s[base + k];
        nnz += f;
        tr += (f != prev);
        prev = f;
    }
    wave_sync();
    return group_sum<16>(nnz + tr) + 4;
}

// sub_tokens in registers: the same count from the sub-blocks' row masks, no LDS and no barrier
// (the VBS run's LDS budget).  Lane l holds rows r0 = l & 3 and r0 + 4 of sub-block l >> 2; the
// quad of lanes of a sub-block gathers all 8 row masks (byte i of lo / hi = row i / i + 4), then
// each lane counts the scan-order transitions that start in its two rows (block_tokens' three
// kinds of consecutive pairs, for N = 8):
//   inside a diagonal  (i, j) -> (i+1, j-1), j >= 1, i <= 6: bits 1..7 of M_i vs M_{i+1} << 1;
//   diagonal k <= 6 ends at (k, 0), the next starts at (0, k+1): M_k bit 0 vs M_0 bit k+1;
//   diagonal k >= 7 ends at (7, k-7), the next starts at (m, 7), m = k-6 in 1..7: M_7 bit m-1
//   vs M_m bit 7.
SO_DEV int sub_tokens_reg(int l, const int (&q)[2][8]) {
    const int r0 = l & 3;
    uint32_t m0 = 0, m1 = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        m0 |= (q[0][c] != 0 ? 1u : 0u) << c;
        m1 |= (q[1][c] != 0 ? 1u : 0u) << c;
    }
    uint32_t lo = m0 << (8 * r0), hi = m1 << (8 * r0);
    lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
    hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0xB1, 0xF, 0xF, false);
    lo |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
    hi |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi, 0x4E, 0xF, 0xF, false);
    const uint32_t n0 = r0 < 3 ? (lo >> (8 * r0 + 8)) & 255u : hi & 255u;    // M_{r0+1}
    const uint32_t n1 = r0 < 3 ? (hi >> (8 * r0 + 8)) & 255u : 0u;           // M_{r0+5}
    const uint32_t M0 = lo & 255u, M7 = hi >> 24;
    int tr = __builtin_popcount((m0 ^ (n0 << 1)) & 0xFEu) + (int)((m0 & 1u) ^ ((M0 >> (r0 + 1)) & 1u)) +
             (int)(((M7 >> (r0 + 3)) & 1u) ^ (m1 >> 7));
    if (r0 < 3) tr += __builtin_popcount((m1 ^ (n1 << 1)) & 0xFEu) + (int)((m1 & 1u) ^ ((M0 >> (r0 + 5)) & 1u));
    if (r0 >= 1) tr += (int)(((M7 >> (r0 - 1)) & 1u) ^ (m0 >> 7));
    return group_sum<16>(__builtin_popcount(m0) + __builtin_popcount(m1) + tr) + 4;
}

// calculate_RD_cost (Encoder.py:1133-1158): lam * bits + mae, two roundings (no FMA:
// this translation unit is compiled with -ffp-contract=off).
SO_DEV double rd_cost(double lam, int bits, double mae) {
    const double lb = lam * (double)bits;
    return lb + mae;
}

}  // namespace so
