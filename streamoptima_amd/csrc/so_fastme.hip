// so_fastme.hip — fast_me (Encoder.py:719-742) for gfx950, integer-pel and FME.
//
// fast_motion_estimation searches the 3x3 neighbourhood of a predictor mvp over
// refs[:nRefFrames], at (x, y) -- or (2x, 2y) on the frac frame with FME:
//   * candidate (dx, dy) in mvp + {-1, 0, 1}^2 (ref outer, dx middle, dy inner) is valid iff
//       0 <= X+dx < PW-n  and  0 <= X+dx+2n < PW-n   (and the same for y)
//     -- the second test is the reference's FME bound, applied even without FME (:727);
//   * the strictly smaller MAE wins: the first found minimum in scan order;
//   * it returns (best_mv, best_ref_idx): best_mv = mvp when no candidate is valid, and the
//     caller uses best_ref_idx AS THE BLOCK'S MAE (:742).  The kernels therefore write
//     (dx, dy, ref, ref * n * n) into the ME record -- so_inter_tq_recon reads the last
//     field as MAE * n^2 -- and (mvp.dx, mvp.dy, mvp.ref, 0) when nothing is valid.
// The predictor chain of inter_prediction's serial branch (:462-585): mvp starts at
// (0, 0, 0) and becomes each block's full-block mv in raster order (:581); the VBS
// sub-blocks of a block use the same mvp as the block itself.  This is a true serial
// dependence, so `serial` runs ONE wavefront along the frame; its loads for a block depend
// only on the previous block's mv.  Under ParallelMode 2 (inter_prediction_parallel
// :587-676) every block's mvp is (0, 0, 0) with nRefFrames 1: one wavefront per block.
//
// Lane mapping: a bs x bs block is (row i, dword c) -> lane i * (bs/4) + c; the four
// (bs/2) sub-blocks of VBS take one 16-lane DPP row each (bs 16) with the same mapping.
// A lane reads its 4 reference bytes as two aligned dwords + v_alignbyte (any column);
// with FME the stride-2 sample of F at (X+dx, Y+dy) is 4 CONSECUTIVE bytes of phase plane
// P_ab (a = (Y+dy) & 1, b = (X+dx) & 1), see so_me.hip FmePhase.
#include "so_common.h"
#include "so_dpp.h"

namespace so {

struct FastRefs {
    const uint8_t* p[4 * kMaxRef];   // integer: refs; FME: phase planes 4 r + 2a + b
};

SO_DEV uint32_t unaligned_u32(const uint8_t* p) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(a & ~(uintptr_t)3);
    return __builtin_amdgcn_alignbyte(q[1], q[0], (uint32_t)(a & 3));
}

// sum over aligned groups of G lanes (4: quads, 16: DPP rows, 64: the wave), result in
// every lane of the group
template <int G>
SO_DEV uint32_t group_sum_u32(uint32_t v) {
    if constexpr (G == 64) return wave_sum_u32(v);
    else if constexpr (G == 16) return row_sum_u32(v);
    else return quad_sum_u32(v);
}

struct Mvp {
    int dx, dy, ref;
};

// One fast search of an n x n block at frame position (x, y) by the lanes of a G-lane
// group; (lane_i, lane_c) = the lane's block row / dword, `act` = the lane holds pixels.
// Writes the record (dx, dy, ref, mae * n * n), identical in every lane of the group.
template <bool FME, int G>
SO_DEV void fast_search(const uint8_t* __restrict__ cur, const FastRefs& R, int nref, int H, int W, int x, int y,
                        int n, Mvp mvp, int lane_i, int lane_c, bool act, int32_t out[4]) {
    const int k = FME ? 2 : 1;
    const int PW = FME ? 2 * W - 1 : W, PH = FME ? 2 * H - 1 : H;
    const int X = k * x, Y = k * y;
    const uint32_t cw = *reinterpret_cast<const uint32_t*>(cur + (size_t)(y + (act ? lane_i : 0)) * W + x +
                                                           4 * (act ? lane_c : 0));
    uint32_t best = 0xFFFFFFFFu;   // (sad << 8) | candidate index r * 9 + ci
#pragma unroll 1
    for (int r = 0; r < nref; ++r) {
        // all nine candidates' bytes are loaded before any is used (one latency per ref):
        // the addresses are clamped into the plane, invalid candidates are masked below
        uint32_t wv[9];
#pragma unroll
        for (int ci = 0; ci < 9; ++ci) {
            const int px = X + mvp.dx - 1 + ci / 3, py = Y + mvp.dy - 1 + ci % 3;
            const uint8_t* p;
            if constexpr (FME) {
                int row = (py >> 1) + lane_i, col = (px >> 1) + 4 * lane_c;
                row = row < 0 ? 0 : (row > H - 1 ? H - 1 : row);
                col = col < 0 ? 0 : (col > W - 4 ? W - 4 : col);
                p = R.p[4 * r + 2 * (py & 1) + (px & 1)] + (size_t)row * W + col;
            } else {
                int row = py + lane_i, col = px + 4 * lane_c;
                row = row < 0 ? 0 : (row > H - 1 ? H - 1 : row);
                col = col < 0 ? 0 : (col > W - 4 ? W - 4 : col);
                p = R.p[r] + (size_t)row * W + col;
            }
            wv[ci] = unaligned_u32(p);
        }
#pragma unroll
        for (int ci = 0; ci < 9; ++ci) {
            const int px = X + mvp.dx - 1 + ci / 3, py = Y + mvp.dy - 1 + ci % 3;
            const bool ok = 0 <= px && px < PW - n && 0 <= py && py < PH - n && px + 2 * n < PW - n &&
                            py + 2 * n < PH - n;   // uniform over the group
            const uint32_t s = group_sum_u32<G>(act ? __builtin_amdgcn_sad_u8(cw, wv[ci], 0u) : 0u);
            const uint32_t key = (s << 8) | (uint32_t)(r * 9 + ci);
            best = (ok && key < best) ? key : best;
        }
    }
    if (best == 0xFFFFFFFFu) {
        out[0] = mvp.dx; out[1] = mvp.dy; out[2] = mvp.ref; out[3] = 0;
    } else {
        const int c = (int)(best & 255), r = c / 9, ci = c % 9;
        out[0] = mvp.dx - 1 + ci / 3; out[1] = mvp.dy - 1 + ci % 3; out[2] = r; out[3] = r * n * n;
    }
}

// The nine candidates' bytes of one lane for the search of fast_search (clamped addresses).
template <bool FME>
SO_DEV void fast_loads(const FastRefs& R, int r, int H, int W, int X, int Y, Mvp mvp, int lane_i, int lane_c,
                       uint32_t (&wv)[9]) {
#pragma unroll
    for (int ci = 0; ci < 9; ++ci) {
        const int px = X + mvp.dx - 1 + ci / 3, py = Y + mvp.dy - 1 + ci % 3;
        const uint8_t* p;
        if constexpr (FME) {
            int row = (py >> 1) + lane_i, col = (px >> 1) + 4 * lane_c;
            row = row < 0 ? 0 : (row > H - 1 ? H - 1 : row);
            col = col < 0 ? 0 : (col > W - 4 ? W - 4 : col);
            p = R.p[4 * r + 2 * (py & 1) + (px & 1)] + (size_t)row * W + col;
        } else {
            int row = py + lane_i, col = px + 4 * lane_c;
            row = row < 0 ? 0 : (row > H - 1 ? H - 1 : row);
            col = col < 0 ? 0 : (col > W - 4 ? W - 4 : col);
            p = R.p[r] + (size_t)row * W + col;
        }
        wv[ci] = unaligned_u32(p);
    }
}

// fast_search's key update for one reference from the loaded bytes
template <bool FME, int G>
SO_DEV uint32_t fast_keys(uint32_t best, uint32_t cw, const uint32_t (&wv)[9], int r, int H, int W, int X, int Y, int n,
                          Mvp mvp, bool act) {
    const int PW = FME ? 2 * W - 1 : W, PH = FME ? 2 * H - 1 : H;
#pragma unroll
    for (int ci = 0; ci < 9; ++ci) {
        const int px = X + mvp.dx - 1 + ci / 3, py = Y + mvp.dy - 1 + ci % 3;
        const bool ok = 0 <= px && px < PW - n && 0 <= py && py < PH - n && px + 2 * n < PW - n && py + 2 * n < PH - n;
        const uint32_t sv = group_sum_u32<G>(act ? __builtin_amdgcn_sad_u8(cw, wv[ci], 0u) : 0u);
        const uint32_t key = (sv << 8) | (uint32_t)(r * 9 + ci);
        best = (ok && key < best) ? key : best;
    }
    return best;
}

SO_DEV void fast_record(uint32_t best, Mvp mvp, int n, int32_t out[4]) {
    if (best == 0xFFFFFFFFu) {
        out[0] = mvp.dx; out[1] = mvp.dy; out[2] = mvp.ref; out[3] = 0;
    } else {
        const int c = (int)(best & 255), r = c / 9, ci = c % 9;
        out[0] = mvp.dx - 1 + ci / 3; out[1] = mvp.dy - 1 + ci % 3; out[2] = r; out[3] = r * n * n;
    }
}

// fast_block with the sub-block and block searches' loads issued together (one memory latency
// per reference and chain step instead of two); same records.  bs 16 only.
template <bool FME>
SO_DEV Mvp fast_block_vbs16(const uint8_t* __restrict__ cur, const FastRefs& R, int nref, int H, int W, int x, int y,
                            Mvp mvp, int lane, int32_t* __restrict__ ob, int32_t* __restrict__ os) {
    const int k = FME ? 2 : 1;
    const bool sub = x != 0 && y != 0;
    const int j = lane >> 4, si = (lane >> 1) & 7, sc = lane & 1;   // sub-block j, its row / dword
    const int xs = x + (j & 1) * 8, ys = y + (j >> 1) * 8;
    const int fi = lane >> 2, fc = lane & 3;                        // block row / dword
    const uint32_t cws = *reinterpret_cast<const uint32_t*>(cur + (size_t)(ys + si) * W + xs + 4 * sc);
    const uint32_t cwf = *reinterpret_cast<const uint32_t*>(cur + (size_t)(y + fi) * W + x + 4 * fc);
    uint32_t bs_ = 0xFFFFFFFFu, bf = 0xFFFFFFFFu;
#pragma unroll 1
    for (int r = 0; r < nref; ++r) {
        uint32_t ws[9], wf[9];
        if (sub) fast_loads<FME>(R, r, H, W, k * xs, k * ys, mvp, si, sc, ws);
        fast_loads<FME>(R, r, H, W, k * x, k * y, mvp, fi, fc, wf);
        if (sub) bs_ = fast_keys<FME, 16>(bs_, cws, ws, r, H, W, k * xs, k * ys, 8, mvp, true);
        bf = fast_keys<FME, 64>(bf, cwf, wf, r, H, W, k * x, k * y, 16, mvp, true);
    }
    if (sub) {
        int32_t rec[4];
        fast_record(bs_, mvp, 8, rec);
        const int e = lane - 16 * j;   // lanes 16j .. 16j+3 store the sub-block's record
        const int32_t v = e == 0 ? rec[0] : e == 1 ? rec[1] : e == 2 ? rec[2] : rec[3];
        if (e >= 0 && e < 4) os[j * 4 + e] = v;
    }
    int32_t rec[4];
    fast_record(bf, mvp, 16, rec);
    const int32_t v = lane == 0 ? rec[0] : lane == 1 ? rec[1] : lane == 2 ? rec[2] : rec[3];
    if (lane < 4) ob[lane] = v;
    return Mvp{__builtin_amdgcn_readfirstlane(rec[0]), __builtin_amdgcn_readfirstlane(rec[1]),
               __builtin_amdgcn_readfirstlane(rec[2])};   // lane 0 holds the record (all lanes active)
}

// bs 16: full block on 64 lanes (row l >> 2, dword l & 3); sub-blocks on the four 16-lane
// rows (sub j = l >> 4, row (l >> 1) & 7, dword l & 1).  bs 8: full block on lanes 0..15
// (row l >> 1, dword l & 1); 4x4 sub-blocks on 4 lanes each (sub l >> 2, row l & 3).
// Returns the full block's mv (the next predictor of the serial chain), uniform.
template <bool FME, bool SUB, int BS>
SO_DEV Mvp fast_block(const uint8_t* __restrict__ cur, const FastRefs& R, int nref, int H, int W, int x, int y,
                      Mvp mvp, int lane, int32_t* __restrict__ ob, int32_t* __restrict__ os) {
    if constexpr (SUB && BS == 16) return fast_block_vbs16<FME>(cur, R, nref, H, W, x, y, mvp, lane, ob, os);
    constexpr int SBS = BS / 2;
    if constexpr (SUB) {
        if (x != 0 && y != 0) {
            int32_t rec[4];
            int j, i, c;
            if constexpr (BS == 16) { j = lane >> 4; i = (lane >> 1) & 7; c = lane & 1; }
            else { j = (lane >> 2) & 3; i = lane & 3; c = 0; }
            const bool act = BS == 16 || lane < 16;
            const int xs = x + (j & 1) * SBS, ys = y + (j >> 1) * SBS;
            fast_search<FME, BS == 16 ? 16 : 4>(cur, R, nref, H, W, xs, ys, SBS, mvp, i, c, act, rec);
            const int lj = BS == 16 ? 16 * j : 4 * j;
            const int e = lane - lj;   // lanes lj .. lj+3 store the sub-block's record
            const int32_t v = e == 0 ? rec[0] : e == 1 ? rec[1] : e == 2 ? rec[2] : rec[3];
            if (act && e >= 0 && e < 4) os[j * 4 + e] = v;
        }
    }
    int32_t rec[4];
    const int i = BS == 16 ? lane >> 2 : lane >> 1, c = BS == 16 ? lane & 3 : lane & 1;
    const bool act = BS == 16 || lane < 16;
    fast_search<FME, BS == 16 ? 64 : 16>(cur, R, nref, H, W, x, y, BS, mvp, i, c, act, rec);
    const int32_t v = lane == 0 ? rec[0] : lane == 1 ? rec[1] : lane == 2 ? rec[2] : rec[3];
    if (lane < 4) ob[lane] = v;
    // the record is identical in the lanes of the block's group; lane 0 is in it
    return Mvp{__builtin_amdgcn_readfirstlane(rec[0]), __builtin_amdgcn_readfirstlane(rec[1]),
               __builtin_amdgcn_readfirstlane(rec[2])};   // lane 0 holds the record (all lanes active)
}

template <bool FME, bool SUB, int BS>
__global__ void __launch_bounds__(256)
me_fastpred_kernel(const uint8_t* __restrict__ cur, FastRefs R, int nref, int H, int W, int by0, int by1, int serial,
                   int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub) {
    const int nbx = W / BS, nb = nbx * (by1 - by0);
    const int lane = threadIdx.x & 63;
    if (serial) {
        // one wavefront walks the range in raster order; mvp = the previous block's mv
        if (blockIdx.x != 0 || threadIdx.x >= 64) return;
        Mvp mvp{0, 0, 0};
        for (int b = 0; b < nb; ++b) {
            const int x = (b % nbx) * BS, y = (by0 + b / nbx) * BS;
            mvp = fast_block<FME, SUB, BS>(cur, R, nref, H, W, x, y, mvp, lane, out_best + (size_t)b * 4,
                                           out_sub ? out_sub + (size_t)b * 16 : nullptr);
        }
        return;
    }
    const int b = blockIdx.x * 4 + (threadIdx.x >> 6);   // one wave per block, mvp (0,0,0)
    if (b >= nb) return;
    const int x = (b % nbx) * BS, y = (by0 + b / nbx) * BS;
    fast_block<FME, SUB, BS>(cur, R, nref, H, W, x, y, Mvp{0, 0, 0}, lane, out_best + (size_t)b * 4,
                             out_sub ? out_sub + (size_t)b * 16 : nullptr);
}

// ---- the serial chain, speculated by segments ----------------------------------------------
// The chain mv(b) = F_b(mv(b - 1)) is a local descent: from different predictors it falls into
// the same minimum within a few blocks.  So (1) one wavefront per segment of K blocks first
// runs the chain over the WARM blocks before its segment from (0, 0, 0) -- its guess of the
// segment's true predictor -- then the segment itself, storing every record; (2) one wavefront
// walks the segments in order: segment s is exact iff its guessed predictor equals the last mv
// of segment s - 1 (F is deterministic, so equal inputs give equal records), else it re-runs
// the segment from the true predictor.  Bit-identical to the serial walk by construction; the
// chain of 32,400 dependent steps (a 4K frame) becomes K + WARM steps per wavefront plus one
// compare per segment and a K-step redo per wrong guess.
constexpr int kFastSegMax = 4096;                 // segments per launch (the fix kernel's LDS)
// per segment: guessed predictor, last mv, in the caller's scratch (kFastSegWords int32 after
// the ME records, so_p_frame_scratch_elems; the second half of that region is unused)

template <bool FME, int BS>
SO_DEV Mvp fast_chain_mv(const uint8_t* __restrict__ cur, const FastRefs& R, int nref, int H, int W, int x, int y,
                         Mvp mvp, int lane) {
    int32_t rec[4];
    const int i = BS == 16 ? lane >> 2 : lane >> 1, c = BS == 16 ? lane & 3 : lane & 1;
    const bool act = BS == 16 || lane < 16;
    fast_search<FME, BS == 16 ? 64 : 16>(cur, R, nref, H, W, x, y, BS, mvp, i, c, act, rec);
    return Mvp{__builtin_amdgcn_readfirstlane(rec[0]), __builtin_amdgcn_readfirstlane(rec[1]),
               __builtin_amdgcn_readfirstlane(rec[2])};   // lane 0 holds the record (all lanes active)
}

template <bool FME, bool SUB, int BS>
__global__ void __launch_bounds__(64)
me_fastchain_spec_kernel(const uint8_t* __restrict__ cur, FastRefs R, int nref, int H, int W, int by0, int by1, int K,
                         int warm, int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub,
                         int32_t* __restrict__ seg) {
    const int nbx = W / BS, nb = nbx * (by1 - by0);
    const int lane = threadIdx.x;
    const int s = blockIdx.x, b0 = s * K, b1 = b0 + K < nb ? b0 + K : nb;
    Mvp mvp{0, 0, 0};
    for (int b = (b0 - warm > 0 ? b0 - warm : 0); b < b0; ++b)
        mvp = fast_chain_mv<FME, BS>(cur, R, nref, H, W, (b % nbx) * BS, (by0 + b / nbx) * BS, mvp, lane);
    if (lane == 0) {
        seg[s * 6 + 0] = mvp.dx; seg[s * 6 + 1] = mvp.dy; seg[s * 6 + 2] = mvp.ref;
    }
    for (int b = b0; b < b1; ++b)
        mvp = fast_block<FME, SUB, BS>(cur, R, nref, H, W, (b % nbx) * BS, (by0 + b / nbx) * BS, mvp, lane,
                                       out_best + (size_t)b * 4, out_sub ? out_sub + (size_t)b * 16 : nullptr);
    if (lane == 0) {
        seg[s * 6 + 3] = mvp.dx; seg[s * 6 + 4] = mvp.dy; seg[s * 6 + 5] = mvp.ref;
    }
}

template <bool FME, bool SUB, int BS>
__global__ void __launch_bounds__(64)
me_fastchain_fix_kernel(const uint8_t* __restrict__ cur, FastRefs R, int nref, int H, int W, int by0, int by1, int K,
                        int nseg, int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub,
                        const int32_t* __restrict__ segws, int32_t* __restrict__ nfixed) {
    __shared__ int32_t seg[kFastSegMax * 6];
    const int nbx = W / BS, nb = nbx * (by1 - by0);
    const int lane = threadIdx.x;
    for (int i = lane; i < nseg * 6; i += 64) seg[i] = segws[i];
    __syncthreads();
    Mvp truth{seg[3], seg[4], seg[5]};   // segment 0 started from the true (0, 0, 0)
    int fixed = 0;
    for (int s = 1; s < nseg; ++s) {
        if (seg[s * 6] == truth.dx && seg[s * 6 + 1] == truth.dy && seg[s * 6 + 2] == truth.ref) {
            truth = Mvp{seg[s * 6 + 3], seg[s * 6 + 4], seg[s * 6 + 5]};
            continue;
        }
        // wrong guess: the segment again from the true predictor, until the true chain meets
        // the speculated one -- from a block whose true mv equals the stored (speculated) mv,
        // every later block of the segment already had the true predictor
        ++fixed;
        const int b0 = s * K, b1 = b0 + K < nb ? b0 + K : nb;
        bool joined = false;
        for (int b = b0; b < b1 && !joined; ++b) {
            const int32_t* ob = out_best + (size_t)b * 4;
            const int odx = ob[0], ody = ob[1], oref = ob[2];   // the speculated record (before the store)
            truth = fast_block<FME, SUB, BS>(cur, R, nref, H, W, (b % nbx) * BS, (by0 + b / nbx) * BS, truth, lane,
                                             out_best + (size_t)b * 4, out_sub ? out_sub + (size_t)b * 16 : nullptr);
            joined = truth.dx == odx && truth.dy == ody && truth.ref == oref;
        }
        if (joined) truth = Mvp{seg[s * 6 + 3], seg[s * 6 + 4], seg[s * 6 + 5]};
    }
    if (lane == 0 && nfixed) *nfixed = fixed;
}

__device__ int32_t g_fast_fixed;   // segments redone by the last chain (tools / tests)
extern "C" int so_debug_fast_chain_fixed(int* out) {
    return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fast_fixed), sizeof(int));
}

int me_fastpred_launch(const uint8_t* cur, const uint8_t* const* ptrs, int nptr, int nref, int H, int W, int bs,
                       int fme, int by0, int by1, int serial, int32_t* out_best, int32_t* out_sub, int32_t* seg_ws,
                       hipStream_t st) {
    FastRefs R{};
    for (int i = 0; i < nptr && i < 4 * kMaxRef; ++i) R.p[i] = ptrs[i];
    const int nb = (W / bs) * (by1 - by0);
    if (nb <= 0) return SO_OK;
    // SO_OPT_FASTME_SERIAL: the one-wavefront walk; no workspace (so_me_search_ex): the walk
    if (serial && seg_ws && option(SO_OPT_FASTME_SERIAL) != 1) {
        int K = option(SO_OPT_FASTME_SEGMENT), warm = option(SO_OPT_FASTME_WARMUP);
        if ((nb + K - 1) / K > kFastSegMax) K = (nb + kFastSegMax - 1) / kFastSegMax;
        const int nseg = (nb + K - 1) / K;
        int32_t* nfixed = nullptr;
        if (hipGetSymbolAddress(reinterpret_cast<void**>(&nfixed), HIP_SYMBOL(g_fast_fixed)) != hipSuccess)
            nfixed = nullptr;
        const bool sub = out_sub != nullptr;
#define SO_FASTCHAIN(F, S, B)                                                                                       \
        do {                                                                                                        \
            hipLaunchKernelGGL((me_fastchain_spec_kernel<F, S, B>), dim3(nseg), dim3(64), 0, st, cur, R, nref, H,   \
                               W, by0, by1, K, warm, out_best, out_sub, seg_ws);                                    \
            hipLaunchKernelGGL((me_fastchain_fix_kernel<F, S, B>), dim3(1), dim3(64), 0, st, cur, R, nref, H, W,    \
                               by0, by1, K, nseg, out_best, out_sub, seg_ws, nfixed);                               \
        } while (0)
        if (bs == 16) {
            if (fme) { if (sub) SO_FASTCHAIN(true, true, 16); else SO_FASTCHAIN(true, false, 16); }
            else { if (sub) SO_FASTCHAIN(false, true, 16); else SO_FASTCHAIN(false, false, 16); }
        } else {
            if (fme) { if (sub) SO_FASTCHAIN(true, true, 8); else SO_FASTCHAIN(true, false, 8); }
            else { if (sub) SO_FASTCHAIN(false, true, 8); else SO_FASTCHAIN(false, false, 8); }
        }
#undef SO_FASTCHAIN
        return check_launch("me_fastchain_kernel");
    }
    const dim3 grid(serial ? 1 : (nb + 3) / 4), blk(serial ? 64 : 256);
    const bool sub = out_sub != nullptr;
#define SO_FASTPRED(F, S, B)                                                                                 \
    hipLaunchKernelGGL((me_fastpred_kernel<F, S, B>), grid, blk, 0, st, cur, R, nref, H, W, by0, by1, serial, \
                       out_best, out_sub)
    if (bs == 16) {
        if (fme) { if (sub) SO_FASTPRED(true, true, 16); else SO_FASTPRED(true, false, 16); }
        else { if (sub) SO_FASTPRED(false, true, 16); else SO_FASTPRED(false, false, 16); }
    } else {
        if (fme) { if (sub) SO_FASTPRED(true, true, 8); else SO_FASTPRED(true, false, 8); }
        else { if (sub) SO_FASTPRED(false, true, 8); else SO_FASTPRED(false, false, 8); }
    }
#undef SO_FASTPRED
    return check_launch("me_fastpred_kernel");
}

}  // namespace so
