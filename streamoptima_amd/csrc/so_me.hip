// so_me.hip — full-search integer-pel motion estimation for gfx950.
//
// Replaces find_best_match / compute_mae / is_better_mv (Encoder.py:678-717, 314-315,
// 771-773).  Semantics reproduced exactly:
//   * candidates dx, dy in [-sr, sr] for each reference frame; valid iff
//       0 <= x+dx < W-bs  and  0 <= y+dy < H-bs          (strict, Encoder.py:695)
//   * MAE = SAD / bs^2 exactly (power-of-two divisor), so integer SAD compares the same;
//   * keep if mae < best or (mae == best and (|dx|+|dy|, ref) strictly smaller), scanning
//     ref (outer), dx (middle), dy (inner) => the result is the lexicographic minimum of
//       key = (SAD, |dx|+|dy|, ref, scan),  scan = (dx+sr)*(2sr+1) + (dy+sr)
//     which is packed into one uint64 so the argmin is a plain min (LDS atomicMin).
//   * no valid candidate => mv (0,0,0), MAE inf (SAD reported as -1).
//
// Fast path (sr == 16, bs in {16, 8}): a workgroup owns a TB x TB tile of blocks and
// stages the reference window (tile + 2*sr halo) in LDS once per reference.  A task is
// (block, dx): the lane keeps the current block in VGPRs, slides down the 2*sr+bs window
// rows once, and for every (cur row r, window row j) pair adds one 16-px row SAD into
// acc[j - r] with v_sad_u8 (4 byte-|diffs| + accumulate per instruction) after aligning
// the window bytes with v_alignbyte.  All 2*sr+1 dy candidates of the lane's dx share
// each window-row load, so LDS traffic is (bs+2sr)*(bs/4+1) dwords per 33 candidates.
// With VBS the same workgroup also runs the 8x8 sub-block searches on the same window.
//
// Generic path (any sr <= 64): one thread per (block, candidate) with a global atomicMin.
#include <stdlib.h>
#include <string.h>

#include "so_common.h"

namespace so {

SO_DEV uint64_t me_key(uint32_t sad, uint32_t l1, uint32_t ref, uint32_t scan) {
    return ((uint64_t)sad << 32) | ((uint64_t)l1 << 24) | ((uint64_t)ref << 16) | (uint64_t)scan;
}
constexpr uint64_t kNoKey = ~0ull;

SO_DEV void decode_key(uint64_t k, int sr, int32_t* out) {
    if (k == kNoKey) {
        out[0] = 0; out[1] = 0; out[2] = 0; out[3] = -1;
        return;
    }
    const int d = 2 * sr + 1;
    const int scan = (int)(k & 0xFFFF);
    out[0] = scan / d - sr;
    out[1] = scan % d - sr;
    out[2] = (int)((k >> 16) & 0xFF);
    out[3] = (int)(k >> 32);
}

// ---------------------------------------------------------------------------------------
// Fast path
// ---------------------------------------------------------------------------------------
template <int BS>
struct MeTile {
    static constexpr int SR = 16;
    static constexpr int D = 2 * SR + 1;                 // 33 candidates per axis
    static constexpr int TB = (BS == 16) ? 8 : 16;       // blocks per tile side
    static constexpr int TPX = TB * BS;                  // 128 px
    static constexpr int WR = TPX + 2 * SR;              // window rows
    static constexpr int WC = TPX + 2 * SR;              // window cols
    static constexpr int WPD = (WC + 16) / 4 + 1;        // pitch in dwords (+1 breaks bank stride)
    static constexpr int NBLK = TB * TB;
    static constexpr int NWAVES = 11;                    // 704 threads; 33*64 = 3*704
    static constexpr int NTHREADS = NWAVES * 64;
};

// One task: block (or sub-block) of size TBS at frame (x, y), window coordinates of its
// top-left (wrow0, wcol0) = position - (tile origin - SR), candidate column dxi.
// Returns the lane's best key over the 33 dy candidates.
template <int TBS, int SR>
SO_DEV uint64_t me_task(const uint32_t* __restrict__ win, int wpd, const uint8_t* __restrict__ cur,
                        int W, int H, int x, int y, int wrow0, int wcol0, int dxi, int ref) {
    constexpr int D = 2 * SR + 1;
    constexpr int NDW = TBS / 4;  // dwords per block row
    uint32_t cr[TBS][NDW];
#pragma unroll
    for (int r = 0; r < TBS; ++r) {
        const uint8_t* p = cur + (size_t)(y + r) * W + x;
        if constexpr (TBS == 16) {
            uint4 v = *reinterpret_cast<const uint4*>(p);
            cr[r][0] = v.x; cr[r][1] = v.y; cr[r][2] = v.z; cr[r][3] = v.w;
        } else {
            uint2 v = *reinterpret_cast<const uint2*>(p);
            cr[r][0] = v.x; cr[r][1] = v.y;
        }
    }
    uint32_t acc[D];
#pragma unroll
    for (int i = 0; i < D; ++i) acc[i] = 0;

    const int c = wcol0 + dxi;
    const uint32_t sh = (uint32_t)(c & 3);
    const uint32_t* rowp = win + wrow0 * wpd + (c >> 2);
#pragma unroll
    for (int j = 0; j < TBS + 2 * SR; ++j) {
        uint32_t w[NDW + 1];
#pragma unroll
        for (int k = 0; k <= NDW; ++k) w[k] = rowp[j * wpd + k];
        uint32_t rr[NDW];
#pragma unroll
        for (int k = 0; k < NDW; ++k) rr[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
#pragma unroll
        for (int r = 0; r < TBS; ++r) {
            const int di = j - r;
            if (di >= 0 && di < D) {
#pragma unroll
                for (int k = 0; k < NDW; ++k) acc[di] = __builtin_amdgcn_sad_u8(cr[r][k], rr[k], acc[di]);
            }
        }
    }
    const int dx = dxi - SR;
    const bool xok = (x + dx >= 0) && (x + dx < W - TBS);
    uint64_t best = kNoKey;
    if (xok) {
        const uint32_t adx = (uint32_t)(dx < 0 ? -dx : dx);
#pragma unroll
        for (int di = 0; di < D; ++di) {
            const int dy = di - SR;
            const bool ok = (y + dy >= 0) && (y + dy < H - TBS);
            const uint64_t k = me_key(acc[di], adx + (uint32_t)(dy < 0 ? -dy : dy), (uint32_t)ref,
                                      (uint32_t)(dxi * D + di));
            best = (ok && k < best) ? k : best;
        }
    }
    return best;
}

template <int BS, bool SUB>
__global__ void __launch_bounds__(MeTile<BS>::NTHREADS)
me_fast_kernel(const uint8_t* __restrict__ cur, RefSet refs, int nref, int H, int W,
               int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub) {
    using T = MeTile<BS>;
    constexpr int SR = T::SR, D = T::D, TB = T::TB, SB = BS / 2;
    __shared__ uint32_t win[T::WR * T::WPD];
    __shared__ unsigned long long keys[T::NBLK * (SUB ? 5 : 1)];

    const int nbx = W / BS, nby = H / BS;
    const int tiles_x = (nbx + TB - 1) / TB;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int x0 = tx * T::TPX, y0 = ty * T::TPX;
    const int tid = threadIdx.x;

    for (int i = tid; i < T::NBLK * (SUB ? 5 : 1); i += T::NTHREADS) keys[i] = kNoKey;

    constexpr int NFULL = T::NBLK * D;               // 2112 (bs16) / 8448 (bs8)
    constexpr int NSUBT = SUB ? 4 * T::NBLK * D : 0;
    constexpr int NTASK = NFULL + NSUBT;

    for (int r = 0; r < nref; ++r) {
        const uint8_t* ref = refs.p[r];
        __syncthreads();  // previous reference's tasks done with the window
        // stage the window: rows y0-SR .., cols x0-SR .. (dwords; zero outside the frame)
        constexpr int WCD = T::WC / 4;
        for (int i = tid; i < T::WR * T::WPD; i += T::NTHREADS) {
            const int wr = i / T::WPD, wc = i % T::WPD;
            const int gy = y0 - SR + wr, gx = x0 - SR + wc * 4;
            uint32_t v = 0;
            if (wc < WCD && gy >= 0 && gy < H && gx >= 0 && gx + 4 <= W)
                v = *reinterpret_cast<const uint32_t*>(ref + (size_t)gy * W + gx);
            win[i] = v;
        }
        __syncthreads();
        for (int t0 = 0; t0 < NTASK; t0 += T::NTHREADS) {
            const int t = t0 + tid;
            if (t >= NTASK) break;
            if (t < NFULL) {
                const int blk = t / D, dxi = t % D;
                const int bxl = blk % TB, byl = blk / TB;
                const int gbx = tx * TB + bxl, gby = ty * TB + byl;
                if (gbx < nbx && gby < nby) {
                    const uint64_t k = me_task<BS, SR>(win, T::WPD, cur, W, H, gbx * BS, gby * BS,
                                                      byl * BS, bxl * BS, dxi, r);
                    if (k != kNoKey) atomicMin(&keys[blk], (unsigned long long)k);
                }
            } else if constexpr (SUB) {
                const int s = (t - NFULL) / D, dxi = (t - NFULL) % D;
                const int blk = s >> 2, j = s & 3;
                const int bxl = blk % TB, byl = blk / TB;
                const int gbx = tx * TB + bxl, gby = ty * TB + byl;
                if (gbx < nbx && gby < nby) {
                    const int ox = (j & 1) * SB, oy = (j >> 1) * SB;
                    const uint64_t k = me_task<SB, SR>(win, T::WPD, cur, W, H, gbx * BS + ox,
                                                      gby * BS + oy, byl * BS + oy, bxl * BS + ox, dxi, r);
                    if (k != kNoKey) atomicMin(&keys[T::NBLK + s], (unsigned long long)k);
                }
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < T::NBLK * (SUB ? 5 : 1); i += T::NTHREADS) {
        const int blk = i < T::NBLK ? i : (i - T::NBLK) >> 2;
        const int gbx = tx * TB + blk % TB, gby = ty * TB + blk / TB;
        if (gbx >= nbx || gby >= nby) continue;
        const int b = gby * nbx + gbx;
        if (i < T::NBLK) decode_key(keys[i], SR, out_best + (size_t)b * 4);
        else decode_key(keys[i], SR, out_sub + ((size_t)b * 4 + ((i - T::NBLK) & 3)) * 4);
    }
}

// ---------------------------------------------------------------------------------------
// QSAD path (default): one wavefront per (sub-)block, current block in SGPRs.
//
// v_qsad_pk_u16_u8 D, S0(8 ref bytes), S1(4 cur bytes), S2 computes four SADs of S1
// against S0 at byte offsets 0..3 and accumulates them into four packed u16 (16 |diffs|
// per instruction, and the 4-byte-aligned window words need no byte alignment).  A
// 16x16 SAD is at most 65280, so u16 accumulators are exact.
// Lane (s, g), s < 7, g < 9: dx = 4g + i - 16 (i = 0..3), dy = 5s + t - 16 (t = 0..4):
// 63 lanes x 20 candidates >= 33 x 33; invalid slots are masked at the argmin.  The
// lane slides over its 5 + bs - 1 window rows; for every (row, cur row r) pair with
// t = row - r in range it issues bs/4 QSADs.  The current block is wave-uniform, so it
// lives in SGPRs (scalar loads) and feeds S1 directly.
// ---------------------------------------------------------------------------------------
// The current (sub-)block is wave-uniform: read it through the constant address space so
// the compiler issues scalar loads and keeps the pixels in SGPRs (QSAD operand S1).
typedef const __attribute__((address_space(4))) uint32_t* const_u32p;
template <int NR, int NDW>
SO_DEV void load_cur_sgpr(const uint8_t* __restrict__ cur, int W, int x, int y, uint32_t (&cr)[NR][NDW]) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const_u32p p = (const_u32p)(cur + (size_t)(y + r) * W + x);
#pragma unroll
        for (int k = 0; k < NDW; ++k) cr[r][k] = p[k];
    }
}

template <int TBS>
SO_DEV uint64_t me_qsad_task(const uint32_t* __restrict__ win, int wpd, const uint8_t* __restrict__ cur,
                             int lane, int W, int H, int x, int y, int wrow0, int wcol0, int ref) {
    constexpr int SR = 16, D = 33, NDW = TBS / 4, DYS = 5, NG = 9;
    constexpr int HALF = 8, NPASS = TBS / HALF, NROW = DYS + HALF - 1;
    // opaque per call: stops LICM from hoisting 20 per-lane key constants out of the
    // caller's block loop (they were kept live across it and spilled)
    asm volatile("" : "+v"(lane));
    const int s = lane / NG, g = lane - s * NG;
    uint64_t acc[DYS];
#pragma unroll
    for (int t = 0; t < DYS; ++t) acc[t] = 0;
    // the current rows are consumed in passes of 8 (<= 32 SGPRs live)
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
        uint32_t cr[HALF][NDW];
        load_cur_sgpr<HALF, NDW>(cur, W, x, y + pass * HALF, cr);
        const uint32_t* rowp = win + (wrow0 + DYS * s + pass * HALF) * wpd + (wcol0 >> 2) + g;
        // one window row in flight ahead of the one being consumed; the scheduling barrier
        // keeps the compiler from hoisting every row's loads (register pressure -> spills)
        uint32_t wc[NDW + 1], wn[NDW + 1];
#pragma unroll
        for (int k = 0; k <= NDW; ++k) wc[k] = rowp[k];
#pragma unroll
        for (int jj = 0; jj < NROW; ++jj) {
            if (jj + 1 < NROW) {
#pragma unroll
                for (int k = 0; k <= NDW; ++k) wn[k] = rowp[(jj + 1) * wpd + k];
            }
#pragma unroll
            for (int t = 0; t < DYS; ++t) {
                const int r = jj - t;
                if (r >= 0 && r < HALF) {
#pragma unroll
                    for (int k = 0; k < NDW; ++k)
                        acc[t] = __builtin_amdgcn_qsad_pk_u16_u8(((uint64_t)wc[k + 1] << 32) | wc[k], cr[r][k], acc[t]);
                }
            }
#pragma unroll
            for (int k = 0; k <= NDW; ++k) wc[k] = wn[k];
            // row fence: this row's QSADs are complete and the next-next row's loads have not
            // been hoisted above it (an IR-level barrier; sched_barrier alone is not)
            asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]) : : "memory");
        }
    }
    // no branch here: a branch around the epilogue lets the compiler sink every QSAD
    // into it and issue all window loads first (register pressure -> spills)
    const bool lane_ok = s < 7;
    uint64_t best = kNoKey;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int dxi = 4 * g + i, dx = dxi - SR;
        const bool xok = lane_ok && dxi < D && (x + dx >= 0) && (x + dx < W - TBS);
        const uint32_t adx = (uint32_t)(dx < 0 ? -dx : dx);
#pragma unroll
        for (int t = 0; t < DYS; ++t) {
            const int di = DYS * s + t, dy = di - SR;
            const bool ok = xok && di < D && (y + dy >= 0) && (y + dy < H - TBS);
            const uint32_t sad = (uint32_t)((acc[t] >> (16 * i)) & 0xFFFF);
            const uint64_t k = me_key(sad, adx + (uint32_t)(dy < 0 ? -dy : dy), (uint32_t)ref,
                                      (uint32_t)(dxi * D + di));
            best = (ok && k < best) ? k : best;
        }
    }
    return best;
}

SO_DEV uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) {
        const uint32_t lo = __shfl_xor((uint32_t)v, m, 64), hi = __shfl_xor((uint32_t)(v >> 32), m, 64);
        const uint64_t o = ((uint64_t)hi << 32) | lo;
        v = o < v ? o : v;
    }
    return v;
}

// The current (sub-)block is wave-uniform: read it through the constant address space so
// the compiler issues scalar loads and keeps the pixels in SGPRs (QSAD operand S1).
template <int BS, bool SUB>
__global__ void __launch_bounds__(1024)
me_qsad_kernel(const uint8_t* __restrict__ cur, RefSet refs, int nref, int H, int W,
               int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub) {
    using T = MeTile<BS>;
    constexpr int SR = T::SR, TB = T::TB, SB = BS / 2, NW = 16;
    __shared__ uint32_t win[T::WR * T::WPD];
    __shared__ unsigned long long keys[T::NBLK * (SUB ? 5 : 1)];
    const int nbx = W / BS, nby = H / BS;
    const int tiles_x = (nbx + TB - 1) / TB;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int x0 = tx * T::TPX, y0 = ty * T::TPX;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < T::NBLK * (SUB ? 5 : 1); i += NW * 64) keys[i] = kNoKey;
    constexpr int NUNIT = T::NBLK * (SUB ? 5 : 1);
    for (int r = 0; r < nref; ++r) {
        const uint8_t* ref = refs.p[r];
        __syncthreads();
        constexpr int WCD = T::WC / 4;
        for (int i = tid; i < T::WR * T::WPD; i += NW * 64) {
            const int wr = i / T::WPD, wc = i % T::WPD;
            const int gy = y0 - SR + wr, gx = x0 - SR + wc * 4;
            uint32_t v = 0;
            if (wc < WCD && gy >= 0 && gy < H && gx >= 0 && gx + 4 <= W)
                v = *reinterpret_cast<const uint32_t*>(ref + (size_t)gy * W + gx);
            win[i] = v;
        }
        __syncthreads();
        for (int u = wave; u < NUNIT; u += NW) {          // wave-uniform unit index
            if (u < T::NBLK) {
                const int bxl = u % TB, byl = u / TB;
                const int gbx = tx * TB + bxl, gby = ty * TB + byl;
                if (gbx >= nbx || gby >= nby) continue;
                uint64_t k = me_qsad_task<BS>(win, T::WPD, cur, lane, W, H, gbx * BS, gby * BS, byl * BS,
                                              bxl * BS, r);
                k = wave_min_u64(k);
                if (lane == 0 && k != kNoKey) atomicMin(&keys[u], (unsigned long long)k);
            } else if constexpr (SUB) {
                const int sidx = u - T::NBLK, blk = sidx >> 2, j = sidx & 3;
                const int bxl = blk % TB, byl = blk / TB;
                const int gbx = tx * TB + bxl, gby = ty * TB + byl;
                if (gbx >= nbx || gby >= nby) continue;
                const int ox = (j & 1) * SB, oy = (j >> 1) * SB;
                uint64_t k = me_qsad_task<SB>(win, T::WPD, cur, lane, W, H, gbx * BS + ox, gby * BS + oy,
                                              byl * BS + oy, bxl * BS + ox, r);
                k = wave_min_u64(k);
                if (lane == 0 && k != kNoKey) atomicMin(&keys[u], (unsigned long long)k);
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < NUNIT; i += NW * 64) {
        const int blk = i < T::NBLK ? i : (i - T::NBLK) >> 2;
        const int gbx = tx * TB + blk % TB, gby = ty * TB + blk / TB;
        if (gbx >= nbx || gby >= nby) continue;
        const int b = gby * nbx + gbx;
        if (i < T::NBLK) decode_key(keys[i], SR, out_best + (size_t)b * 4);
        else decode_key(keys[i], SR, out_sub + ((size_t)b * 4 + ((i - T::NBLK) & 3)) * 4);
    }
}

// ---------------------------------------------------------------------------------------
// Wave path (default): one wavefront per (sub-)block, current block in SGPRs, v_sad_u8.
//
// Measured on gfx950 (tools/ubench_sad.cpp): v_sad_u8 ~4.4 cycles per wave64 instruction
// (256 |diffs|) vs ~20.8 for v_qsad_pk_u16_u8 (1024 |diffs|), so plain v_sad_u8 it is.
// Phase 1: lane = hh*32 + xi: dx = xi - 16 (xi < 32), dy = 16*hh + t - 16 (t < 17), i.e.
// the two lane halves cover dy in [-16, 0] and [0, 16] (dy 0 twice).  The lane slides
// over its 17 + bs - 1 window rows and adds each aligned 4-byte group into acc[t] for
// every current row r = row - t (current pixels are wave-uniform SGPR operands).
// Phase 2: the dx = +16 column, lanes 0..32 one dy each, full SAD.
// VGPRs: 17 accumulators + one window row; PMC showed the per-lane-block kernel above
// waiting 47% of its time at 2.75 waves/SIMD, this one runs at up to 8 waves/SIMD.
// ---------------------------------------------------------------------------------------
template <int TBS>
SO_DEV uint64_t me_wave_task(const uint32_t* __restrict__ win, int wpd, const uint8_t* __restrict__ cur,
                             int lane, int W, int H, int x, int y, int wrow0, int wcol0, int ref) {
    constexpr int SR = 16, D = 33, NDW = TBS / 4, NT = 17;
    constexpr int HALF = 8, NPASS = TBS / HALF, NROW = NT + HALF - 1;   // <= 32 SGPRs of pixels live
    asm volatile("" : "+v"(lane));   // keep per-lane constants inside the caller's loop
    const int xi = lane & 31, hh = lane >> 5;
    uint32_t acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = 0;
    const int c = wcol0 + xi;
    const uint32_t sh = (uint32_t)(c & 3);
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
        uint32_t cr[HALF][NDW];
        load_cur_sgpr<HALF, NDW>(cur, W, x, y + pass * HALF, cr);
        const uint32_t* rowp = win + (wrow0 + 16 * hh + pass * HALF) * wpd + (c >> 2);
        uint32_t wc[NDW + 1], wn[NDW + 1];
#pragma unroll
        for (int k = 0; k <= NDW; ++k) wc[k] = rowp[k];
#pragma unroll
        for (int jj = 0; jj < NROW; ++jj) {
            if (jj + 1 < NROW) {   // one row in flight ahead of the row being consumed
#pragma unroll
                for (int k = 0; k <= NDW; ++k) wn[k] = rowp[(jj + 1) * wpd + k];
            }
            uint32_t rr[NDW];
#pragma unroll
            for (int k = 0; k < NDW; ++k) rr[k] = __builtin_amdgcn_alignbyte(wc[k + 1], wc[k], sh);
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int r = jj - t;
                if (r >= 0 && r < HALF) {
#pragma unroll
                    for (int k = 0; k < NDW; ++k) acc[t] = __builtin_amdgcn_sad_u8(cr[r][k], rr[k], acc[t]);
                }
            }
#pragma unroll
            for (int k = 0; k <= NDW; ++k) wc[k] = wn[k];
            // row fence (IR level): this row's SADs complete here and no later row's loads or
            // alignments are hoisted above it -- keeps VGPRs ~ 17 acc + 2 rows
            asm volatile("" : "+v"(acc[0]), "+v"(acc[1]), "+v"(acc[2]), "+v"(acc[3]), "+v"(acc[4]), "+v"(acc[5]),
                         "+v"(acc[6]), "+v"(acc[7]), "+v"(acc[8]), "+v"(acc[9]), "+v"(acc[10]), "+v"(acc[11]),
                         "+v"(acc[12]), "+v"(acc[13]), "+v"(acc[14]), "+v"(acc[15]), "+v"(acc[16]) : : "memory");
        }
    }
    uint64_t best = kNoKey;
    {
        const int dx = xi - SR;
        const bool xok = (x + dx >= 0) && (x + dx < W - TBS);
        const uint32_t adx = (uint32_t)(dx < 0 ? -dx : dx);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int di = 16 * hh + t, dy = di - SR;
            const bool ok = xok && (y + dy >= 0) && (y + dy < H - TBS);
            const uint64_t k = me_key(acc[t], adx + (uint32_t)(dy < 0 ? -dy : dy), (uint32_t)ref,
                                      (uint32_t)(xi * D + di));
            best = (ok && k < best) ? k : best;
        }
    }
    // phase 2: dx = +16, lane = di
    {
        const int di = lane < D ? lane : D - 1;
        const int c2 = wcol0 + 32;
        const uint32_t sh2 = (uint32_t)(c2 & 3);
        const uint32_t* rowp = win + (wrow0 + di) * wpd + (c2 >> 2);
        uint32_t a2 = 0;
#pragma unroll
        for (int pass = 0; pass < NPASS; ++pass) {
            uint32_t cr[HALF][NDW];
            load_cur_sgpr<HALF, NDW>(cur, W, x, y + pass * HALF, cr);
#pragma unroll
            for (int r = 0; r < HALF; ++r) {
                uint32_t w[NDW + 1];
#pragma unroll
                for (int k = 0; k <= NDW; ++k) w[k] = rowp[(pass * HALF + r) * wpd + k];
#pragma unroll
                for (int k = 0; k < NDW; ++k)
                    a2 = __builtin_amdgcn_sad_u8(cr[r][k], __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh2), a2);
            }
            asm volatile("" : "+v"(a2) : : "memory");
        }
        const int dx = SR, dy = di - SR;
        const bool ok = lane < D && (x + dx < W - TBS) && (y + dy >= 0) && (y + dy < H - TBS);
        const uint64_t k = me_key(a2, (uint32_t)(dx + (dy < 0 ? -dy : dy)), (uint32_t)ref, (uint32_t)(32 * D + di));
        best = (ok && k < best) ? k : best;
    }
    return best;
}

template <int BS, bool SUB>
__global__ void __launch_bounds__(512)
me_wave_kernel(const uint8_t* __restrict__ cur, RefSet refs, int nref, int H, int W,
               int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub) {
    constexpr int SR = 16, SB = BS / 2, NW = 8;
    constexpr int TBX = (BS == 16) ? 8 : 16, TBY = (BS == 16) ? 4 : 8;   // 128 x 64 px tile
    constexpr int WR = TBY * BS + 2 * SR, WC = TBX * BS + 2 * SR;
    constexpr int WPD = (WC + 16) / 4 + 1, WCD = WC / 4;
    constexpr int NBLK = TBX * TBY, NUNIT = NBLK * (SUB ? 5 : 1);
    __shared__ uint32_t win[WR * WPD];
    __shared__ unsigned long long keys[NUNIT];
    const int nbx = W / BS, nby = H / BS;
    const int tiles_x = (nbx + TBX - 1) / TBX;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int x0 = tx * TBX * BS, y0 = ty * TBY * BS;
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    for (int i = tid; i < NUNIT; i += NW * 64) keys[i] = kNoKey;
    for (int r = 0; r < nref; ++r) {
        const uint8_t* ref = refs.p[r];
        __syncthreads();
        for (int i = tid; i < WR * WPD; i += NW * 64) {
            const int wr = i / WPD, wc = i % WPD;
            const int gy = y0 - SR + wr, gx = x0 - SR + wc * 4;
            uint32_t v = 0;
            if (wc < WCD && gy >= 0 && gy < H && gx >= 0 && gx + 4 <= W)
                v = *reinterpret_cast<const uint32_t*>(ref + (size_t)gy * W + gx);
            win[i] = v;
        }
        __syncthreads();
        for (int u = wave; u < NUNIT; u += NW) {
            if (u < NBLK) {
                const int bxl = u % TBX, byl = u / TBX;
                const int gbx = tx * TBX + bxl, gby = ty * TBY + byl;
                if (gbx >= nbx || gby >= nby) continue;
                uint64_t k = me_wave_task<BS>(win, WPD, cur, lane, W, H, gbx * BS, gby * BS, byl * BS, bxl * BS, r);
                k = wave_min_u64(k);
                if (lane == 0 && k != kNoKey) atomicMin(&keys[u], (unsigned long long)k);
            } else if constexpr (SUB) {
                const int sidx = u - NBLK, blk = sidx >> 2, j = sidx & 3;
                const int bxl = blk % TBX, byl = blk / TBX;
                const int gbx = tx * TBX + bxl, gby = ty * TBY + byl;
                if (gbx >= nbx || gby >= nby) continue;
                const int ox = (j & 1) * SB, oy = (j >> 1) * SB;
                uint64_t k = me_wave_task<SB>(win, WPD, cur, lane, W, H, gbx * BS + ox, gby * BS + oy, byl * BS + oy,
                                              bxl * BS + ox, r);
                k = wave_min_u64(k);
                if (lane == 0 && k != kNoKey) atomicMin(&keys[u], (unsigned long long)k);
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < NUNIT; i += NW * 64) {
        const int blk = i < NBLK ? i : (i - NBLK) >> 2;
        const int gbx = tx * TBX + blk % TBX, gby = ty * TBY + blk / TBX;
        if (gbx >= nbx || gby >= nby) continue;
        const int b = gby * nbx + gbx;
        if (i < NBLK) decode_key(keys[i], SR, out_best + (size_t)b * 4);
        else decode_key(keys[i], SR, out_sub + ((size_t)b * 4 + ((i - NBLK) & 3)) * 4);
    }
}

// ---------------------------------------------------------------------------------------
// Generic path: one thread per (block, ref, candidate); keys in global memory.
// ---------------------------------------------------------------------------------------
// The generic path keeps each unit's key in the first 8 bytes of its own 16-byte output
// record (stride 2 in uint64 units) and decodes it in place at the end.
__global__ void me_generic_init(unsigned long long* keys, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) keys[2 * (size_t)i] = kNoKey;
}

__global__ void me_generic_kernel(const uint8_t* __restrict__ cur, RefSet refs, int nref, int H,
                                  int W, int bs, int sb_mode, int sr,
                                  unsigned long long* __restrict__ keys) {
    // sb_mode 0: full blocks (size bs); 1: sub-blocks (size bs/2, 4 per block)
    const int d = 2 * sr + 1;
    const int nbx = W / bs, nby = H / bs;
    const int nunit = nbx * nby * (sb_mode ? 4 : 1);
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long ntot = (long long)nunit * nref * d * d;
    if (t >= ntot) return;
    const int cand = (int)(t % (d * d));
    const int r = (int)((t / (d * d)) % nref);
    const int u = (int)(t / ((long long)d * d * nref));
    int b = sb_mode ? u >> 2 : u;
    const int tbs = sb_mode ? bs / 2 : bs;
    int x = (b % nbx) * bs, y = (b / nbx) * bs;
    if (sb_mode) { x += (u & 1) * tbs; y += ((u >> 1) & 1) * tbs; }
    const int dxi = cand / d, di = cand % d;
    const int dx = dxi - sr, dy = di - sr;
    if (!(x + dx >= 0 && x + dx < W - tbs && y + dy >= 0 && y + dy < H - tbs)) return;
    const uint8_t* ref = refs.p[r];
    uint32_t sad = 0;
    for (int i = 0; i < tbs; ++i)
        for (int j = 0; j < tbs; ++j) {
            int a = cur[(size_t)(y + i) * W + x + j], c = ref[(size_t)(y + dy + i) * W + x + dx + j];
            sad += (uint32_t)(a > c ? a - c : c - a);
        }
    const uint32_t l1 = (uint32_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy));
    atomicMin(&keys[2 * (size_t)u], (unsigned long long)me_key(sad, l1, (uint32_t)r, (uint32_t)cand));
}

__global__ void me_generic_finalize(int n, int sr, int32_t* __restrict__ out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const unsigned long long k = *reinterpret_cast<const unsigned long long*>(out + (size_t)i * 4);
        decode_key(k, sr, out + (size_t)i * 4);
    }
}

int me_launch(const uint8_t* cur, const RefSet& refs, int nref, int H, int W, int bs, int sr,
              int32_t* out_best, int32_t* out_sub, hipStream_t st) {
    const int nbx = W / bs, nby = H / bs;
    if (sr == 16 && (bs == 16 || bs == 8) && (out_sub == nullptr || bs == 16)) {
        // SO_ME_IMPL (A/B only): "wave" / "qsad" select the alternative kernels; default: v_sad_u8
        // per (block, dx) lane (fastest measured, tools/me_ab.py)
        const char* impl = getenv("SO_ME_IMPL");
        const bool use_wave = impl && strcmp(impl, "wave") == 0;
        const bool use_qsad = impl && strcmp(impl, "qsad") == 0;
        if (use_wave) {
            const int tbx = bs == 16 ? 8 : 16, tby = bs == 16 ? 4 : 8;
            const int tiles = ((nbx + tbx - 1) / tbx) * ((nby + tby - 1) / tby);
            if (bs == 16 && out_sub)
                hipLaunchKernelGGL((me_wave_kernel<16, true>), dim3(tiles), dim3(512), 0, st, cur, refs, nref, H, W,
                                   out_best, out_sub);
            else if (bs == 16)
                hipLaunchKernelGGL((me_wave_kernel<16, false>), dim3(tiles), dim3(512), 0, st, cur, refs, nref, H, W,
                                   out_best, out_sub);
            else
                hipLaunchKernelGGL((me_wave_kernel<8, false>), dim3(tiles), dim3(512), 0, st, cur, refs, nref, H, W,
                                   out_best, nullptr);
            return check_launch("me_wave_kernel");
        }
        if (use_qsad) {
            if (bs == 16) {
                using T = MeTile<16>;
                const int tiles = ((nbx + T::TB - 1) / T::TB) * ((nby + T::TB - 1) / T::TB);
                if (out_sub)
                    hipLaunchKernelGGL((me_qsad_kernel<16, true>), dim3(tiles), dim3(1024), 0, st, cur, refs, nref,
                                       H, W, out_best, out_sub);
                else
                    hipLaunchKernelGGL((me_qsad_kernel<16, false>), dim3(tiles), dim3(1024), 0, st, cur, refs, nref,
                                       H, W, out_best, out_sub);
            } else {
                using T = MeTile<8>;
                const int tiles = ((nbx + T::TB - 1) / T::TB) * ((nby + T::TB - 1) / T::TB);
                hipLaunchKernelGGL((me_qsad_kernel<8, false>), dim3(tiles), dim3(1024), 0, st, cur, refs, nref, H,
                                   W, out_best, nullptr);
            }
            return check_launch("me_qsad_kernel");
        }
        if (bs == 16) {
            using T = MeTile<16>;
            const int tiles = ((nbx + T::TB - 1) / T::TB) * ((nby + T::TB - 1) / T::TB);
            if (out_sub)
                hipLaunchKernelGGL((me_fast_kernel<16, true>), dim3(tiles), dim3(T::NTHREADS), 0, st,
                                   cur, refs, nref, H, W, out_best, out_sub);
            else
                hipLaunchKernelGGL((me_fast_kernel<16, false>), dim3(tiles), dim3(T::NTHREADS), 0, st,
                                   cur, refs, nref, H, W, out_best, out_sub);
        } else {
            using T = MeTile<8>;
            const int tiles = ((nbx + T::TB - 1) / T::TB) * ((nby + T::TB - 1) / T::TB);
            hipLaunchKernelGGL((me_fast_kernel<8, false>), dim3(tiles), dim3(T::NTHREADS), 0, st,
                               cur, refs, nref, H, W, out_best, nullptr);
        }
        return check_launch("me_fast_kernel");
    }
    // generic
    const int d = 2 * sr + 1;
    for (int mode = 0; mode < (out_sub ? 2 : 1); ++mode) {
        const int nunit = nbx * nby * (mode ? 4 : 1);
        int32_t* out = mode ? out_sub : out_best;
        unsigned long long* keys = reinterpret_cast<unsigned long long*>(out);
        hipLaunchKernelGGL(me_generic_init, dim3((nunit + 255) / 256), dim3(256), 0, st, keys, nunit);
        const long long ntot = (long long)nunit * nref * d * d;
        hipLaunchKernelGGL(me_generic_kernel, dim3((unsigned)((ntot + 255) / 256)), dim3(256), 0, st,
                           cur, refs, nref, H, W, bs, mode, sr, keys);
        hipLaunchKernelGGL(me_generic_finalize, dim3((nunit + 255) / 256), dim3(256), 0, st, nunit,
                           sr, out);
    }
    return check_launch("me_generic_kernel");
}

}  // namespace so
