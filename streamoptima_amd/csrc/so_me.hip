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
// Every kernel takes a block-row range [by0, by1) (stripe sharding across GPUs, DESIGN.md
// §5); output records are indexed relative to by0.
//
// Tile path (sr == 16, bs in {16, 8}; default): see me_tile_kernel.
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
// Tile path (default)
//
// A 704-thread workgroup (11 waves) owns a TB x TB tile of blocks (128 x 128 px).  It
// stages the current tile (128 x 128 B) and the reference window (tile + 16-px halo,
// 160 x 160 B) in LDS with coalesced 8-byte loads.  A task is (block, dx): 64 blocks x 33
// dx = 2112 tasks = exactly 3 rounds of 704 lanes.
//
// A lane walks its block's window rows: each row is 5 aligned ds_read_b32 + 4 v_alignbyte
// (win_read) and feeds up to 8 (cur row r, dy) pairs, each 4 v_sad_u8.  v_sad_u8 is the whole VALU budget: measured
// 4.39 cycles per wave64 instruction (tools/ubench_sad.cpp), the same issue cost as any
// other 32-bit VALU op, so the kernel is built to issue almost nothing else:
//   * the current block is held 8 rows at a time (two passes of 40 window rows), which
//     keeps ~80 VGPRs and 2 workgroups (22 waves) per CU so one tile's staging overlaps
//     the other's SADs;
//   * per-lane argmin on 32-bit keys (sad << 11 | |dy| << 6 | dy_index): one v_lshl_or
//     and one v_min per candidate (dx and ref are fixed within a lane, so the order of
//     these keys is the reference's order); dy bounds only for the frame's edge rows.
// The lane's best is widened to the 64-bit key and merged with an LDS atomicMin.
// With VBS the same launch also runs the 4 x 8x8 sub-block searches on the same window.
// ---------------------------------------------------------------------------------------
template <int BS>
struct MeGeo {
    static constexpr int SR = 16;
    static constexpr int D = 2 * SR + 1;                  // 33 candidates per axis
    static constexpr int TB = (BS == 16) ? 8 : 16;        // blocks per tile side
    static constexpr int TPX = TB * BS;                   // 128 px
    static constexpr int WP = TPX + 2 * SR;               // 160: window rows == pitch (bytes)
    static constexpr int CP = TPX;                        // current tile pitch
    static constexpr int NBLK = TB * TB;
    static constexpr int NTHREADS = 704;                  // 11 waves; 33 * 64 = 3 * 704
};

// Aligned LDS row read of N dwords (ds_read_b128 / ds_read_b64).
template <int N>
SO_DEV void lds_read(const uint8_t* p, uint32_t (&v)[N]) {
    if constexpr (N == 4) {
        const uint4 t = *reinterpret_cast<const uint4*>(p);
        v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    } else {
        const uint2 t = *reinterpret_cast<const uint2*>(p);
        v[0] = t.x; v[1] = t.y;
    }
}

// Window-row read of N dwords starting at ANY byte address p: aligned ds_read_b32 x (N+1)
// and N v_alignbyte.  Measured alternatives (tools/me_ab.py, 4K P-frame, same outputs):
// one byte-unaligned ds_read_b128 157.9 us, N byte-unaligned ds_read_b32 576.8 us -- gfx950
// replays misaligned DS reads (cdna_hip_programming.md Guideline 17) -- vs 111.9 us here.
template <int N>
SO_DEV void win_read(const uint8_t* p, uint32_t (&v)[N]) {
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3);
    const uint32_t* q = reinterpret_cast<const uint32_t*>(p - sh);   // keeps the LDS address space
    uint32_t w[N + 1];
#pragma unroll
    for (int k = 0; k <= N; ++k) w[k] = q[k];
#pragma unroll
    for (int k = 0; k < N; ++k) v[k] = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
}

// IR-level fence over the accumulators: the SADs of a window row are issued before any
// later row's LDS load is hoisted above them (bounds VGPRs to acc + cur + 2 rows).
template <int D>
SO_DEV void acc_fence(uint32_t (&a)[D]) {
    static_assert(D == 33, "fence written for 33 accumulators");
    asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                 "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]),
                 "+v"(a[14]), "+v"(a[15]), "+v"(a[16]) : : "memory");
    asm volatile("" : "+v"(a[17]), "+v"(a[18]), "+v"(a[19]), "+v"(a[20]), "+v"(a[21]), "+v"(a[22]),
                 "+v"(a[23]), "+v"(a[24]), "+v"(a[25]), "+v"(a[26]), "+v"(a[27]), "+v"(a[28]), "+v"(a[29]),
                 "+v"(a[30]), "+v"(a[31]), "+v"(a[32]) : : "memory");
}

// One task: (sub-)block of size TBS whose top-left sits at window (wrow, wcol - dxi) and
// current-tile (crow, ccol); wcol already includes dxi.  dy_index in [dlo, dhi] is valid.
// Returns the lane's best 32-bit key, 0xFFFFFFFF if no dy is valid.
template <int TBS, int WP, int CP>
SO_DEV uint32_t me_tile_task(const uint8_t* __restrict__ win, const uint8_t* __restrict__ curt, int wrow,
                             int wcol, int crow, int ccol, int dlo, int dhi) {
    constexpr int D = 33, NDW = TBS / 4, RCH = 8, NR = RCH + D - 1;
    uint32_t acc[D];
#pragma unroll
    for (int i = 0; i < D; ++i) acc[i] = 0;
#pragma unroll
    for (int c0 = 0; c0 < TBS; c0 += RCH) {
        uint32_t cr[RCH][NDW];
#pragma unroll
        for (int r = 0; r < RCH; ++r) lds_read<NDW>(curt + (crow + c0 + r) * CP + ccol, cr[r]);
        const uint8_t* p = win + (wrow + c0) * WP + wcol;
        uint32_t wc[NDW], wn[NDW];
        win_read<NDW>(p, wc);
#pragma unroll
        for (int jj = 0; jj < NR; ++jj) {
            if (jj + 1 < NR) win_read<NDW>(p + (jj + 1) * WP, wn);
#pragma unroll
            for (int r = 0; r < RCH; ++r) {
                const int di = jj - r;
                if (di >= 0 && di < D) {
#pragma unroll
                    for (int k = 0; k < NDW; ++k) acc[di] = __builtin_amdgcn_sad_u8(cr[r][k], wc[k], acc[di]);
                }
            }
#pragma unroll
            for (int k = 0; k < NDW; ++k) wc[k] = wn[k];
            acc_fence<D>(acc);
        }
    }
    uint32_t best = 0xFFFFFFFFu;
    if (dlo == 0 && dhi == D - 1) {
#pragma unroll
        for (int di = 0; di < D; ++di) {
            constexpr int SR = 16;
            const uint32_t low = (uint32_t)(((di < SR ? SR - di : di - SR) << 6) | di);
            const uint32_t k = (acc[di] << 11) | low;
            best = k < best ? k : best;
        }
    } else {
#pragma unroll
        for (int di = 0; di < D; ++di) {
            constexpr int SR = 16;
            const uint32_t low = (uint32_t)(((di < SR ? SR - di : di - SR) << 6) | di);
            uint32_t k = (acc[di] << 11) | low;
            k = (di < dlo || di > dhi) ? 0xFFFFFFFFu : k;
            best = k < best ? k : best;
        }
    }
    return best;
}

template <int BS, bool SUB>
__global__ void __launch_bounds__(MeGeo<BS>::NTHREADS) __attribute__((amdgpu_waves_per_eu(6)))
me_tile_kernel(const uint8_t* __restrict__ cur, RefSet refs, int nref, int H, int W, int by0, int by1,
               int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub) {
    using G = MeGeo<BS>;
    constexpr int SR = G::SR, D = G::D, TB = G::TB, SB = BS / 2, WP = G::WP, CP = G::CP;
    constexpr int NUNIT = G::NBLK * (SUB ? 5 : 1);
    __shared__ uint32_t win32[WP * WP / 4];
    __shared__ uint32_t cur32[G::TPX * CP / 4];
    __shared__ unsigned long long keys[NUNIT];
    uint8_t* win = reinterpret_cast<uint8_t*>(win32);
    uint8_t* curt = reinterpret_cast<uint8_t*>(cur32);

    const int nbx = W / BS;
    const int tiles_x = (nbx + TB - 1) / TB;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int bx0 = tx * TB, byt0 = by0 + ty * TB;       // first block of the tile
    const int x0 = bx0 * BS, y0 = byt0 * BS;
    const int tid = threadIdx.x;

    for (int i = tid; i < NUNIT; i += G::NTHREADS) keys[i] = kNoKey;
    // current tile: 128 rows x 16 chunks of 8 B (zero outside the frame)
    for (int i = tid; i < G::TPX * (CP / 8); i += G::NTHREADS) {
        const int r = i / (CP / 8), c = i % (CP / 8);
        const int gy = y0 + r, gx = x0 + c * 8;
        uint2 v = make_uint2(0, 0);
        if (gy < H && gx + 8 <= W) v = *reinterpret_cast<const uint2*>(cur + (size_t)gy * W + gx);
        *reinterpret_cast<uint2*>(curt + r * CP + c * 8) = v;
    }

    constexpr int NFULL = G::NBLK * D;
    constexpr int NSUBT = SUB ? 4 * G::NBLK * D : 0;
    constexpr int NTASK = NFULL + NSUBT;
    static_assert(NTASK % G::NTHREADS == 0, "tasks must fill whole rounds");

    for (int r = 0; r < nref; ++r) {
        const uint8_t* ref = refs.p[r];
        __syncthreads();  // previous reference's tasks are done with the window
        for (int i = tid; i < WP * (WP / 8); i += G::NTHREADS) {
            const int wr = i / (WP / 8), wc = i % (WP / 8);
            const int gy = y0 - SR + wr, gx = x0 - SR + wc * 8;
            uint2 v = make_uint2(0, 0);
            if (gy >= 0 && gy < H && gx >= 0 && gx + 8 <= W)
                v = *reinterpret_cast<const uint2*>(ref + (size_t)gy * W + gx);
            *reinterpret_cast<uint2*>(win + wr * WP + wc * 8) = v;
        }
        __syncthreads();
#pragma unroll 1
        for (int t = tid; t < NTASK; t += G::NTHREADS) {
            int unit, tbs, dxi, ox, oy, blk;
            if (t < NFULL) {
                blk = t / D; dxi = t - blk * D; unit = blk; tbs = BS; ox = 0; oy = 0;
            } else {
                const int s = (t - NFULL) / D;
                dxi = (t - NFULL) - s * D; blk = s >> 2; unit = G::NBLK + s; tbs = SB;
                ox = (s & 1) * SB; oy = ((s >> 1) & 1) * SB;
            }
            const int bxl = blk % TB, byl = blk / TB;
            if (bx0 + bxl >= nbx || byt0 + byl >= by1) continue;
            const int x = x0 + bxl * BS + ox, y = y0 + byl * BS + oy;
            int dlo = SR - y;               dlo = dlo < 0 ? 0 : dlo;
            int dhi = H - tbs - y + SR - 1; dhi = dhi > D - 1 ? D - 1 : dhi;
            const int wrow = byl * BS + oy, wcol = bxl * BS + ox + dxi;
            uint32_t b32;
            if (t < NFULL) b32 = me_tile_task<BS, WP, CP>(win, curt, wrow, wcol, wrow, bxl * BS + ox, dlo, dhi);
            else if constexpr (SUB) b32 = me_tile_task<SB, WP, CP>(win, curt, wrow, wcol, wrow, bxl * BS + ox, dlo, dhi);
            else b32 = 0xFFFFFFFFu;
            const int dx = dxi - SR;
            const bool xok = (x + dx >= 0) && (x + dx < W - tbs);
            if (xok && b32 != 0xFFFFFFFFu) {
                const uint32_t sad = b32 >> 11, ady = (b32 >> 6) & 31, di = b32 & 63;
                const uint32_t adx = (uint32_t)(dx < 0 ? -dx : dx);
                atomicMin(&keys[unit], (unsigned long long)me_key(sad, adx + ady, (uint32_t)r, (uint32_t)dxi * D + di));
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < NUNIT; i += G::NTHREADS) {
        const int blk = i < G::NBLK ? i : (i - G::NBLK) >> 2;
        const int gbx = bx0 + blk % TB, gby = byt0 + blk / TB;
        if (gbx >= nbx || gby >= by1) continue;
        const size_t b = (size_t)(gby - by0) * nbx + gbx;
        if (i < G::NBLK) decode_key(keys[i], SR, out_best + b * 4);
        else decode_key(keys[i], SR, out_sub + (b * 4 + ((i - G::NBLK) & 3)) * 4);
    }
}

// ---------------------------------------------------------------------------------------
// Round-1 kernel, kept for A/B (SO_ME_IMPL=fast): same tiling and tasks, but the current
// block lives whole in VGPRs (168 VGPRs, 1 workgroup per CU), window rows are aligned
// dword reads + v_alignbyte, and the argmin builds a 64-bit key per candidate.
// ---------------------------------------------------------------------------------------
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
__global__ void __launch_bounds__(MeGeo<BS>::NTHREADS)
me_fast_kernel(const uint8_t* __restrict__ cur, RefSet refs, int nref, int H, int W, int by0, int by1,
               int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub) {
    using G = MeGeo<BS>;
    constexpr int SR = G::SR, D = G::D, TB = G::TB, SB = BS / 2;
    constexpr int WPD = (G::WP + 16) / 4 + 1, WCD = G::WP / 4;
    __shared__ uint32_t win[G::WP * WPD];
    __shared__ unsigned long long keys[G::NBLK * (SUB ? 5 : 1)];

    const int nbx = W / BS;
    const int tiles_x = (nbx + TB - 1) / TB;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int bx0 = tx * TB, byt0 = by0 + ty * TB;
    const int x0 = bx0 * BS, y0 = byt0 * BS;
    const int tid = threadIdx.x;

    for (int i = tid; i < G::NBLK * (SUB ? 5 : 1); i += G::NTHREADS) keys[i] = kNoKey;

    constexpr int NFULL = G::NBLK * D;
    constexpr int NSUBT = SUB ? 4 * G::NBLK * D : 0;
    constexpr int NTASK = NFULL + NSUBT;

    for (int r = 0; r < nref; ++r) {
        const uint8_t* ref = refs.p[r];
        __syncthreads();
        for (int i = tid; i < G::WP * WPD; i += G::NTHREADS) {
            const int wr = i / WPD, wc = i % WPD;
            const int gy = y0 - SR + wr, gx = x0 - SR + wc * 4;
            uint32_t v = 0;
            if (wc < WCD && gy >= 0 && gy < H && gx >= 0 && gx + 4 <= W)
                v = *reinterpret_cast<const uint32_t*>(ref + (size_t)gy * W + gx);
            win[i] = v;
        }
        __syncthreads();
        for (int t0 = 0; t0 < NTASK; t0 += G::NTHREADS) {
            const int t = t0 + tid;
            if (t >= NTASK) break;
            if (t < NFULL) {
                const int blk = t / D, dxi = t % D;
                const int bxl = blk % TB, byl = blk / TB;
                if (bx0 + bxl < nbx && byt0 + byl < by1) {
                    const uint64_t k = me_task<BS, SR>(win, WPD, cur, W, H, x0 + bxl * BS, y0 + byl * BS,
                                                      byl * BS, bxl * BS, dxi, r);
                    if (k != kNoKey) atomicMin(&keys[blk], (unsigned long long)k);
                }
            } else if constexpr (SUB) {
                const int s = (t - NFULL) / D, dxi = (t - NFULL) % D;
                const int blk = s >> 2, j = s & 3;
                const int bxl = blk % TB, byl = blk / TB;
                if (bx0 + bxl < nbx && byt0 + byl < by1) {
                    const int ox = (j & 1) * SB, oy = (j >> 1) * SB;
                    const uint64_t k = me_task<SB, SR>(win, WPD, cur, W, H, x0 + bxl * BS + ox,
                                                      y0 + byl * BS + oy, byl * BS + oy, bxl * BS + ox, dxi, r);
                    if (k != kNoKey) atomicMin(&keys[G::NBLK + s], (unsigned long long)k);
                }
            }
        }
    }
    __syncthreads();
    for (int i = tid; i < G::NBLK * (SUB ? 5 : 1); i += G::NTHREADS) {
        const int blk = i < G::NBLK ? i : (i - G::NBLK) >> 2;
        const int gbx = bx0 + blk % TB, gby = byt0 + blk / TB;
        if (gbx >= nbx || gby >= by1) continue;
        const size_t b = (size_t)(gby - by0) * nbx + gbx;
        if (i < G::NBLK) decode_key(keys[i], SR, out_best + b * 4);
        else decode_key(keys[i], SR, out_sub + (b * 4 + ((i - G::NBLK) & 3)) * 4);
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
                                  int W, int bs, int by0, int nrows, int sb_mode, int sr,
                                  unsigned long long* __restrict__ keys) {
    // sb_mode 0: full blocks (size bs); 1: sub-blocks (size bs/2, 4 per block)
    const int d = 2 * sr + 1;
    const int nbx = W / bs;
    const int nunit = nbx * nrows * (sb_mode ? 4 : 1);
    const long long t = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long ntot = (long long)nunit * nref * d * d;
    if (t >= ntot) return;
    const int cand = (int)(t % (d * d));
    const int r = (int)((t / (d * d)) % nref);
    const int u = (int)(t / ((long long)d * d * nref));
    int b = sb_mode ? u >> 2 : u;
    const int tbs = sb_mode ? bs / 2 : bs;
    int x = (b % nbx) * bs, y = (by0 + b / nbx) * bs;
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

int me_launch(const uint8_t* cur, const RefSet& refs, int nref, int H, int W, int bs, int sr, int by0, int by1,
              int32_t* out_best, int32_t* out_sub, hipStream_t st) {
    const int nbx = W / bs, nrows = by1 - by0;
    if (nrows <= 0) return SO_OK;
    if (sr == 16 && (bs == 16 || bs == 8) && (out_sub == nullptr || bs == 16)) {
        // SO_ME_IMPL=fast selects the round-1 kernel (A/B only, tools/me_ab.py)
        const char* impl = getenv("SO_ME_IMPL");
        const bool use_fast = impl && strcmp(impl, "fast") == 0;
        const int tb = bs == 16 ? MeGeo<16>::TB : MeGeo<8>::TB;
        const dim3 grid(((nbx + tb - 1) / tb) * ((nrows + tb - 1) / tb)), blk(MeGeo<16>::NTHREADS);
        if (use_fast) {
            if (bs == 16 && out_sub)
                hipLaunchKernelGGL((me_fast_kernel<16, true>), grid, blk, 0, st, cur, refs, nref, H, W, by0, by1,
                                   out_best, out_sub);
            else if (bs == 16)
                hipLaunchKernelGGL((me_fast_kernel<16, false>), grid, blk, 0, st, cur, refs, nref, H, W, by0, by1,
                                   out_best, out_sub);
            else
                hipLaunchKernelGGL((me_fast_kernel<8, false>), grid, blk, 0, st, cur, refs, nref, H, W, by0, by1,
                                   out_best, nullptr);
            return check_launch("me_fast_kernel");
        }
        if (bs == 16 && out_sub)
            hipLaunchKernelGGL((me_tile_kernel<16, true>), grid, blk, 0, st, cur, refs, nref, H, W, by0, by1,
                               out_best, out_sub);
        else if (bs == 16)
            hipLaunchKernelGGL((me_tile_kernel<16, false>), grid, blk, 0, st, cur, refs, nref, H, W, by0, by1,
                               out_best, out_sub);
        else
            hipLaunchKernelGGL((me_tile_kernel<8, false>), grid, blk, 0, st, cur, refs, nref, H, W, by0, by1,
                               out_best, nullptr);
        return check_launch("me_tile_kernel");
    }
    // generic
    const int d = 2 * sr + 1;
    for (int mode = 0; mode < (out_sub ? 2 : 1); ++mode) {
        const int nunit = nbx * nrows * (mode ? 4 : 1);
        int32_t* out = mode ? out_sub : out_best;
        unsigned long long* keys = reinterpret_cast<unsigned long long*>(out);
        hipLaunchKernelGGL(me_generic_init, dim3((nunit + 255) / 256), dim3(256), 0, st, keys, nunit);
        const long long ntot = (long long)nunit * nref * d * d;
        hipLaunchKernelGGL(me_generic_kernel, dim3((unsigned)((ntot + 255) / 256)), dim3(256), 0, st,
                           cur, refs, nref, H, W, bs, by0, nrows, mode, sr, keys);
        hipLaunchKernelGGL(me_generic_finalize, dim3((nunit + 255) / 256), dim3(256), 0, st, nunit,
                           sr, out);
    }
    return check_launch("me_generic_kernel");
}

}  // namespace so
