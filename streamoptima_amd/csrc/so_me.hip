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
// Wave path (sr == 16, bs in {16, 8}; default): see me_wave_kernel.
// Generic path (any sr <= 64): one thread per (block, candidate) with a global atomicMin.
#include <stdlib.h>
#include <string.h>

#include <cstring>
#include <map>
#include <mutex>
#include <utility>

#include "so_block.h"
#include "so_common.h"
#include "so_dpp.h"
#include "so_run.h"

namespace so {

SO_DEV uint64_t me_key(uint32_t sad, uint32_t l1, uint32_t ref, uint32_t scan) {
    return ((uint64_t)sad << 32) | ((uint64_t)l1 << 24) | ((uint64_t)ref << 16) | (uint64_t)scan;
}
constexpr uint64_t kNoKey = ~0ull;
// SAD byte operations of one wave_dense_block at bs 16 (2 passes x (17 x 8 + 8) x 4 v_sad_u8
// per lane, 64 lanes, 4 bytes each)
constexpr uint32_t kDenseSadOps = 1152u * 256u;
// only when the run counts (SO_OPT_COUNT_SAD_OPS: bench.py's roofline replay); a uniform
// branch otherwise (the count's LDS atomics cost ~1 % of the P-run)
#define SO_OPS_ADD(p, v) do { if (L.count_ops) atomicAdd((p), (v)); } while (0)

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
// Wave path (default): one wavefront per block, current block in SGPRs, no v_alignbyte.
//
// gfx950 issue costs (tools/ubench_ops.cpp): every VOP3 instruction -- v_sad_u8,
// v_alignbyte_b32, v_add3_u32 -- costs ~4.4 cycles per wave64, a VOP2 v_add ~2.5.  So the
// kernel minimises VOP3 instructions other than v_sad_u8:
//   * the block is wave-uniform: its pixels live in SGPRs (scalar loads, 8 rows per pass)
//     and feed v_sad_u8 directly, so lanes hold only accumulators and one window row;
//   * the window is staged in LDS as FOUR copies shifted by 0..3 bytes, so the 16 bytes at
//     any column are four dword-aligned ds_read_b32 from copy (col & 3) -- the byte
//     alignment is paid once per staged dword instead of once per row per lane (a b128 read
//     would need 16-byte alignment: misaligned wide DS reads are replayed on gfx950);
//   * copy strides are 8 (mod 32) dwords, so the 32-lane b32 reads are bank-conflict free.
// Phase 1: lane = hh*32 + xi covers dx = xi - 16 (xi < 32) and dy = 16*hh + t - 16
// (t < 17): the halves take dy in [-16, 0] and [0, 16] (dy 0 twice, 3% redundant).  The
// lane slides over its 17 + 8 - 1 window rows per pass and adds every row into the t it
// pairs with.  Phase 2: the dx = +16 column, lane = dy index (33 lanes), whose column is
// 4-byte aligned (copy 0).
// VBS: the lane keeps left/right-quadrant accumulators per pass (dwords 0-1 / 2-3), so
// the 8x8 sub-block SADs come out of the same v_sad_u8 work and the 16x16 SAD is their sum.
// Argmin: per-lane 32-bit keys (sad << 5 | ordered |dy| code), widened to the 64-bit key
// and reduced across the wave.
// ---------------------------------------------------------------------------------------
// Tile geometry.  Without VBS a lane needs ~40 VGPRs, so LDS sets the occupancy: a 128 x 64
// tile (96-row window, 4 copies = 62 KB) with 16 waves gives 2 workgroups = 8 waves/SIMD.
// With VBS (~126 VGPRs, 4 waves/SIMD) a 128 x 32 tile with 8 waves.
template <int BS, bool SUB>
struct MeWGeo {
    static constexpr int SR = 16, D = 33, NT = 17;
    static constexpr int TBX = 128 / BS;                  // blocks across (128 px)
    static constexpr int TPY = SUB ? 32 : 64;             // pixel rows per tile
    static constexpr int TBY = TPY / BS;
    static constexpr int TPX = 128;
    static constexpr int WR = TPY + 2 * SR;               // window rows
    // copy row pitch: 40 dwords of window + 1 pad, so reads that walk down a column (dy
    // lanes, survivor rows) hit 32 different banks (41 r mod 32) instead of 4 (40 r mod 32)
    static constexpr int RPD = (TPX + 2 * SR) / 4 + 1;
    // dwords per shifted copy: CSTRIDE = 8 (mod 32) puts the four copies 8 banks apart, so a
    // 32-lane ds_read_b32 (bank = dword mod 32) of lanes xi hits 8*(xi&3) + (xi>>2): no conflict
    static constexpr int CSTRIDE = WR * RPD + 8;
    static constexpr int NBLK = TBX * TBY;
    static constexpr int NW = SUB ? 8 : 16, NTHREADS = NW * 64;
};

typedef const __attribute__((address_space(4))) uint32_t* const_u32p;
// LDS pointer type for volatile reads (address-space inference skips volatile accesses)
typedef const volatile __attribute__((address_space(3))) uint32_t* lds_vu32p;

// NR rows x NDW dwords of the current block into SGPRs (wave-uniform address).
template <int NR, int NDW>
SO_DEV void load_cur_sgpr(const uint8_t* __restrict__ cur, int W, int x, int y, uint32_t (&cr)[NR][NDW]) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        const_u32p p = (const_u32p)(cur + (size_t)(y + r) * W + x);
#pragma unroll
        for (int k = 0; k < NDW; ++k) cr[r][k] = p[k];
    }
}


// Stage a WR x (4 RPD) byte window of `ref` at (gx0, gy0) into LDS as four copies shifted
// by 0..3 bytes (copy s, row r, dword m = window bytes [4m + s, 4m + s + 4); zero outside
// the frame).  Every thread issues all its global loads before any LDS store, so a
// workgroup pays one memory latency for the window instead of one per loop trip.
template <int WR, int RPD, int CS, int NT>
SO_DEV void stage_window(uint32_t* win, const uint8_t* __restrict__ ref, int H, int W, int gx0, int gy0, int tid) {
    constexpr int N = WR * RPD, IT = (N + NT - 1) / NT;
    uint32_t a[IT], b[IT];
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int i = tid + k * NT;
        const int wr = i / RPD, m = i - wr * RPD;
        const int gy = gy0 + wr, gx = gx0 + 4 * m;
        a[k] = 0;
        b[k] = 0;
        if (i < N && gy >= 0 && gy < H) {
            const uint8_t* rp = ref + (size_t)gy * W;
            if (gx >= 0 && gx + 4 <= W) a[k] = *reinterpret_cast<const uint32_t*>(rp + gx);
            if (gx + 4 >= 0 && gx + 8 <= W) b[k] = *reinterpret_cast<const uint32_t*>(rp + gx + 4);
        }
    }
#pragma unroll
    for (int k = 0; k < IT; ++k) {
        const int i = tid + k * NT;
        if (i < N) {
            uint32_t* d = win + i;     // == wr * RPD + m
            d[0] = a[k];
            d[CS] = __builtin_amdgcn_alignbyte(b[k], a[k], 1);
            d[2 * CS] = __builtin_amdgcn_alignbyte(b[k], a[k], 2);
            d[3 * CS] = __builtin_amdgcn_alignbyte(b[k], a[k], 3);
        }
    }
}

template <int N>
SO_DEV void acc_fence_n(uint32_t (&a)[N]) {
    static_assert(N == 17, "fence written for 17 accumulators");
    asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                 "+v"(a[7]), "+v"(a[8]), "+v"(a[9]), "+v"(a[10]), "+v"(a[11]), "+v"(a[12]), "+v"(a[13]),
                 "+v"(a[14]), "+v"(a[15]), "+v"(a[16]) : : "memory");
}

// Lane's best 32-bit key over its 17 phase-1 candidates t: (sad << 5) | (t ^ X), where
// X = 31 for the dy <= 0 half (|dy| = 16 - t) and 0 for the other (|dy| = t) -- within a
// lane dx and ref are fixed, so (sad, this code) orders exactly like (sad, |dx|+|dy|, scan).
// di valid in [dlo, dhi] (di = 16*hh + t); `edge` selects the masked form.
// `ex16`: drop t = 16 of the lower half (the duplicate dy = 0 row) -- the FME row phase
// a = 1 maps it to dy = +1 half-pel, which the upper half's t = 0 already covers, and
// keeping it would break the lane's |dy| order (|-1| == |+1| at t = 15 and t = 16).
// HALF: the SAD is the whole accumulator (0), its low 16 bits (1) or its high 16 bits (2) --
// the VBS dense search keeps a lane's left / right quadrant SADs packed in one register.
template <int HALF = 0>
SO_DEV uint32_t half16(uint32_t v) {
    return HALF == 0 ? v : HALF == 1 ? (v & 0xFFFFu) : (v >> 16);
}
template <int HALF = 0>
SO_DEV uint32_t lane_best17(const uint32_t (&a)[17], uint32_t X, int hh, int dlo, int dhi, bool edge,
                            bool ex16 = false) {
    uint32_t best = 0xFFFFFFFFu;
    if (!edge) {
#pragma unroll
        for (int t = 0; t < 17; ++t) {
            const uint32_t k = ((half16<HALF>(a[t]) << 5) | (uint32_t)t) ^ X;
            best = k < best ? k : best;
        }
    } else {
#pragma unroll
        for (int t = 0; t < 17; ++t) {
            const int di = 16 * hh + t;
            uint32_t k = ((half16<HALF>(a[t]) << 5) | (uint32_t)t) ^ X;
            k = (di < dlo || di > dhi || (t == 16 && ex16 && hh == 0)) ? 0xFFFFFFFFu : k;
            best = k < best ? k : best;
        }
    }
    return best;
}

// ---- FME (FMEEnable, Encoder.py:388-403, 697-705, 1647-1651) ---------------------------------
// The frac frame F ((2H-1) x (2W-1)) is searched at (2x, 2y) over half-pel offsets in
// [-2sr, 2sr] with the block sampled every other row and column.  Candidate (dxh, dyh)
// reads F[2y+dyh+2i][2x+dxh+2j] = P_ab[y+v+i][x+u+j] with dyh = 2v+a, dxh = 2u+b and the
// phase planes P_ab[i][j] = F[2i+a][2j+b] (so_fme_planes).  So the half-pel search is four
// integer-pel searches (u, v in [-16, 16]) over the four planes, with a candidate map:
//   valid   |dxh| <= 2sr and 0 <= 2x+dxh <= 2W-3bs-2 (the reference's strict bound plus
//           its FME bound 0 <= X+dx+2bs < W2-bs, :698); the same for y;
//   key     (SAD, |dxh|+|dyh|, ref, (dxh+2sr)(4sr+1)+(dyh+2sr)), decoded with sr' = 2sr.
struct FmePhase {
    int a, b;
};

SO_DEV bool fme_xok(int x, int dxi, int b, int W, int bsz) {
    const int dxh = 2 * (dxi - 16) + b;
    return dxh >= -32 && dxh <= 32 && 2 * x + dxh >= 0 && 2 * x + dxh <= 2 * W - 3 * bsz - 2;
}

// valid dy indices di in [dlo, dhi] (dyh = 2(di-16)+a)
SO_DEV void fme_drange(int y, int a, int H, int bsz, int& dlo, int& dhi) {
    int lo = -2 * y;             lo = lo < -32 ? -32 : lo;
    int hi = 2 * H - 3 * bsz - 2 - 2 * y; hi = hi > 32 ? 32 : hi;
    dlo = (lo + 33 - a) >> 1;    // ceil((lo + 32 - a) / 2)
    dhi = (hi + 32 - a) >> 1;    // floor, arithmetic shift
}

SO_DEV uint64_t fme_key(uint32_t sad, int dxi, int di, FmePhase ph, int ref) {
    const int dxh = 2 * (dxi - 16) + ph.b, dyh = 2 * (di - 16) + ph.a;
    const uint32_t l1 = (uint32_t)((dxh < 0 ? -dxh : dxh) + (dyh < 0 ? -dyh : dyh));
    return me_key(sad, l1, (uint32_t)ref, (uint32_t)((dxh + 32) * 65 + (dyh + 32)));
}

// Widen a lane's phase-1 best to the 64-bit reference key (kNoKey if none / dx invalid).
SO_DEV uint64_t widen17(uint32_t b32, uint32_t X, int hh, int xi, bool xok, int ref) {
    if (!xok || b32 == 0xFFFFFFFFu) return kNoKey;
    const uint32_t t = (b32 & 31) ^ X, sad = b32 >> 5;
    const int di = 16 * hh + (int)t, dy = di - 16, dx = xi - 16;
    const uint32_t l1 = (uint32_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy));
    return me_key(sad, l1, (uint32_t)ref, (uint32_t)(xi * 33 + di));
}

SO_DEV uint64_t widen17_fme(uint32_t b32, uint32_t X, int hh, int xi, bool xok, int ref, FmePhase ph) {
    if (!xok || b32 == 0xFFFFFFFFu) return kNoKey;
    const uint32_t t = (b32 & 31) ^ X, sad = b32 >> 5;
    return fme_key(sad, xi, 16 * hh + (int)t, ph, ref);
}

// Dense search of one block by one wavefront (phase 1 + phase 2 over the four shifted
// window copies in `win`); merges the block key into keys[u] and, with VBS, the quadrant
// keys into keys[nblk + 4u + j].  Used by me_wave_kernel.
// ONE: the window is a single copy (me_sea2_kernel): the lane's 16 bytes at any column are
// five ds_read_b32 + four v_alignbyte per row instead of four reads of its shifted copy.
// `c1` (dwords from win): copies 1..3 at win + c1 + (s - 1) CS instead of win + s CS (the
// fused tile's dense tiles keep copy 0 in the window and stage the others into its scratch).
template <int BS, bool SUB, int RPD, int CS, bool FME = false, bool ONE = false>
SO_DEV void wave_dense_block(const uint32_t* win, unsigned long long* keys, int nblk, const uint8_t* __restrict__ cur,
                             int W, int H, int x, int y, int bxl, int byl, int u, int tid, int r,
                             FmePhase ph = FmePhase{0, 0}, int c1 = CS) {
    constexpr int SR = 16, NT = 17;
    constexpr int NDW = BS / 4, HALF = 8, NPASS = BS / HALF, NR = NT + HALF - 1;
    // lane identity re-derived per block through an opaque asm: otherwise LICM hoists
    // the ~17 per-lane (16*hh + t) edge constants out of this loop and spills them
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int xi = lane & 31, hh = lane >> 5;
    const uint32_t X = hh ? 0u : 31u;
    // phase-1 lane: window column bxl*BS + xi (dx = xi - 16) in copy xi & 3
    const int q1 = (ONE || (xi & 3) == 0 ? 0 : c1 + ((xi & 3) - 1) * CS) + (byl * BS + 16 * hh) * RPD +
                   ((bxl * BS + xi) >> 2);
    const uint32_t sh1 = (uint32_t)((bxl * BS + xi) & 3);   // ONE: byte shift of the lane's column
    // phase-2 lane: dx = +16 (column bxl*BS + 32, copy 0), dy index = lane (< 33)
    const int d2 = lane < 33 ? lane : 32;
    const int q2 = (byl * BS + d2) * RPD + ((bxl * BS + 32) >> 2);
    // VBS (SUB): acc[t] = left-quadrant SAD | right-quadrant SAD << 16 (v_sad_u8 / v_sad_hi_u8;
    // an 8 x 8 SAD is < 2^14) and S[t] the packed sum over both passes (< 2^15 per half): 34
    // accumulators instead of 51 live through the scan
    uint32_t accL[NT], S[NT];
    uint32_t a2L[NPASS], a2R[NPASS];
#pragma unroll
    for (int t = 0; t < NT; ++t) S[t] = 0;
    uint32_t subb[4];          // VBS: lane best 32-bit key per quadrant (phase 1)
    uint32_t sub2[4];          // VBS: phase-2 quadrant SADs
#pragma unroll
    for (int pass = 0; pass < NPASS; ++pass) {
        // the row index goes through an opaque asm so this pass's scalar loads cannot
        // be hoisted above the previous pass (constant-space loads are otherwise free
        // to move, and two passes of pixels overflow the SGPRs)
        int ycur = y + pass * HALF;
        asm volatile("" : "+s"(ycur));
        uint32_t cr[HALF][NDW];
        load_cur_sgpr<HALF, NDW>(cur, W, x, ycur, cr);
        if (SUB || pass == 0) {   // without VBS accL accumulates the whole block
#pragma unroll
            for (int t = 0; t < NT; ++t) accL[t] = 0;
        }
        // phase 1: rows pass*8 + jj of the lane's 24-row strip
        // volatile: the four dwords stay four ds_read_b32 -- merged into one b128 they
        // are 4-byte but not 16-byte aligned and the LDS replays them (Guideline 17)
        int qo = q1 + pass * HALF * RPD;       // dword offsets into win[] keep the LDS
        asm volatile("" : "+v"(qo));           // address space through the opaque asm
        lds_vu32p qp = (lds_vu32p)(win + qo);
        uint32_t wc[NDW], wn[NDW];
        if constexpr (ONE) {
            uint32_t t[NDW + 1];
#pragma unroll
            for (int k = 0; k <= NDW; ++k) t[k] = qp[k];
#pragma unroll
            for (int k = 0; k < NDW; ++k) wc[k] = __builtin_amdgcn_alignbyte(t[k + 1], t[k], sh1);
        } else {
#pragma unroll
            for (int k = 0; k < NDW; ++k) wc[k] = qp[k];
        }
#pragma unroll
        for (int jj = 0; jj < NR; ++jj) {
            if (jj + 1 < NR) {
                if constexpr (ONE) {
                    uint32_t t[NDW + 1];
#pragma unroll
                    for (int k = 0; k <= NDW; ++k) t[k] = qp[(jj + 1) * RPD + k];
#pragma unroll
                    for (int k = 0; k < NDW; ++k) wn[k] = __builtin_amdgcn_alignbyte(t[k + 1], t[k], sh1);
                } else {
#pragma unroll
                    for (int k = 0; k < NDW; ++k) wn[k] = qp[(jj + 1) * RPD + k];
                }
            }
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                const int rr = jj - t;
                if (rr >= 0 && rr < HALF) {
#pragma unroll
                    for (int k = 0; k < NDW; ++k) {
                        if (SUB && k >= NDW / 2) accL[t] = __builtin_amdgcn_sad_hi_u8(cr[rr][k], wc[k], accL[t]);
                        else accL[t] = __builtin_amdgcn_sad_u8(cr[rr][k], wc[k], accL[t]);
                    }
                }
            }
#pragma unroll
            for (int k = 0; k < NDW; ++k) wc[k] = wn[k];
            acc_fence_n<NT>(accL);
        }
        // phase 2: the dx = +16 candidate of dy index d2, rows pass*8 .. +8
        uint32_t l2 = 0, r2 = 0;
        int q2o = q2 + pass * HALF * RPD;
        asm volatile("" : "+v"(q2o));   // phase-2 reads stay after phase 1
        lds_vu32p q2p = (lds_vu32p)(win + q2o);
#pragma unroll
        for (int rr = 0; rr < HALF; ++rr) {
            lds_vu32p w2 = q2p + rr * RPD;
#pragma unroll
            for (int k = 0; k < NDW; ++k) {
                if (SUB && k >= NDW / 2) r2 = __builtin_amdgcn_sad_u8(cr[rr][k], w2[k], r2);
                else l2 = __builtin_amdgcn_sad_u8(cr[rr][k], w2[k], l2);
            }
            asm volatile("" : "+v"(l2), "+v"(r2) : : "memory");   // one row in flight
        }
        a2L[pass] = l2;
        a2R[pass] = r2;
        if constexpr (SUB) {
            // quadrants (pass 0: TL, TR; pass 1: BL, BR) -- per-lane bests now, the
            // accumulators are reused by the next pass
            const int ys = y + pass * HALF;
            int dlo, dhi;
            if constexpr (FME) {
                fme_drange(ys, ph.a, H, 8, dlo, dhi);
            } else {
                dlo = SR - ys;          dlo = dlo < 0 ? 0 : dlo;
                dhi = H - 8 - ys + SR - 1; dhi = dhi > 32 ? 32 : dhi;
            }
            const bool edge = FME || dlo > 0 || dhi < 32;
            subb[2 * pass] = lane_best17<1>(accL, X, hh, dlo, dhi, edge, FME && ph.a);
            subb[2 * pass + 1] = lane_best17<2>(accL, X, hh, dlo, dhi, edge, FME && ph.a);
            sub2[2 * pass] = l2;
            sub2[2 * pass + 1] = r2;
#pragma unroll
            for (int t = 0; t < NT; ++t) S[t] += accL[t];
        }
    }
    if constexpr (!SUB) {
#pragma unroll
        for (int t = 0; t < NT; ++t) S[t] = accL[t];
    } else {
#pragma unroll
        for (int t = 0; t < NT; ++t) S[t] = (S[t] & 0xFFFFu) + (S[t] >> 16);
    }
    // block keys: phase 1 (lane's 17 candidates) and phase 2 (dx = +16)
    int dlo, dhi;
    bool xok, x2ok;
    if constexpr (FME) {
        fme_drange(y, ph.a, H, BS, dlo, dhi);
        xok = fme_xok(x, xi, ph.b, W, BS);
        x2ok = fme_xok(x, 32, ph.b, W, BS);
    } else {
        dlo = SR - y;            dlo = dlo < 0 ? 0 : dlo;
        dhi = H - BS - y + SR - 1; dhi = dhi > 32 ? 32 : dhi;
        xok = (x + xi - 16 >= 0) && (x + xi - 16 < W - BS);
        x2ok = x + 16 < W - BS;
    }
    const bool edge = FME || dlo > 0 || dhi < 32;
    const uint32_t lb = lane_best17(S, X, hh, dlo, dhi, edge, FME && ph.a);
    uint64_t k;
    if constexpr (FME) k = widen17_fme(lb, X, hh, xi, xok, r, ph);
    else k = widen17(lb, X, hh, xi, xok, r);
    {
        uint32_t s2 = 0;
#pragma unroll
        for (int pass = 0; pass < NPASS; ++pass) s2 += a2L[pass] + a2R[pass];
        const bool ok2 = lane < 33 && x2ok && d2 >= dlo && d2 <= dhi;
        uint64_t k2 = kNoKey;
        if constexpr (FME) {
            if (ok2) k2 = fme_key(s2, 32, d2, ph, r);
        } else {
            if (ok2) k2 = me_key(s2, (uint32_t)(16 + (d2 < 16 ? 16 - d2 : d2 - 16)), (uint32_t)r, (uint32_t)(32 * 33 + d2));
        }
        k = k2 < k ? k2 : k;
    }
    k = wave_min_u64(k);
    if (lane == 0 && k < keys[u]) keys[u] = k;
    if constexpr (SUB) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int xs = x + (j & 1) * 8, ys = y + (j >> 1) * 8;
            uint64_t ks, k2 = kNoKey;
            if constexpr (FME) {
                int sdlo, sdhi;
                fme_drange(ys, ph.a, H, 8, sdlo, sdhi);
                ks = widen17_fme(subb[j], X, hh, xi, fme_xok(xs, xi, ph.b, W, 8), r, ph);
                if (lane < 33 && fme_xok(xs, 32, ph.b, W, 8) && d2 >= sdlo && d2 <= sdhi) k2 = fme_key(sub2[j], 32, d2, ph, r);
            } else {
                const bool sxok = (xs + xi - 16 >= 0) && (xs + xi - 16 < W - 8);
                ks = widen17(subb[j], X, hh, xi, sxok, r);
                const bool ok2 = lane < 33 && (xs + 16 < W - 8) && (ys + d2 - 16 >= 0) && (ys + d2 - 16 < H - 8);
                if (ok2) k2 = me_key(sub2[j], (uint32_t)(16 + (d2 < 16 ? 16 - d2 : d2 - 16)), (uint32_t)r,
                                     (uint32_t)(32 * 33 + d2));
            }
            ks = k2 < ks ? k2 : ks;
            ks = wave_min_u64(ks);
            if (lane == 0 && ks < keys[nblk + 4 * u + j]) keys[nblk + 4 * u + j] = ks;
        }
    }
}

template <int BS, bool SUB>
__global__ void __launch_bounds__((MeWGeo<BS, SUB>::NTHREADS)) __attribute__((amdgpu_waves_per_eu(SUB ? 4 : 8)))
me_wave_kernel(const uint8_t* __restrict__ cur, RefSet refs, int nref, int H, int W, int by0, int by1,
               int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub) {
    using G = MeWGeo<BS, SUB>;
    constexpr int SR = G::SR, TBX = G::TBX, TBY = G::TBY, RPD = G::RPD, CS = G::CSTRIDE;
    constexpr int NUNIT = G::NBLK * (SUB ? 5 : 1);
    __shared__ uint32_t win[4 * CS];
    __shared__ unsigned long long keys[NUNIT];

    const int nbx = W / BS;
    const int tiles_x = (nbx + TBX - 1) / TBX;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int bx0 = tx * TBX, byt0 = by0 + ty * TBY;
    const int x0 = bx0 * BS, y0 = byt0 * BS;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    for (int i = tid; i < NUNIT; i += G::NTHREADS) keys[i] = kNoKey;
    for (int r = 0; r < nref; ++r) {
        const uint8_t* ref = refs.p[r];
        __syncthreads();   // the previous reference's reads of the window are done
        // stage: copy s row wr dword m = window bytes [4m + s, 4m + s + 4); zero off-frame
        stage_window<G::WR, RPD, CS, G::NTHREADS>(win, ref, H, W, x0 - SR, y0 - SR, tid);
        __syncthreads();
#pragma unroll 1
        for (int u = wave; u < G::NBLK; u += G::NW) {
            const int bxl = u % TBX, byl = u / TBX;
            if (bx0 + bxl >= nbx || byt0 + byl >= by1) continue;   // wave-uniform
            const int x = x0 + bxl * BS, y = y0 + byl * BS;
            wave_dense_block<BS, SUB, RPD, CS>(win, keys, G::NBLK, cur, W, H, x, y, bxl, byl, u, tid, r);
        }
    }
    __syncthreads();
    for (int i = tid; i < NUNIT; i += G::NTHREADS) {
        const int blk = i < G::NBLK ? i : (i - G::NBLK) >> 2;
        const int gbx = bx0 + blk % TBX, gby = byt0 + blk / TBX;
        if (gbx >= nbx || gby >= by1) continue;
        const size_t b = (size_t)(gby - by0) * nbx + gbx;
        if (i < G::NBLK) decode_key(keys[i], SR, out_best + b * 4);
        else decode_key(keys[i], SR, out_sub + (b * 4 + ((i - G::NBLK) & 3)) * 4);
    }
}

// FME search (FMEEnable): me_wave_kernel's dense wave search over the four phase planes of
// every reference (virtual references vr = 4 r + 2a + b, planes + vr * pstride; see
// FmePhase above).  Keys are the half-pel keys, decoded with sr' = 2 sr = 32.
template <bool SUB>
__global__ void __launch_bounds__((MeWGeo<16, SUB>::NTHREADS)) __attribute__((amdgpu_waves_per_eu(SUB ? 4 : 8)))
me_fme_kernel(const uint8_t* __restrict__ cur, const uint8_t* __restrict__ planes, size_t pstride, int nref, int H,
              int W, int by0, int by1, int32_t* __restrict__ out_best, int32_t* __restrict__ out_sub) {
    using G = MeWGeo<16, SUB>;
    constexpr int BS = 16, SR = G::SR, TBX = G::TBX, TBY = G::TBY, RPD = G::RPD, CS = G::CSTRIDE;
    constexpr int NUNIT = G::NBLK * (SUB ? 5 : 1);
    __shared__ uint32_t win[4 * CS];
    __shared__ unsigned long long keys[NUNIT];

    const int nbx = W / BS;
    const int tiles_x = (nbx + TBX - 1) / TBX;
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int bx0 = tx * TBX, byt0 = by0 + ty * TBY;
    const int x0 = bx0 * BS, y0 = byt0 * BS;
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

    for (int i = tid; i < NUNIT; i += G::NTHREADS) keys[i] = kNoKey;
    for (int vr = 0; vr < 4 * nref; ++vr) {
        const uint8_t* ref = planes + (size_t)vr * pstride;
        const FmePhase ph{(vr >> 1) & 1, vr & 1};
        const int r = vr >> 2;
        __syncthreads();
        stage_window<G::WR, RPD, CS, G::NTHREADS>(win, ref, H, W, x0 - SR, y0 - SR, tid);
        __syncthreads();
#pragma unroll 1
        for (int u = wave; u < G::NBLK; u += G::NW) {
            const int bxl = u % TBX, byl = u / TBX;
            if (bx0 + bxl >= nbx || byt0 + byl >= by1) continue;   // wave-uniform
            const int x = x0 + bxl * BS, y = y0 + byl * BS;
            wave_dense_block<BS, SUB, RPD, CS, true>(win, keys, G::NBLK, cur, W, H, x, y, bxl, byl, u, tid, r, ph);
        }
    }
    __syncthreads();
    for (int i = tid; i < NUNIT; i += G::NTHREADS) {
        const int blk = i < G::NBLK ? i : (i - G::NBLK) >> 2;
        const int gbx = bx0 + blk % TBX, gby = byt0 + blk / TBX;
        if (gbx >= nbx || gby >= by1) continue;
        const size_t b = (size_t)(gby - by0) * nbx + gbx;
        if (i < G::NBLK) decode_key(keys[i], 2 * SR, out_best + b * 4);
        else decode_key(keys[i], 2 * SR, out_sub + (b * 4 + ((i - G::NBLK) & 3)) * 4);
    }
}

// Phase planes of frac_me_reference_frame (Encoder.py:388-403): P_ab[i][j] = F[2i+a][2j+b],
//   P00 = r,  P01 = ceil(h/2),  P10 = ceil((r[i][j] + r[i+1][j]) / 2),  P11 = ceil((h + h') / 4)
// with h = r[i][j] + r[i][j+1] (mod 256 when `wrap`: the uint8 row sum of the reference,
// see oracle oc_fme_upsample) and h' the same one row down.  Entries past F (last column of
// P01/P11, last row of P10/P11) are 0 and never read by a valid candidate.  One thread per
// 4 pixels of a row: one dword of r and of the next row, plus the next byte of each.
__global__ void __launch_bounds__(256)
fme_planes_kernel(const uint8_t* __restrict__ ref, int H, int W, int wrap, uint8_t* __restrict__ out, size_t pstride) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    const int qpr = W >> 2;
    if (q >= qpr * H) return;
    const int i = q / qpr, j0 = (q - i * qpr) * 4;
    const uint8_t* r0 = ref + (size_t)i * W + j0;
    const bool down = i + 1 < H;
    const uint8_t* r1 = down ? r0 + W : r0;
    uint32_t p00 = 0, p01 = 0, p10 = 0, p11 = 0;
    const uint32_t w0 = *reinterpret_cast<const uint32_t*>(r0), w1 = *reinterpret_cast<const uint32_t*>(r1);
    const bool right = j0 + 4 < W;
    const int e0 = right ? r0[4] : 0, e1 = right ? r1[4] : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int a = (w0 >> (8 * k)) & 255, c = (w1 >> (8 * k)) & 255;
        const bool rk = j0 + k + 1 < W;
        const int a2 = k < 3 ? (int)((w0 >> (8 * k + 8)) & 255) : e0;
        const int c2 = k < 3 ? (int)((w1 >> (8 * k + 8)) & 255) : e1;
        int h0 = a + a2, h1 = c + c2;
        if (wrap) { h0 &= 255; h1 &= 255; }
        p00 |= (uint32_t)a << (8 * k);
        if (rk) p01 |= (uint32_t)((h0 + 1) >> 1) << (8 * k);
        if (down) p10 |= (uint32_t)((a + c + 1) >> 1) << (8 * k);
        if (down && rk) p11 |= (uint32_t)((h0 + h1 + 3) >> 2) << (8 * k);
    }
    const size_t o = (size_t)i * W + j0;
    *reinterpret_cast<uint32_t*>(out + o) = p00;
    *reinterpret_cast<uint32_t*>(out + pstride + o) = p01;
    *reinterpret_cast<uint32_t*>(out + 2 * pstride + o) = p10;
    *reinterpret_cast<uint32_t*>(out + 3 * pstride + o) = p11;
}

int fme_planes_launch(const uint8_t* ref, int H, int W, int wrap, uint8_t* out, size_t pstride, hipStream_t st) {
    const int n = (W / 4) * H;
    hipLaunchKernelGGL(fme_planes_kernel, dim3((n + 255) / 256), dim3(256), 0, st, ref, H, W, wrap, out, pstride);
    return check_launch("fme_planes_kernel");
}

int me_fme_launch(const uint8_t* cur, const uint8_t* planes, size_t pstride, int nref, int H, int W, int by0, int by1,
                  int32_t* out_best, int32_t* out_sub, hipStream_t st) {
    const int nbx = W / 16, nrows = by1 - by0;
    if (nrows <= 0) return SO_OK;
    const bool sub = out_sub != nullptr;
    const int tby = (sub ? MeWGeo<16, true>::TPY : MeWGeo<16, false>::TPY) / 16;
    const dim3 grid(((nbx + 7) / 8) * ((nrows + tby - 1) / tby));
    if (sub)
        hipLaunchKernelGGL((me_fme_kernel<true>), grid, dim3(MeWGeo<16, true>::NTHREADS), 0, st, cur, planes, pstride,
                           nref, H, W, by0, by1, out_best, out_sub);
    else
        hipLaunchKernelGGL((me_fme_kernel<false>), grid, dim3(MeWGeo<16, false>::NTHREADS), 0, st, cur, planes,
                           pstride, nref, H, W, by0, by1, out_best, out_sub);
    return check_launch("me_fme_kernel");
}

// ---------------------------------------------------------------------------------------
// SEA path (me_sea2_kernel and the fused tile kernels; the default for bs 16 without VBS):
// exact successive elimination.
//
// With S = a 4x4 pixel sum (0..4080) and q = S >> 4 (a byte), write S = 16q + r, r < 16.
// Then |S_cur - S_ref| >= 16|q_cur - q_ref| - 15, so for a candidate c
//     SAD(c) >= sum_k |S_cur(k) - S_ref(c, k)| >= 16 * LBq(c) - 240,
//     LBq(c) = sum over the 16 4x4 sub-blocks k of |q_cur(k) - q_ref(c, k)|
// (triangle inequality).  Per block:
//   1. LBq for all 1089 candidates; a candidate's four byte sums of one 4x4 row are one
//      dword, so LBq costs 4 v_sad_u8 per candidate instead of 64 for its SAD;
//   2. U = the full SAD of the valid candidate with the smallest LBq, so U >= min SAD;
//   3. every valid candidate with 16 * LBq - 240 <= U gets its full SAD (survivors,
//      compacted into an LDS list).  Any other candidate has SAD > U >= min SAD, so it can
//      neither be the minimum nor tie it: the lexicographic key result is exactly the full
//      search's.  More than CAP survivors (weak bounds: flat or noise-like content): every
//      valid candidate's SAD, one per lane.
// Layout and scheduling:
//   * ONE copy of the window in LDS (pitch 41 dwords: column walks are conflict free); the
//     byte-shifted reads the search needs are two ds_read_b32 + v_alignbyte;
//   * the window's loads are all issued before any LDS store;
//   * the reference's 4x4 byte sums (B4) are built per tile in LDS by threads owning 4
//     adjacent columns and a band of output rows, all their LDS reads issued up front;
//   * survivors are compacted with one wave ballot per candidate row and the lane's rank in
//     it (mbcnt) -- the list order is irrelevant, the key decides.
// A first SEA kernel with four byte-shifted window copies (59 KB LDS per workgroup) took
// 66-73 us per 4K P-frame, 23 us of it staging and 17 us compacting; it was retired once
// this one replaced it.
// ---------------------------------------------------------------------------------------
#ifndef SO_SEA2_WPE
#define SO_SEA2_WPE 6
#endif
#ifndef SO_SEA_CAP   // survivors per block evaluated from the list; more take the dense fallback
#define SO_SEA_CAP 384   // round 6, 192 -> 384 (the list shares LDS with the transform scratch: no
                         // cost in LDS): configs[4] 2.457 -> 2.41, low texture 2.186 -> 2.112, 4K
                         // 1.568 -> 1.562 ms per GOP, noise unchanged; 512 and 768 slower
                         // (profiles/r06/ab_sea_cap*.log)
#endif
#ifndef SO_SEA_CAP_VBS   // the same for a VBS block's block / sub-block lists (sea_vbs_block): looser
#define SO_SEA_CAP_VBS 384   // sub-block bounds leave more survivors (4K VBS P-run 161.5 -> 158.8 us,
                             // dense blocks 8.9 -> 3.8 %; 768: 161.5, profiles/r03/r03n/vbs_ab.log)
#endif
#ifndef SO_DENSE_THR     // a tile searches dense from the start when the same tile of the
#define SO_DENSE_THR 8   // reference frame had at least this many of its 16 blocks overflow,
#endif                   // except every SO_DENSE_PROBE-th frame, which probes the bound again
#ifndef SO_DENSE_PROBE    // round 6, 4 -> 16: a probe frame pays the bound and the lists of every
#define SO_DENSE_PROBE 16 // block before their dense search -- noise 3.13 -> 2.94 ms per 4K GOP (8:
#endif                    // 3.01, 32: 2.91), textured content unchanged (ab_dense_probe_period.log)
#ifndef SO_VBS_HALVES   // A/B builds: 1 = list B by halves.  Bit-exact, but 4K VBS GOP 3.198 ->
#define SO_VBS_HALVES 0  // 3.359 ms (the second mask, list and four more wave minima cost more than
#endif                   // the passes saved), 1080p 1.437 -> 1.375 (profiles/r06/ab_vbs_halves.log)
#ifndef SO_B4_PD   // byte-sum rows in flight in the SEA bound loop (A/B builds: 3, 4)
#define SO_B4_PD 2
#endif
#ifndef SO_PTILE_WPE16   // waves per SIMD of the 16-wave fused tile kernels (A/B builds only)
#define SO_PTILE_WPE16 8
#endif
// NW_ waves per workgroup: 8 (two blocks per wave; me_sea2_kernel) or 16 (one block per
// wave; p_tile_kernel at 8 waves/SIMD)
// TPX_: tile width, 128 (16 blocks)
template <int NW_, int TPX_ = 128>
struct Sea2GeoT {
    static constexpr int SR = 16, NT = 17;
    static constexpr int TPX = TPX_, TBX = TPX / 16, TPY = 32, TBY = 2;
    static constexpr int WR = TPY + 2 * SR;               // 64 window rows
    static constexpr int WD = (TPX + 2 * SR) / 4;         // 40 (24) data dwords per row
    static constexpr int RP = WD + 1;                     // pitch 41 (25)
    static constexpr int B4R = WR - 3, B4C = TPX + 2 * SR - 3, B4P = 4 * RP;   // 41 dwords: rows 16 apart land 16 banks apart
    // transform phase: blocks per wave (16 lanes each); 4 (waves 0-3 for 16 blocks) or 2
    // (waves 0-3 for 8 blocks: half the per-wave latency)
    static constexpr int TQ_BPW = TPX == 128 ? 4 : 2;
    static constexpr int B4BAND = NW_ >= 16 ? 3 : 6;      // output rows per byte-sum thread
    static constexpr int B4NB = (B4R + B4BAND - 1) / B4BAND;
    static constexpr int B4RS = B4NB * B4BAND;            // stored rows: whole bands, no bounds tests
    static constexpr int NBLK = TBX * TBY;
    static constexpr int NW = NW_, NTHREADS = NW * 64;
    static constexpr int CAP = SO_SEA_CAP, CAPV = SO_SEA_CAP_VBS;
    // list entries per wave (SO_VBS_HALVES: a VBS block's sub-block survivors go to two lists of
    // up to CAPV, its top and bottom halves; in the fused tiles the lists share LDS with the
    // transform scratch, which is larger either way)
    static constexpr int CAPLV = SO_VBS_HALVES ? 2 * CAPV : CAPV;
    static constexpr int CAPL = CAP > CAPLV ? CAP : CAPLV;
    static constexpr int DCS = WR * RP + 8;                // dense tiles: window copy stride (8 mod 32)
    static constexpr int CPD = TPX / 4 + 1;               // current-tile pitch in dwords: 16 rows of
                                                          // one block column land on 16 banks
    static_assert(WD * B4NB <= NTHREADS, "byte-sum threads");
};
using Sea2Geo = Sea2GeoT<8>;

// 4 bytes of window row `row` starting at byte column `col` (single copy, pitch RP dwords)
template <int RP>
SO_DEV uint32_t win_u32(const uint32_t* win, int row, int col) {
    lds_vu32p p = (lds_vu32p)(win + row * RP + (col >> 2));
    return __builtin_amdgcn_alignbyte(p[1], p[0], (uint32_t)(col & 3));
}

#ifdef SO_STAMPS
// Instrumented builds only (tools/sea_stamps.py, tools/run_stamps.py): per-workgroup (per-task
// in p_run_kernel) phase time stamps.  s_stamp_rec is the workgroup's current record.
__device__ unsigned long long* g_sea_stamps = nullptr;
__device__ unsigned long long* g_run_stamps = nullptr;
__shared__ unsigned long long* s_stamp_rec;
#define SO_SEA_STAMP(i, v) do { if (tid == 0 && s_stamp_rec) s_stamp_rec[(i)] = (v); } while (0)
#define SO_STAMP_REC_SET(p) do { if (threadIdx.x == 0) s_stamp_rec = (p); } while (0)
extern "C" int so_debug_set_sea_stamps(void* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_sea_stamps), &p, sizeof(p));
}
extern "C" int so_debug_set_run_stamps(void* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_run_stamps), &p, sizeof(p));
}
#else
#define SO_STAMP_REC_SET(p) do { } while (0)
#define SO_SEA_STAMP(i, v) do { } while (0)
#endif

// ISA census builds (-DSO_MARKS, tools/isa_census.py): a comment line in the assembly at each
// phase boundary of the persistent loop; nothing is emitted otherwise.
// -DSO_MARKS_COUNT (tools/valu_census.py): every marker a wave passes adds 1 to its LDS counter
// (the lowest active lane's ds_add_u32; no VALU beyond the two operand moves), and each
// workgroup adds its counters to g_mark_counts at exit: executions per phase per launch, which
// weight the static census into a dynamic VALU table.
#define SO_MARK_NAMES(X) X(loop_top) X(stage_cur) X(stage_cur_int) X(stage_cur_edge) X(cur_sums) X(wait) \
    X(poll_iter) X(stage_win) X(stage_win_int) X(stage_win_edge) X(dense_tile) X(dense_tile_block) X(byte_sums) \
    X(block_top) X(bound) X(umin) X(umin_edge) X(ballots) X(bal_row) X(dense_fallback) X(survivors) X(sur_one) X(sur_le4) X(sur_pass) \
    X(search_end) X(decode_keys) X(tq_residual) X(tq_fwd) X(tq_quant) X(tq_tokens) X(tq_qtc_store) X(tq_inv) \
    X(tq_recon) X(tq_sse_records) X(post) X(done_flag) X(task_end) X(vbs_block) X(vbs_umin) X(vbs_list_a) \
    X(vbs_pass) X(vbs_list_b) X(vbs_final) X(vbs_dense) X(vbs_fwd) X(vbs_fwd_sub) X(vbs_final_q) X(vbs_inv) \
    X(vbs_inv_split) X(vbs_inv_end) X(wait_w0) X(keys_tail) X(p1_tq) X(p1_flag) X(p2_wait) X(p2_sums) X(p2_tq) \
    X(p2_flag)
#define SO_MARK_ENUM(n) kMark_##n,
enum SoMarkId { SO_MARK_NAMES(SO_MARK_ENUM) kMarkCount };
#undef SO_MARK_ENUM
#if defined(SO_MARKS_COUNT)
__device__ unsigned* g_mark_counts = nullptr;
__shared__ unsigned s_mark_cnt[64];
extern "C" int so_debug_set_mark_counts(void* p) {
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_mark_counts), &p, sizeof(p));
}
SO_DEV void so_mark_hit(int id) {
    uint64_t sv, m;
    uint32_t f;
    asm volatile(   // exec = the lowest active lane (none: s_ff1 gives -1, bit 63 & 0 = 0)
        "s_mov_b64 %0, exec\n\t"
        "s_ff1_i32_b64 %2, exec\n\t"
        "s_lshl_b64 %1, 1, %2\n\t"
        "s_and_b64 exec, exec, %1\n\t"
        "ds_add_u32 %3, %4\n\t"
        "s_mov_b64 exec, %0"
        : "=&s"(sv), "=&s"(m), "=&s"(f)
        : "v"((uint32_t)(uintptr_t)&s_mark_cnt[id]), "v"(1u)
        : "memory", "scc");
}
#define SO_MARK(name) so_mark_hit(kMark_##name)
#elif defined(SO_MARKS)
#define SO_MARK(name) asm volatile(";SO_MARK " #name)
#else
#define SO_MARK(name) do { } while (0)
#endif

// threadIdx.x behind an optimisation barrier: inside p_run_kernel's persistent loop the
// tid-derived addresses are then recomputed per task instead of being hoisted out of the
// loop and held in (spilled) registers across it.
SO_DEV int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// LDS of one SEA tile (me_sea2_kernel, p_tile_kernel).
struct Sea2Lds {
    uint32_t* win;             // [WR * RP + 4] reference window, single copy
    uint32_t* b4w;             // [(B4RS * B4P + 4) / 4] 4x4 byte sums of the window
    uint32_t* curt;            // [TPY * TPX / 4] current tile, 32 rows x 128 B
    uint32_t* a4;              // [NBLK * 4] per block: [j] = 4 byte sums (4x4 >> 4) of row j
    uint16_t* list;            // [NW * CAP] survivor lists
    uint32_t* lcount;          // [NW]
    unsigned long long* keys;  // [NBLK] packed best key per block
    uint32_t* st;              // [3]: dense-fallback blocks, survivors (SO_STAMPS only), SAD byte ops
    int count_ops;             // st[2] is counted (SO_OPT_COUNT_SAD_OPS)
    int dense4;                // dwords from win to the room for window copies 1..3 of a dense tile
                               // (DCS apart, 8 mod 32); 0 = none: dense tiles read the single copy
};

// Exact SEA full search of tile `tile` (16 blocks of 16x16) over nref references.  On
// return (after a barrier) keys[] holds every block's packed best key and win[] the last
// reference's window (zero outside the frame).
struct NoPre {
    SO_DEV void operator()() const {}
};
// `pre` runs (on every wave) after the current tile is staged and before the first
// reference's window is read: p_run_kernel waits there for the reference's tiles, so the
// current-tile staging overlaps that wait.
// Waves per SIMD the VBS run kernel is compiled for: 6 (three 8-wave workgroups per CU: 80
// VGPRs, 53.2 KB of LDS) -- 4K VBS P-frame 120.4 vs 136.3 us at 4 waves / SIMD (128 VGPRs),
// VALU busy 0.868 vs 0.735, 1.03x the VALU instructions (profiles/r05/vbs_ab4.log, pmc_vbs4)
#ifndef SO_VBS_WPE
#define SO_VBS_WPE 6
#endif
// SO_VBS_LEAN: the VBS search / transforms hold fewer values in VGPRs (block bounds recomputed
// where used, current rows re-read per survivor pass, levels requantised from the coefficients)
// at the price of ~3 % more VALU -- what the 80-VGPR (6 waves / SIMD) build needs; at 128 VGPRs
// (4 waves / SIMD) the plain forms are faster
#ifndef SO_VBS_LEAN
#define SO_VBS_LEAN (SO_VBS_WPE >= 6)
#endif
// ---- VBSEnable: exact SEA for a block and its four 8x8 sub-blocks (sea_vbs_block) ----------
// The block search of find_best_match plus the sub-block searches of inter_prediction
// (Encoder.py:512-544: find_best_match of each 8x8 sub-block over its own +-16 window), for a
// block with x != 0, y != 0 away from the right / bottom frame edge (x, y <= W - 48, H - 48):
// there every one of the 1089 candidates is valid for the block AND for each sub-block (the
// sub-blocks' larger valid ranges only differ within 32 px of those edges; such blocks take the
// dense search), so all five minima run over the same candidate set.
//   1. One pass over the 4x4 byte sums gives, per candidate, the four sub-block bounds packed
//      in two dwords (TL | TR << 16, BL | BR << 16: v_sad_u8 / v_sad_hi_u8 on the cell-sum
//      dwords masked to the sub-block's two cells); the block bound is their sum.
//      SAD_j >= 16 sum_j |dq| - 60, SAD >= 16 sum |dq| - 240 (q = 4x4 sum >> 4).
//   2. A: U = the SAD of the smallest-bound candidate; every candidate with block bound <= U
//      is evaluated exactly (four lanes per candidate), giving the block minimum and, from the
//      same SADs split by quadrant, U_j = the smallest sub-block SAD seen.
//   3. B: every remaining candidate with some sub-block bound <= U_j is evaluated exactly.
// Any other candidate has SAD > U >= min (block) and SAD_j > U_j >= min_j for every j, so the
// five lexicographic minima (SAD, |dx|+|dy|, ref, scan) are exactly the full searches'.  More
// than CAP survivors in A or B: returns false and the caller runs the dense search.
template <class G>
SO_DEV void vbs_eval_list(const Sea2Lds& L, const uint16_t* list, uint32_t n, int cs, int bxl, int byl, int lane,
                          uint64_t& bestB, uint32_t& best0, uint32_t& best1) {
    constexpr int RP = G::RP, CPD = G::CPD;
    const int sidx = lane >> 2, q = lane & 3;
    const int crow0 = byl * 16 * CPD + bxl * 4;
    // SO_VBS_LEAN: the current rows are re-read from LDS per pass (a list is mostly one pass of
    // 16): held across the loop they take 16 VGPRs while the 34 packed sub-bounds are live
    uint32_t cr[4][4];
    if constexpr (!SO_VBS_LEAN) {
#pragma unroll
        for (int rr = 0; rr < 4; ++rr)
#pragma unroll
            for (int k = 0; k < 4; ++k) cr[rr][k] = L.curt[crow0 + (4 * q + rr) * CPD + k];
    }
#pragma unroll 1
    for (uint32_t s0 = 0; s0 < n; s0 += 16) {
        SO_MARK(vbs_pass);
        const bool act = s0 + (uint32_t)sidx < n;
        const int cand = act ? (int)list[s0 + sidx] : cs;
        const int dxi = cand / 33, di = cand - dxi * 33;
        const int col = bxl * 16 + dxi;
        const uint32_t sh = (uint32_t)(col & 3);
        int wo = (byl * 16 + di + 4 * q) * RP + (col >> 2);
        asm volatile("" : "+v"(wo));
        uint32_t sl = 0, srr = 0;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            lds_vu32p p = (lds_vu32p)(L.win + wo + rr * RP);
            lds_vu32p c = (lds_vu32p)(L.curt + crow0 + (4 * q + rr) * CPD);
            const uint32_t q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3], q4 = p[4];
            const uint32_t c0 = SO_VBS_LEAN ? c[0] : cr[rr][0], c1 = SO_VBS_LEAN ? c[1] : cr[rr][1];
            const uint32_t c2 = SO_VBS_LEAN ? c[2] : cr[rr][2], c3 = SO_VBS_LEAN ? c[3] : cr[rr][3];
            sl = __builtin_amdgcn_sad_u8(c0, __builtin_amdgcn_alignbyte(q1, q0, sh), sl);
            sl = __builtin_amdgcn_sad_u8(c1, __builtin_amdgcn_alignbyte(q2, q1, sh), sl);
            srr = __builtin_amdgcn_sad_u8(c2, __builtin_amdgcn_alignbyte(q3, q2, sh), srr);
            srr = __builtin_amdgcn_sad_u8(c3, __builtin_amdgcn_alignbyte(q4, q3, sh), srr);
        }
        // quad lanes q = 0, 1 hold rows 0-7 (top sub-blocks), 2, 3 rows 8-15: pair them up
        uint32_t v = sl | (srr << 16);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppQuad1032, 0xF, 0xF, false);   // (L | R << 16) of the half
        uint32_t hb = __builtin_amdgcn_sad_u16(v, 0u, 0u);                                       // the half's SAD
        hb += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hb, kDppQuad2301, 0xF, 0xF, false);  // the block's
        const int dx = dxi - 16, dy = di - 16;
        const uint32_t md = (uint32_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy));
        const uint64_t tail = ((uint64_t)md << 24) | (uint64_t)cand;
        const uint64_t kb = ((uint64_t)hb << 32) | tail;
        // sub-block keys in 32 bits: SAD_j < 2^14 (64 pixels), |dx| + |dy| <= 32, cand < 2^11
        const uint32_t t32 = (md << 11) | (uint32_t)cand;
        const uint32_t k0 = ((v & 0xFFFFu) << 17) | t32, k1 = ((v >> 16) << 17) | t32;
        bestB = (act && kb < bestB) ? kb : bestB;
        best0 = (act && k0 < best0) ? k0 : best0;
        best1 = (act && k1 < best1) ? k1 : best1;
    }
}

// List B by halves (SO_VBS_HALVES): a candidate not in list A can only improve sub-block
// minima, and mostly passes one sub-block bound, so B holds (candidate, half) entries -- the
// top half's list at listT, the bottom half's at listBo -- and a pass evaluates 16 entries of
// each: lanes 0-31 the top ones, lanes 32-63 the bottom ones, two lanes per entry (4 of its
// 8 rows each), paired by one DPP add into the half's left / right quadrant SADs.  32-bit
// sub-block keys as vbs_eval_list's, into c0 (left quadrant) and c1 (right) of the lane's half.
template <class G>
SO_DEV void vbs_eval_halves(const Sea2Lds& L, const uint16_t* listT, uint32_t nT, const uint16_t* listBo,
                            uint32_t nBo, int cs, int bxl, int byl, int lane, uint32_t& c0, uint32_t& c1) {
    constexpr int RP = G::RP, CPD = G::CPD;
    const bool bot = lane >= 32;
    const int e = (lane & 31) >> 1;
    const int r0 = (bot ? 8 : 0) + 4 * (lane & 1);
    const uint16_t* const list = bot ? listBo : listT;
    const uint32_t n = bot ? nBo : nT, nmax = nT > nBo ? nT : nBo;
    const int crow0 = byl * 16 * CPD + bxl * 4 + r0 * CPD;
#pragma unroll 1
    for (uint32_t s0 = 0; s0 < nmax; s0 += 16) {
        SO_MARK(vbs_pass);
        const bool act = s0 + (uint32_t)e < n;
        const int cand = act ? (int)list[s0 + e] : cs;
        const int dxi = cand / 33, di = cand - dxi * 33;
        const int col = bxl * 16 + dxi;
        const uint32_t sh = (uint32_t)(col & 3);
        int wo = (byl * 16 + di + r0) * RP + (col >> 2);
        asm volatile("" : "+v"(wo));
        uint32_t sl = 0, srr = 0;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
            lds_vu32p p = (lds_vu32p)(L.win + wo + rr * RP);
            lds_vu32p c = (lds_vu32p)(L.curt + crow0 + rr * CPD);
            const uint32_t q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3], q4 = p[4];
            sl = __builtin_amdgcn_sad_u8(c[0], __builtin_amdgcn_alignbyte(q1, q0, sh), sl);
            sl = __builtin_amdgcn_sad_u8(c[1], __builtin_amdgcn_alignbyte(q2, q1, sh), sl);
            srr = __builtin_amdgcn_sad_u8(c[2], __builtin_amdgcn_alignbyte(q3, q2, sh), srr);
            srr = __builtin_amdgcn_sad_u8(c[3], __builtin_amdgcn_alignbyte(q4, q3, sh), srr);
        }
        uint32_t v = sl | (srr << 16);
        v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, kDppQuad1032, 0xF, 0xF, false);   // lanes l, l ^ 1
        const int dx = dxi - 16, dy = di - 16;
        const uint32_t md = (uint32_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy));
        const uint32_t t32 = (md << 11) | (uint32_t)cand;
        const uint32_t k0 = ((v & 0xFFFFu) << 17) | t32, k1 = ((v >> 16) << 17) | t32;
        c0 = (act && k0 < c0) ? k0 : c0;
        c1 = (act && k1 < c1) ? k1 : c1;
    }
}

#ifndef SO_VBS_BALLOT_LATENCY   // A/B builds: 0 = mask-built lists in latency-bound runs too.
#define SO_VBS_BALLOT_LATENCY 1  // 1080p VBS GOP 1.433 -> 1.399 ms (profiles/r06/ab_vbs_ballot_
#endif                           // latency.log); the uniform-QP run as two instantiations, 4K
                                 // unchanged (ab_vbs_latency_twin.log)
#ifndef SO_VBS_MASKLIST   // bit 0: list A, bit 1: list B built from masks (0: one ballot per
#define SO_VBS_MASKLIST 3   // candidate row, round 5).  4K VBS GOP 3.271 -> 3.201 ms (B alone 3.212,
#endif                      // A alone 3.251); 1080p VBS 1.394 -> 1.430, latency-bound there (a wave
                            // runs its lanes' longest bit loop) -- profiles/r06/ab_vbs_masklist*.log
// A VBS survivor list from per-lane candidate masks (bit t < NT: candidate cbase + t; bit NT:
// c2, the dx = +16 column's): each lane's entries at its offset in the wave's prefix sum of the
// masks' popcounts, the set bits written in a loop the wave runs max-popcount times (the lists'
// candidates sit a few to a lane).  Returns the list length (uniform); past `cap` nothing is
// written.  The order differs from the one-ballot-per-row build, which the lists' minima over
// keys unique by candidate do not see.
template <int NT>
SO_DEV uint32_t vbs_list_from_masks(uint16_t* list, uint32_t m, int cbase, int c2, uint32_t cap) {
    const uint32_t c = (uint32_t)__builtin_popcount(m);
    const uint32_t inc = wave_incl_scan_u32(c);   // (a prefix by bit planes of c, five ballots:
    const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)inc, 63);   // slower)
    uint32_t pos = inc - c;
    if (tot > cap) return tot;
    while (m) {
        const int t = __builtin_ctz(m);
        m &= m - 1u;
        list[pos++] = (uint16_t)(t < NT ? cbase + t : c2);
    }
    return tot;
}

template <class G>
SO_DEV bool sea_vbs_block(const Sea2Lds& L, int u, int bxl, int byl, int tid, bool ballot_lists = false) {
    constexpr int NT = G::NT, B4P = G::B4P, CAP = G::CAPV, RP = G::RP, CPD = G::CPD;
    SO_MARK(vbs_block);
    int lane = tid & 63;
    asm volatile("" : "+v"(lane));
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int xi = lane & 31, hh = lane >> 5;
    const int d2 = lane < 33 ? lane : 32;
    uint32_t AL[4], AR[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const uint32_t a = L.a4[u * 4 + j];
        AL[j] = a & 0xFFFFu;
        AR[j] = a & 0xFFFF0000u;
    }
    // ---- 1. packed sub-block bounds ----------------------------------------------------------
    const int cB = bxl * 16 + xi;
    const int lb0 = (byl * 16 + 16 * hh) * B4P + (cB & 3) * G::WD + (cB >> 2);   // byte offset
    const uint32_t bsh = (uint32_t)lb0 & 3;
    int lo1 = lb0 >> 2;
    asm volatile("" : "+v"(lo1));
    lds_vu32p p1 = (lds_vu32p)(L.b4w + lo1);
    uint32_t T[NT], Bt[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) { T[t] = 0; Bt[t] = 0; }
    constexpr int PD = 2;
    uint32_t n0[PD], n1[PD];
#pragma unroll
    for (int k = 0; k < PD; ++k) { n0[k] = p1[k * (B4P / 4)]; n1[k] = p1[k * (B4P / 4) + 1]; }
#pragma unroll
    for (int sr_ = 0; sr_ < NT + 12; ++sr_) {
        const uint32_t w0 = n0[sr_ % PD], w1 = n1[sr_ % PD];
        if (sr_ + PD < NT + 12) {
            n0[sr_ % PD] = p1[(sr_ + PD) * (B4P / 4)];
            n1[sr_ % PD] = p1[(sr_ + PD) * (B4P / 4) + 1];
        }
        const uint32_t P = __builtin_amdgcn_alignbyte(w1, w0, bsh);
        const uint32_t PL = P & 0xFFFFu, PR = P & 0xFFFF0000u;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int t = sr_ - 4 * j;
            if (t >= 0 && t < NT) {
                uint32_t& acc = j < 2 ? T[t] : Bt[t];
                acc = __builtin_amdgcn_sad_hi_u8(AR[j], PR, __builtin_amdgcn_sad_u8(AL[j], PL, acc));
            }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t)
            if (t <= sr_) asm volatile("" : "+v"(T[t]), "+v"(Bt[t]) : : "memory");
    }
    uint32_t l2T = 0, l2B = 0;   // the dx = +16 column (lanes < 33: dy index d2)
    {
        int lo2 = ((byl * 16 + d2) * B4P + ((bxl * 16 + 32) >> 2)) >> 2;
        asm volatile("" : "+v"(lo2));
        lds_vu32p p2 = (lds_vu32p)(L.b4w + lo2);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const uint32_t qv = p2[4 * j * (B4P / 4)];
            uint32_t& acc = j < 2 ? l2T : l2B;
            acc = __builtin_amdgcn_sad_hi_u8(AR[j], qv & 0xFFFF0000u, __builtin_amdgcn_sad_u8(AL[j], qv & 0xFFFFu, acc));
        }
    }
    // block bounds LBq(t): the four sub-block bounds summed (SO_VBS_LEAN: recomputed where used,
    // the list-A test, instead of held in 17 more VGPRs through the lists)
    SO_MARK(vbs_umin);
    const auto blb0 = [&](int t) { return __builtin_amdgcn_sad_u16(T[t], 0u, __builtin_amdgcn_sad_u16(Bt[t], 0u, 0u)); };
    uint32_t lbs[SO_VBS_LEAN ? 1 : NT];
    if constexpr (!SO_VBS_LEAN) {
#pragma unroll
        for (int t = 0; t < NT; ++t) lbs[t] = blb0(t);
    }
    const auto blb = [&](int t) { return SO_VBS_LEAN ? blb0(t) : lbs[SO_VBS_LEAN ? 0 : t]; };
    const uint32_t lb2 = __builtin_amdgcn_sad_u16(l2T, 0u, __builtin_amdgcn_sad_u16(l2B, 0u, 0u));
    const bool ok2 = lane < 33;
    // ---- 2. U and the block survivors (A) -------------------------------------------------------
    uint32_t kt = 0xFFFFFFFFu;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
        const uint32_t k = (blb(t) << 16) | (uint32_t)t;
        kt = k < kt ? k : kt;
    }
    uint32_t kl = ((kt >> 16) << 11) | (uint32_t)(xi * 33 + 16 * hh + (kt & 31));
    {
        const uint32_t k2 = (lb2 << 11) | (uint32_t)(32 * 33 + d2);
        kl = (ok2 && k2 < kl) ? k2 : kl;
    }
    const uint32_t kmin = wave_min_u32(kl);
    // SAD byte operations: the packed bounds (136 + 8 lane instructions), U (1)
    if (lane == 0) SO_OPS_ADD(&L.st[2], 145u * 256u);
    const int cs = (int)(kmin & 2047), cdx = cs / 33, cdi = cs - cdx * 33;
    const int crow0 = byl * 16 * CPD + bxl * 4;
    uint32_t U;
    {
        const int row = lane >> 2, kk = lane & 3;
        const uint32_t w = win_u32<RP>(L.win, byl * 16 + cdi + row, bxl * 16 + cdx + 4 * kk);
        U = wave_sum_u32(__builtin_amdgcn_sad_u8(L.curt[crow0 + row * CPD + kk], w, 0u));
    }
    const uint32_t qU = (U + 240) >> 4;
    SO_MARK(vbs_list_a);
    // list-A membership of the lane's 17 candidates as a bit mask (the list-B test reads it)
    uint32_t amask = 0;
#pragma unroll
    for (int t = 0; t < NT; ++t) amask |= (blb(t) <= qU ? 1u : 0u) << t;
    uint16_t* const mylist = L.list + wave * G::CAPL;
    const int cbase = xi * 33 + 16 * hh;
    uint32_t nA = 0;
    if ((SO_VBS_MASKLIST & 1) != 0 && !ballot_lists) {
        nA = vbs_list_from_masks<NT>(mylist, amask | ((ok2 && lb2 <= qU) ? 1u << NT : 0u), cbase, 32 * 33 + d2,
                                     (uint32_t)CAP);
    } else {
#pragma unroll
        for (int t = 0; t <= NT; ++t) {
            const bool pass = t < NT ? ((amask >> t) & 1u) != 0u : (ok2 && lb2 <= qU);
            const uint64_t bal = __builtin_amdgcn_ballot_w64(pass);
            if (bal) {
                const uint32_t pos = nA + lane_prefix(bal);
                if (pass && pos < (uint32_t)CAP) mylist[pos] = (uint16_t)(t < NT ? cbase + t : 32 * 33 + d2);
                nA += (uint32_t)__builtin_popcountll(bal);
            }
        }
    }
    if (nA > (uint32_t)CAP) return false;
    if (lane == 0) SO_OPS_ADD(&L.st[2], 16u * ((nA + 15) / 16) * 256u);   // list A: 16 per 16 candidates
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint64_t bestB = kNoKey;
    uint32_t best0 = ~0u, best1 = ~0u;
    vbs_eval_list<G>(L, mylist, nA, cs, bxl, byl, lane, bestB, best0, best1);
    // U_j: the smallest sub-block SADs among the evaluated candidates (quad lanes 0, 1: top)
    const bool top = (lane & 2) == 0;
    const uint32_t mTL = wave_min_u32(top ? best0 : ~0u), mTR = wave_min_u32(top ? best1 : ~0u);
    const uint32_t mBL = wave_min_u32(top ? ~0u : best0), mBR = wave_min_u32(top ? ~0u : best1);
    const uint32_t uTL = mTL >> 17, uTR = mTR >> 17, uBL = mBL >> 17, uBR = mBR >> 17;
    // ---- 3. the sub-block survivors (B): some sub-block bound <= its U_j, not evaluated in A ----
    SO_MARK(vbs_list_b);
    typedef short so_v2i16 __attribute__((ext_vector_type(2)));
    const uint32_t thT = (((uTL + 60) >> 4) + 1) | ((((uTR + 60) >> 4) + 1) << 16);
    const uint32_t thB = (((uBL + 60) >> 4) + 1) | ((((uBR + 60) >> 4) + 1) << 16);
    const auto any_sub = [&](uint32_t tv, uint32_t bv) {   // a 16-bit half of (bound - (thr + 1)) < 0
        const so_v2i16 dt = __builtin_bit_cast(so_v2i16, tv) - __builtin_bit_cast(so_v2i16, thT);
        const so_v2i16 db = __builtin_bit_cast(so_v2i16, bv) - __builtin_bit_cast(so_v2i16, thB);
        return ((__builtin_bit_cast(uint32_t, dt) | __builtin_bit_cast(uint32_t, db)) & 0x80008000u) != 0u;
    };
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");   // list A read before it is overwritten
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (SO_VBS_HALVES) {
        // (candidate, half) entries: the top list at mylist, the bottom one at mylist + CAP
        const auto pass_half = [](uint32_t v, uint32_t th) {
            const so_v2i16 d = __builtin_bit_cast(so_v2i16, v) - __builtin_bit_cast(so_v2i16, th);
            return (__builtin_bit_cast(uint32_t, d) & 0x80008000u) != 0u;
        };
        uint32_t mT = 0, mBo = 0;
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            mT |= (pass_half(T[t], thT) ? 1u : 0u) << t;
            mBo |= (pass_half(Bt[t], thB) ? 1u : 0u) << t;
        }
        const bool col_b = ok2 && !(lb2 <= qU);
        mT = (mT & ~amask) | ((col_b && pass_half(l2T, thT)) ? 1u << NT : 0u);
        mBo = (mBo & ~amask) | ((col_b && pass_half(l2B, thB)) ? 1u << NT : 0u);
        const uint32_t nT = vbs_list_from_masks<NT>(mylist, mT, cbase, 32 * 33 + d2, (uint32_t)CAP);
        const uint32_t nBo = vbs_list_from_masks<NT>(mylist + CAP, mBo, cbase, 32 * 33 + d2, (uint32_t)CAP);
        if (nT > (uint32_t)CAP || nBo > (uint32_t)CAP) return false;
        const uint32_t nmax = nT > nBo ? nT : nBo;
        if (lane == 0) SO_OPS_ADD(&L.st[2], 16u * ((nmax + 15) / 16) * 256u);   // 32 half-candidates per pass
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t kb = wave_min_u64_dpp(bestB);
        uint32_t c0 = ~0u, c1 = ~0u;
        vbs_eval_halves<G>(L, mylist, nT, mylist + CAP, nBo, cs, bxl, byl, lane, c0, c1);
        SO_MARK(vbs_final);
        const auto widen = [](uint32_t k) {
            return ((uint64_t)(k >> 17) << 32) | ((uint64_t)((k >> 11) & 63u) << 24) | (uint64_t)(k & 2047u);
        };
        const bool bot = lane >= 32;
        const uint32_t hTL = wave_min_u32(bot ? ~0u : c0), hTR = wave_min_u32(bot ? ~0u : c1);
        const uint32_t hBL = wave_min_u32(bot ? c0 : ~0u), hBR = wave_min_u32(bot ? c1 : ~0u);
        const uint64_t kTL = widen(hTL < mTL ? hTL : mTL), kTR = widen(hTR < mTR ? hTR : mTR);
        const uint64_t kBL = widen(hBL < mBL ? hBL : mBL), kBR = widen(hBR < mBR ? hBR : mBR);
        if (lane == 0) {
            unsigned long long* const ks = L.keys;
            if (kb < ks[u]) ks[u] = kb;
            unsigned long long* const sk = ks + G::NBLK + 4 * u;
            if (kTL < sk[0]) sk[0] = kTL;
            if (kTR < sk[1]) sk[1] = kTR;
            if (kBL < sk[2]) sk[2] = kBL;
            if (kBR < sk[3]) sk[3] = kBR;
        }
        return true;
    }
    uint32_t nB = 0;
    if ((SO_VBS_MASKLIST & 2) != 0 && !ballot_lists) {
        uint32_t mB = 0;
#pragma unroll
        for (int t = 0; t < NT; ++t) mB |= (any_sub(T[t], Bt[t]) ? 1u : 0u) << t;
        mB &= ~amask;
        mB |= (ok2 && any_sub(l2T, l2B) && !(lb2 <= qU)) ? 1u << NT : 0u;
        nB = vbs_list_from_masks<NT>(mylist, mB, cbase, 32 * 33 + d2, (uint32_t)CAP);
    } else {
#pragma unroll
        for (int t = 0; t <= NT; ++t) {
            const bool pass = t < NT ? (any_sub(T[t], Bt[t]) && ((amask >> t) & 1u) == 0u)
                                     : (ok2 && any_sub(l2T, l2B) && !(lb2 <= qU));
            const uint64_t bal = __builtin_amdgcn_ballot_w64(pass);
            if (bal) {
                const uint32_t pos = nB + lane_prefix(bal);
                if (pass && pos < (uint32_t)CAP) mylist[pos] = (uint16_t)(t < NT ? cbase + t : 32 * 33 + d2);
                nB += (uint32_t)__builtin_popcountll(bal);
            }
        }
    }
    if (nB > (uint32_t)CAP) return false;
    if (lane == 0) SO_OPS_ADD(&L.st[2], 16u * ((nB + 15) / 16) * 256u);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    vbs_eval_list<G>(L, mylist, nB, cs, bxl, byl, lane, bestB, best0, best1);
    SO_MARK(vbs_final);
    const uint64_t kb = wave_min_u64_dpp(bestB);
    // the 32-bit sub-block keys widened to the 64-bit key layout (SAD << 32 | md << 24 | cand)
    const auto widen = [](uint32_t k) {
        return ((uint64_t)(k >> 17) << 32) | ((uint64_t)((k >> 11) & 63u) << 24) | (uint64_t)(k & 2047u);
    };
    const uint64_t kTL = widen(wave_min_u32(top ? best0 : ~0u)), kTR = widen(wave_min_u32(top ? best1 : ~0u));
    const uint64_t kBL = widen(wave_min_u32(top ? ~0u : best0)), kBR = widen(wave_min_u32(top ? ~0u : best1));
    if (lane == 0) {
        unsigned long long* const ks = L.keys;
        if (kb < ks[u]) ks[u] = kb;
        unsigned long long* const sk = ks + G::NBLK + 4 * u;
        if (kTL < sk[0]) sk[0] = kTL;
        if (kTR < sk[1]) sk[1] = kTR;
        if (kBL < sk[2]) sk[2] = kBL;
        if (kBR < sk[3]) sk[3] = kBR;
    }
    return true;
}

// VBS: blocks with a sub-block search (x != 0 and y != 0, Encoder.py:512) take sea_vbs_block
// (the block and its four 8x8 sub-blocks, keys [NBLK + 4u + j]) or, within 32 px of the right /
// bottom edge or past CAP survivors, the dense wave search, whose v_sad_u8 work yields the
// sub-block SADs with the block's; the other blocks the block's exact SEA.
// dense_flag (LDS, read after `pre`): nonzero = every block of the tile takes the dense search
// directly (p_run_kernel sets it when the same tile of the previous frame had most of its
// blocks overflow the SEA bound: flat or noise-like content, where computing the bound only to
// fall back costs more than it saves).
// prev_mv (optional): the motion records (int16 [nb][12], dx and dy first; rows relative to by0)
// of the frame before `cur` against the same kind of reference -- the co-located block's vector
// there is a second candidate for U (below).  Only a hint: any VALID candidate's SAD bounds the
// minimum from above, so a stale or garbage record (it is read unordered, and is range-checked)
// can cost survivors, never exactness.
// LISTS (VBS): how sea_vbs_block builds its survivor lists -- 1 from lane masks, 2 one ballot
// per candidate row, 0 chosen per launch (below)
template <class G, class Pre = NoPre, bool VBS = false, int LISTS = 0>
SO_DEV void sea2_tile(const Sea2Lds& L, int tile, const uint8_t* __restrict__ cur, const RefSet& refs, int nref,
                      int H, int W, int by0, int by1, int probe, const Pre& pre = Pre(),
                      const int* dense_flag = nullptr, const int16_t* prev_mv = nullptr) {
    constexpr int SR = G::SR, TBX = G::TBX, TBY = G::TBY, RP = G::RP, NT = G::NT;
    constexpr int B4P = G::B4P, CAP = G::CAP, CP = G::TPX;
#ifdef SO_NO_MV_HINT   // A/B builds: U from the smallest-bound candidate only
    prev_mv = nullptr;
#endif
    uint32_t* const win = L.win;
    uint32_t* const b4w = L.b4w;
    uint8_t* const b4 = reinterpret_cast<uint8_t*>(b4w);
    uint32_t* const curt = L.curt;
    uint32_t* const a4 = L.a4;
    uint16_t* const list = L.list;
    unsigned long long* const keys = L.keys;

    const int nbx = W / 16;
    const int tiles_x = (nbx + TBX - 1) / TBX;
    const int tx = tile % tiles_x, ty = tile / tiles_x;
    // a persistent grid with more slots than a frame has tiles runs latency-bound (the chain
    // step of one tile position): there the VBS lists are built one ballot per candidate row,
    // whose cost does not depend on how the survivors cluster in a lane (SO_VBS_MASKLIST)
    const bool ballot_lists = LISTS == 2 || (LISTS == 0 && SO_VBS_BALLOT_LATENCY && VBS &&
                                             tiles_x * ((H / 16 + TBY - 1) / TBY) < (int)gridDim.x);
    const int bx0 = tx * TBX, byt0 = by0 + ty * TBY;
    const int x0 = bx0 * 16, y0 = byt0 * 16;
    const int tid = opaque_tid();
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    // st[0]: blocks of this tile that took the dense fallback (the run adds it to its workspace
    // fallback count: the content-dependence records of bench.py)
    uint32_t& st_fb = L.st[0];
    if (tid == 0) st_fb = 0;
    // st[2]: SAD byte operations executed for this tile (every v_sad_u8 / v_sad_hi_u8 lane
    // instruction counts 4): the current tile's 4x4 sums, here
    uint32_t& st_ops = L.st[2];
    if (tid == 0) {
        // recomputed per tile: the persistent run hoisted this select and spilled it
        uint32_t ops0 = L.count_ops ? G::NBLK * 16 * 4 * 4 : 0u;
        asm volatile("" : "+v"(ops0));
        st_ops = ops0;
    }
#ifdef SO_STAMPS
    uint32_t& st_sur = L.st[1];
    if (tid == 0) st_sur = 0;
    SO_SEA_STAMP(0, __builtin_amdgcn_s_memrealtime());
    SO_SEA_STAMP(1, __builtin_amdgcn_s_memtime());
#endif

    SO_MARK(stage_cur);
    for (int i = tid; i < G::NBLK * (VBS ? 5 : 1); i += G::NTHREADS) keys[i] = kNoKey;
    // interior window (uniform): thread = (row, column phase) with immediate per-dword offsets
    constexpr int WTPR = G::NTHREADS / G::WR, WNPT = (RP + WTPR - 1) / WTPR;
    static_assert(G::NTHREADS % G::WR == 0, "window staging");
    const int wwr = tid / WTPR, wc0 = tid - wwr * WTPR;
    const bool win_int = x0 - SR >= 0 && x0 - SR + 4 * RP <= W && y0 - SR >= 0 && y0 - SR + G::WR <= H;
    if (x0 + CP <= W && y0 + G::TPY <= H) {
        // interior tile (uniform branch): thread = (row, column phase); the loads' and stores'
        // per-dword offsets are immediates, so staging costs a few VALU per thread
        constexpr int TPR = G::NTHREADS / G::TPY, NPT = (CP / 4) / TPR;   // threads per row, dwords per thread
        static_assert(G::NTHREADS % G::TPY == 0 && (CP / 4) % TPR == 0, "current-tile staging");
        SO_MARK(stage_cur_int);
        const int rr = tid / TPR, c0 = tid - rr * TPR;
        const uint32_t* src = reinterpret_cast<const uint32_t*>(cur + (size_t)(y0 + rr) * W + x0) + c0;
        uint32_t v[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) v[k] = src[k * TPR];
#pragma unroll
        for (int k = 0; k < NPT; ++k) curt[rr * G::CPD + c0 + k * TPR] = v[k];
    } else {   // current tile (zero outside the frame / stripe)
        SO_MARK(stage_cur_edge);
        constexpr int N = G::TPY * CP / 4, IT = (N + G::NTHREADS - 1) / G::NTHREADS;
        uint32_t v[IT];
#pragma unroll
        for (int k = 0; k < IT; ++k) {
            const int i = tid + k * G::NTHREADS;
            const int rr = i / (CP / 4), m = i - rr * (CP / 4);
            const int gy = y0 + rr, gx = x0 + 4 * m;
            v[k] = 0;
            if (i < N && gy < H && gx + 4 <= W) v[k] = *reinterpret_cast<const uint32_t*>(cur + (size_t)gy * W + gx);
        }
#pragma unroll
        for (int k = 0; k < IT; ++k)
            if (tid + k * G::NTHREADS < N) {
                const int i = tid + k * G::NTHREADS, rr = i / (CP / 4);
                curt[i + rr] = v[k];   // pitch CP/4 + 1 (G::CPD)
            }
    }
    __syncthreads();
    SO_MARK(cur_sums);
    for (int i = tid; i < G::NBLK * 16; i += G::NTHREADS) {   // (block, j, ii) -> byte ii of a4[blk*4 + j]
        const int blk = i >> 4, j = (i >> 2) & 3, ii = i & 3;
        const int rr = (blk / TBX) * 16 + 4 * j, m = (blk % TBX) * 4 + ii;
        uint32_t sum = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) sum = __builtin_amdgcn_sad_u8(curt[(rr + q) * G::CPD + m], 0u, sum);
        reinterpret_cast<uint8_t*>(a4)[i] = (uint8_t)(sum >> 4);
    }
    // Blocks of the tile go to waves dynamically: wave w starts with block w, then takes the
    // next unclaimed one (an LDS counter), so a wave stuck on a many-survivor or dense-fallback
    // block no longer holds a second block back while the others wait at the barrier.
    // (SO_SEA_STATIC: the fixed u = w, w + NW assignment, A/B builds only.)
    uint32_t* const grab = L.lcount;
    const auto next_block = [&](int u) -> int {
#ifdef SO_SEA_STATIC
        return u + G::NW;
#else
        (void)u;
        uint32_t nx = 0;
        if ((tid & 63) == 0) nx = __hip_atomic_fetch_add(grab, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        return (int)__builtin_amdgcn_readfirstlane(nx);
#endif
    };
    for (int r = 0; r < nref; ++r) {
        const uint8_t* ref = refs.p[r];
        SO_MARK(wait);
        if (r == 0) pre();
        SO_MARK(stage_win);
        if (tid == 0) *grab = (uint32_t)G::NW;   // read after the barrier below
        __syncthreads();
        if (r == 0) SO_SEA_STAMP(2, __builtin_amdgcn_s_memtime());
        if (win_int) {   // all loads first, then the LDS stores
            SO_MARK(stage_win_int);
            uint32_t wv0[WNPT];
            const uint32_t* src = reinterpret_cast<const uint32_t*>(ref + (size_t)(y0 - SR + wwr) * W + (x0 - SR)) + wc0;
#pragma unroll
            for (int k = 0; k < WNPT; ++k)
                if (wc0 + k * WTPR < RP) wv0[k] = src[k * WTPR];
#pragma unroll
            for (int k = 0; k < WNPT; ++k)
                if (wc0 + k * WTPR < RP) win[wwr * RP + wc0 + k * WTPR] = wv0[k];
        } else {   // window: all loads first, then the LDS stores (zero outside the frame)
            SO_MARK(stage_win_edge);
            constexpr int N = G::WR * RP, IT = (N + G::NTHREADS - 1) / G::NTHREADS;
            uint32_t v[IT];
#pragma unroll
            for (int k = 0; k < IT; ++k) {
                const int i = tid + k * G::NTHREADS;
                const int wr = i / RP, m = i - wr * RP;
                const int gy = y0 - SR + wr, gx = x0 - SR + 4 * m;
                v[k] = 0;
                if (i < N && gy >= 0 && gy < H && gx >= 0 && gx + 4 <= W)
                    v[k] = *reinterpret_cast<const uint32_t*>(ref + (size_t)gy * W + gx);
            }
#pragma unroll
            for (int k = 0; k < IT; ++k)
                if (tid + k * G::NTHREADS < N) win[tid + k * G::NTHREADS] = v[k];
        }
        __syncthreads();
        if (r == 0) SO_SEA_STAMP(3, __builtin_amdgcn_s_memtime());
        if (probe == 5) continue;   // phase-attribution builds (SO_PROF_PHASE=2): no search at all
        if (dense_flag && __builtin_amdgcn_readfirstlane(*dense_flag)) {   // uniform: the whole tile dense
            SO_MARK(dense_tile);
            // the window's byte-shifted copies 1..3 into the free scratch (no byte sums or lists
            // here): every row the scan reads is then four aligned ds_read_b32 instead of five
            // plus four v_alignbyte (me_wave_kernel's layout)
            const int c1 = L.dense4;
            if (c1 != 0) {
                uint32_t* const cp = win + c1;
                for (int i = tid; i < G::WR * RP; i += G::NTHREADS) {
                    const uint32_t a = win[i], b = win[i + 1];
                    cp[i] = __builtin_amdgcn_alignbyte(b, a, 1);
                    cp[G::DCS + i] = __builtin_amdgcn_alignbyte(b, a, 2);
                    cp[2 * G::DCS + i] = __builtin_amdgcn_alignbyte(b, a, 3);
                }
                __syncthreads();
            }
#pragma unroll 1
            for (int u = wave; u < G::NBLK; u = next_block(u)) {
                SO_MARK(dense_tile_block);
                const int bxl = u % TBX, byl = u / TBX;
                if (bx0 + bxl >= nbx || byt0 + byl >= by1) continue;   // wave-uniform
                const int x = x0 + bxl * 16, y = y0 + byl * 16;
                if (c1 != 0) {
                    if (VBS && x != 0 && y != 0)
                        wave_dense_block<16, true, RP, G::DCS>(win, keys, G::NBLK, cur, W, H, x, y, bxl, byl, u, tid, r,
                                                               FmePhase{0, 0}, c1);
                    else
                        wave_dense_block<16, false, RP, G::DCS>(win, keys, G::NBLK, cur, W, H, x, y, bxl, byl, u, tid,
                                                                r, FmePhase{0, 0}, c1);
                } else if (VBS && x != 0 && y != 0)
                    wave_dense_block<16, true, RP, 0, false, true>(win, keys, G::NBLK, cur, W, H, x, y, bxl, byl, u,
                                                                   tid, r);
                else
                    wave_dense_block<16, false, RP, 0, false, true>(win, keys, G::NBLK, cur, W, H, x, y, bxl, byl, u,
                                                                    tid, r);
                if ((tid & 63) == 0) {
                    atomicAdd(&st_fb, 1u);
                    SO_OPS_ADD(&st_ops, kDenseSadOps);
                }
            }
            continue;
        }
        // 4x4 byte sums B4(row, c) = (sum of the 4x4 window block at (row, c)) >> 4, stored at
        // b4[row * B4P + (c & 3) * WD + (c >> 2)] (a candidate's four sums of one 4x4 row --
        // columns c, c+4, c+8, c+12 -- are then consecutive bytes).  Thread = (dword column m:
        // columns 4m..4m+3, band of B4BAND output rows).
        SO_MARK(byte_sums);
        if (tid == 0) SO_OPS_ADD(&st_ops, (uint32_t)(G::WD * G::B4NB * (G::B4BAND + 3) * 4 * 4));
        if (tid < G::WD * G::B4NB) {
            const int m = tid % G::WD, band = tid / G::WD;
            const int r0 = band * G::B4BAND;
            constexpr int NR = G::B4BAND + 3;
            // row sums of 4 bytes at byte shifts k = 0..3, two per dword as 16-bit halves
            // (v_sad_hi_u8 adds its sum << 16): h[i][0] = (k 0 | k 2 << 16), h[i][1] = (k 1 | k 3
            // << 16).  A 4x4 sum is <= 4080, so the column sums below never carry across halves
            // The last band reads up to 5 rows past the window (the next LDS fields, or 0 past
            // the allocation): those rows only feed sums >= B4R, which no valid candidate reads.
            uint32_t h[NR][2];
            lds_vu32p p = (lds_vu32p)(win + r0 * RP + m);
#pragma unroll
            for (int i = 0; i < NR; ++i) {
                const uint32_t w0 = p[i * RP], w1 = p[i * RP + 1];
                h[i][0] = __builtin_amdgcn_sad_hi_u8(__builtin_amdgcn_alignbyte(w1, w0, 2), 0u,
                                                     __builtin_amdgcn_sad_u8(w0, 0u, 0u));
                h[i][1] = __builtin_amdgcn_sad_hi_u8(__builtin_amdgcn_alignbyte(w1, w0, 3), 0u,
                                                     __builtin_amdgcn_sad_u8(__builtin_amdgcn_alignbyte(w1, w0, 1), 0u, 0u));
            }
            // whole bands, every column: rows >= B4R and columns >= B4C hold sums no valid
            // candidate reads (the storage is B4RS rows), so the stores need no bounds tests.
            // One packed shift per two sums; the high byte goes out by ds_write_b8_d16_hi.
            typedef unsigned short so_v2u16 __attribute__((ext_vector_type(2)));
            uint8_t* const ob = b4 + r0 * B4P + m;
#pragma unroll
            for (int i = 0; i < G::B4BAND; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j) {
                    const uint32_t sum = h[i][j] + h[i + 1][j] + h[i + 2][j] + h[i + 3][j];
                    const uint32_t q = __builtin_bit_cast(uint32_t, __builtin_bit_cast(so_v2u16, sum) >> (so_v2u16){4, 4});
                    ob[i * B4P + j * G::WD] = (uint8_t)q;
                    ob[i * B4P + (j + 2) * G::WD] = (uint8_t)(q >> 16);
                }
        }
        __syncthreads();
        if (r == 0) SO_SEA_STAMP(4, __builtin_amdgcn_s_memtime());
        if (probe == 1) continue;   // timing probe (tools/me_ab2.py): staging + byte sums only
#pragma unroll 1
        for (int u = wave; u < G::NBLK; u = next_block(u)) {
            SO_MARK(block_top);
            const int bxl = u % TBX, byl = u / TBX;
            if (bx0 + bxl >= nbx || byt0 + byl >= by1) continue;   // wave-uniform
            const int x = x0 + bxl * 16, y = y0 + byl * 16;
            // the co-located block's vector in the previous frame (issued now, used after the bounds)
            uint32_t pmv = 0x80008000u;   // (-32768, -32768): no hint
            if (!VBS && prev_mv != nullptr && r == 0)
                pmv = __builtin_amdgcn_readfirstlane(
                    *reinterpret_cast<const uint32_t*>(prev_mv + ((size_t)(byt0 + byl - by0) * nbx + bx0 + bxl) * 12));
            if constexpr (VBS) {
                if (x != 0 && y != 0) {   // uniform: block + sub-block search
#ifndef SO_VBS_DENSE_ONLY   // A/B builds: every sub-searched block dense
                    if (x + 48 <= W && y + 48 <= H && sea_vbs_block<G>(L, u, bxl, byl, tid, ballot_lists)) continue;
#endif
                    if ((tid & 63) == 0) {
                        atomicAdd(&st_fb, 1u);   // counted as a dense fallback
                        SO_OPS_ADD(&st_ops, kDenseSadOps);
                    }
#ifndef SO_TEST_NODENSE
                    SO_MARK(vbs_dense);
                    wave_dense_block<16, true, RP, 0, false, true>(win, keys, G::NBLK, cur, W, H, x, y, bxl, byl, u,
                                                                   tid, r);
#endif
                    continue;
                }
            }
            int lane = tid & 63;
            asm volatile("" : "+v"(lane));
            const int xi = lane & 31, hh = lane >> 5;
            const int d2 = lane < 33 ? lane : 32;
            SO_MARK(bound);
            uint32_t A[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) A[j] = a4[u * 4 + j];
            // ---- 1. lower bounds --------------------------------------------------------------
            const int cB = bxl * 16 + xi;
            const int lb0 = (byl * 16 + 16 * hh) * B4P + (cB & 3) * G::WD + (cB >> 2);   // byte offset
            const uint32_t bsh = (uint32_t)lb0 & 3;
            int lo1 = lb0 >> 2;
            asm volatile("" : "+v"(lo1));
#ifdef SO_B4_READ2   // A/B: plain (mergeable into ds_read2_b32) reads of the byte-sum rows
            typedef const __attribute__((address_space(3))) uint32_t* lds_u32p_;
            lds_u32p_ p1 = (lds_u32p_)(b4w + lo1);
#else
            lds_vu32p p1 = (lds_vu32p)(b4w + lo1);
#endif
            // lb[t] = (LBq << 16) | t: v_sad_hi_u8 accumulates each sum << 16 onto the initial t
            // (an inline constant), so the smallest-bound key below needs no shifts or ORs
            // (LBq <= 16 * 255 < 2^16)
            uint32_t lb[NT];
#pragma unroll
            for (int t = 0; t < NT; ++t) lb[t] = (uint32_t)t;
            // byte-sum rows through a ring of PD rows in flight: the row used in step sr_ was
            // loaded PD steps earlier, so LDS latency overlaps PD steps of v_sad_u8 work
            // (one step ahead left every step waiting on its own loads)
            constexpr int PD = SO_B4_PD;
            uint32_t n0[PD], n1[PD];
#pragma unroll
            for (int k = 0; k < PD; ++k) { n0[k] = p1[k * (B4P / 4)]; n1[k] = p1[k * (B4P / 4) + 1]; }
#pragma unroll
            for (int sr_ = 0; sr_ < NT + 12; ++sr_) {
                const uint32_t w0 = n0[sr_ % PD], w1 = n1[sr_ % PD];
                if (sr_ + PD < NT + 12) {
                    n0[sr_ % PD] = p1[(sr_ + PD) * (B4P / 4)];
                    n1[sr_ % PD] = p1[(sr_ + PD) * (B4P / 4) + 1];
                }
                const uint32_t P = __builtin_amdgcn_alignbyte(w1, w0, bsh);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int t = sr_ - 4 * j;
                    if (t >= 0 && t < NT) lb[t] = __builtin_amdgcn_sad_hi_u8(A[j], P, lb[t]);
                }
                // fence the started accumulators only: a not yet started one stays the inline
                // constant t that its first v_sad_hi_u8 takes directly
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    if (t <= sr_) asm volatile("" : "+v"(lb[t]) : : "memory");
            }
            uint32_t lb2 = 0;
            {
                int lo2 = ((byl * 16 + d2) * B4P + ((bxl * 16 + 32) >> 2)) >> 2;
                asm volatile("" : "+v"(lo2));
                lds_vu32p p2 = (lds_vu32p)(b4w + lo2);
#pragma unroll
                for (int j = 0; j < 4; ++j) lb2 = __builtin_amdgcn_sad_u8(A[j], p2[4 * j * (B4P / 4)], lb2);
            }
            SO_MARK(umin);
            constexpr uint32_t kBig = 0x7FFFFFFFu;   // a masked row: above every (LBq << 16) | t
            int dlo = SR - y;              dlo = dlo < 0 ? 0 : dlo;
            int dhi = H - 16 - y + SR - 1; dhi = dhi > 32 ? 32 : dhi;
            const bool xok = (x + xi - 16 >= 0) && (x + xi - 16 < W - 16);
            const bool x2ok = x + 16 < W - 16;
            const bool ok2 = lane < 33 && x2ok && d2 >= dlo && d2 <= dhi;
            if (dlo > 0 || dhi < 32) {
                SO_MARK(umin_edge);
                const int tlo = dlo - 16 * hh, thi = dhi - 16 * hh;
#pragma unroll
                for (int t = 0; t < NT; ++t) lb[t] = (t < tlo || t > thi) ? kBig : lb[t];
            }
            // ---- 2. U = SAD of the smallest-bound candidate ----------------------------------
            uint32_t kt = lb[0];
#pragma unroll
            for (int t = 1; t < NT; ++t) kt = lb[t] < kt ? lb[t] : kt;
            uint32_t kl = (xok && kt != kBig) ? ((kt >> 16) << 11) | (uint32_t)(xi * 33 + 16 * hh + (kt & 31))
                                              : 0xFFFFFFFFu;
            {
                const uint32_t k2 = (lb2 << 11) | (uint32_t)(32 * 33 + d2);
                kl = (ok2 && k2 < kl) ? k2 : kl;
            }
            const uint32_t kmin = wave_min_u32(kl);
            // the bound pass: 68 + 4 SAD lane instructions, the U evaluation: 1 (2 with a valid hint)
            if (lane == 0) SO_OPS_ADD(&st_ops, kmin == 0xFFFFFFFFu ? 72u * 256u : 73u * 256u);
            if (kmin == 0xFFFFFFFFu) continue;                 // no valid candidate: key stays none
            const int cs = (int)(kmin & 2047), cdx = cs / 33, cdi = cs - cdx * 33;
            const int crow0 = byl * 16 * G::CPD + bxl * 4;   // current block in curt (dwords)
            // U = min(SAD of the smallest-bound candidate, SAD at the previous frame's vector of
            // this block when that is a valid candidate): both SADs in one wave sum, packed in the
            // 16-bit halves (each <= 65,280).  The previous frame's vector is close to the minimum
            // for most blocks; with it a 4K bench P-frame leaves 9.5 instead of 15.9 survivors per
            // block, 0.18 % instead of 1.4 % past the cap (tests/analysis/sea_u_sources.py)
            const int pdx = (int)(int16_t)(pmv & 0xFFFFu), pdy = (int)pmv >> 16;
            const bool pv = pdx >= -SR && pdx <= SR && pdy >= -SR && pdy <= SR && x + pdx >= 0 && x + pdx < W - 16 &&
                            y + pdy >= 0 && y + pdy < H - 16;   // uniform
            uint32_t U;
            {
                const int row = lane >> 2, kk = lane & 3;
                const uint32_t c = curt[crow0 + row * G::CPD + kk];
                const uint32_t w = win_u32<RP>(win, byl * 16 + cdi + row, bxl * 16 + cdx + 4 * kk);
                uint32_t sp = __builtin_amdgcn_sad_u8(c, w, 0u);
                if (pv) {
                    const uint32_t wp = win_u32<RP>(win, byl * 16 + SR + pdy + row, bxl * 16 + SR + pdx + 4 * kk);
                    sp = __builtin_amdgcn_sad_hi_u8(c, wp, sp);
                }
                const uint32_t both = wave_sum_u32(sp);
                U = both & 0xFFFFu;
                if (pv && (both >> 16) < U) U = both >> 16;
                if (pv && lane == 0) SO_OPS_ADD(&st_ops, 256u);
            }
            if (probe == 2) {
                if (lane == 0 && U < keys[u]) keys[u] = U;
                continue;
            }
            // ---- 3. survivors: 16 LBq - 240 <= U, i.e. LBq <= qU = (U + 240) >> 4 ------------
            SO_MARK(ballots);
            const uint32_t qU = (U + 240) >> 4;
            // per-lane threshold (dx-invalid lanes: -1, nothing passes), opaque so that the
            // compare stays a plain v_cmp whose mask IS the ballot (folded back into
            // `xok && lb <= qU` it costs a 0/1 select and a second compare per row)
            int thr = xok ? (int)((qU << 16) | 0xFFFFu) : -1;
            asm volatile("" : "+v"(thr));
            // survivors by one wave ballot per candidate row t (t = NT: the dx = +16 column,
            // lanes < 33): rows nobody passes cost one compare and a scalar branch; the others
            // write their candidates at the running count + the lane's rank in the ballot (no
            // per-lane bit loops, no LDS atomics).  Writes past CAP are dropped: that block
            // takes the dense fallback below.
            uint16_t* mylist = list + wave * G::CAPL;
            const int cbase = xi * 33 + 16 * hh;
            uint32_t nsur = 0;
#pragma unroll
            for (int t = 0; t <= NT; ++t) {
                const bool pass = t < NT ? (int)lb[t] <= thr : (ok2 && lb2 <= qU);
                const uint64_t bal = __builtin_amdgcn_ballot_w64(pass);
                if (bal) {   // uniform
                    SO_MARK(bal_row);
                    const uint32_t pos = nsur + lane_prefix(bal);
                    if (pass && pos < (uint32_t)CAP) mylist[pos] = (uint16_t)(t < NT ? cbase + t : 32 * 33 + d2);
                    nsur += (uint32_t)__builtin_popcountll(bal);
                }
            }
#ifdef SO_STAMPS
            if (lane == 0) atomicAdd(&st_sur, nsur);
#endif
            if (nsur > (uint32_t)CAP) {
                if (lane == 0) {
                    atomicAdd(&st_fb, 1u);
                    SO_OPS_ADD(&st_ops, kDenseSadOps);
                }
                if (probe == 3) continue;
                SO_MARK(dense_fallback);
                // fallback: the dense wave search on the single-copy window
                wave_dense_block<16, false, RP, 0, false, true>(win, keys, G::NBLK, cur, W, H, x, y, bxl, byl, u, tid,
                                                                r);
                continue;
            }
            if (probe == 4) continue;
            SO_MARK(survivors);
            if (nsur == 1) {
                // the smallest-bound candidate cs always survives (16 LBq(cs) - 240 <= SAD(cs) = U),
                // so a lone survivor IS cs and its SAD is U: no second evaluation (the median
                // block on textured content)
                SO_MARK(sur_one);
                const int dx = cdx - 16, dy = cdi - 16;
                const uint64_t key = me_key(U, (uint32_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy)), (uint32_t)r,
                                            (uint32_t)cs);
                if (lane == 0 && key < keys[u]) keys[u] = key;
                continue;
            }
            if (lane == 0) SO_OPS_ADD(&st_ops, (nsur <= 4 ? 4u : 16u * ((nsur + 15) / 16)) * 256u);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            uint64_t best = kNoKey;
            if (nsur <= 4) {
                // one pass: 16 lanes (one DPP row) per survivor, a row per lane
                SO_MARK(sur_le4);
                const int sidx = lane >> 4, row = lane & 15;
                const uint32_t* cr_ = curt + crow0 + row * G::CPD;
                const uint32_t c0 = cr_[0], c1 = cr_[1], c2 = cr_[2], c3 = cr_[3];
                const bool act = (uint32_t)sidx < nsur;
                const int cand = act ? (int)mylist[sidx] : cs;
                const int dxi = cand / 33, di = cand - dxi * 33;
                const int col = bxl * 16 + dxi;
                int wo = (byl * 16 + di + row) * RP + (col >> 2);
                asm volatile("" : "+v"(wo));
                lds_vu32p p = (lds_vu32p)(win + wo);
                const uint32_t sh = (uint32_t)(col & 3);
                const uint32_t q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3], q4 = p[4];
                uint32_t sad = __builtin_amdgcn_sad_u8(c0, __builtin_amdgcn_alignbyte(q1, q0, sh), 0u);
                sad = __builtin_amdgcn_sad_u8(c1, __builtin_amdgcn_alignbyte(q2, q1, sh), sad);
                sad = __builtin_amdgcn_sad_u8(c2, __builtin_amdgcn_alignbyte(q3, q2, sh), sad);
                sad = __builtin_amdgcn_sad_u8(c3, __builtin_amdgcn_alignbyte(q4, q3, sh), sad);
                sad = row_sum_u32(sad);
                const int dx = dxi - 16, dy = di - 16;
                const uint64_t key = me_key(sad, (uint32_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy)),
                                            (uint32_t)r, (uint32_t)cand);
                best = (act && key < best) ? key : best;
            } else {
                // four lanes (one DPP quad) per survivor, rows 4q..4q+3 per lane: sixteen
                // survivors per pass (one survivor per lane left 3/4 of the lanes idle at the
                // typical 5..16 survivors)
                const int sidx = lane >> 2, q = lane & 3;
                uint32_t cr[4][4];
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
#pragma unroll
                    for (int k = 0; k < 4; ++k) cr[rr][k] = curt[crow0 + (4 * q + rr) * G::CPD + k];
#pragma unroll 1
                for (uint32_t s0 = 0; s0 < nsur; s0 += 16) {
                    SO_MARK(sur_pass);
                    const bool act = s0 + (uint32_t)sidx < nsur;
                    const int cand = act ? (int)mylist[s0 + sidx] : cs;
                    const int dxi = cand / 33, di = cand - dxi * 33;
                    const int col = bxl * 16 + dxi;
                    const uint32_t sh = (uint32_t)(col & 3);
                    int wo = (byl * 16 + di + 4 * q) * RP + (col >> 2);
                    asm volatile("" : "+v"(wo));
                    uint32_t sad = 0;
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr) {
                        lds_vu32p p = (lds_vu32p)(win + wo + rr * RP);
                        const uint32_t q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3], q4 = p[4];
                        sad = __builtin_amdgcn_sad_u8(cr[rr][0], __builtin_amdgcn_alignbyte(q1, q0, sh), sad);
                        sad = __builtin_amdgcn_sad_u8(cr[rr][1], __builtin_amdgcn_alignbyte(q2, q1, sh), sad);
                        sad = __builtin_amdgcn_sad_u8(cr[rr][2], __builtin_amdgcn_alignbyte(q3, q2, sh), sad);
                        sad = __builtin_amdgcn_sad_u8(cr[rr][3], __builtin_amdgcn_alignbyte(q4, q3, sh), sad);
                    }
                    sad = quad_sum_u32(sad);
                    const int dx = dxi - 16, dy = di - 16;
                    const uint64_t key = me_key(sad, (uint32_t)((dx < 0 ? -dx : dx) + (dy < 0 ? -dy : dy)),
                                                (uint32_t)r, (uint32_t)cand);
                    best = (act && key < best) ? key : best;
                }
            }
            best = wave_min_u64_dpp(best);
            if (lane == 0 && best < keys[u]) keys[u] = best;
        }
    }
    SO_MARK(search_end);
    __syncthreads();
}

__global__ void __launch_bounds__(Sea2Geo::NTHREADS) __attribute__((amdgpu_waves_per_eu(SO_SEA2_WPE)))
me_sea2_kernel(const uint8_t* __restrict__ cur, RefSet refs, int nref, int H, int W, int by0, int by1,
               int32_t* __restrict__ out_best, int probe) {
    using G = Sea2Geo;
    constexpr int SR = G::SR, TBX = G::TBX, TBY = G::TBY, RP = G::RP, B4P = G::B4P;
    __shared__ uint32_t win[G::WR * RP + 4];
    __shared__ uint32_t b4w[(G::B4RS * B4P + 4) / 4];
    __shared__ uint32_t curt[G::TPY * G::CPD];
    __shared__ uint32_t a4[G::NBLK * 4];
    __shared__ uint16_t list[G::NW * G::CAPL];
    __shared__ uint32_t lcount[G::NW];
    __shared__ unsigned long long keys[G::NBLK];
    __shared__ uint32_t st[3];
    const Sea2Lds L{win, b4w, curt, a4, list, lcount, keys, st};
    SO_STAMP_REC_SET(g_sea_stamps ? g_sea_stamps + (size_t)blockIdx.x * 12 : nullptr);
    sea2_tile<Sea2Geo>(L, blockIdx.x, cur, refs, nref, H, W, by0, by1, probe);

    const int tid = threadIdx.x;
    const int nbx = W / 16;
    const int tiles_x = (nbx + TBX - 1) / TBX;
    const int bx0 = (blockIdx.x % tiles_x) * TBX, byt0 = by0 + (blockIdx.x / tiles_x) * TBY;
    SO_SEA_STAMP(5, __builtin_amdgcn_s_memtime());
    for (int i = tid; i < G::NBLK; i += G::NTHREADS) {
        const int gbx = bx0 + i % TBX, gby = byt0 + i / TBX;
        if (gbx >= nbx || gby >= by1) continue;
        decode_key(keys[i], SR, out_best + ((size_t)(gby - by0) * nbx + gbx) * 4);
    }
#ifdef SO_STAMPS
    if (tid == 0) {
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        SO_SEA_STAMP(6, __builtin_amdgcn_s_memtime());
        SO_SEA_STAMP(7, __builtin_amdgcn_s_memrealtime());
        SO_SEA_STAMP(8, ((unsigned long long)xcc << 32) | hw);
        SO_SEA_STAMP(9, ((unsigned long long)st[0] << 32) | st[1]);
    }
#endif
}

// ---------------------------------------------------------------------------------------
// Fused P-frame tile (p_tile_kernel, the default for bs 16 / sr 16 / no VBS / one reference):
// the SEA search of a 128x32 tile (sea2_tile) followed, in the same workgroup, by the
// transform / quantisation / token / reconstruction of its 16 blocks -- the arithmetic of
// inter_tq_kernel<16, false, false> (so_tq.hip), which replaces calculate_inter_frame_residual
// (Encoder.py:432-460), apply_2d_dct (:779), quantize_TC (:787), len(entropy_encoder_block)
// (:1086) and reconstruct_frame (:824-932).
//   * One launch per frame (or stripe) instead of two: the ME launch's ramp / tail overlaps
//     other workgroups' transform work and vice versa.
//   * The prediction rows come from the LDS window the search used (it spans +-16 around the
//     tile and is zero outside the frame, which is also handle_boundary_conditions' zero
//     fill for the no-valid-candidate case), the current rows from the LDS tile: the
//     transform phase reads nothing from HBM.
//   * The transposes' FP64 scratch reuses the LDS of the byte sums and survivor lists.
// Waves 0-3 run the transforms (16 lanes per block); the ME records are also written to
// `out_best` when it is given (SO_REUSE_ME, the two-pass RC's second pass, reads them).
//
// p_run_kernel runs a whole run of P-frames (so_encode_p_run) as one persistent launch:
// workgroups take (frame, tile) tasks from a queue in frame-major raster order, and a tile
// of frame f starts once the 3x3 tiles of frame f-1 its +-16 px window reads are done, so
// frame f's first rows overlap frame f-1's last ones and only the run's last frame has a
// launch tail (a launch per frame leaves ~25% of the machine idle in its tail,
// tools/sea_stamps.py).  Per-tile flags (not per-row counters) matter at 1080p, where
// fewer tiles than resident workgroups make the frame-to-frame latency the limit.
// ---------------------------------------------------------------------------------------
// FP64 transpose scratch per block of the fused tile: 16 x 17 doubles.  (Two-half transposes,
// 16 x 9, would let 4 workgroups fit per CU but spill at 64-80 VGPRs: measured slower, DESIGN.md.)
constexpr int kTqScratch = 16 * 17;
// The tokens-only pass-1 tile (p_tile_kernel<8, true>) transforms through half of it (16 x 9,
// xform2d_fwd_i_half): 33.7 KB of LDS per workgroup, four workgroups per CU instead of three
#ifndef SO_PTILE_TOK_HALF
#define SO_PTILE_TOK_HALF 1
#endif
constexpr int kTqScratchHalf = 16 * 9;
// SO_FWD_MFMA=1: the fused tiles' forward transform on the matrix cores with an exactness
// certificate (fwd_mfma).  Bit-exact (the GPU suite passes through it) but measured slower, so
// off: 73.6 vs 67.0 us per 4K P-frame -- the FP32 MFMA runs at the FP32 vector rate and does not
// hide behind the other waves' VALU here, and the certificate costs ~19 lane operations per
// coefficient against ~7 for the FP64 pocketfft forward it replaces.
#ifndef SO_FWD_MFMA
#define SO_FWD_MFMA 0
#endif
template <class G, bool HALFTQ = false>
struct PTileGeo {
    static constexpr int B4 = (G::B4RS * G::B4P + 4) / 4;             // dwords
    static constexpr int LIST = G::NW * G::CAPL / 2;                  // dwords
    static constexpr int TQD = G::NBLK * (HALFTQ ? kTqScratchHalf : kTqScratch);   // doubles
    static constexpr int U64 = ((B4 + LIST + 1) / 2 > TQD) ? (B4 + LIST + 1) / 2 : TQD;
};
// VBSEnable (tq16_vbs): 16 x 18 doubles per block (the 16 x 17 transpose of the block, or the
// four 8 x 9 of its sub-blocks); between tq16_vbs_fwd and tq16_vbs_inv the same scratch holds the
// block's chosen levels (16 lanes x 8 packed int16 pairs).  Sub-block tokens: registers
// (sub_tokens_reg).  LDS per tile 53.9 KB: three workgroups per CU (160 KB).
constexpr int kTqScratchVbs = 288;
template <class G>
struct PTileGeoVbs {
    static constexpr int TQD = G::NBLK * kTqScratchVbs;
    static constexpr int U64 = ((PTileGeo<G>::B4 + PTileGeo<G>::LIST + 1) / 2 > TQD)
                                   ? (PTileGeo<G>::B4 + PTileGeo<G>::LIST + 1) / 2 : TQD;
};

// 16 bytes of window row `row` from byte column `col`, as 4 dwords (5 aligned ds_read_b32
// + v_alignbyte: misaligned wide DS reads are replayed on gfx950)
template <int RP>
SO_DEV void win_row16(const uint32_t* win, int row, int col, uint32_t (&w)[4]) {
    lds_vu32p p = (lds_vu32p)(win + row * RP + (col >> 2));
    const uint32_t sh = (uint32_t)(col & 3);
    const uint32_t q0 = p[0], q1 = p[1], q2 = p[2], q3 = p[3], q4 = p[4];
    w[0] = __builtin_amdgcn_alignbyte(q1, q0, sh);
    w[1] = __builtin_amdgcn_alignbyte(q2, q1, sh);
    w[2] = __builtin_amdgcn_alignbyte(q3, q2, sh);
    w[3] = __builtin_amdgcn_alignbyte(q4, q3, sh);
}

typedef uint32_t so_v4u __attribute__((ext_vector_type(4)));

// A decoded ME record in LDS: dx, dy, ref as int16 and the SAD as uint16 (a 16 x 16 SAD is at
// most 65,280; 0xFFFF = no valid candidate, decode_key's -1).  Half the bytes of four int32:
// the VBS tile's 80 records then leave its LDS at 53.2 KB, under the 53,760 B at which a CU
// still holds three workgroups (tools/ubench_lds_occ.cpp: 53,880 B gives two, although the
// occupancy API reports three).
struct MeRec {
    uint16_t v[4];
    SO_DEV int operator[](int k) const { return k < 3 ? (int)(int16_t)v[k] : (v[3] == 0xFFFFu ? -1 : (int)v[3]); }
    SO_DEV void set(const int32_t (&r)[4]) {
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = (uint16_t)r[k];
    }
};

// The LDS of one fused tile.
// VBS: keys / mer hold the 16 blocks' records, then the 4 sub-blocks of each (NBLK + 4 g + j).
template <class G, bool VBS = false, bool HALFTQ = false>
struct PTileLds {
    static constexpr int NU = G::NBLK * (VBS ? 5 : 1);
    uint32_t win[G::WR * G::RP + 4];
    uint32_t curt[G::TPY * G::CPD];
    uint32_t a4[G::NBLK * 4];
    uint32_t lcount[G::NW];
    unsigned long long keys[NU];
    uint32_t st[3];
    MeRec mer[NU];                         // decoded ME records (dx, dy, ref, sad)
    int32_t msum[G::TBY];                  // two-pass runs: pass-1 token sum of each block row
    uint32_t fwd_flags;                    // fwd_mfma: blocks whose levels need the FP64 forward
    alignas(16) double un[VBS ? PTileGeoVbs<G>::U64 : PTileGeo<G, HALFTQ>::U64];   // byte sums + survivor lists | FP64 transposes
    // VBS: each block's split state (0 block, 1 split, 2 none) between tq16_vbs_fwd and
    // tq16_vbs_inv (its levels wait in its transpose scratch)
    uint8_t vsp[VBS ? G::NBLK : 1];
};

// Boundary rows of a rank's stripe that the neighbouring ranks read (so_encode_p_run_stripe):
// rows [y0s, up_end) are also stored into the up neighbour's landing plane of the frame, rows
// [dn_begin, y1s) into the down neighbour's ("virtual" full-frame bases: row y of the frame is
// at base + y * W).  Null = no such neighbour.
struct PHalo {
    uint8_t* up;
    uint8_t* dn;
    int up_end, dn_begin;
};

// The exact transform path of one block: 16 lanes (l = row) run scipy.fftpack's pocketfft
// DCT-II / DCT-III sequence in FP64 (so_dct.h) -- the arithmetic of inter_tq_kernel<16,
// false, false>.  `scratch` = 16 x 17 doubles of LDS owned by the calling lanes.
// `qs` (fwd_mfma): the block's levels, already certified (16 x 16 int16 at the start of
// `scratch`); null = run the FP64 forward transform here.
// The twiddles of tq16_exact's transforms: scalar loads from the constant table, behind one
// optimisation barrier per 2-D transform (dct::tw16_table); -DSO_TQ_TW_LITERAL: as literals.
#ifdef SO_TQ_TW_LITERAL
#define SO_TQ_TW() dct::TW16{}
#define SO_TQ_TW8() dct::TW8{}
#else
#define SO_TQ_TW() dct::tw16_table()
#define SO_TQ_TW8() dct::tw8_table()
#endif
// ZSKIP (SO_OPT_RUN_ZERO_SKIP): a wave whose four blocks all quantised to zero skips the IDCT
template <class G, bool SC1, bool HALO = false, bool TOK = false, bool HALFTQ = false, bool ZSKIP = false>
SO_DEV void tq16_exact(PTileLds<G, false, HALFTQ>& S, int g, int l, double* scratch, int bx0, int byt0, int nbx, int by0, int by1,
                       int W, int qp_rd, const int32_t* __restrict__ qp_row, const int32_t* __restrict__ qp_map,
                       const PFrameOut& o, const PHalo& hl = PHalo{}, bool qs = false) {
    constexpr int SR = G::SR, TBX = G::TBX;
    const int bxl = g % TBX, byl = g / TBX;
    const int gbx = bx0 + bxl, gby = byt0 + byl;
    if (gbx < nbx && gby < by1) {   // uniform over the block's 16 lanes
        const size_t b = (size_t)(gby - by0) * nbx + gbx;
        const int x = gbx * 16, y = gby * 16;
        const int qpr = qp_map ? qp_map[(size_t)gby * nbx + gbx] : (qp_row ? qp_row[gby] : qp_rd);
        const int dx = S.mer[g][0], dy = S.mer[g][1], rf = S.mer[g][2], sad = S.mer[g][3];
        const int prow = byl * 16 + SR + dy + l, pcol = bxl * 16 + SR + dx;   // window coordinates
        const uint32_t* crow = S.curt + (byl * 16 + l) * G::CPD + bxl * 4;
        double* dl = scratch;
        // np.round to int by the 1.5 * 2^52 shift (|values| < 2^51): x + kRne rounds x to an
        // integer half-to-even, held in the low mantissa dword as two's complement -- one
        // v_add_f64 instead of v_rndne + v_cvt_i32
        constexpr double kRne = 0x1.8p52;
        int q[16];
        if (qs) {
            const so_v4u* qr = reinterpret_cast<const so_v4u*>(reinterpret_cast<const int16_t*>(dl) + l * 16);
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const so_v4u v = qr[h];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    q[8 * h + 2 * e] = (int)(int16_t)(v[e] & 0xFFFFu);
                    q[8 * h + 2 * e + 1] = (int)v[e] >> 16;
                }
            }
        } else {
            SO_MARK(tq_residual);
            int res[16];
            {
                uint32_t pw[4];
                win_row16<G::RP>(S.win, prow, pcol, pw);
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t cw = crow[k];
#pragma unroll
                    for (int e = 0; e < 4; ++e)
                        res[4 * k + e] = (int)((cw >> (8 * e)) & 255) - (int)((pw[k] >> (8 * e)) & 255);
                }
            }
            double tcr[16];
            SO_MARK(tq_fwd);
            static_assert(!HALFTQ || TOK, "the half scratch carries the forward transform only");
            if constexpr (HALFTQ)
                xform2d_fwd_i_half(dl, l, res, tcr, SO_TQ_TW());
            else
                xform2d_rows<16, false>(dl, l, res, tcr, SO_TQ_TW());
            SO_MARK(tq_quant);
#pragma unroll
            for (int c = 0; c < 16; ++c)
                q[c] = (int)(uint32_t)__builtin_bit_cast(
                    uint64_t, __builtin_amdgcn_ldexp(__builtin_rint(tcr[c]), -q_exp_fast<16>(l, c, qpr)) + kRne);
        }
        SO_MARK(tq_tokens);
        const int tok = block_tokens<16>(nullptr, l, q);
        if constexpr (TOK) {   // pass 1 of two-pass RC: the token count is all that is used
            if (l == 0) o.tokens[b] = tok;
            return;
        }
        SO_MARK(tq_qtc_store);
        store_row_i16<16>(o.qtc + b * 256 + l * 16, q);
        // the reconstruction row's store (write-through, plus the neighbours' halo rows) and
        // its SSE: the tail of both paths below
        const auto finish = [&](const int (&rec)[16]) -> int {
            if constexpr (SC1) {
                so_v4u v;
#pragma unroll
                for (int k = 0; k < 4; ++k)
                    v[k] = (uint32_t)(rec[4 * k] & 255) | ((uint32_t)(rec[4 * k + 1] & 255) << 8) |
                           ((uint32_t)(rec[4 * k + 2] & 255) << 16) | ((uint32_t)(rec[4 * k + 3] & 255) << 24);
                uint8_t* rp = o.recon + (size_t)(y + l) * W + x;
                asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(rp), "v"(v) : "memory");
                if constexpr (HALO) {
                    // the rows a neighbouring rank's window reads: system-scope write-through
                    // stores into its uncached landing plane (peer memory over xGMI)
                    if (hl.up && y + l < hl.up_end) {
                        uint8_t* q2 = hl.up + (size_t)(y + l) * W + x;
                        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q2), "v"(v) : "memory");
                    }
                    if (hl.dn && y + l >= hl.dn_begin) {
                        uint8_t* q2 = hl.dn + (size_t)(y + l) * W + x;
                        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q2), "v"(v) : "memory");
                    }
                }
            } else {
                store_row_u8<16>(o.recon, W, x, y + l, rec);
            }
            SO_MARK(tq_sse_records);
            int e2 = 0;
            if (o.sse) {
#pragma unroll
                for (int k = 0; k < 4; ++k) {
                    const uint32_t cw = crow[k];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int d = (int)((cw >> (8 * e)) & 255) - (rec[4 * k + e] & 255);
                        e2 += d * d;
                    }
                }
                e2 = group_sum<16>(e2);
            }
            return e2;
        };
        const auto full = [&]() -> int {   // dequantisation, IDCT, prediction + inverse
            int dq[16];
            double rd[16];
            dequant_row_int<16>(q, l, qpr, dq);
            SO_MARK(tq_inv);
            xform2d_rows<16, true>(dl, l, dq, rd, SO_TQ_TW());
            SO_MARK(tq_recon);
            int rec[16];
            {
                uint32_t pw[4];
                win_row16<G::RP>(S.win, prow, pcol, pw);
#pragma unroll
                for (int c = 0; c < 16; ++c)
                    rec[c] = (int)((pw[c >> 2] >> (8 * (c & 3))) & 255) +
                             (int)(uint32_t)__builtin_bit_cast(uint64_t, rd[c] + kRne);
            }
            return finish(rec);
        };
        int sse;
        if constexpr (ZSKIP) {
            // a block whose levels are all zero (tok == 1: no non-zero, one zero run) has an
            // exactly zero inverse (every step of pocketfft's sequence on zeros gives +-0,
            // rounded to 0): a wave whose blocks are all such reconstructs its prediction rows
            // as they stand.  Its own instantiation (SO_OPT_RUN_ZERO_SKIP), chosen by the host
            // for content where most blocks quantise to zero: in the default kernel the branch
            // cost two spills and +0.3-0.5 % on textured content
            if (__builtin_amdgcn_ballot_w64(tok != 1) == 0) {
                int rec[16];
                uint32_t pw[4];
                win_row16<G::RP>(S.win, prow, pcol, pw);
#pragma unroll
                for (int c = 0; c < 16; ++c) rec[c] = (int)((pw[c >> 2] >> (8 * (c & 3))) & 255);
                sse = finish(rec);
            } else {
                sse = full();
            }
        } else {
            sse = full();
        }
        if (l < 12) o.mv[b * 12 + l] = (int16_t)(l == 0 ? dx : l == 1 ? dy : l == 2 ? rf : 0);
        if (l == 0) {
            o.split[b] = 0;
            o.tokens[b] = tok;
            o.mae[b] = sad;
            if (o.sse) o.sse[b] = sse;
        }
    }
}

// ---- the forward transform on the matrix cores (SO_FWD_MFMA) -------------------------------
// fwd_mfma: Z = C R C^T of one block on one wave's 64 lanes, 8 v_mfma_f32_16x16x4_f32, then a
// certificate per coefficient that the FP32 result quantises to the level pocketfft's FP64
// one does (tq16_exact: the arithmetic of Encoder.py:781-789):
//  * bound: an MFMA step is a k-ordered chain of single-rounding FP32 FMAs, so a 16-term chain
//    is within gamma_16 ~ 16u sum|a b| of its exact value (u = 2^-24); the matrix entries
//    (dct16_f32) are within u relative of C.  The two products together:
//    |z - Z| <= 34.04 u max|C_ur C_vk| sum|R| <= 2.512e-7 sum|R|  (max|C_ur C_vk| = 0.1238),
//    and pocketfft's FP64 result is within 1e-11 of Z.
//  * the level q(Z) = rne(rint(Z) / 2^k) is, for k >= 1, constant in Z except for steps at
//    mid +- 1/2, mid = (floor(Z / 2^k) + 1/2) 2^k.  When ||z - mid| - 1/2| > delta (both
//    differences exact where they matter, Sterbenz), no step lies within delta of z and
//    q(z) == q(pocketfft).  k = 0 (qp 0) steps at every half-integer: such blocks are flagged.
// A flagged block (some coefficient within delta of mid +- 1/2: ~4 delta / 2^k of them, 3-6 %
// of the blocks at QP 4) gets the FP64 forward in phase B.
__constant__ float kDctCos32[17] = {
    0x1.6a09e6p-2f, 0x1.684b9cp-2f, 0x1.63150cp-2f, 0x1.5a730cp-2f, 0x1.4e7aeap-2f, 0x1.3f4a24p-2f,
    0x1.2d062ep-2f, 0x1.17dc14p-2f, 0x1.000000p-2f, 0x1.cb598cp-3f, 0x1.92469cp-3f, 0x1.5553e4p-3f,
    0x1.1517a8p-3f, 0x1.a4608ap-4f, 0x1.1a855ep-4f, 0x1.1be352p-5f, 0.0f};   // fl32(sqrt(1/8) cos(pi j / 32))

// C[u][r] of the orthonormal 16-point DCT-II (scipy.fftpack.dct norm='ortho') in FP32
SO_DEV float dct16_f32(int u, int r) {
    if (u == 0) return 0.25f;
    const int j = ((2 * r + 1) * u) & 63;
    const int m = j <= 32 ? j : 64 - j;
    return m <= 16 ? kDctCos32[m] : -kDctCos32[32 - m];
}

typedef float so_v4f __attribute__((ext_vector_type(4)));
constexpr float kFwdBound = 2.6e-7f;   // >= 2.512e-7 (above) + the rounding of delta itself

// One block on one wave: lane (c4 = ln >> 4, r = ln & 15) feeds R[r][4 c4 + s] and
// C[r][4 c4 + s] at MFMA step s (A[i][k] = lane (k, i), B[k][j] = lane (k, j)); the first
// product's D (lane (c4, v): Y[4 c4 + i][v]) is the second's B operand as it stands.  Writes
// the 256 levels as int16 rows to the start of the block's scratch and flags the block in
// S.fwd_flags when the certificate fails.
template <class G>
SO_DEV void fwd_mfma(PTileLds<G>& S, int g, int ln, const float (&cs)[4], int bx0, int byt0, int nbx, int by1,
                     int qp_rd, const int32_t* __restrict__ qp_row, const int32_t* __restrict__ qp_map) {
    constexpr int SR = G::SR, TBX = G::TBX;
    const int bxl = g % TBX, byl = g / TBX;
    const int gbx = bx0 + bxl, gby = byt0 + byl;
    if (gbx >= nbx || gby >= by1) return;   // uniform over the wave
    const int qpr = qp_map ? qp_map[(size_t)gby * nbx + gbx] : (qp_row ? qp_row[gby] : qp_rd);
    const int r = ln & 15, c4 = ln >> 4;
    const int dx = S.mer[g][0], dy = S.mer[g][1];
    const uint32_t cw = S.curt[(byl * 16 + r) * G::CPD + bxl * 4 + c4];
    const uint32_t pw = win_u32<G::RP>(S.win, byl * 16 + SR + dy + r, bxl * 16 + SR + dx + 4 * c4);
    float a[4];
    uint32_t sab = 0;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
        const int d = (int)((cw >> (8 * s)) & 255) - (int)((pw >> (8 * s)) & 255);
        a[s] = (float)d;
        sab += (uint32_t)(d < 0 ? -d : d);
    }
    sab = wave_sum_u32(sab);
    so_v4f y = {0.f, 0.f, 0.f, 0.f}, z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < 4; ++s) y = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s], cs[s], y, 0, 0, 0);   // Y = R C^T
#pragma unroll
    for (int s = 0; s < 4; ++s) z = __builtin_amdgcn_mfma_f32_16x16x4f32(cs[s], y[s], z, 0, 0, 0);   // Z = C Y
    const float delta = __builtin_fmaf((float)sab, kFwdBound, 0x1p-20f);
    bool near = qpr < 1;
    int16_t* qd = reinterpret_cast<int16_t*>(S.un + g * kTqScratch);
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // z[i] = Z[4 c4 + i][r]
        const int u = 4 * c4 + i, k = q_exp_fast<16>(u, r, qpr);
        const float zi = z[i];
        const float mid = __builtin_amdgcn_ldexpf(__builtin_floorf(__builtin_amdgcn_ldexpf(zi, -k)) + 0.5f, k);
        near |= __builtin_fabsf(__builtin_fabsf(zi - mid) - 0.5f) <= delta;
        qd[u * 16 + r] = (int16_t)(int)__builtin_rintf(__builtin_amdgcn_ldexpf(__builtin_rintf(zi), -k));
    }
#ifdef SO_FWD_FORCE   // A/B timing builds only: 0 = never flagged (wrong levels), 1 = always
    near = SO_FWD_FORCE;
#endif
    if (__builtin_amdgcn_ballot_w64(near) != 0 && ln == 0) atomicOr(&S.fwd_flags, 1u << g);
}

// Phase-B position p -> block: the flagged blocks first (so their FP64 forwards share waves),
// then the rest, each in block order.
template <int NBLK>
SO_DEV int fwd_order(uint32_t m, int p) {
    const int nf = __builtin_popcount(m);
    uint32_t s = p < nf ? m : (~m & ((1u << NBLK) - 1u));
    for (int t = p < nf ? p : p - nf; t > 0; --t) s &= s - 1u;
    return __builtin_ctz(s);
}

// 8 bytes of window row `row` from byte column `col`, as 2 dwords (3 aligned ds_read_b32 +
// v_alignbyte)
template <int RP>
SO_DEV void win_row8(const uint32_t* win, int row, int col, uint32_t (&w)[2]) {
    lds_vu32p p = (lds_vu32p)(win + row * RP + (col >> 2));
    const uint32_t sh = (uint32_t)(col & 3);
    const uint32_t q0 = p[0], q1 = p[1], q2 = p[2];
    w[0] = __builtin_amdgcn_alignbyte(q1, q0, sh);
    w[1] = __builtin_amdgcn_alignbyte(q2, q1, sh);
}

// One 16-byte (or 8-byte) reconstruction row: local store write-through (sc1) and, for the
// multi-GPU hand-off, the same bytes into a neighbour's landing plane (system scope).
template <bool SC1, bool HALO>
SO_DEV void store_rec_row(const PFrameOut& o, const PHalo& hl, int W, int x, int yy, const int* rec, int n) {
    uint8_t* rp = o.recon + (size_t)yy * W + x;
    if (n == 16) {
        so_v4u v;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = (uint32_t)(rec[4 * k] & 255) | ((uint32_t)(rec[4 * k + 1] & 255) << 8) |
                   ((uint32_t)(rec[4 * k + 2] & 255) << 16) | ((uint32_t)(rec[4 * k + 3] & 255) << 24);
        if constexpr (SC1) {
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(rp), "v"(v) : "memory");
            if constexpr (HALO) {
                if (hl.up && yy < hl.up_end) {
                    uint8_t* q = hl.up + (size_t)yy * W + x;
                    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q), "v"(v) : "memory");
                }
                if (hl.dn && yy >= hl.dn_begin) {
                    uint8_t* q = hl.dn + (size_t)yy * W + x;
                    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q), "v"(v) : "memory");
                }
            }
        } else {
            *reinterpret_cast<so_v4u*>(rp) = v;
        }
    } else {
        typedef uint32_t so_v2u __attribute__((ext_vector_type(2)));
        so_v2u v;
#pragma unroll
        for (int k = 0; k < 2; ++k)
            v[k] = (uint32_t)(rec[4 * k] & 255) | ((uint32_t)(rec[4 * k + 1] & 255) << 8) |
                   ((uint32_t)(rec[4 * k + 2] & 255) << 16) | ((uint32_t)(rec[4 * k + 3] & 255) << 24);
        if constexpr (SC1) {
            asm volatile("global_store_dwordx2 %0, %1, off sc1" ::"v"(rp), "v"(v) : "memory");
            if constexpr (HALO) {
                if (hl.up && yy < hl.up_end) {
                    uint8_t* q = hl.up + (size_t)yy * W + x;
                    asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(q), "v"(v) : "memory");
                }
                if (hl.dn && yy >= hl.dn_begin) {
                    uint8_t* q = hl.dn + (size_t)yy * W + x;
                    asm volatile("global_store_dwordx2 %0, %1, off sc0 sc1" ::"v"(q), "v"(v) : "memory");
                }
            }
        } else {
            *reinterpret_cast<so_v2u*>(rp) = v;
        }
    }
}

// The VBSEnable transform path of one block inside the fused tile: the arithmetic of
// inter_tq_kernel<16, true, false> (so_tq.hip) -- DCT of the block at the RD QP, the four 8x8
// sub-blocks at max(QP - 1, 0) when x != 0 and y != 0, calculate_RD_cost of both and the
// split decision !(cost_bs < cost_vbs) (Encoder.py:512-578, :1133-1158), then the chosen
// path's requantisation at the block's final QP, IDCT and reconstruction -- with every pixel
// read from the LDS tile (current rows) and window (predictions: block and sub-block MVs lie
// inside the window's +-16 px, zero outside the frame as handle_boundary_conditions).
// 16 lanes (l = row); `scratch` 288 doubles, `flags` 256 bytes of LDS owned by the lanes.
// int16 pairs: the transform coefficients and quantised levels (|v| <= 4080) that must survive
// the RD decision live packed, two per VGPR (the VBS tile kernel is register-bound)
template <int N>
SO_DEV void pack_i16(const int* v, uint32_t* p) {
#pragma unroll
    for (int k = 0; k < N / 2; ++k) p[k] = ((uint32_t)v[2 * k] & 0xFFFFu) | ((uint32_t)v[2 * k + 1] << 16);
}
template <int N>
SO_DEV void unpack_i16(const uint32_t* p, int* v) {
#pragma unroll
    for (int k = 0; k < N / 2; ++k) {
        v[2 * k] = (int)(int16_t)(p[k] & 0xFFFFu);
        v[2 * k + 1] = (int)p[k] >> 16;
    }
}

template <class G, bool SC1, bool HALO = false>
SO_DEV void tq16_vbs_fwd(PTileLds<G, true>& S, int g, int l, double* scratch, int bx0, int byt0, int nbx,
                         int by0, int by1, int W, int qp_rd, const int32_t* __restrict__ qp_row,
                         const int32_t* __restrict__ qp_map, double lam, const PFrameOut& o) {
    constexpr int SR = G::SR, TBX = G::TBX;
    const int bxl = g % TBX, byl = g / TBX;
    const int gbx = bx0 + bxl, gby = byt0 + byl;
    if (gbx >= nbx || gby >= by1) {   // uniform over the block's 16 lanes
        if (l == 0) S.vsp[g] = 2;        // no block: no inverse
        return;
    }
    const size_t b = (size_t)(gby - by0) * nbx + gbx;
    const int x = gbx * 16, y = gby * 16;
    const int qpr = qp_map ? qp_map[(size_t)gby * nbx + gbx] : (qp_row ? qp_row[gby] : qp_rd);
    const int dx = S.mer[g][0], dy = S.mer[g][1], rf = S.mer[g][2], sad = S.mer[g][3];
    const int prow = byl * 16 + SR + dy + l, pcol = bxl * 16 + SR + dx;   // window coordinates
    const uint32_t* crow = S.curt + (byl * 16 + l) * G::CPD + bxl * 4;
    // The chosen levels go to the block's QTC rows.  The block's levels at the RD QP are stored
    // there as soon as they exist: when the block is not split and its QP is the RD QP (no
    // per-row / per-block QP: always), that store is final, neither the levels nor their tokens
    // are recomputed, and tq16_vbs_inv reads them back from there (after the tile's barrier; the
    // same workgroup, so the same L1).  A split block's levels also wait in its scratch for the
    // inverse.  Only the block's coefficients stay in registers through the sub-block
    // transforms (packed int16 pairs, |TC| <= 4080), to requantise at another QP.
    uint32_t tcp[8];
    int tok_b = 0;
    SO_MARK(vbs_fwd);
    {
        int res[16];
        uint32_t pw[4];
        win_row16<G::RP>(S.win, prow, pcol, pw);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t cw = crow[k];
#pragma unroll
            for (int e = 0; e < 4; ++e) res[4 * k + e] = (int)((cw >> (8 * e)) & 255) - (int)((pw[k] >> (8 * e)) & 255);
        }
        double tcr[16];
        xform2d_rows<16, false>(scratch, l, res, tcr, SO_TQ_TW());
        int tc[16], q[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) tc[c] = (int)__builtin_rint(tcr[c]);
        quant_row_int<16>(tc, l, qp_rd, q);
        tok_b = block_tokens<16>(nullptr, l, q);
        store_row_i16<16>(o.qtc + b * 256 + l * 16, q);
        pack_i16<16>(tc, tcp);
    }
    bool split = false;
    int mae_num = sad, tok = tok_b;
    const int j = l >> 2, r0 = l & 3;
    const int qpm1_rd = qp_rd > 0 ? qp_rd - 1 : qp_rd;
    if (x != 0 && y != 0) {   // uniform
        SO_MARK(vbs_fwd_sub);
        const MeRec& sm = S.mer[G::NBLK + 4 * g + j];
        const int sdx = sm[0], sdy = sm[1], sref = sm[2];
        const int sxl = bxl * 16 + (j & 1) * 8, syl = byl * 16 + (j >> 1) * 8;   // sub-block in the tile (px)
        int sres[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = r0 + 4 * h;
            uint32_t pw[2];
            win_row8<G::RP>(S.win, syl + SR + sdy + row, sxl + SR + sdx, pw);
            const uint32_t* cr = S.curt + (syl + row) * G::CPD + (sxl >> 2);
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t cw = cr[k];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    sres[h][4 * k + e] = (int)((cw >> (8 * e)) & 255) - (int)((pw[k] >> (8 * e)) & 255);
            }
        }
        double std_[2][8];
        xform2d_sub<false>(scratch, l, sres, std_, SO_TQ_TW8());
        int stc[2][8], qs[2][8];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
#pragma unroll
            for (int c = 0; c < 8; ++c) stc[h][c] = (int)__builtin_rint(std_[h][c]);
            quant_row_int<8>(stc[h], r0 + 4 * h, qpm1_rd, qs[h]);
        }
        const int tok_v = sub_tokens_reg(l, qs);
        // the sub-blocks' levels and coefficients wait in the (now free) transpose scratch, packed:
        // [l * 8, +8) the levels (an int16 row pair per lane, as the QTC rows hold them), [128 + l
        // * 8, +8) the coefficients -- through the decision the lanes hold only the block's tcp
        uint32_t* const sl = reinterpret_cast<uint32_t*>(scratch);
        {
            uint32_t pq[8], pc[8];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                pack_i16<8>(qs[h], pq + 4 * h);
                pack_i16<8>(stc[h], pc + 4 * h);
            }
            so_v4u* const d = reinterpret_cast<so_v4u*>(sl + l * 8);
            d[0] = so_v4u{pq[0], pq[1], pq[2], pq[3]};
            d[1] = so_v4u{pq[4], pq[5], pq[6], pq[7]};
            so_v4u* const e = reinterpret_cast<so_v4u*>(sl + 128 + l * 8);
            e[0] = so_v4u{pc[0], pc[1], pc[2], pc[3]};
            e[1] = so_v4u{pc[4], pc[5], pc[6], pc[7]};
        }
        int ssum = 0;
        bool vinf = false;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int sk = S.mer[G::NBLK + 4 * g + k][3];
            vinf |= sk < 0;
            ssum += sk;
        }
        const double mae_b = sad < 0 ? __builtin_inf() : (double)sad / 256.0;
        const double mae_v = vinf ? __builtin_inf() : (double)ssum / 256.0;
        const double c_v = rd_cost(lam, 64 + 8 * tok_v, mae_v);
        const double c_b = rd_cost(lam, 16 + 8 * tok_b, mae_b);
        split = !(c_b < c_v);
        mae_num = vinf ? -1 : ssum;   // the sub-blocks' SAD sum, split or not (as inter_tq_kernel)
        SO_MARK(vbs_final_q);
        if (split) {   // uniform: the sub-blocks' levels at the block's final QP - 1
            const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
            so_v4u* const d = reinterpret_cast<so_v4u*>(sl + l * 8);
            if (qpm1 != qpm1_rd) {   // uniform: requantise the coefficients at the block's QP - 1
                const so_v4u* const e = reinterpret_cast<const so_v4u*>(sl + 128 + l * 8);
                int qf[2][8];
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const so_v4u v = e[h];
                    const uint32_t pc[4] = {v[0], v[1], v[2], v[3]};
                    int t8[8];
                    unpack_i16<8>(pc, t8);
                    int rq = r0 + 4 * h;
                    asm volatile("" : "+v"(rq));   // (as lq below)
                    quant_row_int<8>(t8, rq, qpm1, qf[h]);
                }
                tok = sub_tokens_reg(l, qf);
                uint32_t pq[8];
#pragma unroll
                for (int h = 0; h < 2; ++h) pack_i16<8>(qf[h], pq + 4 * h);
                d[0] = so_v4u{pq[0], pq[1], pq[2], pq[3]};
                d[1] = so_v4u{pq[4], pq[5], pq[6], pq[7]};
            } else {
                tok = tok_v;
            }
            // the packed pairs are the QTC rows' int16 layout: 16-byte stores as they stand
#pragma unroll
            for (int h = 0; h < 2; ++h)
                *reinterpret_cast<so_v4u*>(o.qtc + b * 256 + j * 64 + (r0 + 4 * h) * 8) = d[h];
            if (r0 < 3) o.mv[b * 12 + 3 * j + r0] = (int16_t)(r0 == 0 ? sdx : r0 == 1 ? sdy : sref);
        }
    }
    // the row index behind an optimisation barrier for the requantisations below: otherwise the
    // per-coefficient exponents of the RD-QP quantisation are kept (spilled) to be reused here
    int lq = l;
    asm volatile("" : "+v"(lq));
    if (!split) {
        if (qpr != qp_rd) {   // uniform: requantise at the block's own QP
            int tc[16], q[16];
            unpack_i16<16>(tcp, tc);
            quant_row_int<16>(tc, lq, qpr, q);
            tok = block_tokens<16>(nullptr, l, q);
            store_row_i16<16>(o.qtc + b * 256 + l * 16, q);
        }
        if (l < 12) o.mv[b * 12 + l] = (int16_t)(l == 0 ? dx : l == 1 ? dy : l == 2 ? rf : 0);
    }
    if (l == 0) {
        S.vsp[g] = (uint8_t)split;
        o.split[b] = (uint8_t)split;
        o.tokens[b] = tok;
        o.mae[b] = mae_num;
    }
}

// The inverse half of the VBS transform path, for slot k of the tile's blocks in split-sorted
// order (unsplit blocks first, then split ones, then none): the four blocks of a wave then
// take one of the two inverse paths -- a wave with both ran both (about two waves in three on
// the bench content, split ~50 %), now at most one wave per tile does.  Reads the levels
// tq16_vbs_fwd left -- an unsplit block's in its QTC rows (this workgroup's stores, before the
// barrier), a split one's packed in its scratch; dequantisation, IDCT, reconstruction and SSE.  `un`: the tile's transpose scratch (slot k's
// lanes use block g's part, un + g * kTqScratchVbs: the slot -> block map is a permutation).
template <class G, bool SC1, bool HALO = false>
SO_DEV void tq16_vbs_inv(PTileLds<G, true>& S, int k, int l, double* un, int bx0, int byt0, int nbx,
                         int by0, int by1, int W, int qp_rd, const int32_t* __restrict__ qp_row,
                         const int32_t* __restrict__ qp_map, const PFrameOut& o, const PHalo& hl = PHalo{}) {
    constexpr int SR = G::SR, TBX = G::TBX;
    // slot k -> block g: the k-th unsplit block, else the (k - #unsplit)-th split one
    uint32_t mns = 0, ms = 0;
#pragma unroll
    for (int i = 0; i < G::NBLK; ++i) {
        const uint32_t v = S.vsp[i];
        mns |= (v == 0 ? 1u : 0u) << i;
        ms |= (v == 1 ? 1u : 0u) << i;
    }
    const int nns = __builtin_popcount(mns);
    int kk = k < nns ? k : k - nns;
    uint32_t m = k < nns ? mns : ms;
    if (kk >= __builtin_popcount(m)) return;   // uniform over the 16 lanes: no block
#pragma unroll 1
    for (; kk > 0; --kk) m &= m - 1;           // drop the kk lowest set bits
    const int g = __builtin_ctz(m);
    const bool split = k >= nns;
    const int bxl = g % TBX, byl = g / TBX;
    const int gbx = bx0 + bxl, gby = byt0 + byl;
    const size_t b = (size_t)(gby - by0) * nbx + gbx;
    const int x = gbx * 16, y = gby * 16;
    const int qpr = qp_map ? qp_map[(size_t)gby * nbx + gbx] : (qp_row ? qp_row[gby] : qp_rd);
    SO_MARK(vbs_inv);
    double* const scratch = un + g * kTqScratchVbs;
    const uint32_t* crow = S.curt + (byl * 16 + l) * G::CPD + bxl * 4;
    const int j = l >> 2, r0 = l & 3;
    int sse = 0;
    if (!split) {
        const int dx = S.mer[g][0], dy = S.mer[g][1];
        const int prow = byl * 16 + SR + dy + l, pcol = bxl * 16 + SR + dx;   // window coordinates
        int q[16], dq[16];
        load_row_i16<16>(o.qtc + b * 256 + l * 16, q);
        dequant_row_int<16>(q, l, qpr, dq);
        double rd[16];
        xform2d_rows<16, true>(scratch, l, dq, rd, SO_TQ_TW());
        int rec[16];
        {
            uint32_t pw[4];
            win_row16<G::RP>(S.win, prow, pcol, pw);
#pragma unroll
            for (int c = 0; c < 16; ++c)
                rec[c] = (int)((pw[c >> 2] >> (8 * (c & 3))) & 255) + (int)__builtin_rint(rd[c]);
        }
        store_rec_row<SC1, HALO>(o, hl, W, x, y + l, rec, 16);
        if (o.sse) {
#pragma unroll
            for (int kq = 0; kq < 4; ++kq) {
                const uint32_t cw = crow[kq];
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int d = (int)((cw >> (8 * e)) & 255) - (rec[4 * kq + e] & 255);
                    sse += d * d;
                }
            }
        }
    } else {
        SO_MARK(vbs_inv_split);
        const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
        const MeRec& sm = S.mer[G::NBLK + 4 * g + j];
        const int sdx = sm[0], sdy = sm[1];
        const int sxl = bxl * 16 + (j & 1) * 8, syl = byl * 16 + (j >> 1) * 8;   // sub-block in the tile (px)
        int sdq[2][8];
        {   // the levels tq16_vbs_fwd left packed in the block's scratch (read before the transposes)
            const so_v4u* const d = reinterpret_cast<const so_v4u*>(reinterpret_cast<const uint32_t*>(scratch) + l * 8);
            const so_v4u v0 = d[0], v1 = d[1];
            wave_sync();
            const uint32_t pq[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                int qs[8];
                unpack_i16<8>(pq + 4 * h, qs);
                dequant_row_int<8>(qs, r0 + 4 * h, qpm1, sdq[h]);
            }
        }
        double srd[2][8];
        xform2d_sub<true>(scratch, l, sdq, srd, SO_TQ_TW8());
        const int xs = x + (j & 1) * 8, ys = y + (j >> 1) * 8;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int row = r0 + 4 * h;
            uint32_t pw[2];
            win_row8<G::RP>(S.win, syl + SR + sdy + row, sxl + SR + sdx, pw);
            int rec[8];
#pragma unroll
            for (int c = 0; c < 8; ++c)
                rec[c] = (int)((pw[c >> 2] >> (8 * (c & 3))) & 255) + (int)__builtin_rint(srd[h][c]);
            store_rec_row<SC1, HALO>(o, hl, W, xs, ys + row, rec, 8);
            if (o.sse) {
                const uint32_t* cr = S.curt + (syl + row) * G::CPD + (sxl >> 2);
#pragma unroll
                for (int kq = 0; kq < 2; ++kq) {
                    const uint32_t cw = cr[kq];
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const int d = (int)((cw >> (8 * e)) & 255) - (rec[4 * kq + e] & 255);
                        sse += d * d;
                    }
                }
            }
        }
    }
    SO_MARK(vbs_inv_end);
    if (o.sse) {
        sse = group_sum<16>(sse);
        if (l == 0) o.sse[b] = sse;
    }
}

// Search + transforms of tile `tile` of one frame.  SC1: the reconstruction rows are stored
// write-through (global_store sc1), so another XCD that later reads them (p_run_kernel's
// next frame) gets them from memory without a release fence.  Ends with every wave's
// stores retired (s_waitcnt vmcnt(0)) and a workgroup barrier.  `pre`: as sea2_tile's.
// write-through (sc1) stores: the value is in memory once the store retires
SO_DEV void store_sc1_i16(int16_t* p, int v) {
    asm volatile("global_store_short %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}
SO_DEV void store_sc1_i32(int32_t* p, int v) {
    asm volatile("global_store_dword %0, %1, off sc1" ::"v"(p), "v"(v) : "memory");
}

template <class G, bool SC1, class Pre = NoPre, bool HALO = false, bool TOK = false, bool VBS = false,
          class Post = NoPre, bool HALFTQ = false, bool ZSKIP = false, int LISTS = 0>
SO_DEV void ptile_body(PTileLds<G, VBS, HALFTQ>& S, int tile, const uint8_t* __restrict__ cur, const uint8_t* ref, int H, int W,
                       int by0, int by1, int qp_rd, const int32_t* __restrict__ qp_row,
                       const int32_t* __restrict__ qp_map, int32_t* __restrict__ out_best, const PFrameOut& o,
                       const Pre& pre = Pre(), const PHalo& hl = PHalo{}, double lam = 0.0,
                       const int* dense_flag = nullptr, int32_t* fb_out = nullptr, int count_ops = 0,
                       const Post& post = Post(), const int16_t* prev_mv = nullptr) {
    constexpr int SR = G::SR, TBX = G::TBX, TBY = G::TBY;
    using P = PTileGeo<G>;
    uint32_t* const b4w = reinterpret_cast<uint32_t*>(S.un);
    uint16_t* const list = reinterpret_cast<uint16_t*>(b4w + P::B4);
    // room for a dense tile's three shifted window copies in the scratch, 8 (mod 32) dwords on
    constexpr int kUnDw = 2 * (VBS ? PTileGeoVbs<G>::U64 : PTileGeo<G, HALFTQ>::U64);
    int dense4 = 0;
#ifndef SO_DENSE_ONE   // A/B builds: dense tiles read the single window copy
    if constexpr (3 * G::DCS + 32 <= kUnDw) {
        const int d = (int)((reinterpret_cast<uintptr_t>(b4w) - reinterpret_cast<uintptr_t>(S.win)) / 4);
        dense4 = d + ((8 - d) & 31);
    }
#endif
    const Sea2Lds L{S.win, b4w, S.curt, S.a4, list, S.lcount, S.keys, S.st, count_ops, dense4};
    RefSet refs{};
    refs.p[0] = ref;
#ifndef SO_PROF_PHASE   // phase-attribution A/B builds only (tools/prun_phase.py): 1 = no transforms
#define SO_PROF_PHASE 0  // (the tile's current rows stored as its reconstruction), 2 = no search
#endif                   // (window staged, every block at mv (0, 0))
    sea2_tile<G, Pre, VBS, LISTS>(L, tile, cur, refs, 1, H, W, by0, by1, SO_PROF_PHASE == 2 ? 5 : 0, pre,
                           dense_flag, prev_mv);   // ends with a barrier

    const int tid = opaque_tid();
    SO_SEA_STAMP(5, __builtin_amdgcn_s_memtime());
    const int nbx = W / 16;
    const int tiles_x = (nbx + TBX - 1) / TBX;
    const int bx0 = (tile % tiles_x) * TBX, byt0 = by0 + (tile / tiles_x) * TBY;
    for (int i = tid; i < PTileLds<G, VBS>::NU; i += G::NTHREADS) {
        SO_MARK(decode_keys);
        int32_t rec4[4];
        decode_key(S.keys[i], SR, rec4);
        S.mer[i].set(rec4);
        const int gbx = bx0 + i % TBX, gby = byt0 + i / TBX;
        if (out_best && i < G::NBLK && gbx < nbx && gby < by1) {
            int32_t* ob = out_best + ((size_t)(gby - by0) * nbx + gbx) * 4;
            ob[0] = S.mer[i][0]; ob[1] = S.mer[i][1]; ob[2] = S.mer[i][2]; ob[3] = S.mer[i][3];
        }
    }
    SO_MARK(keys_tail);
    // the tile's dense-block count (p_run_kernel: the next frame's same tile reads it), stored
    // write-through now so that the drain below covers it
    if (fb_out != nullptr && tid == 0) store_sc1_i32(fb_out, (int)S.st[0]);
    if (tid == 0) S.fwd_flags = 0u;
    __syncthreads();
    SO_SEA_STAMP(6, __builtin_amdgcn_s_memtime());
    constexpr bool kFwdMfma = !VBS && SO_FWD_MFMA && SO_PROF_PHASE != 1;
    if constexpr (kFwdMfma) {   // every wave: blocks w, w + NW on the matrix cores
        const int ln = tid & 63;
        float cs[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) cs[s] = dct16_f32(ln & 15, 4 * (ln >> 4) + s);
        for (int g = tid >> 6; g < G::NBLK; g += G::NW)
            fwd_mfma<G>(S, g, ln, cs, bx0, byt0, nbx, by1, qp_rd, qp_row, qp_map);
        __syncthreads();
#ifdef SO_FWD_COUNT   // A/B builds only: the flagged blocks replace the SAD count (words 66..67)
        if (tid == 0) S.st[2] = (uint32_t)__builtin_popcount(S.fwd_flags);
#endif
    }
    {   // block g = wave * TQ_BPW + (lane >> 4) on lanes [0, 16 * TQ_BPW) of waves 0..NBLK/TQ_BPW-1
        // (the even waves, or every wave with 2 blocks, measured slower: 4K 71.8 / 79.8 vs
        // 67.2 us per frame, 1088p 30.7 / 31.7 vs 28.7); after fwd_mfma, the flagged blocks first
        const int ln = tid & 63, w = tid >> 6;
        int gq = w * G::TQ_BPW + (ln >> 4);
        bool qs = false;
        if constexpr (kFwdMfma) {
            const uint32_t m = S.fwd_flags;
            if (m != 0u && gq < G::NBLK) gq = fwd_order<G::NBLK>(m, gq);
            qs = !((m >> gq) & 1u);
        }
        if (SO_PROF_PHASE == 1 && ln < 16 * G::TQ_BPW && gq < G::NBLK) {
            // no transforms: the current rows stand in for the reconstruction, so the next
            // frame searches realistic content
            const int bxl = gq % G::TBX, byl = gq / G::TBX, l = ln & 15;
            const int gbx = bx0 + bxl, gby = byt0 + byl;
            if (gbx < nbx && gby < by1) {
                const uint32_t* crow = S.curt + (byl * 16 + l) * G::CPD + bxl * 4;
                so_v4u v;
                for (int k = 0; k < 4; ++k) v[k] = crow[k];
                *reinterpret_cast<so_v4u*>(o.recon + (size_t)(gby * 16 + l) * W + gbx * 16) = v;
            }
        } else if (ln < 16 * G::TQ_BPW && gq < G::NBLK) {
            if constexpr (VBS)
                tq16_vbs_fwd<G, SC1, HALO>(S, gq, ln & 15, S.un + gq * kTqScratchVbs, bx0, byt0, nbx, by0, by1, W, qp_rd,
                                           qp_row, qp_map, lam, o);
            else
                tq16_exact<G, SC1, HALO, TOK, HALFTQ, ZSKIP>(S, gq, ln & 15, S.un + gq * (HALFTQ ? kTqScratchHalf : kTqScratch), bx0,
                                              byt0, nbx, by0, by1, W, qp_rd,
                                              qp_row, qp_map, o, hl, qs);
        }
    }
    if constexpr (VBS) {
        if (SO_PROF_PHASE != 1) {
            __syncthreads();   // every block's levels and split state in LDS
            const int ln = tid & 63, gq = (tid >> 6) * G::TQ_BPW + (ln >> 4);
            if (ln < 16 * G::TQ_BPW && gq < G::NBLK)
                tq16_vbs_inv<G, SC1, HALO>(S, gq, ln & 15, S.un, bx0, byt0, nbx, by0, by1, W, qp_rd,
                                           qp_row, qp_map, o, hl);
        }
    }
    SO_SEA_STAMP(7, __builtin_amdgcn_s_memtime());
    SO_MARK(post);
    post();   // p_run_kernel: the next task's dequeue, in flight with the drain below
    if constexpr (SC1) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every storing wave
    SO_SEA_STAMP(14, __builtin_amdgcn_s_memtime());
    __syncthreads();
}

// ---- two-pass rate control inside the persistent run (so_encode_p_run_2pass) ---------------
// The per-frame flow of encode() with RCFlag 3: pass 1 encodes the frame
// at the rate-control row QP, so_qp_map turns each block's pass-1 token count t against its
// block row's sum m (n blocks) into delta = [t n >= 2m] + [t n >= 4m] - [2 t n < m] -
// [4 t n < m], qp = clamp(row QP + delta + roi, lo, hi), and pass 2 re-runs the transforms
// with those QPs on pass 1's motion vectors.  In the run a tile is two tasks: pass 1 (search +
// forward transform + token count: the pass-1 QTC and reconstruction are never used) and
// pass 2 (the transforms at the block QPs, from the ME records pass 1 stored); a pass-2 task
// starts once every tile of its tile row finished pass 1 (the row sums).


// pass 1 of one block (16 lanes, l = row): residual from the LDS window / tile as tq16_exact,
// the forward transform, quantisation at the row QP and the token count.  Stores the ME
// record (mv / mae / split: final, pass 2 keeps them) and the pass-1 tokens to t1, write-
// through (pass-2 tasks on other CUs read them).
template <class G>
SO_DEV void tq16_pass1(PTileLds<G>& S, int g, int l, double* scratch, int bx0, int byt0, int nbx, int by1, int qp_rd,
                       const int32_t* __restrict__ qp_row, const PFrameOut& o, int32_t* __restrict__ t1) {
    constexpr int SR = G::SR, TBX = G::TBX;
    const int bxl = g % TBX, byl = g / TBX;
    const int gbx = bx0 + bxl, gby = byt0 + byl;
    if (gbx < nbx && gby < by1) {   // uniform over the block's 16 lanes
        const size_t b = (size_t)gby * nbx + gbx;
        const int qpr = qp_row ? qp_row[gby] : qp_rd;
        const int dx = S.mer[g][0], dy = S.mer[g][1], rf = S.mer[g][2], sad = S.mer[g][3];
        const int prow = byl * 16 + SR + dy + l, pcol = bxl * 16 + SR + dx;
        const uint32_t* crow = S.curt + (byl * 16 + l) * G::CPD + bxl * 4;
        int res[16];
        {
            uint32_t pw[4];
            win_row16<G::RP>(S.win, prow, pcol, pw);
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t cw = crow[k];
#pragma unroll
                for (int e = 0; e < 4; ++e)
                    res[4 * k + e] = (int)((cw >> (8 * e)) & 255) - (int)((pw[k] >> (8 * e)) & 255);
            }
            // the prediction row waits for pass 2 in the block's reconstruction rows (write-
            // through; pass 2 overwrites them with the reconstruction before the tile's done
            // flag, which every reader of the plane waits for): pass 2 then needs neither the
            // vector nor a load that depends on it
            const so_v4u pv{pw[0], pw[1], pw[2], pw[3]};
            uint8_t* const rp = o.recon + (size_t)(gby * 16 + l) * (nbx * 16) + gbx * 16;
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(rp), "v"(pv) : "memory");
        }
        double tcr[16];
        xform2d_rows<16, false>(scratch, l, res, tcr, SO_TQ_TW());
        // TC = np.round(DCT) as int32 (the 1.5 * 2^52 shift rounds half to even, as rint), the
        // pass-1 levels at the row QP by the exact integer round-half-even shift
        constexpr double kRne = 0x1.8p52;
        int tc[16], q[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) tc[c] = (int)(uint32_t)__builtin_bit_cast(uint64_t, tcr[c] + kRne);
        quant_row_int<16>(tc, l, qpr, q);
        const int tok = block_tokens<16>(nullptr, l, q);
        // the coefficients wait for pass 2 in the block's QTC rows (|TC| <= 4080: int16), stored
        // write-through like the ME records: pass 2 requantises them at the block's QP instead
        // of forming the residual and running the forward transform again (same MV, same
        // planes, so the same TC)
        {
            uint32_t w[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) w[k] = (uint32_t)(uint16_t)tc[2 * k] | ((uint32_t)tc[2 * k + 1] << 16);
            const so_v4u v0{w[0], w[1], w[2], w[3]}, v1{w[4], w[5], w[6], w[7]};
            int16_t* const qp_ = o.qtc + b * 256 + l * 16;
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(qp_), "v"(v0) : "memory");
            asm volatile("global_store_dwordx4 %0, %1, off offset:16 sc1" ::"v"(qp_), "v"(v1) : "memory");
        }
        if (l < 12) store_sc1_i16(o.mv + b * 12 + l, l == 0 ? dx : l == 1 ? dy : l == 2 ? rf : 0);
        if (l == 0) {
            o.split[b] = 0;
            o.mae[b] = sad;
            store_sc1_i32(t1 + b, tok);
        }
    }
}

// pass 2 of one block: the QP from the row's pass-1 statistics, then tq16_exact's transform
// path with the prediction / current rows read from the planes (this task staged no window)
// at pass 1's motion vector.  Stores QTC, tokens, reconstruction (write-through), SSE, QP.
// 16 bytes of a plane row from byte `p` (any alignment): five aligned dwords + v_alignbyte (at a
// valid candidate, x + dx + 16 < W, the last dword ends at most 3 bytes past the row)
SO_DEV void row16_any(const uint8_t* p, uint32_t (&w)[4]) {
    const uint32_t* pa = reinterpret_cast<const uint32_t*>((uintptr_t)p & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)((uintptr_t)p & 3);
    uint32_t q5[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) q5[k] = pa[k];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = __builtin_amdgcn_alignbyte(q5[k + 1], q5[k], sh);
}
SO_DEV void row16_aligned(const uint8_t* p, uint32_t (&w)[4]) {
    const so_v4u c4 = *reinterpret_cast<const so_v4u*>(p);
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = c4[k];
}

// pass 2 of one block: the QP from the row's pass-1 statistics, then tq16_exact's transform
// path with the prediction / current rows read from the planes (this task staged no window)
// at pass 1's motion vector -- read again (L1 / L2) after the transforms instead of being
// held across them.  Stores QTC, tokens, reconstruction (write-through), SSE, QP.
template <class G>
SO_DEV void tq16_pass2(PTileLds<G>& S, int g, int l, double* scratch, int bx0, int byt0, int nbx, int by1, int W,
                       int qp_rd, const int32_t* __restrict__ qp_row, const int32_t* __restrict__ roi, int qp_lo,
                       int qp_hi, const uint8_t* __restrict__ cur, const uint8_t* /*ref*/, const PFrameOut& o,
                       const int32_t* __restrict__ t1, uint8_t* push = nullptr) {
    constexpr int TBX = G::TBX;
    const int bxl = g % TBX, byl = g / TBX;
    const int gbx = bx0 + bxl, gby = byt0 + byl;
    if (gbx < nbx && gby < by1) {
        const size_t b = (size_t)gby * nbx + gbx;
        const int x = gbx * 16, y = gby * 16;
        // No address here derives from another task's output: pass 1 left the prediction rows
        // in the block's reconstruction rows and the coefficients in its QTC rows.  (Round 5
        // read pass 1's motion vector and loaded the prediction at it: after a timed-out wait,
        // when the run's later waits return at once (SO_RUN_ABORT_CHECK), a pass-2 unit could
        // run before its row's pass 1 and address ~125 MB past the plane with an unwritten
        // record -- the frame pipeline's hipErrorIllegalAddress)
        int qpr;
        {   // qp_map_kernel (so_capi.hip), per block
            const long long tn = (long long)t1[b] * nbx, m = S.msum[byl];
            const int d = (tn >= 2 * m) + (tn >= 4 * m) - (2 * tn < m) - (4 * tn < m);
            qpr = (qp_row ? qp_row[gby] : qp_rd) + d + (roi ? roi[b] : 0);
            qpr = qpr < qp_lo ? qp_lo : (qpr > qp_hi ? qp_hi : qpr);
        }
        const uint8_t* crow = cur + (size_t)(y + l) * W + x;
        const uint8_t* prow = o.recon + (size_t)(y + l) * W + x;   // pass 1's prediction row
        constexpr double kRne = 0x1.8p52;
        // the coefficients pass 1 left in the QTC rows (after the wait's acquire), requantised
        // at the block's QP: q = np.round(TC / 2^k), the exact integer round-half-even shift
        int tc[16], q[16];
        load_row_i16<16>(o.qtc + b * 256 + l * 16, tc);
        quant_row_int<16>(tc, l, qpr, q);
        const int tok = block_tokens<16>(nullptr, l, q);
        store_row_i16<16>(o.qtc + b * 256 + l * 16, q);
        int dq[16];
        double rd[16];
        dequant_row_int<16>(q, l, qpr, dq);
        xform2d_rows<16, true>(scratch, l, dq, rd, SO_TQ_TW());
        int rec[16];
        {
            uint32_t pw[4];
            row16_aligned(prow, pw);
#pragma unroll
            for (int c = 0; c < 16; ++c)
                rec[c] = (int)((pw[c >> 2] >> (8 * (c & 3))) & 255) +
                         (int)(uint32_t)__builtin_bit_cast(uint64_t, rd[c] + kRne);
        }
        so_v4u v;
#pragma unroll
        for (int k = 0; k < 4; ++k)
            v[k] = (uint32_t)(rec[4 * k] & 255) | ((uint32_t)(rec[4 * k + 1] & 255) << 8) |
                   ((uint32_t)(rec[4 * k + 2] & 255) << 16) | ((uint32_t)(rec[4 * k + 3] & 255) << 24);
        uint8_t* rp = o.recon + (size_t)(y + l) * W + x;
        asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(rp), "v"(v) : "memory");
        if (push) {   // frame pipeline: the next rank's landing plane (system scope, over xGMI)
            uint8_t* q = push + (size_t)(y + l) * W + x;
            asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q), "v"(v) : "memory");
        }
        int sse = 0;
        if (o.sse) {
            uint32_t cw[4];
            row16_aligned(crow, cw);
#pragma unroll
            for (int k = 0; k < 4; ++k)
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    const int dd = (int)((cw[k] >> (8 * e)) & 255) - (rec[4 * k + e] & 255);
                    sse += dd * dd;
                }
            sse = group_sum<16>(sse);
        }
        if (l == 0) {
            o.tokens[b] = tok;
            if (o.sse) o.sse[b] = sse;
            if (o.qpmap) o.qpmap[b] = qpr;
        }
    }
}

#ifndef SO_PTILE_NW
#define SO_PTILE_NW 8
#endif
template <int NW, bool TOK = false>
__global__ void __launch_bounds__(NW * 64) __attribute__((amdgpu_waves_per_eu(
    NW >= 16 ? SO_PTILE_WPE16 : (TOK && SO_PTILE_TOK_HALF ? 8 : SO_SEA2_WPE))))
p_tile_kernel(const uint8_t* __restrict__ cur, RefSet refs, int H, int W, int by0, int by1, int qp_rd,
              const int32_t* __restrict__ qp_row, const int32_t* __restrict__ qp_map, int32_t* __restrict__ out_best,
              PFrameOut o, const int16_t* prev_mv) {
    using G = Sea2GeoT<NW>;
    __shared__ PTileLds<G, false, TOK && SO_PTILE_TOK_HALF> S;
    SO_STAMP_REC_SET(g_sea_stamps ? g_sea_stamps + (size_t)blockIdx.x * 12 : nullptr);
    ptile_body<G, false, NoPre, false, TOK>(S, blockIdx.x, cur, refs.p[0], H, W, by0, by1, qp_rd, qp_row, qp_map,
                                            out_best, o, NoPre(), PHalo{}, 0.0, nullptr, nullptr, 0, NoPre(), prev_mv);
#ifdef SO_STAMPS
    const int tid = threadIdx.x;
    if (tid == 0) {   // tools/sea_stamps.py (STAMP_FUSED=1): epilogue = records + transforms
        uint32_t hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        SO_SEA_STAMP(6, __builtin_amdgcn_s_memtime());
        SO_SEA_STAMP(7, __builtin_amdgcn_s_memrealtime());
        SO_SEA_STAMP(8, ((unsigned long long)xcc << 32) | hw);
        SO_SEA_STAMP(9, ((unsigned long long)S.st[0] << 32) | S.st[1]);
    }
#endif
}

// prev_mv (may be null): the previous frame's motion records, the search's U hint (sea2_tile)
int p_tile_launch(const uint8_t* cur, const RefSet& refs, int H, int W, int by0, int by1, int qp_rd,
                  const int32_t* qp_row, const int32_t* qp_map, int32_t* out_best, uint8_t* out_split,
                  int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae, uint8_t* out_recon,
                  int32_t* out_sse, hipStream_t st, bool tokens_only, const int16_t* prev_mv) {
    const int nbx = W / 16, nrows = by1 - by0;
    if (nrows <= 0) return SO_OK;
    const dim3 grid(((nbx + Sea2Geo::TBX - 1) / Sea2Geo::TBX) * ((nrows + Sea2Geo::TBY - 1) / Sea2Geo::TBY));
    const PFrameOut o{out_split, out_mv, out_qtc, out_tokens, out_mae, out_recon, out_sse, nullptr};
    if (tokens_only)
        hipLaunchKernelGGL((p_tile_kernel<SO_PTILE_NW, true>), grid, dim3(SO_PTILE_NW * 64), 0, st, cur, refs, H, W,
                           by0, by1, qp_rd, qp_row, qp_map, out_best, o, prev_mv);
    else
        hipLaunchKernelGGL((p_tile_kernel<SO_PTILE_NW, false>), grid, dim3(SO_PTILE_NW * 64), 0, st, cur, refs, H, W,
                           by0, by1, qp_rd, qp_row, qp_map, out_best, o, prev_mv);
    return check_launch("p_tile_kernel");
}

// ---- persistent run of P-frames ------------------------------------------------------------
// Frame i of a launch predicts from ref[i]; dep[i] = j >= 0 when that plane is frame j's
// reconstruction in the same launch (its tiles are waited for), -1 when it is complete before
// the launch (stream order).  One run: dep[i] = i - 1.  Several independent runs interleaved
// (so_encode_p_runs: other GOPs' P-frames) keep more tiles in flight than one frame offers.
// The stripe / frame-pipeline modes use i - 1 (and their own reference planes).
struct PRunArgs {
    const uint8_t* cur[kRunMax];
    const uint8_t* ref[kRunMax];
    int dep[kRunMax];
    PFrameOut out[kRunMax];
};

// Workspace words: [0] task counter, [1] exit counter, [2] epoch of the last finished launch,
// [32] timeout count, [64 + f * ntiles + t] = the launch's epoch once tile t of frame f is
// done.  The caller zeroes the workspace once; a launch runs with epoch [2] + 1 and its last
// workgroup resets [0], [1] and stores the epoch in [2], so no launch needs a memset.  [32] is
// the CALLER's: it accumulates over launches and calls until the caller reads and clears it
// (Engine.check_run), so a timeout in any launch of a GOP is seen.
#ifndef SO_RUN_ACQUIRE
#define SO_RUN_ACQUIRE 1
#endif
#ifndef SO_RUN_ABORT_CHECK
#define SO_RUN_ABORT_CHECK 1
#endif
#ifndef SO_RUN_TIMEOUT_WORD
#define SO_RUN_TIMEOUT_WORD 32
#endif
#ifndef SO_RUN_DONE_BASE
#define SO_RUN_DONE_BASE 128
#endif
// the task counter (hammered by every workgroup's dequeue), the timeout count, the fallback and
// SAD counts, the wait diagnostic record and the done flags live on separate 128-byte lines
constexpr int kRunTimeoutWord = SO_RUN_TIMEOUT_WORD, kRunDoneBase = SO_RUN_DONE_BASE;
// [1], [2] on the task counter's line: touched once per workgroup.  [64] (a line of its own):
// blocks whose SEA search took the dense fallback, summed over launches until the caller clears
// it (SO_P_RUN_FALLBACK_WORD); each workgroup adds its total once, on its way out.  (Adding per
// tile on the timeout word's line, which every waiting workgroup reads, cost +17 % per frame.)
// [66..67] (same line, 64-bit): the search's executed SAD byte operations, added the same way.
constexpr int kRunExitWord = 1, kRunEpochWord = 2, kRunFallbackWord = 64, kRunSadOpsWord = SO_P_RUN_SAD_OPS_WORD;
// The waits' health words on the timeout word's line (written only when something unusual
// happened, so the per-tile read of the timeout word stays a clean hit):
//   [33] waits whose relaxed polls kept missing a flag that an atomic read then found set
//        (evidence of a stale copy; the wait itself goes on with atomic reads and completes);
//   [34] poll intervals of >= 1 ms (the wave was descheduled: queue preemption / CWSR), which
//        do not count towards the wait's bound;
//   [35] the diagnostic record's claim counter.
// [96..127]: the record of the first wait that timed out (SO_P_RUN_DIAG_WORD, layout in
// include/streamoptima.h; Engine.check_run prints it).
constexpr int kRunStaleWord = SO_P_RUN_STALE_WORD, kRunGapWord = SO_P_RUN_GAP_WORD, kRunClaimWord = 35;
constexpr int kRunDiagWord = SO_P_RUN_DIAG_WORD;
static_assert(kRunDoneBase >= kRunDiagWord + 32, "the diagnostic record precedes the done flags");
// kRunFPipe2P: the frame pipeline with two-pass RC (each tile a pass-1 and a pass-2 task as
// kRunTwoPass; the reference arrives in the landing planes as kRunFPipe, and pass 2 pushes
// the final reconstruction on to the rank encoding the next frame)
constexpr int kRunSingle = 0, kRunStripe = 1, kRunFPipe = 2, kRunTwoPass = 3, kRunFPipe2P = 4;
// SO_RUN_PROFILE builds (tools/rc2p_ab.py): per-phase shader cycles >> 10 accumulated by wave 0
// into workspace words 48.. (48 pass-1 task, 49 pass-2 task, 50 pass-2 row wait, 51 reference
// wait); A/B diagnostics only
#ifdef SO_RUN_PROFILE
#define SO_RUN_PROF(word, cyc) \
    do { if (wave == 0) __hip_atomic_fetch_add(&ws[(word)], lane == 0 ? (uint32_t)((cyc) >> 10) : 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); } while (0)
#else
#define SO_RUN_PROF(word, cyc) do { } while (0)
#endif

// ---- dependency waits ---------------------------------------------------------------------------
// What a wave polls for: lane l waits on *c (when need) until it reads `want` (agent-scope
// flags of this GPU) or `sys_want` (sysl: another rank's flags, system scope).
struct RunWait {
    int task, f, dep, tile, mode;
    uint32_t want, sys_want;
    unsigned long long limit;   // polling time bound, 100 MHz s_memrealtime ticks
};
constexpr unsigned long long kRunGapTicks = 100000ull;        // 1 ms: a descheduled wave
constexpr unsigned long long kRunEscalateTicks = 100000ull;   // 1 ms of polling: atomic reads

SO_DEV uint32_t rmw_read(const uint32_t* c) {
    return __hip_atomic_fetch_add(const_cast<uint32_t*>(c), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Called by every lane of ONE wave (wave-uniform control flow throughout: a lane-0 branch
// around a loop with a barrier after it gets structurised into a hang, see p_run_kernel).
// Relaxed polls with s_sleep; the elapsed time counts only poll-to-poll intervals shorter than
// 1 ms, so a wave that was descheduled (queue preemption) is not mistaken for a lost flag;
// after 1 ms of polling the awaited local flags are read with atomic RMWs instead (these cannot
// be served from a stale cached copy; a first RMW that finds a flag the loads kept missing is
// counted in ws[kRunStaleWord]).  Past `limit` the wave counts a timeout and, if it is the
// first, writes the diagnostic record (ws[kRunDiagWord..+31]) and keeps reading the awaited
// flags for up to 50 ms more to record when they arrive.  Returns the lane's last raw value.
// (Durations in 32 bits of 100 MHz ticks: the wait state is a handful of SGPRs.)
SO_DEV uint32_t run_poll(const uint32_t* c, bool need, bool sysl, uint32_t* ws, const RunWait& w) {
    const int lane = threadIdx.x & 63;
    const uint32_t one = lane == 0 ? 1u : 0u;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    uint32_t last = 0, susp = 0, raw = 0;   // ticks since t0 at the last poll; descheduled ticks
    bool esc = false, first = true;
    for (;;) {
        if (sysl)
            raw = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        else if (esc && need)
            raw = rmw_read(c);
        else
            raw = __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const bool ok = raw == (sysl ? w.sys_want : w.want);
        SO_MARK(poll_iter);
        if (__builtin_amdgcn_ballot_w64(need && !ok) == 0) break;
#if SO_RUN_ABORT_CHECK
        // the timeout count, read once per wait and only when it has to wait: after one timeout
        // the later waits of the run return at once (the run is already flagged wrong), so a
        // lost flag cannot stall the launch for 50 ms per remaining tile.  (Read ahead of every
        // first poll it put a memory round trip on every tile's path; polled in the loop it put
        // every waiting workgroup on one word: +70 % per frame.)
        if (first) {
            first = false;
            if (__builtin_amdgcn_readfirstlane(__hip_atomic_load(ws + kRunTimeoutWord, __ATOMIC_RELAXED,
                                                                 __HIP_MEMORY_SCOPE_AGENT)) != 0u)
                break;
        }
#endif
        __builtin_amdgcn_s_sleep(1);
        const uint32_t now = (uint32_t)(__builtin_amdgcn_s_memrealtime() - t0), gap = now - last;
        last = now;
        if (gap >= (uint32_t)kRunGapTicks) {
            susp += gap;
            __hip_atomic_fetch_add(&ws[kRunGapWord], one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        const uint32_t active = now - susp;
        if (!esc && active > (uint32_t)kRunEscalateTicks) {
            esc = true;
            // a stale copy, not a late arrival: the RMW (served by L2) finds the flag set AND a
            // relaxed load issued after it still misses it.  Comparing the RMW with `raw`, the
            // load from before the s_sleep, counted a flag set inside that window as stale
            // (ADVICE r05); flags only grow (launch epochs), so a coherent load after the RMW
            // must see at least what the RMW saw.
            const uint32_t v2 = (need && !sysl) ? rmw_read(c) : raw;
            const uint32_t v3 = (need && !sysl) ? __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : raw;
            if (__builtin_amdgcn_ballot_w64(need && !sysl && !ok && v2 == w.want && v3 != w.want) != 0)
                __hip_atomic_fetch_add(&ws[kRunStaleWord], one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        if (active > (uint32_t)w.limit) {
            __hip_atomic_fetch_add(&ws[kRunTimeoutWord], one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const uint32_t claim = __builtin_amdgcn_readfirstlane(
                __hip_atomic_fetch_add(&ws[kRunClaimWord], one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
            if (claim == 0u) {   // uniform: the first timed-out wait of the workspace records itself
                const uint32_t rv = (need && !sysl) ? rmw_read(c) : raw;
                const uint64_t bneed = __builtin_amdgcn_ballot_w64(need);
                const uint64_t bsys = __builtin_amdgcn_ballot_w64(need && sysl);
                const uint64_t brmw = __builtin_amdgcn_ballot_w64(need && !sysl && rv == w.want);
                const uint32_t other = (uint32_t)__builtin_amdgcn_ds_bpermute(((lane - 20) & 63) << 2, (int)raw);
                uint32_t hw, xcc;
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
                asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
                // words 1..19 from lane 0 (a per-lane select chain here had its 19 lane masks
                // hoisted out of the persistent loop into spilled SGPRs), words 20..31: the flags
                if (lane >= 20 && lane < 32)
                    __hip_atomic_store(&ws[kRunDiagWord + lane], other, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lane == 0) {
                    const uint32_t rec[19] = {(uint32_t)w.task, (uint32_t)w.f, (uint32_t)w.dep, (uint32_t)w.tile, w.want,
                                              w.sys_want, (uint32_t)w.mode | (esc ? 1u << 12 : 0u), (uint32_t)bneed,
                                              (uint32_t)bsys, active, now, susp, 0u, 0xFFFFFFFFu, hw, xcc,
                                              (uint32_t)blockIdx.x, (uint32_t)gridDim.x, (uint32_t)brmw};
#pragma unroll
                    for (int i = 0; i < 19; ++i)
                        __hip_atomic_store(&ws[kRunDiagWord + 1 + i], rec[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                }
                // keep reading the awaited flags (atomically) for up to 50 ms: when -- whether --
                // they arrive tells a slow holder from a lost or unseen flag
                const unsigned long long ta = __builtin_amdgcn_s_memrealtime();
                uint32_t arrive = 0xFFFFFFFFu;
                for (;;) {
                    const uint32_t x = sysl ? __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)
                                            : (need ? rmw_read(c) : 0u);
                    const uint32_t el = (uint32_t)(__builtin_amdgcn_s_memrealtime() - ta);
                    if (__builtin_amdgcn_ballot_w64(need && x != (sysl ? w.sys_want : w.want)) == 0) {
                        arrive = el;
                        break;
                    }
                    if (el > 5000000u) break;
                    __builtin_amdgcn_s_sleep(8);
                }
                if (lane == 14)
                    __hip_atomic_store(&ws[kRunDiagWord + 14], arrive, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (lane == 0)
                    __hip_atomic_store(&ws[kRunDiagWord], SO_P_RUN_DIAG_MAGIC, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
        }
    }
    return raw;
}


// The run's task dequeue, called by a whole wave: ONE returning atomic add of 1 to ws[0] (exec =
// lane 0 inside the asm), then s_waitcnt vmcnt(0), which also drains the wave's earlier stores.
// Returns the task index in lane 0.  (Written as `fetch_add(ws, lane == 0 ? 1 : 0)` by every
// lane, the compiler's atomic optimizer turned it into a 64-iteration readlane / writelane scan
// over the lanes before the atomic, and waited on the result right after it; a `lane == 0`
// branch ahead of the loop's barrier was structurised into a hang, tools/ubench_rowdeps.cpp.)
SO_DEV uint32_t run_dequeue(uint32_t* ws) {
    uint32_t r;
    uint64_t sv;
    asm volatile(
        "s_mov_b64 %1, exec\n\t"
        "s_mov_b64 exec, 1\n\t"
        "global_atomic_add %0, %2, %3, off sc0\n\t"
        "s_waitcnt vmcnt(0)\n\t"
        "s_mov_b64 exec, %1"
        : "=&v"(r), "=&s"(sv)
        : "v"(ws), "v"(1u)
        : "memory");
    return r;
}

// VBS: VBSEnable (the block + sub-block SEA and the RD split, tq16_vbs_fwd / _inv; 80 VGPRs, 6 waves per SIMD)
// HOOKS: the measurement / test hooks -- the searches' SAD byte-operation count
// (SO_OPT_COUNT_SAD_OPS) and the deliberately lost done flag (SO_OPT_TEST_LOSE_FLAG).  Only
// kRunSingle has a HOOKS instantiation, launched only while one of those options is set, so the
// timed kernels carry neither (count_ops folds to the constant 0 and its atomics are dead code).
// UQP (VBS runs without a row-QP schedule): every block at the RD QP, known at compile time --
// the block coefficients tq16_vbs_fwd would hold through the sub-block transforms for a
// requantisation at another QP are then dead (VBS run spills 30 -> 23; 4K VBS GOP 3.311 ->
// 3.265 ms, profiles/r06/ab_vbs_uqp.log).
// ZSKIP (one-GPU plain run, SO_OPT_RUN_ZERO_SKIP): tq16_exact's all-zero-wave IDCT skip.  On the
// one-GPU uniform-QP VBS run the same slot selects the latency-bound twin: its VBS survivor lists
// built one ballot per candidate row (sea2_tile's LISTS = 2; the host launches it when the grid
// has more slots than a frame has tiles), the other one building them from lane masks (LISTS = 1)
template <int NW, int MODE, bool VBS = false, bool HOOKS = false, bool UQP = false, bool ZSKIP = false>
__global__ void __launch_bounds__(NW * 64)
__attribute__((amdgpu_waves_per_eu(VBS ? SO_VBS_WPE : (NW >= 16 ? SO_PTILE_WPE16 : SO_SEA2_WPE))))
p_run_kernel(const PRunArgs a, int nframes, const uint8_t* __restrict__ ref0, int H, int W,
             int qp_rd, const int32_t* __restrict__ qp_row_arg, uint32_t* __restrict__ ws, int ws_stamp_base,
             const PRunStripe sp, double lam) {
    static_assert(!UQP || VBS, "the uniform-QP instantiation is the VBS run's");
    static_assert(!ZSKIP || (MODE == kRunSingle && !HOOKS && (!VBS || UQP)),
                  "the zero-skip / latency-lists instantiation is the one-GPU run's");
    constexpr int LISTS = VBS && MODE == kRunSingle && UQP ? (ZSKIP ? 2 : 1) : 0;
    const int32_t* __restrict__ const qp_row = UQP ? nullptr : qp_row_arg;
    using G = Sea2GeoT<NW>;
    __shared__ PTileLds<G, VBS> S;
    __shared__ int s_task;
    __shared__ int s_dense;   // kRunSingle: this tile searches dense (sea2_tile's dense_flag)
    const int tid = threadIdx.x;
    const int nbx = W / 16;
    constexpr bool STRIPE = MODE == kRunStripe, FPIPE = MODE == kRunFPipe || MODE == kRunFPipe2P;
    constexpr bool TWOP = MODE == kRunTwoPass || MODE == kRunFPipe2P;
    static_assert(!(VBS && (TWOP || MODE == kRunStripe)), "VBS runs: one GPU and the frame pipeline");
    static_assert(!HOOKS || MODE == kRunSingle, "test hooks: the one-GPU run only");
    const int count_ops = HOOKS ? sp.count_ops : 0;   // a compile-time 0 without HOOKS
    const int by0 = STRIPE ? sp.by0 : 0, by1 = STRIPE ? sp.by1 : H / 16;
    const int tiles_x = (nbx + G::TBX - 1) / G::TBX, ntr = (by1 - by0 + G::TBY - 1) / G::TBY;
    const int ntiles = tiles_x * ntr;
    // two-pass: 2 tasks per tile; per frame the pass-1 tasks of tile row r + 1 are queued ahead
    // of the pass-2 tasks of row r (which wait for all of row r's pass 1), so every wait is
    // on tasks earlier in the queue
    // kRunTwoPass (one GPU): each task runs a pass-2 unit, then a pass-1 unit (MERGE2P, below):
    // nframes * ntiles units of each, the pass-2 units lag2 = ntiles - (tiles_x + 1) tasks behind
    constexpr bool MERGE2P = MODE == kRunTwoPass;
    const int lag2 = ntiles - (tiles_x + 1);
    const int per_frame = TWOP && !MERGE2P ? 2 * ntiles : ntiles;
    const int ntasks = per_frame * nframes + (MERGE2P ? lag2 : 0);
    uint32_t* const done = ws + kRunDoneBase;
    // kRunSingle: per (frame, tile) the count of blocks that searched dense (after the done
    // flags, the pass-1 flags and token counts: p_run_workspace_words)
    uint32_t* const tilefb = ws + kRunDoneBase + 2 * (size_t)kRunMax * ntiles + (size_t)kRunMax * nbx * (H / 16);
    // Every queue / flag access is made by ALL lanes of wave 0 under a wave-uniform branch
    // (lane 0 adds 1, the others 0): a `tid == 0` branch ahead of a barrier inside this loop
    // gets structurised into a divergent inner loop that never re-runs the dequeue (a hang;
    // tools/ubench_rowdeps.cpp).
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const uint32_t one = lane == 0 ? 1u : 0u;
    __shared__ uint32_t s_fbsum;   // this workgroup's dense-searched blocks over its tasks (LDS: a
    __shared__ unsigned long long s_ops;   // register kept live across the loop cost spills)
    if (tid == 0) {                        // and its SAD byte operations
        s_fbsum = 0;
        s_ops = 0;
    }
#ifdef SO_MARKS_COUNT
    if (tid < 64) s_mark_cnt[tid] = 0u;   // visible after the loop's first barrier
#endif
    // this launch's epoch: ws[2] + 1 (ws[2] = the last finished launch's; written by that
    // launch's last workgroup, so every workgroup here reads it before it can change).  Done
    // flags hold the epoch of the launch that set them: nothing is zeroed between launches.
    const uint32_t ep0 = __builtin_amdgcn_readfirstlane(
        __hip_atomic_load(&ws[kRunEpochWord], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) + 1u;
#ifndef SO_EP_REG
    // inside the loop the epoch is re-read from LDS where it is used: a register held across
    // the persistent loop was spilled to scratch and reloaded per task on wave 0's path
    __shared__ uint32_t s_ep;
    if (tid == 0) s_ep = ep0;   // visible after the dequeue barrier below
#define ep ((uint32_t)__builtin_amdgcn_readfirstlane(*(lds_vu32p)&s_ep))
#else
    const uint32_t ep = ep0;
#endif
    // The plain run dequeues its next task at the end of the current one (ptile_body's `post`,
    // before the drain of the tile's stores), so the atomic's round trip overlaps the drain
    // instead of following the done flag.  Still deadlock-free: a workgroup holds at most one
    // not-yet-started task, and the lowest unfinished task is either running or held by a
    // workgroup whose current task (dequeued before it) has finished.
    uint32_t nxt_v = 0;       // wave 0: the atomic's result (VGPR; read at the loop top)
    bool nxt_taken = false;   // uniform
    for (;;) {
        SO_MARK(loop_top);
        if (wave == 0) {
            if (!nxt_taken) nxt_v = run_dequeue(ws);
            s_task = (int)__builtin_amdgcn_readfirstlane(nxt_v);
            s_dense = 0;
        }
        nxt_taken = false;
        __syncthreads();
        const int task = __builtin_amdgcn_readfirstlane(s_task);
        if (task >= ntasks) break;   // uniform: every wave leaves
#ifdef SO_STAMPS
        unsigned long long* const rec = g_run_stamps ? g_run_stamps + (size_t)(ws_stamp_base + task) * 16 : nullptr;
        SO_STAMP_REC_SET(rec);
        if (tid == 0 && rec) rec[8] = __builtin_amdgcn_s_memrealtime();
#endif
        // MERGE2P: the task's pass-1 unit (frame-major (f, tile); none in the trailing lag2 tasks,
        // which then name their pass-2 unit here) and its pass-2 unit u2 (none while < 0)
        const int u2 = MERGE2P ? task - lag2 : -1;
        const bool has1 = !MERGE2P || task < nframes * ntiles;
        const int u = has1 ? task : u2;
        const int f = u / per_frame;
        int tile = u - f * per_frame, pass = has1 ? 1 : 2;
        if constexpr (TWOP && !MERGE2P) {
            // [P1 rows 0..L-1] [P1 row L][P2 row 0] [P1 row L+1][P2 row 1] ... [P2 rows ntr-L..]:
            // a pass-2 task is queued L tile rows after its row's pass 1 (L = sp.p2lag, about
            // one grid's worth of tasks), so it rarely waits holding its slot
            const int L = sp.p2lag, k = tile, k1 = k - L * tiles_x, nb2 = (ntr - L) * 2 * tiles_x;
            if (k1 < 0) {
                tile = k;
            } else if (k1 < nb2) {
                const int j = k1 / (2 * tiles_x), rem = k1 - j * 2 * tiles_x;
                if (rem < tiles_x) {
                    tile = (j + L) * tiles_x + rem;
                } else {
                    pass = 2;
                    tile = j * tiles_x + rem - tiles_x;
                }
            } else {
                pass = 2;
                tile = (ntr - L) * tiles_x + (k1 - nb2);
            }
        }
        const int ty = tile / tiles_x, tx = tile - ty * tiles_x;
        const bool first_row = ty == 0, last_row = ty == ntr - 1;
        // in-launch reference frame, or -1
        const int dep = (MODE == kRunSingle || MODE == kRunTwoPass) ? a.dep[f] : f - 1;
        // the 3x3 tiles of frame f-1 around this one (the window's +-16 px), one flag per lane,
        // all polled in one round trip by wave 0 once the current tile is staged (ptile_body's
        // `pre`; the barrier after it releases the other waves).  Stripe: lanes 9-11 (12-14)
        // poll the up (down) neighbour's hand-off flags of the frame before.  Every task they
        // stand for was dequeued before this one by a running workgroup (here or on the
        // neighbour), so the wait always ends; it is bounded all the same (50 ms of
        // s_memrealtime): a timeout flags the run (Engine.check_run raises) and the tile proceeds.
        const auto wait_ref = [&]() {
            if (wave != 0) return;
            const int gprev = (STRIPE ? sp.gbase : 0) + f - 1;   // global index of the reference frame
            const bool remote = STRIPE && (first_row ? sp.my_up_flags != nullptr : false);
            const bool remote_dn = STRIPE && (last_row ? sp.my_dn_flags != nullptr : false);
            if (!FPIPE && dep < 0 && !remote && !remote_dn) return;
            SO_MARK(wait_w0);
#ifdef SO_STAMPS
            if (lane == 0 && rec) rec[9] = __builtin_amdgcn_s_memrealtime();
#endif
            const int lane = opaque_tid() & 63;   // recomputed per task (hoisted, it was spilled)
            const int nx = tx + lane % 3 - 1, ny = ty + lane / 3 - 1;
            const bool need = (FPIPE || dep >= 0) && lane < 9 && nx >= 0 && nx < tiles_x && ny >= 0 && ny < ntr;
            const uint32_t* c = done + (size_t)(dep > 0 ? dep : 0) * ntiles + (need ? ny * tiles_x + nx : 0);
            bool rneed = false;
            if constexpr (FPIPE) {   // the previous frame's tiles arrive from the previous rank
                c = sp.my_dn_flags + (size_t)(sp.gbase + f) * ntiles + (need ? ny * tiles_x + nx : 0);
                rneed = need;
            }
            if constexpr (STRIPE) {
                const int rx = tx + (lane - 9) % 3 - 1;
                if (lane >= 9 && lane < 12 && remote && rx >= 0 && rx < tiles_x) {
                    c = sp.my_up_flags + (size_t)gprev * tiles_x + rx;
                    rneed = true;
                } else if (lane >= 12 && lane < 15 && remote_dn && rx >= 0 && rx < tiles_x) {
                    c = sp.my_dn_flags + (size_t)gprev * tiles_x + rx;
                    rneed = true;
                }
            }
            // 50 ms of polling within one GPU; 2 s where the flags come from another rank, whose
            // host may enqueue its launch late (a rank's kernel can start waiting on a neighbour
            // whose process is descheduled, e.g. several ranks time-sharing one GPU)
            constexpr unsigned long long kWaitLimit = (STRIPE || FPIPE) ? 200000000ull : 5000000ull;
            // one GPU: lane 9 reads, in the same round trips, the dense-block count of the same tile
            // of the reference frame (a heuristic only -- dense and SEA searches are both exact --
            // so it is read unordered with the flags)
            const bool fbl = MODE == kRunSingle && lane == 9 && dep >= 0;
            if (fbl) c = tilefb + (size_t)dep * ntiles + tile;
#ifdef SO_RUN_PROFILE
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
#endif
            const RunWait rw{task, f, dep, tile, MODE | (VBS ? 16 : 0) | (pass << 8), ep, sp.epoch, kWaitLimit};
            const uint32_t raw = run_poll(c, need || rneed, (STRIPE || FPIPE) && rneed, ws, rw);
            SO_RUN_PROF(51, (__builtin_amdgcn_s_memrealtime() - t0) * 25);   // 100 MHz ticks -> ~2.5 GHz cycles
#ifdef SO_STAMPS
            if (lane == 0 && rec) rec[10] = __builtin_amdgcn_s_memrealtime();
#endif
#if SO_RUN_ACQUIRE
            // consumer side of the hand-off (MI355X_MICROARCH.md, "Valid forms"): one relaxed
            // poll, ONE agent-scope acquire (invalidates this CU's L1), its completion awaited
            // before the barrier that releases the other waves to the window loads.  (A
            // stripe's planes are uncached: the neighbour's rows come from memory either way.)
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
            // the same tile of the reference frame had most of its blocks overflow the SEA bound
            // -> this one searches dense from the start, except every SO_DENSE_PROBE-th frame,
            // which probes the bound again
            if (MODE == kRunSingle && dep >= 0 && (f & (SO_DENSE_PROBE - 1)) != 0) {
                const uint32_t fb = (uint32_t)__builtin_amdgcn_readlane((int)raw, 9);
                if (lane == 0) s_dense = fb >= (uint32_t)SO_DENSE_THR ? 1 : 0;
            }
        };
        // ptile_body's `post`: the next task's dequeue, before the tile's drain (one-GPU,
        // frame-pipeline and stripe runs)
#ifndef SO_DEQ_LATE   // A/B builds: dequeue at the loop top, after the done flag
        const auto take_next = [&]() {
            if (wave == 0) nxt_v = run_dequeue(ws);   // waits for the tile's stores too
            nxt_taken = true;
        };
#else
        const NoPre take_next{};
#endif
        const uint8_t* ref = FPIPE ? sp.land0 + (long long)(sp.gbase + f) * sp.stride
                                   : (MODE == kRunSingle || TWOP) ? a.ref[f] : (f ? a.out[f - 1].recon : ref0);
        if constexpr (TWOP) {
            const int nb = nbx * (H / 16);
#ifdef SO_RUN_PROFILE
            const unsigned long long pt0 = __builtin_amdgcn_s_memtime();
#endif
            // pass 1 of (f, tile): the search (after the 3x3 reference tiles' done flags) and the
            // forward transform for the token counts; stores the ME records and tokens, then p1done
            const auto pass1_unit = [&]() {
                int32_t* const t1 = sp.t1 + (size_t)f * nb;
                const int bx0 = tx * G::TBX, byt0 = ty * G::TBY;
                using P = PTileGeo<G>;
                uint32_t* const b4w = reinterpret_cast<uint32_t*>(S.un);
                const Sea2Lds L{S.win, b4w, S.curt, S.a4, reinterpret_cast<uint16_t*>(b4w + P::B4), S.lcount, S.keys,
                                S.st, count_ops};
                RefSet refs{};
                refs.p[0] = ref;
                sea2_tile<G>(L, tile, a.cur[f], refs, 1, H, W, 0, by1, 0, wait_ref, nullptr,
                             MODE == kRunTwoPass && dep >= 0 ? a.out[dep].mv : nullptr);   // ends with a barrier
                for (int i = tid; i < G::NBLK; i += G::NTHREADS) {
                    int32_t rec4[4];
                    decode_key(S.keys[i], G::SR, rec4);
                    S.mer[i].set(rec4);
                }
                __syncthreads();
                SO_MARK(p1_tq);
                const int t2 = opaque_tid(), ln = t2 & 63, gq = (t2 >> 6) * G::TQ_BPW + (ln >> 4);
                if (ln < 16 * G::TQ_BPW && gq < G::NBLK)
                    tq16_pass1<G>(S, gq, ln & 15, S.un + gq * kTqScratch, bx0, byt0, nbx, by1, qp_rd, qp_row, a.out[f],
                                  t1);
                SO_MARK(p1_flag);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
                if (wave == 0)
                    __hip_atomic_store(sp.p1done + (size_t)f * ntiles + tile, ep, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                SO_RUN_PROF(48, __builtin_amdgcn_s_memtime() - pt0);
            };
            // pass 2 of (f2, tile2): after its tile row's p1done flags, the row's token sums, the
            // block QPs and the transforms on pass 1's records; stores the symbols and the
            // reconstruction, then the done flag
            const auto pass2_unit = [&](int f2, int tile2) {
                int32_t* const t1 = sp.t1 + (size_t)f2 * nb;
                const int ty2 = tile2 / tiles_x;
                const int bx0 = (tile2 - ty2 * tiles_x) * G::TBX, byt0 = ty2 * G::TBY;
                const uint8_t* const ref2 = FPIPE ? sp.land0 + (long long)(sp.gbase + f2) * sp.stride : a.ref[f2];
                SO_MARK(p2_wait);
                if (wave == 0) {   // every tile of this tile row finished pass 1 (tiles_x <= 64)
                    const uint32_t* c = sp.p1done + (size_t)f2 * ntiles + ty2 * tiles_x + (lane < tiles_x ? lane : 0);
                    // 50 ms of polling; 2 s in the frame pipeline, whose pass-1 tasks may wait that
                    // long on another rank's reconstruction
                    const RunWait rw{task, f2, -2, tile2, MODE | (2 << 8), ep, sp.epoch, FPIPE ? 200000000ull : 5000000ull};
                    run_poll(c, lane < tiles_x, false, ws, rw);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    SO_RUN_PROF(50, __builtin_amdgcn_s_memtime() - pt0);
                }
                __syncthreads();
                SO_MARK(p2_sums);
                if (wave < G::TBY) {   // pass-1 token sum of block row byt0 + wave
                    const int row = byt0 + wave;
                    uint32_t sum = 0;
                    if (row < by1)
                        for (int bx = lane; bx < nbx; bx += 64) sum += (uint32_t)t1[(size_t)row * nbx + bx];
                    sum = wave_sum_u32(sum);
                    if (lane == 0) S.msum[wave] = (int32_t)sum;
                }
                __syncthreads();
                // frame pipeline: where the final reconstruction goes (kRunFPipe's push code)
                const int code = FPIPE ? a.dep[f2] : -1;
                uint8_t* const push = code >= 0 ? ((code & 1) ? sp.peer_up0 : sp.peer_dn0) +
                                                      (long long)(code >> 1) * sp.stride : nullptr;
                SO_MARK(p2_tq);
                const int t2 = opaque_tid(), ln = t2 & 63, gq = (t2 >> 6) * G::TQ_BPW + (ln >> 4);
                if (ln < 16 * G::TQ_BPW && gq < G::NBLK)
                    tq16_pass2<G>(S, gq, ln & 15, S.un + gq * kTqScratch, bx0, byt0, nbx, by1, W, qp_rd, qp_row, sp.roi,
                                  sp.qp_lo, sp.qp_hi, a.cur[f2], ref2, a.out[f2], t1, push);
                SO_MARK(p2_flag);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // local and remote stores retired
                __syncthreads();
                if (wave == 0) {
                    __hip_atomic_store(done + (size_t)f2 * ntiles + tile2, ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (lane == 0 && code >= 0)
                        __hip_atomic_store(((code & 1) ? sp.peer_up_flags : sp.peer_dn_flags) +
                                               (size_t)(code >> 1) * ntiles + tile2,
                                           sp.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                SO_RUN_PROF(49, __builtin_amdgcn_s_memtime() - pt0);
            };
            if constexpr (MERGE2P) {
                // task k: pass 2 of unit k - lag2, then pass 1 of unit k.  Pass 1 of (f, t) needs
                // frame f-1's tiles up to t + tiles_x + 1, whose pass-2 units run in tasks up to
                // k (this one: unit k - lag2 = (f-1, t + tiles_x + 1)); pass 2 of unit j needs the
                // pass 1 of its tile row, units up to j + tiles_x - 1, in tasks before j + lag2
                // when 2 tiles_x < ntiles (the launcher checks).  So every wait is on this task's
                // own first part or on earlier tasks: deadlock-free as the one-pass run.
                if (u2 >= 0) {
                    const int f2 = u2 / ntiles;
                    pass2_unit(f2, u2 - f2 * ntiles);
                }
                if (has1) pass1_unit();
            } else if (pass == 1) {
                pass1_unit();
            } else {
                pass2_unit(f, tile);
            }
        } else if constexpr (FPIPE) {
            // where frame f's reconstruction goes (the ring direction alternates per block of N
            // frames): a.dep[f] = slot * 2 + (0: peer_dn, 1: peer_up) of the rank encoding frame
            // f + 1, or -1 when no frame follows (the GOP's last frame: nothing is pushed)
            const int code = a.dep[f];
            const int slot = code >> 1;
            uint8_t* const pbase = (code & 1) ? sp.peer_up0 : sp.peer_dn0;
            uint32_t* const pflags = (code & 1) ? sp.peer_up_flags : sp.peer_dn_flags;
            PHalo hl{};
            hl.dn = code >= 0 ? pbase + (long long)slot * sp.stride : nullptr;   // every row of the tile
            hl.dn_begin = 0;
            ptile_body<G, true, decltype(wait_ref), true, false, VBS, decltype(take_next)>(
                S, tile, a.cur[f], ref, H, W, 0, by1, qp_rd, qp_row, nullptr, nullptr, a.out[f], wait_ref, hl, lam,
                nullptr, nullptr, count_ops, take_next);
            // ptile_body ended with every wave's stores (local and remote) retired and a barrier
            if (wave == 0) {
                __hip_atomic_store(done + (size_t)f * ntiles + tile, ep, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                if (lane == 0 && code >= 0)
                    __hip_atomic_store(pflags + (size_t)slot * ntiles + tile, sp.epoch, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else if constexpr (STRIPE) {
            const int gf = sp.gbase + f;
            PHalo hl{};
            if (first_row && sp.peer_up0) {
                hl.up = sp.peer_up0 + (long long)gf * sp.stride;
                hl.up_end = by0 * 16 + 16;
            }
            if (last_row && sp.peer_dn0) {
                hl.dn = sp.peer_dn0 + (long long)gf * sp.stride;
                hl.dn_begin = by1 * 16 - 16;
            }
            ptile_body<G, true, decltype(wait_ref), true, false, false, decltype(take_next)>(
                S, tile, a.cur[f], ref, H, W, by0, by1, qp_rd, qp_row, nullptr, nullptr, a.out[f], wait_ref, hl, 0.0,
                nullptr, nullptr, count_ops, take_next, f > 0 ? a.out[f - 1].mv : nullptr);
            // ptile_body ended with every wave's stores (local and remote) retired and a barrier
            if (wave == 0) {
                __hip_atomic_store(done + (size_t)f * ntiles + tile, ep, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                if (lane == 0 && hl.up)
                    __hip_atomic_store(sp.peer_up_flags + (size_t)gf * tiles_x + tx, sp.epoch, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
                if (lane == 1 && hl.dn)
                    __hip_atomic_store(sp.peer_dn_flags + (size_t)gf * tiles_x + tx, sp.epoch, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
            }
        } else {
#ifdef SO_RUN_PROFILE
            const unsigned long long pt0 = __builtin_amdgcn_s_memtime();
#endif
            ptile_body<G, true, decltype(wait_ref), false, false, VBS, decltype(take_next), false, ZSKIP && !VBS, LISTS>(
                S, tile, a.cur[f], ref, H, W, 0, by1, qp_rd, qp_row, nullptr, nullptr, a.out[f], wait_ref, PHalo{}, lam,
                &s_dense, reinterpret_cast<int32_t*>(tilefb) + (size_t)f * ntiles + tile, count_ops, take_next,
                // VBS: the same hint for the block's U measured slower (4K VBS P-frame 123.1 vs
                // 121.3 us: 8 more VGPR spills; profiles/r05/hint_ab_vbs.log), appended to list A
                // (its quadrant SADs bounding the sub-block U_j) 117.8 vs 115.9 us (6 more spills;
                // profiles/r05/vbs_ab6_lista_hint.log)
                !VBS && dep >= 0 ? a.out[dep].mv : nullptr);
            SO_RUN_PROF(52, __builtin_amdgcn_s_memtime() - pt0);
            SO_MARK(done_flag);
            // ptile_body ended with every wave's write-through stores retired and a barrier
            // (sp.lose_task: SO_OPT_TEST_LOSE_FLAG, the wait diagnostics' test -- that task's flag
            // is never set, so its dependants time out and record themselves)
            if (wave == 0 && !(HOOKS && task + 1 == sp.lose_task))
                __hip_atomic_store(done + (size_t)f * ntiles + tile, ep, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
        }
        SO_MARK(task_end);
        if (pass == 1 && tid == 0) {   // this tile's dense-searched blocks and SAD byte operations
            s_fbsum += S.st[0];
            if constexpr (HOOKS) s_ops += S.st[2];
        }
#ifdef SO_STAMPS
        if (tid == 0 && rec) {
            uint32_t hw, xcc;
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
            asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
            rec[11] = __builtin_amdgcn_s_memrealtime();
            rec[12] = ((unsigned long long)xcc << 32) | hw;
            rec[13] = __builtin_amdgcn_s_memtime();
        }
#endif
    }
#ifdef SO_MARKS_COUNT
    __syncthreads();
    if (tid < kMarkCount && g_mark_counts) atomicAdd(&g_mark_counts[tid], s_mark_cnt[tid]);
#endif
    // the last workgroup out resets the task and exit counters and publishes the epoch
    if (wave == 0) {
        const uint32_t fbsum = __builtin_amdgcn_readfirstlane(s_fbsum);
        if (fbsum != 0u)
            __hip_atomic_fetch_add(&ws[kRunFallbackWord], lane == 0 ? fbsum : 0u, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long ops = s_ops;
        if (ops != 0ull)
            __hip_atomic_fetch_add(reinterpret_cast<unsigned long long*>(ws + kRunSadOpsWord), lane == 0 ? ops : 0ull,
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (wave == 0) {
        const uint32_t o = __builtin_amdgcn_readfirstlane(
            __hip_atomic_fetch_add(&ws[kRunExitWord], one, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
        if (o == gridDim.x - 1) {
            __hip_atomic_store(&ws[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ws[kRunExitWord], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(&ws[kRunEpochWord], ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}
#ifndef SO_EP_REG
#undef ep
#endif

// [kRunDoneBase, +kRunMax * ntiles64) done flags, then (two-pass runs) kRunMax * ntiles128
// pass-1 done flags and kRunMax * nb pass-1 token counts
static size_t run_tiles(int H, int W, int tbx, int tby) {
    return (size_t)((W / 16 + tbx - 1) / tbx) * ((H / 16 + tby - 1) / tby);
}
size_t p_run_workspace_words(int H, int W) {
    using G = Sea2Geo;
    return (size_t)kRunDoneBase + 3 * (size_t)kRunMax * run_tiles(H, W, G::TBX, G::TBY) +
           (size_t)kRunMax * (W / 16) * (H / 16);   // + the per-tile dense counts
}

// Launch the run in <= kRunMax-frame launches.  max_wg > 0 caps the resident grid (several
// ranks sharing one GPU in the tests).
// The calling thread's current device: its CU count and the kernel's resident workgroups per CU
// (the occupancy API), cached per (device, kernel) under a mutex -- a process may drive several
// devices from several host threads.  (The grid only sizes the run: a workgroup that is not
// resident holds no task, so an over-estimate costs speed, never progress.)
constexpr size_t kLdsPerCuObserved = 161280;   // gfx950: 3 x 53,760 B resident at once (ubench_lds_occ)
// the VBS run holds three workgroups per CU only while its LDS (PTileLds + the kernel's few
// scalars) stays within 53,760 B: a later LDS increase must not silently drop it to two
static_assert(sizeof(PTileLds<Sea2GeoT<SO_PTILE_NW>, true>) + 64 <= kLdsPerCuObserved / 3,
              "the VBS run's LDS no longer fits three workgroups per gfx950 CU");
static int run_shape(const void* kernel, int* ncu, int* per_cu) {
    static std::mutex mu;
    static std::map<std::pair<int, const void*>, std::pair<int, int>> cache;
    int dev = 0;
    const hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) {
        set_error("p_run: hipGetDevice: %s", hipGetErrorString(e));
        return (int)e;
    }
    std::lock_guard<std::mutex> lk(mu);
    const auto key = std::make_pair(dev, kernel);
    auto it = cache.find(key);
    if (it == cache.end()) {
        int n = 0, p = 0;
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&p, kernel, SO_PTILE_NW * 64, 0) != hipSuccess || p <= 0) p = 1;
        // The occupancy API over-counts near the LDS limit on gfx950: it reports three
        // 512-thread workgroups per CU for 53,880 B of LDS, but a CU runs only two of them at
        // once (three up to 53,760 B; tools/ubench_lds_occ.cpp, profiles/r05/ubench_lds_occ.log).
        // Count 512-B granules against the 161,280 B three such workgroups were seen to share.
        // (an observation on gfx950 only: other devices keep the occupancy API's count)
        hipDeviceProp_t prop{};
        const bool gfx950 = hipGetDeviceProperties(&prop, dev) == hipSuccess &&
                            std::strncmp(prop.gcnArchName, "gfx950", 6) == 0;
        hipFuncAttributes fa{};
        if (gfx950 && hipFuncGetAttributes(&fa, kernel) == hipSuccess && fa.sharedSizeBytes > 0) {
            const size_t g = (fa.sharedSizeBytes + 511) & ~(size_t)511;
            const int by_lds = (int)(kLdsPerCuObserved / g);
            if (by_lds >= 1 && by_lds < p) p = by_lds;
        }
        it = cache.emplace(key, std::make_pair(n, p)).first;
    }
    *ncu = it->second.first;
    *per_cu = it->second.second;
    return SO_OK;
}

// Resident workgroups of the persistent run kernel on the current device (so_p_run_resident_
// workgroups): the grid a launch uses when nothing caps it.
// mode < 0: the smallest over every instantiation a run of that VBS setting may launch (the
// one-GPU run with and without test hooks, the stripe, frame-pipeline and two-pass modes): the
// ranks sharing one device size their claims by it, whichever kernel each of them launches.
int p_run_capacity(int vbs, int mode) {
    constexpr int NW = SO_PTILE_NW;
    const void* ks[13];
    int n = 0;
    const auto add = [&](int m, const void* k) {
        if (mode < 0 || mode == m) ks[n++] = k;
    };
    if (vbs) {
        add(kRunSingle, reinterpret_cast<const void*>(p_run_kernel<NW, kRunSingle, true>));
        add(kRunSingle, reinterpret_cast<const void*>(p_run_kernel<NW, kRunSingle, true, true>));
        add(kRunSingle, reinterpret_cast<const void*>(p_run_kernel<NW, kRunSingle, true, false, true>));
        add(kRunSingle, reinterpret_cast<const void*>(p_run_kernel<NW, kRunSingle, true, true, true>));
        add(kRunSingle, reinterpret_cast<const void*>(p_run_kernel<NW, kRunSingle, true, false, true, true>));
        add(kRunFPipe, reinterpret_cast<const void*>(p_run_kernel<NW, kRunFPipe, true>));
        add(kRunFPipe, reinterpret_cast<const void*>(p_run_kernel<NW, kRunFPipe, true, false, true>));
    } else {
        add(kRunSingle, reinterpret_cast<const void*>(p_run_kernel<NW, kRunSingle, false>));
        add(kRunSingle, reinterpret_cast<const void*>(p_run_kernel<NW, kRunSingle, false, true>));
        add(kRunSingle, reinterpret_cast<const void*>(p_run_kernel<NW, kRunSingle, false, false, false, true>));
        add(kRunStripe, reinterpret_cast<const void*>(p_run_kernel<NW, kRunStripe, false>));
        add(kRunFPipe, reinterpret_cast<const void*>(p_run_kernel<NW, kRunFPipe, false>));
        add(kRunTwoPass, reinterpret_cast<const void*>(p_run_kernel<NW, kRunTwoPass, false>));
        add(kRunFPipe2P, reinterpret_cast<const void*>(p_run_kernel<NW, kRunFPipe2P, false>));
    }
    if (n == 0) return -SO_E_INVALID;
    int best = 0;
    for (int i = 0; i < n; ++i) {
        int ncu = 0, per_cu = 0;
        const int rc = run_shape(ks[i], &ncu, &per_cu);
        if (rc != SO_OK) return -rc;
        if (i == 0 || ncu * per_cu < best) best = ncu * per_cu;
    }
    return best;
}

// refs / deps (may be null: one run, frame g predicting from g - 1 and frame 0 from ref0): frame g
// predicts from outs[deps[g]].recon when deps[g] >= 0 (0 <= deps[g] < g), else from refs[g].
// conc: independent runs interleaved in the list (their tiles are in flight together).
template <int MODE, bool VBS = false>
static int p_run_launch_t(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int qp_rd,
                          const int32_t* qp_row, const PFrameOut* outs, uint32_t* ws, const PRunStripe& sp0,
                          int max_wg, hipStream_t st, const uint8_t* const* refs = nullptr,
                          const int* deps = nullptr, int conc = 1, double lam = 0.0) {
    using G = Sea2GeoT<SO_PTILE_NW>;
    // the test-hook instantiation (one GPU only) while SO_OPT_COUNT_SAD_OPS / _TEST_LOSE_FLAG is set
    const bool hook_set = option(SO_OPT_COUNT_SAD_OPS) != 0 || option(SO_OPT_TEST_LOSE_FLAG) != 0;
    if (hook_set && MODE != kRunSingle) {   // no hook instantiation here: refuse rather than ignore
        set_error("p_run: SO_OPT_COUNT_SAD_OPS / SO_OPT_TEST_LOSE_FLAG apply to the one-GPU run only (so_encode_p_run, "
                  "so_encode_p_runs); this run kind has no hook instantiation");
        return SO_E_INVALID;
    }
    const bool hooks = MODE == kRunSingle && hook_set;
    // VBS without a row-QP schedule: the uniform-QP instantiation (p_run_kernel's UQP)
    const bool uqp = VBS && qp_row == nullptr;
    // the plain one-GPU run with the all-zero-wave IDCT skip (SO_OPT_RUN_ZERO_SKIP; not with hooks)
    constexpr bool ZS_OK = MODE == kRunSingle && !VBS;
    const bool zskip = ZS_OK && !hooks && option(SO_OPT_RUN_ZERO_SKIP) != 0;
    // the uniform-QP VBS run's latency-bound twin (p_run_kernel's ZSKIP slot on VBS): chosen below
    // when the grid has more slots than a frame has tiles
    constexpr bool VL_OK = MODE == kRunSingle && VBS;
    const bool vlat_ok = VL_OK && uqp && !hooks && SO_VBS_BALLOT_LATENCY;
    const void* const kfn =
        hooks ? (uqp ? reinterpret_cast<const void*>(p_run_kernel<SO_PTILE_NW, MODE, VBS, MODE == kRunSingle, VBS>)
                     : reinterpret_cast<const void*>(p_run_kernel<SO_PTILE_NW, MODE, VBS, MODE == kRunSingle>))
              : (uqp     ? reinterpret_cast<const void*>(p_run_kernel<SO_PTILE_NW, MODE, VBS, false, VBS>)
                 : zskip ? reinterpret_cast<const void*>(p_run_kernel<SO_PTILE_NW, MODE, VBS, false, false, ZS_OK>)
                         : reinterpret_cast<const void*>(p_run_kernel<SO_PTILE_NW, MODE, VBS, false>));
    if (hooks && option(SO_OPT_TEST_LOSE_FLAG) != 0) {
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) {
            set_error("p_run: SO_OPT_TEST_LOSE_FLAG is set while the stream is capturing (the graph would lose a "
                      "flag on every replay)");
            return SO_E_INVALID;
        }
    }
    int ncu = 0, per_cu = 0;
    {
        const int rc = run_shape(kfn, &ncu, &per_cu);
        if (rc != SO_OK) return rc;
    }
    const int nbx = W / 16;
    const int rows = MODE == kRunStripe ? sp0.by1 - sp0.by0 : H / 16;
    const long ntiles = (long)((nbx + G::TBX - 1) / G::TBX) * ((rows + G::TBY - 1) / G::TBY);
    for (int f0 = 0; f0 < nframes; f0 += kRunMax) {
        const int n = nframes - f0 < kRunMax ? nframes - f0 : kRunMax;
        PRunArgs a{};
        for (int i = 0; i < n; ++i) {
            const int g = f0 + i;
            const int d = deps ? deps[g] : g - 1;
            a.cur[i] = curs[g];
            a.out[i] = outs[g];
            if (MODE == kRunFPipe || MODE == kRunFPipe2P) {   // deps = the per-frame push codes (slot * 2 + peer)
                a.ref[i] = nullptr;
                a.dep[i] = deps ? deps[g] : -1;
                continue;
            }
            a.ref[i] = d >= 0 ? outs[d].recon : (refs ? refs[g] : ref0);
            a.dep[i] = d >= f0 ? d - f0 : -1;   // an earlier launch's frame is complete (stream order)
        }
        // nothing to reset: the kernel leaves the task / exit counters at 0 and done flags are
        // compared with the launch's epoch (the caller zeroes the workspace once)
        // A frame with fewer tiles than resident slots (1080p: 510 tiles, 768 slots) gets
        // ceil(ntiles / ncu) workgroups per CU: every CU then runs its share of a frame's tiles
        // side by side, instead of some CUs running three (slower) while the next frame's tiles
        // wait on others -- a frame's time is its slowest tile's (1080p: 30 vs 33 us/frame).
        int pcu = (int)((ntiles * conc + ncu - 1) / ncu);
        if (pcu > per_cu) pcu = per_cu;
#ifdef SO_AB
        if (const char* e = getenv("SO_RUN_PER_CU")) {   // A/B builds only: resident workgroups per CU
            const int v = atoi(e);
            if (v > 0 && v <= per_cu) pcu = v;
        }
#endif
        long grid = (long)ncu * pcu;
        if (grid > ntiles * n) grid = ntiles * n;
        if (max_wg > 0 && grid > max_wg) grid = max_wg;
        PRunStripe sp = sp0;
        sp.gbase = sp0.gbase + f0;
        sp.count_ops = option(SO_OPT_COUNT_SAD_OPS);
        sp.lose_task = f0 == 0 ? option(SO_OPT_TEST_LOSE_FLAG) : 0;
        if (MODE == kRunTwoPass || MODE == kRunFPipe2P) {   // pass 2 of a row about one grid's worth of tasks after its pass 1
            const int tiles_x = (nbx + G::TBX - 1) / G::TBX, ntr = (rows + G::TBY - 1) / G::TBY;
            // about one grid's worth of tile rows (a pass-2 task then rarely waits holding its
            // slot), capped by the caller's lag (the frame pipeline: consecutive frames on
            // different ranks trail each other by ~lag + 2 rows, so more ranks want less)
            int lag = (int)((grid + tiles_x - 1) / tiles_x);
            if (sp0.p2lag > 0 && sp0.p2lag < lag) lag = sp0.p2lag;
#ifdef SO_AB
            if (const char* e = getenv("SO_P2LAG")) lag = atoi(e);   // A/B builds only
#endif
            sp.p2lag = lag < 1 ? 1 : (lag > ntr ? ntr : lag);
        }
        const uint8_t* const r0 = f0 ? outs[f0 - 1].recon : ref0;
#define SO_P_RUN_GO(HK, UQ, ZS)                                                                                         \
    hipLaunchKernelGGL((p_run_kernel<SO_PTILE_NW, MODE, VBS, HK, UQ, ZS>), dim3((unsigned)grid), dim3(SO_PTILE_NW * 64), \
                       0, st, a, n, r0, H, W, qp_rd, qp_row, ws, (int)(f0 * ntiles), sp, lam)
        if (hooks && uqp)
            SO_P_RUN_GO(MODE == kRunSingle, VBS, false);
        else if (hooks)
            SO_P_RUN_GO(MODE == kRunSingle, false, false);
        else if (uqp && vlat_ok && ntiles < grid)
            SO_P_RUN_GO(false, VBS, VL_OK);
        else if (uqp)
            SO_P_RUN_GO(false, VBS, false);
        else if (zskip)
            SO_P_RUN_GO(false, false, ZS_OK);
        else
            SO_P_RUN_GO(false, false, false);
#undef SO_P_RUN_GO
        const int rc = check_launch("p_run_kernel");
        if (rc != SO_OK) return rc;
    }
    return SO_OK;
}

// One GPU: 128-px tiles (64-px tiles -- 8 blocks, one per wave in the search -- measured no
// faster where a frame has fewer tiles than resident workgroups, 1088p 29.5 vs 28.3 us per
// frame, and 1.56x slower at 4K: removed).
int p_run_launch(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int qp_rd,
                 const int32_t* qp_row, int vbs, double lam, const PFrameOut* outs, uint32_t* ws, hipStream_t st) {
    PRunStripe sp{};
    sp.by0 = 0;
    sp.by1 = H / 16;
    if (vbs)
        return p_run_launch_t<kRunSingle, true>(curs, nframes, ref0, H, W, qp_rd, qp_row, outs, ws, sp, 0, st, nullptr,
                                                nullptr, 1, lam);
    return p_run_launch_t<kRunSingle>(curs, nframes, ref0, H, W, qp_rd, qp_row, outs, ws, sp, 0, st);
}

// Several independent runs in one list (so_encode_p_runs): frame g predicts from
// outs[deps[g]].recon (deps[g] < g) or, with deps[g] < 0, from refs[g].
int p_runs_launch(const uint8_t* const* curs, int nframes, const uint8_t* const* refs, const int* deps, int conc,
                  int H, int W, int qp_rd, const int32_t* qp_row, int vbs, double lam, const PFrameOut* outs,
                  uint32_t* ws, hipStream_t st) {
    PRunStripe sp{};
    sp.by0 = 0;
    sp.by1 = H / 16;
    if (vbs)
        return p_run_launch_t<kRunSingle, true>(curs, nframes, nullptr, H, W, qp_rd, qp_row, outs, ws, sp, 0, st, refs,
                                                deps, conc, lam);
    return p_run_launch_t<kRunSingle>(curs, nframes, nullptr, H, W, qp_rd, qp_row, outs, ws, sp, 0, st, refs, deps,
                                           conc);
}

// The workspace's pass-1 token region (kRunMax * nb words; the per-frame two-pass sequence of
// so_encode_p_run_2pass keeps its ME records there)
int32_t* p_run_t1_region(uint32_t* ws, int H, int W) {
    return reinterpret_cast<int32_t*>(ws + kRunDoneBase + 2 * (size_t)kRunMax * run_tiles(H, W, Sea2Geo::TBX, Sea2Geo::TBY));
}

// The merged two-pass schedule's deadlock-freedom needs 2 tiles_x < ntiles: three tile rows or more
bool p_run_2pass_fused_ok(int H, int W) {
    const int tiles_x = (W / 16 + Sea2Geo::TBX - 1) / Sea2Geo::TBX;
    return 2 * tiles_x < run_tiles(H, W, Sea2Geo::TBX, Sea2Geo::TBY);
}

// Two-pass rate control over a run (so_encode_p_run_2pass): one run as p_run_launch, each tile
// as a pass-1 and a pass-2 task (kRunTwoPass).
int p_run_2pass_launch(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int qp_rd,
                       const int32_t* qp_row, const int32_t* roi, int qp_lo, int qp_hi, const PFrameOut* outs,
                       uint32_t* ws, hipStream_t st) {
    if (!p_run_2pass_fused_ok(H, W)) {
        set_error("so_encode_p_run_2pass (fused): needs three tile rows (H > %d)", 2 * 16 * Sea2Geo::TBY);
        return SO_E_UNSUPPORTED;
    }
    PRunStripe sp{};
    sp.by0 = 0;
    sp.by1 = H / 16;
    sp.p1done = ws + kRunDoneBase + (size_t)kRunMax * run_tiles(H, W, Sea2Geo::TBX, Sea2Geo::TBY);
    sp.t1 = reinterpret_cast<int32_t*>(sp.p1done + (size_t)kRunMax * run_tiles(H, W, Sea2Geo::TBX, Sea2Geo::TBY));
    sp.roi = roi;
    sp.qp_lo = qp_lo;
    sp.qp_hi = qp_hi;
    return p_run_launch_t<kRunTwoPass>(curs, nframes, ref0, H, W, qp_rd, qp_row, outs, ws, sp, 0, st, nullptr,
                                            nullptr, 2);
}

int p_run_stripe_launch(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int qp_rd,
                        const int32_t* qp_row, const PFrameOut* outs, uint32_t* ws, const PRunStripe& sp, int max_wg,
                        hipStream_t st) {
    return p_run_launch_t<kRunStripe>(curs, nframes, ref0, H, W, qp_rd, qp_row, outs, ws, sp, max_wg, st);
}

int p_run_fpipe_launch(const uint8_t* const* curs, int nframes, int H, int W, int qp_rd, const int32_t* qp_row,
                       int vbs, double lam, const PFrameOut* outs, uint32_t* ws, const PRunStripe& sp, int max_wg,
                       hipStream_t st, const int* push) {
    if (vbs)
        return p_run_launch_t<kRunFPipe, true>(curs, nframes, nullptr, H, W, qp_rd, qp_row, outs, ws, sp, max_wg, st,
                                               nullptr, push, 1, lam);
    return p_run_launch_t<kRunFPipe>(curs, nframes, nullptr, H, W, qp_rd, qp_row, outs, ws, sp, max_wg, st,
                                          nullptr, push);
}

// The frame pipeline with two-pass RC (kRunFPipe2P): sp as p_run_fpipe_launch plus the ROI / QP
// clamp; the pass-1 flags and token counts live in the workspace as in p_run_2pass_launch.
int p_run_fpipe_2pass_launch(const uint8_t* const* curs, int nframes, int H, int W, int qp_rd, const int32_t* qp_row,
                             const PFrameOut* outs, uint32_t* ws, const PRunStripe& sp0, int max_wg, hipStream_t st,
                             const int* push) {
    PRunStripe sp = sp0;
    sp.p1done = ws + kRunDoneBase + (size_t)kRunMax * run_tiles(H, W, Sea2Geo::TBX, Sea2Geo::TBY);
    sp.t1 = reinterpret_cast<int32_t*>(sp.p1done + (size_t)kRunMax * run_tiles(H, W, Sea2Geo::TBX, Sea2Geo::TBY));
    return p_run_launch_t<kRunFPipe2P>(curs, nframes, nullptr, H, W, qp_rd, qp_row, outs, ws, sp, max_wg, st,
                                           nullptr, push, 2);
}

// The I-frame's hand-off (the P-frame run's frame 0 reads its boundary rows): copy the
// stripe's top 16 rows into the up neighbour's plane and its bottom 16 rows into the down
// neighbour's, then set their flags [gf * tiles_x + tx] = epoch.  One workgroup per (tile
// column, direction): 16 rows x 128 bytes, one dwordx4 per thread, system-scope write-through.
__global__ void __launch_bounds__(128) stripe_halo_push_kernel(const uint8_t* __restrict__ plane, int W, int y0, int y1,
                                                               uint8_t* up, uint8_t* dn, uint32_t* up_flags,
                                                               uint32_t* dn_flags, int gf, int tiles_x,
                                                               uint32_t epoch) {
    const int tx = blockIdx.x % tiles_x, dir = blockIdx.x / tiles_x;   // 0 up, 1 down
    uint8_t* dst = dir == 0 ? up : dn;
    if (dst == nullptr) return;   // uniform
    const int r = threadIdx.x >> 3, c = (threadIdx.x & 7) * 16;       // 16 rows x 8 dwordx4
    const int y = (dir == 0 ? y0 : y1 - 16) + r, x = tx * 128 + c;
    if (x < W && y >= y0 && y < y1) {
        const so_v4u v = *reinterpret_cast<const so_v4u*>(plane + (size_t)y * W + x);
        uint8_t* q = dst + (size_t)y * W + x;
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q), "v"(v) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
        __hip_atomic_store((dir == 0 ? up_flags : dn_flags) + (size_t)gf * tiles_x + tx, epoch, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
}

int stripe_halo_push_launch(const uint8_t* plane, int W, int by0, int by1, uint8_t* up, uint8_t* dn,
                            uint32_t* up_flags, uint32_t* dn_flags, int gf, uint32_t epoch, hipStream_t st) {
    const int tiles_x = (W / 16 + Sea2Geo::TBX - 1) / Sea2Geo::TBX;
    hipLaunchKernelGGL(stripe_halo_push_kernel, dim3(2 * tiles_x), dim3(128), 0, st, plane, W, by0 * 16, by1 * 16, up,
                       dn, up_flags, dn_flags, gf, tiles_x, epoch);
    return check_launch("stripe_halo_push_kernel");
}

// The I-frame's hand-off in the frame pipeline (kRunFPipe): the whole reconstruction into
// the next rank's landing plane `dst`, tile by tile (128 x 32 px: one dwordx4 per thread,
// system-scope write-through), each tile's flag flags[t] = epoch once its stores drained.
__global__ void __launch_bounds__(256) frame_push_kernel(const uint8_t* __restrict__ plane, int H, int W,
                                                         uint8_t* dst, uint32_t* flags, int tiles_x, uint32_t epoch) {
    const int t = blockIdx.x, tx = t % tiles_x, ty = t / tiles_x;
    const int r = threadIdx.x >> 3, c = (threadIdx.x & 7) * 16;       // 32 rows x 8 dwordx4
    const int y = ty * 32 + r, x = tx * 128 + c;
    if (x < W && y < H) {
        const so_v4u v = *reinterpret_cast<const so_v4u*>(plane + (size_t)y * W + x);
        uint8_t* q = dst + (size_t)y * W + x;
        asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(q), "v"(v) : "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(flags + t, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int frame_push_launch(const uint8_t* plane, int H, int W, uint8_t* dst, uint32_t* flags, uint32_t epoch,
                      hipStream_t st) {
    const int tiles_x = (W / 16 + Sea2Geo::TBX - 1) / Sea2Geo::TBX;
    const int ntr = (H / 16 + Sea2Geo::TBY - 1) / Sea2Geo::TBY;
    hipLaunchKernelGGL(frame_push_kernel, dim3(tiles_x * ntr), dim3(256), 0, st, plane, H, W, dst, flags, tiles_x,
                       epoch);
    return check_launch("frame_push_kernel");
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

// `planes` != NULL: FME (FmePhase above) -- the candidates are the half-pel offsets in
// [-2sr, 2sr] at (2x, 2y) on the frac frame, read from its phase planes, with the
// reference's FME bound (find_best_match :697-705); the scan index runs over that range.
__global__ void me_generic_kernel(const uint8_t* __restrict__ cur, RefSet refs, const uint8_t* __restrict__ planes,
                                  size_t pstride, int nref, int H, int W, int bs, int by0, int nrows, int sb_mode,
                                  int sr, unsigned long long* __restrict__ keys) {
    // sb_mode 0: full blocks (size bs); 1: sub-blocks (size bs/2, 4 per block)
    const bool fme = planes != nullptr;
    const int R = fme ? 2 * sr : sr;
    const int d = 2 * R + 1;
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
    const int dx = dxi - R, dy = di - R;
    uint32_t sad = 0;
    if (fme) {
        const int W2 = 2 * W - 1, H2 = 2 * H - 1, px = 2 * x + dx, py = 2 * y + dy;
        if (!(px >= 0 && px < W2 - tbs && py >= 0 && py < H2 - tbs && px + 2 * tbs < W2 - tbs &&
              py + 2 * tbs < H2 - tbs))
            return;
        const uint8_t* pl = planes + (size_t)(4 * r + 2 * (py & 1) + (px & 1)) * pstride;
        for (int i = 0; i < tbs; ++i)
            for (int j = 0; j < tbs; ++j) {
                int a = cur[(size_t)(y + i) * W + x + j], c = pl[(size_t)((py >> 1) + i) * W + (px >> 1) + j];
                sad += (uint32_t)(a > c ? a - c : c - a);
            }
    } else {
        if (!(x + dx >= 0 && x + dx < W - tbs && y + dy >= 0 && y + dy < H - tbs)) return;
        const uint8_t* ref = refs.p[r];
        for (int i = 0; i < tbs; ++i)
            for (int j = 0; j < tbs; ++j) {
                int a = cur[(size_t)(y + i) * W + x + j], c = ref[(size_t)(y + dy + i) * W + x + dx + j];
                sad += (uint32_t)(a > c ? a - c : c - a);
            }
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

int me_generic_launch(const uint8_t* cur, const RefSet& refs, const uint8_t* planes, size_t pstride, int nref, int H,
                      int W, int bs, int sr, int by0, int by1, int32_t* out_best, int32_t* out_sub, hipStream_t st);

int me_launch(const uint8_t* cur, const RefSet& refs, int nref, int H, int W, int bs, int sr, int by0, int by1,
              int32_t* out_best, int32_t* out_sub, hipStream_t st) {
    const int nbx = W / bs, nrows = by1 - by0;
    if (nrows <= 0) return SO_OK;
    if (sr == 16 && (bs == 16 || bs == 8) && (out_sub == nullptr || bs == 16)) {
#ifdef SO_AB   // A/B builds: SO_ME_IMPL=dense selects the dense wave kernel where SEA would run
        const char* impl = getenv("SO_ME_IMPL");
        const bool use_dense = impl && strcmp(impl, "dense") == 0;
        const char* pr = getenv("SO_SEA_PROBE");   // timing probes only (tools/me_ab2.py)
#else
        const bool use_dense = false;
        const char* pr = nullptr;
#endif
        if (!use_dense && bs == 16 && out_sub == nullptr) {
            const dim3 sgrid(((nbx + Sea2Geo::TBX - 1) / Sea2Geo::TBX) * ((nrows + Sea2Geo::TBY - 1) / Sea2Geo::TBY));
            hipLaunchKernelGGL(me_sea2_kernel, sgrid, dim3(Sea2Geo::NTHREADS), 0, st, cur, refs, nref, H, W, by0, by1,
                               out_best, pr ? atoi(pr) : 0);
            return check_launch("me_sea2_kernel");
        }
        const bool sub = out_sub != nullptr;
        const int tbx = 128 / bs;
        const int tby = (sub ? MeWGeo<16, true>::TPY : MeWGeo<16, false>::TPY) / bs;
        const dim3 wgrid(((nbx + tbx - 1) / tbx) * ((nrows + tby - 1) / tby));
        const dim3 wblk(sub ? MeWGeo<16, true>::NTHREADS : MeWGeo<16, false>::NTHREADS);
        if (bs == 16 && out_sub)
            hipLaunchKernelGGL((me_wave_kernel<16, true>), wgrid, wblk, 0, st, cur, refs, nref, H, W, by0, by1,
                               out_best, out_sub);
        else if (bs == 16)
            hipLaunchKernelGGL((me_wave_kernel<16, false>), wgrid, wblk, 0, st, cur, refs, nref, H, W, by0, by1,
                               out_best, out_sub);
        else
            hipLaunchKernelGGL((me_wave_kernel<8, false>), wgrid, wblk, 0, st, cur, refs, nref, H, W, by0, by1,
                               out_best, nullptr);
        return check_launch("me_wave_kernel");
    }
    return me_generic_launch(cur, refs, nullptr, 0, nref, H, W, bs, sr, by0, by1, out_best, out_sub, st);
}

int me_generic_launch(const uint8_t* cur, const RefSet& refs, const uint8_t* planes, size_t pstride, int nref, int H,
                      int W, int bs, int sr, int by0, int by1, int32_t* out_best, int32_t* out_sub, hipStream_t st) {
    const int nbx = W / bs, nrows = by1 - by0;
    if (nrows <= 0) return SO_OK;
    const int R = planes ? 2 * sr : sr;
    const int d = 2 * R + 1;
    for (int mode = 0; mode < (out_sub ? 2 : 1); ++mode) {
        const int nunit = nbx * nrows * (mode ? 4 : 1);
        int32_t* out = mode ? out_sub : out_best;
        unsigned long long* keys = reinterpret_cast<unsigned long long*>(out);
        hipLaunchKernelGGL(me_generic_init, dim3((nunit + 255) / 256), dim3(256), 0, st, keys, nunit);
        const long long ntot = (long long)nunit * nref * d * d;
        hipLaunchKernelGGL(me_generic_kernel, dim3((unsigned)((ntot + 255) / 256)), dim3(256), 0, st,
                           cur, refs, planes, pstride, nref, H, W, bs, by0, nrows, mode, sr, keys);
        hipLaunchKernelGGL(me_generic_finalize, dim3((nunit + 255) / 256), dim3(256), 0, st, nunit,
                           R, out);
    }
    return check_launch("me_generic_kernel");
}

}  // namespace so
