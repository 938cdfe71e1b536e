// so_pack.hip — the symbols of a frame as one packed byte stream on the device, so a host
// caller downloads the bitstream's content (symbols out of the timed region)
// instead of the dense int16 QTC planes (2 B per pixel).
//
// The content is exactly what the reference's two text lines carry per frame: the block's
// split flag and motion vectors (differential_encoder_frame, Encoder.py:1419-1520, before its
// differencing) and the RLE token list of every (sub-)block (entropy_encoder_block,
// :1086-1131, which entropy_encoder_frame joins, :1522-1542).  Per block, in raster order:
//     split | mv values | tokens of each (sub-)block
// every number a zigzag LEB128 varint (zz(v) = 2v for v >= 0, -2v-1 for v < 0; 7 bits per
// byte, high bit = more).  mv values: inter (dx, dy, ref) once, or 4x in Z order when split;
// intra dx once or 4x.  A (sub-)block's token list is self-delimiting: "-L" and L values
// cover L coefficients, "Z" (> 0) covers Z zeros, "0" ends the block (the trailing zero
// run), and a list ends after n*n coefficients otherwise.  bitstream.unpack_frame restores
// the lists and MVs on the host.
//
// Two passes over the frame (one wave per block): byte counts, an exclusive scan per frame
// (one workgroup), then the bytes at their offsets.  HBM-bound: the dense QTC read once per
// pass (2 B/px) against the packed stream written once.  A block whose bytes would pass the
// caller's capacity is not written (the caller compares offs[nb] with it).
#include "so_common.h"

namespace so {

// Worst case bytes of one block: split + 4 x 3 mv varints + the token list of bs*bs
// coefficients (at most nn values + nn/2 + 1 run tokens, 3 bytes for any int16).
size_t pack_block_bound(int bs) { return 1 + 12 * 3 + (size_t)3 * (bs * bs + bs * bs / 2 + 4); }
constexpr int kPackStage = 1 + 12 * 3 + 3 * (256 + 128 + 4);   // pack_block_bound(16)

// scan position -> row-major index in an n x n block (anti-diagonal order, :1093-1123)
__constant__ uint8_t c_scan16[256];
__constant__ uint8_t c_scan8[64];

static bool g_scan_ready = false;

static int init_scan_tables() {
    if (g_scan_ready) return SO_OK;
    uint8_t t16[256], t8[64];
    for (int n : {16, 8}) {
        uint8_t* t = n == 16 ? t16 : t8;
        int p = 0;
        for (int k = 0; k < 2 * n - 1; ++k) {
            int i = k < n ? 0 : k - n + 1, j = k < n ? k : n - 1;
            while (i < n && j >= 0) t[p++] = (uint8_t)(i * n + j), ++i, --j;
        }
    }
    if (hipMemcpyToSymbol(HIP_SYMBOL(c_scan16), t16, sizeof(t16)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(c_scan8), t8, sizeof(t8)) != hipSuccess) {
        set_error("so_pack_frames: scan tables: %s", hipGetErrorString(hipGetLastError()));
        return SO_E_INVALID;
    }
    g_scan_ready = true;
    return SO_OK;
}

SO_DEV uint32_t zz(int v) { return ((uint32_t)v << 1) ^ (uint32_t)(v >> 31); }
// LEB128 length: floor(bit_length(z | 1) - 1) / 7) + 1, the division as (x * 37) >> 8 (exact
// for x < 32); no compares, so no VCC round trips per value
SO_DEV int vlen(uint32_t z) { return (((31 - __builtin_clz(z | 1u)) * 37) >> 8) + 1; }

SO_DEV void put_varint(uint8_t* p, int v) {
    uint32_t z = zz(v);
    do {
        *p++ = (uint8_t)(z & 0x7F) | (z > 0x7F ? 0x80 : 0);
        z >>= 7;
    } while (z);
}

// exclusive prefix sum over the wave; *total = the wave's sum
SO_DEV int wave_excl_scan(int x, int lane, int* total) {
    int s = x;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int y = __shfl_up(s, d);
        if (lane >= d) s += y;
    }
    *total = __shfl(s, 63);
    return s - x;
}

struct PackFrame {
    const uint8_t* split;
    const int16_t* mv;
    const int16_t* qtc;
    uint32_t* offs;        // [nb + 1] exclusive offsets (pass 1 writes counts)
    uint8_t* out;          // packed bytes
    int frame_type;
};
constexpr int kPackMax = 32;
struct PackArgs {
    PackFrame f[kPackMax];
};

// One wave per block; lane l owns the R = nn / 64 consecutive scan positions P = R*l + j.
// The block goes through LDS into scan order.  A position starts a run when it opens a
// (sub-)block segment (256 positions unsplit, 4 x 64 split, 64 for 8x8) or its non-zero flag
// differs from the previous position's; a run's length is the distance to the next start
// (inside the lane, else the first start of the next lane that has one: one ballot and one
// bpermute).  A position's bytes are its run token if it starts a run, then its value if
// non-zero; one wave prefix sum over the lanes' byte counts places them after the header
// (split, then the mv values; wave-uniform).  WRITE = false stores the block's byte count.
// A block's inputs, loaded one block ahead (every load of a block is independent of the
// others, so the wave pays one memory latency per block, not a chain of them).
struct PackIn {
    uint2 q;          // this lane's 4 coefficients (row-major)
    int sp;           // split flag
    int hv;           // header value of lane h: split (h = 0) or mv value h - 1
    uint32_t o0, o1;  // offs[b], offs[b + 1] (write pass)
};

template <bool WRITE, int bs>
SO_DEV PackIn pack_load(const PackFrame& f, int b, int nb, int lane) {
    // branch-free (b clamped, every lane loads) so the compiler can wait for exactly these
    // loads one block later instead of draining everything in flight
    b = b < nb ? b : nb - 1;
    constexpr int nn = bs * bs;
    const int nmv = f.frame_type == 1 ? 12 : 4;
    const int qi = lane * 4 < nn ? lane * 4 : 0;
    const int mi = lane >= 1 && lane <= nmv ? lane - 1 : 0;
    // the split byte's address goes through an opaque zero so that the load stays a vector
    // load (a uniform one becomes readfirstlane right after it, i.e. an immediate wait)
    int z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    PackIn in;
    in.q = *reinterpret_cast<const uint2*>(f.qtc + (size_t)b * nn + qi);
    in.sp = f.split[b + z];
    in.hv = f.mv[(size_t)b * nmv + mi];
    in.o0 = WRITE ? f.offs[b] : 0;
    in.o1 = WRITE ? f.offs[b + 1] : 0;
    return in;
}

// One block by one wave; lane l owns the R = nn / 64 consecutive scan positions P = R*l + j.
// The block goes through LDS into scan order.  A position starts a run when it opens a
// (sub-)block segment (256 positions unsplit, 4 x 64 split, 64 for 8x8) or its non-zero flag
// differs from the previous position's; a run's length is the distance to the next start
// (inside the lane, else the first start of the next lane that has one: one ballot and one
// bpermute).  A position's bytes are its run token if it starts a run, then its value if
// non-zero.  The header (split, then the mv values) sits on lanes 0..H-1; one wave prefix sum
// of (header bytes << 16 | token bytes) places both.  WRITE = false stores the byte count.
template <bool WRITE, int bs>
SO_DEV void pack_one_block(const PackFrame& f, int b, unsigned long long cap, int lane, const PackIn& in,
                           int16_t* __restrict__ sq, uint8_t* __restrict__ stage, const int* idx_whole,
                           const int* idx_split) {
    constexpr int nn = bs * bs, R = nn >> 6;
    if (lane * 4 < nn) *reinterpret_cast<uint2*>(&sq[lane * 4]) = in.q;
    const int sp = in.sp;
    const int inter = f.frame_type == 1, H = 1 + (sp ? 4 : 1) * (inter ? 3 : 1);
    const int S = (sp && bs == 16) ? 64 : nn;   // segment length in scan positions
    __builtin_amdgcn_wave_barrier();   // LDS ops of one wave run in order; no fence (it would
                                       // also wait for the next block's loads in flight)

    int v[4];
    unsigned nzb = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        v[j] = 0;
        if (j < R) {
            v[j] = sq[S == 64 && bs == 16 ? idx_split[j] : idx_whole[j]];
            nzb |= (v[j] != 0) << j;
        }
    }
    // run starts: bit j of stb
    const unsigned prev_last = __shfl_up((nzb >> (R - 1)) & 1, 1);
    const unsigned prevb = ((nzb << 1) | (lane > 0 ? prev_last : 0u)) & ((1u << R) - 1);
    unsigned stb = nzb ^ prevb;
    if ((R * lane) % S == 0) stb |= 1u;           // a segment opens at this lane's first position
    const unsigned long long lanes_with_start = __ballot(stb != 0);
    const unsigned long long above = lane == 63 ? 0ull : lanes_with_start & (~0ull << (lane + 1));
    const int nl = above ? __builtin_ctzll(above) : lane;
    const int nfs = __shfl((int)__builtin_ctz(stb | 0x10u), nl);
    const int next_lane_start = above ? R * nl + nfs : nn;

    int tok[4];
    int nbytes = 0;
#pragma unroll
    for (int j = 0; j < R; ++j) {   // branch-free: every position computes its would-be token
        const unsigned later = stb & ~((2u << j) - 1);
        const int nxt = later ? R * lane + __builtin_ctz(later | 0x10u) : next_lane_start;
        const int run = nxt - (R * lane + j);
        const int nzj = (nzb >> j) & 1, stj = (stb >> j) & 1;
        tok[j] = nzj ? -run : ((nxt & (S - 1)) == 0 ? 0 : run);   // a trailing zero run is one 0
        nbytes += (vlen(zz(tok[j])) & -stj) + (vlen(zz(v[j])) & -nzj);
    }
    const int hv = lane == 0 ? sp : in.hv;
    const int hb = lane < H ? vlen(zz(hv)) : 0;
    int tot;
    const int ex = wave_excl_scan((hb << 16) | nbytes, lane, &tot);
    const int hsum = tot >> 16, total = hsum + (tot & 0xFFFF);
    if (!WRITE) {
        if (lane == 0) f.offs[b] = (uint32_t)total;
        return;
    }
    if (in.o1 > cap) return;
    // bytes into the wave's LDS stage, then out with consecutive lanes on consecutive bytes
    if (lane < H) put_varint(stage + (ex >> 16), hv);
    uint8_t* p = stage + hsum + (ex & 0xFFFF);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j >= R) break;
        if ((stb >> j) & 1) {
            put_varint(p, tok[j]);
            p += vlen(zz(tok[j]));
        }
        if (v[j] != 0) {
            put_varint(p, v[j]);
            p += vlen(zz(v[j]));
        }
    }
    __builtin_amdgcn_wave_barrier();
    uint8_t* out = f.out + in.o0;
    for (int i = lane; i < total; i += 64) out[i] = stage[i];
}

// Each wave packs blocks b = wave, wave + nwaves, ... of its frame (blockIdx.y), loading the
// next block's inputs before packing the current one.
template <bool WRITE, int bs>
__global__ void __launch_bounds__(256) pack_block_kernel(const PackArgs a, int nb, unsigned long long cap) {
    __shared__ alignas(16) int16_t sq[4][256];
    __shared__ uint8_t stage[WRITE ? 4 : 1][WRITE ? kPackStage : 1];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int w0 = __builtin_amdgcn_readfirstlane(blockIdx.x * 4 + wv), nw = gridDim.x * 4;
    const PackFrame f = a.f[blockIdx.y];   // a copy: its pointers stay in SGPRs
    // this lane's scan positions as element indices, unsplit and split (4 x 8x8 segments)
    constexpr int R = (bs * bs) >> 6;
    int idx_whole[4], idx_split[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int P = R * lane + j;
        idx_whole[j] = j < R ? (bs == 16 ? c_scan16[P] : c_scan8[P]) : 0;
        idx_split[j] = j < R ? (P & ~63) + c_scan8[P & 63] : 0;
    }
    // two blocks per iteration, each one's inputs loaded one block ahead, in two register sets
    // (a loop-carried copy of a register still being loaded would wait for it)
    PackIn x = pack_load<WRITE, bs>(f, w0, nb, lane);
    for (int b = w0; b < nb; b += 2 * nw) {
        const PackIn y = pack_load<WRITE, bs>(f, b + nw, nb, lane);
        pack_one_block<WRITE, bs>(f, b, cap, lane, x, sq[wv], stage[WRITE ? wv : 0], idx_whole, idx_split);
        if (b + nw >= nb) break;
        x = pack_load<WRITE, bs>(f, b + 2 * nw, nb, lane);
        pack_one_block<WRITE, bs>(f, b + nw, cap, lane, y, sq[wv], stage[WRITE ? wv : 0], idx_whole, idx_split);
    }
}

// exclusive scan of offs[0..nb) in place, total in offs[nb] (and in totals[blockIdx.x] when
// given -- host-mapped memory: a system-scope store): one 1024-thread workgroup per frame,
// the counts in tiles of 8192 -- loaded and stored coalesced (consecutive lanes on
// consecutive counts) through LDS, scanned 8 consecutive counts per thread (one wave scan of
// the threads' sums, one of the 16 wave totals), the tile's total carried into the next.
// Round 6: replaces a chunk-per-thread scan whose lanes read 128 B apart (52 us for a 2-frame
// P-run chunk, on the host-stream region's critical path at its end).
constexpr int kScanTile = 8192;
__global__ void __launch_bounds__(1024) pack_scan_kernel(const PackArgs a, int nb, uint32_t* totals) {
    __shared__ alignas(16) uint32_t tile[kScanTile];
    __shared__ uint32_t wtot[16];
    uint32_t* offs = a.f[blockIdx.x].offs;
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint32_t carry = 0;
    for (int base = 0; base < nb; base += kScanTile) {
        const int n = nb - base < kScanTile ? nb - base : kScanTile;
#pragma unroll
        for (int i = 0; i < kScanTile / 1024; ++i) {
            const int e = t + 1024 * i;
            tile[e] = e < n ? offs[base + e] : 0u;
        }
        __syncthreads();
        const uint4 lo = reinterpret_cast<const uint4*>(tile)[2 * t];
        const uint4 hi = reinterpret_cast<const uint4*>(tile)[2 * t + 1];
        const uint32_t s = lo.x + lo.y + lo.z + lo.w + hi.x + hi.y + hi.z + hi.w;
        int wsum;
        const uint32_t wex = (uint32_t)wave_excl_scan((int)s, lane, &wsum);
        if (lane == 0) wtot[wv] = (uint32_t)wsum;
        __syncthreads();
        uint32_t before = carry, all = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            const uint32_t v = wtot[w];
            before += w < wv ? v : 0u;
            all += v;
        }
        uint32_t r = before + wex;
        uint4 o0, o1;
        o0.x = r; r += lo.x; o0.y = r; r += lo.y; o0.z = r; r += lo.z; o0.w = r; r += lo.w;
        o1.x = r; r += hi.x; o1.y = r; r += hi.y; o1.z = r; r += hi.z; o1.w = r;
        reinterpret_cast<uint4*>(tile)[2 * t] = o0;
        reinterpret_cast<uint4*>(tile)[2 * t + 1] = o1;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kScanTile / 1024; ++i) {
            const int e = t + 1024 * i;
            if (e < n) offs[base + e] = tile[e];
        }
        carry += all;
        __syncthreads();   // the tile and wave totals are reused
    }
    if (t == 0) {
        offs[nb] = carry;
        if (totals) __hip_atomic_store(totals + blockIdx.x, carry, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// ---- unpack (so_unpack_frames): the packed stream back to split / mv / qtc ----------------
// One thread per block parses its bytes [offs[b], offs[b+1]) sequentially: the header, then
// each (sub-)block's tokens -- "-L" and L values, "Z" zeros, "0" the trailing zeros -- into
// the zeroed block in scan order.  Malformed input (a varint or token list running past the
// block's bytes, bytes left over, a run past n*n) sets *err = 1 + that block's index.
struct UnpackFrame {
    const uint8_t* in;
    const uint32_t* offs;
    uint8_t* split;
    int16_t* mv;
    int16_t* qtc;
    int frame_type;
};
struct UnpackArgs {
    UnpackFrame f[kPackMax];
};

template <int BS>
__global__ void __launch_bounds__(256) unpack_block_kernel(const UnpackArgs a, int nb, int32_t* __restrict__ err) {
    const int b = blockIdx.x * 256 + threadIdx.x;
    if (b >= nb) return;
    const UnpackFrame& f = a.f[blockIdx.y];
    const uint8_t* p = f.in + f.offs[b];
    const uint8_t* const end = f.in + f.offs[b + 1];
    bool bad = f.offs[b + 1] < f.offs[b];
    auto next = [&]() -> int {
        uint32_t z = 0;
        for (int sh = 0; sh < 35; sh += 7) {
            if (p >= end) break;
            const uint32_t c = *p++;
            z |= (c & 0x7Fu) << sh;
            if (!(c & 0x80u)) return (int)(z >> 1) ^ -(int)(z & 1u);
        }
        bad = true;
        return 0;
    };
    constexpr int NN = BS * BS;
    int16_t* q = f.qtc + (size_t)b * NN;
#pragma unroll
    for (int i = 0; i < NN / 8; ++i) reinterpret_cast<uint4*>(q)[i] = make_uint4(0, 0, 0, 0);
    const int sp = bad ? 0 : next();
    if (sp != 0 && (sp != 1 || BS != 16)) bad = true;
    f.split[b] = (uint8_t)(sp == 1 && !bad);
    const int inter = f.frame_type == 1, nmv = (sp == 1) ? 4 : 1;
    if (inter) {
        int16_t* m = f.mv + (size_t)b * 12;
        for (int j = 0; j < 12; ++j) m[j] = (int16_t)(j < 3 * nmv && !bad ? next() : 0);
    } else {
        int16_t* m = f.mv + (size_t)b * 4;
        for (int j = 0; j < 4; ++j) m[j] = (int16_t)(j < nmv && !bad ? next() : 0);
    }
    const int nsub = sp == 1 ? 4 : 1, n = sp == 1 ? 8 : BS, nn = n * n;
    const uint8_t* scan = n == 16 ? c_scan16 : c_scan8;
    for (int j = 0; j < nsub && !bad; ++j) {
        int16_t* qs = q + j * nn;
        int k = 0;
        while (k < nn && !bad) {
            const int t = next();
            if (t < 0) {
                if (-t > nn - k) { bad = true; break; }
                for (int i = 0; i < -t && !bad; ++i) qs[scan[k + i]] = (int16_t)next();
                k -= t;
            } else if (t == 0) {
                break;
            } else {
                if (t > nn - k) { bad = true; break; }
                k += t;
            }
        }
    }
    if (p != end) bad = true;
    if (bad) __hip_atomic_store(err, b + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

int unpack_frames_launch(const UnpackFrame* frames, int nframes, int nb, int bs, int32_t* err, hipStream_t st) {
    const int trc = init_scan_tables();
    if (trc != SO_OK) return trc;
    for (int f0 = 0; f0 < nframes; f0 += kPackMax) {
        const int n = nframes - f0 < kPackMax ? nframes - f0 : kPackMax;
        UnpackArgs a{};
        for (int i = 0; i < n; ++i) a.f[i] = frames[f0 + i];
        const dim3 grid((nb + 255) / 256, n);
        if (bs == 16) hipLaunchKernelGGL(unpack_block_kernel<16>, grid, dim3(256), 0, st, a, nb, err);
        else hipLaunchKernelGGL(unpack_block_kernel<8>, grid, dim3(256), 0, st, a, nb, err);
        const int rc = check_launch("unpack_block_kernel");
        if (rc != SO_OK) return rc;
    }
    return SO_OK;
}

int pack_frames_launch(const PackFrame* frames, int nframes, int nb, int bs, unsigned long long cap, uint32_t* totals,
                       hipStream_t st) {
    const int trc = init_scan_tables();
    if (trc != SO_OK) return trc;
    for (int f0 = 0; f0 < nframes; f0 += kPackMax) {
        const int n = nframes - f0 < kPackMax ? nframes - f0 : kPackMax;
        PackArgs a{};
        for (int i = 0; i < n; ++i) a.f[i] = frames[f0 + i];
        const int per_wave = 8;
        const dim3 grid((nb + 4 * per_wave - 1) / (4 * per_wave), n);
        if (bs == 16) hipLaunchKernelGGL((pack_block_kernel<false, 16>), grid, dim3(256), 0, st, a, nb, cap);
        else hipLaunchKernelGGL((pack_block_kernel<false, 8>), grid, dim3(256), 0, st, a, nb, cap);
        hipLaunchKernelGGL(pack_scan_kernel, dim3(n), dim3(1024), 0, st, a, nb, totals ? totals + f0 : nullptr);
        if (bs == 16) hipLaunchKernelGGL((pack_block_kernel<true, 16>), grid, dim3(256), 0, st, a, nb, cap);
        else hipLaunchKernelGGL((pack_block_kernel<true, 8>), grid, dim3(256), 0, st, a, nb, cap);
        const int rc = check_launch("pack kernels");
        if (rc != SO_OK) return rc;
    }
    return SO_OK;
}

}  // namespace so
