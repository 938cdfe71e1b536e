// so_capi.hip — the extern "C" boundary of libstreamoptima_hip.so (include/streamoptima.h).
// Argument validation, thread-local error text, launches; no device allocation, no host
// synchronisation (every entry point is capturable into a hipGraph).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <vector>

#include <hip/hip_ext.h>

#include "so_common.h"
#include "so_run.h"

namespace so {

static thread_local char g_err[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

// so_set_option / so_get_option (SO_OPT_*): index = option id
static std::atomic<int> g_opt[8] = {0, 1, 0, 32, 32, 0, 0, 0};   // SO_OPT_RUN_2PASS_FUSED on by default

int option(int id) {
    return (id > 0 && id < 8) ? g_opt[id].load(std::memory_order_relaxed) : 0;
}

int me_launch(const uint8_t* cur, const RefSet& refs, int nref, int H, int W, int bs, int sr, int by0, int by1,
              int32_t* out_best, int32_t* out_sub, hipStream_t st);
int me_generic_launch(const uint8_t* cur, const RefSet& refs, const uint8_t* planes, size_t pstride, int nref, int H,
                      int W, int bs, int sr, int by0, int by1, int32_t* out_best, int32_t* out_sub, hipStream_t st);
int me_fme_launch(const uint8_t* cur, const uint8_t* planes, size_t pstride, int nref, int H, int W, int by0, int by1,
                  int32_t* out_best, int32_t* out_sub, hipStream_t st);
int fme_planes_launch(const uint8_t* ref, int H, int W, int wrap, uint8_t* out, size_t pstride, hipStream_t st);
int me_fastpred_launch(const uint8_t* cur, const uint8_t* const* ptrs, int nptr, int nref, int H, int W, int bs,
                       int fme, int by0, int by1, int serial, int32_t* out_best, int32_t* out_sub, int32_t* seg_ws,
                       hipStream_t st);
constexpr size_t kFastSegWords = 2 * 4096 * 6;   // so_fastme.hip: the speculated chain's segment records
int p_tile_launch(const uint8_t* cur, const RefSet& refs, int H, int W, int by0, int by1, int qp_rd,
                  const int32_t* qp_row, const int32_t* qp_map, int32_t* out_best, uint8_t* out_split,
                  int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae, uint8_t* out_recon,
                  int32_t* out_sse, hipStream_t st, bool tokens_only = false, const int16_t* prev_mv = nullptr);

struct PackFrame {
    const uint8_t* split;
    const int16_t* mv;
    const int16_t* qtc;
    uint32_t* offs;
    uint8_t* out;
    int frame_type;
};
size_t pack_block_bound(int bs);
struct UnpackFrame {
    const uint8_t* in;
    const uint32_t* offs;
    uint8_t* split;
    int16_t* mv;
    int16_t* qtc;
    int frame_type;
};
int unpack_frames_launch(const UnpackFrame* frames, int nframes, int nb, int bs, int32_t* err, hipStream_t st);
int pack_frames_launch(const PackFrame* frames, int nframes, int nb, int bs, unsigned long long cap, uint32_t* totals,
                       hipStream_t st);
int stripe_halo_push_launch(const uint8_t* plane, int W, int by0, int by1, uint8_t* up, uint8_t* dn,
                            uint32_t* up_flags, uint32_t* dn_flags, int gf, uint32_t epoch, hipStream_t st);
int frame_push_launch(const uint8_t* plane, int H, int W, uint8_t* dst, uint32_t* flags, uint32_t epoch,
                      hipStream_t st);

#ifdef SO_AB
// A/B builds only (not in the header): tools that set the SO_AB environment knobs
// (tools/ab_guard.py) check for this symbol, so a knob can never silently measure the default path
extern "C" int so_debug_ab_build(void) { return 1; }
#endif

// The fused search + transform tile kernel (so_me.hip p_tile_kernel) covers the headline
// configuration: bs 16, sr 16, full search, no VBS / FME, one reference.  SO_FUSED=0 or an
// SO_ME_IMPL A/B selection keeps the two-launch path (ME kernel + inter_tq_kernel).
static bool use_fused(int bs, int sr, int vbs, int nref) {
    if (bs != 16 || sr != 16 || vbs || nref != 1) return false;
#ifdef SO_AB   // A/B builds only
    const char* f = getenv("SO_FUSED");
    if (f && strcmp(f, "0") == 0) return false;
    const char* impl = getenv("SO_ME_IMPL");
    return impl == nullptr || impl[0] == 0;
#else
    return true;
#endif
}

int inter_tq_launch(const uint8_t* cur, const RefSet& refs, const uint8_t* planes, size_t pstride, int H, int W,
                    int bs, int by0, int by1, const int32_t* best, const int32_t* sub, int qp_rd, const int32_t* qp_row,
                    const int32_t* qp_map, int vbs, double lam, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens,
                    int32_t* out_mae, uint8_t* out_recon, int32_t* out_sse, hipStream_t st);
int inter_tq_2pass_launch(const uint8_t* cur, const RefSet& refs, int H, int W, const int32_t* best, const int32_t* t1,
                          int qp_rd, const int32_t* qp_row, const int32_t* roi, int qp_lo, int qp_hi,
                          int32_t* out_qpmap, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc,
                          int32_t* out_tokens, int32_t* out_mae, uint8_t* out_recon, int32_t* out_sse,
                          hipStream_t st);
int inter_recon_launch(const RefSet& refs, const uint8_t* planes, size_t pstride, int H, int W, int bs, int qp,
                       const int32_t* qp_row, const int32_t* qp_map, const uint8_t* split, const int16_t* mv, const int16_t* qtc,
                       uint8_t* out_recon, hipStream_t st);
int intra_encode_launch(const uint8_t* cur, int H, int W, int bs, int sr, int by0, int by1, int qp_rd,
                        const int32_t* qp_row, const int32_t* qp_map, int vbs, double lam, uint8_t* out_split, int16_t* out_mv,
                        int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae, uint8_t* out_recon,
                        int32_t* out_sse, uint8_t* idres, hipStream_t st);
int intra_recon_launch(int H, int W, int bs, int sr, int qp, const int32_t* qp_row, const int32_t* qp_map,
                       const uint8_t* split,
                       const int16_t* mv, const int16_t* qtc, uint8_t* out_recon, uint8_t* idres,
                       hipStream_t st);

// ---- validation ------------------------------------------------------------------------------
// VBSEnable flag and calculate_RD_cost's lambda (Encoder.py:1133-1158)
static int check_vbs(const char* fn, int vbs, double lam) {
    if (vbs != 0 && vbs != 1) {
        set_error("%s: vbs must be 0 or 1", fn);
        return SO_E_INVALID;
    }
    if (vbs && !(lam >= 0.0 && lam < 1e300)) {
        set_error("%s: lambda %g (VBSEnable needs a finite lambda >= 0)", fn, lam);
        return SO_E_INVALID;
    }
    return SO_OK;
}

static int check_geom(const char* fn, int H, int W, int bs, int vbs) {
    if (bs != 16 && bs != 8) {
        set_error("%s: block_size %d not built (gfx950 kernels exist for 16 and 8)", fn, bs);
        return SO_E_UNSUPPORTED;
    }
    if (vbs && bs != 16) {
        set_error("%s: VBSEnable needs block_size 16 (8x8 sub-blocks)", fn);
        return SO_E_UNSUPPORTED;
    }
    if (H <= 0 || W <= 0 || H % bs || W % bs) {
        set_error("%s: frame %dx%d must be a positive multiple of block_size %d (pad with pad_hw)", fn, W, H, bs);
        return SO_E_INVALID;
    }
    if ((long long)H * W > (1ll << 31)) {
        set_error("%s: frame too large", fn);
        return SO_E_INVALID;
    }
    return SO_OK;
}

static int check_sr(const char* fn, int sr) {
    if (sr < 0 || sr > 64) {
        set_error("%s: search_range %d outside [0, 64]", fn, sr);
        return SO_E_UNSUPPORTED;
    }
    return SO_OK;
}

static int check_intra_width(const char* fn, int W) {
    if (W > 8192) {   // intra_recon_kernel keeps one pixel row (12 B/px) in LDS
        set_error("%s: intra frames wider than 8192 px are not built", fn);
        return SO_E_UNSUPPORTED;
    }
    return SO_OK;
}

static int check_rows(const char* fn, int H, int bs, int by0, int by1) {
    if (by0 < 0 || by1 < by0 || by1 > H / bs) {
        set_error("%s: block-row range [%d, %d) outside [0, %d]", fn, by0, by1, H / bs);
        return SO_E_INVALID;
    }
    return SO_OK;
}

static int check_qp(const char* fn, int qp) {
    if (qp < 0 || qp > 20) {
        set_error("%s: Qp %d outside [0, 20]", fn, qp);
        return SO_E_INVALID;
    }
    return SO_OK;
}

static int make_refs(const char* fn, const uint8_t* const* refs, int nref, RefSet* rs) {
    if (refs == nullptr || nref < 1 || nref > kMaxRef) {
        set_error("%s: nref %d outside [1, %d]", fn, nref, kMaxRef);
        return SO_E_INVALID;
    }
    for (int i = 0; i < kMaxRef; ++i) rs->p[i] = i < nref ? refs[i] : refs[0];
    for (int i = 0; i < nref; ++i)
        if (!refs[i]) {
            set_error("%s: refs[%d] is NULL", fn, i);
            return SO_E_INVALID;
        }
    return SO_OK;
}

#define SO_TRY(x)                 \
    do {                          \
        int _rc = (x);            \
        if (_rc != SO_OK) return _rc; \
    } while (0)

#define SO_NEED(p, fn)                                  \
    do {                                                \
        if (!(p)) {                                     \
            set_error("%s: %s is NULL", fn, #p);        \
            return SO_E_INVALID;                        \
        }                                               \
    } while (0)

// ---- per-frame sums of the encode kernels' per-block / per-row SSE ---------------------------
constexpr int kSumMax = 64;
struct SumArgs {
    const int32_t* p[kSumMax];
};

// one workgroup of 1024 threads per array: int64 sum of len int32 values into out[blockIdx.x];
// 16-byte loads, eight in flight per thread (a 4K frame's 32,400 per-block values are ~130 KB:
// 256 threads left it latency-bound at 10 us for 30 frames)
constexpr int kSumThreads = 1024;
__global__ void __launch_bounds__(kSumThreads) sum_rows_kernel(const SumArgs a, int len, long long* __restrict__ out) {
    __shared__ long long part[kSumThreads / 64];
    const int32_t* p = a.p[blockIdx.x];
    long long acc = 0;
    const int n4 = (reinterpret_cast<uintptr_t>(p) & 15) ? 0 : len / 4;
    const int4* p4 = reinterpret_cast<const int4*>(p);
    int i = threadIdx.x;
    // guarded loads, all eight issued before the adds (a separate remainder loop ran its loads
    // one round trip at a time: 8 us for a 4K GOP's 30 frames)
    for (; i < n4; i += 8 * kSumThreads) {
        int4 v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = i + k * kSumThreads < n4 ? p4[i + k * kSumThreads] : make_int4(0, 0, 0, 0);
#pragma unroll
        for (int k = 0; k < 8; ++k) acc += (long long)v[k].x + v[k].y + v[k].z + v[k].w;
    }
    for (int j = 4 * n4 + threadIdx.x; j < len; j += kSumThreads) acc += p[j];
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) {
        long long t = 0;
#pragma unroll
        for (int w = 0; w < kSumThreads / 64; ++w) t += part[w];
        out[blockIdx.x] = t;
    }
}

// ---- SSE (PSNR) -------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) sse_kernel(const uint8_t* __restrict__ a, const uint8_t* __restrict__ b,
                                                  int64_t n, unsigned long long* __restrict__ out) {
    __shared__ unsigned long long part[4];
    unsigned long long acc = 0;
    const int64_t n16 = n / 16;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
        const uint4 va = reinterpret_cast<const uint4*>(a)[i];
        const uint4 vb = reinterpret_cast<const uint4*>(b)[i];
        const uint32_t wa[4] = {va.x, va.y, va.z, va.w}, wb[4] = {vb.x, vb.y, vb.z, vb.w};
        uint32_t s = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                const int d = (int)((wa[k] >> (8 * e)) & 255) - (int)((wb[k] >> (8 * e)) & 255);
                s += (uint32_t)(d * d);
            }
        acc += s;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int64_t i = n16 * 16; i < n; ++i) {
            const int d = (int)a[i] - (int)b[i];
            acc += (unsigned long long)(d * d);
        }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(out, part[0] + part[1] + part[2] + part[3]);
}

// Per-block QP map (build extension, DESIGN.md "ROI and two-pass rate control"): one
// workgroup per block row.  Two-pass: with pass-1 token counts t (stripe-local records) the
// row mean is m / n (m = sum, n = blocks per row) and
//   delta = [t n >= 2m] + [t n >= 4m] - [2 t n < m] - [4 t n < m]      (in [-2, 2], exact)
// i.e. blocks at >= 2x / 4x the row's mean bits are quantised 1 / 2 QP coarser and blocks at
// < 1/2 / < 1/4 of it 1 / 2 QP finer.  qp = clamp(base + delta + roi, qp_lo, qp_hi) with
// base = qp_row[by] (rate-control schedule) or qp_rd.  tokens == NULL: ROI only (delta 0).
__global__ void __launch_bounds__(256)
qp_map_kernel(const int32_t* __restrict__ tokens, int nbx, int by0, int qp_rd, const int32_t* __restrict__ qp_row,
              const int32_t* __restrict__ roi, int qp_lo, int qp_hi, int32_t* __restrict__ out) {
    __shared__ long long part[4];
    const int by = by0 + blockIdx.x;
    const int32_t* t = tokens ? tokens + (size_t)blockIdx.x * nbx : nullptr;
    long long m = 0;
    if (t) {
        for (int bx = threadIdx.x; bx < nbx; bx += blockDim.x) m += t[bx];
#pragma unroll
        for (int s = 32; s >= 1; s >>= 1) m += __shfl_xor(m, s, 64);
        if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = m;
        __syncthreads();
        m = part[0] + part[1] + part[2] + part[3];
    }
    const int base = qp_row ? qp_row[by] : qp_rd;
    for (int bx = threadIdx.x; bx < nbx; bx += blockDim.x) {
        int d = 0;
        if (t) {
            const long long tn = (long long)t[bx] * nbx;
            d = (tn >= 2 * m) + (tn >= 4 * m) - (2 * tn < m) - (4 * tn < m);
        }
        int q = base + d + (roi ? roi[(size_t)by * nbx + bx] : 0);
        q = q < qp_lo ? qp_lo : (q > qp_hi ? qp_hi : q);
        out[(size_t)by * nbx + bx] = q;
    }
}

}  // namespace so

using namespace so;

extern "C" {

int so_abi_version(void) { return SO_ABI_VERSION; }

int so_set_option(int opt, int value) {
    const bool ok = (opt == SO_OPT_RUN_2PASS_FUSED || opt == SO_OPT_FASTME_SERIAL || opt == SO_OPT_COUNT_SAD_OPS ||
                     opt == SO_OPT_RUN_ZERO_SKIP)
                        ? (value == 0 || value == 1)
                    : opt == SO_OPT_FASTME_SEGMENT                               ? value >= 1
                    : opt == SO_OPT_FASTME_WARMUP || opt == SO_OPT_TEST_LOSE_FLAG ? value >= 0
                                                                                 : false;
    if (!ok) {
        set_error("so_set_option: option %d value %d is unknown or out of range", opt, value);
        return SO_E_INVALID;
    }
    g_opt[opt].store(value, std::memory_order_relaxed);
    return SO_OK;
}

int so_get_option(int opt) { return option(opt); }

const char* so_last_error(void) { return g_err; }

int so_me_full_search(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W, int bs,
                      int sr, int32_t* out_best, int32_t* out_sub, void* stream) {
    const char* fn = "so_me_full_search";
    SO_TRY(check_geom(fn, H, W, bs, out_sub != nullptr));
    SO_TRY(check_sr(fn, sr));
    SO_NEED(cur, fn);
    SO_NEED(out_best, fn);
    RefSet rs;
    SO_TRY(make_refs(fn, refs, nref, &rs));
    return me_launch(cur, rs, nref, H, W, bs, sr, 0, H / bs, out_best, out_sub, (hipStream_t)stream);
}

int so_inter_tq_recon(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W, int bs,
                      const int32_t* best, const int32_t* sub, int qp_rd, const int32_t* qp_row, int vbs,
                      double lam, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens,
                      int32_t* out_mae_num, uint8_t* out_recon, int32_t* out_sse, void* stream) {
    const char* fn = "so_inter_tq_recon";
    SO_TRY(check_geom(fn, H, W, bs, vbs));
    SO_TRY(check_qp(fn, qp_rd));
    SO_NEED(cur, fn); SO_NEED(best, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn);
    SO_NEED(out_qtc, fn); SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn);
    if (vbs) SO_NEED(sub, fn);
    RefSet rs;
    SO_TRY(make_refs(fn, refs, nref, &rs));
    for (int i = 0; i < nref; ++i)
        if (refs[i] == out_recon) {
            set_error("%s: out_recon aliases refs[%d]", fn, i);
            return SO_E_INVALID;
        }
    return inter_tq_launch(cur, rs, nullptr, 0, H, W, bs, 0, H / bs, best, vbs ? sub : nullptr, qp_rd, qp_row, nullptr, vbs, lam,
                           out_split, out_mv, out_qtc, out_tokens, out_mae_num, out_recon, out_sse,
                           (hipStream_t)stream);
}

size_t so_p_frame_scratch_elems(int H, int W, int bs, int vbs) {
    if (bs <= 0) return 0;
    const size_t nb = (size_t)(W / bs) * (size_t)(H / bs);
    return nb * 4 + (vbs ? nb * 16 : 0) + kFastSegWords;
}

int so_encode_p_rows(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W, int bs, int sr,
                     int by0, int by1, int qp_rd, const int32_t* qp_row, int vbs, double lam, uint8_t* out_split,
                     int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae_num,
                     uint8_t* out_recon, int32_t* out_sse, int32_t* scratch, void* stream) {
    const char* fn = "so_encode_p_rows";
    SO_TRY(check_geom(fn, H, W, bs, vbs));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    SO_TRY(check_rows(fn, H, bs, by0, by1));
    SO_NEED(cur, fn); SO_NEED(scratch, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn);
    SO_NEED(out_qtc, fn); SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn);
    RefSet rs;
    SO_TRY(make_refs(fn, refs, nref, &rs));
    for (int i = 0; i < nref; ++i)
        if (refs[i] == out_recon) {
            set_error("%s: out_recon aliases refs[%d]", fn, i);
            return SO_E_INVALID;
        }
    const size_t nbs = (size_t)(W / bs) * (size_t)(by1 - by0);
    int32_t* best = scratch;
    int32_t* sub = vbs ? scratch + nbs * 4 : nullptr;
    hipStream_t st = (hipStream_t)stream;
    if (use_fused(bs, sr, vbs, nref))
        return p_tile_launch(cur, rs, H, W, by0, by1, qp_rd, qp_row, nullptr, best, out_split, out_mv, out_qtc,
                             out_tokens, out_mae_num, out_recon, out_sse, st);
    SO_TRY(me_launch(cur, rs, nref, H, W, bs, sr, by0, by1, best, sub, st));
    return inter_tq_launch(cur, rs, nullptr, 0, H, W, bs, by0, by1, best, sub, qp_rd, qp_row, nullptr, vbs, lam, out_split,
                           out_mv, out_qtc, out_tokens, out_mae_num, out_recon, out_sse, st);
}

int so_encode_p_frame(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W, int bs, int sr,
                      int qp_rd, const int32_t* qp_row, int vbs, double lam, uint8_t* out_split,
                      int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae_num,
                      uint8_t* out_recon, int32_t* out_sse, int32_t* scratch, void* stream) {
    if (bs <= 0) {
        set_error("so_encode_p_frame: block_size %d", bs);
        return SO_E_UNSUPPORTED;
    }
    return so_encode_p_rows(cur, refs, nref, H, W, bs, sr, 0, H / bs, qp_rd, qp_row, vbs, lam, out_split, out_mv,
                            out_qtc, out_tokens, out_mae_num, out_recon, out_sse, scratch, stream);
}

// ---- P-frame runs: one persistent launch (so_me.hip p_run_kernel) -----------------------
size_t so_p_run_workspace_elems(int H, int W) {
    if (H <= 0 || W <= 0) return 0;
    return p_run_workspace_words(H, W);
}

int so_p_run_resident_workgroups(int vbs) {
    const int n = p_run_capacity(vbs ? 1 : 0);
    if (n <= 0) {
        set_error("so_p_run_resident_workgroups: device query failed");
        return SO_E_INVALID;
    }
    return n;
}

int so_p_run_2pass_fused(int H, int W) {
    return H > 0 && W > 0 && option(SO_OPT_RUN_2PASS_FUSED) == 1 && p_run_2pass_fused_ok(H, W) ? 1 : 0;
}

int so_p_run_mode_resident_workgroups(int mode, int vbs) {
    if (mode < 0 || mode > 4 || (vbs && mode != 0 && mode != 2)) {
        set_error("so_p_run_mode_resident_workgroups: mode %d%s", mode, vbs ? " with vbs (modes 0, 2)" : " (0..4)");
        return SO_E_INVALID;
    }
    const int n = p_run_capacity(vbs ? 1 : 0, mode);
    if (n <= 0) {
        set_error("so_p_run_mode_resident_workgroups: device query failed");
        return SO_E_INVALID;
    }
    return n;
}

int so_encode_p_run(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int bs, int sr,
                    int qp_rd, const int32_t* qp_row, int vbs, double lam, uint8_t* const* out_split,
                    int16_t* const* out_mv, int16_t* const* out_qtc, int32_t* const* out_tokens,
                    int32_t* const* out_mae_num, uint8_t* const* out_recon, int32_t* const* out_sse,
                    uint32_t* workspace, void* stream) {
    const char* fn = "so_encode_p_run";
    SO_TRY(check_geom(fn, H, W, bs, vbs));
    SO_TRY(check_vbs(fn, vbs, lam));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    if (bs != 16 || sr != 16 || W % 128 != 0) {
        set_error("%s: covers bs 16 / sr 16 / W %% 128 == 0 (call so_encode_p_frame per frame)", fn);
        return SO_E_UNSUPPORTED;
    }
    if (nframes <= 0) return SO_OK;
    SO_NEED(curs, fn); SO_NEED(ref0, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn); SO_NEED(out_qtc, fn);
    SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn); SO_NEED(workspace, fn);
    std::vector<PFrameOut> outs((size_t)nframes);
    for (int i = 0; i < nframes; ++i) {
        SO_NEED(curs[i], fn); SO_NEED(out_split[i], fn); SO_NEED(out_mv[i], fn); SO_NEED(out_qtc[i], fn);
        SO_NEED(out_tokens[i], fn); SO_NEED(out_mae_num[i], fn); SO_NEED(out_recon[i], fn);
        for (int j = -1; j < i; ++j)
            if (out_recon[i] == (j < 0 ? ref0 : out_recon[j])) {
                set_error("%s: out_recon[%d] aliases ref0 or another frame's reconstruction", fn, i);
                return SO_E_INVALID;
            }
        outs[i] = PFrameOut{out_split[i], out_mv[i], out_qtc[i], out_tokens[i], out_mae_num[i], out_recon[i],
                            out_sse ? out_sse[i] : nullptr};
    }
    return p_run_launch(curs, nframes, ref0, H, W, qp_rd, qp_row, vbs, lam, outs.data(), workspace,
                        (hipStream_t)stream);
}

int so_encode_p_runs(const uint8_t* const* curs, int nframes, const uint8_t* const* refs, const int32_t* ref_frame,
                     int H, int W, int bs, int sr, int qp_rd, const int32_t* qp_row, int vbs, double lam,
                     uint8_t* const* out_split, int16_t* const* out_mv, int16_t* const* out_qtc,
                     int32_t* const* out_tokens, int32_t* const* out_mae_num, uint8_t* const* out_recon,
                     int32_t* const* out_sse, uint32_t* workspace, void* stream) {
    const char* fn = "so_encode_p_runs";
    SO_TRY(check_geom(fn, H, W, bs, vbs));
    SO_TRY(check_vbs(fn, vbs, lam));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    if (bs != 16 || sr != 16 || W % 128 != 0) {
        set_error("%s: covers bs 16 / sr 16 / W %% 128 == 0 (call so_encode_p_frame per frame)", fn);
        return SO_E_UNSUPPORTED;
    }
    if (nframes <= 0) return SO_OK;
    SO_NEED(curs, fn); SO_NEED(refs, fn); SO_NEED(ref_frame, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn);
    SO_NEED(out_qtc, fn); SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn);
    SO_NEED(workspace, fn);
    std::vector<PFrameOut> outs((size_t)nframes);
    std::vector<int> deps((size_t)nframes);
    int conc = 0;   // runs starting from a plane outside the list: interleaved chains
    for (int i = 0; i < nframes; ++i) {
        SO_NEED(curs[i], fn); SO_NEED(out_split[i], fn); SO_NEED(out_mv[i], fn); SO_NEED(out_qtc[i], fn);
        SO_NEED(out_tokens[i], fn); SO_NEED(out_mae_num[i], fn); SO_NEED(out_recon[i], fn);
        const int d = ref_frame[i];
        if (d >= i || d < -1) {
            set_error("%s: ref_frame[%d] = %d (must be -1 or an earlier frame of the list)", fn, i, d);
            return SO_E_INVALID;
        }
        if (d < 0) {
            SO_NEED(refs[i], fn);
            ++conc;
        }
        deps[(size_t)i] = d;
        for (int j = 0; j < nframes; ++j)
            if ((j != i && out_recon[i] == out_recon[j]) || (ref_frame[j] < 0 && out_recon[i] == refs[j])) {
                set_error("%s: out_recon[%d] aliases a reference plane or another frame's reconstruction", fn, i);
                return SO_E_INVALID;
            }
        outs[(size_t)i] = PFrameOut{out_split[i], out_mv[i], out_qtc[i], out_tokens[i], out_mae_num[i], out_recon[i],
                                    out_sse ? out_sse[i] : nullptr};
    }
    return p_runs_launch(curs, nframes, refs, deps.data(), conc, H, W, qp_rd, qp_row, vbs, lam, outs.data(), workspace,
                         (hipStream_t)stream);
}

int so_encode_p_run_2pass(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int bs, int sr,
                          int qp_rd, const int32_t* qp_row, const int32_t* roi, int qp_lo, int qp_hi,
                          uint8_t* const* out_split, int16_t* const* out_mv, int16_t* const* out_qtc,
                          int32_t* const* out_tokens, int32_t* const* out_mae_num, uint8_t* const* out_recon,
                          int32_t* const* out_sse, int32_t* const* out_qp_map, uint32_t* workspace, void* stream) {
    const char* fn = "so_encode_p_run_2pass";
    SO_TRY(check_geom(fn, H, W, bs, 0));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    if (bs != 16 || sr != 16 || W % 128 != 0 || W > 8192) {
        set_error("%s: covers bs 16 / sr 16 / W %% 128 == 0, W <= 8192 (encode per frame otherwise)", fn);
        return SO_E_UNSUPPORTED;
    }
    if (qp_lo < 0 || qp_hi > 20 || qp_lo > qp_hi) {
        set_error("%s: QP clamp [%d, %d] outside [0, 20]", fn, qp_lo, qp_hi);
        return SO_E_INVALID;
    }
    if (nframes <= 0) return SO_OK;
    SO_NEED(curs, fn); SO_NEED(ref0, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn); SO_NEED(out_qtc, fn);
    SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn); SO_NEED(out_qp_map, fn);
    SO_NEED(workspace, fn);
    std::vector<PFrameOut> outs((size_t)nframes);
    for (int i = 0; i < nframes; ++i) {
        SO_NEED(curs[i], fn); SO_NEED(out_split[i], fn); SO_NEED(out_mv[i], fn); SO_NEED(out_qtc[i], fn);
        SO_NEED(out_tokens[i], fn); SO_NEED(out_mae_num[i], fn); SO_NEED(out_recon[i], fn); SO_NEED(out_qp_map[i], fn);
        for (int j = -1; j < i; ++j)
            if (out_recon[i] == (j < 0 ? ref0 : out_recon[j])) {
                set_error("%s: out_recon[%d] aliases ref0 or another frame's reconstruction", fn, i);
                return SO_E_INVALID;
            }
        outs[(size_t)i] = PFrameOut{out_split[i], out_mv[i], out_qtc[i], out_tokens[i], out_mae_num[i], out_recon[i],
                                    out_sse ? out_sse[i] : nullptr, out_qp_map[i]};
    }
    hipStream_t st = (hipStream_t)stream;
    // default: both passes of every frame in one persistent launch (each task the pass 2 of one
    // tile and the pass 1 of another), for frames of three tile rows or
    // more; otherwise, or with SO_OPT_RUN_2PASS_FUSED = 0, the per-frame sequence below
    if (so_p_run_2pass_fused(H, W))
        return p_run_2pass_launch(curs, nframes, ref0, H, W, qp_rd, qp_row, roi, qp_lo, qp_hi, outs.data(), workspace,
                                  st);
    // per frame, pass 1 (fused search + tokens only) and pass 2 (the QP map from pass 1's token
    // counts, then the transforms on pass 1's ME records, kept in the workspace), enqueued from
    // here with no host round trip per frame
    // the workspace's pass-1 region (kRunMax >= 5 blocks' words per block): the ME records
    // (4 words per block), then the pass-1 token counts (1 word per block)
    int32_t* best = p_run_t1_region(workspace, H, W);
    const int nbx = W / 16, nby = H / 16;
    int32_t* t1 = best + (size_t)4 * nbx * nby;
    static_assert(kRunMax >= 5, "the pass-1 region holds 4 + 1 words per block");
    for (int i = 0; i < nframes; ++i) {
        RefSet rs{};
        rs.p[0] = i ? out_recon[i - 1] : ref0;
        const PFrameOut& o = outs[(size_t)i];
        // pass 1 with the previous frame's (final) motion records as the search's U hint
        SO_TRY(p_tile_launch(curs[i], rs, H, W, 0, nby, qp_rd, qp_row, nullptr, best, o.split, o.mv, o.qtc, t1,
                             o.mae, o.recon, o.sse, st, true, i ? out_mv[i - 1] : nullptr));
        // pass 2 derives the QP map from the pass-1 tokens itself (qp_map_kernel's rule) and
        // stores it: no separate QP-map launch per frame
        SO_TRY(inter_tq_2pass_launch(curs[i], rs, H, W, best, t1, qp_rd, qp_row, roi, qp_lo, qp_hi, o.qpmap, o.split,
                                     o.mv, o.qtc, o.tokens, o.mae, o.recon, o.sse, st));
    }
    return SO_OK;
}

// ---- one GOP across GPUs: a rank's stripe of every frame (so_me.hip PRunStripe) -------------
int so_encode_p_run_stripe(const uint8_t* const* curs, int nframes, const uint8_t* ref0, int H, int W, int bs, int sr,
                           int by0, int by1, int qp_rd, const int32_t* qp_row, uint8_t* const* out_split,
                           int16_t* const* out_mv, int16_t* const* out_qtc, int32_t* const* out_tokens,
                           int32_t* const* out_mae_num, uint8_t* const* out_recon, int32_t* const* out_sse,
                           uint32_t* workspace, int gbase, uint8_t* peer_up0, uint8_t* peer_dn0, long long stride,
                           const uint32_t* my_up_flags, const uint32_t* my_dn_flags, uint32_t* peer_up_flags,
                           uint32_t* peer_dn_flags, uint32_t epoch, int max_wg, void* stream) {
    const char* fn = "so_encode_p_run_stripe";
    SO_TRY(check_geom(fn, H, W, bs, 0));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    if (bs != 16 || sr != 16 || W % 128 != 0) {
        set_error("%s: covers bs 16 / sr 16 / W %% 128 == 0", fn);
        return SO_E_UNSUPPORTED;
    }
    if (by0 < 0 || by1 > H / 16 || by1 <= by0 || gbase < 1) {
        set_error("%s: bad stripe [%d, %d) of %d block rows or gbase %d", fn, by0, by1, H / 16, gbase);
        return SO_E_INVALID;
    }
    if ((peer_up0 != nullptr) != (peer_up_flags != nullptr) || (peer_dn0 != nullptr) != (peer_dn_flags != nullptr) ||
        (peer_up0 != nullptr) != (my_up_flags != nullptr) || (peer_dn0 != nullptr) != (my_dn_flags != nullptr) ||
        (peer_up0 && by0 == 0) || (peer_dn0 && by1 == H / 16)) {
        set_error("%s: a neighbour needs its plane, its flags and mine, and none past the frame edge", fn);
        return SO_E_INVALID;
    }
    if (nframes <= 0) return SO_OK;
    SO_NEED(curs, fn); SO_NEED(ref0, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn); SO_NEED(out_qtc, fn);
    SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn); SO_NEED(workspace, fn);
    std::vector<PFrameOut> outs((size_t)nframes);
    for (int i = 0; i < nframes; ++i) {
        SO_NEED(curs[i], fn); SO_NEED(out_split[i], fn); SO_NEED(out_mv[i], fn); SO_NEED(out_qtc[i], fn);
        SO_NEED(out_tokens[i], fn); SO_NEED(out_mae_num[i], fn); SO_NEED(out_recon[i], fn);
        outs[i] = PFrameOut{out_split[i], out_mv[i], out_qtc[i], out_tokens[i], out_mae_num[i], out_recon[i],
                            out_sse ? out_sse[i] : nullptr};
    }
    PRunStripe sp{by0, by1, peer_up0, peer_dn0, stride, my_up_flags, my_dn_flags, peer_up_flags, peer_dn_flags,
                  epoch, gbase, nullptr};
    return p_run_stripe_launch(curs, nframes, ref0, H, W, qp_rd, qp_row, outs.data(), workspace, sp, max_wg,
                               (hipStream_t)stream);
}

int so_stripe_halo_push(const uint8_t* plane, int H, int W, int by0, int by1, int gf, uint8_t* peer_up,
                        uint8_t* peer_dn, uint32_t* peer_up_flags, uint32_t* peer_dn_flags, uint32_t epoch,
                        void* stream) {
    const char* fn = "so_stripe_halo_push";
    SO_TRY(check_geom(fn, H, W, 16, 0));
    if (W % 128 != 0 || by0 < 0 || by1 > H / 16 || by1 <= by0 || gf < 0 || by1 - by0 < 1) {
        set_error("%s: bad stripe [%d, %d) / frame %d", fn, by0, by1, gf);
        return SO_E_INVALID;
    }
    if ((peer_up != nullptr) != (peer_up_flags != nullptr) || (peer_dn != nullptr) != (peer_dn_flags != nullptr)) {
        set_error("%s: a neighbour plane needs its flags", fn);
        return SO_E_INVALID;
    }
    SO_NEED(plane, fn);
    if (!peer_up && !peer_dn) return SO_OK;
    return stripe_halo_push_launch(plane, W, by0, by1, peer_up, peer_dn, peer_up_flags, peer_dn_flags, gf, epoch,
                                   (hipStream_t)stream);
}

// ---- one GOP across GPUs: consecutive frames on consecutive ranks (so_me.hip kRunFPipe) -----
// The frame pipeline's argument checks and launch, with (two_pass) or without two-pass RC.
static int fpipe_run(const char* fn, bool two_pass, const uint8_t* const* curs, int nframes, int H, int W, int bs,
                     int sr, int qp_rd, const int32_t* qp_row, int vbs, double lam, const int32_t* roi, int qp_lo,
                     int qp_hi,
                     uint8_t* const* out_split, int16_t* const* out_mv, int16_t* const* out_qtc,
                     int32_t* const* out_tokens, int32_t* const* out_mae_num, uint8_t* const* out_recon,
                     int32_t* const* out_sse, int32_t* const* out_qp_map, uint32_t* workspace, const uint8_t* land0,
                     const uint32_t* land_flags, int slot0, uint8_t* peer_land0, uint32_t* peer_flags,
                     uint8_t* peer2_land0, uint32_t* peer2_flags, const int32_t* push_to, int nslots, long long stride,
                     uint32_t epoch, int max_wg, int p2lag, void* stream) {
    SO_TRY(check_geom(fn, H, W, bs, vbs));
    SO_TRY(check_vbs(fn, vbs, lam));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    if (two_pass && vbs) {
        set_error("%s: two-pass RC with VBSEnable is not built for the frame pipeline", fn);
        return SO_E_UNSUPPORTED;
    }
    if (bs != 16 || sr != 16 || W % 128 != 0 || (two_pass && W > 8192)) {
        set_error("%s: covers bs 16 / sr 16 / W %% 128 == 0%s", fn, two_pass ? ", W <= 8192" : "");
        return SO_E_UNSUPPORTED;
    }
    if (two_pass && (qp_lo < 0 || qp_hi > 20 || qp_lo > qp_hi)) {
        set_error("%s: QP clamp [%d, %d] outside [0, 20]", fn, qp_lo, qp_hi);
        return SO_E_INVALID;
    }
    // every rank owns `nslots` landing slots: this run reads slots [slot0, slot0 + nframes) and
    // writes (system scope, over xGMI) only slots below nslots of its peers
    if (p2lag < 0) {
        set_error("%s: p2lag %d < 0", fn, p2lag);
        return SO_E_INVALID;
    }
    if (slot0 < 0 || nslots < 1 || slot0 + nframes > nslots || stride < (long long)H * W) {
        set_error("%s: slot0 %d + %d frames / nslots %d / stride %lld", fn, slot0, nframes, nslots, stride);
        return SO_E_INVALID;
    }
    if (nframes <= 0) return SO_OK;
    SO_NEED(curs, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn); SO_NEED(out_qtc, fn); SO_NEED(out_tokens, fn);
    SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn); SO_NEED(workspace, fn); SO_NEED(land0, fn);
    SO_NEED(land_flags, fn); SO_NEED(peer_land0, fn); SO_NEED(peer_flags, fn); SO_NEED(peer2_land0, fn);
    SO_NEED(peer2_flags, fn); SO_NEED(push_to, fn);
    if (two_pass) SO_NEED(out_qp_map, fn);
    std::vector<PFrameOut> outs((size_t)nframes);
    std::vector<int> push((size_t)nframes);
    const uint8_t* land_end = land0 + (long long)(slot0 + nframes) * stride;
    for (int i = 0; i < nframes; ++i) {
        SO_NEED(curs[i], fn); SO_NEED(out_split[i], fn); SO_NEED(out_mv[i], fn); SO_NEED(out_qtc[i], fn);
        SO_NEED(out_tokens[i], fn); SO_NEED(out_mae_num[i], fn); SO_NEED(out_recon[i], fn);
        if (two_pass) SO_NEED(out_qp_map[i], fn);
        if (out_recon[i] >= land0 && out_recon[i] < land_end) {
            set_error("%s: out_recon[%d] lies in the landing planes", fn, i);
            return SO_E_INVALID;
        }
        if (push_to[i] < -1 || (push_to[i] >> 1) >= nslots) {   // -1: nothing follows, no push
            set_error("%s: push_to[%d] = %d (nslots %d)", fn, i, push_to[i], nslots);
            return SO_E_INVALID;
        }
        push[(size_t)i] = push_to[i];
        outs[i] = PFrameOut{out_split[i], out_mv[i], out_qtc[i], out_tokens[i], out_mae_num[i], out_recon[i],
                            out_sse ? out_sse[i] : nullptr, two_pass ? out_qp_map[i] : nullptr};
    }
    PRunStripe sp{0, H / 16, peer2_land0, peer_land0, stride, nullptr, land_flags, peer2_flags, peer_flags,
                  epoch, slot0, land0};
    if (two_pass) {
        sp.roi = roi;
        sp.qp_lo = qp_lo;
        sp.qp_hi = qp_hi;
        sp.p2lag = p2lag;
        return p_run_fpipe_2pass_launch(curs, nframes, H, W, qp_rd, qp_row, outs.data(), workspace, sp, max_wg,
                                        (hipStream_t)stream, push.data());
    }
    return p_run_fpipe_launch(curs, nframes, H, W, qp_rd, qp_row, vbs, lam, outs.data(), workspace, sp, max_wg,
                              (hipStream_t)stream, push.data());
}

int so_encode_p_run_fpipe2(const uint8_t* const* curs, int nframes, int H, int W, int bs, int sr, int qp_rd,
                           const int32_t* qp_row, int vbs, double lam, uint8_t* const* out_split, int16_t* const* out_mv,
                           int16_t* const* out_qtc, int32_t* const* out_tokens, int32_t* const* out_mae_num,
                           uint8_t* const* out_recon, int32_t* const* out_sse, uint32_t* workspace,
                           const uint8_t* land0, const uint32_t* land_flags, int slot0, uint8_t* peer_land0,
                           uint32_t* peer_flags, uint8_t* peer2_land0, uint32_t* peer2_flags, const int32_t* push_to,
                           int nslots, long long stride, uint32_t epoch, int max_wg, void* stream) {
    return fpipe_run("so_encode_p_run_fpipe2", false, curs, nframes, H, W, bs, sr, qp_rd, qp_row, vbs, lam, nullptr, 0, 0,
                     out_split, out_mv, out_qtc, out_tokens, out_mae_num, out_recon, out_sse, nullptr, workspace, land0,
                     land_flags, slot0, peer_land0, peer_flags, peer2_land0, peer2_flags, push_to, nslots, stride, epoch,
                     max_wg, 0, stream);
}

int so_encode_p_run_fpipe_2pass(const uint8_t* const* curs, int nframes, int H, int W, int bs, int sr, int qp_rd,
                                const int32_t* qp_row, const int32_t* roi, int qp_lo, int qp_hi,
                                uint8_t* const* out_split, int16_t* const* out_mv, int16_t* const* out_qtc,
                                int32_t* const* out_tokens, int32_t* const* out_mae_num, uint8_t* const* out_recon,
                                int32_t* const* out_sse, int32_t* const* out_qp_map, uint32_t* workspace,
                                const uint8_t* land0, const uint32_t* land_flags, int slot0, uint8_t* peer_land0,
                                uint32_t* peer_flags, uint8_t* peer2_land0, uint32_t* peer2_flags,
                                const int32_t* push_to, int nslots, long long stride, uint32_t epoch, int max_wg,
                                int p2lag, void* stream) {
    return fpipe_run("so_encode_p_run_fpipe_2pass", true, curs, nframes, H, W, bs, sr, qp_rd, qp_row, 0, 0.0, roi, qp_lo,
                     qp_hi,
                     out_split, out_mv, out_qtc, out_tokens, out_mae_num, out_recon, out_sse, out_qp_map, workspace,
                     land0, land_flags, slot0, peer_land0, peer_flags, peer2_land0, peer2_flags, push_to, nslots, stride,
                     epoch, max_wg, p2lag, stream);
}

int so_frame_push(const uint8_t* plane, int H, int W, uint8_t* peer_plane, uint32_t* peer_flags, uint32_t epoch,
                  void* stream) {
    const char* fn = "so_frame_push";
    SO_TRY(check_geom(fn, H, W, 16, 0));
    if (W % 128 != 0) {
        set_error("%s: W %% 128 != 0", fn);
        return SO_E_UNSUPPORTED;
    }
    SO_NEED(plane, fn); SO_NEED(peer_plane, fn); SO_NEED(peer_flags, fn);
    return frame_push_launch(plane, H, W, peer_plane, peer_flags, epoch, (hipStream_t)stream);
}

// ---- memory the ranks share (uncached landing planes, IPC) ----------------------------------
int so_alloc_uncached(size_t bytes, void** out) {
    if (!out || bytes == 0) {
        set_error("so_alloc_uncached: bad arguments");
        return SO_E_INVALID;
    }
    const hipError_t e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached);
    if (e != hipSuccess) {
        set_error("so_alloc_uncached(%zu): %s", bytes, hipGetErrorString(e));
        return (int)e;
    }
    return SO_OK;
}

int so_free_device(void* p) {
    const hipError_t e = hipFree(p);
    if (e != hipSuccess) {
        set_error("so_free_device: %s", hipGetErrorString(e));
        return (int)e;
    }
    return SO_OK;
}

int so_ipc_export(void* p, uint8_t* out_handle) {
    static_assert(sizeof(hipIpcMemHandle_t) <= SO_IPC_HANDLE_BYTES, "IPC handle size");
    if (!p || !out_handle) {
        set_error("so_ipc_export: bad arguments");
        return SO_E_INVALID;
    }
    hipIpcMemHandle_t h;
    const hipError_t e = hipIpcGetMemHandle(&h, p);
    if (e != hipSuccess) {
        set_error("so_ipc_export: %s", hipGetErrorString(e));
        return (int)e;
    }
    memset(out_handle, 0, SO_IPC_HANDLE_BYTES);
    memcpy(out_handle, &h, sizeof(h));
    return SO_OK;
}

int so_ipc_open(const uint8_t* handle, void** out) {
    if (!handle || !out) {
        set_error("so_ipc_open: bad arguments");
        return SO_E_INVALID;
    }
    hipIpcMemHandle_t h;
    memcpy(&h, handle, sizeof(h));
    const hipError_t e = hipIpcOpenMemHandle(out, h, hipIpcMemLazyEnablePeerAccess);
    if (e != hipSuccess) {
        set_error("so_ipc_open: %s", hipGetErrorString(e));
        return (int)e;
    }
    return SO_OK;
}

int so_copy_d2d(void* dst, const void* src, size_t bytes, void* stream) {
    if ((!dst || !src) && bytes) {
        set_error("so_copy_d2d: bad arguments");
        return SO_E_INVALID;
    }
    const hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, (hipStream_t)stream);
    if (e != hipSuccess) {
        set_error("so_copy_d2d: %s", hipGetErrorString(e));
        return (int)e;
    }
    return SO_OK;
}

int so_memset_d8(void* dst, int value, size_t bytes, void* stream) {
    const hipError_t e = hipMemsetAsync(dst, value, bytes, (hipStream_t)stream);
    if (e != hipSuccess) {
        set_error("so_memset_d8: %s", hipGetErrorString(e));
        return (int)e;
    }
    return SO_OK;
}

int so_ipc_close(void* p) {
    const hipError_t e = hipIpcCloseMemHandle(p);
    if (e != hipSuccess) {
        set_error("so_ipc_close: %s", hipGetErrorString(e));
        return (int)e;
    }
    return SO_OK;
}

size_t so_i_frame_scratch_elems(int H, int W, int bs) {
    if (bs <= 0) return 0;
    const size_t nb = (size_t)(W / bs) * (size_t)(H / bs);
    return nb * (size_t)bs * bs + nb * 8;
}

int so_encode_i_rows(const uint8_t* cur, int H, int W, int bs, int sr, int by0, int by1, int qp_rd,
                     const int32_t* qp_row, int vbs, double lam, uint8_t* out_split, int16_t* out_mv,
                     int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae_num, uint8_t* out_recon,
                     int32_t* out_sse, int32_t* scratch, void* stream) {
    const char* fn = "so_encode_i_rows";
    SO_TRY(check_geom(fn, H, W, bs, vbs));
    SO_TRY(check_intra_width(fn, W));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    SO_TRY(check_rows(fn, H, bs, by0, by1));
    SO_NEED(cur, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn); SO_NEED(out_qtc, fn);
    SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn); SO_NEED(scratch, fn);
    return intra_encode_launch(cur, H, W, bs, sr, by0, by1, qp_rd, qp_row, nullptr, vbs, lam, out_split, out_mv, out_qtc,
                               out_tokens, out_mae_num, out_recon, out_sse, reinterpret_cast<uint8_t*>(scratch),
                               (hipStream_t)stream);
}

int so_encode_i_frame(const uint8_t* cur, int H, int W, int bs, int sr, int qp_rd, const int32_t* qp_row,
                      int vbs, double lam, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc,
                      int32_t* out_tokens, int32_t* out_mae_num, uint8_t* out_recon, int32_t* out_sse,
                      int32_t* scratch, void* stream) {
    if (bs <= 0) {
        set_error("so_encode_i_frame: block_size %d", bs);
        return SO_E_UNSUPPORTED;
    }
    return so_encode_i_rows(cur, H, W, bs, sr, 0, H / bs, qp_rd, qp_row, vbs, lam, out_split, out_mv, out_qtc,
                            out_tokens, out_mae_num, out_recon, out_sse, scratch, stream);
}

int so_inter_recon(const uint8_t* const* refs, int nref, int H, int W, int bs, int qp, const int32_t* qp_row,
                   const uint8_t* split, const int16_t* mv, const int16_t* qtc, uint8_t* out_recon, void* stream) {
    const char* fn = "so_inter_recon";
    SO_TRY(check_geom(fn, H, W, bs, 0));
    SO_TRY(check_qp(fn, qp));
    SO_NEED(split, fn); SO_NEED(mv, fn); SO_NEED(qtc, fn); SO_NEED(out_recon, fn);
    RefSet rs;
    SO_TRY(make_refs(fn, refs, nref, &rs));
    return inter_recon_launch(rs, nullptr, 0, H, W, bs, qp, qp_row, nullptr, split, mv, qtc, out_recon,
                              (hipStream_t)stream);
}

int so_intra_recon(int H, int W, int bs, int qp, const int32_t* qp_row, const uint8_t* split, const int16_t* mv,
                   const int16_t* qtc, uint8_t* out_recon, int32_t* scratch, void* stream) {
    const char* fn = "so_intra_recon";
    SO_TRY(check_geom(fn, H, W, bs, 0));
    SO_TRY(check_intra_width(fn, W));
    SO_TRY(check_qp(fn, qp));
    SO_NEED(split, fn); SO_NEED(mv, fn); SO_NEED(qtc, fn); SO_NEED(out_recon, fn); SO_NEED(scratch, fn);
    // the recon kernel only needs sr to size its ring: the largest reachable offset is 64
    return intra_recon_launch(H, W, bs, 64, qp, qp_row, nullptr, split, mv, qtc, out_recon,
                              reinterpret_cast<uint8_t*>(scratch), (hipStream_t)stream);
}

size_t so_fme_plane_stride(int H, int W) {
    if (H <= 0 || W <= 0) return 0;
    return (((size_t)H * W + 64) + 255) & ~(size_t)255;   // 64 B of slack for aligned row reads
}

size_t so_fme_workspace_bytes(int H, int W, int nref) {
    return nref <= 0 ? 0 : (size_t)nref * 4 * so_fme_plane_stride(H, W);
}

int so_fme_planes(const uint8_t* ref, int H, int W, int wrap, uint8_t* out_planes, void* stream) {
    const char* fn = "so_fme_planes";
    SO_NEED(ref, fn); SO_NEED(out_planes, fn);
    if (H <= 1 || W <= 1 || W % 4) {
        set_error("%s: frame %dx%d (W must be a multiple of 4)", fn, W, H);
        return SO_E_INVALID;
    }
    return fme_planes_launch(ref, H, W, wrap, out_planes, so_fme_plane_stride(H, W), (hipStream_t)stream);
}

// shared validation + dispatch of the ME variants into best / sub
static int me_ex(const char* fn, const uint8_t* cur, const uint8_t* const* refs, int nref, const RefSet& rs, int H,
                 int W, int bs, int sr, int by0, int by1, int me_mode, int fme, int fme_wrap, uint8_t* planes,
                 int32_t* best, int32_t* sub, hipStream_t st, int32_t* seg_ws = nullptr) {
    if (me_mode < SO_ME_FULL || me_mode > SO_ME_FAST_PAR) {
        set_error("%s: me_mode %d", fn, me_mode);
        return SO_E_INVALID;
    }
    if (me_mode == SO_ME_FAST_PAR && sub) {
        set_error("%s: fast_me under ParallelMode 2 with VBSEnable (the reference raises NameError, "
                  "Encoder.py:609)", fn);
        return SO_E_UNSUPPORTED;
    }
    if (me_mode == SO_ME_FAST && by0 != 0) {
        set_error("%s: fast_me's predictor chain runs over the whole frame (no stripes)", fn);
        return SO_E_UNSUPPORTED;
    }
    const size_t ps = so_fme_plane_stride(H, W);
    if (fme) {
        SO_NEED(planes, fn);
        if (me_mode == SO_ME_FULL && sr > 63) {
            set_error("%s: FME search_range %d > 63", fn, sr);
            return SO_E_UNSUPPORTED;
        }
        for (int r = 0; r < nref; ++r)
            SO_TRY(fme_planes_launch(refs[r], H, W, fme_wrap, planes + (size_t)r * 4 * ps, ps, st));
    }
    if (me_mode == SO_ME_FULL) {
        if (!fme) return me_launch(cur, rs, nref, H, W, bs, sr, by0, by1, best, sub, st);
        if (bs == 16 && sr == 16) return me_fme_launch(cur, planes, ps, nref, H, W, by0, by1, best, sub, st);
        return me_generic_launch(cur, rs, planes, ps, nref, H, W, bs, sr, by0, by1, best, sub, st);
    }
    const uint8_t* ptrs[4 * kMaxRef];
    const int nfast = me_mode == SO_ME_FAST_PAR ? 1 : nref;
    int nptr = 0;
    for (int r = 0; r < nfast; ++r) {
        if (fme)
            for (int p = 0; p < 4; ++p) ptrs[nptr++] = planes + (size_t)(4 * r + p) * ps;
        else
            ptrs[nptr++] = refs[r];
    }
    return me_fastpred_launch(cur, ptrs, nptr, nfast, H, W, bs, fme, by0, by1, me_mode == SO_ME_FAST, best, sub, seg_ws,
                              st);
}

int so_me_search_ex(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W, int bs, int sr,
                    int me_mode, int fme, int fme_wrap, uint8_t* fme_planes, int32_t* out_best, int32_t* out_sub,
                    void* stream) {
    const char* fn = "so_me_search_ex";
    SO_TRY(check_geom(fn, H, W, bs, out_sub != nullptr));
    SO_TRY(check_sr(fn, sr));
    SO_NEED(cur, fn);
    SO_NEED(out_best, fn);
    RefSet rs;
    SO_TRY(make_refs(fn, refs, nref, &rs));
    return me_ex(fn, cur, refs, nref, rs, H, W, bs, sr, 0, H / bs, me_mode, fme, fme_wrap, fme_planes, out_best,
                 out_sub, (hipStream_t)stream);
}

int so_encode_p_rows_ex(const uint8_t* cur, const uint8_t* const* refs, int nref, int H, int W, int bs, int sr,
                        int by0, int by1, int qp_rd, const int32_t* qp_row, const int32_t* qp_map, int vbs, double lam,
                        int me_mode, int fme, int fme_wrap, uint8_t* fme_planes, int flags, uint8_t* out_split, int16_t* out_mv, int16_t* out_qtc,
                        int32_t* out_tokens, int32_t* out_mae_num, uint8_t* out_recon, int32_t* out_sse,
                        int32_t* scratch, void* stream) {
    const char* fn = "so_encode_p_rows_ex";
    if (me_mode == SO_ME_FULL && !fme && !qp_map && !(flags & (SO_REUSE_ME | SO_TOKENS_ONLY)))
        return so_encode_p_rows(cur, refs, nref, H, W, bs, sr, by0, by1, qp_rd, qp_row, vbs, lam, out_split, out_mv,
                                out_qtc, out_tokens, out_mae_num, out_recon, out_sse, scratch, stream);
    SO_TRY(check_geom(fn, H, W, bs, vbs));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    SO_TRY(check_rows(fn, H, bs, by0, by1));
    SO_NEED(cur, fn); SO_NEED(scratch, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn);
    SO_NEED(out_qtc, fn); SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn);
    RefSet rs;
    SO_TRY(make_refs(fn, refs, nref, &rs));
    for (int i = 0; i < nref; ++i)
        if (refs[i] == out_recon) {
            set_error("%s: out_recon aliases refs[%d]", fn, i);
            return SO_E_INVALID;
        }
    const size_t nbs = (size_t)(W / bs) * (size_t)(by1 - by0);
    int32_t* best = scratch;
    int32_t* sub = vbs ? scratch + nbs * 4 : nullptr;
    hipStream_t st = (hipStream_t)stream;
    if (flags & SO_REUSE_ME) {
        // pass 2 of two-pass RC: the ME records (and FME planes) of the previous call stay
        if (fme) SO_NEED(fme_planes, fn);
    } else if (me_mode == SO_ME_FULL && !fme && use_fused(bs, sr, vbs, nref)) {
        return p_tile_launch(cur, rs, H, W, by0, by1, qp_rd, qp_row, qp_map, best, out_split, out_mv, out_qtc,
                             out_tokens, out_mae_num, out_recon, out_sse, st, (flags & SO_TOKENS_ONLY) != 0);
    } else {
        SO_TRY(me_ex(fn, cur, refs, nref, rs, H, W, bs, sr, by0, by1, me_mode, fme, fme_wrap, fme_planes, best, sub,
                     st, scratch + nbs * 4 + (vbs ? nbs * 16 : 0)));
    }
    return inter_tq_launch(cur, rs, fme ? fme_planes : nullptr, so_fme_plane_stride(H, W), H, W, bs, by0, by1, best,
                           sub, qp_rd, qp_row, qp_map, vbs, lam, out_split, out_mv, out_qtc, out_tokens, out_mae_num, out_recon,
                           out_sse, st);
}

int so_inter_recon_ex(const uint8_t* const* refs, int nref, int H, int W, int bs, int qp, const int32_t* qp_row,
                      const int32_t* qp_map, int fme, int fme_wrap, uint8_t* fme_planes, const uint8_t* split, const int16_t* mv,
                      const int16_t* qtc, uint8_t* out_recon, void* stream) {
    const char* fn = "so_inter_recon_ex";
    SO_TRY(check_geom(fn, H, W, bs, 0));
    SO_TRY(check_qp(fn, qp));
    SO_NEED(split, fn); SO_NEED(mv, fn); SO_NEED(qtc, fn); SO_NEED(out_recon, fn);
    if (fme) SO_NEED(fme_planes, fn);
    RefSet rs;
    SO_TRY(make_refs(fn, refs, nref, &rs));
    const size_t ps = so_fme_plane_stride(H, W);
    hipStream_t st = (hipStream_t)stream;
    if (fme)
        for (int r = 0; r < nref; ++r)
            SO_TRY(fme_planes_launch(refs[r], H, W, fme_wrap, fme_planes + (size_t)r * 4 * ps, ps, st));
    return inter_recon_launch(rs, fme ? fme_planes : nullptr, ps, H, W, bs, qp, qp_row, qp_map, split, mv, qtc,
                              out_recon, st);
}

int so_encode_i_rows_ex(const uint8_t* cur, int H, int W, int bs, int sr, int by0, int by1, int qp_rd,
                        const int32_t* qp_row, const int32_t* qp_map, int vbs, double lam, uint8_t* out_split,
                        int16_t* out_mv, int16_t* out_qtc, int32_t* out_tokens, int32_t* out_mae_num,
                        uint8_t* out_recon, int32_t* out_sse, int32_t* scratch, void* stream) {
    const char* fn = "so_encode_i_rows_ex";
    SO_TRY(check_geom(fn, H, W, bs, vbs));
    SO_TRY(check_intra_width(fn, W));
    SO_TRY(check_sr(fn, sr));
    SO_TRY(check_qp(fn, qp_rd));
    SO_TRY(check_rows(fn, H, bs, by0, by1));
    SO_NEED(cur, fn); SO_NEED(out_split, fn); SO_NEED(out_mv, fn); SO_NEED(out_qtc, fn);
    SO_NEED(out_tokens, fn); SO_NEED(out_mae_num, fn); SO_NEED(out_recon, fn); SO_NEED(scratch, fn);
    return intra_encode_launch(cur, H, W, bs, sr, by0, by1, qp_rd, qp_row, qp_map, vbs, lam, out_split, out_mv,
                               out_qtc, out_tokens, out_mae_num, out_recon, out_sse, reinterpret_cast<uint8_t*>(scratch),
                               (hipStream_t)stream);
}

int so_intra_recon_ex(int H, int W, int bs, int qp, const int32_t* qp_row, const int32_t* qp_map,
                      const uint8_t* split, const int16_t* mv, const int16_t* qtc, uint8_t* out_recon,
                      int32_t* scratch, void* stream) {
    const char* fn = "so_intra_recon_ex";
    SO_TRY(check_geom(fn, H, W, bs, 0));
    SO_TRY(check_intra_width(fn, W));
    SO_TRY(check_qp(fn, qp));
    SO_NEED(split, fn); SO_NEED(mv, fn); SO_NEED(qtc, fn); SO_NEED(out_recon, fn); SO_NEED(scratch, fn);
    return intra_recon_launch(H, W, bs, 64, qp, qp_row, qp_map, split, mv, qtc, out_recon,
                              reinterpret_cast<uint8_t*>(scratch), (hipStream_t)stream);
}

int so_qp_map(const int32_t* tokens, int H, int W, int bs, int by0, int by1, int qp_rd, const int32_t* qp_row,
              const int32_t* roi, int qp_lo, int qp_hi, int32_t* out_qp_map, void* stream) {
    const char* fn = "so_qp_map";
    if (bs <= 0 || H <= 0 || W <= 0 || H % bs || W % bs) {
        set_error("%s: bad geometry", fn);
        return SO_E_INVALID;
    }
    SO_TRY(check_rows(fn, H, bs, by0, by1));
    SO_NEED(out_qp_map, fn);
    if (qp_lo < 0 || qp_hi > 20 || qp_lo > qp_hi) {
        set_error("%s: QP clamp [%d, %d] outside [0, 20]", fn, qp_lo, qp_hi);
        return SO_E_INVALID;
    }
    if (by1 <= by0) return SO_OK;
    hipLaunchKernelGGL(qp_map_kernel, dim3(by1 - by0), dim3(256), 0, (hipStream_t)stream, tokens, W / bs, by0, qp_rd,
                       qp_row, roi, qp_lo, qp_hi, out_qp_map);
    return check_launch("qp_map_kernel");
}

int so_sum_i32_rows(const int32_t* const* rows, int n, int len, int64_t* out, void* stream) {
    const char* fn = "so_sum_i32_rows";
    if (n < 0 || len < 0) {
        set_error("%s: n %d / len %d", fn, n, len);
        return SO_E_INVALID;
    }
    if (n == 0) return SO_OK;
    SO_NEED(rows, fn); SO_NEED(out, fn);
    for (int i0 = 0; i0 < n; i0 += kSumMax) {
        const int m = n - i0 < kSumMax ? n - i0 : kSumMax;
        SumArgs a{};
        for (int i = 0; i < m; ++i) {
            SO_NEED(rows[i0 + i], fn);
            a.p[i] = rows[i0 + i];
        }
        hipLaunchKernelGGL(sum_rows_kernel, dim3(m), dim3(kSumThreads), 0, (hipStream_t)stream, a, len,
                           reinterpret_cast<long long*>(out + i0));
        const int rc = check_launch("sum_rows_kernel");
        if (rc != SO_OK) return rc;
    }
    return SO_OK;
}

int so_sse_u8(const uint8_t* a, const uint8_t* b, int64_t n, uint64_t* out_sse, void* stream) {
    const char* fn = "so_sse_u8";
    SO_NEED(a, fn); SO_NEED(b, fn); SO_NEED(out_sse, fn);
    if (n < 0) {
        set_error("%s: n < 0", fn);
        return SO_E_INVALID;
    }
    if ((reinterpret_cast<uintptr_t>(a) | reinterpret_cast<uintptr_t>(b)) & 15) {
        set_error("%s: planes must be 16-byte aligned", fn);
        return SO_E_INVALID;
    }
    int64_t blocks = (n / 16 + 255) / 256;
    if (blocks < 1) blocks = 1;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(sse_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, b, n,
                       reinterpret_cast<unsigned long long*>(out_sse));
    return check_launch("sse_kernel");
}

// ---- packed symbol stream (so_pack.hip) -----------------------------------------------------
size_t so_pack_bound(int nb, int bs) {
    if (nb <= 0 || (bs != 16 && bs != 8)) return 0;
    return (size_t)nb * pack_block_bound(bs);
}

int so_pack_frames(int nframes, const int32_t* frame_types, const uint8_t* const* split, const int16_t* const* mv,
                   const int16_t* const* qtc, int nb, int bs, uint32_t* const* offs, uint8_t* const* out,
                   unsigned long long cap, void* stream) {
    return so_pack_frames_ex(nframes, frame_types, split, mv, qtc, nb, bs, offs, out, cap, nullptr, stream);
}

int so_pack_frames_ex(int nframes, const int32_t* frame_types, const uint8_t* const* split, const int16_t* const* mv,
                      const int16_t* const* qtc, int nb, int bs, uint32_t* const* offs, uint8_t* const* out,
                      unsigned long long cap, uint32_t* totals, void* stream) {
    const char* fn = "so_pack_frames";
    if (bs != 16 && bs != 8) {
        set_error("%s: block_size %d not built", fn, bs);
        return SO_E_UNSUPPORTED;
    }
    if (nb <= 0 || nframes < 0) {
        set_error("%s: nb %d / nframes %d", fn, nb, nframes);
        return SO_E_INVALID;
    }
    if (nframes == 0) return SO_OK;
    SO_NEED(frame_types, fn); SO_NEED(split, fn); SO_NEED(mv, fn); SO_NEED(qtc, fn); SO_NEED(offs, fn); SO_NEED(out, fn);
    std::vector<PackFrame> fr((size_t)nframes);
    for (int i = 0; i < nframes; ++i) {
        SO_NEED(split[i], fn); SO_NEED(mv[i], fn); SO_NEED(qtc[i], fn); SO_NEED(offs[i], fn); SO_NEED(out[i], fn);
        if (frame_types[i] != 0 && frame_types[i] != 1) {
            set_error("%s: frame_types[%d] = %d", fn, i, frame_types[i]);
            return SO_E_INVALID;
        }
        fr[i] = PackFrame{split[i], mv[i], qtc[i], offs[i], out[i], frame_types[i]};
    }
    return pack_frames_launch(fr.data(), nframes, nb, bs, cap, totals, (hipStream_t)stream);
}

int so_unpack_frames(int nframes, const int32_t* frame_types, const uint8_t* const* packed, const uint32_t* const* offs,
                     int nb, int bs, uint8_t* const* split, int16_t* const* mv, int16_t* const* qtc, int32_t* err,
                     void* stream) {
    const char* fn = "so_unpack_frames";
    if (bs != 16 && bs != 8) {
        set_error("%s: block_size %d not built", fn, bs);
        return SO_E_UNSUPPORTED;
    }
    if (nb <= 0 || nframes < 0) {
        set_error("%s: nb %d / nframes %d", fn, nb, nframes);
        return SO_E_INVALID;
    }
    if (nframes == 0) return SO_OK;
    SO_NEED(frame_types, fn); SO_NEED(packed, fn); SO_NEED(offs, fn); SO_NEED(split, fn); SO_NEED(mv, fn);
    SO_NEED(qtc, fn); SO_NEED(err, fn);
    std::vector<UnpackFrame> fr((size_t)nframes);
    for (int i = 0; i < nframes; ++i) {
        SO_NEED(packed[i], fn); SO_NEED(offs[i], fn); SO_NEED(split[i], fn); SO_NEED(mv[i], fn); SO_NEED(qtc[i], fn);
        if (frame_types[i] != 0 && frame_types[i] != 1) {
            set_error("%s: frame_types[%d] = %d", fn, i, frame_types[i]);
            return SO_E_INVALID;
        }
        fr[i] = UnpackFrame{packed[i], offs[i], split[i], mv[i], qtc[i], frame_types[i]};
    }
    return unpack_frames_launch(fr.data(), nframes, nb, bs, err, (hipStream_t)stream);
}

}  // extern "C"
