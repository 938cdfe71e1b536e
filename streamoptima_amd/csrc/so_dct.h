// so_dct.h — FP64 DCT-II / DCT-III for gfx950 that is BITWISE identical to
// scipy.fftpack.dct/idct(norm='ortho') (the reference's apply_2d_dct / apply_2d_idct,
// Encoder.py:779-817, decoder.py:455-462).
//
// scipy.fftpack reaches pocketfft (C++, inside SciPy 1.15.3): T_dcst23 folds the DCT into
// a length-N real FFT (rfftp) made of radix-4 / radix-2 passes.  A DCT coefficient that
// is mathematically an exact .5 (e.g. the DC term when the block sum == 8 mod 16) is
// rounded by np.round on whichever side pocketfft's own float64 error lands, so matching
// the reference bit-for-bit requires the same operations in the same order with the same
// (not correctly rounded) twiddles.  Everything below is straight-line code after
// unrolling; the kernels are compiled with -ffp-contract=off so no FMA contraction can
// change a rounding.
//
// N = 16: rfftp factors [4, 4];  N = 8: [2, 4].  One lane transforms one length-N vector
// held in registers.
#pragma once
#include "so_common.h"

namespace so {
namespace dct {

// pocketfft T_dcst23 twiddle[i] ~= cos(pi (i+1) / (2N)) (4N-point sincos table values)
constexpr double kTw16Dct[15] = {
    0x1.fd88da3d12526p-1, 0x1.f6297cff75cb0p-1, 0x1.e9f4156c62ddap-1, 0x1.d906bcf328d46p-1,
    0x1.c38b2f180bdb1p-1, 0x1.a9b66290ea1a3p-1, 0x1.8bc806b151741p-1, 0x1.6a09e667f3bccp-1,
    0x1.44cf325091dd6p-1, 0x1.1c73b39ae68c8p-1, 0x1.e2b5d3806f639p-2, 0x1.87de2a6aea961p-2,
    0x1.294062ed59f04p-2, 0x1.8f8b83c69a60ap-3, 0x1.917a6bc29b424p-4};
// rfftp first-factor twiddles, pocketfft layout wa[i + x*(ido-1)], ido = 4
constexpr double kTw16Rf[9] = {
    0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2, 0.0,
    0x1.6a09e667f3bccp-1, 0x1.6a09e667f3bcdp-1, 0.0,
    0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1, 0.0};
constexpr double kSqrt2 = 0x1.6a09e667f3bcdp+0;
constexpr double kHsqt2 = 0x1.6a09e667f3bcdp-1;

// Every constant a pass multiplies by goes through these accessors (the halved and doubled
// twiddles are exact: scaling by a power of two).  TW16 / TW8 fold them into the code as
// literals; TW16R reads the same values from kTw16Tab through a pointer (below).
struct TW16 {
    SO_DEV double dct(int i) const { return kTw16Dct[i]; }
    SO_DEV double hdct(int i) const { return 0.5 * kTw16Dct[i]; }
    SO_DEV double dct2x(int i) const { return 2 * kTw16Dct[i]; }
    SO_DEV double rf(int i) const { return kTw16Rf[i]; }
    SO_DEV double fct() const { return 0x1.6a09e667f3bcdp-3; }   // T(1/sqrt(32))
    SO_DEV double sqrt2() const { return kSqrt2; }
    SO_DEV double hsqrt2() const { return kSqrt2 * 0.5; }
    SO_DEV double hsqt2() const { return kHsqt2; }
};
constexpr double kTw8Dct[7] = {
    0x1.f6297cff75cb0p-1, 0x1.d906bcf328d46p-1, 0x1.a9b66290ea1a3p-1, 0x1.6a09e667f3bccp-1,
    0x1.1c73b39ae68c8p-1, 0x1.87de2a6aea963p-2, 0x1.8f8b83c69a60ap-3};
constexpr double kTw8Rf[2] = {0x1.6a09e667f3bccp-1, 0x1.6a09e667f3bcdp-1};
struct TW8 {
    SO_DEV double dct(int i) const { return kTw8Dct[i]; }
    SO_DEV double hdct(int i) const { return 0.5 * kTw8Dct[i]; }
    SO_DEV double dct2x(int i) const { return 2 * kTw8Dct[i]; }
    SO_DEV double rf(int i) const { return kTw8Rf[i]; }
    SO_DEV double fct() const { return 0x1.0p-2; }   // T(1/sqrt(16))
    SO_DEV double sqrt2() const { return kSqrt2; }
    SO_DEV double hsqrt2() const { return kSqrt2 * 0.5; }
    SO_DEV double hsqt2() const { return kHsqt2; }
};

// The N = 16 constants as one table in constant memory, read by scalar loads through TW16R.
// A kernel that runs the transforms inside a persistent loop takes the table's address through
// an optimisation barrier once per pass (tw16_table()): the loads then stay in the pass, where
// the values live in SGPRs for its length only.  As literals, the ~45 constants were hoisted
// out of the loop, held in SGPRs across it and spilled to VGPR lanes (a v_writelane /
// v_readlane pair per constant and task).
#define SO_TW_D(i) kTw16Dct[i]
#define SO_TW_H(i) (0.5 * kTw16Dct[i])
static __constant__ double kTw16Tab[45] = {
    SO_TW_D(0), SO_TW_D(1), SO_TW_D(2), SO_TW_D(3), SO_TW_D(4), SO_TW_D(5), SO_TW_D(6), SO_TW_D(7),
    SO_TW_D(8), SO_TW_D(9), SO_TW_D(10), SO_TW_D(11), SO_TW_D(12), SO_TW_D(13), SO_TW_D(14),
    SO_TW_H(0), SO_TW_H(1), SO_TW_H(2), SO_TW_H(3), SO_TW_H(4), SO_TW_H(5), SO_TW_H(6), SO_TW_H(7),
    SO_TW_H(8), SO_TW_H(9), SO_TW_H(10), SO_TW_H(11), SO_TW_H(12), SO_TW_H(13), SO_TW_H(14),
    kTw16Rf[0], kTw16Rf[1], kTw16Rf[2], kTw16Rf[3], kTw16Rf[4], kTw16Rf[5], kTw16Rf[6], kTw16Rf[7], kTw16Rf[8],
    0x1.6a09e667f3bcdp-3, kSqrt2, kSqrt2 * 0.5, kHsqt2, 2 * kTw16Dct[7], 0.0};
#undef SO_TW_D
#undef SO_TW_H
typedef const __attribute__((address_space(4))) double* so_cdp;
struct TW16R {
    so_cdp p;
    SO_DEV double dct(int i) const { return p[i]; }
    SO_DEV double hdct(int i) const { return p[15 + i]; }
    SO_DEV double dct2x(int i) const { return i == 7 ? p[43] : 2 * p[i]; }   // only i = 7 is used
    SO_DEV double rf(int i) const { return p[30 + i]; }
    SO_DEV double fct() const { return p[39]; }
    SO_DEV double sqrt2() const { return p[40]; }
    SO_DEV double hsqrt2() const { return p[41]; }
    SO_DEV double hsqt2() const { return p[42]; }
};
SO_DEV TW16R tw16_table() {
    so_cdp q = (so_cdp)kTw16Tab;
    asm volatile("" : "+s"(q));
    return TW16R{q};
}
// The same for N = 8 (the VBS sub-blocks).
static __constant__ double kTw8Tab[21] = {
    kTw8Dct[0], kTw8Dct[1], kTw8Dct[2], kTw8Dct[3], kTw8Dct[4], kTw8Dct[5], kTw8Dct[6],
    0.5 * kTw8Dct[0], 0.5 * kTw8Dct[1], 0.5 * kTw8Dct[2], 0.5 * kTw8Dct[3], 0.5 * kTw8Dct[4],
    0.5 * kTw8Dct[5], 0.5 * kTw8Dct[6],
    kTw8Rf[0], kTw8Rf[1], 0x1.0p-2, kSqrt2, kSqrt2 * 0.5, kHsqt2, 2 * kTw8Dct[3]};
struct TW8R {
    so_cdp p;
    SO_DEV double dct(int i) const { return p[i]; }
    SO_DEV double hdct(int i) const { return p[7 + i]; }
    SO_DEV double dct2x(int i) const { return i == 3 ? p[20] : 2 * p[i]; }   // only i = 3 is used
    SO_DEV double rf(int i) const { return p[14 + i]; }
    SO_DEV double fct() const { return 0x1.0p-2; }   // an inline constant
    SO_DEV double sqrt2() const { return p[17]; }
    SO_DEV double hsqrt2() const { return p[18]; }
    SO_DEV double hsqt2() const { return p[19]; }
};
SO_DEV TW8R tw8_table() {
    so_cdp q = (so_cdp)kTw8Tab;
    asm volatile("" : "+s"(q));
    return TW8R{q};
}

#define SO_PM(a, b, c, d) { a = (c) + (d); b = (c) - (d); }
#define SO_MULPM(a, b, c, d, e, f) { a = (c) * (e) + (d) * (f); b = (c) * (f) - (d) * (e); }

// ---- real-FFT passes (radix 2 / radix 4), compile-time ido / l1 ----------------------
template <int IDO, int L1, class TW>
SO_DEV void radf2(const double* cc, double* ch, const TW& tw) {
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 2 * (c))]
#define WA(x, i) tw.rf((i) + (x) * (IDO - 1))
#pragma unroll
    for (int k = 0; k < L1; k++) SO_PM(CH(0, 0, k), CH(IDO - 1, 1, k), CC(0, k, 0), CC(0, k, 1));
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            CH(0, 1, k) = -CC(IDO - 1, k, 1);
            CH(IDO - 1, 0, k) = CC(IDO - 1, k, 0);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; k++)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                double tr2, ti2;
                SO_MULPM(tr2, ti2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
                SO_PM(CH(i - 1, 0, k), CH(ic - 1, 1, k), CC(i - 1, k, 0), tr2);
                SO_PM(CH(i, 0, k), CH(ic, 1, k), ti2, CC(i, k, 0));
            }
    }
#undef CC
#undef CH
}

template <int IDO, int L1, class TW>
SO_DEV void radf4(const double* cc, double* ch, const TW& tw) {
#define CC(a, b, c) cc[(a) + IDO * ((b) + L1 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + 4 * (c))]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        double tr1, tr2;
        SO_PM(tr1, CH(0, 2, k), CC(0, k, 3), CC(0, k, 1));
        SO_PM(tr2, CH(IDO - 1, 1, k), CC(0, k, 0), CC(0, k, 2));
        SO_PM(CH(0, 0, k), CH(IDO - 1, 3, k), tr2, tr1);
    }
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            double ti1 = -tw.hsqt2() * (CC(IDO - 1, k, 1) + CC(IDO - 1, k, 3));
            double tr1 = tw.hsqt2() * (CC(IDO - 1, k, 1) - CC(IDO - 1, k, 3));
            SO_PM(CH(IDO - 1, 0, k), CH(IDO - 1, 2, k), CC(IDO - 1, k, 0), tr1);
            SO_PM(CH(0, 3, k), CH(0, 1, k), ti1, CC(IDO - 1, k, 2));
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; k++)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                double ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
                SO_MULPM(cr2, ci2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
                SO_MULPM(cr3, ci3, WA(1, i - 2), WA(1, i - 1), CC(i - 1, k, 2), CC(i, k, 2));
                SO_MULPM(cr4, ci4, WA(2, i - 2), WA(2, i - 1), CC(i - 1, k, 3), CC(i, k, 3));
                SO_PM(tr1, tr4, cr4, cr2);
                SO_PM(ti1, ti4, ci2, ci4);
                SO_PM(tr2, tr3, CC(i - 1, k, 0), cr3);
                SO_PM(ti2, ti3, CC(i, k, 0), ci3);
                SO_PM(CH(i - 1, 0, k), CH(ic - 1, 3, k), tr2, tr1);
                SO_PM(CH(i, 0, k), CH(ic, 3, k), ti1, ti2);
                SO_PM(CH(i - 1, 2, k), CH(ic - 1, 1, k), tr3, ti4);
                SO_PM(CH(i, 2, k), CH(ic, 1, k), tr4, ti3);
            }
    }
#undef CC
#undef CH
}

template <int IDO, int L1, class TW>
SO_DEV void radb2(const double* cc, double* ch, const TW& tw) {
#define CC(a, b, c) cc[(a) + IDO * ((b) + 2 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#pragma unroll
    for (int k = 0; k < L1; k++) SO_PM(CH(0, k, 0), CH(0, k, 1), CC(0, 0, k), CC(IDO - 1, 1, k));
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            CH(IDO - 1, k, 0) = 2.0 * CC(IDO - 1, 0, k);
            CH(IDO - 1, k, 1) = -2.0 * CC(0, 1, k);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; ++k)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                const int ic = IDO - i;
                double ti2, tr2;
                SO_PM(CH(i - 1, k, 0), tr2, CC(i - 1, 0, k), CC(ic - 1, 1, k));
                SO_PM(ti2, CH(i, k, 0), CC(i, 0, k), CC(ic, 1, k));
                SO_MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ti2, tr2);
            }
    }
#undef CC
#undef CH
}

template <int IDO, int L1, class TW>
SO_DEV void radb4(const double* cc, double* ch, const TW& tw) {
#define CC(a, b, c) cc[(a) + IDO * ((b) + 4 * (c))]
#define CH(a, b, c) ch[(a) + IDO * ((b) + L1 * (c))]
#pragma unroll
    for (int k = 0; k < L1; k++) {
        double tr1, tr2;
        SO_PM(tr2, tr1, CC(0, 0, k), CC(IDO - 1, 3, k));
        // tr3 = 2 x, tr4 = 2 z and then tr2 +- tr3, tr1 +- tr4: 2x is exact, so
        // fma(+-2, x, tr2) rounds once, exactly like tr2 +- fl(2x)
        const double x = CC(IDO - 1, 1, k), z = CC(0, 2, k);
        CH(0, k, 0) = __builtin_fma(2.0, x, tr2);
        CH(0, k, 2) = __builtin_fma(-2.0, x, tr2);
        CH(0, k, 3) = __builtin_fma(2.0, z, tr1);
        CH(0, k, 1) = __builtin_fma(-2.0, z, tr1);
    }
    if constexpr ((IDO & 1) == 0) {
#pragma unroll
        for (int k = 0; k < L1; k++) {
            double tr1, tr2, ti1, ti2;
            SO_PM(ti1, ti2, CC(0, 3, k), CC(0, 1, k));
            SO_PM(tr2, tr1, CC(IDO - 1, 0, k), CC(IDO - 1, 2, k));
            CH(IDO - 1, k, 0) = tr2 + tr2;
            CH(IDO - 1, k, 1) = tw.sqrt2() * (tr1 - ti1);
            CH(IDO - 1, k, 2) = ti2 + ti2;
            CH(IDO - 1, k, 3) = -tw.sqrt2() * (tr1 + ti1);
        }
    }
    if constexpr (IDO > 2) {
#pragma unroll
        for (int k = 0; k < L1; ++k)
#pragma unroll
            for (int i = 2; i < IDO; i += 2) {
                double ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
                const int ic = IDO - i;
                SO_PM(tr2, tr1, CC(i - 1, 0, k), CC(ic - 1, 3, k));
                SO_PM(ti1, ti2, CC(i, 0, k), CC(ic, 3, k));
                SO_PM(tr4, ti3, CC(i, 2, k), CC(ic, 1, k));
                SO_PM(tr3, ti4, CC(i - 1, 2, k), CC(ic - 1, 1, k));
                SO_PM(CH(i - 1, k, 0), cr3, tr2, tr3);
                SO_PM(CH(i, k, 0), ci3, ti2, ti3);
                SO_PM(cr4, cr2, tr1, tr4);
                SO_PM(ci2, ci4, ti1, ti4);
                SO_MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ci2, cr2);
                SO_MULPM(CH(i, k, 2), CH(i - 1, k, 2), WA(1, i - 2), WA(1, i - 1), ci3, cr3);
                SO_MULPM(CH(i, k, 3), CH(i - 1, k, 3), WA(2, i - 2), WA(2, i - 1), ci4, cr4);
            }
    }
#undef CC
#undef CH
#undef WA
}

// halfcomplex -> real (unscaled), then copy_and_norm(fct)
template <int N> struct Rfft;
template <> struct Rfft<16> {
    using TW = TW16;
    template <class T>
    static SO_DEV void backward(double* c, const T& tw) {
        double ch[16];
        radb4<4, 1>(c, ch, tw);
        radb4<1, 4>(ch, c, tw);
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] *= tw.fct();
    }
    template <class T>
    static SO_DEV void forward(double* c, const T& tw) {
        double ch[16];
        radf4<1, 4>(c, ch, tw);
        radf4<4, 1>(ch, c, tw);
#pragma unroll
        for (int i = 0; i < 16; ++i) c[i] *= tw.fct();
    }
};
template <> struct Rfft<8> {
    using TW = TW8;
    template <class T>
    static SO_DEV void backward(double* c, const T& tw) {
        double ch[8];
        radb2<4, 1>(c, ch, tw);
        radb4<1, 2>(ch, c, tw);
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] *= tw.fct();
    }
    template <class T>
    static SO_DEV void forward(double* c, const T& tw) {
        double ch[8];
        radf4<1, 2>(c, ch, tw);
        radf2<4, 1>(ch, c, tw);
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] *= tw.fct();
    }
};

// DCT-II, ortho (pocketfft T_dcst23::exec type 2, cosine)
template <int N, class TW = typename Rfft<N>::TW>
SO_DEV void dct2(double* c, const TW& tw = TW{}) {
    constexpr int NS2 = (N + 1) / 2;
    c[0] *= 2;
    c[N - 1] *= 2;
#pragma unroll
    for (int k = 1; k < N - 1; k += 2) {
        double t = c[k + 1];
        c[k + 1] -= c[k];
        c[k] += t;
    }
    Rfft<N>::backward(c, tw);
    // 0.5 (t1 +- t2) with the 0.5 folded into the twiddles: scaling by a power of two
    // commutes with every rounding (no under/overflow at these magnitudes), so
    // (0.5 w) a + (0.5 v) b == 0.5 (w a + v b) bit for bit
#pragma unroll
    for (int k = 1; k < NS2; ++k) {
        const int kc = N - k;
        const double ha = tw.hdct(k - 1), hb = tw.hdct(kc - 1);
        double t1 = ha * c[kc] + hb * c[k];
        double t2 = ha * c[k] - hb * c[kc];
        c[k] = t1 + t2;
        c[kc] = t1 - t2;
    }
    c[NS2] *= tw.dct(NS2 - 1);
    c[0] *= tw.hsqrt2();
}

// DCT-III, ortho (pocketfft T_dcst23::exec type 3, cosine)
template <int N, class TW = typename Rfft<N>::TW>
SO_DEV void dct3(double* c, const TW& tw = TW{}) {
    constexpr int NS2 = (N + 1) / 2;
    c[0] *= tw.sqrt2();
#pragma unroll
    for (int k = 1; k < NS2; ++k) {
        const int kc = N - k;
        double t1 = c[k] + c[kc], t2 = c[k] - c[kc];
        c[k] = tw.dct(k - 1) * t2 + tw.dct(kc - 1) * t1;
        c[kc] = tw.dct(k - 1) * t1 - tw.dct(kc - 1) * t2;
    }
    c[NS2] *= tw.dct2x(NS2 - 1);
    Rfft<N>::forward(c, tw);
#pragma unroll
    for (int k = 1; k < N - 1; k += 2) {
        double t = c[k];
        c[k] -= c[k + 1];
        c[k + 1] += t;
    }
}

// ---- integer inputs (the first pass of a 2-D transform) ------------------------------------
// dct2<16> / dct3<16> of a vector of integers (residuals; dequantised coefficients).  An FP64
// add, subtract or doubling of integers below 2^24 is exact, so every such step of the sequence
// above is done in int32 (a 2-cycle VALU op on gfx950 against 4 for FP64) and its value
// converted where it first meets a twiddle: the same doubles bit for bit, with as many
// conversions as loading the 16 inputs as doubles took.  54 of dct2's FP64 ops and 14 of
// dct3's move to the integer pipe.
template <class TW = TW16>
SO_DEV void dct2_16_i(const int (&x)[16], double (&c)[16], const TW& tw = TW{}) {
    int y[16];   // T_dcst23 type-2 prelude
    y[0] = 2 * x[0];
    y[15] = 2 * x[15];
#pragma unroll
    for (int k = 1; k < 15; k += 2) {
        y[k + 1] = x[k + 1] - x[k];
        y[k] = x[k] + x[k + 1];
    }
    // radb4<4, 1>: CC(a, 0, c) = y[a + 4 c], CH(a, 0, c) = h[a + 4 c]; ih = the integer entries
    int ih0, ih1, ih2, ih3, ih4, ih8, ih11, ih12;
    double h5, h6, h7, h9, h10, h13, h14, h15;
    {
        const int tr2 = y[0] + y[15], tr1 = y[0] - y[15];
        ih0 = tr2 + 2 * y[7];
        ih8 = tr2 - 2 * y[7];
        ih12 = tr1 + 2 * y[8];
        ih4 = tr1 - 2 * y[8];
    }
    {
        const int ti1 = y[12] + y[4], ti2 = y[12] - y[4];
        const int tr2 = y[3] + y[11], tr1 = y[3] - y[11];
        ih3 = tr2 + tr2;
        h7 = tw.sqrt2() * (double)(tr1 - ti1);
        ih11 = ti2 + ti2;
        h15 = -tw.sqrt2() * (double)(tr1 + ti1);
    }
    {
        const int tr2 = y[1] + y[13], tr1 = y[1] - y[13];
        const int ti1 = y[2] + y[14], ti2 = y[2] - y[14];
        const int tr4 = y[10] + y[6], ti3 = y[10] - y[6];
        const int tr3 = y[9] + y[5], ti4 = y[9] - y[5];
        ih1 = tr2 + tr3;
        const double cr3 = (double)(tr2 - tr3);
        ih2 = ti2 + ti3;
        const double ci3 = (double)(ti2 - ti3);
        const double cr4 = (double)(tr1 + tr4), cr2 = (double)(tr1 - tr4);
        const double ci2 = (double)(ti1 + ti4), ci4 = (double)(ti1 - ti4);
        h6 = tw.rf(0) * ci2 + tw.rf(1) * cr2;
        h5 = tw.rf(0) * cr2 - tw.rf(1) * ci2;
        h10 = tw.rf(3) * ci3 + tw.rf(4) * cr3;
        h9 = tw.rf(3) * cr3 - tw.rf(4) * ci3;
        h14 = tw.rf(6) * ci4 + tw.rf(7) * cr4;
        h13 = tw.rf(6) * cr4 - tw.rf(7) * ci4;
    }
    // radb4<1, 4>: CC(0, b, k) = h[b + 4 k], CH(0, k, j) = c[k + 4 j]
    {   // k = 0: all four inputs integers
        const int tr2 = ih0 + ih3, tr1 = ih0 - ih3;
        c[0] = (double)(tr2 + 2 * ih1);
        c[8] = (double)(tr2 - 2 * ih1);
        c[12] = (double)(tr1 + 2 * ih2);
        c[4] = (double)(tr1 - 2 * ih2);
    }
    {   // k = 1
        const double a = (double)ih4, tr2 = a + h7, tr1 = a - h7;
        c[1] = __builtin_fma(2.0, h5, tr2);
        c[9] = __builtin_fma(-2.0, h5, tr2);
        c[13] = __builtin_fma(2.0, h6, tr1);
        c[5] = __builtin_fma(-2.0, h6, tr1);
    }
    {   // k = 2
        const double tr2 = (double)(ih8 + ih11), tr1 = (double)(ih8 - ih11);
        c[2] = __builtin_fma(2.0, h9, tr2);
        c[10] = __builtin_fma(-2.0, h9, tr2);
        c[14] = __builtin_fma(2.0, h10, tr1);
        c[6] = __builtin_fma(-2.0, h10, tr1);
    }
    {   // k = 3
        const double a = (double)ih12, tr2 = a + h15, tr1 = a - h15;
        c[3] = __builtin_fma(2.0, h13, tr2);
        c[11] = __builtin_fma(-2.0, h13, tr2);
        c[15] = __builtin_fma(2.0, h14, tr1);
        c[7] = __builtin_fma(-2.0, h14, tr1);
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] *= tw.fct();
    // dct2's post-twiddles, unchanged
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        const int kc = 16 - k;
        const double ha = tw.hdct(k - 1), hb = tw.hdct(kc - 1);
        double t1 = ha * c[kc] + hb * c[k];
        double t2 = ha * c[k] - hb * c[kc];
        c[k] = t1 + t2;
        c[kc] = t1 - t2;
    }
    c[8] *= tw.dct(7);
    c[0] *= tw.hsqrt2();
}

template <class TW = TW16>
SO_DEV void dct3_16_i(const int (&x)[16], double (&c)[16], const TW& tw = TW{}) {
    c[0] = (double)x[0] * tw.sqrt2();
#pragma unroll
    for (int k = 1; k < 8; ++k) {
        const int kc = 16 - k;
        const double t1 = (double)(x[k] + x[kc]), t2 = (double)(x[k] - x[kc]);
        c[k] = tw.dct(k - 1) * t2 + tw.dct(kc - 1) * t1;
        c[kc] = tw.dct(k - 1) * t1 - tw.dct(kc - 1) * t2;
    }
    c[8] = (double)x[8] * tw.dct2x(7);
    Rfft<16>::forward(c, tw);
#pragma unroll
    for (int k = 1; k < 15; k += 2) {
        double t = c[k];
        c[k] -= c[k + 1];
        c[k + 1] += t;
    }
}

// The same for N = 8 (the VBS sub-blocks): rfftp [2, 4]; 24 of dct2<8>'s FP64 ops and 6 of
// dct3<8>'s move to int32.
template <class TW = TW8>
SO_DEV void dct2_8_i(const int (&x)[8], double (&c)[8], const TW& tw = TW{}) {
    int y[8];
    y[0] = 2 * x[0];
    y[7] = 2 * x[7];
#pragma unroll
    for (int k = 1; k < 7; k += 2) {
        y[k + 1] = x[k + 1] - x[k];
        y[k] = x[k] + x[k + 1];
    }
    // radb2<4, 1>: CC(a, b, 0) = y[a + 4 b], CH(a, 0, c) = h[a + 4 c]
    const int ih0 = y[0] + y[7], ih4 = y[0] - y[7];
    const int ih3 = 2 * y[3], ih7 = -2 * y[4];
    const int ih1 = y[1] + y[5], tr2 = y[1] - y[5];
    const int ti2 = y[2] + y[6], ih2 = y[2] - y[6];
    const double h6 = tw.rf(0) * (double)ti2 + tw.rf(1) * (double)tr2;
    const double h5 = tw.rf(0) * (double)tr2 - tw.rf(1) * (double)ti2;
    // radb4<1, 2>: CC(0, b, k) = h[b + 4 k], CH(0, k, j) = c[k + 2 j]
    {   // k = 0: all four inputs integers
        const int t2 = ih0 + ih3, t1 = ih0 - ih3;
        c[0] = (double)(t2 + 2 * ih1);
        c[4] = (double)(t2 - 2 * ih1);
        c[6] = (double)(t1 + 2 * ih2);
        c[2] = (double)(t1 - 2 * ih2);
    }
    {   // k = 1: h[4], h[7] integers, h[5], h[6] not
        const double t2 = (double)(ih4 + ih7), t1 = (double)(ih4 - ih7);
        c[1] = __builtin_fma(2.0, h5, t2);
        c[5] = __builtin_fma(-2.0, h5, t2);
        c[7] = __builtin_fma(2.0, h6, t1);
        c[3] = __builtin_fma(-2.0, h6, t1);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] *= tw.fct();
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const int kc = 8 - k;
        const double ha = tw.hdct(k - 1), hb = tw.hdct(kc - 1);
        double t1 = ha * c[kc] + hb * c[k];
        double t2 = ha * c[k] - hb * c[kc];
        c[k] = t1 + t2;
        c[kc] = t1 - t2;
    }
    c[4] *= tw.dct(3);
    c[0] *= tw.hsqrt2();
}

template <class TW = TW8>
SO_DEV void dct3_8_i(const int (&x)[8], double (&c)[8], const TW& tw = TW{}) {
    c[0] = (double)x[0] * tw.sqrt2();
#pragma unroll
    for (int k = 1; k < 4; ++k) {
        const int kc = 8 - k;
        const double t1 = (double)(x[k] + x[kc]), t2 = (double)(x[k] - x[kc]);
        c[k] = tw.dct(k - 1) * t2 + tw.dct(kc - 1) * t1;
        c[kc] = tw.dct(k - 1) * t1 - tw.dct(kc - 1) * t2;
    }
    c[4] = (double)x[4] * tw.dct2x(3);
    Rfft<8>::forward(c, tw);
#pragma unroll
    for (int k = 1; k < 7; k += 2) {
        double t = c[k];
        c[k] -= c[k + 1];
        c[k + 1] += t;
    }
}

#undef SO_PM
#undef SO_MULPM

}  // namespace dct
}  // namespace so
