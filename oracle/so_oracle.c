/*
 * so_oracle.c — CPU ORACLE for the StreamOptima per-block encode path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is a plain-C restatement of the reference
 * encoder's algorithm (Suyashagarw/StreamOptima, Encoder.py / decoder.py) and of the
 * pocketfft DCT that the reference reaches through scipy.fftpack.  It is compiled into
 * oracle/_build/libso_oracle.so and may only be loaded by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg, as the CHECKER.
 * The product path (streamoptima_amd/, libstreamoptima_hip.so) never links or calls it.
 *
 * Parity pinning: every function here is checked against golden vectors produced by
 * running the reference itself in the development container (tests/golden/make_golden.py,
 * fixtures in tests/golden/ as .npz) - see tests/test_oracle_golden.py.
 *
 * Third-party arithmetic restated here: scipy.fftpack.dct/idct (SciPy 1.15.3) ->
 * pocketfft C++ (scipy/fft/_pocketfft), type-2/type-3 DCT via a real FFT (rfftp with
 * radix-4/radix-2 passes).  Twiddle factors are pocketfft's own (not correctly rounded)
 * double values, listed in SURVEY.md Appendix A.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define EXPORT __attribute__((visibility("default")))
#define SO_ORACLE_MAX_REF 16

/* ------------------------------------------------------------------------------------ */
/* pocketfft restatement (rfftp + T_dcst23), N in {8, 16}                                */
/* ------------------------------------------------------------------------------------ */

/* DCT twiddles tw[i] ~= cos(pi*(i+1)/(2N)) (pocketfft T_dcst23 twiddle[], 4N-point
 * sincos table).  SURVEY.md Appendix A. */
static const double DCT_TW16[15] = {
    0x1.fd88da3d12526p-1, 0x1.f6297cff75cb0p-1, 0x1.e9f4156c62ddap-1, 0x1.d906bcf328d46p-1,
    0x1.c38b2f180bdb1p-1, 0x1.a9b66290ea1a3p-1, 0x1.8bc806b151741p-1, 0x1.6a09e667f3bccp-1,
    0x1.44cf325091dd6p-1, 0x1.1c73b39ae68c8p-1, 0x1.e2b5d3806f639p-2, 0x1.87de2a6aea961p-2,
    0x1.294062ed59f04p-2, 0x1.8f8b83c69a60ap-3, 0x1.917a6bc29b424p-4};
static const double DCT_TW8[7] = {
    0x1.f6297cff75cb0p-1, 0x1.d906bcf328d46p-1, 0x1.a9b66290ea1a3p-1, 0x1.6a09e667f3bccp-1,
    0x1.1c73b39ae68c8p-1, 0x1.87de2a6aea963p-2, 0x1.8f8b83c69a60ap-3};

/* rfftp twiddles of the first factor: (cos, sin)(2*pi*m/N), pocketfft values. */
static const double RF_TW16[9] = {  /* factor 4, ido 4: tw[(j-1)*(ido-1) + 2i-2 (+1)], j=1..3, i=1 */
    0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2, 0.0,
    0x1.6a09e667f3bccp-1, 0x1.6a09e667f3bcdp-1, 0.0,
    0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1, 0.0};
static const double RF_TW8[2] = {   /* factor 2, ido 4: j=1, i=1 */
    0x1.6a09e667f3bccp-1, 0x1.6a09e667f3bcdp-1};

static const double SQRT2 = 0x1.6a09e667f3bcdp+0;   /* T0(1.41421356...L) */
static const double HSQT2 = 0x1.6a09e667f3bcdp-1;   /* T0(0.70710678...L) */

#define PM(a, b, c, d) { a = (c) + (d); b = (c) - (d); }
#define MULPM(a, b, c, d, e, f) { a = (c) * (e) + (d) * (f); b = (c) * (f) - (d) * (e); }

/* radf2 (pocketfft rfftp::radf2) */
static void radf2(size_t ido, size_t l1, const double *cc, double *ch, const double *wa) {
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + 2 * (c))]
#define WA(x, i) wa[(i) + (x) * (ido - 1)]
    for (size_t k = 0; k < l1; k++) PM(CH(0, 0, k), CH(ido - 1, 1, k), CC(0, k, 0), CC(0, k, 1));
    if ((ido & 1) == 0)
        for (size_t k = 0; k < l1; k++) {
            CH(0, 1, k) = -CC(ido - 1, k, 1);
            CH(ido - 1, 0, k) = CC(ido - 1, k, 0);
        }
    if (ido <= 2) return;
    for (size_t k = 0; k < l1; k++)
        for (size_t i = 2; i < ido; i += 2) {
            size_t ic = ido - i;
            double tr2, ti2;
            MULPM(tr2, ti2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
            PM(CH(i - 1, 0, k), CH(ic - 1, 1, k), CC(i - 1, k, 0), tr2);
            PM(CH(i, 0, k), CH(ic, 1, k), ti2, CC(i, k, 0));
        }
#undef CC
#undef CH
}

/* radf4 (pocketfft rfftp::radf4) */
static void radf4(size_t ido, size_t l1, const double *cc, double *ch, const double *wa) {
#define CC(a, b, c) cc[(a) + ido * ((b) + l1 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + 4 * (c))]
    for (size_t k = 0; k < l1; k++) {
        double tr1, tr2;
        PM(tr1, CH(0, 2, k), CC(0, k, 3), CC(0, k, 1));
        PM(tr2, CH(ido - 1, 1, k), CC(0, k, 0), CC(0, k, 2));
        PM(CH(0, 0, k), CH(ido - 1, 3, k), tr2, tr1);
    }
    if ((ido & 1) == 0)
        for (size_t k = 0; k < l1; k++) {
            double ti1 = -HSQT2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3));
            double tr1 = HSQT2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3));
            PM(CH(ido - 1, 0, k), CH(ido - 1, 2, k), CC(ido - 1, k, 0), tr1);
            PM(CH(0, 3, k), CH(0, 1, k), ti1, CC(ido - 1, k, 2));
        }
    if (ido <= 2) return;
    for (size_t k = 0; k < l1; k++)
        for (size_t i = 2; i < ido; i += 2) {
            size_t ic = ido - i;
            double ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
            MULPM(cr2, ci2, WA(0, i - 2), WA(0, i - 1), CC(i - 1, k, 1), CC(i, k, 1));
            MULPM(cr3, ci3, WA(1, i - 2), WA(1, i - 1), CC(i - 1, k, 2), CC(i, k, 2));
            MULPM(cr4, ci4, WA(2, i - 2), WA(2, i - 1), CC(i - 1, k, 3), CC(i, k, 3));
            PM(tr1, tr4, cr4, cr2);
            PM(ti1, ti4, ci2, ci4);
            PM(tr2, tr3, CC(i - 1, k, 0), cr3);
            PM(ti2, ti3, CC(i, k, 0), ci3);
            PM(CH(i - 1, 0, k), CH(ic - 1, 3, k), tr2, tr1);
            PM(CH(i, 0, k), CH(ic, 3, k), ti1, ti2);
            PM(CH(i - 1, 2, k), CH(ic - 1, 1, k), tr3, ti4);
            PM(CH(i, 2, k), CH(ic, 1, k), tr4, ti3);
        }
#undef CC
#undef CH
}

/* radb2 (pocketfft rfftp::radb2) */
static void radb2(size_t ido, size_t l1, const double *cc, double *ch, const double *wa) {
#define CC(a, b, c) cc[(a) + ido * ((b) + 2 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
    for (size_t k = 0; k < l1; k++) PM(CH(0, k, 0), CH(0, k, 1), CC(0, 0, k), CC(ido - 1, 1, k));
    if ((ido & 1) == 0)
        for (size_t k = 0; k < l1; k++) {
            CH(ido - 1, k, 0) = 2.0 * CC(ido - 1, 0, k);
            CH(ido - 1, k, 1) = -2.0 * CC(0, 1, k);
        }
    if (ido <= 2) return;
    for (size_t k = 0; k < l1; ++k)
        for (size_t i = 2; i < ido; i += 2) {
            size_t ic = ido - i;
            double ti2, tr2;
            PM(CH(i - 1, k, 0), tr2, CC(i - 1, 0, k), CC(ic - 1, 1, k));
            PM(ti2, CH(i, k, 0), CC(i, 0, k), CC(ic, 1, k));
            MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ti2, tr2);
        }
#undef CC
#undef CH
}

/* radb4 (pocketfft rfftp::radb4) */
static void radb4(size_t ido, size_t l1, const double *cc, double *ch, const double *wa) {
#define CC(a, b, c) cc[(a) + ido * ((b) + 4 * (c))]
#define CH(a, b, c) ch[(a) + ido * ((b) + l1 * (c))]
    for (size_t k = 0; k < l1; k++) {
        double tr1, tr2;
        PM(tr2, tr1, CC(0, 0, k), CC(ido - 1, 3, k));
        double tr3 = 2.0 * CC(ido - 1, 1, k);
        double tr4 = 2.0 * CC(0, 2, k);
        PM(CH(0, k, 0), CH(0, k, 2), tr2, tr3);
        PM(CH(0, k, 3), CH(0, k, 1), tr1, tr4);
    }
    if ((ido & 1) == 0)
        for (size_t k = 0; k < l1; k++) {
            double tr1, tr2, ti1, ti2;
            PM(ti1, ti2, CC(0, 3, k), CC(0, 1, k));
            PM(tr2, tr1, CC(ido - 1, 0, k), CC(ido - 1, 2, k));
            CH(ido - 1, k, 0) = tr2 + tr2;
            CH(ido - 1, k, 1) = SQRT2 * (tr1 - ti1);
            CH(ido - 1, k, 2) = ti2 + ti2;
            CH(ido - 1, k, 3) = -SQRT2 * (tr1 + ti1);
        }
    if (ido <= 2) return;
    for (size_t k = 0; k < l1; ++k)
        for (size_t i = 2; i < ido; i += 2) {
            double ci2, ci3, ci4, cr2, cr3, cr4, ti1, ti2, ti3, ti4, tr1, tr2, tr3, tr4;
            size_t ic = ido - i;
            PM(tr2, tr1, CC(i - 1, 0, k), CC(ic - 1, 3, k));
            PM(ti1, ti2, CC(i, 0, k), CC(ic, 3, k));
            PM(tr4, ti3, CC(i, 2, k), CC(ic, 1, k));
            PM(tr3, ti4, CC(i - 1, 2, k), CC(ic - 1, 1, k));
            PM(CH(i - 1, k, 0), cr3, tr2, tr3);
            PM(CH(i, k, 0), ci3, ti2, ti3);
            PM(cr4, cr2, tr1, tr4);
            PM(ci2, ci4, ti1, ti4);
            MULPM(CH(i, k, 1), CH(i - 1, k, 1), WA(0, i - 2), WA(0, i - 1), ci2, cr2);
            MULPM(CH(i, k, 2), CH(i - 1, k, 2), WA(1, i - 2), WA(1, i - 1), ci3, cr3);
            MULPM(CH(i, k, 3), CH(i - 1, k, 3), WA(2, i - 2), WA(2, i - 1), ci4, cr4);
        }
#undef CC
#undef CH
#undef WA
}

/* pocketfft factorisation: N=16 -> [4,4], N=8 -> [2,4].  Only factor 0 carries twiddles. */
static int rf_factors(int n, int fct[2], const double **tw0) {
    if (n == 16) { fct[0] = 4; fct[1] = 4; *tw0 = RF_TW16; return 2; }
    if (n == 8) { fct[0] = 2; fct[1] = 4; *tw0 = RF_TW8; return 2; }
    return 0;
}

/* rfftp::exec(c, fct, r2hc) */
static void rfftp_exec(double *c, int n, double fct, int r2hc) {
    int fac[2]; const double *tw0; int nf = rf_factors(n, fac, &tw0);
    double ch[32];
    double *p1 = c, *p2 = ch, *tmp;
    if (r2hc) {
        size_t l1 = (size_t)n;
        for (int k1 = 0; k1 < nf; ++k1) {
            int k = nf - k1 - 1;
            size_t ip = (size_t)fac[k];
            size_t ido = (size_t)n / l1;
            l1 /= ip;
            const double *tw = (k == 0) ? tw0 : NULL;
            if (ip == 4) radf4(ido, l1, p1, p2, tw); else radf2(ido, l1, p1, p2, tw);
            tmp = p1; p1 = p2; p2 = tmp;
        }
    } else {
        size_t l1 = 1;
        for (int k = 0; k < nf; k++) {
            size_t ip = (size_t)fac[k], ido = (size_t)n / (ip * l1);
            const double *tw = (k == 0) ? tw0 : NULL;
            if (ip == 4) radb4(ido, l1, p1, p2, tw); else radb2(ido, l1, p1, p2, tw);
            tmp = p1; p1 = p2; p2 = tmp;
            l1 *= ip;
        }
    }
    /* copy_and_norm */
    if (p1 != c) {
        if (fct != 1.0) for (int i = 0; i < n; ++i) c[i] = fct * p1[i];
        else for (int i = 0; i < n; ++i) c[i] = p1[i];
    } else if (fct != 1.0) {
        for (int i = 0; i < n; ++i) c[i] *= fct;
    }
}

static double ortho_fct(int n) {  /* T(1/sqrt(2N)) from long double */
    return (double)(1.0L / sqrtl((long double)(2 * n)));
}

/* T_dcst23::exec, type 2, cosine, ortho  == scipy.fftpack.dct(x, norm='ortho') */
EXPORT void oc_dct2_1d(double *c, int n) {
    const double *tw = (n == 16) ? DCT_TW16 : DCT_TW8;
    int ns2 = (n + 1) / 2;
    c[0] *= 2;
    if ((n & 1) == 0) c[n - 1] *= 2;
    for (int k = 1; k < n - 1; k += 2) { double t = c[k + 1]; c[k + 1] -= c[k]; c[k] += t; }
    rfftp_exec(c, n, ortho_fct(n), 0);
    for (int k = 1, kc = n - 1; k < ns2; ++k, --kc) {
        double t1 = tw[k - 1] * c[kc] + tw[kc - 1] * c[k];
        double t2 = tw[k - 1] * c[k] - tw[kc - 1] * c[kc];
        c[k] = 0.5 * (t1 + t2);
        c[kc] = 0.5 * (t1 - t2);
    }
    if ((n & 1) == 0) c[ns2] *= tw[ns2 - 1];
    c[0] *= SQRT2 * 0.5;
}

/* T_dcst23::exec, type 3, cosine, ortho  == scipy.fftpack.idct(x, norm='ortho') */
EXPORT void oc_dct3_1d(double *c, int n) {
    const double *tw = (n == 16) ? DCT_TW16 : DCT_TW8;
    int ns2 = (n + 1) / 2;
    c[0] *= SQRT2;
    for (int k = 1, kc = n - 1; k < ns2; ++k, --kc) {
        double t1 = c[k] + c[kc], t2 = c[k] - c[kc];
        c[k] = tw[k - 1] * t2 + tw[kc - 1] * t1;
        c[kc] = tw[k - 1] * t1 - tw[kc - 1] * t2;
    }
    if ((n & 1) == 0) c[ns2] *= 2 * tw[ns2 - 1];
    rfftp_exec(c, n, ortho_fct(n), 1);
    for (int k = 1; k < n - 1; k += 2) { double t = c[k]; c[k] -= c[k + 1]; c[k + 1] += t; }
}

/* dct(dct(x, axis=0), axis=1) on an n x n row-major block (Encoder.py:781) */
EXPORT void oc_dct2_2d(const double *in, double *out, int n) {
    double v[16];
    memcpy(out, in, sizeof(double) * n * n);
    for (int col = 0; col < n; ++col) {
        for (int r = 0; r < n; ++r) v[r] = out[r * n + col];
        oc_dct2_1d(v, n);
        for (int r = 0; r < n; ++r) out[r * n + col] = v[r];
    }
    for (int row = 0; row < n; ++row) oc_dct2_1d(out + row * n, n);
}

/* idct(idct(x, axis=0), axis=1) (Encoder.py:812) */
EXPORT void oc_idct2_2d(const double *in, double *out, int n) {
    double v[16];
    memcpy(out, in, sizeof(double) * n * n);
    for (int col = 0; col < n; ++col) {
        for (int r = 0; r < n; ++r) v[r] = out[r * n + col];
        oc_dct3_1d(v, n);
        for (int r = 0; r < n; ++r) out[r * n + col] = v[r];
    }
    for (int row = 0; row < n; ++row) oc_dct3_1d(out + row * n, n);
}

/* apply_2d_dct: np.round(...).astype(int) (Encoder.py:779-784) */
EXPORT void oc_apply_2d_dct(const int32_t *res, int32_t *tc, int n) {
    double a[256], b[256];
    for (int i = 0; i < n * n; ++i) a[i] = (double)res[i];
    oc_dct2_2d(a, b, n);
    for (int i = 0; i < n * n; ++i) tc[i] = (int32_t)nearbyint(b[i]);
}

/* apply_2d_idct on rescaled coefficients (Encoder.py:810-817) */
EXPORT void oc_apply_2d_idct(const int32_t *deq, int32_t *out, int n) {
    double a[256], b[256];
    for (int i = 0; i < n * n; ++i) a[i] = (double)deq[i];
    oc_idct2_2d(a, b, n);
    for (int i = 0; i < n * n; ++i) out[i] = (int32_t)nearbyint(b[i]);
}

/* generate_Q_matrix exponent (Encoder.py:938-945): Q[x][y] = 2^(QP + (x+y<i-1 ? 0 : x+y==i-1 ? 1 : 2)) */
static int q_exp(int x, int y, int n, int qp) {
    int s = x + y;
    return qp + (s < n - 1 ? 0 : (s == n - 1 ? 1 : 2));
}

/* quantize_TC: np.round(TC / Q) (Encoder.py:787-789) */
EXPORT void oc_quantize(const int32_t *tc, int16_t *q, int n, int qp) {
    for (int x = 0; x < n; ++x)
        for (int y = 0; y < n; ++y) {
            double qv = ldexp(1.0, q_exp(x, y, n, qp));
            q[x * n + y] = (int16_t)nearbyint((double)tc[x * n + y] / qv);
        }
}

/* rescale_QTC: QTC * Q (Encoder.py:820-821) */
static void dequantize(const int16_t *q, int32_t *deq, int n, int qp) {
    for (int x = 0; x < n; ++x)
        for (int y = 0; y < n; ++y) deq[x * n + y] = (int32_t)q[x * n + y] << q_exp(x, y, n, qp);
}

/* entropy_encoder_block (Encoder.py:1086-1131): returns the token list length and
 * optionally writes the list itself. */
EXPORT int oc_rle(const int16_t *blk, int n, int32_t *out) {
    int len = 0, flag = 1, zero_count = 0, nz_count = 0;
    int32_t nzv[256];
    for (int k = 0; k < 2 * n - 1; ++k) {
        int i, j;
        if (k < n) { i = 0; j = k; } else { i = k - n + 1; j = n - 1; }
        while (i < n && j >= 0) {
            int v = blk[i * n + j];
            if (v != 0) {
                if (flag == 0) {
                    if (zero_count) { if (out) out[len] = zero_count; len++; zero_count = 0; }
                    nz_count = 0;
                    flag = 1;
                }
                nzv[nz_count++] = v;
            } else {
                if (flag == 1) {
                    if (nz_count) {
                        if (out) out[len] = -nz_count;
                        len++;
                        for (int t = 0; t < nz_count; ++t) { if (out) out[len] = nzv[t]; len++; }
                        nz_count = 0;
                    }
                    zero_count = 0;
                    flag = 0;
                }
                zero_count++;
            }
            i++; j--;
        }
    }
    if (nz_count) {
        if (out) out[len] = -nz_count;
        len++;
        for (int t = 0; t < nz_count; ++t) { if (out) out[len] = nzv[t]; len++; }
    }
    if (zero_count) { if (out) out[len] = 0; len++; }
    return len;
}

/* ------------------------------------------------------------------------------------ */
/* Motion estimation, prediction, reconstruction                                         */
/* ------------------------------------------------------------------------------------ */

typedef struct { int dx, dy, ref; long sad; } om_mv;   /* sad < 0 == "inf" */

/* find_best_match (Encoder.py:678-717): refs outer, dx middle, dy inner; strict bound
 * 0 <= x+dx < W-bs and 0 <= y+dy < H-bs on the REFERENCE frame shape; keep if mae <
 * best or (== and (|dx|+|dy|, ref) strictly smaller, is_better_mv :771-773).
 * mae = SAD / bs^2 exactly (power-of-two divisor), so integer SAD compares identically. */
static om_mv find_best_match(const uint8_t *cur, int cstride, const uint8_t *const *refs,
                             int nref, int H, int W, int x, int y, int bs, int sr) {
    om_mv best = {0, 0, 0, -1};
    for (int r = 0; r < nref; ++r) {
        const uint8_t *ref = refs[r];
        for (int dx = -sr; dx <= sr; ++dx)
            for (int dy = -sr; dy <= sr; ++dy) {
                if (!(0 <= x + dx && x + dx < W - bs && 0 <= y + dy && y + dy < H - bs)) continue;
                long sad = 0;
                for (int i = 0; i < bs; ++i)
                    for (int j = 0; j < bs; ++j)
                        sad += labs((long)cur[i * cstride + j] - (long)ref[(y + dy + i) * W + x + dx + j]);
                if (best.sad < 0 || sad < best.sad) {
                    best.dx = dx; best.dy = dy; best.ref = r; best.sad = sad;
                } else if (sad == best.sad) {
                    int l1n = abs(dx) + abs(dy), l1b = abs(best.dx) + abs(best.dy);
                    if (l1n < l1b || (l1n == l1b && r < best.ref)) {
                        best.dx = dx; best.dy = dy; best.ref = r;
                    }
                }
            }
    }
    return best;
}

static int block_tokens(const int16_t *q, int n) { return oc_rle(q, n, NULL); }

/* calculate_RD_cost (Encoder.py:1133-1158) given token counts. */
static double rd_cost(int frame_type, int split, double mae, int tok_total, double lam) {
    int bits;
    if (split == 0) bits = (frame_type == 0 ? 8 : 16) + 8 * tok_total;
    else bits = (frame_type == 0 ? 32 : 64) + 8 * tok_total;
    volatile double lb = lam * (double)bits;   /* keep lam*bits + mae as two roundings */
    return lb + mae;
}

static void tq_block(const int32_t *res, int n, int qp, int16_t *qtc) {
    int32_t tc[256];
    oc_apply_2d_dct(res, tc, n);
    oc_quantize(tc, qtc, n, qp);
}

static inline uint8_t wrap_u8(long v) { return (uint8_t)(v & 255); }

/* ------------------------------------------------------------------------------------ */
/* Fractional (half-pel) ME and fast ME                                                   */
/* ------------------------------------------------------------------------------------ */

/* frac_me_reference_frame (Encoder.py:388-403, decoder.py:468-483): a (2H-1) x (2W-1)
 * frame.  Rows first: each row r becomes [r0, (r0+r1)/2, r1, ..., r_{W-1}] in float; then
 * each column of that the same way, and np.ceil of the result.  Every value is a multiple
 * of 1/4, so in integers:
 *   F[2i][2j]     = r[i][j]
 *   F[2i][2j+1]   = ceil(h(i,j) / 2)             h(i,j) = r[i][j] + r[i][j+1]
 *   F[2i+1][2j]   = ceil((r[i][j] + r[i+1][j]) / 2)
 *   F[2i+1][2j+1] = ceil((h(i,j) + h(i+1,j)) / 4)
 * `wrap`: np.copy(ref_frames) is uint8 when every reference is a uint8 reconstruction, and
 * then `row + np.roll(row, -1)` wraps mod 256 (h &= 255).  The column pass already runs in
 * float64 (the rows were promoted by vstack), so it never wraps.  A list that still holds
 * the float64 all-128 start frame (Encoder.py:1798) is float64: no wrap. */
EXPORT void oc_fme_upsample(const uint8_t *ref, int H, int W, int wrap, uint8_t *out) {
    const int W2 = 2 * W - 1;
    for (int i = 0; i < H; ++i)
        for (int j = 0; j < W; ++j) {
            const int a = ref[(size_t)i * W + j];
            out[(size_t)(2 * i) * W2 + 2 * j] = (uint8_t)a;
            int h0 = 0;
            if (j + 1 < W) {
                h0 = a + ref[(size_t)i * W + j + 1];
                if (wrap) h0 &= 255;
                out[(size_t)(2 * i) * W2 + 2 * j + 1] = (uint8_t)((h0 + 1) >> 1);
            }
            if (i + 1 < H) {
                const int c = ref[(size_t)(i + 1) * W + j];
                out[(size_t)(2 * i + 1) * W2 + 2 * j] = (uint8_t)((a + c + 1) >> 1);
                if (j + 1 < W) {
                    int h1 = c + ref[(size_t)(i + 1) * W + j + 1];
                    if (wrap) h1 &= 255;
                    out[(size_t)(2 * i + 1) * W2 + 2 * j + 1] = (uint8_t)((h0 + h1 + 3) >> 2);
                }
            }
        }
}

/* A search plane: the reference frame itself (step 1) or its frac_me frame (step 2, FME:
 * the block is sampled every other row/column, Encoder.py:699-700). */
typedef struct { const uint8_t *const *p; int H, W, step; } om_planes;

/* Integer SAD of a bs x bs block on a step-1 plane.  Same value as the generic loop below;
 * written over uint8 rows with an int accumulator so gcc vectorises it (psadbw): the large
 * parity fixtures (tests/golden/make_large_fixtures.py, 4K x 120 frames) need it. */
static long plane_sad1(const uint8_t *restrict cur, int cstride, const uint8_t *restrict pl, size_t PW, int bs) {
    int sad = 0;
    if (bs == 16) {
        for (int i = 0; i < 16; ++i) {
            const uint8_t *a = cur + (size_t)i * cstride, *b = pl + (size_t)i * PW;
            for (int j = 0; j < 16; ++j) sad += abs((int)a[j] - (int)b[j]);
        }
        return (long)sad;
    }
    for (int i = 0; i < bs; ++i) {
        const uint8_t *a = cur + (size_t)i * cstride, *b = pl + (size_t)i * PW;
        for (int j = 0; j < bs; ++j) sad += abs((int)a[j] - (int)b[j]);
    }
    return (long)sad;
}

static long plane_sad(const uint8_t *cur, int cstride, const uint8_t *pl, int PW, int X, int Y, int bs,
                      int step) {
    if (step == 1) return plane_sad1(cur, cstride, pl + (size_t)Y * PW + X, (size_t)PW, bs);
    long sad = 0;
    for (int i = 0; i < bs; ++i)
        for (int j = 0; j < bs; ++j)
            sad += labs((long)cur[i * cstride + j] - (long)pl[(size_t)(Y + step * i) * PW + X + step * j]);
    return sad;
}

/* find_best_match (Encoder.py:678-717) incl. the FMEEnable branch (:697-705): at (X, Y)
 * (= 2x, 2y with FME) over dx, dy in [-R, R] (R = 2 sr with FME, :1649); FME candidates
 * also need 0 <= X+dx+2bs < W2-bs (and y), and compare the stride-2 sample. */
static om_mv search_full(const uint8_t *cur, int cstride, om_planes P, int nref, int X, int Y, int bs,
                         int R) {
    om_mv best = {0, 0, 0, -1};
    const int fme = P.step == 2;
    for (int r = 0; r < nref; ++r)
        for (int dx = -R; dx <= R; ++dx)
            for (int dy = -R; dy <= R; ++dy) {
                if (!(0 <= X + dx && X + dx < P.W - bs && 0 <= Y + dy && Y + dy < P.H - bs)) continue;
                if (fme && !(0 <= X + dx + 2 * bs && X + dx + 2 * bs < P.W - bs && 0 <= Y + dy + 2 * bs &&
                             Y + dy + 2 * bs < P.H - bs))
                    continue;
                const long sad = plane_sad(cur, cstride, P.p[r], P.W, X + dx, Y + dy, bs, P.step);
                if (best.sad < 0 || sad < best.sad) {
                    best.dx = dx; best.dy = dy; best.ref = r; best.sad = sad;
                } else if (sad == best.sad) {
                    int l1n = abs(dx) + abs(dy), l1b = abs(best.dx) + abs(best.dy);
                    if (l1n < l1b || (l1n == l1b && r < best.ref)) {
                        best.dx = dx; best.dy = dy; best.ref = r;
                    }
                }
            }
    return best;
}

/* fast_motion_estimation (Encoder.py:719-742): the 3x3 neighbourhood of the predictor
 * mvp over refs[:nref]; a candidate needs the strict bound AND 0 <= X+dx+2bs < W-bs (and
 * y) even without FME (:727); strictly smaller MAE wins (first found, no is_better_mv).
 * Returns (best_mv, best_ref_idx): best_mv = mvp when nothing is valid, and the second
 * value -- used by the caller as the block's MAE -- is the reference INDEX (:742).  Here
 * .sad carries that index. */
static om_mv search_fast(const uint8_t *cur, int cstride, om_planes P, int nref, int X, int Y, int bs,
                         om_mv mvp) {
    om_mv best = {mvp.dx, mvp.dy, mvp.ref, 0};
    long best_sad = -1;
    for (int r = 0; r < nref; ++r)
        for (int dx = mvp.dx - 1; dx <= mvp.dx + 1; ++dx)
            for (int dy = mvp.dy - 1; dy <= mvp.dy + 1; ++dy) {
                if (!(0 <= X + dx && X + dx < P.W - bs && 0 <= Y + dy && Y + dy < P.H - bs)) continue;
                if (!(0 <= X + dx + 2 * bs && X + dx + 2 * bs < P.W - bs && 0 <= Y + dy + 2 * bs &&
                      Y + dy + 2 * bs < P.H - bs))
                    continue;
                const long sad = plane_sad(cur, cstride, P.p[r], P.W, X + dx, Y + dy, bs, P.step);
                if (best_sad < 0 || sad < best_sad) {
                    best_sad = sad;
                    best.dx = dx; best.dy = dy; best.ref = r; best.sad = r;
                }
            }
    return best;
}

/* Prediction of calculate_inter_frame_residual (Encoder.py:432-460) and reconstruct_frame
 * (:831-932) on a search plane, at plane position (px, py), block size bs:
 *   strict bound 0 <= px < W-bs (and y)  -> integer: the bs x bs block;
 *                                           FME: if 0 <= px+ext < W-lim (and y) the
 *                                           stride-2 sample, else all 128;
 *   otherwise handle_boundary_conditions (:750-768): zero-filled contiguous overlap.
 * (ext, lim) = (2bs, bs) in the residual and the unsplit recon; a split sub-block's recon
 * uses (BS, BS) of the FULL block size (:908-909), stricter than its search. */
static void fetch_pred2(const uint8_t *pl, int PH, int PW, int step, int px, int py, int bs, int ext, int lim,
                        int32_t *pred) {
    if (0 <= px && px < PW - bs && 0 <= py && py < PH - bs) {
        if (step == 2) {
            const int ok = 0 <= px + ext && px + ext < PW - lim && 0 <= py + ext && py + ext < PH - lim;
            for (int i = 0; i < bs; ++i)
                for (int j = 0; j < bs; ++j)
                    pred[i * bs + j] = ok ? pl[(size_t)(py + 2 * i) * PW + px + 2 * j] : 128;
        } else {
            for (int i = 0; i < bs; ++i)
                for (int j = 0; j < bs; ++j) pred[i * bs + j] = pl[(size_t)(py + i) * PW + px + j];
        }
        return;
    }
    for (int i = 0; i < bs; ++i)
        for (int j = 0; j < bs; ++j) {
            int yy = py + i, xx = px + j;
            pred[i * bs + j] = (yy >= 0 && yy < PH && xx >= 0 && xx < PW) ? pl[(size_t)yy * PW + xx] : 0;
        }
}

/*
 * One P-frame through complete_inter_flow (Encoder.py:1644-1709): inter_prediction
 * (:462-585), per-block DCT/quant/tokens with the per-row QP (:1665-1697) and
 * reconstruct_frame (:831-932).
 *
 *   cur     : padded current frame, Hp x Wp uint8 (pad_hw values)
 *   refs    : nref reference frames, H x W uint8 (H = Hp, W = Wp required)
 *   qp_rd   : QP in effect during inter_prediction (RD decisions)
 *   qp_row  : per block-row QP (NULL => qp_rd everywhere)
 *   qp_map  : per-block QP (build extension: ROI / two-pass RC, oc_qp_map); overrides qp_row
 *   me_mode : 0 find_best_match (full search);
 *             1 fast_me, serial branch: the predictor is the previous block's mv in raster
 *               order, starting at (0,0,0) (:462, :581), over all nref refs;
 *             2 fast_me under ParallelMode 2 (inter_prediction_parallel :587-676): every
 *               block's predictor is (0,0,0) and nRefFrames is 1 (:589-590, :641-642);
 *               VBS is rejected there (the reference raises NameError on `mvp`, :609)
 *   fme     : FMEEnable: search/predict on frac_me_reference_frame(refs) at (2x, 2y)
 *             with range 2 sr, MVs in half-pel units (:1647-1651)
 *   fme_wrap: the frac frame's uint8 wrap (oc_fme_upsample)
 * outputs (nb = Hp/bs * Wp/bs):
 *   split[nb], mv[nb][4][3], qtc[nb][bs*bs], tokens[nb], mae_num[nb] (MAE*bs*bs as an
 *   integer, -1 = inf), recon[H*W]
 */
EXPORT int oc_inter_frame_ex(const uint8_t *cur, int Hp, int Wp, const uint8_t *const *refs,
                             int nref, int H, int W, int bs, int sr, int qp_rd,
                             const int32_t *qp_row, const int32_t *qp_map, int vbs, double lam, int me_mode, int fme,
                             int fme_wrap, uint8_t *split, int16_t *mv, int16_t *qtc,
                             int32_t *tokens, int64_t *mae_num, uint8_t *recon) {
    if (bs != 16 && bs != 8) return -1;
    if (H != Hp || W != Wp) return -2;
    if (me_mode == 2 && vbs) return -3;
    const int sb = bs / 2, nbx = Wp / bs, nby = Hp / bs, bb = bs * bs;
    int32_t res[256], pred[256], deq[256], idc[256];
    int16_t qfull[256], qsub[4][64];
    uint8_t *up[SO_ORACLE_MAX_REF] = {0};
    om_planes P = {refs, H, W, 1};
    if (fme) {
        for (int r = 0; r < nref; ++r) {
            up[r] = (uint8_t *)malloc((size_t)(2 * H - 1) * (2 * W - 1));
            oc_fme_upsample(refs[r], H, W, fme_wrap, up[r]);
        }
        P.p = (const uint8_t *const *)up;
        P.H = 2 * H - 1; P.W = 2 * W - 1; P.step = 2;
    }
    const int k = fme ? 2 : 1;            /* block origin scale on the search plane */
    const int R = fme ? 2 * sr : sr;
    const int nref_fast = me_mode == 2 ? 1 : nref;
    om_mv mvp = {0, 0, 0, 0};
    memset(recon, 0, (size_t)H * W);
    for (int by = 0; by < nby; ++by)
        for (int bx = 0; bx < nbx; ++bx) {
            const int b = by * nbx + bx, x = bx * bs, y = by * bs;
            const uint8_t *cb = cur + (size_t)y * Wp + x;
            const int qpr = qp_map ? qp_map[b] : (qp_row ? qp_row[by] : qp_rd);
            const int eligible = vbs && x != 0 && y != 0;
            if (me_mode == 2) { mvp.dx = 0; mvp.dy = 0; mvp.ref = 0; }
            om_mv sm[4];
            long vbs_sum = 0; int vbs_inf = 0;
            int32_t sres[4][64];
            if (eligible) {
                for (int j = 0; j < 4; ++j) {
                    int xs = x + (j & 1) * sb, ys = y + (j >> 1) * sb;
                    const uint8_t *cs = cur + (size_t)ys * Wp + xs;
                    if (me_mode) {
                        sm[j] = search_fast(cs, Wp, P, nref_fast, k * xs, k * ys, sb, mvp);
                        vbs_sum += sm[j].sad * sb * sb;     /* "mae" = ref index */
                    } else {
                        sm[j] = search_full(cs, Wp, P, nref, k * xs, k * ys, sb, R);
                        if (sm[j].sad < 0) vbs_inf = 1; else vbs_sum += sm[j].sad;
                    }
                    fetch_pred2(P.p[sm[j].ref], P.H, P.W, P.step, k * xs + sm[j].dx, k * ys + sm[j].dy, sb, 2 * sb, sb,
                                pred);
                    for (int i = 0; i < sb; ++i)
                        for (int q = 0; q < sb; ++q)
                            sres[j][i * sb + q] = (int32_t)cb[(size_t)((j >> 1) * sb + i) * Wp + (j & 1) * sb + q] - pred[i * sb + q];
                }
            }
            om_mv m;
            long mae_b_num;          /* MAE * bb */
            int m_inf = 0;
            if (me_mode) {
                m = search_fast(cb, Wp, P, nref_fast, k * x, k * y, bs, mvp);
                mae_b_num = m.sad * bb;
            } else {
                m = search_full(cb, Wp, P, nref, k * x, k * y, bs, R);
                m_inf = m.sad < 0;
                mae_b_num = m.sad;
            }
            int32_t fpred[256];
            fetch_pred2(P.p[m.ref], P.H, P.W, P.step, k * x + m.dx, k * y + m.dy, bs, 2 * bs, bs, fpred);
            for (int i = 0; i < bb; ++i) res[i] = (int32_t)cb[(size_t)(i / bs) * Wp + i % bs] - fpred[i];
            int do_split = 0;
            if (eligible) {
                const int qpm1_rd = qp_rd > 0 ? qp_rd - 1 : qp_rd;
                tq_block(res, bs, qp_rd, qfull);
                int tok_b = block_tokens(qfull, bs), tok_v = 0;
                for (int j = 0; j < 4; ++j) { tq_block(sres[j], sb, qpm1_rd, qsub[j]); tok_v += block_tokens(qsub[j], sb); }
                double mae_b = m_inf ? INFINITY : (double)mae_b_num / bb;
                double mae_v = vbs_inf ? INFINITY : ((double)vbs_sum / (sb * sb)) / 4.0;
                double c_v = rd_cost(1, 1, mae_v, tok_v, lam);
                double c_b = rd_cost(1, 0, mae_b, tok_b, lam);
                do_split = !(c_b < c_v);
                mae_num[b] = vbs_inf ? -1 : vbs_sum;   /* mae = vbs_mae (:575) */
            } else {
                mae_num[b] = m_inf ? -1 : mae_b_num;
            }
            if (me_mode == 1) mvp = m;              /* mvp = mv (:581), the full block's */
            split[b] = (uint8_t)do_split;
            int16_t *mvb = mv + (size_t)b * 12;
            memset(mvb, 0, 12 * sizeof(int16_t));
            int16_t *qb = qtc + (size_t)b * bb;
            if (!do_split) {
                mvb[0] = (int16_t)m.dx; mvb[1] = (int16_t)m.dy; mvb[2] = (int16_t)m.ref;
                tq_block(res, bs, qpr, qb);
                tokens[b] = block_tokens(qb, bs);
                dequantize(qb, deq, bs, qpr);
                oc_apply_2d_idct(deq, idc, bs);
                for (int i = 0; i < bs; ++i)
                    for (int q = 0; q < bs; ++q)
                        recon[(size_t)(y + i) * W + x + q] = wrap_u8((long)fpred[i * bs + q] + idc[i * bs + q]);
            } else {
                const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
                int tk = 0;
                for (int j = 0; j < 4; ++j) {
                    mvb[3 * j] = (int16_t)sm[j].dx; mvb[3 * j + 1] = (int16_t)sm[j].dy; mvb[3 * j + 2] = (int16_t)sm[j].ref;
                    int16_t *qs = qb + j * sb * sb;
                    tq_block(sres[j], sb, qpm1, qs);
                    tk += block_tokens(qs, sb);
                    int xs = x + (j & 1) * sb, ys = y + (j >> 1) * sb;
                    fetch_pred2(P.p[sm[j].ref], P.H, P.W, P.step, k * xs + sm[j].dx, k * ys + sm[j].dy, sb, bs, bs,
                                pred);
                    dequantize(qs, deq, sb, qpm1);
                    oc_apply_2d_idct(deq, idc, sb);
                    for (int i = 0; i < sb; ++i)
                        for (int q = 0; q < sb; ++q)
                            recon[(size_t)(ys + i) * W + xs + q] = wrap_u8((long)pred[i * sb + q] + idc[i * sb + q]);
                }
                tokens[b] = tk;
            }
        }
    for (int r = 0; r < nref; ++r) free(up[r]);
    return 0;
}

EXPORT int oc_inter_frame(const uint8_t *cur, int Hp, int Wp, const uint8_t *const *refs,
                          int nref, int H, int W, int bs, int sr, int qp_rd,
                          const int32_t *qp_row, int vbs, double lam, uint8_t *split,
                          int16_t *mv, int16_t *qtc, int32_t *tokens, int64_t *mae_num,
                          uint8_t *recon) {
    return oc_inter_frame_ex(cur, Hp, Wp, refs, nref, H, W, bs, sr, qp_rd, qp_row, NULL, vbs, lam, 0, 0, 0, split, mv,
                             qtc, tokens, mae_num, recon);
}

/* intra_find_best_match_horizontal (Encoder.py:1010-1045) on the in-loop canvas, which
 * equals the ORIGINAL pixels left of the block's column bx0 and 128 from bx0 on
 * (intra_prediction writes pred + unquantised residual == original, :1329-1338).
 * Tie rule: mae == best and |dx| <= |best| replaces => last-found among min (SAD, |dx|). */
static void intra_search(const uint8_t *cur, int Wp, int x, int y, int bx0, int bs, int sr,
                         int *best_mv, long *best_sad, int32_t *res) {
    long best = -1; int bm = 0;
    if (x == 0) {
        long s = 0;
        for (int i = 0; i < bs; ++i)
            for (int j = 0; j < bs; ++j) {
                int v = (int)cur[(size_t)(y + i) * Wp + x + j] - 128;
                s += labs(v);
                if (res) res[i * bs + j] = v;
            }
        *best_mv = -1; *best_sad = s;
        return;
    }
    for (int dx = -sr; dx <= sr; ++dx) {
        if (!(x + dx >= 0 && x + dx + bs <= Wp)) continue;
        long s = 0;
        for (int i = 0; i < bs; ++i)
            for (int j = 0; j < bs; ++j) {
                int cx = x + dx + j;
                int rv = cx < bx0 ? cur[(size_t)(y + i) * Wp + cx] : 128;
                s += labs((long)cur[(size_t)(y + i) * Wp + x + j] - rv);
            }
        if (best < 0 || s < best) { best = s; bm = dx; }
        else if (s == best && abs(dx) <= abs(bm)) { bm = dx; }
    }
    *best_mv = bm; *best_sad = best;
    if (res) {
        for (int i = 0; i < bs; ++i)
            for (int j = 0; j < bs; ++j) {
                int cx = x + bm + j;
                int rv = cx < bx0 ? cur[(size_t)(y + i) * Wp + cx] : 128;
                res[i * bs + j] = (int)cur[(size_t)(y + i) * Wp + x + j] - rv;
            }
    }
}

/*
 * One I-frame through complete_intra_flow (Encoder.py:1582-1642), intra_mode 0:
 * intra_prediction (:1238-1347, canvas generalised to Hp x Wp), per-block DCT/quant/
 * tokens with per-row QP, reconstruct_frame_intra (:1350-1417; unclipped float canvas,
 * final astype(uint8) == mod-256 wrap).
 * mv[nb][4]: dx per (sub-)block, -1 for x == 0.
 */
EXPORT int oc_intra_frame_ex(const uint8_t *cur, int Hp, int Wp, int bs, int sr, int qp_rd,
                             const int32_t *qp_row, const int32_t *qp_map, int vbs, double lam,
                             uint8_t *split, int16_t *mv, int16_t *qtc, int32_t *tokens,
                             int64_t *mae_num, uint8_t *recon) {
    if (bs != 16 && bs != 8) return -1;
    const int sb = bs / 2, nbx = Wp / bs, nby = Hp / bs, bb = bs * bs;
    int32_t res[256], sres[4][64], deq[256];
    int16_t qfull[256], qsub[4][64];
    int32_t *idres = (int32_t *)malloc(sizeof(int32_t) * (size_t)nbx * nby * bb);
    for (int by = 0; by < nby; ++by)
        for (int bx = 0; bx < nbx; ++bx) {
            const int b = by * nbx + bx, x = bx * bs, y = by * bs;
            const int qpr = qp_map ? qp_map[(size_t)by * nbx + bx] : (qp_row ? qp_row[by] : qp_rd);
            const int eligible = vbs && x != 0 && y != 0;
            int smv[4]; long ssad[4]; long vsum = 0;
            if (eligible)
                for (int j = 0; j < 4; ++j) {
                    int xs = x + (j & 1) * sb, ys = y + (j >> 1) * sb;
                    intra_search(cur, Wp, xs, ys, x, sb, sr, &smv[j], &ssad[j], sres[j]);
                    vsum += ssad[j];
                }
            int m; long msad;
            intra_search(cur, Wp, x, y, x, bs, sr, &m, &msad, res);
            int do_split = 0;
            if (eligible) {
                const int qpm1_rd = qp_rd > 0 ? qp_rd - 1 : qp_rd;
                tq_block(res, bs, qp_rd, qfull);
                int tok_b = block_tokens(qfull, bs), tok_v = 0;
                for (int j = 0; j < 4; ++j) { tq_block(sres[j], sb, qpm1_rd, qsub[j]); tok_v += block_tokens(qsub[j], sb); }
                double mae_b = (double)msad / bb;
                double mae_v = ((double)vsum / (sb * sb)) / 4.0;
                double c_v = rd_cost(0, 1, mae_v, tok_v, lam);
                double c_b = rd_cost(0, 0, mae_b, tok_b, lam);
                do_split = !(c_b < c_v);
                mae_num[b] = vsum;
            } else {
                mae_num[b] = msad;
            }
            split[b] = (uint8_t)do_split;
            int16_t *mvb = mv + (size_t)b * 4;
            int16_t *qb = qtc + (size_t)b * bb;
            int32_t *rb = idres + (size_t)b * bb;
            if (!do_split) {
                mvb[0] = (int16_t)m; mvb[1] = mvb[2] = mvb[3] = 0;
                tq_block(res, bs, qpr, qb);
                tokens[b] = block_tokens(qb, bs);
                dequantize(qb, deq, bs, qpr);
                oc_apply_2d_idct(deq, rb, bs);
            } else {
                const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
                int tk = 0;
                for (int j = 0; j < 4; ++j) {
                    mvb[j] = (int16_t)smv[j];
                    int16_t *qs = qb + j * sb * sb;
                    tq_block(sres[j], sb, qpm1, qs);
                    tk += block_tokens(qs, sb);
                    dequantize(qs, deq, sb, qpm1);
                    oc_apply_2d_idct(deq, rb + j * sb * sb, sb);
                }
                tokens[b] = tk;
            }
        }
    /* reconstruct_frame_intra, mode 0: row-sequential on an unclipped canvas */
    long *canvas = (long *)malloc(sizeof(long) * (size_t)Hp * Wp);
    for (size_t i = 0; i < (size_t)Hp * Wp; ++i) canvas[i] = 128;
    long blk[256];
    for (int by = 0; by < nby; ++by)
        for (int bx = 0; bx < nbx; ++bx) {
            const int b = by * nbx + bx, x = bx * bs, y = by * bs;
            const int32_t *rb = idres + (size_t)b * bb;
            const int16_t *mvb = mv + (size_t)b * 4;
            if (x == 0) {
                for (int i = 0; i < bb; ++i) blk[i] = 128 + rb[i];
            } else if (!split[b]) {
                for (int i = 0; i < bs; ++i)
                    for (int k = 0; k < bs; ++k)
                        blk[i * bs + k] = canvas[(size_t)(y + i) * Wp + x + mvb[0] + k] + rb[i * bs + k];
            } else {
                for (int j = 0; j < 4; ++j) {
                    int oy = (j >> 1) * sb, ox = (j & 1) * sb;
                    for (int i = 0; i < sb; ++i)
                        for (int k = 0; k < sb; ++k)
                            blk[(oy + i) * bs + ox + k] =
                                canvas[(size_t)(y + oy + i) * Wp + x + ox + mvb[j] + k] + rb[j * sb * sb + i * sb + k];
                }
            }
            for (int i = 0; i < bs; ++i)
                for (int k = 0; k < bs; ++k) canvas[(size_t)(y + i) * Wp + x + k] = blk[i * bs + k];
        }
    for (size_t i = 0; i < (size_t)Hp * Wp; ++i) recon[i] = wrap_u8(canvas[i]);
    free(canvas);
    free(idres);
    return 0;
}

/* Decoder inter recon (decoder.py:97-211 == reconstruct_frame :831-932), with the FME
 * branch (frac frames of the references, half-pel MVs; decoder.py:102-103, 121-141,
 * 168-187): `fme_wrap` as in oc_fme_upsample. */
EXPORT int oc_intra_frame(const uint8_t *cur, int Hp, int Wp, int bs, int sr, int qp_rd,
                          const int32_t *qp_row, int vbs, double lam, uint8_t *split,
                          int16_t *mv, int16_t *qtc, int32_t *tokens, int64_t *mae_num,
                          uint8_t *recon) {
    return oc_intra_frame_ex(cur, Hp, Wp, bs, sr, qp_rd, qp_row, NULL, vbs, lam, split, mv, qtc, tokens, mae_num,
                             recon);
}

EXPORT int oc_inter_recon_ex(const uint8_t *const *refs, int nref, int H, int W, int bs, int qp_rd,
                             const int32_t *qp_row, const int32_t *qp_map, int fme, int fme_wrap, const uint8_t *split,
                             const int16_t *mv, const int16_t *qtc, uint8_t *recon) {
    const int sb = bs / 2, nbx = W / bs, nby = H / bs, bb = bs * bs;
    int32_t pred[256], deq[256], idc[256];
    uint8_t *up[SO_ORACLE_MAX_REF] = {0};
    om_planes P = {refs, H, W, 1};
    if (fme) {
        for (int r = 0; r < nref; ++r) {
            up[r] = (uint8_t *)malloc((size_t)(2 * H - 1) * (2 * W - 1));
            oc_fme_upsample(refs[r], H, W, fme_wrap, up[r]);
        }
        P.p = (const uint8_t *const *)up;
        P.H = 2 * H - 1; P.W = 2 * W - 1; P.step = 2;
    }
    const int k = fme ? 2 : 1;
    memset(recon, 0, (size_t)H * W);
    for (int by = 0; by < nby; ++by)
        for (int bx = 0; bx < nbx; ++bx) {
            const int b = by * nbx + bx, x = bx * bs, y = by * bs;
            const int qpr = qp_map ? qp_map[b] : (qp_row ? qp_row[by] : qp_rd);
            const int16_t *mvb = mv + (size_t)b * 12;
            const int16_t *qb = qtc + (size_t)b * bb;
            if (!split[b]) {
                fetch_pred2(P.p[mvb[2]], P.H, P.W, P.step, k * x + mvb[0], k * y + mvb[1], bs, 2 * bs, bs, pred);
                dequantize(qb, deq, bs, qpr);
                oc_apply_2d_idct(deq, idc, bs);
                for (int i = 0; i < bs; ++i)
                    for (int q = 0; q < bs; ++q)
                        recon[(size_t)(y + i) * W + x + q] = wrap_u8((long)pred[i * bs + q] + idc[i * bs + q]);
            } else {
                const int qpm1 = qpr > 0 ? qpr - 1 : qpr;
                for (int j = 0; j < 4; ++j) {
                    int xs = x + (j & 1) * sb, ys = y + (j >> 1) * sb;
                    fetch_pred2(P.p[mvb[3 * j + 2]], P.H, P.W, P.step, k * xs + mvb[3 * j], k * ys + mvb[3 * j + 1],
                                sb, bs, bs, pred);
                    dequantize(qb + j * sb * sb, deq, sb, qpm1);
                    oc_apply_2d_idct(deq, idc, sb);
                    for (int i = 0; i < sb; ++i)
                        for (int q = 0; q < sb; ++q)
                            recon[(size_t)(ys + i) * W + xs + q] = wrap_u8((long)pred[i * sb + q] + idc[i * sb + q]);
                }
            }
        }
    for (int r = 0; r < nref; ++r) free(up[r]);
    return 0;
}

EXPORT int oc_inter_recon(const uint8_t *const *refs, int H, int W, int bs, int qp_rd,
                          const int32_t *qp_row, const uint8_t *split, const int16_t *mv,
                          const int16_t *qtc, uint8_t *recon) {
    int nref = 0;   /* the MVs name their reference; the plain path never upsamples */
    return oc_inter_recon_ex(refs, nref, H, W, bs, qp_rd, qp_row, NULL, 0, 0, split, mv, qtc, recon);
}

/* sum of squared differences for PSNR (Encoder.py:934-935) */
EXPORT int64_t oc_sse_u8(const uint8_t *a, const uint8_t *b, int64_t n) {
    int64_t s = 0;
    for (int64_t i = 0; i < n; ++i) { int64_t d = (int64_t)a[i] - b[i]; s += d * d; }
    return s;
}

/* find_best_match for one block (Encoder.py:678-717); out = (dx, dy, ref, sad or -1) */
EXPORT void oc_me_block(const uint8_t *cur, int cstride, const uint8_t *const *refs, int nref, int H,
                        int W, int x, int y, int bs, int sr, int32_t *out) {
    om_mv m = find_best_match(cur + (size_t)y * cstride + x, cstride, refs, nref, H, W, x, y, bs, sr);
    out[0] = m.dx; out[1] = m.dy; out[2] = m.ref; out[3] = (int32_t)m.sad;
}

/* Per-block QP map of ROI / two-pass rate control (build extension; restates
 * so_capi.hip qp_map_kernel): tokens = pass-1 token counts [nby*nbx] or NULL,
 * roi = offsets [nby*nbx] or NULL. */
EXPORT void oc_qp_map(const int32_t *tokens, int nbx, int nby, int qp_rd, const int32_t *qp_row,
                      const int32_t *roi, int qp_lo, int qp_hi, int32_t *out) {
    for (int by = 0; by < nby; ++by) {
        long long m = 0;
        if (tokens)
            for (int bx = 0; bx < nbx; ++bx) m += tokens[(size_t)by * nbx + bx];
        const int base = qp_row ? qp_row[by] : qp_rd;
        for (int bx = 0; bx < nbx; ++bx) {
            int d = 0;
            if (tokens) {
                const long long tn = (long long)tokens[(size_t)by * nbx + bx] * nbx;
                d = (tn >= 2 * m) + (tn >= 4 * m) - (2 * tn < m) - (4 * tn < m);
            }
            int q = base + d + (roi ? roi[(size_t)by * nbx + bx] : 0);
            q = q < qp_lo ? qp_lo : (q > qp_hi ? qp_hi : q);
            out[(size_t)by * nbx + bx] = q;
        }
    }
}
