// Host build of the device DCT header (streamoptima_amd/csrc/so_dct.h) checked bit for bit
// against the C oracle's pocketfft restatement (oracle/so_oracle.c oc_dct2_1d / oc_dct3_1d)
// on random and tie-heavy integer vectors.  Built and run by tests/test_host.py (CPU):
//   hipcc -O2 -ffp-contract=off -x c++ dct_host_check.cpp -L oracle/_build -lso_oracle
// Exit status 0 = every output identical.
#define SO_DEV inline
#include "../../streamoptima_amd/csrc/so_dct.h"

#include <stdint.h>
#include <stdio.h>
#include <string.h>

extern "C" void oc_dct2_1d(double* c, int n);
extern "C" void oc_dct3_1d(double* c, int n);

static uint64_t rng = 0x9E3779B97F4A7C15ull;
static uint64_t next() {
    rng += 0x9E3779B97F4A7C15ull;
    uint64_t z = rng;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

template <int N>
static long check(long iters) {
    long bad = 0;
    for (long it = 0; it < iters; ++it) {
        double a[N], b[N];
        const int mode = (int)(it % 4);
        for (int i = 0; i < N; ++i) {
            int64_t v;
            if (mode == 0) v = (int64_t)(next() % 511) - 255;                  // residual range
            else if (mode == 1) v = ((int64_t)(next() % 9) - 4) * 40;           // tie-heavy levels
            else if (mode == 2) v = ((int64_t)(next() % 33) - 16) << (next() % 8);  // dequantised
            else v = (int64_t)(next() % 8161) - 4080;                           // TC range
            a[i] = b[i] = (double)v;
        }
        const bool inv = (it / 4) % 2;
        if (inv) { so::dct::dct3<N>(a); oc_dct3_1d(b, N); }
        else { so::dct::dct2<N>(a); oc_dct2_1d(b, N); }
        if (memcmp(a, b, sizeof a) != 0) {
            if (bad < 5) fprintf(stderr, "N=%d it=%ld %s mismatch\n", N, it, inv ? "dct3" : "dct2");
            ++bad;
        }
    }
    return bad;
}

int main(int argc, char** argv) {
    const long iters = argc > 1 ? atol(argv[1]) : 200000;
    const long b16 = check<16>(iters), b8 = check<8>(iters);
    printf("dct host check: N=16 %ld/%ld, N=8 %ld/%ld mismatches\n", b16, iters, b8, iters);
    return (b16 || b8) ? 1 : 0;
}
