// Host check: dct2_16_i / dct3_16_i / dct2_8_i / dct3_8_i (so_dct.h) against dct2<N> / dct3<N> on the same
// integers converted to double -- bit for bit.
//   hipcc -O2 -ffp-contract=off -DSO_DEV=inline tools/check_dct_int.cpp -o /tmp/check_dct_int && /tmp/check_dct_int
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <random>

#include "../streamoptima_amd/csrc/so_dct.h"

int main() {
    std::mt19937_64 rng(12345);
    long bad2 = 0, bad3 = 0, n = 0;
    for (int it = 0; it < 4000000; ++it) {
        int x[16];
        const int mode = it % 4;
        for (int i = 0; i < 16; ++i) {
            if (mode == 0) x[i] = (int)(rng() % 511) - 255;                         // residuals
            else if (mode == 1) x[i] = (rng() & 1) ? 255 : -255;                    // extremes
            else if (mode == 2) x[i] = ((int)(rng() % 401) - 200) * (1 << (rng() % 8));   // dequantised
            else x[i] = (int)(rng() % 131071) - 65535;
        }
        double a[16], b[16];
        for (int i = 0; i < 16; ++i) a[i] = (double)x[i];
        so::dct::dct2<16>(a);
        so::dct::dct2_16_i(x, b);
        if (std::memcmp(a, b, sizeof a)) ++bad2;
        for (int i = 0; i < 16; ++i) a[i] = (double)x[i];
        so::dct::dct3<16>(a);
        so::dct::dct3_16_i(x, b);
        if (std::memcmp(a, b, sizeof a)) ++bad3;
        int x8[8];
        for (int i = 0; i < 8; ++i) x8[i] = x[i] + x[i + 8];
        double a8[8], b8[8];
        for (int i = 0; i < 8; ++i) a8[i] = (double)x8[i];
        so::dct::dct2<8>(a8);
        so::dct::dct2_8_i(x8, b8);
        if (std::memcmp(a8, b8, sizeof a8)) ++bad2;
        for (int i = 0; i < 8; ++i) a8[i] = (double)x8[i];
        so::dct::dct3<8>(a8);
        so::dct::dct3_8_i(x8, b8);
        if (std::memcmp(a8, b8, sizeof a8)) ++bad3;
        ++n;
    }
    std::printf("vectors %ld  dct2 mismatches %ld  dct3 mismatches %ld\n", n, bad2, bad3);
    return (bad2 || bad3) ? 1 : 0;
}
