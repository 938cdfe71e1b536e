// so_common.h — shared definitions for the StreamOptima MI355X (gfx950) kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/streamoptima.h"

#ifndef SO_DEV
#define SO_DEV __device__ __forceinline__
#endif

namespace so {

// Thread-local last error message (so_last_error()).
void set_error(const char* fmt, ...);

// The current value of a process-wide option (so_set_option, SO_OPT_*).
int option(int id);

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error("%s: %s", what, hipGetErrorString(e));
        return (int)e;
    }
    return SO_OK;
}

// Maximum reference frames carried in a kernel argument (nRefFrames, Encoder.py:24).
constexpr int kMaxRef = SO_MAX_REF;

struct RefSet {
    const uint8_t* p[kMaxRef];
};

// Anti-diagonal scan position of (i, j) in an n x n block (entropy_encoder_block,
// Encoder.py:1095-1123): diagonal k = i + j; inside a diagonal i increases.
constexpr int scan_pos(int n, int i, int j) {
    int k = i + j, before = 0;
    for (int d = 0; d < k; ++d) before += (d < n) ? d + 1 : 2 * n - 1 - d;
    int first_i = (k < n) ? 0 : k - n + 1;
    return before + (i - first_i);
}

// Q-matrix exponent (generate_Q_matrix, Encoder.py:938-945).
SO_DEV int q_exp(int x, int y, int n, int qp) {
    int s = x + y;
    return qp + (s < n - 1 ? 0 : (s == n - 1 ? 1 : 2));
}

// np.round(TC / 2^k) with TC integral: exact round-half-to-even in integer arithmetic.
SO_DEV int quant_rne(int tc, int k) {
    if (k <= 0) return tc;
    int a = tc < 0 ? -tc : tc;
    int q = a >> k;
    int rem = a & ((1 << k) - 1);
    int half = 1 << (k - 1);
    q += (rem > half) || (rem == half && (q & 1));
    return tc < 0 ? -q : q;
}

}  // namespace so
