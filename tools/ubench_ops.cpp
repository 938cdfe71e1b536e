// Microbenchmark: VALU issue cost on gfx950 by instruction and operand kind.
//   sad_vvv   v_sad_u8 v_acc, v_a[i], v_b[i], v_acc      (3 distinct VGPR sources)
//   sad_vsv   v_sad_u8 v_acc, v_a[i], s_b, v_acc         (one SGPR source)
//   sad_vsv4  as sad_vsv with 4 different SGPRs rotating
//   add3_vvv  v_add3_u32 with 3 distinct VGPR sources
//   add_vv    v_add_u32 (2 VGPR sources)
//   align_vvs v_alignbyte_b32 v, v_a[i], v_b[i], s_sh
// NACC independent accumulators per lane; loop body = the instruction under test.
// hipcc --offload-arch=gfx950 -O3 tools/ubench_ops.cpp -o tools/ubench_ops
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITER 1024
#define NACC 16

#define KERNEL(NAME, BODY)                                                                    \
    __global__ void NAME(const uint32_t* in, uint32_t* out, int n_iter, uint32_t s0, uint32_t s1, \
                         uint32_t s2, uint32_t s3) {                                         \
        uint32_t a[NACC], b[NACC], acc[NACC];                                                \
        _Pragma("unroll") for (int i = 0; i < NACC; ++i) {                                   \
            a[i] = in[threadIdx.x + i + 1];                                                  \
            b[i] = in[threadIdx.x + 2 * i + 3];                                              \
            acc[i] = i;                                                                      \
        }                                                                                    \
        const uint32_t sv[4] = {s0, s1, s2, s3};                                             \
        (void)sv;                                                                            \
        for (int it = 0; it < n_iter; ++it) {                                                \
            _Pragma("unroll") for (int i = 0; i < NACC; ++i) { BODY; }                       \
        }                                                                                    \
        uint32_t s = 0;                                                                      \
        _Pragma("unroll") for (int i = 0; i < NACC; ++i) s += acc[i];                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                      \
    }

KERNEL(k_sad_vvv, acc[i] = __builtin_amdgcn_sad_u8(a[i], b[i], acc[i]))
KERNEL(k_sad_vsv, acc[i] = __builtin_amdgcn_sad_u8(a[i], s0, acc[i]))
KERNEL(k_sad_vsv4, acc[i] = __builtin_amdgcn_sad_u8(a[i], sv[i & 3], acc[i]))
KERNEL(k_add3_vvv, asm volatile("v_add3_u32 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a[i]), "v"(b[i])))
KERNEL(k_add_vv, acc[i] = acc[i] + a[i])
KERNEL(k_align_vvs, acc[i] = __builtin_amdgcn_alignbyte(a[i], acc[i], s0))

// FP64 VALU (the pocketfft-exact transforms): is a wave64 v_add/mul/fma_f64 4 cycles?
#define KERNELD(NAME, BODY)                                                                   \
    __global__ void NAME(const uint32_t* in, uint32_t* out, int n_iter, uint32_t s0, uint32_t s1, \
                         uint32_t s2, uint32_t s3) {                                         \
        double a[NACC], b[NACC], acc[NACC];                                                  \
        _Pragma("unroll") for (int i = 0; i < NACC; ++i) {                                   \
            a[i] = 1.0 + 1e-9 * in[threadIdx.x + i + 1];                                     \
            b[i] = 1e-9 * in[threadIdx.x + 2 * i + 3];                                       \
            acc[i] = i;                                                                      \
        }                                                                                    \
        for (int it = 0; it < n_iter; ++it) {                                                \
            _Pragma("unroll") for (int i = 0; i < NACC; ++i) { BODY; }                       \
        }                                                                                    \
        double s = 0;                                                                        \
        _Pragma("unroll") for (int i = 0; i < NACC; ++i) s += acc[i];                        \
        out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s;                            \
    }
KERNELD(k_add_f64, acc[i] = acc[i] + a[i])
KERNELD(k_mul_f64, acc[i] = acc[i] * a[i])
KERNELD(k_fma_f64, acc[i] = __builtin_fma(acc[i], a[i], b[i]))
KERNELD(k_rndne_f64, acc[i] = __builtin_rint(acc[i] + b[i]))

template <typename K>
static void run(K kern, const char* name, int blocks, int threads, uint32_t* din, uint32_t* dout) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, N_ITER, 1u, 2u, 3u, 5u);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r)
        hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, N_ITER, 1u, 2u, 3u, 5u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double instr = 5.0 * blocks * (threads / 64) * (double)N_ITER * NACC;
    const double per_s = instr / (ms * 1e-3);
    printf("%-10s %8.3f ms  %.3e wave-instr/s  -> %.2f cycles/wave-instr/SIMD @2.4GHz\n", name, ms, per_s,
           1024 * 2.4e9 / per_s);
}

int main() {
    uint32_t *din, *dout;
    (void)hipMalloc(&din, 8192 * 4);
    (void)hipMalloc(&dout, 1 << 24);
    (void)hipMemset(din, 7, 8192 * 4);
    for (int waves_per_simd : {2, 4, 8}) {
        const int threads = 256, blocks = 256 * waves_per_simd;
        printf("-- %d waves/SIMD\n", waves_per_simd);
        run(k_sad_vvv, "sad_vvv", blocks, threads, din, dout);
        run(k_sad_vsv, "sad_vsv", blocks, threads, din, dout);
        run(k_sad_vsv4, "sad_vsv4", blocks, threads, din, dout);
        run(k_add3_vvv, "add3_vvv", blocks, threads, din, dout);
        run(k_add_vv, "add_vv", blocks, threads, din, dout);
        run(k_align_vvs, "align_vvs", blocks, threads, din, dout);
        run(k_add_f64, "add_f64", blocks, threads, din, dout);
        run(k_mul_f64, "mul_f64", blocks, threads, din, dout);
        run(k_fma_f64, "fma_f64", blocks, threads, din, dout);
        run(k_rndne_f64, "add+rndne", blocks, threads, din, dout);
    }
    return 0;
}
