// Microbenchmark: VALU issue cost per wave64 instruction on gfx950 for the instruction kinds
// a block transform can be built from (FP64 scalar, FP32 scalar and packed, int32), at 2 / 4 / 8
// waves per SIMD.  Each lane runs NACC independent chains; the loop body is the instruction
// under test (inline asm, so the compiler cannot fold or re-associate it).
// hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.cpp -o tools/ubench_valu && tools/ubench_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITER 512
#define NACC 16

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ inline f2 F2(float x, float y) { f2 v; v.x = x; v.y = y; return v; }

#define KERNEL(NAME, T, INIT_A, INIT_ACC, BODY, FOLD)                                           \
    __global__ void NAME(const uint32_t* in, uint32_t* out, int n_iter) {                       \
        T a[NACC], acc[NACC];                                                                   \
        _Pragma("unroll") for (int i = 0; i < NACC; ++i) {                                      \
            const uint32_t u = in[threadIdx.x + i + 1];                                         \
            a[i] = INIT_A;                                                                      \
            acc[i] = INIT_ACC;                                                                  \
        }                                                                                       \
        for (int it = 0; it < n_iter; ++it) {                                                   \
            _Pragma("unroll") for (int i = 0; i < NACC; ++i) { BODY; }                          \
        }                                                                                       \
        uint32_t s = 0;                                                                         \
        _Pragma("unroll") for (int i = 0; i < NACC; ++i) s += FOLD;                             \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                         \
    }

KERNEL(k_add_u32, uint32_t, u, (uint32_t)i, asm volatile("v_add_u32 %0, %0, %1" : "+v"(acc[i]) : "v"(a[i])), acc[i])
KERNEL(k_sad_u8, uint32_t, u, (uint32_t)i, asm volatile("v_sad_u8 %0, %1, %1, %0" : "+v"(acc[i]) : "v"(a[i])), acc[i])
KERNEL(k_bfe_u32, uint32_t, u, (uint32_t)i, asm volatile("v_bfe_u32 %0, %0, 3, 8" : "+v"(acc[i]) : "v"(a[i])), acc[i])
KERNEL(k_add_f32, float, 1.0f + u * 1e-9f, (float)i, asm volatile("v_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(a[i])),
       (uint32_t)acc[i])
KERNEL(k_fma_f32, float, 1.0f + u * 1e-9f, (float)i,
       asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(a[i])), (uint32_t)acc[i])
KERNEL(k_pk_add_f32, f2, (F2(1.0f + u * 1e-9f, 2.0f)), (F2((float)i, 1.0f)),
       asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(a[i])), (uint32_t)(acc[i].x + acc[i].y))
KERNEL(k_pk_fma_f32, f2, (F2(1.0f + u * 1e-9f, 2.0f)), (F2((float)i, 1.0f)),
       asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(a[i])), (uint32_t)(acc[i].x + acc[i].y))
KERNEL(k_pk_mul_f32, f2, (F2(1.0f + u * 1e-9f, 2.0f)), (F2((float)i, 1.0f)),
       asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(acc[i]) : "v"(a[i])), (uint32_t)(acc[i].x + acc[i].y))
KERNEL(k_add_f64, double, 1.0 + u * 1e-9, (double)i, asm volatile("v_add_f64 %0, %0, %1" : "+v"(acc[i]) : "v"(a[i])),
       (uint32_t)acc[i])
KERNEL(k_mul_f64, double, 1.0 + u * 1e-9, (double)i, asm volatile("v_mul_f64 %0, %0, %1" : "+v"(acc[i]) : "v"(a[i])),
       (uint32_t)acc[i])
KERNEL(k_fma_f64, double, 1.0 + u * 1e-9, (double)i,
       asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(acc[i]) : "v"(a[i])), (uint32_t)acc[i])
KERNEL(k_rndne_f64, double, 1.0 + u * 1e-9, (double)i, asm volatile("v_rndne_f64 %0, %0" : "+v"(acc[i])),
       (uint32_t)acc[i])
KERNEL(k_cvt_f64_i32, double, 1.0 + u * 1e-9, (double)i,
       asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(acc[i]) : "v"((int)a[i])), (uint32_t)acc[i])
KERNEL(k_cvt_f32_i32, float, 1.0f + u * 1e-9f, (float)i,
       asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(acc[i])), (uint32_t)acc[i])
KERNEL(k_dot2_f32_bf16, float, __builtin_bit_cast(float, u | 0x3f803f80u), (float)i,
       asm volatile("v_dot2_f32_bf16 %0, %1, %1, %0" : "+v"(acc[i]) : "v"(a[i])), (uint32_t)acc[i])

template <typename K>
static void run(K kern, const char* name, int blocks, int threads, uint32_t* din, uint32_t* dout) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, N_ITER);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout, N_ITER);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double instr = 5.0 * blocks * (threads / 64) * (double)N_ITER * NACC;
    const double per_s = instr / (ms * 1e-3);
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    printf("%-14s %8.3f ms  -> %.2f cycles/wave-instr/SIMD @2.4GHz\n", name, ms, 4.0 * ncu * 2.4e9 / per_s);
}

int main() {
    uint32_t *din, *dout;
    (void)hipMalloc(&din, 8192 * 4);
    (void)hipMalloc(&dout, 1 << 26);
    (void)hipMemset(din, 7, 8192 * 4);
    int ncu = 0;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
    for (int waves_per_simd : {2, 4, 8}) {
        const int threads = 256, blocks = ncu * waves_per_simd;
        printf("-- %d waves/SIMD (%d CUs)\n", waves_per_simd, ncu);
        run(k_add_u32, "add_u32", blocks, threads, din, dout);
        run(k_sad_u8, "sad_u8", blocks, threads, din, dout);
        run(k_bfe_u32, "bfe_u32", blocks, threads, din, dout);
        run(k_add_f32, "add_f32", blocks, threads, din, dout);
        run(k_fma_f32, "fma_f32", blocks, threads, din, dout);
        run(k_pk_add_f32, "pk_add_f32", blocks, threads, din, dout);
        run(k_pk_mul_f32, "pk_mul_f32", blocks, threads, din, dout);
        run(k_pk_fma_f32, "pk_fma_f32", blocks, threads, din, dout);
        run(k_add_f64, "add_f64", blocks, threads, din, dout);
        run(k_mul_f64, "mul_f64", blocks, threads, din, dout);
        run(k_fma_f64, "fma_f64", blocks, threads, din, dout);
        run(k_rndne_f64, "rndne_f64", blocks, threads, din, dout);
        run(k_cvt_f64_i32, "cvt_f64_i32", blocks, threads, din, dout);
        run(k_cvt_f32_i32, "cvt_f32_i32", blocks, threads, din, dout);
        run(k_dot2_f32_bf16, "dot2_f32_bf16", blocks, threads, din, dout);
    }
    return 0;
}
