// Microbenchmark: issue throughput of the byte-SAD instructions on gfx950.
//   v_sad_u8          4 |diffs| + accumulate        (one 32-bit lane op)
//   v_qsad_pk_u16_u8  4 SADs at 4 byte offsets       (16 |diffs|, 4 x u16 accumulators)
//   v_add_u32         reference full-rate op
// Each lane runs NACC independent accumulator chains with loop-invariant operands, so
// the loop body is nothing but the instruction under test (check the .s with --save-temps).
// hipcc --offload-arch=gfx950 -O3 tools/ubench_sad.cpp -o tools/ubench_sad && tools/ubench_sad
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITER 2048
#define NACC 16

__global__ void k_sad(const uint32_t* in, uint32_t* out, int n_iter) {
    uint32_t a[NACC], acc[NACC];
    const uint32_t b = in[threadIdx.x];
#pragma unroll
    for (int i = 0; i < NACC; ++i) { a[i] = in[threadIdx.x + i + 1]; acc[i] = i; }
    for (int it = 0; it < n_iter; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_sad_u8(a[i], b, acc[i]);
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_qsad(const uint32_t* in, uint32_t* out, int n_iter) {
    uint64_t a[NACC], acc[NACC];
    const uint32_t b = in[threadIdx.x];
#pragma unroll
    for (int i = 0; i < NACC; ++i) { a[i] = ((uint64_t)in[threadIdx.x + i + 2] << 32) | in[threadIdx.x + i + 1]; acc[i] = i; }
    for (int it = 0; it < n_iter; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_qsad_pk_u16_u8(a[i], b, acc[i]);
    }
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void k_add(const uint32_t* in, uint32_t* out, int n_iter) {
    uint32_t a[NACC], acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) { a[i] = in[threadIdx.x + i + 1]; acc[i] = i; }
    for (int it = 0; it < n_iter; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = acc[i] * 3u + a[i];   // v_mad_u32_u24 or mul+add
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

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
    const double instr = 5.0 * blocks * (threads / 64) * (double)N_ITER * NACC;  // wave-instructions
    const double per_s = instr / (ms * 1e-3);
    // cycles per wave-instruction per SIMD at 2.4 GHz (1024 SIMDs)
    printf("%-18s %8.3f ms  %.3e wave-instr/s  -> %.2f cycles/wave-instr/SIMD @2.4GHz\n", name, ms, per_s,
           1024 * 2.4e9 / per_s);
}

int main() {
    uint32_t *din, *dout;
    (void)hipMalloc(&din, 8192 * 4);
    (void)hipMalloc(&dout, 1 << 24);
    (void)hipMemset(din, 7, 8192 * 4);
    for (int waves_per_simd : {1, 2, 4, 8}) {
        const int threads = 256, blocks = 256 * waves_per_simd;  // 4 waves per block = 1 per SIMD
        printf("-- %d waves/SIMD\n", waves_per_simd);
        run(k_sad, "v_sad_u8", blocks, threads, din, dout);
        run(k_qsad, "v_qsad_pk_u16_u8", blocks, threads, din, dout);
        run(k_add, "mul+add (2 instr)", blocks, threads, din, dout);
    }
    return 0;
}
