// Microbenchmark: issue throughput of the byte-SAD instructions on gfx950.
//   v_sad_u8          4 |diffs| + accumulate        (one 32-bit lane op)
//   v_qsad_pk_u16_u8  4 SADs at 4 byte offsets       (16 |diffs|, 4 x u16 accumulators)
//   v_alignbyte_b32   byte funnel shift              (reference for a plain 32-bit op)
// hipcc --offload-arch=gfx950 -O3 tools/ubench_sad.cpp -o /tmp/ubench_sad && /tmp/ubench_sad
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITER 4096
#define N_ACC 8

__global__ void k_sad(const uint32_t* in, uint32_t* out) {
    uint32_t a = in[threadIdx.x], b = in[threadIdx.x + 1];
    uint32_t acc[N_ACC];
#pragma unroll
    for (int i = 0; i < N_ACC; ++i) acc[i] = i;
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < N_ACC; ++i) acc[i] = __builtin_amdgcn_sad_u8(a + i, b, acc[i]);
        a ^= acc[0];
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < N_ACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void k_qsad(const uint32_t* in, uint32_t* out) {
    uint64_t a = ((uint64_t)in[threadIdx.x] << 32) | in[threadIdx.x + 2];
    uint32_t b = in[threadIdx.x + 1];
    uint64_t acc[N_ACC];
#pragma unroll
    for (int i = 0; i < N_ACC; ++i) acc[i] = i;
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < N_ACC; ++i) acc[i] = __builtin_amdgcn_qsad_pk_u16_u8(a + i, b, acc[i]);
        b ^= (uint32_t)acc[0];
    }
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < N_ACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void k_align(const uint32_t* in, uint32_t* out) {
    uint32_t a = in[threadIdx.x], b = in[threadIdx.x + 1];
    uint32_t acc[N_ACC];
#pragma unroll
    for (int i = 0; i < N_ACC; ++i) acc[i] = i;
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < N_ACC; ++i) acc[i] = __builtin_amdgcn_alignbyte(acc[i], a, b + i);
        a += acc[1];
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < N_ACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static double run(K kern, const char* name, int blocks, int threads, uint32_t* din, uint32_t* dout) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(kern, dim3(blocks), dim3(threads), 0, 0, din, dout);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    double instr = 5.0 * blocks * (threads / 64) * (double)N_ITER * N_ACC;  // wave-instructions
    double per_s = instr / (ms * 1e-3);
    printf("%-18s %8.3f ms  %.3e wave-instr/s  = %.3f wave-instr/clk/CU @2.4GHz\n", name, ms, per_s,
           per_s / 256 / 2.4e9);
    return per_s;
}

int main() {
    uint32_t *din, *dout;
    hipMalloc(&din, 4096 * 4);
    hipMalloc(&dout, 1 << 24);
    hipMemset(din, 7, 4096 * 4);
    for (int waves_per_cu : {4, 8, 16}) {
        int threads = 256, blocks = 256 * waves_per_cu / 4;
        printf("-- %d waves/CU\n", waves_per_cu);
        run(k_sad, "v_sad_u8", blocks, threads, din, dout);
        run(k_qsad, "v_qsad_pk_u16_u8", blocks, threads, din, dout);
        run(k_align, "v_alignbyte_b32", blocks, threads, din, dout);
    }
    return 0;
}
