// Microbenchmark + semantics check: ds_read_b32 at a byte address that is not a multiple of 4
// on gfx950 (does it return the four bytes at that address, and at what issue cost against an
// aligned read?).  The SEA bound loop reads one such dword per candidate row and today pays
// two aligned reads and a v_alignbyte (VOP3, ~4.4 cycles) for it.
// hipcc --offload-arch=gfx950 -O3 tools/ubench_lds_unaligned.cpp -o tools/ubench_lds_unaligned
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define N_ITER 4096

__global__ void k_sem(uint32_t* out, int off) {
    __shared__ uint8_t b[4096 + 64];
    for (int i = threadIdx.x; i < 4096 + 64; i += blockDim.x) b[i] = (uint8_t)(i * 7 + 3);
    __syncthreads();
    const uint32_t addr = (uint32_t)(uintptr_t)(b) + threadIdx.x * 4 + off;
    uint32_t v;
    asm volatile("ds_read_b32 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(addr) : "memory");
    out[threadIdx.x] = v;
}

// every lane reads NR dwords per iteration at byte offset `off` past a 4-aligned address
template <int NR>
__global__ void k_time(uint32_t* out, int off, int n_iter) {
    __shared__ uint8_t b[8192 + 64];
    for (int i = threadIdx.x; i < 8192 + 64; i += blockDim.x) b[i] = (uint8_t)i;
    __syncthreads();
    uint32_t base = (uint32_t)(uintptr_t)(b) + (threadIdx.x & 63) * 4 + off;
    uint32_t acc = 0;
    for (int it = 0; it < n_iter; ++it) {
        uint32_t v[NR];
#pragma unroll
        for (int r = 0; r < NR; ++r)
            asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v[r]) : "v"(base), "i"(r * 256) : "memory");
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
        for (int r = 0; r < NR; ++r) acc += v[r];
        base ^= 4096;
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main() {
    uint32_t *dout, hout[256];
    (void)hipMalloc(&dout, 1 << 24);
    for (int off = 0; off < 4; ++off) {
        hipLaunchKernelGGL(k_sem, dim3(1), dim3(256), 0, 0, dout, off);
        (void)hipMemcpy(hout, dout, sizeof(hout), hipMemcpyDeviceToHost);
        int bad = 0;
        for (int t = 0; t < 256; ++t) {
            uint32_t want = 0;
            for (int k = 0; k < 4; ++k) want |= (uint32_t)(uint8_t)((t * 4 + off + k) * 7 + 3) << (8 * k);
            bad += hout[t] != want;
        }
        printf("offset %d: %d of 256 lanes differ from the bytes at the address\n", off, bad);
    }
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int off = 0; off < 4; ++off) {
        const int blocks = 256 * 8, threads = 256;   // 8 waves per SIMD
        hipLaunchKernelGGL(k_time<8>, dim3(blocks), dim3(threads), 0, 0, dout, off, N_ITER);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL(k_time<8>, dim3(blocks), dim3(threads), 0, 0, dout, off, N_ITER);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double instr = (double)blocks * (threads / 64) * N_ITER * 8;   // wave-level ds_read_b32
        printf("offset %d: %.3f ms, %.2f cycles per wave ds_read_b32 per CU @2.4GHz\n", off, ms,
               ms * 1e-3 * 2.4e9 * 256 / instr);
    }
    return 0;
}
