// LDS-per-workgroup occupancy on gfx950: what the occupancy API reports for 512-thread
// workgroups holding N bytes of static LDS, and how many such workgroups one CU actually
// runs at once (every workgroup spins until all of a CU's co-resident ones have arrived,
// bounded by a timeout; the count per CU is read back).
//   hipcc --offload-arch=gfx950 -O2 tools/ubench_lds_occ.cpp -o tools/ubench_lds_occ
#include <hip/hip_runtime.h>
#include <stdio.h>

template <int N>
__global__ void __launch_bounds__(512) k(unsigned* cnt, unsigned* out) {
    __shared__ unsigned char buf[N];
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const unsigned cu = ((xcc & 7) << 8) | ((hw >> 8) & 0xF) << 4 | ((hw >> 13) & 0x7) << 1 | ((hw >> 12) & 1);
    buf[threadIdx.x] = (unsigned char)threadIdx.x;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned c = atomicAdd(&cnt[cu & 2047], 1u) + 1;
        unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned m = c;
        while (__builtin_amdgcn_s_memrealtime() - t0 < 200000ull) {   // 2 ms: let co-resident ones arrive
            const unsigned v = __hip_atomic_load(&cnt[cu & 2047], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            m = v > m ? v : m;
        }
        atomicMax(&out[0], m);
        atomicSub(&cnt[cu & 2047], 1u);   // concurrency, not arrivals: leave before the next one comes in
        out[1 + blockIdx.x] = buf[5];
    }
}

template <int N>
void run() {
    int occ = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, k<N>, 512, 0);
    unsigned *cnt, *out;
    hipMalloc(&cnt, 2048 * 4);
    hipMalloc(&out, 4096 * 4);
    hipMemset(cnt, 0, 2048 * 4);
    hipMemset(out, 0, 4096 * 4);
    hipLaunchKernelGGL(k<N>, dim3(256 * 4), dim3(512), 0, 0, cnt, out);
    hipDeviceSynchronize();
    unsigned m = 0;
    hipMemcpy(&m, out, 4, hipMemcpyDeviceToHost);
    printf("lds %6d B: occupancy API %d workgroups/CU, observed max co-resident %u\n", N, occ, m);
    hipFree(cnt);
    hipFree(out);
}

int main() {
    run<50296>();
    run<52224>();
    run<53248>();
    run<53760>();
    run<53880>();
    run<54272>();
    run<54613>();
    return 0;
}
