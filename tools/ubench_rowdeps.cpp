// Microtest of the p_run_kernel dependency scheme: a persistent queue of tasks in rows of C
// tasks; task (row r) waits until row r-1 is complete (done[r-1] == C), then increments
// done[r].  Each wait is bounded by 2 ms of s_memrealtime.  Every queue / counter access is
// made by ALL lanes of wave 0 under a wave-uniform (SGPR) branch: a `tid == 0` branch ahead
// of a barrier inside the loop gets structurised into a divergent inner loop that never
// re-runs the atomic (a hang).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_rowdeps.cpp -o tools/ubench_rowdeps
#include <hip/hip_runtime.h>
#include <stdio.h>

#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

template <int MODE>   // 0: no waits; 1: relaxed agent load poll
__global__ void rowdeps(unsigned* ws, int ntasks, int C, unsigned* out) {
    __shared__ int s_task;
    unsigned* done = ws + 2;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool lane0 = (threadIdx.x & 63) == 0;
    for (;;) {
        if (wave == 0) {
            const unsigned v = __hip_atomic_fetch_add(&ws[0], lane0 ? 1u : 0u, RLX_AGENT);
            s_task = (int)__builtin_amdgcn_readfirstlane(v);
        }
        __syncthreads();
        const int t = __builtin_amdgcn_readfirstlane(s_task);
        __syncthreads();
        if (t >= ntasks) break;
        const int r = t / C;
        if (MODE > 0 && r > 0 && wave == 0) {
            const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
            for (;;) {
                const unsigned v = __builtin_amdgcn_readfirstlane(__hip_atomic_load(done + r - 1, RLX_AGENT));
                if (v >= (unsigned)C) break;
                __builtin_amdgcn_s_sleep(2);
                if (__builtin_amdgcn_s_memrealtime() - t0 > 200000ull) {   // 2 ms at 100 MHz
                    __hip_atomic_fetch_add(&ws[1], lane0 ? 1u : 0u, RLX_AGENT);
                    break;
                }
            }
        }
        __syncthreads();
        float acc = threadIdx.x;
        for (int i = 0; i < 2000; ++i) acc = acc * 1.0001f + 0.5f;
        if (acc == 12345.f) out[0] = 1;
        __syncthreads();
        if (wave == 0) __hip_atomic_fetch_add(done + r, lane0 ? 1u : 0u, RLX_AGENT);
    }
}

template <int M>
void run(const char* name, unsigned* ws, unsigned* out, int ntasks, int C, int grid) {
    (void)hipMemset(ws, 0, (2 + ntasks / C + 1) * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((rowdeps<M>), dim3(grid), dim3(256), 0, 0, ws, ntasks, C, out);
    (void)hipEventRecord(e1);
    (void)hipDeviceSynchronize();
    float ms; (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned h[2]; (void)hipMemcpy(h, ws, 8, hipMemcpyDeviceToHost);
    unsigned d[4]; (void)hipMemcpy(d, ws + 2, 16, hipMemcpyDeviceToHost);
    printf("%-12s tasks %u (expect %d + grid) timeouts %u  done[0..3] %u %u %u %u  %.3f ms\n", name, h[0], ntasks,
           h[1], d[0], d[1], d[2], d[3], ms);
    fflush(stdout);
}

int main() {
    const int C = 64, rows = 100, ntasks = C * rows, grid = 512;
    unsigned *ws, *out;
    (void)hipMalloc(&ws, (2 + rows + 1) * 4);
    (void)hipMalloc(&out, ntasks * 4);
    run<0>("no waits", ws, out, ntasks, C, grid);
    run<1>("load poll", ws, out, ntasks, C, grid);
    run<1>("load poll", ws, out, ntasks, C, grid);
    return 0;
}
