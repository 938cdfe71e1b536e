// FETCH_SIZE calibration on gfx950 for the access widths the encoder's kernels use.
// MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a wide (16 B / lane) coalesced
// streaming read.  The encoder's window / tile staging reads 4 B per lane; this measures what
// FETCH_SIZE reports for exactly 256 MiB read by (a) 4-B and (b) 16-B coalesced loads, so the
// roofline's `traffic` can be corrected by a measured factor instead of an assumed one.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_fetch.cpp -o tools/ubench_fetch
//   rocprofv3 --pmc FETCH_SIZE -- ./tools/ubench_fetch
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void read_b32(const uint32_t* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        acc ^= p[i];
    if (acc == 0x12345678u) out[0] = acc;
}

__global__ void read_b128(const uint4* __restrict__ p, size_t n, uint32_t* out) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = p[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) out[0] = acc;
}

int main() {
    const size_t bytes = 256ull << 20;
    void* buf;
    uint32_t* out;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    hipMemset(buf, 1, bytes);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(read_b32, dim3(4096), dim3(256), 0, 0, (const uint32_t*)buf, bytes / 4, out);
        hipLaunchKernelGGL(read_b128, dim3(4096), dim3(256), 0, 0, (const uint4*)buf, bytes / 16, out);
    }
    hipDeviceSynchronize();
    printf("read %zu bytes per dispatch (read_b32: 4 B/lane, read_b128: 16 B/lane)\n", bytes);
    hipFree(buf);
    hipFree(out);
    return 0;
}
