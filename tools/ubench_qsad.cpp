// Microbenchmark + semantics check: v_qsad_pk_u16_u8 on gfx950 (four 4-byte SADs of one
// reference dword against the byte windows [i, i+4) of an 8-byte source, i = 0..3, each added
// to its own 16-bit half of a 64-bit accumulator) against v_sad_u8 (one 4-byte SAD).
//   semantics: GPU results of random operands against the CPU model, wrap vs saturate
//   issue:     NACC independent accumulators per lane, 2 / 4 / 8 waves per SIMD
// hipcc --offload-arch=gfx950 -O3 tools/ubench_qsad.cpp -o tools/ubench_qsad
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define N_ITER 1024
#define NACC 8

__global__ void k_sem(const uint64_t* a, const uint32_t* b, const uint64_t* c, uint64_t* o, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) o[i] = __builtin_amdgcn_qsad_pk_u16_u8(a[i], b[i], c[i]);
}

__global__ void k_qsad(const uint32_t* in, uint32_t* out, int n_iter) {
    uint64_t a[NACC], acc[NACC];
    uint32_t b[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) {
        a[i] = ((uint64_t)in[threadIdx.x + i + 1] << 32) | in[threadIdx.x + i + 2];
        b[i] = in[threadIdx.x + 2 * i + 3];
        acc[i] = i;
    }
    for (int it = 0; it < n_iter; ++it) {
#pragma unroll
        for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_qsad_pk_u16_u8(a[i], b[i], acc[i]);
    }
    uint64_t s = 0;
#pragma unroll
    for (int i = 0; i < NACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = (uint32_t)s ^ (uint32_t)(s >> 32);
}

__global__ void k_sad(const uint32_t* in, uint32_t* out, int n_iter) {
    uint32_t a[2 * NACC], b[2 * NACC], acc[2 * NACC];   // the same VGPR count of accumulators
#pragma unroll
    for (int i = 0; i < 2 * NACC; ++i) {
        a[i] = in[threadIdx.x + i + 1];
        b[i] = in[threadIdx.x + 2 * i + 3];
        acc[i] = i;
    }
    for (int it = 0; it < n_iter; ++it) {
#pragma unroll
        for (int i = 0; i < 2 * NACC; ++i) acc[i] = __builtin_amdgcn_sad_u8(a[i], b[i], acc[i]);
    }
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < 2 * NACC; ++i) s += acc[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static uint64_t model(uint64_t a, uint32_t b, uint64_t c, bool sat) {
    uint64_t r = 0;
    for (int i = 0; i < 4; ++i) {
        uint32_t s = 0;
        for (int j = 0; j < 4; ++j) {
            const int x = (int)((a >> (8 * (i + j))) & 255), y = (int)((b >> (8 * j)) & 255);
            s += (uint32_t)(x > y ? x - y : y - x);
        }
        uint32_t v = (uint32_t)((c >> (16 * i)) & 0xFFFF) + s;
        v = sat ? (v > 0xFFFF ? 0xFFFF : v) : (v & 0xFFFF);
        r |= (uint64_t)v << (16 * i);
    }
    return r;
}

static uint64_t rnd64() { return ((uint64_t)rand() << 42) ^ ((uint64_t)rand() << 21) ^ (uint64_t)rand(); }

int main() {
    const int n = 1 << 16;
    uint64_t *ha = (uint64_t*)malloc(n * 8), *hc = (uint64_t*)malloc(n * 8), *ho = (uint64_t*)malloc(n * 8);
    uint32_t* hb = (uint32_t*)malloc(n * 4);
    srand(7);
    for (int i = 0; i < n; ++i) {
        ha[i] = rnd64();
        hb[i] = (uint32_t)rnd64();
        hc[i] = rnd64();
        if (i % 4 == 1) hc[i] |= 0xFFF0FFF0FFF0FFF0ull;   // near the 16-bit limit: wrap or saturate
        if (i % 4 == 2) hc[i] &= 0x0FFF0FFF0FFF0FFFull;
    }
    uint64_t *da, *dc, *dout;
    uint32_t* db;
    (void)hipMalloc(&da, n * 8);
    (void)hipMalloc(&dc, n * 8);
    (void)hipMalloc(&dout, n * 8);
    (void)hipMalloc(&db, n * 4);
    (void)hipMemcpy(da, ha, n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(dc, hc, n * 8, hipMemcpyHostToDevice);
    (void)hipMemcpy(db, hb, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_sem, dim3(n / 256), dim3(256), 0, 0, da, db, dc, dout, n);
    (void)hipMemcpy(ho, dout, n * 8, hipMemcpyDeviceToHost);
    int bad_wrap = 0, bad_sat = 0;
    for (int i = 0; i < n; ++i) {
        bad_wrap += ho[i] != model(ha[i], hb[i], hc[i], false);
        bad_sat += ho[i] != model(ha[i], hb[i], hc[i], true);
    }
    printf("semantics: %d cases, mismatches wrap-model %d, saturate-model %d\n", n, bad_wrap, bad_sat);
    if (bad_wrap && bad_sat)
        for (int i = 0; i < n; ++i)
            if (ho[i] != model(ha[i], hb[i], hc[i], false)) {
                printf("  a=%016llx b=%08x c=%016llx gpu=%016llx wrap=%016llx\n", (unsigned long long)ha[i], hb[i],
                       (unsigned long long)hc[i], (unsigned long long)ho[i],
                       (unsigned long long)model(ha[i], hb[i], hc[i], false));
                break;
            }

    uint32_t *din, *dsink;
    (void)hipMalloc(&din, 8192 * 4);
    (void)hipMalloc(&dsink, 1 << 24);
    (void)hipMemset(din, 7, 8192 * 4);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    for (int wps : {2, 4, 8}) {
        const int threads = 256, blocks = 256 * wps;
        for (int which = 0; which < 2; ++which) {
            auto launch = [&]() {
                if (which == 0) hipLaunchKernelGGL(k_sad, dim3(blocks), dim3(threads), 0, 0, din, dsink, N_ITER);
                else hipLaunchKernelGGL(k_qsad, dim3(blocks), dim3(threads), 0, 0, din, dsink, N_ITER);
            };
            launch();
            (void)hipDeviceSynchronize();
            (void)hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) launch();
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            float ms = 0;
            (void)hipEventElapsedTime(&ms, e0, e1);
            const double instr = 5.0 * blocks * (threads / 64) * (double)N_ITER * (which ? NACC : 2 * NACC);
            const double per_s = instr / (ms * 1e-3);
            const double bytes = per_s * 64 * (which ? 16 : 4);   // |diff| byte operations per second
            printf("%d waves/SIMD %-16s %8.3f ms  %.2f cycles/wave-instr/SIMD @2.4GHz  %.3e byte-ops/s\n", wps,
                   which ? "v_qsad_pk_u16_u8" : "v_sad_u8", ms, 1024 * 2.4e9 / per_s, bytes);
        }
    }
    return 0;
}
