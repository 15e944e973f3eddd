// Micro-benchmark: can f64 MFMA and f64 VALU work overlap on gfx950?
// Kernels (one launch each, timed with hipEvents, 256 CUs x waves/SIMD):
//   mfma    ITERS x 4 chains of v_mfma_f64_16x16x4_f64
//   valu    ITERS x 16 independent v_fma_f64 (the same issue slots a softmax uses)
//   mixed   both streams interleaved in one wave
//   split   2 waves per SIMD: even waves the MFMA stream, odd waves the VALU stream
//   mfma4   ITERS x 4 chains of v_mfma_f64_4x4x4_f64 (4 blocks)
//   ldsexp  ITERS x 4 table lookups (ds_read_b64 at lane-varying indices)
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma_valu_mix.hip -o scripts/bin/mfma_valu_mix
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 1024;

__device__ __forceinline__ void mfma_step(d4 (&acc)[4], double a, double b) {
#pragma unroll
    for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
}
__device__ __forceinline__ void valu_step(double (&v)[16], double b, double cc) {
#pragma unroll
    for (int c = 0; c < 16; ++c) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(v[c]) : "v"(b), "v"(cc));
}

template <int KIND>
__global__ __launch_bounds__(1024) void k(double *out, double seed) {
    d4 acc[4];
    for (int c = 0; c < 4; ++c) acc[c] = d4{seed, seed, seed, seed};
    double v[16];
    for (int c = 0; c < 16; ++c) v[c] = seed + threadIdx.x * 1e-3 + c;
    const double a = seed + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-9, cc = 1e-12;
    const int wave = threadIdx.x >> 6;
    double s4[4] = {seed, seed, seed, seed};
    __shared__ double table[64];
    if (threadIdx.x < 64) table[threadIdx.x] = 1.0 + threadIdx.x * 1e-3;
    __syncthreads();
    int idx = (threadIdx.x * 37) & 63;
    double tacc = 0.0;
    for (int i = 0; i < ITERS; ++i) {
        if (KIND == 0) mfma_step(acc, a, b);
        if (KIND == 1) valu_step(v, b, cc);
        if (KIND == 2) { mfma_step(acc, a, b); valu_step(v, b, cc); }
        // waves w and w + 4 share SIMD w % 4 (round-robin placement): one of each kind per SIMD
        if (KIND == 3) { if ((wave >> 2) & 1) valu_step(v, b, cc); else mfma_step(acc, a, b); }
        if (KIND == 4) {
#pragma unroll
            for (int c = 0; c < 4; ++c) s4[c] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, s4[c], 0, 0, 0);
        }
        if (KIND == 5) {
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                tacc += table[(idx + 13 * c) & 63];
                idx = (idx * 5 + 7) & 63;
            }
        }
    }
    double s = tacc;
    for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3] + s4[c];
    for (int c = 0; c < 16; ++c) s += v[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    double *out;
    hipMalloc(&out, sizeof(double) * 1024 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const char *names[] = {"mfma16x16x4", "valu_fma16", "mixed_same_wave", "split_waves", "mfma4x4x4", "lds_table"};
    void (*fns[])(double *, double) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>};
    for (int wps = 1; wps <= 4; ++wps) {
        for (int kind = 0; kind < 6; ++kind) {
            if (kind == 3 && wps != 2) continue;
            if ((kind == 0 || kind == 2) && wps > 2) continue;
            const int threads = 256 * wps;   // 4 or 8 waves per block, one block per CU
            auto launch = [&] { hipLaunchKernelGGL(fns[kind], dim3(256), dim3(threads), 0, 0, out, 1.0); };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double us = ms * 1e3 / 5;
            // per-SIMD instruction issue: waves per SIMD x ITERS x instrs
            printf("{\"kernel\": \"%s\", \"waves_per_simd\": %d, \"us\": %.2f}\n", names[kind], wps, us);
        }
    }
    return 0;
}
