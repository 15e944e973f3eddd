// Micro-benchmark: issue rate of v_mfma_f64_16x16x4_f64 on gfx950 against
// v_fma_f64, to choose the Optimize-v0 image-set kernel's GEMM unit.
// Each wave runs ITERS iterations over CH independent accumulators; chip
// TFLOP/s from hipEvents (one launch of `blocks` x `threads`).
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma_f64.hip -o scripts/bin/mfma_f64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 2048;
constexpr int CH = 4;

__global__ __launch_bounds__(256) void k_mfma(double *out, double seed) {
    d4 acc[CH];
    for (int c = 0; c < CH; ++c) acc[c] = d4{seed, seed, seed, seed};
    double a = seed + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-6;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < CH; ++c) acc[c] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[c], 0, 0, 0);
    }
    double s = 0;
    for (int c = 0; c < CH; ++c) s += acc[c][0] + acc[c][1] + acc[c][2] + acc[c][3];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_fma(double *out, double seed) {
    double a[8];
    for (int c = 0; c < 8; ++c) a[c] = seed + threadIdx.x * 1e-3 + c;
    const double b = 1.0000001, cc = 1e-9;
    for (int i = 0; i < ITERS; ++i) {
#pragma unroll
        for (int c = 0; c < 8; ++c) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "v"(cc));
    }
    double s = 0;
    for (int c = 0; c < 8; ++c) s += a[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
    double *out;
    hipMalloc(&out, sizeof(double) * 256 * 8 * 1024);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int wps = 1; wps <= 4; wps *= 2) {      // waves per SIMD
        const int blocks = 256 * wps;            // 4 waves per block = 1 per SIMD
        for (int kind = 0; kind < 2; ++kind) {
            auto launch = [&] {
                if (kind == 0) hipLaunchKernelGGL(k_mfma, dim3(blocks), dim3(256), 0, 0, out, 1.0);
                else hipLaunchKernelGGL(k_fma, dim3(blocks), dim3(256), 0, 0, out, 1.0);
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            for (int r = 0; r < 5; ++r) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double waves = blocks * 4.0;
            const double flops = kind == 0 ? waves * ITERS * CH * 2.0 * 16 * 16 * 4
                                           : waves * 64.0 * ITERS * 8 * 2.0;
            printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"tflops\": %.2f, \"ms\": %.4f}\n",
                   kind == 0 ? "v_mfma_f64_16x16x4_f64" : "v_fma_f64", wps,
                   flops * 5 / (ms * 1e-3) / 1e12, ms / 5);
        }
    }
    return 0;
}
