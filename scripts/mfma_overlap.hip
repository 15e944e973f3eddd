// Micro-benchmark (round 6): what a row wave's VALU can do while its own f64
// MFMA runs.  One wave per SIMD (256 CUs x 4 waves), every instruction in
// inline asm so the issue order is exactly the source order:
//   per iteration ONE v_mfma_f64_16x16x4_f64 (4 accumulator chains, each
//   read 4 MFMAs after it was written) followed by N independent VALU ops of
//   one kind (f64 fma, f32 fma, u32 add, u32 and), N = 0..16;  and the same N
//   VALU ops with no MFMA.  If the VALU work runs under the MFMA, the mixed
//   time stays at the MFMA-only time until N fills it; if the f64 units are
//   shared, it grows by the VALU-only time.
//   A second family puts the MFMA stream and the VALU stream in two waves of
//   the same SIMD (waves w, w + 4).
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma_overlap.hip -o scripts/bin/mfma_overlap
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 4096;

template <int KIND>
__device__ __forceinline__ void valu1(double &d, float &f, unsigned &u, double b64, float b32, unsigned bu) {
    if constexpr (KIND == 0) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(d) : "v"(b64));
    if constexpr (KIND == 1) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(f) : "v"(b32));
    if constexpr (KIND == 2) asm volatile("v_add_u32 %0, %0, %1" : "+v"(u) : "v"(bu));
    if constexpr (KIND == 3) asm volatile("v_and_b32 %0, %0, %1" : "+v"(u) : "v"(bu));
}

// MODE 0: VALU only; 1: MFMA + N VALU in one wave; 2: split (waves 0-3 MFMA, 4-7 VALU)
template <int KIND, int N, int MODE>
__global__ __launch_bounds__(512) void k(double *out, double seed) {
    d4 acc0 = {seed, seed, seed, seed}, acc1 = acc0, acc2 = acc0, acc3 = acc0;
    double dv[16];
    float fv[16];
    unsigned uv[16];
#pragma unroll
    for (int c = 0; c < 16; ++c) {
        dv[c] = seed + threadIdx.x * 1e-3 + c;
        fv[c] = static_cast<float>(dv[c]);
        uv[c] = threadIdx.x * 7 + c;
    }
    const double a = seed + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-9;
    const float b32 = 1.0f - threadIdx.x * 1e-7f;
    const unsigned bu = 0x7fffffffu - threadIdx.x;
    const int wave = threadIdx.x >> 6;
    const bool do_mfma = MODE == 1 || (MODE == 2 && wave < 4);
    const bool do_valu = MODE != 2 || wave >= 4;
    for (int i = 0; i < ITERS; i += 4) {
#define ONE(ACC)                                                                                 \
    if (do_mfma) asm volatile("v_mfma_f64_16x16x4_f64 %0, %1, %2, %0" : "+v"(ACC) : "v"(a), "v"(b)); \
    if (do_valu) {                                                                                 \
        _Pragma("unroll") for (int c = 0; c < N; ++c) valu1<KIND>(dv[c], fv[c], uv[c], b, b32, bu); \
    }
        ONE(acc0) ONE(acc1) ONE(acc2) ONE(acc3)
#undef ONE
    }
    double s = acc0[0] + acc1[1] + acc2[2] + acc3[3];
#pragma unroll
    for (int c = 0; c < 16; ++c) s += dv[c] + fv[c] + uv[c];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int KIND, int N, int MODE>
double run(double *out, hipEvent_t e0, hipEvent_t e1) {
    const int threads = MODE == 2 ? 512 : 256;
    auto launch = [&] { hipLaunchKernelGGL((k<KIND, N, MODE>), dim3(256), dim3(threads), 0, 0, out, 1.0); };
    launch();
    hipDeviceSynchronize();
    hipEventRecord(e0);
    for (int r = 0; r < 10; ++r) launch();
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    return ms * 1e6 / 10 / ITERS;   // ns per iteration
}

template <int KIND, int N>
void row(const char *kind, double *out, hipEvent_t e0, hipEvent_t e1, double mfma_only) {
    const double v = run<KIND, N, 0>(out, e0, e1);
    const double m = run<KIND, N, 1>(out, e0, e1);
    const double s = run<KIND, N, 2>(out, e0, e1);
    printf("{\"valu\": \"%s\", \"n\": %d, \"ns_valu_only\": %.2f, \"ns_mfma_only\": %.2f, "
           "\"ns_same_wave\": %.2f, \"ns_split_waves\": %.2f}\n", kind, N, v, mfma_only, m, s);
    fflush(stdout);
}

template <int KIND>
void family(const char *kind, double *out, hipEvent_t e0, hipEvent_t e1, double mo) {
    row<KIND, 1>(kind, out, e0, e1, mo);
    row<KIND, 2>(kind, out, e0, e1, mo);
    row<KIND, 4>(kind, out, e0, e1, mo);
    row<KIND, 6>(kind, out, e0, e1, mo);
    row<KIND, 8>(kind, out, e0, e1, mo);
    row<KIND, 12>(kind, out, e0, e1, mo);
    row<KIND, 16>(kind, out, e0, e1, mo);
}

int main() {
    double *out;
    hipMalloc(&out, sizeof(double) * 512 * 256);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    // warm the clock: 200 ms of MFMA-only launches
    for (int r = 0; r < 40; ++r) run<0, 0, 1>(out, e0, e1);
    const double mo = run<0, 0, 1>(out, e0, e1);
    family<0>("f64_fma", out, e0, e1, mo);
    family<1>("f32_fma", out, e0, e1, mo);
    family<2>("u32_add", out, e0, e1, mo);
    family<3>("b32_and", out, e0, e1, mo);
    hipFree(out);
    return 0;
}
