// Micro-benchmark: SIMD issue cost of the float64 VALU instructions the
// Optimize-v0 row loop uses, on gfx950.  Each wave runs ITERS iterations of
// CH independent chains of one instruction (inline asm so nothing is
// folded); s_memtime around the loop gives shader cycles per wave.  With W
// waves per SIMD, cycles-per-instruction at the SIMD = ticks / (ITERS*CH*W).
//   hipcc --offload-arch=gfx950 -O3 scripts/f64_costs.hip -o scripts/bin/f64_costs
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

constexpr int ITERS = 256;
#ifndef CH_N
#define CH_N 8
#endif
constexpr int CH = CH_N;

#define OP_KERNEL(NAME, ASM)                                                        \
    __global__ __launch_bounds__(1024) void NAME(double *out, unsigned long long *t, \
                                                 double seed) {                     \
        double a[CH];                                                               \
        for (int c = 0; c < CH; ++c) a[c] = seed + threadIdx.x * 1e-3 + c;         \
        const double b = 1.0000001, cc = 1e-9;                                      \
        (void)b; (void)cc;                                                          \
        unsigned long long t0 = __builtin_amdgcn_s_memtime();                      \
        for (int i = 0; i < ITERS; ++i) {                                           \
            _Pragma("unroll") for (int c = 0; c < CH; ++c) ASM;                     \
        }                                                                           \
        unsigned long long t1 = __builtin_amdgcn_s_memtime();                      \
        double s = 0;                                                               \
        for (int c = 0; c < CH; ++c) s += a[c];                                     \
        out[blockIdx.x * blockDim.x + threadIdx.x] = s;                             \
        if ((threadIdx.x & 63) == 0) t[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0; \
    }

OP_KERNEL(k_fma, asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[c]) : "v"(b), "v"(cc)))
OP_KERNEL(k_mul, asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
OP_KERNEL(k_add, asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[c]) : "v"(cc)))
OP_KERNEL(k_rcp, asm volatile("v_rcp_f64 %0, %0" : "+v"(a[c])))
OP_KERNEL(k_rndne, asm volatile("v_rndne_f64 %0, %0" : "+v"(a[c])))
OP_KERNEL(k_ldexp, asm volatile("v_ldexp_f64 %0, %0, 1" : "+v"(a[c])))
OP_KERNEL(k_min, asm volatile("v_min_f64 %0, %0, %1" : "+v"(a[c]) : "v"(b)))
OP_KERNEL(k_cmp, asm volatile("v_cmp_lt_f64 vcc, %0, %1" : : "v"(a[c]), "v"(b) : "vcc"))
OP_KERNEL(k_cvt, { int tmp_; asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(tmp_) : "v"(a[c])); })
OP_KERNEL(k_fma32, asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(*reinterpret_cast<float *>(&a[c])) : "v"(1.0f), "v"(1e-9f)))
OP_KERNEL(k_cnd, asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(*reinterpret_cast<int *>(&a[c])) : "v"(3)))

using K = void (*)(double *, unsigned long long *, double);

int main() {
    struct { const char *name; K k; } ops[] = {
        {"v_fma_f64", k_fma}, {"v_mul_f64", k_mul}, {"v_add_f64", k_add},
        {"v_rcp_f64", k_rcp}, {"v_rndne_f64", k_rndne}, {"v_ldexp_f64", k_ldexp},
        {"v_min_f64", k_min}, {"v_cmp_lt_f64", k_cmp}, {"v_cvt_i32_f64", k_cvt},
        {"v_fma_f32", k_fma32}, {"v_cndmask_b32", k_cnd}};
    const int blocks = 256, threads = 1024;   // 4 waves per SIMD on every CU
    double *out;
    unsigned long long *t;
    hipMalloc(&out, sizeof(double) * blocks * threads);
    hipMalloc(&t, sizeof(unsigned long long) * blocks * threads / 64);
    std::vector<unsigned long long> h(blocks * threads / 64);
    for (auto &op : ops) {
        for (int cfg = 0; cfg < 2; ++cfg) {
            const int nb = cfg == 0 ? blocks : 1, nt = cfg == 0 ? threads : 64;
            hipLaunchKernelGGL(op.k, dim3(nb), dim3(nt), 0, 0, out, t, 1.5);
            hipLaunchKernelGGL(op.k, dim3(nb), dim3(nt), 0, 0, out, t, 1.5);
            hipDeviceSynchronize();
            const int nw = nb * nt / 64;
            hipMemcpy(h.data(), t, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
            std::sort(h.begin(), h.begin() + nw);
            const double med = static_cast<double>(h[nw / 2]);
            const int wps = cfg == 0 ? 4 : 1;   // waves per SIMD
            printf("{\"op\": \"%s\", \"chains\": %d, \"waves_per_simd\": %d, \"cycles_per_instr_simd\": %.2f, \"cycles_per_instr_wave\": %.2f}\n",
                   op.name, CH, wps, med / (ITERS * CH * wps), med / (ITERS * CH));
        }
    }
    return 0;
}
