// Micro-benchmark: cycles per two-class row (TwoClassModel::row, float64)
// with rows held in registers (no LDS, no global traffic), for U rows in
// flight per lane and W waves per SIMD.  Isolates the row math's issue /
// latency behaviour from the kernel's memory phases.
//   hipcc --offload-arch=gfx950 -O3 -I include -I custom_envs_amd/csrc \
//         scripts/row_costs.hip -o scripts/bin/row_costs
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#include "optimize_kernels.h"

constexpr int F = 10;
constexpr int ROWS = 256;

template <int U>
__global__ __launch_bounds__(1024) void rows_kernel(double *out, unsigned long long *t, double seed) {
    using Model = ce::TwoClassModel<double, F>;
    const int lane = threadIdx.x & 63;
    double wd[F], x[U][F];
#pragma unroll
    for (int f = 0; f < F; ++f) {
        wd[f] = 0.3 * ((f * 7 + lane) % 11 - 5) * seed;
#pragma unroll
        for (int u = 0; u < U; ++u) x[u][f] = 0.1 * ((f * 3 + lane + u) % 13 - 6);
    }
    double acc[16] = {0}, loss = 0, prod = 1;
    int hits = 0;
    Model::Watch wt;
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ROWS; i += U) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            x[u][0] += 1e-3;   // a new row each iteration
            Model::row<true, false>(x[u], wd, nullptr, 0, true, acc, loss, prod, hits, wt);
        }
        if ((i & 15) == 15) { loss -= ce::log_pos(prod); prod = 1; }
    }
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    double s = loss + hits + wt.tmax;
    for (int j = 0; j < 16; ++j) s += acc[j];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) t[(blockIdx.x * blockDim.x + threadIdx.x) >> 6] = t1 - t0;
}

int main() {
    double *out;
    unsigned long long *t;
    const int maxw = 256 * 16;
    if (hipMalloc(&out, sizeof(double) * maxw * 64) != hipSuccess) return 1;
    if (hipMalloc(&t, sizeof(unsigned long long) * maxw) != hipSuccess) return 1;
    std::vector<unsigned long long> h(maxw);
    using K = void (*)(double *, unsigned long long *, double);
    struct { int u; K k; } ks[] = {{1, rows_kernel<1>}, {2, rows_kernel<2>}, {4, rows_kernel<4>}};
    for (auto &kk : ks)
        for (int wps : {1, 2, 4}) {
            const int threads = 256 * wps;          // one block per CU, wps waves per SIMD
            for (int rep = 0; rep < 2; ++rep)
                hipLaunchKernelGGL(kk.k, dim3(256), dim3(threads), 0, 0, out, t, 1.0);
            if (hipDeviceSynchronize() != hipSuccess) return 2;
            const int nw = 256 * threads / 64;
            if (hipMemcpy(h.data(), t, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost) != hipSuccess) return 3;
            std::sort(h.begin(), h.begin() + nw);
            const double med = static_cast<double>(h[nw / 2]);
            printf("{\"U\": %d, \"waves_per_simd\": %d, \"cycles_per_row_per_wave\": %.1f, "
                   "\"simd_cycles_per_row\": %.1f}\n", kk.u, wps, med / ROWS, med / ROWS / wps);
        }
    return 0;
}
