// Launch cost vs per-wave resources: an (almost) empty kernel of 256
// workgroups replayed back to back in a hipGraph, with 512- or 1024-thread
// workgroups, a forced VGPR allocation (inline asm touching v127 / v255) and
// a dynamic LDS allocation.  Also the spread of wave start times
// (s_memrealtime, 100 MHz) of one launch whose waves each live ~5 us (so
// workgroups that do not fit at once start a round later).
//   hipcc --offload-arch=gfx950 -O3 scripts/launch_res.hip -o scripts/bin/launch_res
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <algorithm>

template <int BLOCK, int VG>
__global__ __launch_bounds__(BLOCK) void touch(float *out, unsigned long long *st, int n) {
    extern __shared__ float lds[];
    unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    if constexpr (VG >= 128) asm volatile("v_mov_b32 v127, 0" ::: "v127");
    if constexpr (VG >= 256) asm volatile("v_mov_b32 v255, 0" ::: "v255");
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (threadIdx.x == 0) lds[0] = 1.0f;
    if (i < n) out[i] = 1.0f;
    if (st) {   // the start-spread launch: every wave lives ~5 us
        while (__builtin_amdgcn_s_memrealtime() - t0 < 500) __builtin_amdgcn_s_sleep(2);
        if ((threadIdx.x & 63) == 0) st[i >> 6] = t0;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int BLOCK, int VG>
int run(hipStream_t s, float *buf, unsigned long long *st, int lds_bytes) {
    const int grid = 256, K = 500;
    if (lds_bytes > 65536)
        CK(hipFuncSetAttribute(reinterpret_cast<const void *>(touch<BLOCK, VG>),
                               hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < K; ++k)
        hipLaunchKernelGGL((touch<BLOCK, VG>), dim3(grid), dim3(BLOCK), lds_bytes, s, buf, nullptr, grid * BLOCK);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int r = 0; r < 4; ++r) CK(hipGraphLaunch(ge, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    // start spread of one launch (after a warm launch)
    const int waves = grid * BLOCK / 64;
    hipLaunchKernelGGL((touch<BLOCK, VG>), dim3(grid), dim3(BLOCK), lds_bytes, s, buf, st, grid * BLOCK);
    hipLaunchKernelGGL((touch<BLOCK, VG>), dim3(grid), dim3(BLOCK), lds_bytes, s, buf, st, grid * BLOCK);
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(waves);
    CK(hipMemcpy(h.data(), st, waves * 8, hipMemcpyDeviceToHost));
    std::sort(h.begin(), h.end());
    printf("{\"block\": %d, \"vgpr\": %d, \"lds\": %d, \"us_per_launch\": %.3f, \"start_p50_us\": %.2f, \"start_p90_us\": %.2f, \"start_max_us\": %.2f}\n",
           BLOCK, VG, lds_bytes, ms * 1e3 / (4 * K), (h[waves / 2] - h[0]) / 100.0,
           (h[waves * 9 / 10] - h[0]) / 100.0, (h[waves - 1] - h[0]) / 100.0);
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return 0;
}

int main() {
    float *buf;
    unsigned long long *st;
    CK(hipMalloc(&buf, 64 << 20));
    CK(hipMalloc(&st, 8 << 20));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    for (int lds : {0, 49152, 73728}) {
        if (run<256, 32>(s, buf, st, lds)) return 1;
        if (run<256, 256>(s, buf, st, lds)) return 1;
        if (run<512, 32>(s, buf, st, lds)) return 1;
        if (run<512, 128>(s, buf, st, lds)) return 1;
        if (run<512, 256>(s, buf, st, lds)) return 1;
        if (run<1024, 32>(s, buf, st, lds)) return 1;
        if (run<1024, 128>(s, buf, st, lds)) return 1;
    }
    return 0;
}
