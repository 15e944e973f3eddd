// Launch-floor microbenchmark: how long does an (almost) empty kernel of a
// given grid shape take per launch when replayed back to back in a hipGraph?
// Also reports the shader clock seen by s_memtime vs s_memrealtime (100 MHz).
//   hipcc --offload-arch=gfx950 -O3 scripts/launch_floor.hip -o /tmp/launch_floor
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void touch(float *out, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = 1.0f;
}

__global__ void clock_probe(unsigned long long *o) {
    if (threadIdx.x == 0) {
        unsigned long long t0 = __builtin_amdgcn_s_memtime();
        unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
        double acc = 1.0;
        for (int i = 0; i < 200000; ++i) acc = fma(acc, 1.0000001, 1e-9);
        unsigned long long t1 = __builtin_amdgcn_s_memtime();
        unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
        o[blockIdx.x * 3 + 0] = t1 - t0;
        o[blockIdx.x * 3 + 1] = r1 - r0;
        o[blockIdx.x * 3 + 2] = acc > 0 ? 1 : 0;
    }
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

int main() {
    float *buf;
    CK(hipMalloc(&buf, 64 << 20));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    struct Shape { int grid, block; } shapes[] = {
        {1, 64}, {256, 64}, {1024, 256}, {256, 1024}, {4096, 64}, {512, 512}, {2048, 256}, {16384, 64}};
    const int K = 500;
    for (auto sh : shapes) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int k = 0; k < K; ++k)
            hipLaunchKernelGGL(touch, dim3(sh.grid), dim3(sh.block), 0, s, buf, sh.grid * sh.block);
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        CK(hipGraphLaunch(ge, s));
        CK(hipStreamSynchronize(s));
        CK(hipEventRecord(a, s));
        for (int r = 0; r < 4; ++r) CK(hipGraphLaunch(ge, s));
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        printf("{\"grid\": %d, \"block\": %d, \"waves\": %d, \"us_per_launch\": %.3f}\n", sh.grid, sh.block,
               sh.grid * ((sh.block + 63) / 64), ms * 1e3 / (4 * K));
        CK(hipGraphExecDestroy(ge));
        CK(hipGraphDestroy(g));
    }
    unsigned long long *o;
    CK(hipMalloc(&o, 3 * 8 * 256));
    hipLaunchKernelGGL(clock_probe, dim3(256), dim3(64), 0, s, o);
    CK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(3 * 256);
    CK(hipMemcpy(h.data(), o, h.size() * 8, hipMemcpyDeviceToHost));
    double sum = 0;
    for (int i = 0; i < 256; ++i) sum += double(h[3 * i]) / double(h[3 * i + 1]) * 100.0;
    printf("{\"memtime_mhz_busy_probe\": %.1f}\n", sum / 256);
    return 0;
}
