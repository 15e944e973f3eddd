// Which XCD runs workgroup b of launch k?  Each workgroup records its
// HW_REG_XCC_ID; 8 launches of 256 workgroups (one per CU).  Then a latency
// probe: kernel W stores a 4 KB slice per workgroup, kernel R (next launch,
// same workgroup ids) times one dependent load of its slice, once with the
// slice chosen by workgroup id and once by an XCD-stable remap
// (slot = 8 * (b / 8) + xcc).
//   hipcc --offload-arch=gfx950 -O3 scripts/xcd_map.hip -o scripts/bin/xcd_map
#include <hip/hip_runtime.h>
#include <cstdio>
#include <algorithm>
#include <vector>

__device__ __forceinline__ unsigned xcc_id() {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

__global__ void map_kernel(unsigned *out) {
    if (threadIdx.x == 0) out[blockIdx.x] = xcc_id();
}

__device__ __forceinline__ unsigned slot_of(bool remap) {
    const unsigned b = blockIdx.x;
    return remap ? 8 * (b / 8) + xcc_id() : b;
}

__global__ void write_kernel(double *buf, bool remap, double v) {
    const unsigned s = slot_of(remap);
    for (int i = threadIdx.x; i < 512; i += blockDim.x) buf[s * 512 + i] = v + i;
}

__global__ void read_kernel(const double *buf, bool remap, unsigned long long *lat, double *sink) {
    const unsigned s = slot_of(remap);
    unsigned long long t0 = __builtin_amdgcn_s_memtime();
    double x = buf[s * 512 + threadIdx.x];
    x += buf[s * 512 + 256 + threadIdx.x];
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) lat[blockIdx.x] = t1 - t0;
    if (x == -1.0) sink[0] = x;
}

int main() {
    const int nb = 256, nl = 8;
    unsigned *d;
    hipMalloc(&d, nb * nl * sizeof(unsigned));
    for (int k = 0; k < nl; ++k) hipLaunchKernelGGL(map_kernel, dim3(nb), dim3(64), 0, 0, d + k * nb);
    std::vector<unsigned> h(nb * nl);
    hipMemcpy(h.data(), d, h.size() * sizeof(unsigned), hipMemcpyDeviceToHost);
    printf("{\"map\": [");
    for (int k = 0; k < nl; ++k) {
        printf("%s[", k ? ", " : "");
        for (int b = 0; b < 16; ++b) printf("%s%u", b ? ", " : "", h[k * nb + b]);
        printf("]");
    }
    printf("]}\n");
    double *buf, *sink;
    unsigned long long *lat;
    hipMalloc(&buf, nb * 512 * sizeof(double));
    hipMalloc(&sink, 8);
    hipMalloc(&lat, nb * sizeof(unsigned long long));
    for (int remap = 0; remap < 2; ++remap) {
        std::vector<unsigned long long> all;
        for (int rep = 0; rep < 20; ++rep) {
            hipLaunchKernelGGL(write_kernel, dim3(nb), dim3(256), 0, 0, buf, remap != 0, 1.0 * rep);
            hipLaunchKernelGGL(read_kernel, dim3(nb), dim3(256), 0, 0, buf, remap != 0, lat, sink);
            std::vector<unsigned long long> l(nb);
            hipMemcpy(l.data(), lat, nb * sizeof(unsigned long long), hipMemcpyDeviceToHost);
            if (rep >= 2) all.insert(all.end(), l.begin(), l.end());
        }
        std::sort(all.begin(), all.end());
        printf("{\"remap\": %d, \"load_ticks_p10\": %llu, \"p50\": %llu, \"p90\": %llu}\n", remap,
               all[all.size() / 10], all[all.size() / 2], all[all.size() * 9 / 10]);
    }
    return 0;
}
