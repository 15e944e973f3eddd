// Accuracy of v_rcp_f64 + k Newton steps on d in [1, 4] (the range
// rcp_unit sees: d = 1 + t, t in [0, 1] ... plus margin), against IEEE 1/d.
// Prints max |ulp| error for k = 0, 1, 2 as one JSON line.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <cstring>
#include <vector>

__global__ void rcp_k(const double *d, double *o0, double *o1, double *o2, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    double x = d[i];
    double r = __builtin_amdgcn_rcp(x);
    o0[i] = r;
    double e = fma(-x, r, 1.0);
    double r1 = fma(r, e, r);
    o1[i] = r1;
    e = fma(-x, r1, 1.0);
    o2[i] = fma(r1, e, r1);
}

static int64_t ulps(double a, double b) {
    int64_t ia, ib;
    std::memcpy(&ia, &a, 8); std::memcpy(&ib, &b, 8);
    return ia > ib ? ia - ib : ib - ia;
}

int main() {
    const int n = 1 << 22;
    std::vector<double> h(n);
    uint64_t s = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        h[i] = 1.0 + 3.0 * (double)(s >> 11) * 0x1.0p-53;
    }
    h[0] = 1.0; h[1] = 2.0; h[2] = 4.0; h[3] = std::nextafter(1.0, 2.0); h[4] = std::nextafter(2.0, 1.0);
    double *d, *o[3];
    (void)hipMalloc(&d, n * 8);
    for (auto &p : o) (void)hipMalloc(&p, n * 8);
    (void)hipMemcpy(d, h.data(), n * 8, hipMemcpyHostToDevice);
    rcp_k<<<n / 256, 256>>>(d, o[0], o[1], o[2], n);
    if (hipDeviceSynchronize() != hipSuccess) return 1;
    std::vector<double> r(n);
    printf("{\"n\": %d", n);
    for (int k = 0; k < 3; ++k) {
        (void)hipMemcpy(r.data(), o[k], n * 8, hipMemcpyDeviceToHost);
        int64_t mx = 0; double sum = 0;
        for (int i = 0; i < n; ++i) { int64_t u = ulps(r[i], 1.0 / h[i]); mx = u > mx ? u : mx; sum += u; }
        printf(", \"newton%d_max_ulp\": %lld, \"newton%d_mean_ulp\": %.4f", k, (long long)mx, k, sum / n);
    }
    printf("}\n");
    return 0;
}
