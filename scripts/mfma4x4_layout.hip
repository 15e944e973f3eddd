// Probe (round 6): the operand / result lane layout of v_mfma_f64_4x4x4f64
// (4 blocks of 4x4x4) on gfx950, and whether its products are the FMA chain
// of the 16x16x4 form.  For every lane j: A[l] = l + 1 (distinct per lane),
// B[l] = (l == j), C = 0; the lanes of D that become nonzero, and the A
// value each holds, name (block, row m, k) of A lane and (block, k, col n) of
// B lane j.  One wave, no other work.
//   hipcc --offload-arch=gfx950 -O3 scripts/mfma4x4_layout.hip -o /tmp/mfma4x4_layout
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(double *out) {
    const int l = threadIdx.x;
    for (int j = 0; j < 64; ++j) {
        const double a = l + 1.0, b = l == j ? 1.0 : 0.0;
        const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
        out[j * 64 + l] = d;
    }
}

int main() {
    double *d_out, h_out[64 * 64];
    if (hipMalloc(&d_out, sizeof(h_out)) != hipSuccess) return 1;
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d_out);
    if (hipMemcpy(h_out, d_out, sizeof(h_out), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    printf("{\"instr\": \"v_mfma_f64_4x4x4f64\", \"by_b_lane\": [");
    for (int j = 0; j < 64; ++j) {
        printf("%s[", j ? ", " : "");
        bool first = true;
        for (int l = 0; l < 64; ++l)
            if (h_out[j * 64 + l] != 0.0) {
                printf("%s[%d, %d]", first ? "" : ", ", l, static_cast<int>(h_out[j * 64 + l]) - 1);
                first = false;
            }
        printf("]");
    }
    printf("]}\n");
    return hipFree(d_out) == hipSuccess ? 0 : 1;
}
