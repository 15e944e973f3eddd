// Launchers of the runtime-shape f64 MFMA Optimize-v0 kernel: one instance
// per forward k-step count NK = ceil(F / 4), in a translation unit of its own.
#include "optimize_mfma.h"

#include "common.h"
#include "optimize_mfma_kernel.h"

namespace ce {

namespace {

using GenFn = void (*)(const StepArgs<double> &, hipStream_t);

template <int NK>
void launch_nk(const StepArgs<double> &a, hipStream_t stream) {
    const int grid = (a.E + kGenWaves - 1) / kGenWaves;
    hipLaunchKernelGGL((optimize_mfma_kernel<NK>), dim3(grid), dim3(kGenBlock),
                       gen_lds_bytes((NK + 3) / 4), stream, a);
}

template <int... NKs>
struct Table {
    static constexpr GenFn steps[sizeof...(NKs)] = {launch_nk<NKs>...};
    static int set_lds_limits() {
        const void *fns[] = {reinterpret_cast<const void *>(optimize_mfma_kernel<NKs>)...};
        const int ft[] = {((NKs + 3) / 4)...};
        for (size_t i = 0; i < sizeof...(NKs); ++i)
            CE_HIP(hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize,
                                       static_cast<int>(gen_lds_bytes(ft[i]))));
        return CE_OK;
    }
};
using Gen = Table<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>;
static_assert(16 == kGenMaxF / 4, "one instance per k-step count");

}  // namespace

int gen_stride_of(int n_features) { return gen_stride(gen_ft(n_features)); }
int gen_rows_padded_of(int n_rows) { return gen_rows_padded(n_rows); }
int gen_set_lds_limits() { return Gen::set_lds_limits(); }

void gen_launch_step(const StepArgs<double> &a, hipStream_t stream) {
    Gen::steps[(a.F + 3) / 4 - 1](a, stream);
}

void gen_launch_reset(const StepArgs<double> &a, hipStream_t stream) {
    const int grid = (a.E + kGenResetWaves - 1) / kGenResetWaves;
    hipLaunchKernelGGL(optimize_reset_rt_kernel, dim3(grid), dim3(kWave * kGenResetWaves), 0,
                       stream, a);
}

}  // namespace ce
