// Launchers of the runtime-shape f64 MFMA Optimize-v0 kernel: one instance
// per forward k-step count NK = ceil(F / 4), in a translation unit of its own.
#include "optimize_mfma.h"

#include "common.h"
#include "optimize_cat_kernel.h"
#include "optimize_lr_mfma.h"
#include "optimize_mfma_kernel.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

namespace ce {

namespace {

using GenFn = void (*)(const StepArgs<double> &, hipStream_t);

// The class-concatenated full-batch kernel (optimize_cat_kernel.h), compiled
// for the shapes listed in kCatShapes; gen_cat = 0 (CE_GEN_CAT=0) keeps the
// one-env-per-wave kernel.
template <int NK, bool TAIL, int K>
void launch_cat(const StepArgs<double> &a, hipStream_t stream) {
    const int grid = (a.E + kCatEnvs - 1) / kCatEnvs;
    hipLaunchKernelGGL((optimize_cat_kernel<NK, TAIL, K>), dim3(grid), dim3(kCatBlock),
                       cat_lds_bytes((NK + 3) / 4, cat_mt(K)), stream, a);
}
struct CatShape {
    int nk, tail, k;
    GenFn fn;
    const void *kernel;
    size_t lds;
};
#define CE_CAT(NK, TAIL, K)                                                                   \
    {NK, TAIL, K, launch_cat<NK, TAIL, K>,                                                   \
     reinterpret_cast<const void *>(optimize_cat_kernel<NK, TAIL, K>),                       \
     cat_lds_bytes((NK + 3) / 4, cat_mt(K))}
// the reference's image sets (49 features, 10 classes) and the smaller
// shapes that exercise the same paths in tests (no tail, class padding)
const CatShape kCatShapes[] = {CE_CAT(13, true, 10), CE_CAT(5, true, 10), CE_CAT(4, false, 10),
                               CE_CAT(3, false, 3), CE_CAT(8, false, 16)};
#undef CE_CAT

const CatShape *find_cat(const StepArgs<double> &a) {
    const int nk = (a.F + 3) / 4;
    const int tail = a.F == 4 * (nk - 1) + 1 && nk % 4 == 1 && nk > 1 ? 1 : 0;
    for (const auto &c : kCatShapes)
        if (c.nk == nk && c.tail == tail && c.k == a.K) return &c;
    return nullptr;
}

template <int NK>
void launch_nk(const StepArgs<double> &a, hipStream_t stream) {
    if (a.B == a.N && a.gen_cat)
        if (const CatShape *c = find_cat(a)) {
            c->fn(a, stream);
            return;
        }
    const int grid = (a.E + kGenWaves - 1) / kGenWaves;
    // F = 16 (FT - 1) + 1 with the full data set: the last feature on the VALU
    if constexpr (NK % 4 == 1 && NK > 1) {
        if (a.F == 4 * (NK - 1) + 1 && a.B == a.N && a.gen_tail) {
            hipLaunchKernelGGL((optimize_mfma_kernel<NK, true>), dim3(grid), dim3(kGenBlock),
                               gen_lds_bytes((NK + 3) / 4), stream, a);
            return;
        }
    }
    hipLaunchKernelGGL((optimize_mfma_kernel<NK, false>), dim3(grid), dim3(kGenBlock),
                       gen_lds_bytes((NK + 3) / 4), stream, a);
}

template <int... NKs>
struct Table {
    static constexpr GenFn steps[sizeof...(NKs)] = {launch_nk<NKs>...};
    static int set_lds_limits() {
        const void *fns[] = {reinterpret_cast<const void *>(optimize_mfma_kernel<NKs, false>)...,
                             reinterpret_cast<const void *>(optimize_mfma_kernel<NKs, (NKs % 4 == 1 && NKs > 1)>)...};
        const int ft[] = {((NKs + 3) / 4)..., ((NKs + 3) / 4)...};
        for (size_t i = 0; i < 2 * sizeof...(NKs); ++i)
            CE_HIP(hipFuncSetAttribute(fns[i], hipFuncAttributeMaxDynamicSharedMemorySize,
                                       static_cast<int>(gen_lds_bytes(ft[i]))));
        return CE_OK;
    }
};
using Gen = Table<1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16>;
static_assert(16 == kGenMaxF / 4, "one instance per k-step count");

// The wave count W and row-loop mode of a launch.  Wave count: 4 waves per
// workgroup (one per SIMD, tiles 4 at a time, software-pipelined) when every
// wave gets whole groups of 4 tiles and either the grid fills the chip or
// there is one group per wave: at 256 x 10, 5.96 us per 4096-env launch
// against 6.06 at 8 waves and 7.0 at 16, and 5.44 / 5.54 / 6.49 at 1024
// envs (the row work is the same f64 work at every wave
// count; more waves cost more in the fixed phases).  Otherwise 8 waves,
// which halve each wave's rows when a small grid has many of them.
// lr_waves = 4, 8 or 16 (CE_LR_WAVES at ce_create) forces one.  The mode is
// lr_mode capped by mode_cap (CE_LR_MODE at ce_create) and by what the wave count is compiled for
// (4 tiles per group at W <= 4, 2 at W <= 8).
void lr_choice(int E, int N, int lr_waves, int mode_cap, int *w_out, int *mode_out) {
    const int groups = (E + kLrEnvs - 1) / kLrEnvs;
    const int ntiles = (N + 15) / 16;
    const int w = lr_waves ? lr_waves : lr_mode(N, 4) == 3 && (groups >= 256 || ntiles <= 16) ? 4 : 8;
    int mode = std::min(lr_mode(N, w), mode_cap);
    if (mode == 3 && w > 4) mode = 2;
    if (mode == 2 && w > 8) mode = 1;
    *w_out = w;
    *mode_out = mode;
}

// E | F << 24: the two-class kernel's preloaded size word (E < 2^24, F <= 16)
unsigned lr_ef(const StepArgs<double> &a) {
    return static_cast<unsigned>(a.E) | (static_cast<unsigned>(a.F) << 24);
}

template <int NKF, int W>
void launch_lr_w(const StepArgs<double> &a, int mode, hipStream_t stream) {
    const int grid = (a.E + kLrEnvs - 1) / kLrEnvs;
    const dim3 block(LrShape<W>::kBlock);
    if constexpr (W <= 4) {
        if (mode == 3) {
            hipLaunchKernelGGL((optimize_lr_mfma_kernel<NKF, 3, W>), dim3(grid), block, 0, stream, a.W, a.act,
                               a.data, a.G, a.step, a.L, lr_ef(a), a.N, a);
            return;
        }
    }
    if constexpr (W <= 8) {   // 16 waves take their tiles one at a time (128 registers)
        if (mode == 2) {
            hipLaunchKernelGGL((optimize_lr_mfma_kernel<NKF, 2, W>), dim3(grid), block, 0, stream, a.W, a.act,
                               a.data, a.G, a.step, a.L, lr_ef(a), a.N, a);
            return;
        }
    }
    if (mode >= 1)
        hipLaunchKernelGGL((optimize_lr_mfma_kernel<NKF, 1, W>), dim3(grid), block, 0, stream, a.W, a.act,
                               a.data, a.G, a.step, a.L, lr_ef(a), a.N, a);
    else
        hipLaunchKernelGGL((optimize_lr_mfma_kernel<NKF, 0, W>), dim3(grid), block, 0, stream, a.W, a.act,
                               a.data, a.G, a.step, a.L, lr_ef(a), a.N, a);
}

template <int NKF>
void launch_lr(const StepArgs<double> &a, hipStream_t stream) {
    int w, mode;
    lr_choice(a.E, a.N, a.lr_waves, a.lr_mode_cap, &w, &mode);
    if (w == 16) launch_lr_w<NKF, 16>(a, mode, stream);
    else if (w == 4) launch_lr_w<NKF, 4>(a, mode, stream);
    else launch_lr_w<NKF, 8>(a, mode, stream);
}
constexpr GenFn kLrSteps[4] = {launch_lr<1>, launch_lr<2>, launch_lr<3>, launch_lr<4>};

}  // namespace

bool lr_shape_ok(int n_features, int n_classes) { return lr_mfma_shape(n_features, n_classes); }

size_t lr_image_doubles(int n_features, int n_rows) {
    return static_cast<size_t>((n_rows + 15) / 16) * lr_tile_doubles(lr_nkf(n_features)) + kLrMaxF +
           kLrExpTab;
}

void lr_build_image(int F, int N, const double *x, const int32_t *y, double *img) {
    const int nkf = lr_nkf(F), TD = lr_tile_doubles(nkf), ntiles = (N + 15) / 16;
    // sign-folded rows s_y x (s_y = +1 for y = 0, -1 for y = 1): exact
    auto xt = [&](int r, int f) -> double {
        if (r >= N || f >= F) return 0.0;
        return y[r] != 0 ? -x[static_cast<size_t>(r) * F + f] : x[static_cast<size_t>(r) * F + f];
    };
    auto label = [&](int r) -> int32_t { return r < N ? y[r] : -1; };
    for (int t = 0; t < ntiles; ++t) {
        double *ti = img + static_cast<size_t>(t) * TD;
        for (int l = 0; l < kWave; ++l) {
            const int c = l & 15, h = l >> 4;
            for (int k = 0; k < nkf; ++k) ti[k * kWave + l] = xt(16 * t + c, 4 * k + h);
            for (int q = 0; q < 4; ++q) ti[(nkf + q) * kWave + l] = xt(16 * t + h + 4 * q, c);
            int32_t lab[4];
            for (int q = 0; q < 4; ++q) lab[q] = label(16 * t + h + 4 * q);
            std::memcpy(&ti[(nkf + 4) * kWave + l], &lab[0], 8);
            std::memcpy(&ti[(nkf + 5) * kWave + l], &lab[2], 8);
        }
    }
    double *colmax = img + static_cast<size_t>(ntiles) * TD;   // the |u| bound's column maxima
    for (int f = 0; f < kLrMaxF; ++f) {
        double m = 0.0;
        for (int r = 0; f < F && r < N; ++r) m = std::max(m, std::fabs(x[static_cast<size_t>(r) * F + f]));
        colmax[f] = m;
    }
    // then T[j] = 2^(j/2048), rounded to float64 (exp_neg_tab, exp2_table.h)
    static const double kTab[kLrExpTab] = CE_EXP2_TAB;
    std::memcpy(colmax + kLrMaxF, kTab, sizeof(kTab));
}

void lr_launch_step(const StepArgs<double> &a, hipStream_t stream) {
    kLrSteps[lr_nkf(a.F) - 1](a, stream);
}

std::string lr_kernel_name(int n_envs, int n_rows, int n_features, int lr_waves, int mode_cap) {
    int w, mode;
    lr_choice(n_envs, n_rows, lr_waves, mode_cap, &w, &mode);
    return "optimize_lr_mfma_kernel<" + std::to_string(lr_nkf(n_features)) + "," +
           std::to_string(mode) + "," + std::to_string(w) + ">";
}

int gen_stride_of(int n_features) { return gen_stride(gen_ft(n_features)); }
int gen_rows_padded_of(int n_rows) { return gen_rows_padded(n_rows); }
int gen_set_lds_limits() {
    for (const auto &c : kCatShapes)
        CE_HIP(hipFuncSetAttribute(c.kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                   static_cast<int>(c.lds)));
    return Gen::set_lds_limits();
}

std::string gen_kernel_name(int n_envs, int n_rows, int batch, int n_features, int n_classes,
                            int gen_cat) {
    (void)n_envs;
    StepArgs<double> a{};
    a.N = n_rows;
    a.B = batch;
    a.F = n_features;
    a.K = n_classes;
    const int nk = (n_features + 3) / 4;
    if (batch == n_rows && gen_cat)
        if (const CatShape *c = find_cat(a))
            return "optimize_cat_kernel<" + std::to_string(nk) + "," + (c->tail ? "true" : "false") +
                   "," + std::to_string(n_classes) + ">";
    return "optimize_mfma_kernel<" + std::to_string(nk) + ">";
}

void gen_launch_step(const StepArgs<double> &a, hipStream_t stream) {
    Gen::steps[(a.F + 3) / 4 - 1](a, stream);
}

void gen_launch_reset(const StepArgs<double> &a, hipStream_t stream) {
    const int grid = (a.E + kGenResetWaves - 1) / kGenResetWaves;
    hipLaunchKernelGGL(optimize_reset_rt_kernel, dim3(grid), dim3(kWave * kGenResetWaves), 0,
                       stream, a);
}

}  // namespace ce
