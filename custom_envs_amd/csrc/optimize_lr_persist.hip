// Launchers of the K-step two-class kernel (optimize_lr_persist.h): one
// instance per forward k-step count NKF = ceil(F / 4), row tiles per wave
// TPW and padding, in a translation unit of its own.
#include "optimize_mfma.h"

#include "common.h"
#include "optimize_lr_persist.h"

#include <cstdlib>
#include <cstring>

namespace ce {

namespace {

using PersistFn = void (*)(const StepArgs<double> &, const ManyArgs &, hipStream_t);

template <int NKF, int TPW, bool PAD, int W>
void launch_persist(const StepArgs<double> &a, const ManyArgs &m, hipStream_t stream) {
    const int grid = (a.E + kLrEnvs - 1) / kLrEnvs;
    hipLaunchKernelGGL((optimize_lr_persist_kernel<NKF, TPW, PAD, W>), dim3(grid), dim3(kWave * W), 0,
                       stream, a, m);
}

template <int NKF, int TPW, bool PAD>
void launch_persist_ws(const StepArgs<double> &a, const ManyArgs &m, hipStream_t stream) {
    const int grid = (a.E + kLrEnvs - 1) / kLrEnvs;
    // the prologue's pointers and sizes lead (preloaded into SGPRs, build.py);
    // E | F << 24 as the one-step kernel's size word (E < 2^24, F <= 16)
    const unsigned ef = static_cast<unsigned>(a.E) | (static_cast<unsigned>(a.F) << 24);
    hipLaunchKernelGGL((optimize_lr_persist_ws_kernel<NKF, TPW, PAD>), dim3(grid), dim3(512), 0, stream,
                       a.W, a.act, a.data, a.G, a.step, a.L, ef, a.N, a, m);
}

template <int NKF, bool PAD>
constexpr PersistFn kWsByTpw[3] = {launch_persist_ws<NKF, 1, PAD>, launch_persist_ws<NKF, 2, PAD>,
                                   launch_persist_ws<NKF, 4, PAD>};

template <bool PAD>
PersistFn pick_ws(int nkf, int tpw) {
    const int i = tpw == 1 ? 0 : tpw == 2 ? 1 : 2;
    switch (nkf) {
        case 1: return kWsByTpw<1, PAD>[i];
        case 2: return kWsByTpw<2, PAD>[i];
        case 3: return kWsByTpw<3, PAD>[i];
        default: return kWsByTpw<4, PAD>[i];
    }
}

// the wave-specialised form (row waves + epilogue waves): CE_LP_FORM=plain
// selects the all-roles form instead (A/B runs)
bool lp_ws() {
    static const bool ws = [] {
        const char *v = std::getenv("CE_LP_FORM");
        return !(v && std::strcmp(v, "plain") == 0);
    }();
    return ws;
}

template <int NKF, bool PAD, int W>
constexpr PersistFn kByTpw[4] = {launch_persist<NKF, 1, PAD, W>, launch_persist<NKF, 2, PAD, W>,
                                 launch_persist<NKF, 4, PAD, W>, launch_persist<NKF, 8, PAD, W>};

int tpw_index(int tpw) { return tpw == 1 ? 0 : tpw == 2 ? 1 : tpw == 4 ? 2 : 3; }

template <bool PAD, int W>
PersistFn pick(int nkf, int tpw) {
    const int i = tpw_index(tpw);
    switch (nkf) {
        case 1: return kByTpw<1, PAD, W>[i];
        case 2: return kByTpw<2, PAD, W>[i];
        case 3: return kByTpw<3, PAD, W>[i];
        default: return kByTpw<4, PAD, W>[i];
    }
}

// waves per workgroup: CE_LP_WAVES=8 (two per SIMD, A/B runs) for the
// benchmark's NKF = 3; 4 otherwise
int lp_waves(int nkf) {
    static const int w = [] {
        const char *v = std::getenv("CE_LP_WAVES");
        return v && std::atoi(v) == 8 ? 8 : 4;
    }();
    return nkf == 3 ? w : 4;
}

}  // namespace

bool lr_persist_ok(int n_rows) { return n_rows > 0 && lp_tpw(n_rows) > 0; }

void lr_launch_persist(const StepArgs<double> &a, int k, long long act_stride, long long out_step,
                       hipStream_t stream) {
    const ManyArgs m{k, act_stride, out_step};
    const int nkf = lr_nkf(a.F);
    const int w = lp_waves(nkf);
    if (w == 8 && lp_tpw(a.N, 8) > 0 && lp_tpw(a.N, 8) <= 4) {
        const int tpw = lp_tpw(a.N, 8);
        const PersistFn fn3[2][3] = {{launch_persist<3, 1, false, 8>, launch_persist<3, 2, false, 8>,
                                      launch_persist<3, 4, false, 8>},
                                     {launch_persist<3, 1, true, 8>, launch_persist<3, 2, true, 8>,
                                      launch_persist<3, 4, true, 8>}};
        fn3[lp_pad(a.N, 8) ? 1 : 0][tpw_index(tpw)](a, m, stream);
        return;
    }
    const int tpw = lp_tpw(a.N);
    if (lp_ws() && tpw <= 4) {   // 8 tiles per wave do not fit two waves per SIMD
        (lp_pad(a.N) ? pick_ws<true>(nkf, tpw) : pick_ws<false>(nkf, tpw))(a, m, stream);
        return;
    }
    (lp_pad(a.N) ? pick<true, 4>(nkf, tpw) : pick<false, 4>(nkf, tpw))(a, m, stream);
}

std::string lr_persist_name(int n_rows, int n_features) {
    const int nkf = lr_nkf(n_features);
    const int w = lp_waves(nkf) == 8 && lp_tpw(n_rows, 8) > 0 && lp_tpw(n_rows, 8) <= 4 ? 8 : 4;
    if (w == 4 && lp_ws() && lp_tpw(n_rows) <= 4)
        return "optimize_lr_persist_ws_kernel<" + std::to_string(nkf) + "," +
               std::to_string(lp_tpw(n_rows)) + "," + (lp_pad(n_rows) ? "true" : "false") + ">";
    return "optimize_lr_persist_kernel<" + std::to_string(nkf) + "," +
           std::to_string(lp_tpw(n_rows, w)) + "," + (lp_pad(n_rows, w) ? "true" : "false") + "," +
           std::to_string(w) + ">";
}

}  // namespace ce
