// C-ABI implementation of the MI355X Optimize-v0 engine (include/custom_envs_amd.h).
//
// Host responsibilities: own the device copy of the dataset and the per-env
// state (struct-of-arrays, one contiguous [E][P] slab per quantity so a
// wave's P values are one coalesced segment), stage host actions/outputs
// through pinned buffers, and launch one fused step kernel per VecEnv.step
// (optimize_kernels.h).  The env RNG is native (seeding.cpp): W0 and the
// reset permutation are drawn once per seed and uploaded, because
// use_random_state never advances the env RNG (custom_envs/utils/
// utils_math.py:9-22), so every reset replays the same draws.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include <algorithm>
#include <thread>

#include "common.h"
#include "mlp_kernels.h"
#include "net_engine.h"
#include "optimize_kernels.h"
#include "optimize_mfma.h"
#include "optimize_pair_kernel.h"
#include "seeding.h"

namespace {

using ce::fail;

using StepFn = void (*)(const void *args, int grid, size_t lds, hipStream_t stream);

template <typename T, int F, int K, bool STAGED>
void launch_step(const void *args, int grid, size_t lds, hipStream_t stream) {
    hipLaunchKernelGGL((ce::optimize_step_kernel<T, F, K, STAGED>), dim3(grid),
                       dim3(ce::kBlock), STAGED ? lds : 0, stream,
                       *static_cast<const ce::StepArgs<T> *>(args));
}

// Two envs per wave (optimize_pair_kernel.h): grid = ceil(E / 16) blocks.
template <typename T, int F, int K, int U>
void launch_pair(const void *args, int, size_t lds, hipStream_t stream) {
    if constexpr (ce::pair_shape(F, K)) {
        const auto &a = *static_cast<const ce::StepArgs<T> *>(args);
        const int grid = (a.E + ce::kPairEnvsPerBlock - 1) / ce::kPairEnvsPerBlock;
        hipLaunchKernelGGL((ce::optimize_pair_kernel<T, F, U>), dim3(grid), dim3(ce::kPairBlock),
                           lds + ce::pair_scratch_bytes<T>(F), stream, a);
    }
}

template <typename T, int F, int K>
void launch_reset(const void *args, int grid, size_t, hipStream_t stream) {
    hipLaunchKernelGGL((ce::optimize_reset_kernel<T, F, K>), dim3(grid), dim3(ce::kBlock), 0,
                       stream, *static_cast<const ce::StepArgs<T> *>(args));
}

struct KernelEntry {
    int precision, F, K;
    StepFn step_staged, step_global, reset;
    StepFn step_pair[2];   // U = 1, 2 (nullptr where the shape has no pair path)
};

// Shapes with a compiled register-path instance.
#define CE_SHAPES(X) \
    X(2, 2) X(4, 2) X(4, 3) X(5, 2) X(8, 2) X(10, 2) X(16, 2) X(20, 2) X(10, 3) X(10, 4) X(3, 3)

#define CE_PAIRS(T, F, K)                                                                   \
    {ce::pair_shape(F, K) ? launch_pair<T, F, K, 1> : nullptr,                              \
     ce::pair_shape(F, K) ? launch_pair<T, F, K, 2> : nullptr}
#define CE_ENTRY(F, K)                                                                \
    {CE_F64, F, K, launch_step<double, F, K, true>, launch_step<double, F, K, false>, \
     launch_reset<double, F, K>, CE_PAIRS(double, F, K)},                             \
    {CE_F32, F, K, launch_step<float, F, K, true>, launch_step<float, F, K, false>,   \
     launch_reset<float, F, K>, CE_PAIRS(float, F, K)},

const KernelEntry kKernels[] = {CE_SHAPES(CE_ENTRY)};

const KernelEntry *find_kernel(int precision, int F, int K) {
    for (const auto &k : kKernels)
        if (k.precision == precision && k.F == F && k.K == K) return &k;
    return nullptr;
}


}  // namespace

struct ce_engine {
    ce_config cfg{};
    int P = 0, obs_dim = 0;
    bool mlp = false;  // CE_PROBLEM_MLP
    ce::NetPlan *net = nullptr;   // CE_PROBLEM_MLP on the layered path (net_engine.hip)
    ce::NetGeom net_geo{};        // its weight-image geometry: W / W0 are [E][Pimg] images
    std::vector<int> dims;        // network: F, hidden..., K
    bool mlp_split = false;  // two launches per step (CE_MLP_SPLIT=1 or CE_MLP_PHASES)
    int mlp_phases = 3;  // bit 0: train kernel, bit 1: info kernel (CE_MLP_PHASES, profiling)
    size_t tsize = 8;  // element size of W / W0
    size_t gsize = 8;  // element size of G (grad_hist)
    const KernelEntry *kern = nullptr;
    hipStream_t own_stream = nullptr;
    hipStream_t stream = nullptr;
    // device state
    void *X = nullptr;
    float *Xs = nullptr;   // MLP: dataset in MFMA operand order (mlp_kernels.h)
    int32_t *label = nullptr;
    void *W = nullptr, *G = nullptr, *W0 = nullptr;
    double *L = nullptr;
    int32_t *step = nullptr;
    int32_t *perm = nullptr, *order = nullptr, *order_sel = nullptr;
    float *d_act = nullptr;
    // outputs: one region on the device, a pinned mirror on the host
    size_t off[6] = {0};
    size_t out_bytes = 0;
    char *d_out = nullptr;
    char *h_out = nullptr;
    float *h_act = nullptr;
    bool was_reset = false;
    bool staged = false;      // dataset fits the per-block LDS stage
    StepFn pair = nullptr;    // two-envs-per-wave step kernel, when the shape has one
    int gen_ft = 0;           // > 0: the runtime-shape MFMA kernel with this many feature tiles
    bool lr_mfma = false;     // two-class full-batch MFMA kernel (optimize_lr_mfma.h)
    std::string kernel_name;  // what ce_step_kernel reports
    size_t stage_bytes = 0;
    ce::GraphCache graphs;   // ce_step_many
    // ce_step_many: k <= many_direct steps are plain launches, longer runs a
    // cached hipGraph.  Measured (4096 envs, pair kernel): 20 steps 7.7 us
    // per step direct vs 8.0 graph; 100 and 2000 steps equal.
    int many_direct = 32;
    int lr_waves = 0;         // CE_LR_WAVES: force the two-class MFMA kernel's wave count
    int gen_tail = 1;         // CE_GEN_TAIL=0: the runtime-shape kernel's last feature on MFMA too
    int gen_cat = 1;          // CE_GEN_CAT=0: full batch on the one-env-per-wave kernel
    int lr_mode_cap = 3;      // CE_LR_MODE: cap on the two-class MFMA kernel's row-loop mode
    bool compact = false;     // ce_set_compact_outputs: device-pointer calls write the compact form
    // the persistent K-step kernel (optimize_lr_persist.h): available for the
    // shape, and chosen (ce_set_persistent; CE_PERSIST=0 at create turns it off)
    bool persist = false, persist_on = true;
    std::string many_name;    // what ce_step_many_kernel reports when persistent
    unsigned long long *diag = nullptr;   // CE_DIAG builds: per-wave phase stamps
};

namespace {

ce_outputs region_view(const ce_engine *e, char *base) {
    ce_outputs o;
    o.obs = reinterpret_cast<float *>(base + e->off[0]);
    o.reward = reinterpret_cast<float *>(base + e->off[1]);
    o.objective = reinterpret_cast<float *>(base + e->off[2]);
    o.accuracy = reinterpret_cast<float *>(base + e->off[3]);
    o.episode_len = reinterpret_cast<int32_t *>(base + e->off[4]);
    o.done = reinterpret_cast<uint8_t *>(base + e->off[5]);
    return o;
}

template <typename T>
ce::StepArgs<T> make_args(const ce_engine *e, const float *act, const ce_outputs &o,
                          bool compact = false) {
    ce::StepArgs<T> a;
    a.E = e->cfg.num_envs;
    a.N = e->cfg.n_rows;
    a.B = e->cfg.batch_size;
    a.max_steps = e->cfg.max_steps;
    a.auto_reset = e->cfg.auto_reset;
    a.F = e->cfg.n_features;
    a.K = e->cfg.n_classes;
    a.data = static_cast<const unsigned char *>(e->X);
    a.W = static_cast<T *>(e->W);
    a.G = static_cast<T *>(e->G);
    a.L = e->L;
    a.step = e->step;
    a.W0 = static_cast<const T *>(e->W0);
    a.perm = e->perm;
    a.order = e->order;
    a.order_sel = e->order_sel;
    a.act = act;
    a.obs = o.obs;
    a.reward = o.reward;
    a.done = o.done;
    a.objective = o.objective;
    a.accuracy = o.accuracy;
    a.episode_len = o.episode_len;
    a.diag = e->diag;
    a.inv_B = 1.0 / static_cast<double>(e->cfg.batch_size);
    const int P = e->cfg.n_features * e->cfg.n_classes;
    a.p_mul = (65536 + P - 1) / P;
    a.lr_waves = e->lr_waves;
    a.gen_tail = e->gen_tail;
    a.gen_cat = e->gen_cat;
    a.lr_mode_cap = e->lr_mode_cap;
    a.obs_stride = compact ? P + 1 : 2 * P + 1;
    a.obs_lo = compact ? P : 0;
    return a;
}

int grid_of(const ce_engine *e) {
    return (e->cfg.num_envs + ce::kWavesPerBlock - 1) / ce::kWavesPerBlock;
}

ce::MlpArgs make_mlp_args(const ce_engine *e, const float *act, const ce_outputs &o) {
    ce::MlpArgs a;
    a.E = e->cfg.num_envs;
    a.N = e->cfg.n_rows;
    a.F = e->cfg.n_features;
    a.K = e->cfg.n_classes;
    a.P = e->P;
    a.max_steps = e->cfg.max_steps;
    a.auto_reset = e->cfg.auto_reset;
    a.X = static_cast<const float *>(e->X);
    a.Xs = e->Xs;
    a.diag = e->diag;
    a.label = e->label;
    a.W = static_cast<float *>(e->W);
    a.W0 = static_cast<const float *>(e->W0);
    a.G = static_cast<double *>(e->G);
    a.L = e->L;
    a.step = e->step;
    a.perm = e->perm;
    a.order = e->order;
    a.order_sel = e->order_sel;
    a.act = act;
    a.obs = o.obs;
    a.reward = o.reward;
    a.done = o.done;
    a.objective = o.objective;
    a.accuracy = o.accuracy;
    a.episode_len = o.episode_len;
    return a;
}

// compact: the caller's device outputs are in the compact form
// (ce_set_compact_outputs; only the two-class MFMA path writes it)
ce::NetArgs make_net_args(const ce_engine *e, const float *act, const ce_outputs &o) {
    ce::NetArgs a{};
    a.E = e->cfg.num_envs;
    a.N = e->cfg.n_rows;
    a.F = e->cfg.n_features;
    a.K = e->cfg.n_classes;
    a.B = e->cfg.batch_size;
    a.P = e->P;
    a.max_steps = e->cfg.max_steps;
    a.auto_reset = e->cfg.auto_reset;
    a.n_hidden = static_cast<int>(e->dims.size()) - 2;
    for (int l = 0; l < a.n_hidden; ++l) a.hidden[l] = e->dims[l + 1];
    a.X = static_cast<const float *>(e->X);
    a.label = e->label;
    a.W = static_cast<float *>(e->W);
    a.W0 = static_cast<const float *>(e->W0);
    a.G = static_cast<double *>(e->G);
    a.L = e->L;
    a.step = e->step;
    a.perm = e->perm;
    a.order = e->order;
    a.order_sel = e->order_sel;
    a.act = act;
    a.obs = o.obs;
    a.reward = o.reward;
    a.done = o.done;
    a.objective = o.objective;
    a.accuracy = o.accuracy;
    a.episode_len = o.episode_len;
    return a;
}

int launch(const ce_engine *e, bool reset, const float *act, const ce_outputs &o,
           hipStream_t stream, bool compact = false) {
    if (e->net) {
        const ce::NetArgs a = make_net_args(e, act, o);
        return reset ? ce::net_reset(e->net, a, stream) : ce::net_step(e->net, a, stream);
    }
    if (e->mlp) {
        const ce::MlpArgs a = make_mlp_args(e, act, o);
        const dim3 grid(e->cfg.num_envs), block(ce::kMlpBlock);
        const bool even = (e->P & 1) == 0;   // pair accesses aligned in every env
        if (reset) {
            hipLaunchKernelGGL(ce::mlp_reset_kernel, grid, block, 0, stream, a);
        } else if (!e->mlp_split) {
            if (even) hipLaunchKernelGGL(ce::mlp_step_kernel<true>, grid, block, 0, stream, a);
            else hipLaunchKernelGGL(ce::mlp_step_kernel<false>, grid, block, 0, stream, a);
        } else {
            if (e->mlp_phases & 1) {
                if (even) hipLaunchKernelGGL(ce::mlp_train_kernel<true>, grid, block, 0, stream, a);
                else hipLaunchKernelGGL(ce::mlp_train_kernel<false>, grid, block, 0, stream, a);
            }
            if (e->mlp_phases & 2) {
                if (even) hipLaunchKernelGGL(ce::mlp_info_kernel<true>, grid, block, 0, stream, a);
                else hipLaunchKernelGGL(ce::mlp_info_kernel<false>, grid, block, 0, stream, a);
            }
        }
        return CE_OK;
    }
    if (e->lr_mfma) {
        auto a = make_args<double>(e, act, o, compact);
        if (reset)
            ce::gen_launch_reset(a, stream);
        else
            ce::lr_launch_step(a, stream);
        return CE_OK;
    }
    if (e->gen_ft) {
        auto a = make_args<double>(e, act, o);
        if (reset)
            ce::gen_launch_reset(a, stream);
        else
            ce::gen_launch_step(a, stream);
        return CE_OK;
    }
    StepFn fn = reset ? e->kern->reset
                      : (e->pair ? e->pair : (e->staged ? e->kern->step_staged : e->kern->step_global));
    if (e->cfg.precision == CE_F64) {
        auto a = make_args<double>(e, act, o);
        fn(&a, grid_of(e), e->stage_bytes, stream);
    } else {
        auto a = make_args<float>(e, act, o);
        fn(&a, grid_of(e), e->stage_bytes, stream);
    }
    return CE_OK;
}

// The outputs of step s of a strided run: every pointer out_step bytes per step.
ce_outputs advance(const ce_outputs &o, int64_t bytes) {
    auto adv = [bytes](auto *p) { return p ? reinterpret_cast<decltype(p)>(reinterpret_cast<char *>(p) + bytes) : p; };
    ce_outputs r;
    r.obs = adv(o.obs);
    r.reward = adv(o.reward);
    r.done = adv(o.done);
    r.objective = adv(o.objective);
    r.accuracy = adv(o.accuracy);
    r.episode_len = adv(o.episode_len);
    return r;
}

// k steps of every env, actions s * stride apart, outputs s * out_step bytes
// apart (one launch per step).
int launch_steps(const ce_engine *e, int k, const float *actions, int64_t stride,
                 const ce_outputs &o, int64_t out_step = 0) {
    for (int s = 0; s < k; ++s) {
        const int rc = launch(e, false, actions + s * stride, out_step ? advance(o, s * out_step) : o,
                              e->stream, e->compact);
        if (rc != CE_OK) return rc;
    }
    return CE_OK;
}

// The k steps as ONE launch of the persistent kernel (optimize_lr_persist.h).
int launch_persist(const ce_engine *e, int k, const float *actions, int64_t stride,
                   const ce_outputs &o, int64_t out_step) {
    const auto a = make_args<double>(e, actions, o, e->compact);
    ce::lr_launch_persist(a, k, stride, out_step, e->stream);
    return CE_OK;
}

// Convert host float64 values to a device array of `elem`-byte floats.
int upload_typed(ce_engine *e, void *dst, const double *src, size_t count, size_t elem) {
    if (elem == sizeof(double)) {
        CE_HIP(hipMemcpyAsync(dst, src, count * sizeof(double), hipMemcpyHostToDevice, e->stream));
    } else {
        std::vector<float> tmp(count);
        for (size_t i = 0; i < count; ++i) tmp[i] = static_cast<float>(src[i]);
        CE_HIP(hipMemcpyAsync(dst, tmp.data(), count * sizeof(float), hipMemcpyHostToDevice,
                              e->stream));
        CE_HIP(hipStreamSynchronize(e->stream));
    }
    return CE_OK;
}

int download_typed(ce_engine *e, double *dst, const void *src, size_t count, size_t elem) {
    if (elem == sizeof(double)) {
        CE_HIP(hipMemcpyAsync(dst, src, count * sizeof(double), hipMemcpyDeviceToHost, e->stream));
        CE_HIP(hipStreamSynchronize(e->stream));
    } else {
        std::vector<float> tmp(count);
        CE_HIP(hipMemcpyAsync(tmp.data(), src, count * sizeof(float), hipMemcpyDeviceToHost,
                              e->stream));
        CE_HIP(hipStreamSynchronize(e->stream));
        for (size_t i = 0; i < count; ++i) dst[i] = tmp[i];
    }
    return CE_OK;
}

// The network path's weight images <-> the flat float64 vectors of ce_state
int net_download(ce_engine *e, double *dst, const void *img) {
    const size_t E = e->cfg.num_envs, P = e->P, PI = static_cast<size_t>(e->net_geo.Pimg);
    std::vector<float> tmp(E * PI), flat(P);
    CE_HIP(hipMemcpyAsync(tmp.data(), img, E * PI * sizeof(float), hipMemcpyDeviceToHost, e->stream));
    CE_HIP(hipStreamSynchronize(e->stream));
    for (size_t i = 0; i < E; ++i) {
        ce::net_image_to_flat(e->net_geo, &tmp[i * PI], flat.data());
        for (size_t p = 0; p < P; ++p) dst[i * P + p] = flat[p];
    }
    return CE_OK;
}

int net_upload(ce_engine *e, void *img, const double *src) {
    const size_t E = e->cfg.num_envs, P = e->P, PI = static_cast<size_t>(e->net_geo.Pimg);
    std::vector<float> tmp(E * PI), flat(P);
    for (size_t i = 0; i < E; ++i) {
        for (size_t p = 0; p < P; ++p) flat[p] = static_cast<float>(src[i * P + p]);
        ce::net_flat_to_image(e->net_geo, flat.data(), &tmp[i * PI]);
    }
    CE_HIP(hipMemcpyAsync(img, tmp.data(), E * PI * sizeof(float), hipMemcpyHostToDevice, e->stream));
    CE_HIP(hipStreamSynchronize(e->stream));
    return CE_OK;
}

void copy_out(const ce_engine *e, const ce_outputs &src, const ce_outputs *dst) {
    const size_t E = e->cfg.num_envs;
    if (!dst) return;
    if (dst->obs) std::memcpy(dst->obs, src.obs, E * e->obs_dim * sizeof(float));
    if (dst->reward) std::memcpy(dst->reward, src.reward, E * sizeof(float));
    if (dst->done) std::memcpy(dst->done, src.done, E);
    if (dst->objective) std::memcpy(dst->objective, src.objective, E * sizeof(float));
    if (dst->accuracy) std::memcpy(dst->accuracy, src.accuracy, E * sizeof(float));
    if (dst->episode_len) std::memcpy(dst->episode_len, src.episode_len, E * sizeof(int32_t));
}

// every output pointer set (the compact form may leave done null)
bool complete(const ce_outputs *o, bool compact = false) {
    // the compact form has no done (episode_len >= max_steps) and no reward
    // (-objective: B = N)
    return o && o->obs && (o->reward || compact) && (o->done || compact) && o->objective &&
           o->accuracy && o->episode_len;
}

int do_step(ce_engine *e, const float *actions, const ce_outputs *out, uint32_t flags,
            bool sync) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_CLEAR_STALE_ERROR();
    if (!e->was_reset) return fail(CE_ESTATE, "step() before the first reset()");
    if (!actions) return fail(CE_EINVAL, "null actions");
    const size_t E = e->cfg.num_envs;
    if (flags & CE_PTR_DEVICE) {
        if (e->compact && !out) return fail(CE_EINVAL, "compact outputs need caller buffers");
        ce_outputs o = out ? *out : region_view(e, e->d_out);
        if (out && !complete(out, e->compact)) return fail(CE_EINVAL, "device outputs must all be set");
        const int rc = launch(e, false, actions, o, e->stream, e->compact);
        if (rc != CE_OK) return rc;
        CE_HIP(hipGetLastError());
        if (sync) CE_HIP(hipStreamSynchronize(e->stream));
        return CE_OK;
    }
    std::memcpy(e->h_act, actions, E * e->P * sizeof(float));
    CE_HIP(hipMemcpyAsync(e->d_act, e->h_act, E * e->P * sizeof(float), hipMemcpyHostToDevice,
                          e->stream));
    const int rc = launch(e, false, e->d_act, region_view(e, e->d_out), e->stream);
    if (rc != CE_OK) return rc;
    CE_HIP(hipGetLastError());
    CE_HIP(hipMemcpyAsync(e->h_out, e->d_out, e->out_bytes, hipMemcpyDeviceToHost, e->stream));
    if (sync) {
        CE_HIP(hipStreamSynchronize(e->stream));
        copy_out(e, region_view(e, e->h_out), out);
    }
    return CE_OK;
}

}  // namespace

extern "C" {

int ce_abi_version(void) { return CE_ABI_VERSION; }

const char *ce_last_error(void) { return ce::last_error().c_str(); }

int ce_seed_draws(uint64_t seed, int32_t n_features, int32_t n_classes, int32_t n_rows,
                  double *init_weights, int32_t *perm) {
    if (n_features <= 0 || n_classes <= 0 || n_rows < 0)
        return fail(CE_EINVAL, "ce_seed_draws: bad shape");
    ce::reset_draws(seed, n_features, n_classes, n_rows, init_weights, perm);
    return CE_OK;
}

int ce_seed_draws_mlp(uint64_t seed, int32_t n_features, int32_t n_hidden, int32_t n_classes,
                      int32_t n_rows, float *init_weights, int32_t *perm) {
    if (n_features <= 0 || n_hidden <= 0 || n_classes <= 0 || n_rows < 0)
        return fail(CE_EINVAL, "ce_seed_draws_mlp: bad shape");
    ce::reset_draws_mlp(seed, n_features, n_hidden, n_classes, n_rows, init_weights, perm);
    return CE_OK;
}

int ce_create(const ce_config *cfg, const double *features, const int32_t *labels,
              ce_engine **out) {
    if (!cfg || !features || !labels || !out) return fail(CE_EINVAL, "ce_create: null argument");
    *out = nullptr;
    if (cfg->abi_version != CE_ABI_VERSION)
        return fail(CE_EINVAL, "ce_create: ABI version mismatch");
    if (cfg->problem != CE_PROBLEM_SOFTMAX && cfg->problem != CE_PROBLEM_MLP)
        return fail(CE_EUNSUPPORTED, "ce_create: unknown problem");
    if (cfg->precision != CE_F64 && cfg->precision != CE_F32)
        return fail(CE_EINVAL, "ce_create: unknown precision");
    if (cfg->num_envs <= 0 || cfg->n_rows <= 0 || cfg->n_features <= 0 || cfg->n_classes <= 0)
        return fail(CE_EINVAL, "ce_create: sizes must be positive");
    if (cfg->batch_size <= 0 || cfg->batch_size > cfg->n_rows)
        return fail(CE_EINVAL, "ce_create: batch_size must be in [1, n_rows]");
    if (cfg->max_steps <= 0) return fail(CE_EINVAL, "ce_create: max_steps must be positive");
    const bool mlp = cfg->problem == CE_PROBLEM_MLP;
    const KernelEntry *kern = nullptr;
    bool lr_path = false;
    bool net_path = false;
    std::vector<int> dims;
    if (mlp) {
        if (cfg->precision != CE_F32)
            return fail(CE_EUNSUPPORTED, "ce_create: the MLP problem computes in float32");
        if (cfg->n_layers < 0 || cfg->n_layers > ce::kNetMaxHidden)
            return fail(CE_EUNSUPPORTED, "ce_create: the network takes 1 to 4 hidden layers");
        dims.push_back(cfg->n_features);
        if (cfg->n_layers == 0) dims.push_back(cfg->n_hidden);
        for (int l = 0; l < cfg->n_layers; ++l) dims.push_back(cfg->hidden[l]);
        dims.push_back(cfg->n_classes);
        for (int d : dims)
            if (d <= 0) return fail(CE_EINVAL, "ce_create: network widths must be positive");
        // the fused config-3 kernel (mlp_kernels.h: 784 -> 64 -> 10, B = 32)
        // where its shape holds; every other network on the layered path
        // (net_engine.hip); CE_MLP_NET=1 forces the layered path (tests)
        const char *fn = std::getenv("CE_MLP_NET");
        const bool fused = !(fn && fn[0] == '1') && dims.size() == 3 &&
                           dims[1] == ce::kMlpHidden && cfg->batch_size == ce::kMlpBatch &&
                           cfg->n_features % 8 == 0 && cfg->n_classes <= ce::kMlpMaxK &&
                           cfg->n_rows % 64 == 0 && cfg->batch_size < cfg->n_rows;
        net_path = !fused;
        if (net_path) {   // the hand-written network kernels' limits (net_engine.h)
            ce::NetGeom geo;
            const int rc = ce::net_geometry(static_cast<int>(dims.size()) - 2, dims.data(), &geo);
            if (rc != CE_OK) return rc;
        }
    } else {
        // a register-path instance when the shape has one (unless CE_GENERIC=1
        // forces the runtime-shape kernel, for tests), else the MFMA kernel
        const char *force = std::getenv("CE_GENERIC");
        const bool generic = force && force[0] == '1';
        // The two-class full-batch float64 shapes (the benchmark's) run on
        // the MFMA kernel with envs along N (optimize_lr_mfma.h): 6.09 us
        // per 4096-env step against 6.3 for the two-envs-per-wave register
        // kernel.  CE_LR_MFMA=0 (or CE_PAIR_U) selects the
        // register kernel instead.
        const char *lrm = std::getenv("CE_LR_MFMA");
        lr_path = !generic && !(lrm && lrm[0] == '0') && !std::getenv("CE_PAIR_U") &&
                  cfg->precision == CE_F64 && cfg->batch_size == cfg->n_rows &&
                  cfg->num_envs < (1 << 24) &&      // its packed E | F << 24 argument
                  ce::lr_shape_ok(cfg->n_features, cfg->n_classes);
        if (!generic && !lr_path)
            kern = find_kernel(cfg->precision, cfg->n_features, cfg->n_classes);
        if (!kern && !lr_path) {
            if (cfg->precision != CE_F64 || cfg->n_features > ce::kGenMaxF ||
                cfg->n_classes > ce::kGenMaxClasses)
                return fail(CE_EUNSUPPORTED,
                            "ce_create: no kernel for F=" + std::to_string(cfg->n_features) +
                                " K=" + std::to_string(cfg->n_classes) +
                                (cfg->precision != CE_F64
                                     ? " in float32 (any F <= 64, K <= 16 runs in float64)"
                                     : " (the float64 MFMA kernel takes F <= 64, K <= 16)"));
        }
    }
    for (int i = 0; i < cfg->n_rows; ++i)
        if (labels[i] < 0 || labels[i] >= cfg->n_classes)
            return fail(CE_EINVAL, "ce_create: label out of range");

    ce_engine *e = new (std::nothrow) ce_engine();
    if (!e) return fail(CE_ENOMEM, "ce_create: host allocation failed");
    e->cfg = *cfg;
    e->kern = kern;
    e->mlp = mlp;
    e->dims = dims;
    if (const char *md = std::getenv("CE_MANY_DIRECT")) e->many_direct = std::atoi(md);
    if (const char *lw = std::getenv("CE_LR_WAVES")) e->lr_waves = std::atoi(lw);
    if (const char *gt = std::getenv("CE_GEN_TAIL")) e->gen_tail = std::atoi(gt);
    if (const char *gc = std::getenv("CE_GEN_CAT")) e->gen_cat = std::atoi(gc);
    if (const char *lm = std::getenv("CE_LR_MODE")) e->lr_mode_cap = std::atoi(lm);
    // experiment switch: launch one phase only, to time each kernel alone
    if (const char *ph = std::getenv("CE_MLP_PHASES")) {
        if (std::strcmp(ph, "train") == 0) e->mlp_phases = 1;
        if (std::strcmp(ph, "info") == 0) e->mlp_phases = 2;
        e->mlp_split = true;
    }
    if (const char *sp = std::getenv("CE_MLP_SPLIT")) e->mlp_split = e->mlp_split || sp[0] == '1';
    if (mlp) {
        const int64_t P = ce::net_params(cfg->n_features, cfg->n_classes,
                                         static_cast<int>(dims.size()) - 2, dims.data() + 1);
        if (P > (int64_t(1) << 30)) {
            delete e;
            return fail(CE_EUNSUPPORTED, "ce_create: network too large (P > 2^30)");
        }
        e->P = static_cast<int>(P);
        e->tsize = sizeof(float);
        e->gsize = sizeof(double);
    } else {
        e->P = cfg->n_features * cfg->n_classes;
        e->tsize = cfg->precision == CE_F64 ? sizeof(double) : sizeof(float);
        e->gsize = e->tsize;
    }
    e->obs_dim = 2 * e->P + 1;
    auto bail = [&](int code) {
        ce_destroy(e);
        return code;
    };
    int rc;
#define CE_TRY(call)                                                   \
    do {                                                               \
        hipError_t err_ = (call);                                      \
        if (err_ != hipSuccess)                                        \
            return bail(fail(CE_EHIP, std::string(#call " failed: ") + \
                                          hipGetErrorString(err_)));   \
    } while (0)
    CE_TRY(hipSetDevice(cfg->device));
    CE_TRY(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking));
    e->stream = e->own_stream;

    const size_t E = cfg->num_envs, N = cfg->n_rows, F = cfg->n_features, P = e->P;
    if (mlp) {
        CE_TRY(hipMalloc(&e->X, N * F * sizeof(float)));
        if (!net_path) CE_TRY(hipMalloc(&e->Xs, N * F * sizeof(float)));
        CE_TRY(hipMalloc(&e->label, N * sizeof(int32_t)));
    } else if (lr_path) {
        e->lr_mfma = true;
        CE_TRY(hipMalloc(&e->X, ce::lr_image_doubles(cfg->n_features, cfg->n_rows) *
                                    sizeof(double)));
    } else if (!kern) {
        e->gen_ft = (cfg->n_features + 15) / 16;
        CE_TRY(hipMalloc(&e->X, static_cast<size_t>(ce::gen_rows_padded_of(cfg->n_rows)) *
                                    ce::gen_stride_of(cfg->n_features) * sizeof(double)));
        if (ce::gen_set_lds_limits() != CE_OK) return bail(CE_EHIP);
    } else {
        CE_TRY(hipMalloc(&e->X, ce::stage_bytes_total(cfg->n_features, cfg->n_rows,
                                                      static_cast<int>(e->tsize))));
    }
    // the network path keeps W / W0 as per-env weight images (net_kernels.h),
    // zero-padded; G stays in the flat parameter order
    size_t wper = P;
    if (net_path) {
        (void)ce::net_geometry(static_cast<int>(dims.size()) - 2, dims.data(), &e->net_geo);
        wper = static_cast<size_t>(e->net_geo.Pimg);
    }
    CE_TRY(hipMalloc(&e->W, E * wper * e->tsize));
    CE_TRY(hipMalloc(&e->G, E * P * e->gsize));
    CE_TRY(hipMalloc(&e->W0, E * wper * e->tsize));
    if (net_path) {
        CE_TRY(hipMemset(e->W, 0, E * wper * e->tsize));
        CE_TRY(hipMemset(e->W0, 0, E * wper * e->tsize));
    }
    CE_TRY(hipMalloc(&e->L, E * sizeof(double)));
    CE_TRY(hipMalloc(&e->step, E * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->d_act, E * P * sizeof(float)));
    CE_TRY(hipHostMalloc(reinterpret_cast<void **>(&e->h_act), E * P * sizeof(float)));
    if (cfg->batch_size < cfg->n_rows) {
        CE_TRY(hipMalloc(&e->perm, E * N * sizeof(int32_t)));
        CE_TRY(hipMalloc(&e->order, 2 * E * N * sizeof(int32_t)));
        CE_TRY(hipMalloc(&e->order_sel, E * sizeof(int32_t)));
        std::vector<int32_t> ident(E * N);
        for (size_t i = 0; i < E; ++i)
            for (size_t r = 0; r < N; ++r) ident[i * N + r] = static_cast<int32_t>(r);
        CE_TRY(hipMemcpy(e->order, ident.data(), E * N * sizeof(int32_t), hipMemcpyHostToDevice));
        CE_TRY(hipMemcpy(e->perm, ident.data(), E * N * sizeof(int32_t), hipMemcpyHostToDevice));
        CE_TRY(hipMemset(e->order_sel, 0, E * sizeof(int32_t)));
    }
    size_t off = 0;
    const size_t sizes[6] = {E * e->obs_dim * sizeof(float), E * sizeof(float), E * sizeof(float),
                             E * sizeof(float), E * sizeof(int32_t), E};
    for (int i = 0; i < 6; ++i) {
        e->off[i] = off;
        off = ce::align16(off + sizes[i]);
    }
    e->out_bytes = off;
    CE_TRY(hipMalloc(&e->d_out, e->out_bytes));
#ifdef CE_DIAG
    CE_TRY(hipMalloc(&e->diag, E * ce::kStamps * sizeof(unsigned long long)));
#endif
    CE_TRY(hipHostMalloc(reinterpret_cast<void **>(&e->h_out), e->out_bytes));
    CE_TRY(hipMemset(e->d_out, 0, e->out_bytes));
    std::memset(e->h_out, 0, e->out_bytes);
    CE_TRY(hipMemset(e->G, 0, E * P * e->gsize));
    CE_TRY(hipMemset(e->L, 0, E * sizeof(double)));
    CE_TRY(hipMemset(e->step, 0, E * sizeof(int32_t)));
    if (mlp) {
        std::vector<float> x32(N * F);
        for (size_t i = 0; i < N * F; ++i) x32[i] = static_cast<float>(features[i]);
        CE_TRY(hipMemcpy(e->X, x32.data(), N * F * sizeof(float), hipMemcpyHostToDevice));
        if (!net_path) {   // the fused kernel's operand-ordered copy
            std::vector<float> xs(N * F);
            const size_t chunks = F / 8;
            for (size_t t = 0; t < N / 32; ++t)
                for (size_t c = 0; c < chunks; ++c)
                    for (size_t l = 0; l < 64; ++l)
                        for (size_t j = 0; j < 4; ++j)
                            xs[((t * chunks + c) * 64 + l) * 4 + j] =
                                x32[(32 * t + (l & 31)) * F + 8 * c + 4 * (l >> 5) + j];
            CE_TRY(hipMemcpy(e->Xs, xs.data(), N * F * sizeof(float), hipMemcpyHostToDevice));
        }
        CE_TRY(hipMemcpy(e->label, labels, N * sizeof(int32_t), hipMemcpyHostToDevice));
        if (net_path) {
            const ce::NetArgs a = make_net_args(e, nullptr, region_view(e, e->d_out));
            if ((rc = ce::net_create(&e->net, a, cfg->device)) != CE_OK) return bail(rc);
            std::string name = "net<";
            for (size_t i = 0; i < dims.size(); ++i) name += (i ? "," : "") + std::to_string(dims[i]);
            // ":mfma": the hand-written MFMA kernels of net_kernels.h; ":wide":
            // a hidden layer wider than 256, the tiled kernels of net_wide.h
            e->kernel_name = name + (e->net_geo.wide ? ">:wide" : ">:mfma");
        }
    }
#undef CE_TRY
    if (e->lr_mfma) {
        std::vector<double> img(ce::lr_image_doubles(cfg->n_features, cfg->n_rows));
        ce::lr_build_image(cfg->n_features, cfg->n_rows, features, labels, img.data());
        if (hipMemcpy(e->X, img.data(), img.size() * sizeof(double), hipMemcpyHostToDevice) !=
            hipSuccess)
            return bail(fail(CE_EHIP, "ce_create: dataset upload failed"));
        e->kernel_name = ce::lr_kernel_name(cfg->num_envs, cfg->n_rows, cfg->n_features,
                                            e->lr_waves, e->lr_mode_cap);
        e->persist = ce::lr_persist_ok(cfg->n_rows);
        if (e->persist) e->many_name = ce::lr_persist_name(cfg->n_rows, cfg->n_features);
        if (const char *pe = std::getenv("CE_PERSIST")) e->persist_on = pe[0] != '0';
    } else if (e->gen_ft) {
        // [Npad][RS] float64: F features, zeros to 16 FT + 1, the label as a
        // double in the last column; rows N..Npad-1 are zeros with label -1
        const int RS = ce::gen_stride_of(cfg->n_features);
        const size_t npad = ce::gen_rows_padded_of(cfg->n_rows);
        std::vector<double> img(npad * RS, 0.0);
        for (size_t r = 0; r < npad; ++r) {
            if (r < N)
                for (size_t f = 0; f < F; ++f) img[r * RS + f] = features[r * F + f];
            img[r * RS + RS - 1] = r < N ? static_cast<double>(labels[r]) : -1.0;
        }
        if (hipMemcpy(e->X, img.data(), img.size() * sizeof(double), hipMemcpyHostToDevice) !=
            hipSuccess)
            return bail(fail(CE_EHIP, "ce_create: dataset upload failed"));
        e->kernel_name = ce::gen_kernel_name(cfg->num_envs, cfg->n_rows, cfg->batch_size,
                                             cfg->n_features, cfg->n_classes, e->gen_cat);
    } else if (!mlp) {
    // [rows | labels]: row-major rows padded to ce::row_stride elements (zeros
    // in the pad), then the int32 labels, in one buffer staged with one copy.
    // Two-class shapes store s_y x with s_y = +1 (y = 0) / -1 (y = 1)
    // (ce::signed_rows, optimize_kernels.h): exact, and it folds the label
    // into the row's dot product.
    const size_t RS = ce::row_stride(cfg->n_features, static_cast<int>(e->tsize));
    const size_t xbytes = ce::align16(N * RS * e->tsize);
    const bool sign_fold = ce::signed_rows(cfg->n_features, cfg->n_classes);
    std::vector<unsigned char> blob(ce::align16(xbytes + 4 * N), 0);
    for (size_t r = 0; r < N; ++r)
        for (size_t f = 0; f < F; ++f) {
            const double v = (sign_fold && labels[r] != 0) ? -features[r * F + f]
                                                           : features[r * F + f];
            if (cfg->precision == CE_F64) {
                std::memcpy(&blob[(r * RS + f) * 8], &v, 8);
            } else {
                const float v32 = static_cast<float>(v);
                std::memcpy(&blob[(r * RS + f) * 4], &v32, 4);
            }
        }
    std::memcpy(&blob[xbytes], labels, 4 * N);
    if (hipMemcpy(e->X, blob.data(), blob.size(), hipMemcpyHostToDevice) != hipSuccess)
        return bail(fail(CE_EHIP, "ce_create: dataset upload failed"));
    e->stage_bytes = ce::stage_bytes_total(cfg->n_features, cfg->n_rows, static_cast<int>(e->tsize));
    e->staged = e->stage_bytes <= ce::kStageLimit;
    if (const char *ns = std::getenv("CE_NO_STAGE"))   // experiment switch: rows from L1/L2
        if (ns[0] == '1') e->staged = false;
    // Two envs per wave where the shape allows it.  U = rows each lane keeps
    // in flight: 2 for float64 (its dependent-issue latency, ~10 cycles,
    // needs the second chain at 2 waves per SIMD), 1 for float32; measured
    // at 4096 envs.  CE_PAIR_U = 0 / 1 / 2 overrides (0 = one
    // env per wave).
    {
        int u = cfg->precision == CE_F64 ? 2 : 1;
        if (const char *pu = std::getenv("CE_PAIR_U")) u = std::atoi(pu);
        if (e->staged && (u == 1 || u == 2)) e->pair = e->kern->step_pair[u - 1];
        const std::string args = std::string(cfg->precision == CE_F64 ? "double" : "float") +
                                 "," + std::to_string(cfg->n_features);
        e->kernel_name = e->pair ? "optimize_pair_kernel<" + args + "," + std::to_string(u) + ">"
                                 : "optimize_step_kernel<" + args + "," +
                                       std::to_string(cfg->n_classes) +
                                       (e->staged ? ",true>" : ",false>");
    }
    }
    // Unseeded envs behave like np_random(None): os.urandom seeds.  The host
    // side normally seeds explicitly; default to seed = env index here.
    std::vector<uint64_t> seeds(E);
    for (size_t i = 0; i < E; ++i) seeds[i] = i;
    if ((rc = ce_seed(e, seeds.data(), static_cast<int32_t>(E))) != CE_OK) return bail(rc);
    if (hipStreamSynchronize(e->stream) != hipSuccess)
        return bail(fail(CE_EHIP, "ce_create: sync failed"));
    *out = e;
    return CE_OK;
}

void ce_destroy(ce_engine *e) {
    if (!e) return;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    e->graphs.release();
    ce::net_destroy(e->net);
    void *dev[] = {e->X, e->Xs, e->label, e->W, e->G, e->W0, e->L, e->step,
                   e->perm, e->order, e->order_sel, e->d_act, e->d_out, e->diag};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (e->h_out) (void)hipHostFree(e->h_out);
    if (e->h_act) (void)hipHostFree(e->h_act);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    delete e;
}

int ce_set_stream(ce_engine *e, void *stream) {
    if (!e) return fail(CE_EINVAL, "null engine");
    e->stream = stream ? static_cast<hipStream_t>(stream) : e->own_stream;
    return CE_OK;
}

int ce_set_compact_outputs(ce_engine *e, int32_t on) {
    if (!e) return fail(CE_EINVAL, "null engine");
    if (on && !e->lr_mfma)
        return fail(CE_EUNSUPPORTED, "ce_set_compact_outputs: only the two-class full-batch "
                                     "float64 kernel (" + std::string("optimize_lr_mfma_kernel") +
                                     ") writes the compact form; this engine runs " + e->kernel_name);
    if (e->compact != (on != 0)) e->graphs.release();   // captured launches carry the form
    e->compact = on != 0;
    return CE_OK;
}

int ce_num_envs(const ce_engine *e) { return e ? e->cfg.num_envs : CE_EINVAL; }
int ce_obs_dim(const ce_engine *e) { return e ? e->obs_dim : CE_EINVAL; }
int ce_act_dim(const ce_engine *e) { return e ? e->P : CE_EINVAL; }

int ce_seed(ce_engine *e, const uint64_t *seeds, int32_t n) {
    if (!e || !seeds) return fail(CE_EINVAL, "ce_seed: null argument");
    if (n != e->cfg.num_envs) return fail(CE_EINVAL, "ce_seed: need one seed per env");
    const size_t E = n, P = e->P, N = e->cfg.n_rows;
    const bool with_perm = e->perm != nullptr;
    if (e->mlp) {
        std::vector<float> w0(E * P);
        std::vector<int32_t> perm(with_perm ? E * N : 0);
        const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
        const size_t nt = std::min<size_t>(hw, E);
        std::vector<std::thread> pool;
        for (size_t t = 0; t < nt; ++t)
            pool.emplace_back([&, t] {
                for (size_t i = t; i < E; i += nt)
                    ce::reset_draws_net(seeds[i], static_cast<int>(e->dims.size()),
                                        e->dims.data(), static_cast<int>(N), &w0[i * P],
                                        with_perm ? &perm[i * N] : nullptr);
            });
        for (auto &th : pool) th.join();
        if (e->net) {   // the weight images (net_kernels.h)
            const size_t PI = static_cast<size_t>(e->net_geo.Pimg);
            std::vector<float> img(E * PI);
            for (size_t i = 0; i < E; ++i) ce::net_flat_to_image(e->net_geo, &w0[i * P], &img[i * PI]);
            CE_HIP(hipMemcpyAsync(e->W0, img.data(), E * PI * sizeof(float), hipMemcpyHostToDevice,
                                  e->stream));
            CE_HIP(hipStreamSynchronize(e->stream));
        } else {
            CE_HIP(hipMemcpyAsync(e->W0, w0.data(), E * P * sizeof(float), hipMemcpyHostToDevice,
                                  e->stream));
        }
        if (with_perm)
            CE_HIP(hipMemcpyAsync(e->perm, perm.data(), E * N * sizeof(int32_t),
                                  hipMemcpyHostToDevice, e->stream));
        CE_HIP(hipStreamSynchronize(e->stream));
        return CE_OK;
    }
    std::vector<double> w0(E * P);
    std::vector<int32_t> perm(with_perm ? E * N : 0);
    for (size_t i = 0; i < E; ++i)
        ce::reset_draws(seeds[i], e->cfg.n_features, e->cfg.n_classes, static_cast<int>(N),
                        &w0[i * P], with_perm ? &perm[i * N] : nullptr);
    int rc = upload_typed(e, e->W0, w0.data(), E * P, e->tsize);
    if (rc != CE_OK) return rc;
    if (with_perm)
        CE_HIP(hipMemcpyAsync(e->perm, perm.data(), E * N * sizeof(int32_t),
                              hipMemcpyHostToDevice, e->stream));
    CE_HIP(hipStreamSynchronize(e->stream));
    return CE_OK;
}

int ce_reset(ce_engine *e, const ce_outputs *out, uint32_t flags) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_CLEAR_STALE_ERROR();
    if (flags & CE_PTR_DEVICE) {
        if (e->compact && !out) return fail(CE_EINVAL, "compact outputs need caller buffers");
        if (out && !complete(out, e->compact)) return fail(CE_EINVAL, "device outputs must all be set");
        ce_outputs o = out ? *out : region_view(e, e->d_out);
        const int rc = launch(e, true, nullptr, o, e->stream, e->compact);
        if (rc != CE_OK) return rc;
        CE_HIP(hipGetLastError());
        e->was_reset = true;
        return CE_OK;
    }
    const int rc = launch(e, true, nullptr, region_view(e, e->d_out), e->stream);
    if (rc != CE_OK) return rc;
    CE_HIP(hipGetLastError());
    CE_HIP(hipMemcpyAsync(e->h_out, e->d_out, e->out_bytes, hipMemcpyDeviceToHost, e->stream));
    CE_HIP(hipStreamSynchronize(e->stream));
    e->was_reset = true;
    if (out && out->obs)
        std::memcpy(out->obs, region_view(e, e->h_out).obs,
                    static_cast<size_t>(e->cfg.num_envs) * e->obs_dim * sizeof(float));
    return CE_OK;
}

int ce_step(ce_engine *e, const float *actions, const ce_outputs *out, uint32_t flags) {
    return do_step(e, actions, out, flags, true);
}

int ce_step_async(ce_engine *e, const float *actions, const ce_outputs *out, uint32_t flags) {
    return do_step(e, actions, out, flags, false);
}

int ce_wait(ce_engine *e) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_HIP(hipStreamSynchronize(e->stream));
    return CE_OK;
}

namespace {

int many_graph(ce_engine *e, int32_t k, const float *actions, int64_t stride,
               const ce_outputs *out, hipGraphExec_t *exec) {
    if (!e) return fail(CE_EINVAL, "null engine");
    if (!e->was_reset) return fail(CE_ESTATE, "step_many() before the first reset()");
    if (k <= 0 || !actions || stride < 0) return fail(CE_EINVAL, "ce_step_many: bad arguments");
    if (e->compact && !out) return fail(CE_EINVAL, "compact outputs need caller buffers");
    if (out && !complete(out, e->compact)) return fail(CE_EINVAL, "device outputs must all be set");
    const ce_outputs o = out ? *out : region_view(e, e->d_out);
    return e->graphs.get(ce::graph_key(k, 0, actions, stride, e->stream, o), [&] {
        (void)launch_steps(e, k, actions, stride, o);
    }, exec);
}

}  // namespace

namespace {

bool aligned16(const void *p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

// the arguments every k-step form checks
int many_args_ok(const ce_engine *e, int32_t k, const float *actions, int64_t stride,
                 const ce_outputs *out) {
    if (!e) return fail(CE_EINVAL, "null engine");
    if (!e->was_reset) return fail(CE_ESTATE, "step_many() before the first reset()");
    if (k <= 0 || !actions || stride < 0) return fail(CE_EINVAL, "ce_step_many: bad arguments");
    if (e->compact && !out) return fail(CE_EINVAL, "compact outputs need caller buffers");
    if (out && !complete(out, e->compact)) return fail(CE_EINVAL, "device outputs must all be set");
    return CE_OK;
}

bool use_persist(const ce_engine *e, const ce_outputs &o) {
    return e->persist && e->persist_on && aligned16(o.obs);
}

// The persistent kernel stores the observation block as 16-B units: a
// caller's misaligned obs is refused, never served by another form while
// ce_step_many_kernel() names the persistent one
int persist_obs_ok(const ce_engine *e, const ce_outputs &o) {
    if (e->persist && e->persist_on && !aligned16(o.obs))
        return fail(CE_EINVAL, "the persistent K-step kernel needs a 16-byte aligned obs "
                               "(ce_set_persistent(e, 0) selects the per-step launches)");
    return CE_OK;
}

}  // namespace

int ce_step_many(ce_engine *e, int32_t k, const float *actions, int64_t stride,
                 const ce_outputs *out) {
    if (e && e->persist && e->persist_on) {
        const int rc = many_args_ok(e, k, actions, stride, out);
        if (rc != CE_OK) return rc;
        const ce_outputs o = out ? *out : region_view(e, e->d_out);
        if (persist_obs_ok(e, o) != CE_OK) return CE_EINVAL;
        if (use_persist(e, o)) {
            CE_CLEAR_STALE_ERROR();
            (void)launch_persist(e, k, actions, stride, o, 0);
            CE_HIP(hipGetLastError());
            return CE_OK;
        }
    }
    if (e && k <= e->many_direct) {
        if (!e->was_reset) return fail(CE_ESTATE, "step_many() before the first reset()");
        if (k <= 0 || !actions || stride < 0) return fail(CE_EINVAL, "ce_step_many: bad arguments");
        if (e->compact && !out) return fail(CE_EINVAL, "compact outputs need caller buffers");
        if (out && !complete(out, e->compact)) return fail(CE_EINVAL, "device outputs must all be set");
        const ce_outputs o = out ? *out : region_view(e, e->d_out);
        CE_CLEAR_STALE_ERROR();
        const int rc = launch_steps(e, k, actions, stride, o);
        if (rc != CE_OK) return rc;
        CE_HIP(hipGetLastError());
        return CE_OK;
    }
    hipGraphExec_t exec;
    const int rc = many_graph(e, k, actions, stride, out, &exec);
    if (rc != CE_OK) return rc;
    CE_HIP(hipGraphLaunch(exec, e->stream));
    return CE_OK;
}

int ce_step_many_prepare(ce_engine *e, int32_t k, const float *actions, int64_t stride,
                         const ce_outputs *out) {
    if (e && e->persist && e->persist_on) {   // one launch: nothing to instantiate
        const int rc = many_args_ok(e, k, actions, stride, out);
        if (rc != CE_OK) return rc;
        const ce_outputs o = out ? *out : region_view(e, e->d_out);
        if (persist_obs_ok(e, o) != CE_OK) return CE_EINVAL;
        if (use_persist(e, o)) return CE_OK;
    }
    hipGraphExec_t exec;
    return many_graph(e, k, actions, stride, out, &exec);
}

int ce_step_many_strided(ce_engine *e, int32_t k, const float *actions, int64_t stride,
                         const ce_outputs *out, int64_t out_step) {
    int rc = many_args_ok(e, k, actions, stride, out);
    if (rc != CE_OK) return rc;
    if (!out) return fail(CE_EINVAL, "ce_step_many_strided: needs caller output buffers");
    if (out_step < 0 || out_step % 16 != 0 || !aligned16(out->obs))
        return fail(CE_EINVAL, "ce_step_many_strided: obs must be 16-byte aligned and "
                               "out_step_bytes a non-negative multiple of 16");
    CE_CLEAR_STALE_ERROR();
    rc = use_persist(e, *out) ? launch_persist(e, k, actions, stride, *out, out_step)
                              : launch_steps(e, k, actions, stride, *out, out_step);
    if (rc != CE_OK) return rc;
    CE_HIP(hipGetLastError());
    return CE_OK;
}

int ce_set_persistent(ce_engine *e, int32_t on) {
    if (!e) return fail(CE_EINVAL, "null engine");
    e->persist_on = on != 0;
    return CE_OK;
}

const char *ce_step_many_kernel(const ce_engine *e) {
    if (!e) return "";
    if (e->persist && e->persist_on) return e->many_name.c_str();
    return ce_step_kernel(e);
}

int64_t ce_stale_error_count(void) { return ce::stale_errors().count.load(); }

const char *ce_stale_error_note(void) {
    static thread_local std::string copy;
    std::lock_guard<std::mutex> lock(ce::stale_errors().mu);
    copy = ce::stale_errors().note;
    return copy.c_str();
}

// Test hook (not part of include/custom_envs_amd.h): record a stale error as
// an entry point would, so the bookkeeping is testable without a GPU.
int ce_test_note_stale_error(int32_t code) {
    ce::note_stale(code, "injected by a test", "ce_test_note_stale_error");
    return CE_OK;
}

const char *ce_step_kernel(const ce_engine *e) {
    if (!e) return "";
    if (e->mlp && !e->net)
        return e->mlp_split ? "mlp_train_kernel+mlp_info_kernel"
                            : "mlp_step_kernel";
    return e->kernel_name.c_str();
}

int ce_host_outputs(ce_engine *e, ce_outputs *view) {
    if (!e || !view) return fail(CE_EINVAL, "null argument");
    *view = region_view(e, e->h_out);
    return CE_OK;
}

#ifdef CE_DIAG
// Diagnostic builds only (not part of include/custom_envs_amd.h).
int ce_diag_stamps(ce_engine *e, unsigned long long *out) {
    if (!e || !out) return fail(CE_EINVAL, "null argument");
    CE_HIP(hipStreamSynchronize(e->stream));
    CE_HIP(hipMemcpy(out, e->diag, sizeof(unsigned long long) * e->cfg.num_envs * ce::kStamps,
                     hipMemcpyDeviceToHost));
    return CE_OK;
}
#endif

int ce_get_state(ce_engine *e, const ce_state *st) {
    if (!e || !st) return fail(CE_EINVAL, "null argument");
    const size_t E = e->cfg.num_envs, P = e->P, N = e->cfg.n_rows;
    int rc;
    CE_HIP(hipStreamSynchronize(e->stream));
    if (e->net) {
        if (st->weights && (rc = net_download(e, st->weights, e->W)) != CE_OK) return rc;
        if (st->init_weights && (rc = net_download(e, st->init_weights, e->W0)) != CE_OK) return rc;
    } else {
        if (st->weights && (rc = download_typed(e, st->weights, e->W, E * P, e->tsize)) != CE_OK) return rc;
        if (st->init_weights && (rc = download_typed(e, st->init_weights, e->W0, E * P, e->tsize)) != CE_OK)
            return rc;
    }
    if (st->grad_hist && (rc = download_typed(e, st->grad_hist, e->G, E * P, e->gsize)) != CE_OK) return rc;
    if (st->loss_hist) CE_HIP(hipMemcpy(st->loss_hist, e->L, E * sizeof(double), hipMemcpyDeviceToHost));
    if (st->step) CE_HIP(hipMemcpy(st->step, e->step, E * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (st->order) {
        if (!e->order) return fail(CE_ESTATE, "row order is only tracked when batch_size < n_rows");
        std::vector<int32_t> sel(E), both(2 * E * N);
        CE_HIP(hipMemcpy(sel.data(), e->order_sel, E * sizeof(int32_t), hipMemcpyDeviceToHost));
        CE_HIP(hipMemcpy(both.data(), e->order, 2 * E * N * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < E; ++i)
            std::memcpy(st->order + i * N, &both[sel[i] * E * N + i * N], N * sizeof(int32_t));
    }
    return CE_OK;
}

int ce_set_state(ce_engine *e, const ce_state *st) {
    if (!e || !st) return fail(CE_EINVAL, "null argument");
    const size_t E = e->cfg.num_envs, P = e->P, N = e->cfg.n_rows;
    int rc;
    CE_HIP(hipStreamSynchronize(e->stream));
    if (e->net) {
        if (st->weights && (rc = net_upload(e, e->W, st->weights)) != CE_OK) return rc;
        if (st->init_weights && (rc = net_upload(e, e->W0, st->init_weights)) != CE_OK) return rc;
    } else {
        if (st->weights && (rc = upload_typed(e, e->W, st->weights, E * P, e->tsize)) != CE_OK) return rc;
        if (st->init_weights && (rc = upload_typed(e, e->W0, st->init_weights, E * P, e->tsize)) != CE_OK)
            return rc;
    }
    if (st->grad_hist && (rc = upload_typed(e, e->G, st->grad_hist, E * P, e->gsize)) != CE_OK) return rc;
    if (st->loss_hist) CE_HIP(hipMemcpy(e->L, st->loss_hist, E * sizeof(double), hipMemcpyHostToDevice));
    if (st->step) CE_HIP(hipMemcpy(e->step, st->step, E * sizeof(int32_t), hipMemcpyHostToDevice));
    if (st->order) {
        if (!e->order) return fail(CE_ESTATE, "row order is only tracked when batch_size < n_rows");
        CE_HIP(hipMemcpy(e->order, st->order, E * N * sizeof(int32_t), hipMemcpyHostToDevice));
        CE_HIP(hipMemset(e->order_sel, 0, E * sizeof(int32_t)));
    }
    CE_HIP(hipStreamSynchronize(e->stream));
    e->was_reset = true;
    return CE_OK;
}

}  // extern "C"
