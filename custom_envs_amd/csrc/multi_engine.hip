// C-ABI implementation of the MultiOptLRs-v0 engine (ce_multi_* in
// include/custom_envs_amd.h).  Same conventions as engine.hip: the engine
// owns the struct-of-arrays state; host mode stages actions/outputs through
// pinned buffers and synchronises; CE_PTR_DEVICE calls are stream-ordered.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "common.h"
#include "multiopt_kernels.h"

namespace {

using ce::fail;

using MultiFn = void (*)(const ce::MultiArgs &, int grid, hipStream_t);

// one lane per (env, agent): E groups of Group<P>::G lanes
template <int P>
int multi_grid(int E) {
    const long lanes = static_cast<long>(E) * ce::Group<P>::G;
    return static_cast<int>((lanes + ce::kMultiBlock - 1) / ce::kMultiBlock);
}
template <int P>
void launch_multi_step(const ce::MultiArgs &a, int, hipStream_t s) {
    // LDS stage of the observation rows: per wave 64/G envs x P rows x 3H
    const size_t lds = a.H <= ce::kMultiStageH
                           ? ce::kMultiBlock / 64 * (64 / ce::Group<P>::G) * P * 3 * a.H * sizeof(float)
                           : 0;
#ifndef CE_MULTI_HC
#define CE_MULTI_HC 1   // A/B switch: 0 runs the any-H kernel for every history length
#endif
    if (CE_MULTI_HC && a.H == 5)   // the reference's default history (multioptlrs.py:39)
        hipLaunchKernelGGL((ce::multi_step_kernel<P, 5>), dim3(multi_grid<P>(a.E)),
                           dim3(ce::kMultiBlock), lds, s, a);
    else
        hipLaunchKernelGGL((ce::multi_step_kernel<P, 0>), dim3(multi_grid<P>(a.E)),
                           dim3(ce::kMultiBlock), lds, s, a);
}
// K steps in one launch (multi_persist_kernel): the reference default history
// H = 5 only (the compile-time instance the kernel needs)
// the split forms: five waves (state, sums, ratio, rows, info; the default),
// four (CE_MULTI_FORM=four: the state wave keeps the raw history), three
// (CE_MULTI_FORM=three: state, rows, info) or one (CE_MULTI_FORM=one), A/B
int multi_form() {
    static const int form = [] {
        const char *v = std::getenv("CE_MULTI_FORM");
        if (v && std::strcmp(v, "one") == 0) return 1;
        if (v && std::strcmp(v, "three") == 0) return 3;
        if (v && std::strcmp(v, "four") == 0) return 4;
        return 5;
    }();
    return form;
}
template <int P>
void launch_multi_persist(const ce::MultiArgs &a, int k, long long act_stride, long long out_step,
                          hipStream_t s) {
    const long lanes = static_cast<long>(a.E) * ce::Group<P>::G;
    const dim3 grid(static_cast<int>((lanes + 63) / 64));
    if (multi_form() == 5) {
        hipLaunchKernelGGL((ce::multi_persist5_kernel<P, 5>), grid, dim3(320), 0, s, a, k, act_stride,
                           out_step);
        return;
    }
    if (multi_form() == 4) {
        hipLaunchKernelGGL((ce::multi_persist4_kernel<P, 5>), grid, dim3(256), 0, s, a, k, act_stride,
                           out_step);
        return;
    }
    if (multi_form() == 3) {
        hipLaunchKernelGGL((ce::multi_persist2_kernel<P, 5>), grid, dim3(192), 0, s, a, k, act_stride,
                           out_step);
        return;
    }
    const size_t lds = ce::kMultiBlock / 64 * (64 / ce::Group<P>::G) * P * 3 * 5 * sizeof(float);
    hipLaunchKernelGGL((ce::multi_persist_kernel<P, 5>), dim3(multi_grid<P>(a.E)), dim3(ce::kMultiBlock),
                       lds, s, a, k, act_stride, out_step);
}
template <int P>
void launch_multi_reset(const ce::MultiArgs &a, int, hipStream_t s) {
    hipLaunchKernelGGL(ce::multi_reset_kernel<P>, dim3(multi_grid<P>(a.E)),
                       dim3(ce::kMultiBlock), 0, s, a);
}

using MultiPersistFn = void (*)(const ce::MultiArgs &, int, long long, long long, hipStream_t);

struct MultiEntry {
    int P;
    MultiFn step, reset;
    MultiPersistFn persist;
};

// every even dimension count up to CE_MULTI_MAX_PARAMS (one lane per agent:
// an env's agents are a group of 2..64 lanes of one wave)
#define CE_MULTI_ENTRY(P) {P, launch_multi_step<P>, launch_multi_reset<P>, launch_multi_persist<P>},
#define CE_MULTI_ENTRY8(P) CE_MULTI_ENTRY(P) CE_MULTI_ENTRY(P + 2) CE_MULTI_ENTRY(P + 4) CE_MULTI_ENTRY(P + 6)
const MultiEntry kMulti[] = {CE_MULTI_ENTRY8(2) CE_MULTI_ENTRY8(10) CE_MULTI_ENTRY8(18)
                                 CE_MULTI_ENTRY8(26) CE_MULTI_ENTRY8(34) CE_MULTI_ENTRY8(42)
                                     CE_MULTI_ENTRY8(50) CE_MULTI_ENTRY8(58)};

}  // namespace

struct ce_multi_engine {
    ce_multi_config cfg{};
    const MultiEntry *kern = nullptr;
    hipStream_t own_stream = nullptr, stream = nullptr;
    int32_t agent_row[ce::kMultiMaxP] = {};   // output row of each agent (sorted names)
    float *theta = nullptr, *grad = nullptr, *hl = nullptr, *hg = nullptr, *hw = nullptr;
    float *ol = nullptr, *og = nullptr, *ow = nullptr;   // adjusted history, observation form
    double *sa = nullptr;                               // its per-entry |.| sums
    int32_t *step = nullptr;
    float *d_act = nullptr, *h_act = nullptr;
    size_t off[5] = {0};
    size_t out_bytes = 0;
    char *d_out = nullptr, *h_out = nullptr;
    bool was_reset = false;
    ce::GraphCache graphs;   // ce_multi_step_many
    // the K-step launch (multi_persist_kernel): max_history == 5, and chosen
    // (ce_multi_set_persistent; CE_PERSIST=0 at create turns it off)
    bool persist = false, persist_on = true;
    std::string many_name, step_name;
};

namespace {

ce_multi_outputs region(const ce_multi_engine *e, char *base) {
    ce_multi_outputs o;
    o.obs = reinterpret_cast<float *>(base + e->off[0]);
    o.reward = reinterpret_cast<float *>(base + e->off[1]);
    o.info = reinterpret_cast<float *>(base + e->off[2]);
    o.episode_len = reinterpret_cast<int32_t *>(base + e->off[3]);
    o.done = reinterpret_cast<uint8_t *>(base + e->off[4]);
    return o;
}

ce::MultiArgs make_args(const ce_multi_engine *e, const float *act, const ce_multi_outputs &o) {
    ce::MultiArgs a;
    a.E = e->cfg.num_envs;
    a.H = e->cfg.max_history;
    a.max_batches = e->cfg.max_batches;
    a.auto_reset = e->cfg.auto_reset;
    for (int i = 0; i < ce::kMultiMaxP; ++i) {
        a.init[i] = i < e->cfg.n_params ? e->cfg.initial_points[i] : 0.0f;
        a.init_g[i] = 0.0f;
        a.agent_row[i] = e->agent_row[i];
    }
    ce::rosenbrock_ref(a.init, e->cfg.n_params, a.init_g, &a.init_l);
    a.theta = e->theta;
    a.grad = e->grad;
    a.hl = e->hl;
    a.hg = e->hg;
    a.hw = e->hw;
    a.ol = e->ol;
    a.og = e->og;
    a.ow = e->ow;
    a.sa = e->sa;
    a.step = e->step;
    a.act = act;
    a.obs = o.obs;
    a.reward = o.reward;
    a.done = o.done;
    a.info = o.info;
    a.episode_len = o.episode_len;
    return a;
}

int grid_of(const ce_multi_engine *e) {
    return (e->cfg.num_envs + ce::kMultiBlock - 1) / ce::kMultiBlock;
}

bool complete(const ce_multi_outputs *o) {
    return o && o->obs && o->reward && o->done && o->info && o->episode_len;
}

void copy_out(const ce_multi_engine *e, const ce_multi_outputs &src, const ce_multi_outputs *dst) {
    if (!dst) return;
    const size_t E = e->cfg.num_envs, P = e->cfg.n_params, H = e->cfg.max_history;
    if (dst->obs) std::memcpy(dst->obs, src.obs, E * P * 3 * H * sizeof(float));
    if (dst->reward) std::memcpy(dst->reward, src.reward, E * P * sizeof(float));
    if (dst->done) std::memcpy(dst->done, src.done, E * P);
    if (dst->info) std::memcpy(dst->info, src.info, E * CE_MULTI_INFO * sizeof(float));
    if (dst->episode_len) std::memcpy(dst->episode_len, src.episode_len, E * sizeof(int32_t));
}

int do_step(ce_multi_engine *e, const float *actions, const ce_multi_outputs *out,
            uint32_t flags, bool sync) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_CLEAR_STALE_ERROR();
    if (!e->was_reset) return fail(CE_ESTATE, "step() before the first reset()");
    if (!actions) return fail(CE_EINVAL, "null actions");
    const size_t rows = static_cast<size_t>(e->cfg.num_envs) * e->cfg.n_params;
    if (flags & CE_PTR_DEVICE) {
        if (out && !complete(out)) return fail(CE_EINVAL, "device outputs must all be set");
        const ce_multi_outputs o = out ? *out : region(e, e->d_out);
        e->kern->step(make_args(e, actions, o), grid_of(e), e->stream);
        CE_HIP(hipGetLastError());
        if (sync) CE_HIP(hipStreamSynchronize(e->stream));
        return CE_OK;
    }
    std::memcpy(e->h_act, actions, rows * sizeof(float));
    CE_HIP(hipMemcpyAsync(e->d_act, e->h_act, rows * sizeof(float), hipMemcpyHostToDevice,
                          e->stream));
    e->kern->step(make_args(e, e->d_act, region(e, e->d_out)), grid_of(e), e->stream);
    CE_HIP(hipGetLastError());
    CE_HIP(hipMemcpyAsync(e->h_out, e->d_out, e->out_bytes, hipMemcpyDeviceToHost, e->stream));
    if (sync) {
        CE_HIP(hipStreamSynchronize(e->stream));
        copy_out(e, region(e, e->h_out), out);
    }
    return CE_OK;
}

}  // namespace

extern "C" {

int ce_multi_create(const ce_multi_config *cfg, ce_multi_engine **out) {
    if (!cfg || !out) return fail(CE_EINVAL, "ce_multi_create: null argument");
    *out = nullptr;
    if (cfg->abi_version != CE_ABI_VERSION)
        return fail(CE_EINVAL, "ce_multi_create: ABI version mismatch");
    if (cfg->function != CE_FUNC_ROSENBROCK_PAIRS)
        return fail(CE_EUNSUPPORTED, "ce_multi_create: unknown function");
    if (cfg->num_envs <= 0 || cfg->max_history <= 0 || cfg->max_batches <= 0)
        return fail(CE_EINVAL, "ce_multi_create: sizes must be positive");
    if (cfg->n_params < 2 || cfg->n_params % 2 || cfg->n_params > CE_MULTI_MAX_PARAMS)
        return fail(CE_EINVAL, "ce_multi_create: n_params must be even, 2..16");
    {   // the step kernel's 32-bit element offsets: every ring plane and the
        // observation block stay below 2^31 elements
        const long long EP = static_cast<long long>(cfg->num_envs) * cfg->n_params;
        const long long planes = std::max(cfg->max_history, 5);
        if (EP * planes >= (1LL << 28) || EP * 3 * cfg->max_history >= (1LL << 28))
            return fail(CE_EUNSUPPORTED, "ce_multi_create: num_envs * n_params * max(max_history, 5) "
                                         "and the observation block must stay below 2^28 elements");
    }
    const MultiEntry *kern = nullptr;
    for (const auto &k : kMulti)
        if (k.P == cfg->n_params) kern = &k;
    if (!kern)
        return fail(CE_EUNSUPPORTED, "ce_multi_create: no kernel for n_params=" +
                                         std::to_string(cfg->n_params));
    ce_multi_engine *e = new (std::nothrow) ce_multi_engine();
    if (!e) return fail(CE_ENOMEM, "ce_multi_create: host allocation failed");
    e->cfg = *cfg;
    e->kern = kern;
    e->persist = cfg->max_history == 5;
    if (const char *pe = std::getenv("CE_PERSIST")) e->persist_on = pe[0] != '0';
    e->step_name = "multi_step_kernel<" + std::to_string(cfg->n_params) + "," +
                   std::to_string(cfg->max_history == 5 ? 5 : 0) + ">";
    e->many_name = std::string(multi_form() == 5   ? "multi_persist5_kernel<"
                               : multi_form() == 4 ? "multi_persist4_kernel<"
                               : multi_form() == 3 ? "multi_persist2_kernel<"
                                                   : "multi_persist_kernel<") +
                   std::to_string(cfg->n_params) + ",5>";
    auto bail = [&](int code) {
        ce_multi_destroy(e);
        return code;
    };
#define CE_TRY(call)                                                           \
    do {                                                                       \
        hipError_t err_ = (call);                                              \
        if (err_ != hipSuccess)                                                \
            return bail(fail(CE_EHIP, std::string(#call " failed: ") +         \
                                          hipGetErrorString(err_)));           \
    } while (0)
    CE_TRY(hipSetDevice(cfg->device));
    CE_TRY(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking));
    e->stream = e->own_stream;
    const size_t E = cfg->num_envs, P = cfg->n_params, H = cfg->max_history;
    CE_TRY(hipMalloc(&e->theta, P * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->grad, P * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->hl, ce::kRawHist * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->hg, ce::kRawHist * P * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->hw, ce::kRawHist * P * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->ol, H * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->og, H * P * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->ow, H * P * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->sa, H * P * E * sizeof(double)));
    CE_TRY(hipMalloc(&e->step, E * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->d_act, E * P * sizeof(float)));
    CE_TRY(hipHostMalloc(reinterpret_cast<void **>(&e->h_act), E * P * sizeof(float)));
    const size_t sizes[5] = {E * P * 3 * H * sizeof(float), E * P * sizeof(float),
                             E * CE_MULTI_INFO * sizeof(float), E * sizeof(int32_t), E * P};
    size_t off = 0;
    for (int i = 0; i < 5; ++i) {
        e->off[i] = off;
        off = ce::align16(off + sizes[i]);
    }
    e->out_bytes = off;
    CE_TRY(hipMalloc(&e->d_out, e->out_bytes));
    CE_TRY(hipHostMalloc(reinterpret_cast<void **>(&e->h_out), e->out_bytes));
    CE_TRY(hipMemset(e->d_out, 0, e->out_bytes));
    std::memset(e->h_out, 0, e->out_bytes);
    // OptEnvRunner rows: agent names sorted as strings (optvecenv.py:10-14,22-23)
    std::vector<std::string> names(P);
    for (size_t i = 0; i < P; ++i) names[i] = "parameter-" + std::to_string(i);
    std::vector<int32_t> order(P);
    for (size_t i = 0; i < P; ++i) order[i] = static_cast<int32_t>(i);
    std::sort(order.begin(), order.end(), [&](int32_t x, int32_t y) { return names[x] < names[y]; });
    for (size_t r = 0; r < P; ++r) e->agent_row[order[r]] = static_cast<int32_t>(r);
#undef CE_TRY
    *out = e;
    return CE_OK;
}

void ce_multi_destroy(ce_multi_engine *e) {
    if (!e) return;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    e->graphs.release();
    void *dev[] = {e->theta, e->grad, e->hl, e->hg, e->hw,
                   e->ol, e->og, e->ow, e->sa, e->step, e->d_act, e->d_out};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (e->h_out) (void)hipHostFree(e->h_out);
    if (e->h_act) (void)hipHostFree(e->h_act);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    delete e;
}

int ce_multi_set_stream(ce_multi_engine *e, void *stream) {
    if (!e) return fail(CE_EINVAL, "null engine");
    e->stream = stream ? static_cast<hipStream_t>(stream) : e->own_stream;
    return CE_OK;
}

int ce_multi_reset(ce_multi_engine *e, const ce_multi_outputs *out, uint32_t flags) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_CLEAR_STALE_ERROR();
    if (flags & CE_PTR_DEVICE) {
        if (out && !complete(out)) return fail(CE_EINVAL, "device outputs must all be set");
        const ce_multi_outputs o = out ? *out : region(e, e->d_out);
        e->kern->reset(make_args(e, nullptr, o), grid_of(e), e->stream);
        CE_HIP(hipGetLastError());
        e->was_reset = true;
        return CE_OK;
    }
    e->kern->reset(make_args(e, nullptr, region(e, e->d_out)), grid_of(e), e->stream);
    CE_HIP(hipGetLastError());
    CE_HIP(hipMemcpyAsync(e->h_out, e->d_out, e->out_bytes, hipMemcpyDeviceToHost, e->stream));
    CE_HIP(hipStreamSynchronize(e->stream));
    e->was_reset = true;
    if (out && out->obs) {
        const size_t n = static_cast<size_t>(e->cfg.num_envs) * e->cfg.n_params * 3 *
                         e->cfg.max_history;
        std::memcpy(out->obs, region(e, e->h_out).obs, n * sizeof(float));
    }
    return CE_OK;
}

int ce_multi_step(ce_multi_engine *e, const float *actions, const ce_multi_outputs *out,
                  uint32_t flags) {
    return do_step(e, actions, out, flags, true);
}

int ce_multi_step_async(ce_multi_engine *e, const float *actions, const ce_multi_outputs *out,
                        uint32_t flags) {
    return do_step(e, actions, out, flags, false);
}

int ce_multi_wait(ce_multi_engine *e) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_HIP(hipStreamSynchronize(e->stream));
    return CE_OK;
}

namespace {

int multi_graph(ce_multi_engine *e, int32_t k, const float *actions, int64_t stride,
                const ce_multi_outputs *out, hipGraphExec_t *exec) {
    if (!e) return fail(CE_EINVAL, "null engine");
    if (!e->was_reset) return fail(CE_ESTATE, "step_many() before the first reset()");
    if (k <= 0 || !actions || stride < 0) return fail(CE_EINVAL, "bad arguments");
    if (out && !complete(out)) return fail(CE_EINVAL, "device outputs must all be set");
    const ce_multi_outputs o = out ? *out : region(e, e->d_out);
    return e->graphs.get(ce::graph_key(k, 0, actions, stride, e->stream, o), [&] {
        for (int s = 0; s < k; ++s)
            e->kern->step(make_args(e, actions + s * stride, o), grid_of(e), e->stream);
    }, exec);
}

}  // namespace

namespace {

int multi_many_ok(const ce_multi_engine *e, int32_t k, const float *actions, int64_t stride,
                  const ce_multi_outputs *out) {
    if (!e) return fail(CE_EINVAL, "null engine");
    if (!e->was_reset) return fail(CE_ESTATE, "step_many() before the first reset()");
    if (k <= 0 || !actions || stride < 0) return fail(CE_EINVAL, "bad arguments");
    if (out && !complete(out)) return fail(CE_EINVAL, "device outputs must all be set");
    return CE_OK;
}

}  // namespace

int ce_multi_step_many(ce_multi_engine *e, int32_t k, const float *actions, int64_t stride,
                       const ce_multi_outputs *out) {
    if (e && e->persist && e->persist_on) {
        const int rc = multi_many_ok(e, k, actions, stride, out);
        if (rc != CE_OK) return rc;
        CE_CLEAR_STALE_ERROR();
        const ce_multi_outputs o = out ? *out : region(e, e->d_out);
        e->kern->persist(make_args(e, actions, o), k, stride, 0, e->stream);
        CE_HIP(hipGetLastError());
        return CE_OK;
    }
    hipGraphExec_t exec;
    const int rc = multi_graph(e, k, actions, stride, out, &exec);
    if (rc != CE_OK) return rc;
    CE_HIP(hipGraphLaunch(exec, e->stream));
    return CE_OK;
}

int ce_multi_step_many_prepare(ce_multi_engine *e, int32_t k, const float *actions,
                               int64_t stride, const ce_multi_outputs *out) {
    if (e && e->persist && e->persist_on) return multi_many_ok(e, k, actions, stride, out);
    hipGraphExec_t exec;
    return multi_graph(e, k, actions, stride, out, &exec);
}

int ce_multi_step_many_strided(ce_multi_engine *e, int32_t k, const float *actions, int64_t stride,
                               const ce_multi_outputs *out, int64_t out_step) {
    int rc = multi_many_ok(e, k, actions, stride, out);
    if (rc != CE_OK) return rc;
    if (!out) return fail(CE_EINVAL, "ce_multi_step_many_strided: needs caller output buffers");
    if (out_step < 0 || out_step % 16 != 0)
        return fail(CE_EINVAL, "ce_multi_step_many_strided: out_step_bytes must be a non-negative "
                               "multiple of 16");
    CE_CLEAR_STALE_ERROR();
    if (e->persist && e->persist_on) {
        e->kern->persist(make_args(e, actions, *out), k, stride, out_step, e->stream);
    } else {
        for (int s = 0; s < k; ++s) {
            ce_multi_outputs o = *out;
            const int64_t b = s * out_step;
            o.obs = reinterpret_cast<float *>(reinterpret_cast<char *>(o.obs) + b);
            o.reward = reinterpret_cast<float *>(reinterpret_cast<char *>(o.reward) + b);
            o.done = o.done + b;
            o.info = reinterpret_cast<float *>(reinterpret_cast<char *>(o.info) + b);
            o.episode_len = reinterpret_cast<int32_t *>(reinterpret_cast<char *>(o.episode_len) + b);
            e->kern->step(make_args(e, actions + s * stride, o), grid_of(e), e->stream);
        }
    }
    CE_HIP(hipGetLastError());
    return CE_OK;
}

int ce_multi_set_persistent(ce_multi_engine *e, int32_t on) {
    if (!e) return fail(CE_EINVAL, "null engine");
    e->persist_on = on != 0;
    return CE_OK;
}

const char *ce_multi_step_many_kernel(const ce_multi_engine *e) {
    if (!e) return "";
    return (e->persist && e->persist_on ? e->many_name : e->step_name).c_str();
}

int ce_multi_host_outputs(ce_multi_engine *e, ce_multi_outputs *view) {
    if (!e || !view) return fail(CE_EINVAL, "null argument");
    *view = region(e, e->h_out);
    return CE_OK;
}

int ce_multi_get_state(ce_multi_engine *e, float *theta, int32_t *step) {
    if (!e) return fail(CE_EINVAL, "null engine");
    const size_t E = e->cfg.num_envs, P = e->cfg.n_params;
    CE_HIP(hipStreamSynchronize(e->stream));
    if (theta) {
        CE_HIP(hipMemcpy(theta, e->theta, P * E * sizeof(float), hipMemcpyDeviceToHost));
    }
    if (step) CE_HIP(hipMemcpy(step, e->step, E * sizeof(int32_t), hipMemcpyDeviceToHost));
    return CE_OK;
}

}  // extern "C"
