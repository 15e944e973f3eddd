// C-ABI implementation of MultiOptLRs-v0 over the OptimizeNN problem (ce_nn_*
// in include/custom_envs_amd.h).  Same conventions as multi_engine.hip: the
// engine owns the struct-of-arrays state; host mode stages actions/outputs
// through pinned buffers and synchronises; CE_PTR_DEVICE calls are
// stream-ordered.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "multinn_kernels.h"
#include "seeding.h"

struct ce_nn_engine {
    ce_nn_config cfg{};
    ce::NnArgs base{};                 // shapes, offsets and state pointers
    int P = 0;
    size_t Ps = 0;
    hipStream_t own_stream = nullptr, stream = nullptr;
    float *X = nullptr;
    int32_t *label = nullptr;
    float *theta_buf[2] = {nullptr, nullptr}, *g_buf[2] = {nullptr, nullptr};
    int parity = 0;                    // theta_buf[parity], g_buf[parity] are current
    float *theta0 = nullptr, *gU = nullptr, *loss_b = nullptr;
    float *rw = nullptr, *rg = nullptr, *hl = nullptr;
    double *al = nullptr, *sw = nullptr, *sg = nullptr, *hsg = nullptr;
    double *part_u = nullptr, *part_c = nullptr;
    int32_t *step = nullptr, *cursor = nullptr, *order = nullptr, *order_sel = nullptr;
    int32_t *reset_perm = nullptr, *epoch_perm = nullptr, *agent_row = nullptr;
    int32_t *row_agent = nullptr;
    float *d_act = nullptr, *h_act = nullptr;
    size_t off[5] = {0};
    size_t out_bytes = 0;
    char *d_out = nullptr, *h_out = nullptr;
    unsigned long long *diag = nullptr;    // CE_DIAG builds: [2][E][kNnStamps]
    bool seeded = false, was_reset = false;
    ce::GraphCache graphs;   // ce_nn_step_many
};

namespace {

using ce::fail;

int host_ld(int w) { return ((w + 31) & ~31) + ce::kNnPad; }

ce_multi_outputs region(const ce_nn_engine *e, char *base) {
    ce_multi_outputs o;
    o.obs = reinterpret_cast<float *>(base + e->off[0]);
    o.reward = reinterpret_cast<float *>(base + e->off[1]);
    o.info = reinterpret_cast<float *>(base + e->off[2]);
    o.episode_len = reinterpret_cast<int32_t *>(base + e->off[3]);
    o.done = reinterpret_cast<uint8_t *>(base + e->off[4]);
    return o;
}

ce::NnArgs make_args(const ce_nn_engine *e, const float *act, const ce_multi_outputs &o) {
    ce::NnArgs a = e->base;
    a.theta = e->theta_buf[e->parity];
    a.theta_n = e->theta_buf[1 - e->parity];
    a.gprev = e->g_buf[e->parity];
    a.gN = e->g_buf[1 - e->parity];
    a.act = act;
    a.obs = o.obs;
    a.reward = o.reward;
    a.done = o.done;
    a.info = o.info;
    a.episode_len = o.episode_len;
    return a;
}

bool complete(const ce_multi_outputs *o) {
    return o && o->obs && o->reward && o->done && o->info && o->episode_len;
}

// one step's five launches; the ping-pong pairs swap afterwards
void launch_step(ce_nn_engine *e, const float *act, const ce_multi_outputs &o, hipStream_t s) {
    const ce::NnArgs a = make_args(e, act, o);
    const size_t stage = (static_cast<size_t>(ce::kNnRows) * 3 * a.H + 4) * sizeof(float);
    hipLaunchKernelGGL(ce::nn_grad_kernel, dim3(a.E), dim3(ce::kNnBlock), a.lds_bytes, s, a);
    hipLaunchKernelGGL(ce::nn_update_kernel, dim3(a.nchunk_u, a.E), dim3(ce::kNnChunk), 0, s, a);
    hipLaunchKernelGGL(ce::nn_step_kernel, dim3(a.E), dim3(ce::kNnBlock), a.lds_bytes, s, a);
    hipLaunchKernelGGL(ce::nn_agent_rows_kernel, dim3(a.nchunk, a.E), dim3(ce::kNnRows), stage, s, a);
    hipLaunchKernelGGL(ce::nn_finalize_kernel, dim3(a.E), dim3(ce::kNnChunk), 0, s, a);
    e->parity ^= 1;
}

void copy_out(const ce_nn_engine *e, const ce_multi_outputs &src, const ce_multi_outputs *dst) {
    if (!dst) return;
    const size_t E = e->cfg.num_envs, P = e->P, H = e->cfg.max_history;
    if (dst->obs) std::memcpy(dst->obs, src.obs, E * P * 3 * H * sizeof(float));
    if (dst->reward) std::memcpy(dst->reward, src.reward, E * P * sizeof(float));
    if (dst->done) std::memcpy(dst->done, src.done, E * P);
    if (dst->info) std::memcpy(dst->info, src.info, E * CE_MULTI_INFO * sizeof(float));
    if (dst->episode_len) std::memcpy(dst->episode_len, src.episode_len, E * sizeof(int32_t));
}

int do_step(ce_nn_engine *e, const float *actions, const ce_multi_outputs *out, uint32_t flags,
            bool sync) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_CLEAR_STALE_ERROR();
    if (!e->was_reset) return fail(CE_ESTATE, "step() before the first reset()");
    if (!actions) return fail(CE_EINVAL, "null actions");
    const size_t rows = static_cast<size_t>(e->cfg.num_envs) * e->P;
    if (flags & CE_PTR_DEVICE) {
        if (out && !complete(out)) return fail(CE_EINVAL, "device outputs must all be set");
        const ce_multi_outputs o = out ? *out : region(e, e->d_out);
        launch_step(e, actions, o, e->stream);
        CE_HIP(hipGetLastError());
        if (sync) CE_HIP(hipStreamSynchronize(e->stream));
        return CE_OK;
    }
    std::memcpy(e->h_act, actions, rows * sizeof(float));
    CE_HIP(hipMemcpyAsync(e->d_act, e->h_act, rows * sizeof(float), hipMemcpyHostToDevice,
                          e->stream));
    launch_step(e, e->d_act, region(e, e->d_out), e->stream);
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

int ce_nn_create(const ce_nn_config *cfg, const float *features, const int32_t *labels,
                 ce_nn_engine **out) {
    if (!cfg || !out || !features || !labels) return fail(CE_EINVAL, "ce_nn_create: null argument");
    *out = nullptr;
    if (cfg->abi_version != CE_ABI_VERSION) return fail(CE_EINVAL, "ce_nn_create: ABI version mismatch");
    const int L = cfg->n_hidden;
    if (cfg->num_envs <= 0 || cfg->n_rows <= 0 || cfg->n_features <= 0 || cfg->max_batches <= 0)
        return fail(CE_EINVAL, "ce_nn_create: sizes must be positive");
    if (L < 1 || L > CE_NN_MAX_HIDDEN)
        return fail(CE_EUNSUPPORTED, "ce_nn_create: 1..4 hidden layers");
    for (int l = 0; l < L; ++l)
        if (cfg->hidden[l] <= 0 || cfg->hidden[l] % 32 || cfg->hidden[l] > ce::kNnMaxWidth)
            return fail(CE_EUNSUPPORTED, "ce_nn_create: hidden widths must be multiples of 32, <= 512");
    if (cfg->n_classes < 2 || cfg->n_classes > ce::kNnMaxK)
        return fail(CE_EUNSUPPORTED, "ce_nn_create: 2..32 classes");
    if (cfg->batch_size <= 0 || cfg->batch_size > ce::kNnBatch)
        return fail(CE_EUNSUPPORTED, "ce_nn_create: batch_size must be 1..32");
    if (cfg->num_envs > 65535) return fail(CE_EUNSUPPORTED, "ce_nn_create: at most 65535 envs");
    if (cfg->max_history <= 0 || cfg->max_history > ce::kNnMaxH)
        return fail(CE_EUNSUPPORTED, "ce_nn_create: max_history must be 1..16");
    if (cfg->n_features > 1024) return fail(CE_EUNSUPPORTED, "ce_nn_create: n_features <= 1024");
    for (int i = 0; i < cfg->n_rows; ++i)
        if (labels[i] < 0 || labels[i] >= cfg->n_classes)
            return fail(CE_EINVAL, "ce_nn_create: label out of range");

    ce_nn_engine *e = new (std::nothrow) ce_nn_engine();
    if (!e) return fail(CE_ENOMEM, "ce_nn_create: host allocation failed");
    e->cfg = *cfg;
    auto bail = [&](int code) {
        ce_nn_destroy(e);
        return code;
    };
#define CE_TRY(call)                                                                   \
    do {                                                                               \
        hipError_t err_ = (call);                                                      \
        if (err_ != hipSuccess)                                                        \
            return bail(fail(CE_EHIP, std::string(#call " failed: ") + hipGetErrorString(err_))); \
    } while (0)

    ce::NnArgs &a = e->base;
    a.E = cfg->num_envs;
    a.N = cfg->n_rows;
    a.F = cfg->n_features;
    a.K = cfg->n_classes;
    a.L = L;
    a.B = cfg->batch_size;
    a.nb = (a.N + a.B - 1) / a.B;
    a.H = cfg->max_history;
    a.max_batches = cfg->max_batches;
    a.auto_reset = cfg->auto_reset;
    a.dims[0] = a.F;
    for (int l = 0; l < L; ++l) a.dims[l + 1] = cfg->hidden[l];
    a.dims[L + 1] = a.K;
    long P = 0;
    for (int l = 0; l <= L; ++l) {
        a.off_w[l] = static_cast<int>(P);
        P += static_cast<long>(a.dims[l]) * a.dims[l + 1];
        a.off_b[l] = static_cast<int>(P);
        P += a.dims[l + 1];
    }
    e->P = a.P = static_cast<int>(P);
    e->Ps = static_cast<size_t>((P + 63) & ~63L);
    a.Ps = static_cast<int>(e->Ps);
    a.nchunk = static_cast<int>((P + ce::kNnRows - 1) / ce::kNnRows);
    a.nchunk_u = static_cast<int>((P + ce::kNnChunk * ce::kNnUpdPer - 1) /
                                  (ce::kNnChunk * ce::kNnUpdPer));
    // LDS: X, every hidden activation, the logits, the split-k scratch
    int fl = 0;
    a.lds_x = fl;
    fl += ce::kNnBatch * host_ld(a.F);
    a.split = 0;
    for (int l = 0; l < L; ++l) {
        a.lds_h[l] = fl;
        fl += ce::kNnBatch * host_ld(a.dims[l + 1]);
        if (a.dims[l + 1] / 32 < ce::kNnWaves) a.split = 1;
    }
    a.lds_z = fl;
    fl += ce::kNnBatch * host_ld(a.K);
    a.lds_wo = fl;
    fl += (a.dims[L] * a.K + 3) & ~3;
    a.lds_part = fl;
    if (a.split) fl += ce::kNnWaves * 32 * 32;
    a.lds_bytes = fl * static_cast<int>(sizeof(float));
    if (a.lds_bytes > 150 * 1024)
        return bail(fail(CE_EUNSUPPORTED, "ce_nn_create: network too wide for LDS (" +
                                              std::to_string(a.lds_bytes) + " bytes)"));

    CE_TRY(hipSetDevice(cfg->device));
    CE_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(ce::nn_grad_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, a.lds_bytes));
    CE_TRY(hipFuncSetAttribute(reinterpret_cast<const void *>(ce::nn_step_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, a.lds_bytes));
    CE_TRY(hipStreamCreateWithFlags(&e->own_stream, hipStreamNonBlocking));
    e->stream = e->own_stream;
    const size_t E = a.E, N = a.N, Ps = e->Ps, H = a.H;
    CE_TRY(hipMalloc(&e->X, N * a.F * sizeof(float)));
    CE_TRY(hipMalloc(&e->label, N * sizeof(int32_t)));
    CE_TRY(hipMemcpy(e->X, features, N * a.F * sizeof(float), hipMemcpyHostToDevice));
    CE_TRY(hipMemcpy(e->label, labels, N * sizeof(int32_t), hipMemcpyHostToDevice));
    for (int i = 0; i < 2; ++i) {
        CE_TRY(hipMalloc(&e->theta_buf[i], E * Ps * sizeof(float)));
        CE_TRY(hipMalloc(&e->g_buf[i], E * Ps * sizeof(float)));
        CE_TRY(hipMemset(e->theta_buf[i], 0, E * Ps * sizeof(float)));
        CE_TRY(hipMemset(e->g_buf[i], 0, E * Ps * sizeof(float)));
    }
    CE_TRY(hipMalloc(&e->theta0, E * Ps * sizeof(float)));
    CE_TRY(hipMalloc(&e->gU, E * Ps * sizeof(float)));
    CE_TRY(hipMalloc(&e->loss_b, E * sizeof(float)));
    CE_TRY(hipMalloc(&e->part_u, E * a.nchunk_u * 3 * sizeof(double)));
    CE_TRY(hipMalloc(&e->part_c, E * a.nchunk * 5 * sizeof(double)));
    CE_TRY(hipMalloc(&e->rw, H * E * Ps * sizeof(float)));
    CE_TRY(hipMalloc(&e->rg, H * E * Ps * sizeof(float)));
    CE_TRY(hipMalloc(&e->al, H * E * sizeof(double)));
    CE_TRY(hipMalloc(&e->sw, H * E * sizeof(double)));
    CE_TRY(hipMalloc(&e->sg, H * E * sizeof(double)));
    CE_TRY(hipMalloc(&e->hl, ce::kRawHist * E * sizeof(float)));
    CE_TRY(hipMalloc(&e->hsg, ce::kRawHist * E * sizeof(double)));
    CE_TRY(hipMalloc(&e->step, E * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->cursor, E * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->order, 2 * E * N * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->order_sel, E * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->reset_perm, E * N * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->epoch_perm, E * N * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->agent_row, P * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->row_agent, P * sizeof(int32_t)));
    CE_TRY(hipMalloc(&e->d_act, E * P * sizeof(float)));
    CE_TRY(hipHostMalloc(reinterpret_cast<void **>(&e->h_act), E * P * sizeof(float)));
    CE_TRY(hipMemset(e->step, 0, E * sizeof(int32_t)));
    CE_TRY(hipMemset(e->cursor, 0, E * sizeof(int32_t)));
    CE_TRY(hipMemset(e->order_sel, 0, E * sizeof(int32_t)));
    {
        // the dataset object starts in file order (the construction-time
        // shuffle draws from the unseeded global npr, optimize_nn.py:64,
        // and is not reproducible in the reference)
        std::vector<int32_t> ident(E * N);
        for (size_t i = 0; i < E * N; ++i) ident[i] = static_cast<int32_t>(i % N);
        CE_TRY(hipMemcpy(e->order, ident.data(), E * N * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    {
        // OptEnvRunner rows: agent names sorted as strings (optvecenv.py:10-14,22-23)
        std::vector<std::string> names(P);
        for (long i = 0; i < P; ++i) names[i] = "parameter-" + std::to_string(i);
        std::vector<int32_t> order(P), row(P);
        for (long i = 0; i < P; ++i) order[i] = static_cast<int32_t>(i);
        std::sort(order.begin(), order.end(),
                  [&](int32_t x, int32_t y) { return names[x] < names[y]; });
        for (long r = 0; r < P; ++r) row[order[r]] = static_cast<int32_t>(r);
        CE_TRY(hipMemcpy(e->agent_row, row.data(), P * sizeof(int32_t), hipMemcpyHostToDevice));
        CE_TRY(hipMemcpy(e->row_agent, order.data(), P * sizeof(int32_t), hipMemcpyHostToDevice));
    }
    const size_t sizes[5] = {E * P * 3 * H * sizeof(float), E * P * sizeof(float),
                             E * CE_MULTI_INFO * sizeof(float), E * sizeof(int32_t),
                             E * static_cast<size_t>(P)};
    size_t off = 0;
    for (int i = 0; i < 5; ++i) {
        e->off[i] = off;
        off = ce::align16(off + sizes[i]);
    }
    e->out_bytes = off;
    CE_TRY(hipMalloc(&e->d_out, e->out_bytes));
#ifdef CE_DIAG
    CE_TRY(hipMalloc(&e->diag, 2 * E * ce::kNnStamps * sizeof(unsigned long long)));
    a.diag = e->diag;
#endif
    CE_TRY(hipHostMalloc(reinterpret_cast<void **>(&e->h_out), e->out_bytes));
    CE_TRY(hipMemset(e->d_out, 0, e->out_bytes));
    std::memset(e->h_out, 0, e->out_bytes);
#undef CE_TRY
    a.X = e->X;
    a.label = e->label;
    a.theta0 = e->theta0;
    a.gU = e->gU;
    a.loss_b = e->loss_b;
    a.part_u = e->part_u;
    a.part_c = e->part_c;
    a.rw = e->rw;
    a.rg = e->rg;
    a.al = e->al;
    a.sw = e->sw;
    a.sg = e->sg;
    a.hl = e->hl;
    a.hsg = e->hsg;
    a.step = e->step;
    a.cursor = e->cursor;
    a.order = e->order;
    a.order_sel = e->order_sel;
    a.reset_perm = e->reset_perm;
    a.epoch_perm = e->epoch_perm;
    a.agent_row = e->agent_row;
    a.row_agent = e->row_agent;
    *out = e;
    return CE_OK;
}

void ce_nn_destroy(ce_nn_engine *e) {
    if (!e) return;
    if (e->stream) (void)hipStreamSynchronize(e->stream);
    e->graphs.release();
    void *dev[] = {e->X, e->label, e->theta_buf[0], e->theta_buf[1], e->g_buf[0], e->g_buf[1],
                   e->theta0, e->gU, e->loss_b, e->part_u, e->part_c, e->rw, e->rg,
                   e->al, e->sw, e->sg, e->hl, e->hsg, e->step, e->cursor,
                   e->order, e->order_sel, e->reset_perm, e->epoch_perm, e->agent_row, e->row_agent,
                   e->d_act, e->d_out, e->diag};
    for (void *p : dev)
        if (p) (void)hipFree(p);
    if (e->h_out) (void)hipHostFree(e->h_out);
    if (e->h_act) (void)hipHostFree(e->h_act);
    if (e->own_stream) (void)hipStreamDestroy(e->own_stream);
    delete e;
}

int ce_nn_set_stream(ce_nn_engine *e, void *stream) {
    if (!e) return fail(CE_EINVAL, "null engine");
    e->stream = stream ? static_cast<hipStream_t>(stream) : e->own_stream;
    return CE_OK;
}

int ce_nn_n_params(const ce_nn_engine *e) { return e ? e->P : fail(CE_EINVAL, "null engine"); }

int ce_nn_seed_draws(uint64_t seed, int32_t n_dims, const int32_t *dims, int32_t n_rows,
                     float *init_weights, int32_t *reset_perm, int32_t *epoch_perm) {
    if (n_dims < 2 || !dims || n_rows <= 0) return fail(CE_EINVAL, "ce_nn_seed_draws: bad arguments");
    std::vector<int> d(dims, dims + n_dims);
    ce::reset_draws_nn(seed, n_dims, d.data(), n_rows, init_weights, reset_perm, epoch_perm);
    return CE_OK;
}

int ce_nn_seed(ce_nn_engine *e, const uint64_t *seeds, int32_t n) {
    if (!e || !seeds) return fail(CE_EINVAL, "null argument");
    const ce::NnArgs &a = e->base;
    if (n != a.E) return fail(CE_EINVAL, "ce_nn_seed: one seed per env");
    const size_t E = a.E, N = a.N, Ps = e->Ps;
    std::vector<float> th(E * Ps, 0.0f);
    std::vector<int32_t> rp(E * N), ep(E * N);
    const int n_dims = a.L + 2;
    const unsigned workers = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    std::vector<std::thread> pool;
    for (unsigned w = 0; w < workers; ++w) {
        pool.emplace_back([&, w]() {
            for (size_t i = w; i < E; i += workers)
                ce::reset_draws_nn(seeds[i], n_dims, a.dims, a.N, th.data() + i * Ps,
                                   rp.data() + i * N, ep.data() + i * N);
        });
    }
    for (auto &t : pool) t.join();
    // stream-ordered after any step still reading theta0 / the permutations
    // (the engine stream is non-blocking, so null-stream copies would race)
    CE_HIP(hipStreamSynchronize(e->stream));
    CE_HIP(hipMemcpyAsync(e->theta0, th.data(), E * Ps * sizeof(float), hipMemcpyHostToDevice,
                          e->stream));
    CE_HIP(hipMemcpyAsync(e->reset_perm, rp.data(), E * N * sizeof(int32_t),
                          hipMemcpyHostToDevice, e->stream));
    CE_HIP(hipMemcpyAsync(e->epoch_perm, ep.data(), E * N * sizeof(int32_t),
                          hipMemcpyHostToDevice, e->stream));
    CE_HIP(hipStreamSynchronize(e->stream));
    e->seeded = true;
    return CE_OK;
}

int ce_nn_reset(ce_nn_engine *e, const ce_multi_outputs *out, uint32_t flags) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_CLEAR_STALE_ERROR();
    if (!e->seeded) return fail(CE_ESTATE, "reset() before seed()");
    const size_t n = static_cast<size_t>(e->cfg.num_envs) * e->P * 3 * e->cfg.max_history;
    if (flags & CE_PTR_DEVICE) {
        if (out && !complete(out)) return fail(CE_EINVAL, "device outputs must all be set");
        const ce_multi_outputs o = out ? *out : region(e, e->d_out);
        const ce::NnArgs a = make_args(e, nullptr, o);
        hipLaunchKernelGGL(ce::nn_reset_kernel, dim3(a.E), dim3(ce::kNnBlock), 0, e->stream, a);
        CE_HIP(hipGetLastError());
        e->was_reset = true;
        return CE_OK;
    }
    const ce::NnArgs a = make_args(e, nullptr, region(e, e->d_out));
    hipLaunchKernelGGL(ce::nn_reset_kernel, dim3(a.E), dim3(ce::kNnBlock), 0, e->stream, a);
    CE_HIP(hipGetLastError());
    CE_HIP(hipMemcpyAsync(e->h_out, e->d_out, e->out_bytes, hipMemcpyDeviceToHost, e->stream));
    CE_HIP(hipStreamSynchronize(e->stream));
    e->was_reset = true;
    if (out && out->obs) std::memcpy(out->obs, region(e, e->h_out).obs, n * sizeof(float));
    return CE_OK;
}

int ce_nn_step(ce_nn_engine *e, const float *actions, const ce_multi_outputs *out, uint32_t flags) {
    return do_step(e, actions, out, flags, true);
}

int ce_nn_step_async(ce_nn_engine *e, const float *actions, const ce_multi_outputs *out,
                     uint32_t flags) {
    return do_step(e, actions, out, flags, false);
}

int ce_nn_wait(ce_nn_engine *e) {
    if (!e) return fail(CE_EINVAL, "null engine");
    CE_HIP(hipStreamSynchronize(e->stream));
    return CE_OK;
}

namespace {

int nn_graph(ce_nn_engine *e, int32_t k, const float *actions, int64_t stride,
             const ce_multi_outputs *out, hipGraphExec_t *exec) {
    if (!e) return fail(CE_EINVAL, "null engine");
    if (!e->was_reset) return fail(CE_ESTATE, "step_many() before the first reset()");
    if (k <= 0 || !actions || stride < 0) return fail(CE_EINVAL, "bad arguments");
    if (out && !complete(out)) return fail(CE_EINVAL, "device outputs must all be set");
    const ce_multi_outputs o = out ? *out : region(e, e->d_out);
    // the captured launches bake in the ping-pong pointers of their parity
    const int p0 = e->parity;
    const int rc = e->graphs.get(ce::graph_key(k, p0, actions, stride, e->stream, o), [&] {
        for (int s = 0; s < k; ++s) launch_step(e, actions + s * stride, o, e->stream);
    }, exec);
    e->parity = p0;
    return rc;
}

}  // namespace

int ce_nn_step_many(ce_nn_engine *e, int32_t k, const float *actions, int64_t stride,
                    const ce_multi_outputs *out) {
    hipGraphExec_t exec;
    const int rc = nn_graph(e, k, actions, stride, out, &exec);
    if (rc != CE_OK) return rc;
    CE_HIP(hipGraphLaunch(exec, e->stream));
    e->parity ^= (k & 1);
    return CE_OK;
}

int ce_nn_step_many_prepare(ce_nn_engine *e, int32_t k, const float *actions, int64_t stride,
                            const ce_multi_outputs *out) {
    hipGraphExec_t exec;
    return nn_graph(e, k, actions, stride, out, &exec);
}

int ce_nn_host_outputs(ce_nn_engine *e, ce_multi_outputs *view) {
    if (!e || !view) return fail(CE_EINVAL, "null argument");
    *view = region(e, e->h_out);
    return CE_OK;
}

#ifdef CE_DIAG
// Diagnostic builds only (not part of include/custom_envs_amd.h): the eval
// kernels' phase stamps, [2 kernels][E][kNnStamps].
int ce_nn_diag_stamps(ce_nn_engine *e, unsigned long long *out) {
    if (!e || !out) return fail(CE_EINVAL, "null argument");
    CE_HIP(hipStreamSynchronize(e->stream));
    CE_HIP(hipMemcpy(out, e->diag,
                     2 * sizeof(unsigned long long) * e->cfg.num_envs * ce::kNnStamps,
                     hipMemcpyDeviceToHost));
    return CE_OK;
}
#endif

int ce_nn_get_state(ce_nn_engine *e, float *theta, float *gprev, int32_t *step, int32_t *cursor,
                    int32_t *order) {
    if (!e) return fail(CE_EINVAL, "null engine");
    const size_t E = e->cfg.num_envs, P = e->P, Ps = e->Ps, N = e->cfg.n_rows;
    CE_HIP(hipStreamSynchronize(e->stream));
    if (theta)
        CE_HIP(hipMemcpy2D(theta, P * sizeof(float), e->theta_buf[e->parity], Ps * sizeof(float),
                           P * sizeof(float),
                           E, hipMemcpyDeviceToHost));
    if (gprev)
        CE_HIP(hipMemcpy2D(gprev, P * sizeof(float), e->g_buf[e->parity], Ps * sizeof(float),
                           P * sizeof(float),
                           E, hipMemcpyDeviceToHost));
    if (step) CE_HIP(hipMemcpy(step, e->step, E * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (cursor) CE_HIP(hipMemcpy(cursor, e->cursor, E * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (order) {
        std::vector<int32_t> sel(E), all(2 * E * N);
        CE_HIP(hipMemcpy(sel.data(), e->order_sel, E * sizeof(int32_t), hipMemcpyDeviceToHost));
        CE_HIP(hipMemcpy(all.data(), e->order, 2 * E * N * sizeof(int32_t), hipMemcpyDeviceToHost));
        for (size_t i = 0; i < E; ++i)
            std::memcpy(order + i * N, all.data() + (sel[i] * E + i) * N, N * sizeof(int32_t));
    }
    return CE_OK;
}

}  // extern "C"
