// Optimize-v0 over a general OptimizeNN network: the plan (geometry, work
// buffers, the dataset in MFMA operand order) and the step's launch sequence
// (net_kernels.h lists it).  Every dense product is a hand-written MFMA
// kernel; nothing here calls a BLAS library.
#include "net_engine.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.h"
#include "net_kernels.h"
#include "net_wide.h"

namespace ce {

namespace {

template <typename T>
int dev_alloc(T **p, size_t count, bool zero = false) {
    *p = nullptr;
    if (count == 0) return CE_OK;
    CE_HIP(hipMalloc(reinterpret_cast<void **>(p), count * sizeof(T)));
    if (zero) CE_HIP(hipMemset(*p, 0, count * sizeof(T)));
    return CE_OK;
}

int round_up(int v, int m) { return (v + m - 1) / m * m; }

// workgroups per env of the streaming kernels (each loops over its env's rows
// / tasks): enough to fill the chip at a few hundred envs, few enough that
// dispatch is not the bound
constexpr int kNetUpdBlocks = 8;
constexpr int kNetGradBlocks = 8;

}  // namespace

int net_geometry(int n_hidden, const int *dims, NetGeom *g) {
    *g = NetGeom{};
    if (n_hidden < 1 || n_hidden > kNetMaxHidden)
        return fail(CE_EUNSUPPORTED, "network: 1 to 4 hidden layers");
    const int nl = n_hidden + 1;
    g->nl = nl;
    for (int l = 0; l <= nl; ++l)
        if (dims[l] <= 0) return fail(CE_EINVAL, "network: widths must be positive");
    // a hidden layer wider than the MFMA forward's accumulators hold: the
    // wide-layer path (net_wide.h), natural image layout
    for (int l = 1; l < nl; ++l) {
        if (dims[l] > kNetMaxWide)
            return fail(CE_EUNSUPPORTED, "network: hidden widths up to " + std::to_string(kNetMaxWide));
        if (dims[l] > kNetMaxOp) g->wide = 1;
    }
    if (dims[nl] > kNetMaxClasses)
        return fail(CE_EUNSUPPORTED, "network: at most 32 classes");
    if (g->wide) {
        int64_t flat = 0, img = 0;
        int bias = 0;
        for (int l = 0; l < nl; ++l) {
            g->din[l] = dims[l];
            g->dout[l] = dims[l + 1];
            g->op[l] = round_up(dims[l + 1], 64);
            g->nchunk[l] = (dims[l] + kNetChunk - 1) / kNetChunk;
            g->img_off[l] = img;
            g->bias_rel[l] = bias;
            g->flat_w[l] = flat;
            img += static_cast<int64_t>(dims[l]) * g->op[l];
            bias += g->op[l];
            flat += static_cast<int64_t>(dims[l]) * dims[l + 1] + dims[l + 1];
        }
        g->bias_total = bias;
        g->bias_base = img;
        g->Pimg = (img + bias + 63) / 64 * 64;
        g->P = flat;
        return CE_OK;
    }
    // every hidden layer padded to one width (64 or 256 units): the forward
    // is compiled per hidden-layer width (net_fwd_kernel<NCGH>); the output
    // layer (K <= 32) has 64
    int oph = 64;
    for (int l = 1; l < nl; ++l) oph = std::max(oph, round_up(dims[l], 64) > 64 ? kNetMaxOp : 64);
    int64_t flat = 0, img = 0;
    int chunk = 0, row = 0, bias = 0;
    for (int l = 0; l < nl; ++l) {
        g->din[l] = dims[l];
        g->dout[l] = dims[l + 1];
        g->op[l] = l + 1 < nl ? oph : 64;
        g->nchunk[l] = l == 0 ? (dims[0] + kNetChunk - 1) / kNetChunk : g->op[l - 1] / kNetChunk;
        g->chunk0[l] = chunk;
        g->row0[l] = row;
        g->img_off[l] = img;
        g->bias_rel[l] = bias;
        g->flat_w[l] = flat;
        // the forward's chunk sequence: every layer starts on an even chunk
        // (static LDS slot per chunk parity, net_kernels.h); an odd layer-0
        // count gets a padding chunk that is neither loaded nor multiplied
        chunk += (g->nchunk[l] + 1) & ~1;
        row += g->nchunk[l] * kNetChunk;
        img += static_cast<int64_t>(g->nchunk[l]) * kNetChunk * g->op[l];
        bias += g->op[l];
        flat += static_cast<int64_t>(dims[l]) * dims[l + 1] + dims[l + 1];
    }
    g->chunk0[nl] = chunk;
    g->row0[nl] = row;
    g->bias_total = bias;
    g->bias_base = img;
    g->Pimg = (img + bias + 63) / 64 * 64;
    g->P = flat;
    return CE_OK;
}

void net_flat_to_image(const NetGeom &g, const float *flat, float *img) {
    std::memset(img, 0, g.Pimg * sizeof(float));
    for (int l = 0; l < g.nl; ++l) {
        const int din = g.din[l], dout = g.dout[l];
        for (int k = 0; k < din; ++k)
            std::memcpy(img + g.img_off[l] + static_cast<int64_t>(g.wide ? k : net_img_row(l, k)) * g.op[l],
                        flat + g.flat_w[l] + static_cast<int64_t>(k) * dout, dout * sizeof(float));
        const float *b = flat + g.flat_w[l] + static_cast<int64_t>(din) * dout;
        for (int u = 0; u < dout; ++u) img[g.bias_base + g.bias_rel[l] + (g.wide ? u : net_bias_slot(u))] = b[u];
    }
}

void net_image_to_flat(const NetGeom &g, const float *img, float *flat) {
    for (int l = 0; l < g.nl; ++l) {
        const int din = g.din[l], dout = g.dout[l];
        for (int k = 0; k < din; ++k)
            std::memcpy(flat + g.flat_w[l] + static_cast<int64_t>(k) * dout,
                        img + g.img_off[l] + static_cast<int64_t>(g.wide ? k : net_img_row(l, k)) * g.op[l],
                        dout * sizeof(float));
        float *b = flat + g.flat_w[l] + static_cast<int64_t>(din) * dout;
        for (int u = 0; u < dout; ++u) b[u] = img[g.bias_base + g.bias_rel[l] + (g.wide ? u : net_bias_slot(u))];
    }
}

struct NetPlan {
    NetGeom g;
    int E = 0, N = 0, B = 0, T = 0, F16 = 0;
    int Tmb = 0;                             // minibatch tiles (B < N)
    float *Xt = nullptr;                     // [T*64/16][F16][64][4]
    float *Xmb = nullptr;                    // [E][Tmb*64/16][F16][64][4] (B < N)
    int32_t *label_mb = nullptr;             // [E][Tmb*64] (B < N)
    double *part_loss = nullptr;             // [E][T]: info forward
    int32_t *part_hits = nullptr;
    double *mb_loss = nullptr;               // [E][Tmb]: minibatch forward (B < N)
    int32_t *mb_hits = nullptr;
    hipStream_t side = nullptr;              // the gradient chain
    hipEvent_t fork = nullptr, join = nullptr;
    float *act_mb[kNetL] = {nullptr};        // hidden l: [E][B][op_l]
    float *dz_mb[kNetL] = {nullptr};         // hidden l: [E][B][op_l]
    float *dz_out = nullptr;                 // [E][B][op_{nl-1}]
    int task0[kNetL + 1] = {0};
    int ut[kNetL] = {0};
    int tpe = 0;                             // net_grad_kernel tasks per env
    int cus = 256;                           // compute units (the persistent grad grid)
    int upd_blocks = 0;
    float *wide_buf[2] = {nullptr, nullptr}; // wide path, B < N: the info forward's layers [E][N][op_max]
};

int64_t net_params(int F, int K, int n_hidden, const int *hidden) {
    int64_t P = 0;
    int prev = F;
    for (int l = 0; l <= n_hidden; ++l) {
        const int d = l < n_hidden ? hidden[l] : K;
        P += static_cast<int64_t>(prev) * d + d;
        prev = d;
    }
    return P;
}

const NetGeom &net_geom(const NetPlan *p) { return p->g; }

int net_create(NetPlan **out, const NetArgs &a, int device) {
    *out = nullptr;
    int dims[kNetL + 1];
    dims[0] = a.F;
    for (int l = 0; l < a.n_hidden; ++l) dims[l + 1] = a.hidden[l];
    dims[a.n_hidden + 1] = a.K;
    NetGeom geo;
    int rc = net_geometry(a.n_hidden, dims, &geo);
    if (rc != CE_OK) return rc;
    if (geo.P != a.P) return fail(CE_EINVAL, "network: parameter count mismatch");
    if (a.E > 65535) return fail(CE_EUNSUPPORTED, "network: at most 65535 envs per engine");
    NetPlan *p = new (std::nothrow) NetPlan();
    if (!p) return fail(CE_ENOMEM, "network: host allocation failed");
    auto bail = [&](int code) {
        net_destroy(p);
        return code;
    };
    // a HIP failure after the plan exists frees it (CE_HIP would return past it)
#define NET_HIP(call)                                                                     \
    do {                                                                                  \
        const hipError_t err_ = (call);                                                   \
        if (err_ != hipSuccess)                                                           \
            return bail(fail(CE_EHIP, std::string(#call " failed: ") + hipGetErrorString(err_))); \
    } while (0)
    p->g = geo;
    p->E = a.E;
    p->N = a.N;
    p->B = a.B;
    p->T = (a.N + kNetTile - 1) / kNetTile;
    p->F16 = (a.F + 15) / 16;
    const size_t E = a.E, B = a.B, N = a.N;
    if (hipSetDevice(device) != hipSuccess) return bail(fail(CE_EHIP, "network: hipSetDevice"));
    // the dataset in the forward's B-operand order: lane g*16 + n of 16-row
    // block rb, feature group t holds X[16 rb + n][16 t + 4 g .. + 3] (the
    // wide path reads the rows as they are)
    if (!geo.wide) {
        const size_t nrb = static_cast<size_t>(p->T) * (kNetTile / 16);
        std::vector<float> xt(nrb * p->F16 * 64 * 4, 0.0f);
        std::vector<float> xh(N * a.F);
        NET_HIP(hipMemcpy(xh.data(), a.X, xh.size() * sizeof(float), hipMemcpyDeviceToHost));
        for (size_t rb = 0; rb < nrb; ++rb)
            for (int t = 0; t < p->F16; ++t)
                for (int ln = 0; ln < 64; ++ln)
                    for (int q = 0; q < 4; ++q) {
                        const size_t r = rb * 16 + (ln & 15);
                        const int f = 16 * t + 4 * (ln >> 4) + q;
                        if (r < N && f < a.F)
                            xt[((rb * p->F16 + t) * 64 + ln) * 4 + q] = xh[r * a.F + f];
                    }
        if ((rc = dev_alloc(&p->Xt, xt.size())) != CE_OK) return bail(rc);
        NET_HIP(hipMemcpy(p->Xt, xt.data(), xt.size() * sizeof(float), hipMemcpyHostToDevice));
    }
    if (B < N) {
        p->Tmb = (a.B + kNetTile - 1) / kNetTile;
        const size_t rows = static_cast<size_t>(p->Tmb) * kNetTile;
        if (!geo.wide) {     // the MFMA forward's gathered minibatch operands
            if ((rc = dev_alloc(&p->Xmb, E * rows * p->F16 * 16, true)) != CE_OK) return bail(rc);
            if ((rc = dev_alloc(&p->label_mb, E * rows, true)) != CE_OK) return bail(rc);
        } else {             // the wide path's info forward, layer by layer (ping-pong)
            int opm = 64;
            for (int l = 0; l < geo.nl; ++l) opm = std::max(opm, geo.op[l]);
            for (int i = 0; i < 2; ++i)
                if ((rc = dev_alloc(&p->wide_buf[i], E * N * opm, true)) != CE_OK) return bail(rc);
        }
        if ((rc = dev_alloc(&p->mb_loss, E * p->Tmb, true)) != CE_OK) return bail(rc);
        if ((rc = dev_alloc(&p->mb_hits, E * p->Tmb, true)) != CE_OK) return bail(rc);
    }
    if ((rc = dev_alloc(&p->part_loss, E * p->T, true)) != CE_OK) return bail(rc);
    if ((rc = dev_alloc(&p->part_hits, E * p->T, true)) != CE_OK) return bail(rc);
    // (stream priorities were measured: a greatest-priority stream for the
    // forward changed nothing; the persistent grad grid is what keeps the
    // forward's slots)
    if (hipDeviceGetAttribute(&p->cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess)
        return bail(fail(CE_EHIP, "network: device attribute"));
    if (hipStreamCreateWithFlags(&p->side, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&p->fork, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&p->join, hipEventDisableTiming) != hipSuccess)
        return bail(fail(CE_EHIP, "network: side stream / events"));
    const int nl = geo.nl;
    for (int l = 0; l + 1 < nl; ++l) {
        if ((rc = dev_alloc(&p->act_mb[l], E * B * geo.op[l], true)) != CE_OK) return bail(rc);
        if ((rc = dev_alloc(&p->dz_mb[l], E * B * geo.op[l], true)) != CE_OK) return bail(rc);
    }
    // padded classes stay zero: the backward kernels read them as K steps
    if ((rc = dev_alloc(&p->dz_out, E * B * geo.op[nl - 1], true)) != CE_OK) return bail(rc);
    int task = 0;
    for (int l = 0; l < nl; ++l) {
        p->task0[l] = task;
        p->ut[l] = (geo.dout[l] + kNetGradTile - 1) / kNetGradTile;
        task += (geo.din[l] + 1 + 31) / 32 * p->ut[l];
    }
    p->task0[nl] = task;
    p->tpe = task;
    // a few long-lived workgroups per env: one per 16 rows made 85k tiny
    // workgroups at 1024 envs, dispatch-bound (0.99 ms for 3.3 GB)
    const int rows = geo.row0[nl] + (geo.bias_total + 255) / 256;
    p->upd_blocks = std::max(1, std::min(kNetUpdBlocks, (rows + 15) / 16));
    NET_HIP(hipDeviceSynchronize());
#undef NET_HIP
    *out = p;
    return CE_OK;
}

void net_destroy(NetPlan *p) {
    if (!p) return;
    void *bufs[] = {p->Xt, p->Xmb, p->label_mb, p->part_loss, p->part_hits, p->mb_loss, p->mb_hits, p->dz_out};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    if (p->fork) (void)hipEventDestroy(p->fork);
    if (p->join) (void)hipEventDestroy(p->join);
    if (p->side) (void)hipStreamDestroy(p->side);
    for (int l = 0; l < kNetL; ++l) {
        if (p->act_mb[l]) (void)hipFree(p->act_mb[l]);
        if (p->dz_mb[l]) (void)hipFree(p->dz_mb[l]);
    }
    for (float *b : p->wide_buf)
        if (b) (void)hipFree(b);
    delete p;
}

namespace {

NetFinArgs fin_args(const NetPlan *p, const NetArgs &a) {
    NetFinArgs f{};
    f.E = a.E;
    f.N = a.N;
    f.B = a.B;
    f.P = a.P;
    f.T = p->T;
    f.max_steps = a.max_steps;
    f.auto_reset = a.auto_reset;
    f.Pimg = p->g.Pimg;
    f.part_loss = p->part_loss;
    f.part_hits = p->part_hits;
    // B == N: the info forward is the minibatch forward
    f.Tmb = p->Tmb ? p->Tmb : p->T;
    f.mb_loss = p->Tmb ? p->mb_loss : p->part_loss;
    f.mb_hits = p->Tmb ? p->mb_hits : p->part_hits;
    f.img = a.W;
    f.img0 = a.W0;
    f.L = a.L;
    f.step = a.step;
    f.perm = a.perm;
    f.order = a.order;
    f.order_sel = a.order_sel;
    f.obs = a.obs;
    f.reward = a.reward;
    f.done = a.done;
    f.objective = a.objective;
    f.accuracy = a.accuracy;
    f.episode_len = a.episode_len;
    return f;
}

NetGradArgs grad_args(const NetPlan *p, const NetArgs &a) {
    NetGradArgs r{};
    r.g = p->g;
    r.E = a.E;
    r.N = a.N;
    r.B = a.B;
    r.P = a.P;
    r.F = a.F;
    r.max_steps = a.max_steps;
    r.auto_reset = a.auto_reset;
    r.tpe = p->tpe;
    for (int l = 0; l <= kNetL; ++l) r.task0[l] = p->task0[std::min(l, p->g.nl)];
    for (int l = 0; l < kNetL; ++l) {
        r.ut[l] = p->ut[l];
        r.act_mb[l] = p->act_mb[l];
        r.dz_mb[l] = p->dz_mb[l];
    }
    r.X = a.X;
    r.order = a.B < a.N ? a.order : nullptr;
    r.order_sel = a.order_sel;
    r.dz_out = p->dz_out;
    r.step = a.step;
    r.G = a.G;
    r.obs = a.obs;
    return r;
}

int op_max(const NetGeom &g) {
    int m = 64;
    for (int l = 0; l < g.nl; ++l) m = std::max(m, g.op[l]);
    return m;
}

// The wide-layer path (net_wide.h): every launch on the caller's stream.
int net_step_wide(NetPlan *p, const NetArgs &a, hipStream_t s) {
    const NetGeom &g = p->g;
    const int E = a.E, nl = g.nl, B = a.B;
    const bool split = p->Tmb > 0;                          // B < N: a separate info forward
    const int64_t Bs = B;
    {
        WideUpdArgs u{};
        u.g = g;
        u.E = E;
        u.P = a.P;
        u.img = a.W;
        u.act = a.act;
        u.step = a.step;
        const unsigned bx = static_cast<unsigned>(std::min<int64_t>(256, (a.P + 255) / 256));
        hipLaunchKernelGGL(net_wide_update_kernel, dim3(bx, E), dim3(256), 0, s, u);
    }
    auto gemm = [&](const WideGemmArgs &ga) {
        const dim3 grid((ga.N + kWideTile - 1) / kWideTile, (ga.M + kWideTile - 1) / kWideTile, E);
        hipLaunchKernelGGL(net_wide_gemm_kernel, grid, dim3(256), 0, s, ga);
    };
    // H_l = relu(H_{l-1} W'_l + b'_l) (the output layer: the logits)
    auto layer_fwd = [&](int l, int R, const float *in, int64_t in_env, int ldin, bool gather, float *out,
                         int64_t out_env) {
        WideGemmArgs ga{};
        ga.E = E;
        ga.M = R;
        ga.N = g.dout[l];
        ga.K = g.din[l];
        ga.A = in;
        ga.a_env = in_env;
        ga.lda = ldin;
        if (gather) {
            ga.order = a.order;
            ga.order_sel = a.order_sel;
            ga.n_rows = a.N;
        }
        ga.B = a.W + g.img_off[l];
        ga.b_env = g.Pimg;
        ga.ldb = g.op[l];
        ga.bias = a.W + g.bias_base + g.bias_rel[l];
        ga.bias_env = g.Pimg;
        ga.relu = l + 1 < nl;
        ga.C = out;
        ga.c_env = out_env;
        ga.ldc = g.op[l];
        gemm(ga);
    };
    auto loss = [&](int R, int T, float *Z, int64_t z_env, bool gather, bool dz, double *pl, int32_t *ph) {
        WideLossArgs la{};
        la.E = E;
        la.R = R;
        la.K = g.dout[nl - 1];
        la.T = T;
        la.write_dz = dz ? 1 : 0;
        la.Z = Z;
        la.z_env = z_env;
        la.ldz = g.op[nl - 1];
        la.label = a.label;
        if (gather) {
            la.order = a.order;
            la.order_sel = a.order_sel;
            la.n_rows = a.N;
        }
        la.part_loss = pl;
        la.part_hits = ph;
        hipLaunchKernelGGL(net_wide_loss_kernel, dim3(T, E), dim3(64), 0, s, la);
    };
    // the minibatch forward over sequence[0] (B < N: through the env's row
    // order; B == N: every row in order, which is also the info forward)
    for (int l = 0; l < nl; ++l) {
        float *out = l + 1 == nl ? p->dz_out : p->act_mb[l];
        if (l == 0) layer_fwd(0, B, a.X, 0, a.F, split, out, Bs * g.op[0]);
        else layer_fwd(l, B, p->act_mb[l - 1], Bs * g.op[l - 1], g.op[l - 1], false, out, Bs * g.op[l]);
    }
    loss(B, split ? p->Tmb : p->T, p->dz_out, Bs * g.op[nl - 1], split, true, split ? p->mb_loss : p->part_loss,
         split ? p->mb_hits : p->part_hits);
    if (split) {   // info['objective'] / ['accuracy'] over every dataset row at W'
        const int64_t ne = static_cast<int64_t>(a.N) * op_max(g);
        const float *in = a.X;
        int64_t in_env = 0;
        int ldin = a.F;
        for (int l = 0; l < nl; ++l) {
            float *out = p->wide_buf[l & 1];
            layer_fwd(l, a.N, in, in_env, ldin, false, out, ne);
            in = out;
            in_env = ne;
            ldin = g.op[l];
        }
        loss(a.N, p->T, p->wide_buf[(nl - 1) & 1], ne, false, false, p->part_loss, p->part_hits);
    }
    // dZ_l = (dZ_{l+1} W'_{l+1}^T) * (H_l > 0), top down
    for (int lh = nl - 2; lh >= 0; --lh) {
        const int lo = lh + 1;
        WideGemmArgs ga{};
        ga.E = E;
        ga.M = B;
        ga.N = g.dout[lh];
        ga.K = g.dout[lo];
        ga.A = lo == nl - 1 ? p->dz_out : p->dz_mb[lo];
        ga.a_env = Bs * g.op[lo];
        ga.lda = g.op[lo];
        ga.B = a.W + g.img_off[lo];
        ga.b_env = g.Pimg;
        ga.ldb = g.op[lo];
        ga.b_trans = 1;
        ga.mask = p->act_mb[lh];
        ga.mask_env = Bs * g.op[lh];
        ga.ldm = g.op[lh];
        ga.C = p->dz_mb[lh];
        ga.c_env = Bs * g.op[lh];
        ga.ldc = g.op[lh];
        gemm(ga);
    }
    const int grid = 8 * std::min(p->tpe, kNetGradBlocks) * ((E + 7) / 8);
    hipLaunchKernelGGL(net_grad_kernel, dim3((grid + 7) / 8 * 8), dim3(kNetThreads), 0, s, grad_args(p, a));
    hipLaunchKernelGGL(net_finish_kernel, dim3(E), dim3(kNetThreads), 0, s, fin_args(p, a));
    CE_HIP(hipGetLastError());
    return CE_OK;
}

}  // namespace

int net_step(NetPlan *p, const NetArgs &a, hipStream_t s) {
    const NetGeom &g = p->g;
    if (g.wide) return net_step_wide(p, a, s);
    const int E = a.E, nl = g.nl;
    const bool split = p->Tmb > 0;                          // B < N: a separate minibatch forward
    // B <= 32 (the minibatch in waves 0-1): the update rides in the minibatch
    // forward's producer waves (net_producer) -- one kernel instead of the
    // update, the gather and the minibatch forward
#ifndef CE_NET_FUSED
#define CE_NET_FUSED 1
#endif
    const bool fused = CE_NET_FUSED && split && a.B <= 2 * kNetWaveRows;
    if (!fused) {
        NetUpdArgs u{};
        u.g = g;
        u.E = E;
        u.P = a.P;
        u.img = a.W;
        u.act = a.act;
        u.step = a.step;
        hipLaunchKernelGGL(net_update_kernel, dim3(p->upd_blocks, E), dim3(kNetThreads), 0, s, u);
    }
    auto forward = [&](bool mb, hipStream_t st) {
        NetFwdArgs f{};
        f.g = g;
        f.E = E;
        f.F16 = p->F16;
        f.img = a.W;
        if (mb && split) {
            f.rows = a.B;
            f.T = p->Tmb;
            f.Xt = p->Xmb;
            f.xt_env = static_cast<int64_t>(p->Tmb) * kNetTile * p->F16 * 16;
            f.label = p->label_mb;
            f.label_env = static_cast<int64_t>(p->Tmb) * kNetTile;
            f.part_loss = p->mb_loss;
            f.part_hits = p->mb_hits;
        } else {
            f.rows = a.N;
            f.T = p->T;
            f.Xt = p->Xt;
            f.label = a.label;
            f.part_loss = p->part_loss;
            f.part_hits = p->part_hits;
        }
        f.mb = mb ? 1 : 0;
        for (int l = 0; l < kNetL; ++l) f.act_mb[l] = p->act_mb[l];
        f.dz_out = p->dz_out;
        const bool fu = mb && fused;
        if (fu) {
            f.label = a.label;                              // indexed by the dataset row
            f.N = a.N;
            f.F = a.F;
            f.P = a.P;
            f.X = a.X;
            f.act = a.act;
            f.step = a.step;
            f.order = a.order;
            f.order_sel = a.order_sel;
        }
        const unsigned grid = static_cast<unsigned>((E + 7) / 8 * 8) * f.T;
        const bool narrow = g.dout[nl - 1] <= 16;
        constexpr int W4 = kNetMaxOp / 64;
#define CE_NET_FWD(NCGH, NARROW, FU) \
    hipLaunchKernelGGL((net_fwd_kernel<NCGH, NARROW, FU>), dim3(grid), dim3(kNetThreads), 0, st, f)
        if (g.op[0] == kNetMaxOp) {
            if (narrow) {
                if (fu) CE_NET_FWD(W4, true, true);
                else CE_NET_FWD(W4, true, false);
            } else {
                if (fu) CE_NET_FWD(W4, false, true);
                else CE_NET_FWD(W4, false, false);
            }
        } else if (narrow) {
            if (fu) CE_NET_FWD(1, true, true);
            else CE_NET_FWD(1, true, false);
        } else {
            if (fu) CE_NET_FWD(1, false, true);
            else CE_NET_FWD(1, false, false);
        }
#undef CE_NET_FWD
    };
    if (split && !fused) {
        NetGatherArgs ga{};
        ga.E = E;
        ga.N = a.N;
        ga.B = a.B;
        ga.F = a.F;
        ga.F16 = p->F16;
        ga.Tmb = p->Tmb;
        ga.X = a.X;
        ga.label = a.label;
        ga.order = a.order;
        ga.order_sel = a.order_sel;
        ga.Xmb = p->Xmb;
        ga.label_mb = p->label_mb;
        hipLaunchKernelGGL(net_gather_kernel, dim3(p->Tmb * (kNetTile / 16), E), dim3(kNetThreads), 0, s, ga);
    }
    // the minibatch forward (B == N: the info forward too), then the fork:
    // the info forward on this stream, the gradient chain on the side stream
    forward(true, s);
    hipStream_t gs = s;
    if (split) {
        CE_HIP(hipEventRecord(p->fork, s));
        CE_HIP(hipStreamWaitEvent(p->side, p->fork, 0));
        forward(false, s);                                  // first: it takes its 2 workgroups per CU
        gs = p->side;
    }
    for (int lh = nl - 2; lh >= 0; --lh) {
        NetBwdArgs b{};
        b.g = g;
        b.E = E;
        b.B = a.B;
        b.lh = lh;
        b.img = a.W;
        b.dz_next = lh + 1 == nl - 1 ? p->dz_out : p->dz_mb[lh + 1];
        b.act = p->act_mb[lh];
        b.dz = p->dz_mb[lh];
        hipLaunchKernelGGL(net_bwd_kernel, dim3(E), dim3(kNetThreads), 0, gs, b);
    }
    {
        const NetGradArgs r = grad_args(p, a);
        // beside the forward: a fixed grid of ~0.62 workgroups per CU (one per
        // CU is what fits beside the forward's two; fewer spreads the same
        // traffic over the forward's whole run -- A/B in DESIGN 3.7); alone:
        // 8 per env
#ifndef CE_NET_GRAD_PCT
#define CE_NET_GRAD_PCT 62
#endif
        const int grid = split ? std::max(8, CE_NET_GRAD_PCT * p->cus / 100)
                               : 8 * std::min(p->tpe, kNetGradBlocks) * ((E + 7) / 8);
        hipLaunchKernelGGL(net_grad_kernel, dim3((grid + 7) / 8 * 8), dim3(kNetThreads), 0, gs, r);
    }
    if (split) {
        CE_HIP(hipEventRecord(p->join, p->side));
        CE_HIP(hipStreamWaitEvent(s, p->join, 0));
    }
    hipLaunchKernelGGL(net_finish_kernel, dim3(E), dim3(kNetThreads), 0, s, fin_args(p, a));
    CE_HIP(hipGetLastError());
    return CE_OK;
}

int net_reset(NetPlan *p, const NetArgs &a, hipStream_t s) {
    NetResetArgs r{};
    r.E = a.E;
    r.P = a.P;
    r.Pimg = p->g.Pimg;
    r.img = a.W;
    r.img0 = a.W0;
    r.G = a.G;
    r.obs = a.obs;
    const size_t per = std::max<size_t>(2 * static_cast<size_t>(a.P) + 1, p->g.Pimg / 4);
    const unsigned bx = static_cast<unsigned>(std::min<size_t>(1024, (per + kNetThreads - 1) / kNetThreads));
    hipLaunchKernelGGL(net_reset_params_kernel, dim3(bx, a.E), dim3(kNetThreads), 0, s, r);
    hipLaunchKernelGGL(net_reset_env_kernel, dim3(a.E), dim3(kNetThreads), 0, s, fin_args(p, a));
    CE_HIP(hipGetLastError());
    return CE_OK;
}


}  // namespace ce
