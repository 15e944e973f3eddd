// Optimize-v0 over the config-3 MLP problem for gfx950.
//
// One VecEnv.step of E envs is ONE launch, mlp_step_kernel: a 256-thread
// workgroup per env runs the two phases of the step back to back,
//   train phase:
//     Optimize.base_step        custom_envs/envs/optimize.py:69-93
//       W <- W - a              (:74-75), fused into the forward's operand loads
//       minibatch forward/backward of the F -> 64 (relu) -> K softmax MLP
//       (problems/optimize_nn.py:35-52; gradient = d(sum_i CE_i)/dtheta), the
//       flat parameter order [W1 | b1 | W2 | b2] (utils_common.py:199-207)
//       g / B, L' = (loss - L)/(L + 0.1), G' = g/(|G| + 1)   (:78-83)
//       obs = [0 (P) | L' | G' (P)], reward = -loss, done = step >= 40
//   info phase:
//       info objective/accuracy over the full dataset     (optimize.py:94-97)
//       auto-reset of finished envs (utils_venv.py:31): W <- W0, histories 0,
//       row order composed with the reset permutation (inmemorydataset
//       on_epoch_end under use_random_state, optimize.py:58-67)
// The train phase streams the env's state (36 bytes per parameter, HBM-bound),
// the info phase is a 1024 x 784 x 64 GEMM per env (MFMA-bound).  The kernel
// is held to 256 registers so two workgroups share a CU: their phases drift
// apart, and one env's streaming hides under another env's matrix work
// (DESIGN.md 3.7).  The split pair mlp_train_kernel + mlp_info_kernel (same
// bodies, the info pass with twice the accumulators at one wave per SIMD)
// stays for A/B timing (CE_MLP_SPLIT=1).
//
// Matrix work runs on the f32-input MFMA v_mfma_f32_32x32x2_f32 (exact f32
// products, k-ordered fma chain): lane l supplies A[i = l&31][k = l>>5] and
// B[k = l>>5][j = l&31]; the 32x32 result has column j = l&31 on the lane and
// rows (r&3) + 8(r>>2) + 4(l>>5) in accumulator register r.  Hidden units are
// interleaved over the two 32-wide hidden accumulators (accumulator ht holds
// units 2i + ht), so the W1 operand of a lane is one float2 of a 256-B W1 row
// and each dW1 / grad-history element pair is one 16-B access:
//   * forward: H^T (hidden x samples) = W1^T . X_b^T.  A chunk of 8 k's is
//     one float4 of a sample row per lane half (k = 8c + 4h + jj);
//   * logits^T (classes x samples) = W2^T . H^T takes the H^T accumulator
//     as its B operand register by register (no LDS round trip);
//   * dW1 (features x hidden) = X_b^T . dz1, K = 32 samples, one tile per
//     32x32 output block, G' and obs written from the accumulator.
// Shapes: hidden = 64, minibatch B = 32, F % 8 == 0, K <= 16, N % 64 == 0.
// With P odd (odd K) an env's parameter block may start at an odd float: that
// shape runs an instance with its pair accesses split into scalars.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "optimize_kernels.h"   // CE_STAMP, kStamps

namespace ce {

constexpr int kMlpHidden = 64;
constexpr int kMlpBatch = 32;
constexpr int kMlpMaxK = 16;
constexpr int kMlpBlock = 256;    // 4 waves
constexpr int kSplitInfoTiles = 8; // split info kernel: 16 accumulators, 1 wave per SIMD
constexpr int kStepInfoTiles = 4;  // fused kernel: 8 accumulators, 2 workgroups per CU
#ifndef CE_MLP_TRAIN_DEPTH
#define CE_MLP_TRAIN_DEPTH 4
#endif
#ifndef CE_MLP_INFO_DEPTH
#define CE_MLP_INFO_DEPTH 1
#endif
constexpr int kTrainDepth = CE_MLP_TRAIN_DEPTH;    // forward chunks in flight per wave
constexpr int kStepInfoDepth = CE_MLP_INFO_DEPTH;  // fused kernel: info-pass chunks in flight
constexpr int kSplitInfoDepth = 1; // split info kernel (its 16 accumulators leave no room)

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct MlpArgs {
    int E, N, F, K, P, max_steps, auto_reset;
    const float *X;          // [N][F] dataset rows (dataset order)
    const float *Xs;         // the same rows in MFMA operand order:
                             // [N/32 tiles][F/8 chunks][64 lanes][4], element j of
                             // lane l = X[32 t + (l & 31)][8 c + 4 (l >> 5) + j]
    const int32_t *label;    // [N]
    float *W;                // [E][P]
    const float *W0;         // [E][P]
    double *G;               // [E][P] grad_hist[idx] (float64, np.zeros)
    double *L;               // [E]
    int32_t *step;           // [E]
    const int32_t *perm;     // [E][N] reset permutation
    int32_t *order;          // [2][E][N] current row order (ping-pong)
    int32_t *order_sel;      // [E]
    const float *act;        // [E][P]
    float *obs;              // [E][2P+1]
    float *reward;
    uint8_t *done;
    float *objective;
    float *accuracy;
    int32_t *episode_len;
    unsigned long long *diag;   // [E][kStamps] (CE_DIAG builds only)
};

// Diagnostic builds stamp wave 0's phase boundaries (optimize_kernels.h
// CE_STAMP): 0 train entry, 1 forward done, 2 small gradients done, 3 train
// done, 4 info entry, 5 info passes done, 6 info end; the train phase writes
// slots 0-3, the info phase 4-6.
struct MlpStamps {
    unsigned long long stamps[8];
};

// LDS of the two phases of one env's step.
// W2 rows are kMlpW2S = 17 floats apart: the dz1 = dz2 W2^T loop reads
// w2s[j][k] with j across the lanes, and the 16-float stride put a 32-lane
// group on 2 banks (16-way conflicts: 41.1 M conflict cycles per 4096-env
// dispatch, profiles/r03_mlp_pmc.json "train")
constexpr int kMlpW2S = kMlpMaxK + 1;
struct MlpTrainShared {
    float part[4][kMlpHidden][kMlpBatch];     // per-wave partial H^T
    float hs[kMlpBatch][kMlpHidden + 1];      // H, then dz1 (sample-major)
    float w2s[kMlpHidden][kMlpW2S];
    float b1s[kMlpHidden], b2s[kMlpMaxK];
    float dz2[kMlpBatch][kMlpMaxK];
    float ce[kMlpBatch];
    int rows[kMlpBatch];
};
struct MlpInfoShared {
    float w2s[kMlpHidden][kMlpW2S];
    float b1s[kMlpHidden], b2s[kMlpMaxK];
    float red_loss[4];
    int red_hits[4];
};

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// row of accumulator register r for lane half h (32x32 C/D map)
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// pair accesses: one 8-B / 16-B access when the env's block is pair-aligned
template <bool A> __device__ __forceinline__ float2 ld_f2(const float *p) {
    if constexpr (A) return *reinterpret_cast<const float2 *>(p);
    else return make_float2(p[0], p[1]);
}
template <bool A> __device__ __forceinline__ void st_f2(float *p, float2 v) {
    if constexpr (A) *reinterpret_cast<float2 *>(p) = v;
    else { p[0] = v.x; p[1] = v.y; }
}
template <bool A> __device__ __forceinline__ double2 ld_d2(const double *p) {
    if constexpr (A) return *reinterpret_cast<const double2 *>(p);
    else return make_double2(p[0], p[1]);
}
template <bool A> __device__ __forceinline__ void st_d2(double *p, double2 v) {
    if constexpr (A) *reinterpret_cast<double2 *>(p) = v;
    else { p[0] = v.x; p[1] = v.y; }
}

// Streams touched once per step (actions, grad history, obs) go through
// these helpers; CE_MLP_NT experiment builds give them the nontemporal
// policy (measured: no gain, the train phase 8% slower), product builds the
// default policy.
#ifndef CE_MLP_NT
#define __builtin_nontemporal_load(p) (*(p))
#define __builtin_nontemporal_store(v, p) (*(p) = (v))
#endif
typedef float nt_f2 __attribute__((ext_vector_type(2)));
typedef float nt_f4 __attribute__((ext_vector_type(4)));
typedef double nt_d2 __attribute__((ext_vector_type(2)));
template <bool A> __device__ __forceinline__ float2 ld_f2_nt(const float *p) {
    if constexpr (A) {
        const nt_f2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_f2 *>(p));
        return make_float2(v.x, v.y);
    } else {
        return make_float2(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1));
    }
}
template <bool A> __device__ __forceinline__ double2 ld_d2_nt(const double *p) {
    if constexpr (A) {
        const nt_d2 v = __builtin_nontemporal_load(reinterpret_cast<const nt_d2 *>(p));
        return make_double2(v.x, v.y);
    } else {
        return make_double2(__builtin_nontemporal_load(p), __builtin_nontemporal_load(p + 1));
    }
}
template <bool A> __device__ __forceinline__ void st_d2_nt(double *p, double2 v) {
    if constexpr (A) {
        nt_d2 w = {v.x, v.y};
        __builtin_nontemporal_store(w, reinterpret_cast<nt_d2 *>(p));
    } else {
        __builtin_nontemporal_store(v.x, p);
        __builtin_nontemporal_store(v.y, p + 1);
    }
}
__device__ __forceinline__ void st_nt(float *p, float v) { __builtin_nontemporal_store(v, p); }

// LDS byte address of a pointer into __shared__ memory
__device__ __forceinline__ unsigned lds_addr(const void *p) {
    return static_cast<unsigned>(reinterpret_cast<uintptr_t>(
        (const __attribute__((address_space(3))) char *)(p)));
}

// block-wide p[0:n] = 0 with 16-B stores between a scalar head and tail
__device__ __forceinline__ void zero_floats(float *p, int n, int tid, int nthreads) {
    int head = static_cast<int>(((16 - (reinterpret_cast<uintptr_t>(p) & 15)) & 15) / 4);
    head = head < n ? head : n;
    if (tid < head) st_nt(p + tid, 0.0f);
    nt_f4 *q = reinterpret_cast<nt_f4 *>(p + head);
    const int n4 = (n - head) / 4;
    const nt_f4 z = {0.0f, 0.0f, 0.0f, 0.0f};
    for (int i = tid; i < n4; i += nthreads) __builtin_nontemporal_store(z, q + i);
    const int tail = head + 4 * n4;
    if (tid < n - tail) st_nt(p + tail + tid, 0.0f);
}

// A D-deep software pipeline over nunits * D consecutive chunks from c0: the
// ring slot of chunk c + D is refilled as soon as chunk c's registers are
// consumed.  Slot indices are static and the loop has no branches, so the
// compiler's memory-counter waits stay exact (a runtime-indexed or shifted
// ring, or a guarded load, makes it wait for every outstanding access).
// load(stage, c, part) loads part 0, 1 or both (-1) of a stage;
// use(stage, c, refill) calls refill(part) once that part's registers are
// dead (a part still read after its refill would cost a register copy and a
// wait at the loop's back edge).  Scheduling barriers keep each slot's
// accesses in program order, and the first unit is peeled, so the loop is
// entered in the same counter state its back edge carries.
template <int D, typename Stage, typename Load, typename Use>
__device__ __forceinline__ void pipelined(int c0, int nunits, Load &&load, Use &&use) {
    if (nunits <= 0) return;
    Stage ring[D];
#pragma unroll
    for (int s = 0; s < D; ++s) {
        load(ring[s], c0 + s, -1);
        __builtin_amdgcn_sched_barrier(0);
    }
    int c = c0;
    auto unit = [&] {
#pragma unroll
        for (int s = 0; s < D; ++s) {
            use(ring[s], c + s, [&](int part) { load(ring[s], c + s + D, part); });
            __builtin_amdgcn_sched_barrier(0);
        }
        c += D;
    };
    if (nunits > 1) {
        unit();
        for (int u = 2; u < nunits; ++u) unit();
    }
#pragma unroll
    for (int s = 0; s < D; ++s) use(ring[s], c + s, [](int) {});
}

__device__ __forceinline__ void mlp_offsets(const MlpArgs &a, int &ob1, int &oW2, int &ob2) {
    ob1 = a.F * kMlpHidden;
    oW2 = ob1 + kMlpHidden;
    ob2 = oW2 + kMlpHidden * a.K;
}

// G' = g / (|G| + 1) in float64 (optimize.py:82-83 with grad_hist float64);
// obs carries it as float32 after the P zero weight-history entries and L'.
__device__ __forceinline__ void write_grad(const MlpArgs &a, size_t e, int idx, float g) {
    const size_t gi = e * a.P + idx;
    const double gn = static_cast<double>(g) / (fabs(a.G[gi]) + 1.0);
    a.G[gi] = gn;
    a.obs[e * (2 * static_cast<size_t>(a.P) + 1) + a.P + 1 + idx] = static_cast<float>(gn);
}

// Barrier of the phase bodies: the whole workgroup.
struct WgSync {
    __device__ __forceinline__ void operator()() const { __syncthreads(); }
};
// tid: thread index within the 256 threads that run the body; sync: their barrier
template <bool A, typename Sync>
__device__ __forceinline__ void mlp_train_body(const MlpArgs &a, const size_t e, MlpTrainShared &sh,
                                               MlpStamps &ms, const int tid, const Sync &sync) {
    unsigned long long *stamps = ms.stamps;
    (void)stamps;
    CE_STAMP(0);
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar loops)
    const int li = lane & 31, h = lane >> 5;
    const int F = a.F, K = a.K, P = a.P;
    int ob1, oW2, ob2;
    mlp_offsets(a, ob1, oW2, ob2);
    float *W = a.W + e * P;
    const float *act = a.act + e * P;
    double *G = a.G + e * P;
    float *obs = a.obs + e * (2 * static_cast<size_t>(P) + 1);

    if (tid < kMlpBatch) {
        const int sel = a.order_sel[e];
        sh.rows[tid] = a.order[(static_cast<size_t>(sel) * a.E + e) * a.N + tid];
    }
    // small parameters: b1, W2, b2 updated (W <- W - a) and staged
    for (int i = tid; i < P - ob1; i += kMlpBlock) {
        const int idx = ob1 + i;
        const float w = W[idx] - act[idx];
        W[idx] = w;
        if (idx < oW2) sh.b1s[idx - ob1] = w;
        else if (idx < ob2) sh.w2s[(idx - oW2) / K][(idx - oW2) % K] = w;
        else sh.b2s[idx - ob2] = w;
    }
    // obs[0:P] = wght_hist[idx] == 0 (optimize.py:84-86 never leaves zero)
    zero_floats(obs, P, tid, kMlpBlock);
    sync();

    // ---- forward H^T = W1'^T X_b^T, k split over the 4 waves in units of
    // kTrainDepth chunks (a leftover F/8 % D chunks go to wave 3); W1 <- W1 - a.
    {
        const int chunks = F / 8;
        const int units = chunks / kTrainDepth;
        const int u0 = wave * units / 4, u1 = (wave + 1) * units / 4;
        f32x16 acc0 = {}, acc1 = {};
        const float *xrow = a.X + static_cast<size_t>(sh.rows[li]) * F + 4 * h;
        const int wofs = 4 * h * kMlpHidden + 2 * li;   // + (8c + jj) * 64
        struct Stage {
            float4 x;
            float2 w[4], d[4];
        };
        auto load = [&](Stage &st, int c, int part) {
            if (part != 0) st.x = *reinterpret_cast<const float4 *>(xrow + 8 * c);
            if (part != 1) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    st.w[jj] = ld_f2<A>(W + wofs + (8 * c + jj) * kMlpHidden);
                    st.d[jj] = ld_f2_nt<A>(act + wofs + (8 * c + jj) * kMlpHidden);
                }
            }
        };
        // W' = W - a stored back, the W / a slot refilled, W''s 8 MFMAs, then
        // the X slot refilled
        auto use = [&](const Stage &st, int c, auto &&refill) {
            float2 wc[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                wc[jj] = make_float2(st.w[jj].x - st.d[jj].x, st.w[jj].y - st.d[jj].y);
                st_f2<A>(W + wofs + (8 * c + jj) * kMlpHidden, wc[jj]);
            }
            refill(0);
            const float xs[4] = {st.x.x, st.x.y, st.x.z, st.x.w};
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                acc0 = mfma32(wc[jj].x, xs[jj], acc0);
                acc1 = mfma32(wc[jj].y, xs[jj], acc1);
            }
            refill(1);
        };
        pipelined<kTrainDepth, Stage>(u0 * kTrainDepth, u1 - u0, load, use);
        if (wave == 3) {
            for (int c = units * kTrainDepth; c < chunks; ++c) {
                Stage st;
                load(st, c, -1);
                use(st, c, [](int) {});
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            sh.part[wave][2 * acc_row(r, h)][li] = acc0[r];
            sh.part[wave][2 * acc_row(r, h) + 1][li] = acc1[r];
        }
    }
    CE_STAMP(1);
    sync();
    for (int i = tid; i < kMlpHidden * kMlpBatch; i += kMlpBlock) {
        const int j = i / kMlpBatch, s = i % kMlpBatch;
        const float z = ((sh.part[0][j][s] + sh.part[1][j][s]) + (sh.part[2][j][s] + sh.part[3][j][s])) +
                        sh.b1s[j];
        sh.hs[s][j] = z > 0.0f ? z : 0.0f;
    }
    sync();

    // ---- logits, softmax, cross-entropy (utils_math.py:25-34,51-63), P - Y
    if (tid < kMlpBatch) {
        const int s = tid;
        float z[kMlpMaxK];
        float m = -INFINITY;
        for (int k = 0; k < K; ++k) {
            float acc = sh.b2s[k];
            for (int j = 0; j < kMlpHidden; ++j) acc = fmaf(sh.hs[s][j], sh.w2s[j][k], acc);
            z[k] = acc;
            m = fmaxf(m, acc);
        }
        float sum = 0.0f;
        for (int k = 0; k < K; ++k) {
            z[k] = expf(z[k] - m);
            sum += z[k];
        }
        const int y = a.label[sh.rows[s]];
        for (int k = 0; k < K; ++k) {
            const float p = z[k] / sum;
            sh.dz2[s][k] = p - (k == y ? 1.0f : 0.0f);
            if (k == y) sh.ce[s] = -logf(p + 1e-16f);
        }
    }
    sync();

    // ---- small gradients: dW2, db2, dz1 = (dz2 W2^T) * (H > 0), db1
    const float inv_b = 1.0f / kMlpBatch;
    for (int i = tid; i < kMlpHidden * K; i += kMlpBlock) {
        const int j = i / K, k = i % K;
        float acc = 0.0f;
        for (int s = 0; s < kMlpBatch; ++s) acc = fmaf(sh.hs[s][j], sh.dz2[s][k], acc);
        write_grad(a, e, oW2 + i, acc * inv_b);
    }
    if (tid < K) {
        float acc = 0.0f;
        for (int s = 0; s < kMlpBatch; ++s) acc += sh.dz2[s][tid];
        write_grad(a, e, ob2 + tid, acc * inv_b);
    }
    float dz1v[kMlpHidden * kMlpBatch / kMlpBlock];
#pragma unroll
    for (int q = 0; q < kMlpHidden * kMlpBatch / kMlpBlock; ++q) {
        const int i = tid + q * kMlpBlock;
        const int s = i / kMlpHidden, j = i % kMlpHidden;
        float acc = 0.0f;
        for (int k = 0; k < K; ++k) acc = fmaf(sh.dz2[s][k], sh.w2s[j][k], acc);
        dz1v[q] = sh.hs[s][j] > 0.0f ? acc : 0.0f;
    }
    sync();
#pragma unroll
    for (int q = 0; q < kMlpHidden * kMlpBatch / kMlpBlock; ++q) {
        const int i = tid + q * kMlpBlock;
        sh.hs[i / kMlpHidden][i % kMlpHidden] = dz1v[q];
    }
    sync();
    if (tid < kMlpHidden) {
        float acc = 0.0f;
        for (int s = 0; s < kMlpBatch; ++s) acc += sh.hs[s][tid];
        write_grad(a, e, ob1 + tid, acc * inv_b);
    }
    CE_STAMP(2);

    // ---- dW1 = X_b^T dz1 on MFMA: 32 features x 64 hidden per tile (two
    // accumulators sharing the X operand, even / odd hidden units), K = 32
    // samples.  A tile's 16 grad-history pairs and 16 X operands (L2 hits:
    // the forward just read these rows) are issued together ahead of its
    // MFMAs; G' and obs are written from the accumulators, one 512-B G run
    // per row.  Accesses of the partial last tile's rows past F are clamped
    // to row F - 1 (valid memory, discarded), so the loads need no branch.
    {
        const int ftiles = (F + 31) / 32;
        float *og = obs + P + 1;
        for (int ft = wave; ft < ftiles; ft += 4) {
            const int f = ft * 32 + li;
            double2 g[16];
            float x[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int fr = min(ft * 32 + acc_row(r, h), F - 1);
                g[r] = ld_d2_nt<A>(G + fr * kMlpHidden + 2 * li);
            }
#pragma unroll
            for (int ks = 0; ks < 16; ++ks)
                x[ks] = a.X[static_cast<size_t>(sh.rows[2 * ks + h]) * F + min(f, F - 1)];
            f32x16 acc0 = {}, acc1 = {};
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) {
                const int s = 2 * ks + h;
                const float xa = f < F ? x[ks] : 0.0f;
                acc0 = mfma32(xa, sh.hs[s][2 * li], acc0);
                acc1 = mfma32(xa, sh.hs[s][2 * li + 1], acc1);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int fr = ft * 32 + acc_row(r, h);
                if (fr < F) {
                    const int idx = fr * kMlpHidden + 2 * li;
                    const double g0 = static_cast<double>(acc0[r] * inv_b) / (fabs(g[r].x) + 1.0);
                    const double g1 = static_cast<double>(acc1[r] * inv_b) / (fabs(g[r].y) + 1.0);
                    st_d2_nt<A>(G + idx, make_double2(g0, g1));
                    st_nt(og + idx, static_cast<float>(g0));
                    st_nt(og + idx + 1, static_cast<float>(g1));
                }
            }
        }
    }

    CE_STAMP(3);
    // ---- loss recurrence, reward, done (optimize.py:80-81,90-91,102-103)
    if (tid == 0) {
        float loss = 0.0f;
        for (int s = 0; s < kMlpBatch; ++s) loss += sh.ce[s];
        loss /= static_cast<float>(kMlpBatch);
        const double lp = a.L[e];
        const double ln = (static_cast<double>(loss) - lp) / (lp + 0.1);
        a.L[e] = ln;
        obs[P] = static_cast<float>(ln);
        const int s = a.step[e] + 1;
        a.step[e] = s;
        a.reward[e] = -loss;
        a.done[e] = s >= a.max_steps ? 1 : 0;
        a.episode_len[e] = s;
    }
#ifdef CE_DIAG
    if (tid < 4) a.diag[e * kStamps + tid] = stamps[tid];
#endif
}

// Reset one env (block-wide): W <- W0, histories zero, order composed with
// the reset permutation, reset observation = zeros (optimize.py:58-67).
template <typename Sync>
__device__ void mlp_reset_env(const MlpArgs &a, size_t e, bool write_obs, int tid, const Sync &sync) {
    const int P = a.P;
    for (int i = tid; i < P; i += kMlpBlock) {
        a.W[e * P + i] = a.W0[e * P + i];
        a.G[e * P + i] = 0.0;
    }
    if (write_obs) zero_floats(a.obs + e * (2 * static_cast<size_t>(P) + 1), 2 * P + 1, tid, kMlpBlock);
    const int sel = a.order_sel[e];
    const int32_t *cur = a.order + (static_cast<size_t>(sel) * a.E + e) * a.N;
    int32_t *nxt = a.order + (static_cast<size_t>(1 - sel) * a.E + e) * a.N;
    const int32_t *perm = a.perm + e * a.N;
    for (int i = tid; i < a.N; i += kMlpBlock) nxt[i] = cur[perm[i]];
    sync();
    if (tid == 0) {
        a.order_sel[e] = 1 - sel;
        a.L[e] = 0.0;
        a.step[e] = 0;
    }
}

__global__ __launch_bounds__(kMlpBlock) void mlp_reset_kernel(MlpArgs a) {
    mlp_reset_env(a, blockIdx.x, true, threadIdx.x, WgSync{});
}

// Full-dataset forward for info['objective'] / info['accuracy'] with the
// updated weights, then the auto-reset of envs that just finished.  Each wave
// takes T consecutive 32-sample tiles per pass: 2T accumulators live across
// one sweep over K, so every W1 fragment a wave loads feeds 8T MFMAs.
template <int T, int D, bool A, typename Sync>
__device__ __forceinline__ void mlp_info_body(const MlpArgs &a, const size_t e, MlpInfoShared &sh,
                                              MlpStamps &ms, const int tid, const Sync &sync) {
    unsigned long long *stamps = ms.stamps;
    (void)stamps;
    CE_STAMP(4);
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // wave-uniform (scalar loops)
    const int li = lane & 31, h = lane >> 5;
    const int F = a.F, K = a.K, P = a.P;
    int ob1, oW2, ob2;
    mlp_offsets(a, ob1, oW2, ob2);
    const float *W = a.W + e * P;
    for (int i = tid; i < P - ob1; i += kMlpBlock) {
        const int idx = ob1 + i;
        const float w = W[idx];
        if (idx < oW2) sh.b1s[idx - ob1] = w;
        else if (idx < ob2) sh.w2s[(idx - oW2) / K][(idx - oW2) % K] = w;
        else sh.b2s[idx - ob2] = w;
    }
    sync();

    float loss_acc = 0.0f;
    int hits = 0;
    const int tiles = a.N / 32;
    const int chunks = F / 8;
    const size_t tstride = static_cast<size_t>(chunks) * 64 * 4;   // floats per swizzled tile
    const int wofs = 4 * h * kMlpHidden + 2 * li;                   // + (8c + jj) * 64
    for (int t0 = wave * T; t0 < tiles; t0 += 4 * T) {
        const int nt = tiles - t0 < T ? tiles - t0 : T;   // wave-uniform
        f32x16 acc[T][2];
#pragma unroll
        for (int q = 0; q < T; ++q) acc[q][0] = acc[q][1] = f32x16{};
        const float *xb = a.Xs + (static_cast<size_t>(t0) * chunks * 64 + lane) * 4;
        // tiles past the end of a partial pass read tile 0 (valid memory); their
        // accumulators are never used, so the MFMA loop stays branch-free
        size_t toff[T];
#pragma unroll
        for (int q = 0; q < T; ++q) toff[q] = (q < nt ? q : 0) * tstride;
        {
        // a D-deep pipeline of chunk operands: parts 0..T-1 are the
        // tiles' X float4s (refilled once the tile's 8 MFMAs issued), part T
        // the W1 pairs
        struct Stage {
            float4 x[T];
            float2 w[4];
        };
        auto load = [&](Stage &st, int c, int part) {
#pragma unroll
            for (int q = 0; q < T; ++q)
                if (part < 0 || part == q)
                    st.x[q] = *reinterpret_cast<const float4 *>(xb + toff[q] + 256 * c);
            if (part < 0 || part == T) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) st.w[jj] = ld_f2<A>(W + wofs + (8 * c + jj) * kMlpHidden);
            }
        };
        auto use = [&](const Stage &st, int, auto &&refill) {
            // the W1 pairs are copied out and their slot refilled first, so
            // the next visit's W1 loads get a whole chunk of MFMA work as cover
            float2 wc[4];
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) wc[jj] = st.w[jj];
            refill(T);
#pragma unroll
            for (int q = 0; q < T; ++q) {
                const float xs[4] = {st.x[q].x, st.x[q].y, st.x[q].z, st.x[q].w};
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    acc[q][0] = mfma32(wc[jj].x, xs[jj], acc[q][0]);
                    acc[q][1] = mfma32(wc[jj].y, xs[jj], acc[q][1]);
                }
                refill(q);
            }
        };
        const int units = chunks / D;
        pipelined<D, Stage>(0, units, load, use);
        for (int c = units * D; c < chunks; ++c) {
            Stage st;
            load(st, c, -1);
            use(st, c, [](int) {});
        }
        }
#pragma unroll
        for (int q = 0; q < T; ++q) {
            if (q >= nt) continue;
            // bias + relu on H^T, then logits^T = W2^T H^T with H^T as the B operand
            f32x16 lg = {};
#pragma unroll
            for (int ht = 0; ht < 2; ++ht) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int hid = 2 * acc_row(r, h) + ht;
                    const float z = acc[q][ht][r] + sh.b1s[hid];
                    const float hv = z > 0.0f ? z : 0.0f;
                    const float wa = li < K ? sh.w2s[hid][li] : 0.0f;
                    lg = mfma32(wa, hv, lg);
                }
            }
            // lane (sample li, half h) holds classes acc_row(r, h) of its sample
            float m = -INFINITY, best = -INFINITY;
            int arg = 0;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int k = acc_row(r, h);
                if (k < K) {
                    const float z = lg[r] + sh.b2s[k];
                    lg[r] = z;
                    m = fmaxf(m, z);
                }
            }
            m = fmaxf(m, __shfl_xor(m, 32));
            float sum = 0.0f;
            const int row = (t0 + q) * 32 + li;
            const int y = a.label[row];
            float zy = 0.0f;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int k = acc_row(r, h);
                if (k < K) {
                    sum += expf(lg[r] - m);
                    if (k == y) zy = lg[r];
                    if (lg[r] > best || (lg[r] == best && k < arg)) {
                        best = lg[r];
                        arg = k;
                    }
                }
            }
            sum += __shfl_xor(sum, 32);
            zy += __shfl_xor(zy, 32);            // exactly one half owns class y
            const float best_o = __shfl_xor(best, 32);
            const int arg_o = __shfl_xor(arg, 32);
            if (best_o > best || (best_o == best && arg_o < arg)) arg = arg_o;
            if (h == 0) {
                const float p = expf(zy - m) / sum;
                loss_acc += -logf(p + 1e-16f);
                hits += arg == y ? 1 : 0;
            }
        }
    }
    CE_STAMP(5);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        loss_acc += __shfl_xor(loss_acc, off);
        hits += __shfl_xor(hits, off);
    }
    if (lane == 0) {
        sh.red_loss[wave] = loss_acc;
        sh.red_hits[wave] = hits;
    }
    sync();
    if (tid == 0) {
        const float tot = (sh.red_loss[0] + sh.red_loss[1]) + (sh.red_loss[2] + sh.red_loss[3]);
        a.objective[e] = tot / static_cast<float>(a.N);
        a.accuracy[e] = static_cast<float>(sh.red_hits[0] + sh.red_hits[1] + sh.red_hits[2] +
                                           sh.red_hits[3]) /
                        static_cast<float>(a.N);
    }
    const bool wipe = a.auto_reset && a.step[e] >= a.max_steps;
    sync();
    if (wipe) mlp_reset_env(a, e, true, tid, sync);
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CE_STAMP(6);
    if (tid >= 4 && tid < 7) a.diag[e * kStamps + tid] = stamps[tid];
#endif
}

// mlp_step_kernel: the product step.  One 4-wave workgroup per env runs the
// train phase then the info phase; at <= 256 registers two workgroups share
// a CU, and whichever of them is in its info phase keeps the matrix pipe
// busy while the other streams (measured 4.4-4.7 ms per 4096-env step
// against 5.6 ms for the split pair).
template <bool A>
__global__ __launch_bounds__(kMlpBlock, 2) void mlp_step_kernel(MlpArgs a) {
    __shared__ union {
        MlpTrainShared t;
        MlpInfoShared i;
    } sh;
    MlpStamps ms{};
    const size_t e = blockIdx.x;
    mlp_train_body<A>(a, e, sh.t, ms, threadIdx.x, WgSync{});
    __syncthreads();
    mlp_info_body<kStepInfoTiles, kStepInfoDepth, A>(a, e, sh.i, ms, threadIdx.x, WgSync{});
}

// The split pair (CE_MLP_SPLIT=1, and CE_MLP_PHASES=train|info to time one
// phase alone): the train phase at 2 waves per SIMD, the info phase holding
// 16 32x32 accumulators per wave (one wave per SIMD, 512 registers).
template <bool A>
__global__ __launch_bounds__(kMlpBlock) void mlp_train_kernel(MlpArgs a) {
    __shared__ MlpTrainShared sh;
    MlpStamps ms{};
    mlp_train_body<A>(a, blockIdx.x, sh, ms, threadIdx.x, WgSync{});
}

template <bool A>
__global__ __launch_bounds__(kMlpBlock) void mlp_info_kernel(MlpArgs a) {
    __shared__ MlpInfoShared sh;
    MlpStamps ms{};
    mlp_info_body<kSplitInfoTiles, kSplitInfoDepth, A>(a, blockIdx.x, sh, ms, threadIdx.x,
                                                          WgSync{});
}

}  // namespace ce
