// Fused MultiOptLRs-v0 step (learned per-parameter learning rates) for gfx950.
//
// One launch advances E envs x P agents by one OptVecEnv.step:
//   OptVecEnv.step_async/step_wait        custom_envs/vectorize/optvecenv.py:70-88
//   OptEnvRunner.step (rows in sorted agent-name order, reward/done/info
//                      replicated per agent)  optvecenv.py:10-14,38-46
//   BaseEnvironment.step                  custom_envs/envs/baseenvironment.py:30-41
//   MultiOptLRs.base_step (version 3,3,0,6) custom_envs/envs/multioptlrs.py:80-129
//     action v0: lr = 10^(a - 4)          custom_envs/utils/utils_env.py:113-114
//     theta <- theta - grad * lr          (float32, the TF1 variables' dtype)
//     Rosenbrock problem                  custom_envs/problems/optimize_function.py:130-137,
//                                         custom_envs/utils/utils_functions.py:4-6
//     observation v3: ratios of the two newest raw-history entries, nan_to_num
//                                         utils_env.py:126-164
//     History append / build_multistate   custom_envs/utils/utils_common.py:102-196
//     obs_i = clip(nan_to_num(.), +-100) - 1; reward v6 = clip(1 - l~, +-100);
//     early stop at loss > 1e4 with penalty; 14-key info (multioptlrs.py:97-127)
//   auto-reset on done                    concurrentvecenv.py:37 (any(done) on the agent list)
//
// Mapping: one thread per env (P is a handful of agents).  State is struct-
// of-arrays [field][E] so a wave's 64 envs read and write coalesced lines.
// Rings: the raw history keeps 5 entries (multioptlrs.py:42-45), slot
// step % 5; the adjusted history keeps H entries, slot (step - 1) % H;
// a slot not written since the last reset reads as the reset zero.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ce {

constexpr int kRawHist = 5;
constexpr int kMultiBlock = 256;
constexpr int kMultiInfo = 14;   // info keys, order in include/custom_envs_amd.h

struct MultiArgs {
    int E, H, max_batches, auto_reset;
    const float *init;       // [P] initial points
    const int32_t *row_agent;// [P] agent index of row r (sorted agent names)
    float *theta;            // [P][E]
    float *grad;             // [P][E] gradient at theta (newest raw entry)
    float *hl;               // [5][E]
    float *hg;               // [5][P][E]
    float *hw;               // [5][P][E]
    double *al;              // [H][E]
    double *ag;              // [H][P][E]
    double *aw;              // [H][P][E]
    int32_t *step;           // [E]
    const float *act;        // [E][P] rows
    float *obs;              // [E][P][3H] rows
    float *reward;           // [E][P] rows
    uint8_t *done;           // [E][P] rows
    float *info;             // [E][14]
    int32_t *episode_len;    // [E]
};

// Sum of Rosenbrock over coordinate pairs in float32, with TF1's autodiff
// order for the gradient: dL/dy = 200 d, dL/dx = -(2 (200 d)) x - 2 (1 - x),
// d = y - x^2.  Contraction is off so every product rounds as in the oracle.
template <int P>
__device__ __forceinline__ void rosenbrock_pairs(const float (&th)[P], float (&g)[P], float &loss) {
#pragma clang fp contract(off)
    loss = 0.0f;
#pragma unroll
    for (int k = 0; k < P; k += 2) {
        const float x = th[k], y = th[k + 1];
        const float d = y - x * x;
        const float r = 1.0f - x;
        loss = loss + (100.0f * (d * d) + r * r);
        const float t = 200.0f * d;
        g[k] = -((2.0f * t) * x) - 2.0f * r;
        g[k + 1] = t;
    }
}

// numpy.nan_to_num of a / |b| in float64.
__device__ __forceinline__ double ratio(double a, double b) {
    const double q = a / fabs(b);
    if (q != q) return 0.0;
    if (isinf(q)) return q > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308;
    return q;
}

__device__ __forceinline__ double clip100(double v) {
    if (v != v) v = 0.0;
    return v < -100.0 ? -100.0 : (v > 100.0 ? 100.0 : v);
}

template <int P>
__device__ __forceinline__ void multi_reset_env(const MultiArgs &a, int e) {
    const size_t E = a.E;
    float th[P], g[P], loss;
#pragma unroll
    for (int i = 0; i < P; ++i) th[i] = a.init[i];
    rosenbrock_pairs<P>(th, g, loss);
    for (int s = 0; s < kRawHist; ++s) {
        a.hl[s * E + e] = s == 0 ? loss : 0.0f;
#pragma unroll
        for (int i = 0; i < P; ++i) {
            a.hg[(s * P + i) * E + e] = s == 0 ? g[i] : 0.0f;
            a.hw[(s * P + i) * E + e] = s == 0 ? th[i] : 0.0f;
        }
    }
    for (int s = 0; s < a.H; ++s) {
        a.al[s * E + e] = 0.0;
#pragma unroll
        for (int i = 0; i < P; ++i) {
            a.ag[(s * P + i) * E + e] = 0.0;
            a.aw[(s * P + i) * E + e] = 0.0;
        }
    }
#pragma unroll
    for (int i = 0; i < P; ++i) {
        a.theta[i * E + e] = th[i];
        a.grad[i * E + e] = g[i];
    }
    a.step[e] = 0;
}

template <int P>
__global__ __launch_bounds__(kMultiBlock) void multi_reset_kernel(MultiArgs a) {
    const int e = blockIdx.x * kMultiBlock + threadIdx.x;
    if (e >= a.E) return;
    multi_reset_env<P>(a, e);
    const int row = 3 * a.H;
    for (int k = 0; k < P * row; ++k) a.obs[static_cast<size_t>(e) * P * row + k] = -1.0f;
}

template <int P>
__global__ __launch_bounds__(kMultiBlock) void multi_step_kernel(MultiArgs a) {
#pragma clang fp contract(off)
    const int e = blockIdx.x * kMultiBlock + threadIdx.x;
    if (e >= a.E) return;
    const size_t E = a.E;
    const int H = a.H;
    const int s = a.step[e] + 1;

    // ---- update (multioptlrs.py:81-87): rows -> agents, lr = 10^(a - 4)
    float th[P], g[P], lr[P];
#pragma unroll
    for (int r = 0; r < P; ++r) {
        const int i = a.row_agent[r];
        // numpy float32 10 ** (a - 4): the exponent rounds to float32 first;
        // the power is taken in float64 and rounded once (correctly rounded
        // but for ties far below float32 resolution)
        const float x = a.act[static_cast<size_t>(e) * P + r] - 4.0f;
        lr[i] = static_cast<float>(pow(10.0, static_cast<double>(x)));
    }
#pragma unroll
    for (int i = 0; i < P; ++i) {
        th[i] = a.theta[i * E + e];
        g[i] = a.grad[i * E + e];
    }
#pragma unroll
    for (int i = 0; i < P; ++i) th[i] = th[i] - g[i] * lr[i];
    float loss;
    rosenbrock_pairs<P>(th, g, loss);

    // ---- raw history append, observation v3 against the previous entry
    const int slot = s % kRawHist, prev = (s - 1) % kRawHist;
    const double l_prev = a.hl[prev * E + e];
    a.hl[slot * E + e] = loss;
    const double adj_l = ratio(loss, l_prev);
    double adj_w[P], adj_g[P];
    double gdiff = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        const float gp = a.hg[(prev * P + i) * E + e];
        const float wp = a.hw[(prev * P + i) * E + e];
        adj_g[i] = ratio(g[i], gp);
        adj_w[i] = ratio(th[i], wp);
        gdiff += fabs(static_cast<double>(g[i]) - static_cast<double>(gp));
        a.hg[(slot * P + i) * E + e] = g[i];
        a.hw[(slot * P + i) * E + e] = th[i];
    }
    const int aslot = (s - 1) % H;
    a.al[aslot * E + e] = adj_l;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        a.ag[(aslot * P + i) * E + e] = adj_g[i];
        a.aw[(aslot * P + i) * E + e] = adj_w[i];
    }

    // ---- reward v6 + termination (multioptlrs.py:102-107)
    double reward = 1.0 - adj_l;
    reward = reward < -100.0 ? -100.0 : (reward > 100.0 ? 100.0 : reward);
    bool terminal = s >= a.max_batches;
    if (!terminal && loss > 1e4f) {
        terminal = true;
        reward -= static_cast<double>(a.max_batches - s);
    }

    // ---- observations: per agent [w~ (H, newest first) | l~ (H) | g~ (H)]
    const int row = 3 * H;
    float *obs = a.obs + static_cast<size_t>(e) * P * row;
    double st_abs = 0.0;
    const bool wipe = terminal && a.auto_reset;
    for (int k = 0; k < H; ++k) {
        const bool live = k < s;                    // older slots are reset zeros
        const int sl = ((s - 1 - k) % H + H) % H;
        const double lk = live ? a.al[sl * E + e] : 0.0;
        st_abs += P * fabs(lk);
#pragma unroll
        for (int r = 0; r < P; ++r) {
            const int i = a.row_agent[r];
            const double wk = live ? a.aw[(sl * P + i) * E + e] : 0.0;
            const double gk = live ? a.ag[(sl * P + i) * E + e] : 0.0;
            st_abs += fabs(wk) + fabs(gk);
            float *o = obs + r * row;
            o[k] = wipe ? -1.0f : static_cast<float>(clip100(wk) - 1.0);
            o[H + k] = wipe ? -1.0f : static_cast<float>(clip100(lk) - 1.0);
            o[2 * H + k] = wipe ? -1.0f : static_cast<float>(clip100(gk) - 1.0);
        }
    }

    // ---- info (multioptlrs.py:112-127), float64 arithmetic
    double wsum = 0.0, amean = 0.0, gsum = 0.0, lsum = 0.0, adjg = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) {
        wsum += fabs(static_cast<double>(th[i]));
        amean += lr[i];
        adjg += fabs(adj_g[i]);
    }
    amean /= P;
    double avar = 0.0;
#pragma unroll
    for (int i = 0; i < P; ++i) avar += (lr[i] - amean) * (lr[i] - amean);
    for (int k = 0; k < kRawHist; ++k) {
        lsum += a.hl[k * E + e];
#pragma unroll
        for (int i = 0; i < P; ++i) gsum += a.hg[(k * P + i) * E + e];
    }
    float *info = a.info + static_cast<size_t>(e) * kMultiInfo;
    info[0] = terminal ? loss : __builtin_nanf("");          // loss (None -> NaN)
    info[1] = loss;                                           // batch_loss
    info[2] = static_cast<float>(wsum / P);                   // weights_mean
    info[3] = static_cast<float>(wsum);                       // weights_sum
    info[4] = static_cast<float>(amean);                      // actions_mean
    info[5] = static_cast<float>(sqrt(avar / P));             // actions_std
    info[6] = static_cast<float>(st_abs / (P * row));         // states_mean
    info[7] = static_cast<float>(st_abs);                     // states_sum
    info[8] = static_cast<float>(gsum / (kRawHist * P));      // grads_mean
    info[9] = static_cast<float>(gsum);                       // grads_sum
    info[10] = static_cast<float>(lsum / kRawHist);           // loss_mean
    info[11] = static_cast<float>(adj_l);                     // adjusted_loss
    info[12] = static_cast<float>(adjg / P);                  // adjusted_grad
    info[13] = static_cast<float>(gdiff / P);                 // grad_diff
    a.episode_len[e] = s;
#pragma unroll
    for (int r = 0; r < P; ++r) {
        a.reward[static_cast<size_t>(e) * P + r] = static_cast<float>(reward);
        a.done[static_cast<size_t>(e) * P + r] = terminal ? 1 : 0;
    }

    if (wipe) {
        multi_reset_env<P>(a, e);
    } else {
#pragma unroll
        for (int i = 0; i < P; ++i) {
            a.theta[i * E + e] = th[i];
            a.grad[i * E + e] = g[i];
        }
        a.step[e] = s;
    }
}

}  // namespace ce
