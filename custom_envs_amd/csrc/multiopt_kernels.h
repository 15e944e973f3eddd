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
// Mapping: one lane per (env, agent).  An env's agents are a group of G lanes
// (G = P rounded up to a power of two; lanes i >= P idle), so a wave holds
// 64/G envs and every per-env quantity is a shuffle reduction inside the
// group.  Lane i is AGENT i; its output row is agent_row[i] (the sorted-name
// order, which differs from the agent order once P >= 11).  Per-agent state
// is [slot][E][P] so a group's P values are contiguous and a wave's loads and
// stores are coalesced.  Rings: the raw history keeps 5 entries
// (multioptlrs.py:42-45), slot step % 5; the adjusted history keeps H
// entries, slot (step - 1) % H; a slot not written since the last reset
// reads as the reset zero.  The wave's observation rows are one contiguous
// block of the output: they are assembled in LDS and stored lane-contiguous.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "optimize_kernels.h"   // xchg<>: DPP / swizzle lane exchanges

namespace ce {

constexpr int kRawHist = 5;
#ifndef CE_MULTI_WAVES
#define CE_MULTI_WAVES 1
#endif
// One wave per workgroup: config 5's 1024 envs are 64 waves, which then
// spread over 64 CUs instead of sharing 16 (each wave's loads are all issued
// up front, so CU-local load throughput matters).
constexpr int kMultiBlock = 64 * CE_MULTI_WAVES;
constexpr int kMultiInfo = 14;     // info keys, order in include/custom_envs_amd.h
constexpr int kMultiMaxP = 64;
constexpr int kMultiStageH = 20;   // LDS-staged observation rows up to this H

struct MultiArgs {
    int E, H, max_batches, auto_reset;
    float init[kMultiMaxP];      // initial points (agent order)
    float init_g[kMultiMaxP];    // the problem's gradient at them (rosenbrock_ref)
    float init_l;                // and its loss
    int agent_row[kMultiMaxP];   // output row of agent i within its env
    float *theta;            // [E][P]
    float *grad;             // [E][P] gradient at theta (newest raw entry)
    float *hl;               // [5][E]
    float *hg;               // [5][E][P]
    float *hw;               // [5][E][P]
    // adjusted history, kept in observation form: an entry x is stored as
    // float(clip(nan_to_num(x), +-100) - 1), the value every later
    // observation row repeats, plus the float64 |w~| + |g~| + |l~| of the
    // agent's entry for states_sum (multioptlrs.py:116-117)
    float *ol;               // [H][E]    l~
    float *og;               // [H][E][P] g~
    float *ow;               // [H][E][P] w~
    double *sa;              // [H][E][P] |w~| + |g~| + |l~| (raw)
    int32_t *step;           // [E]
    const float *act;        // [E][P] rows
    float *obs;              // [E][P][3H] rows
    float *reward;           // [E][P] rows
    uint8_t *done;           // [E][P] rows
    float *info;             // [E][14]
    int32_t *episode_len;    // [E]
};

// base[idx] with a 32-bit byte offset (idx * sizeof(T) < 2^32, which
// ce_multi_create guarantees): the access is the uniform base in SGPRs plus
// one VGPR offset, with no 64-bit address arithmetic per lane
template <typename T>
__device__ __forceinline__ T &at32(T *base, unsigned idx) {
    return *reinterpret_cast<T *>(reinterpret_cast<char *>(base) + idx * static_cast<unsigned>(sizeof(T)));
}
template <typename T>
__device__ __forceinline__ const T &at32(const T *base, unsigned idx) {
    return *reinterpret_cast<const T *>(reinterpret_cast<const char *>(base) +
                                        idx * static_cast<unsigned>(sizeof(T)));
}

template <int P>
struct Group {
    static constexpr int G = P <= 2 ? 2 : P <= 4 ? 4 : P <= 8 ? 8 : P <= 16 ? 16 : P <= 32 ? 32 : 64;
};

// Sum over a group of G lanes by an xor butterfly on DPP / ds_swizzle
// exchanges (no LDS round trip): every lane of the group gets the total.
template <int G, typename T, int OFF = G / 2>
__device__ __forceinline__ T group_sum(T v) {
    if constexpr (OFF == 0) {
        return v;
    } else {
        v = v + xchg<OFF>(v);
        return group_sum<G, T, OFF / 2>(v);
    }
}

// Lane SRC of each G-lane group, broadcast to the group (G <= 4: DPP
// quad_perm; wider groups: ds_bpermute).
template <int G, int SRC>
__device__ __forceinline__ float group_bcast(float v) {
    if constexpr (G == 4) {
        return __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), SRC * 0x55,
                                                           0xf, 0xf, false));
    } else if constexpr (G == 2) {
        constexpr int c = SRC | (SRC << 2) | ((2 + SRC) << 4) | ((2 + SRC) << 6);
        return __uint_as_float(__builtin_amdgcn_update_dpp(0u, __float_as_uint(v), c, 0xf, 0xf,
                                                           false));
    } else {
        return __shfl(v, SRC, G);
    }
}

template <int G, int P, int Q = 0>
__device__ __forceinline__ float pair_terms_sum(float loss, float term) {
    // loss + term(pair 0) + term(pair 1) + ..., left to right (TF1's add order)
    if constexpr (Q >= P / 2) {
        return loss;
    } else {
        return pair_terms_sum<G, P, Q + 1>(loss + group_bcast<G, 2 * Q>(term), term);
    }
}

// Sum of Rosenbrock over coordinate pairs in float32, with TF1's autodiff
// order for the gradient: dL/dy = 200 d, dL/dx = -(2 (200 d)) x - 2 (1 - x),
// d = y - x^2; the loss sums the pairs left to right.  Lane i holds agent i;
// its pair partner is lane i ^ 1.  Contraction is off so every product
// rounds as in the oracle.
template <int P>
__device__ __forceinline__ void rosenbrock_lane(float th, int i, float &g, float &loss) {
#pragma clang fp contract(off)
    constexpr int G = Group<P>::G;
    const float other = xchg<1>(th);
    const bool is_x = (i & 1) == 0;
    const float x = is_x ? th : other, y = is_x ? other : th;
    const float d = y - x * x;
    const float r = 1.0f - x;
    const float term = 100.0f * (d * d) + r * r;
    const float t = 200.0f * d;
    g = is_x ? -((2.0f * t) * x) - 2.0f * r : t;
    loss = pair_terms_sum<G, P>(0.0f, term);
}

// rosenbrock_lane for a whole point on the host, in the same float32
// operation order (no contraction): the reset point's gradient and loss
inline void rosenbrock_ref(const float *th, int P, float *g, float *loss) {
#pragma clang fp contract(off)
    float l = 0.0f;
    for (int q = 0; q < P / 2; ++q) {
        const float x = th[2 * q], y = th[2 * q + 1];
        const float d = y - x * x;
        const float r = 1.0f - x;
        const float term = 100.0f * (d * d) + r * r;
        const float t = 200.0f * d;
        g[2 * q] = -((2.0f * t) * x) - 2.0f * r;
        g[2 * q + 1] = t;
        l = l + term;
    }
    *loss = l;
}

// numpy.nan_to_num of a / |b| in float64.
__device__ __forceinline__ double ratio(double a, double b) {
    const double q = a / fabs(b);
    if (q != q) return 0.0;
    if (isinf(q)) return q > 0 ? 1.7976931348623157e308 : -1.7976931348623157e308;
    return q;
}

// numpy.nan_to_num(a / |b|) in float64 for float32 a, b (utils_env.py:155-161).
// Finite operands with b != 0 take the hardware reciprocal, one Newton step
// and one residual correction (the IEEE quotient up to a final-rounding tie,
// far below the float32 the result is stored as); anything else takes the
// IEEE division of ratio().  About a third of the float64 work of the
// division sequence.
__device__ __forceinline__ double ratio_fast(float a, float b) {
    const double ad = a, bd = fabs(static_cast<double>(b));
    if (!(bd > 0.0 && bd <= 3.4028234663852886e38 && fabs(ad) <= 3.4028234663852886e38))
        return ratio(a, b);
    double r = __builtin_amdgcn_rcp(bd);
    r = fma(r, fma(-bd, r, 1.0), r);
    const double q = ad * r;
    return fma(fma(-bd, q, ad), r, q);
}

__device__ __forceinline__ double clip100(double v) {
    if (v != v) v = 0.0;
    return v < -100.0 ? -100.0 : (v > 100.0 ? 100.0 : v);
}

// Reset agent i of env e (MultiOptLRs.base_reset, multioptlrs.py:66-78): the
// problem back at its initial point (th0, with gradient g0 and loss l0 from
// rosenbrock_lane, evaluated by every lane of the group), the raw history
// holding that point only, the adjusted history zero.
template <int P>
__device__ __forceinline__ void multi_store_reset(const MultiArgs &a, size_t e, int i, float th0,
                                                  float g0, float l0) {
    const size_t E = a.E;
    for (int s = 0; s < kRawHist; ++s) {
        a.hg[(s * E + e) * P + i] = s == 0 ? g0 : 0.0f;
        a.hw[(s * E + e) * P + i] = s == 0 ? th0 : 0.0f;
        if (i == 0) a.hl[s * E + e] = s == 0 ? l0 : 0.0f;
    }
    for (int s = 0; s < a.H; ++s) {             // the reset zeros: obs form -1
        a.og[(s * E + e) * P + i] = -1.0f;
        a.ow[(s * E + e) * P + i] = -1.0f;
        a.sa[(s * E + e) * P + i] = 0.0;
        if (i == 0) a.ol[s * E + e] = -1.0f;
    }
    a.theta[e * P + i] = th0;
    a.grad[e * P + i] = g0;
    if (i == 0) a.step[e] = 0;
}

template <int P>
__global__ __launch_bounds__(kMultiBlock) void multi_reset_kernel(MultiArgs a) {
    constexpr int G = Group<P>::G;
    const size_t gt = static_cast<size_t>(blockIdx.x) * kMultiBlock + threadIdx.x;
    const size_t e = gt / G;
    const int i = static_cast<int>(gt % G);
    const bool on = e < static_cast<size_t>(a.E) && i < P;
    const float th0 = i < P ? a.init[i] : 0.0f;
    float g0, l0;
    rosenbrock_lane<P>(th0, i, g0, l0);
    if (!on) return;
    multi_store_reset<P>(a, e, i, th0, g0, l0);
    const int row = 3 * a.H;
    float *o = a.obs + (e * P + a.agent_row[i]) * row;
    for (int k = 0; k < row; ++k) o[k] = -1.0f;
}

// HC: the history length when known at compile time (the reference's
// default max_history = 5, multioptlrs.py:39), 0 for any H.  The kernel is
// latency-bound (a few waves per CU), so its time is its dynamic instruction
// count: with HC the ring-age arithmetic is constant and every loop over the
// history unrolls without branches, and the observation rows are staged with
// LDS stores rather than flat stores.
template <int P, int HC = 0>
__global__ __launch_bounds__(kMultiBlock) void multi_step_kernel(MultiArgs a) {
#pragma clang fp contract(off)
    constexpr int G = Group<P>::G;
    extern __shared__ float4 stage4[];        // [waves][64 / G * P * 3H] floats when H <= kMultiStageH
    float *stage = reinterpret_cast<float *>(stage4);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t gt = static_cast<size_t>(blockIdx.x) * kMultiBlock + threadIdx.x;
    const size_t e = gt / G;
    const int i = static_cast<int>(gt % G);
    const size_t E = a.E;
    const bool env_ok = e < E;
    const bool on = env_ok && i < P;
    static_assert(HC <= kMultiStageH, "compile-time histories are staged");
    const int H = HC ? HC : a.H;
    const int row = 3 * H;
    const size_t ec = env_ok ? e : 0;          // clamp so idle lanes read valid memory
    const int ic = i < P ? i : 0;
    // sorted agent names ('parameter-0', 'parameter-1', 'parameter-10', ...)
    // only reorder rows from P = 11 on; below that the row is the agent
    // index and the action load does not wait for the kernarg table
    const int r = P <= 10 ? ic : a.agent_row[ic];

    // ---- every load of the step up front: no address depends on another
    // load (the ring slots are picked from registers once `step` is in), so
    // the wave waits for memory once instead of once per dependent round trip
    // 32-bit offsets (ce_multi_create keeps every ring plane and the
    // observation block below 2^28 elements): every access is a uniform base
    // in SGPRs plus one VGPR byte offset (at32), no 64-bit address arithmetic
    const unsigned Eu = static_cast<unsigned>(E), eu = static_cast<unsigned>(ec);
    const unsigned ep = eu * P + ic;               // this lane's [E][P] element
    const int step_prev = at32(a.step, eu);
    const float act = at32(a.act, eu * P + r);
    // the reset point: loaded here, not after the stores -- vmcnt counts
    // stores too, so a load issued after them would make its first use wait
    // for every one of them to complete
    const float th_init = i < P ? a.init[i] : 0.0f;
    // the reset point's gradient and loss: the same for every env, formed
    // once on the host (rosenbrock_ref, bit-identical to rosenbrock_lane)
    const float g_init = i < P ? a.init_g[i] : 0.0f, l_init = a.init_l;
    const float th0 = at32(a.theta, ep);
    const float g0 = at32(a.grad, ep);
    float hl_v[kRawHist], hg_v[kRawHist], hw_v[kRawHist];
#pragma unroll
    for (int k = 0; k < kRawHist; ++k) {
        hl_v[k] = at32(a.hl, k * Eu + eu);
        hg_v[k] = at32(a.hg, k * Eu * P + ep);
        hw_v[k] = at32(a.hw, k * Eu * P + ep);
    }
    float ol_v[kMultiStageH], og_v[kMultiStageH], ow_v[kMultiStageH];
    double sa_v[kMultiStageH];
#pragma unroll
    for (int j = 0; j < kMultiStageH; ++j) {
        if (j < H) {                             // wave-uniform
            ol_v[j] = at32(a.ol, j * Eu + eu);
            og_v[j] = at32(a.og, j * Eu * P + ep);
            ow_v[j] = at32(a.ow, j * Eu * P + ep);
            sa_v[j] = at32(a.sa, j * Eu * P + ep);
        }
    }

    const int s = step_prev + 1;
    // ---- update (multioptlrs.py:81-87), lr = 10^(a - 4): the exponent rounds
    // to float32 first; the power is taken in float64 and rounded once
    const float x = act - 4.0f;
    const float lr = static_cast<float>(exp10(static_cast<double>(x)));
    const float th = th0 - g0 * lr;
    float g, loss;
    rosenbrock_lane<P>(th, i, g, loss);

    // ---- raw history append, observation v3 against the previous entry
    const int slot = s % kRawHist, prev = (s - 1) % kRawHist;
    double l_prev = 0.0;
    float gp = 0.0f, wp = 0.0f;
    // info sums over the raw ring: this step's entry, then the other four in
    // slot order (the entries being replaced are the loaded ones)
    double lsum = loss, gsum = g;
#pragma unroll
    for (int k = 0; k < kRawHist; ++k) {
        if (k == prev) {
            l_prev = hl_v[k];
            gp = hg_v[k];
            wp = hw_v[k];
        }
        if (k != slot) {
            lsum += hl_v[k];
            gsum += hg_v[k];
        }
    }
    const double adj_l = ratio_fast(loss, static_cast<float>(l_prev));
    const double adj_g = ratio_fast(g, gp);
    const double adj_w = ratio_fast(th, wp);
    // this step's entry in observation form, and its |.| sum (the order of
    // the float64 adds is the one states_sum has always used)
    const float nw = static_cast<float>(clip100(adj_w) - 1.0);
    const float nl = static_cast<float>(clip100(adj_l) - 1.0);
    const float ng = static_cast<float>(clip100(adj_g) - 1.0);
    const double nsum = fabs(adj_w) + fabs(adj_g) + fabs(adj_l);
    const int aslot = (s - 1) % H;

    // ---- reward v6 + termination (multioptlrs.py:102-107)
    double reward = 1.0 - adj_l;
    reward = reward < -100.0 ? -100.0 : (reward > 100.0 ? 100.0 : reward);
    bool terminal = s >= a.max_batches;
    if (!terminal && loss > 1e4f) {
        terminal = true;
        reward -= static_cast<double>(a.max_batches - s);
    }
    const bool wipe = terminal && a.auto_reset;

    // ---- observation row of agent i: [w~ (H, newest first) | l~ (H) | g~ (H)]
    const bool staged = HC || H <= kMultiStageH;
    const int span = 64 / G * P * row;       // floats of one wave's env block
    float *lds = stage + wave * span;
    float *const lrow = lds + ((lane / G) * P + r) * row;
    float *dst = HC ? lrow : staged ? lrow : a.obs + (eu * P + r) * static_cast<unsigned>(row);
    // slot j holds the entry of age k = (s - 1 - j) mod H (age 0 = this
    // step's, written above); slots not written since the reset hold the
    // reset zeros in observation form (-1) with a zero |.| sum
    double st_abs = 0.0;
    // one runtime division by H: the ages step down from k0 = (s - 1) mod H
    const int k0 = aslot;
    auto put = [&](int j, float wk, float gk, float lk, double sk) {
        const int k = k0 - j >= 0 ? k0 - j : k0 - j + H;   // j < H
        if (k == 0) {
            wk = nw;
            gk = ng;
            lk = nl;
            sk = nsum;
        }
        st_abs += sk;
        if (on) {
            dst[k] = wipe ? -1.0f : wk;
            dst[H + k] = wipe ? -1.0f : lk;
            dst[2 * H + k] = wipe ? -1.0f : gk;
        }
    };
#pragma unroll
    for (int j = 0; j < kMultiStageH; ++j)
        if (j < H) put(j, ow_v[j], og_v[j], ol_v[j], sa_v[j]);
    for (int j = kMultiStageH; j < H; ++j)       // long histories: loaded here
        put(j, at32(a.ow, j * Eu * P + ep), at32(a.og, j * Eu * P + ep), at32(a.ol, j * Eu + eu),
            at32(a.sa, j * Eu * P + ep));
    // every loaded value is consumed (the rows staged, st_abs formed) before
    // the first store: vmcnt counts stores too, so a load consumed after a
    // store would wait for that store's completion
    asm volatile("" ::"v"(st_abs) : "memory");
    // this step's raw-history and adjusted-history entries
    if (on) {
        at32(a.hg, slot * Eu * P + ep) = g;
        at32(a.hw, slot * Eu * P + ep) = th;
        at32(a.og, aslot * Eu * P + ep) = ng;
        at32(a.ow, aslot * Eu * P + ep) = nw;
        at32(a.sa, aslot * Eu * P + ep) = nsum;
        if (i == 0) {
            at32(a.hl, slot * Eu + eu) = loss;
            at32(a.ol, aslot * Eu + eu) = nl;
        }
    }
    if (staged) {
        // the wave's rows are obs[e_first * P * row ...] contiguous
        __syncthreads();                        // every thread gets here (no early exit)
        const size_t e_first = (static_cast<size_t>(blockIdx.x) * kMultiBlock + wave * 64) / G;
        const size_t envs = e_first < E ? (E - e_first < static_cast<size_t>(64 / G)
                                               ? E - e_first : static_cast<size_t>(64 / G))
                                        : 0;
        const int n = static_cast<int>(envs) * P * row;
        float *out = a.obs + e_first * P * row;
        // every LDS read of the block issued before its stores, 16 bytes a
        // lane (one dependent LDS round trip per stored float measured 15 x
        // ~100 cycles on the wave's critical path); the span is a multiple of
        // 16 bytes, an unaligned caller pointer or ragged block takes floats
        constexpr int kV = HC ? (64 / G * P * 3 * HC / 4 + 63) / 64 : 1;
        if (HC && (n & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
            const float4 *src = reinterpret_cast<const float4 *>(lds);
            float4 *dst4 = reinterpret_cast<float4 *>(out);
            const int n4 = n >> 2;
            float4 v[kV];
#pragma unroll
            for (int u = 0; u < kV; ++u) {                // clamped, branch-free reads
                const int q = lane + 64 * u;
                v[u] = src[q < n4 ? q : n4 - 1];
            }
#pragma unroll
            for (int u = 0; u < kV; ++u) {                // lanes past the block rewrite its
                const int q = lane + 64 * u;              // last 16 bytes with the same value
                dst4[q < n4 ? q : n4 - 1] = v[u];
            }
        } else {
            for (int q = lane; q < n; q += 64) out[q] = lds[q];
        }
    }

    // ---- info (multioptlrs.py:112-127), float64 group reductions
    const double mine = on ? 1.0 : 0.0;
    const double wsum = group_sum<G>(mine * fabs(static_cast<double>(th)));
    const double amean = group_sum<G>(mine * static_cast<double>(lr)) / P;
    const double dev = static_cast<double>(lr) - amean;
    const double avar = group_sum<G>(mine * dev * dev) / P;
    const double adjg = group_sum<G>(mine * fabs(adj_g)) / P;
    const double gdiff = group_sum<G>(mine * fabs(static_cast<double>(g) - static_cast<double>(gp))) / P;
    const double gsum_all = group_sum<G>(mine * gsum);
    const double st_all = group_sum<G>(mine * st_abs);
    if (on) {
        if (i == 0) {
            float *info = a.info + eu * kMultiInfo;
            info[0] = terminal ? loss : __builtin_nanf("");          // loss (None -> NaN)
            info[1] = loss;                                           // batch_loss
            info[2] = static_cast<float>(wsum / P);                   // weights_mean
            info[3] = static_cast<float>(wsum);                       // weights_sum
            info[4] = static_cast<float>(amean);                      // actions_mean
            info[5] = static_cast<float>(sqrt(avar));                 // actions_std
            info[6] = static_cast<float>(st_all / (P * row));         // states_mean
            info[7] = static_cast<float>(st_all);                     // states_sum
            info[8] = static_cast<float>(gsum_all / (kRawHist * P));  // grads_mean
            info[9] = static_cast<float>(gsum_all);                   // grads_sum
            info[10] = static_cast<float>(lsum / kRawHist);           // loss_mean
            info[11] = static_cast<float>(adj_l);                     // adjusted_loss
            info[12] = static_cast<float>(adjg);                      // adjusted_grad
            info[13] = static_cast<float>(gdiff);                     // grad_diff
            at32(a.episode_len, eu) = s;
        }
        at32(a.reward, eu * P + r) = static_cast<float>(reward);
        at32(a.done, eu * P + r) = terminal ? 1 : 0;
    }

    if (wipe && on) {
        multi_store_reset<P>(a, e, i, th_init, g_init, l_init);
    } else if (on) {
        at32(a.theta, ep) = th;
        at32(a.grad, ep) = g;
        if (i == 0) at32(a.step, eu) = s;
    }
}

}  // namespace ce

namespace ce {

// ---------------------------------------------------------------------------
// K consecutive MultiOptLRs-v0 steps in ONE launch (the reference default
// history HC = 5): ce_multi_step_many_strided / ce_multi_step_many.
//
// An env's whole state -- theta, the gradient, the 5-entry raw ring (loss,
// g, w) and the H-entry adjusted ring in observation form with its |.| sums
// -- is a few dozen values per lane: it is loaded once, lives in VGPRs for
// the K steps (ring slots indexed by the same physical positions
// multi_step_kernel uses, so every sum runs in the same order) and is stored
// once.  Per step a wave reads only its actions (prefetched a step ahead)
// and writes only the step's outputs into output record t (out_step bytes
// apart; 0 = every step into the same record), so the launch floor, the
// state round trip and the ring traffic of K one-step launches are paid
// once.  The arithmetic is multi_step_kernel's, operation for operation
// (tests/test_gpu_multi.py checks the bits against it).
template <int P, int HC>
__global__ __launch_bounds__(kMultiBlock) void multi_persist_kernel(MultiArgs a, int K, long long act_stride,
                                                                   long long out_step) {
#pragma clang fp contract(off)
    constexpr int G = Group<P>::G;
    constexpr int H = HC;
    constexpr int row = 3 * H;
    static_assert(HC > 0 && HC <= kMultiStageH, "compile-time history");
    extern __shared__ float4 stage4[];
    float *stage = reinterpret_cast<float *>(stage4);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t gt = static_cast<size_t>(blockIdx.x) * kMultiBlock + threadIdx.x;
    const size_t e = gt / G;
    const int i = static_cast<int>(gt % G);
    const size_t E = a.E;
    const bool env_ok = e < E;
    const bool on = env_ok && i < P;
    const size_t ec = env_ok ? e : 0;
    const int ic = i < P ? i : 0;
    const int r = P <= 10 ? ic : a.agent_row[ic];
    const unsigned Eu = static_cast<unsigned>(E), eu = static_cast<unsigned>(ec);
    const unsigned ep = eu * P + ic;

    // ---- the state, once
    int s_prev = at32(a.step, eu);
    float act = at32(a.act, eu * P + r);
    const float th_init = i < P ? a.init[i] : 0.0f;
    const float g_init = i < P ? a.init_g[i] : 0.0f, l_init = a.init_l;
    float th = at32(a.theta, ep);
    float gc = at32(a.grad, ep);
    float hl_v[kRawHist], hg_v[kRawHist], hw_v[kRawHist];
#pragma unroll
    for (int k = 0; k < kRawHist; ++k) {
        hl_v[k] = at32(a.hl, k * Eu + eu);
        hg_v[k] = at32(a.hg, k * Eu * P + ep);
        hw_v[k] = at32(a.hw, k * Eu * P + ep);
    }
    float ol_v[H], og_v[H], ow_v[H];
    double sa_v[H];
#pragma unroll
    for (int j = 0; j < H; ++j) {
        ol_v[j] = at32(a.ol, j * Eu + eu);
        og_v[j] = at32(a.og, j * Eu * P + ep);
        ow_v[j] = at32(a.ow, j * Eu * P + ep);
        sa_v[j] = at32(a.sa, j * Eu * P + ep);
    }
    const int span = 64 / G * P * row;       // floats of one wave's env block
    float *lds = stage + wave * span;
    float *const lrow = lds + ((lane / G) * P + r) * row;
    const size_t e_first = (static_cast<size_t>(blockIdx.x) * kMultiBlock + wave * 64) / G;
    const size_t envs = e_first < E ? (E - e_first < static_cast<size_t>(64 / G) ? E - e_first
                                                                                  : static_cast<size_t>(64 / G))
                                    : 0;
    const int nblk = static_cast<int>(envs) * P * row;

    for (int t = 0; t < K; ++t) {
        // step t + 1's action, consumed at the end of this step
        const float act_next = at32(a.act + (t + 1 < K ? (t + 1) * act_stride : 0), eu * P + r);
        const long long ro = t * out_step;     // this step's output record, bytes past record 0
        const int s = s_prev + 1;
        // ---- update (multioptlrs.py:81-87), lr = 10^(a - 4)
        const float x = act - 4.0f;
        const float lr = static_cast<float>(exp10(static_cast<double>(x)));
        const float thn = th - gc * lr;
        float g, loss;
        rosenbrock_lane<P>(thn, i, g, loss);
        // ---- raw history append, observation v3 against the previous entry
        const int slot = s % kRawHist, prev = (s - 1) % kRawHist;
        double l_prev = 0.0;
        float gp = 0.0f, wp = 0.0f;
        double lsum = loss, gsum = g;
#pragma unroll
        for (int k = 0; k < kRawHist; ++k) {
            if (k == prev) {
                l_prev = hl_v[k];
                gp = hg_v[k];
                wp = hw_v[k];
            }
            if (k != slot) {
                lsum += hl_v[k];
                gsum += hg_v[k];
            }
        }
        const double adj_l = ratio_fast(loss, static_cast<float>(l_prev));
        const double adj_g = ratio_fast(g, gp);
        const double adj_w = ratio_fast(thn, wp);
        const float nw = static_cast<float>(clip100(adj_w) - 1.0);
        const float nl = static_cast<float>(clip100(adj_l) - 1.0);
        const float ng = static_cast<float>(clip100(adj_g) - 1.0);
        const double nsum = fabs(adj_w) + fabs(adj_g) + fabs(adj_l);
        const int aslot = (s - 1) % H;
        // ---- reward v6 + termination (multioptlrs.py:102-107)
        double reward = 1.0 - adj_l;
        reward = reward < -100.0 ? -100.0 : (reward > 100.0 ? 100.0 : reward);
        bool terminal = s >= a.max_batches;
        if (!terminal && loss > 1e4f) {
            terminal = true;
            reward -= static_cast<double>(a.max_batches - s);
        }
        const bool wipe = terminal && a.auto_reset;
        // ---- observation row: [w~ (H, newest first) | l~ (H) | g~ (H)]
        double st_abs = 0.0;
        const int k0 = aslot;
#pragma unroll
        for (int j = 0; j < H; ++j) {
            const int kk = k0 - j >= 0 ? k0 - j : k0 - j + H;
            float wk = ow_v[j], gk = og_v[j], lk = ol_v[j];
            double sk = sa_v[j];
            if (kk == 0) {
                wk = nw;
                gk = ng;
                lk = nl;
                sk = nsum;
            }
            st_abs += sk;
            if (on) {
                lrow[kk] = wipe ? -1.0f : wk;
                lrow[H + kk] = wipe ? -1.0f : lk;
                lrow[2 * H + kk] = wipe ? -1.0f : gk;
            }
        }
        // the ring entries of this step, in registers
#pragma unroll
        for (int k = 0; k < kRawHist; ++k)
            if (k == slot) {
                hg_v[k] = g;
                hw_v[k] = thn;
                hl_v[k] = loss;
            }
#pragma unroll
        for (int j = 0; j < H; ++j)
            if (j == aslot) {
                og_v[j] = ng;
                ow_v[j] = nw;
                sa_v[j] = nsum;
                ol_v[j] = nl;
            }
        // the wave's staged rows -> record t (one wave per workgroup: the LDS
        // block is the wave's own, in-order within the wave)
        __builtin_amdgcn_wave_barrier();
        {
            float *out = reinterpret_cast<float *>(reinterpret_cast<char *>(a.obs) + ro) + e_first * P * row;
            constexpr int kV = (64 / G * P * 3 * HC / 4 + 63) / 64;
            if ((nblk & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
                const float4 *src = reinterpret_cast<const float4 *>(lds);
                float4 *dst4 = reinterpret_cast<float4 *>(out);
                const int n4 = nblk >> 2;
                float4 v[kV];
#pragma unroll
                for (int u = 0; u < kV; ++u) {
                    const int q = lane + 64 * u;
                    v[u] = src[q < n4 ? q : n4 - 1];
                }
#pragma unroll
                for (int u = 0; u < kV; ++u) {
                    const int q = lane + 64 * u;
                    if (q < n4) dst4[q] = v[u];
                }
            } else {
                for (int q = lane; q < nblk; q += 64) out[q] = lds[q];
            }
        }
        __builtin_amdgcn_wave_barrier();
        // ---- info (multioptlrs.py:112-127), float64 group reductions.  An
        // idle lane (agent i >= P of a group) carries its own values across
        // the K steps, which may overflow: it contributes by a select, not by
        // multiplying with 0 (the one-step kernel's `mine *`, identical for
        // every finite value)
        auto mine = [&](double v) { return on ? v : 0.0; };
        const double wsum = group_sum<G>(mine(fabs(static_cast<double>(thn))));
        const double amean = group_sum<G>(mine(static_cast<double>(lr))) / P;
        const double dev = static_cast<double>(lr) - amean;
        const double avar = group_sum<G>(mine(dev * dev)) / P;
        const double adjg = group_sum<G>(mine(fabs(adj_g))) / P;
        const double gdiff = group_sum<G>(mine(fabs(static_cast<double>(g) - static_cast<double>(gp)))) / P;
        const double gsum_all = group_sum<G>(mine(gsum));
        const double st_all = group_sum<G>(mine(st_abs));
        if (on) {
            if (i == 0) {
                float *info = reinterpret_cast<float *>(reinterpret_cast<char *>(a.info) + ro) + eu * kMultiInfo;
                info[0] = terminal ? loss : __builtin_nanf("");
                info[1] = loss;
                info[2] = static_cast<float>(wsum / P);
                info[3] = static_cast<float>(wsum);
                info[4] = static_cast<float>(amean);
                info[5] = static_cast<float>(sqrt(avar));
                info[6] = static_cast<float>(st_all / (P * row));
                info[7] = static_cast<float>(st_all);
                info[8] = static_cast<float>(gsum_all / (kRawHist * P));
                info[9] = static_cast<float>(gsum_all);
                info[10] = static_cast<float>(lsum / kRawHist);
                info[11] = static_cast<float>(adj_l);
                info[12] = static_cast<float>(adjg);
                info[13] = static_cast<float>(gdiff);
                at32(reinterpret_cast<int32_t *>(reinterpret_cast<char *>(a.episode_len) + ro), eu) = s;
            }
            at32(reinterpret_cast<float *>(reinterpret_cast<char *>(a.reward) + ro), eu * P + r) =
                static_cast<float>(reward);
            at32(reinterpret_cast<uint8_t *>(a.done) + ro, eu * P + r) = terminal ? 1 : 0;
        }
        // ---- the next step's state: the auto-reset's (multi_store_reset) or this one
        if (wipe) {
#pragma unroll
            for (int k = 0; k < kRawHist; ++k) {
                hg_v[k] = k == 0 ? g_init : 0.0f;
                hw_v[k] = k == 0 ? th_init : 0.0f;
                hl_v[k] = k == 0 ? l_init : 0.0f;
            }
#pragma unroll
            for (int j = 0; j < H; ++j) {
                og_v[j] = -1.0f;
                ow_v[j] = -1.0f;
                ol_v[j] = -1.0f;
                sa_v[j] = 0.0;
            }
            th = th_init;
            gc = g_init;
            s_prev = 0;
        } else {
            th = thn;
            gc = g;
            s_prev = s;
        }
        act = act_next;
    }
    // ---- the state after K steps, once
    if (on) {
        at32(a.theta, ep) = th;
        at32(a.grad, ep) = gc;
#pragma unroll
        for (int k = 0; k < kRawHist; ++k) {
            at32(a.hg, k * Eu * P + ep) = hg_v[k];
            at32(a.hw, k * Eu * P + ep) = hw_v[k];
            if (i == 0) at32(a.hl, k * Eu + eu) = hl_v[k];
        }
#pragma unroll
        for (int j = 0; j < H; ++j) {
            at32(a.og, j * Eu * P + ep) = og_v[j];
            at32(a.ow, j * Eu * P + ep) = ow_v[j];
            at32(a.sa, j * Eu * P + ep) = sa_v[j];
            if (i == 0) at32(a.ol, j * Eu + eu) = ol_v[j];
        }
        if (i == 0) at32(a.step, eu) = s_prev;
    }
}

}  // namespace ce

namespace ce {

// The split form of multi_persist_kernel (multi_persist2_kernel): the same
// 64 / G envs per workgroup, their lanes mirrored in THREE waves on three
// SIMDs.  The STATE wave runs the loop-carried chain only: the update, the
// Rosenbrock pair, the raw history and the three observation ratios.  Two
// waves take what no later step of that chain reads: the ROWS wave keeps the
// adjusted history rings' observation columns and writes the observation
// rows (staged in its own LDS rows, copied out as float4 lines); the INFO
// wave keeps the |.| sums ring and writes the fourteen info values, reward,
// done and length.  Measured per 1024-env step (profiles/r05aa_*, r05v_*):
// one wave ≈1.7 us (latency-bound on the sum); state + one output wave that
// also took the rings 1.21 us, bound by the state wave; rings moved to that
// output wave 1.34 us, bound by it; three waves 0.82 us.  The per-lane
// hand-over (the new ratios and the scalars the outputs need) is
// double-buffered by step parity behind one 192-thread barrier per step.
// Same arithmetic, same operation order as multi_persist_kernel:
// bit-identical outputs.
// Diagnostic builds only (timing which wave bounds the step; outputs wrong):
// bit 0 skips the info wave's work, bit 1 the rows wave's, bit 2 replaces
// the state wave's exp10 by a copy (three-wave form), bit 3 skips the ratio
// wave's work (four-wave form).
#ifndef CE_MP2_DIAG
#define CE_MP2_DIAG 0
#endif
struct MultiXch {
    double adj_g, adj_l, gsum, lsum, nsum, reward;
    float thn, lr, g, gp, loss, nw, nl, ng;
    int s, terminal;
};

template <int P, int HC>
__global__ __launch_bounds__(192) void multi_persist2_kernel(MultiArgs a, int K, long long act_stride,
                                                            long long out_step) {
#pragma clang fp contract(off)
    constexpr int G = Group<P>::G;
    constexpr int H = HC;
    constexpr int row = 3 * H;
    static_assert(HC > 0 && HC <= kMultiStageH, "compile-time history");
    constexpr int span = 64 / G * P * row;                  // floats of the workgroup's env block
    __shared__ __attribute__((aligned(16))) float stage[span];   // the output wave's rows
    __shared__ MultiXch xch[2][64];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t gt = static_cast<size_t>(blockIdx.x) * 64 + lane;   // the lane's (env, agent)
    const size_t e = gt / G;
    const int i = static_cast<int>(gt % G);
    const size_t E = a.E;
    const bool env_ok = e < E;
    const bool on = env_ok && i < P;
    const size_t ec = env_ok ? e : 0;
    const int ic = i < P ? i : 0;
    const int r = P <= 10 ? ic : a.agent_row[ic];
    const unsigned Eu = static_cast<unsigned>(E), eu = static_cast<unsigned>(ec);
    const unsigned ep = eu * P + ic;
    const size_t e_first = static_cast<size_t>(blockIdx.x) * 64 / G;
    const size_t envs = e_first < E ? (E - e_first < static_cast<size_t>(64 / G) ? E - e_first
                                                                                  : static_cast<size_t>(64 / G))
                                    : 0;
    const int nblk = static_cast<int>(envs) * P * row;

    if (wave == 0) {
        // ======================= state wave =======================
        int s_prev = at32(a.step, eu);
        float act = at32(a.act, eu * P + r);
        const float th_init = i < P ? a.init[i] : 0.0f;
        const float g_init = i < P ? a.init_g[i] : 0.0f, l_init = a.init_l;
        float th = at32(a.theta, ep);
        float gc = at32(a.grad, ep);
        float hl_v[kRawHist], hg_v[kRawHist], hw_v[kRawHist];
#pragma unroll
        for (int k = 0; k < kRawHist; ++k) {
            hl_v[k] = at32(a.hl, k * Eu + eu);
            hg_v[k] = at32(a.hg, k * Eu * P + ep);
            hw_v[k] = at32(a.hw, k * Eu * P + ep);
        }
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            const float act_next = at32(a.act + (t + 1 < K ? (t + 1) * act_stride : 0), eu * P + r);
            const int s = s_prev + 1;
            const float x = act - 4.0f;
            const float lr = (CE_MP2_DIAG & 4) ? x : static_cast<float>(exp10(static_cast<double>(x)));
            const float thn = th - gc * lr;
            float g, loss;
            rosenbrock_lane<P>(thn, i, g, loss);
            const int slot = s % kRawHist, prev = (s - 1) % kRawHist;
            double l_prev = 0.0;
            float gp = 0.0f, wp = 0.0f;
            double lsum = loss, gsum = g;
#pragma unroll
            for (int k = 0; k < kRawHist; ++k) {
                if (k == prev) {
                    l_prev = hl_v[k];
                    gp = hg_v[k];
                    wp = hw_v[k];
                }
                if (k != slot) {
                    lsum += hl_v[k];
                    gsum += hg_v[k];
                }
            }
            const double adj_l = ratio_fast(loss, static_cast<float>(l_prev));
            const double adj_g = ratio_fast(g, gp);
            const double adj_w = ratio_fast(thn, wp);
            const float nw = static_cast<float>(clip100(adj_w) - 1.0);
            const float nl = static_cast<float>(clip100(adj_l) - 1.0);
            const float ng = static_cast<float>(clip100(adj_g) - 1.0);
            const double nsum = fabs(adj_w) + fabs(adj_g) + fabs(adj_l);
            double reward = 1.0 - adj_l;
            reward = reward < -100.0 ? -100.0 : (reward > 100.0 ? 100.0 : reward);
            bool terminal = s >= a.max_batches;
            if (!terminal && loss > 1e4f) {
                terminal = true;
                reward -= static_cast<double>(a.max_batches - s);
            }
            const bool wipe = terminal && a.auto_reset;
            MultiXch &xo = xch[buf][lane];
            xo.adj_g = adj_g;
            xo.adj_l = adj_l;
            xo.gsum = gsum;
            xo.lsum = lsum;
            xo.nsum = nsum;
            xo.reward = reward;
            xo.thn = thn;
            xo.lr = lr;
            xo.g = g;
            xo.gp = gp;
            xo.loss = loss;
            xo.nw = nw;
            xo.nl = nl;
            xo.ng = ng;
            xo.s = s;
            xo.terminal = terminal ? 1 : 0;
#pragma unroll
            for (int k = 0; k < kRawHist; ++k)
                if (k == slot) {
                    hg_v[k] = g;
                    hw_v[k] = thn;
                    hl_v[k] = loss;
                }
            if (wipe) {
#pragma unroll
                for (int k = 0; k < kRawHist; ++k) {
                    hg_v[k] = k == 0 ? g_init : 0.0f;
                    hw_v[k] = k == 0 ? th_init : 0.0f;
                    hl_v[k] = k == 0 ? l_init : 0.0f;
                }
                th = th_init;
                gc = g_init;
                s_prev = 0;
            } else {
                th = thn;
                gc = g;
                s_prev = s;
            }
            act = act_next;
            __syncthreads();                                // step t's results -> the output wave
        }
        if (on) {
            at32(a.theta, ep) = th;
            at32(a.grad, ep) = gc;
#pragma unroll
            for (int k = 0; k < kRawHist; ++k) {
                at32(a.hg, k * Eu * P + ep) = hg_v[k];
                at32(a.hw, k * Eu * P + ep) = hw_v[k];
                if (i == 0) at32(a.hl, k * Eu + eu) = hl_v[k];
            }
            if (i == 0) at32(a.step, eu) = s_prev;
        }
    } else if (wave == 1) {
        // ===================== rows wave =====================
        // the adjusted rings' observation columns and the rows
        float ol_v[H], og_v[H], ow_v[H];
#pragma unroll
        for (int j = 0; j < H; ++j) {
            ol_v[j] = at32(a.ol, j * Eu + eu);
            og_v[j] = at32(a.og, j * Eu * P + ep);
            ow_v[j] = at32(a.ow, j * Eu * P + ep);
        }
        float *const lrow = stage + ((lane / G) * P + r) * row;
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // step t's results handed over
            const long long ro = t * out_step;
            const MultiXch &xi = xch[buf][lane];
            if (CE_MP2_DIAG & 2) continue;
            const int s = xi.s;
            const bool wipe = xi.terminal != 0 && a.auto_reset;
            const float nw = xi.nw, ng = xi.ng, nl = xi.nl;
            const int aslot = (s - 1) % H;
            const int k0 = aslot;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int kk = k0 - j >= 0 ? k0 - j : k0 - j + H;
                float wk = ow_v[j], gk = og_v[j], lk = ol_v[j];
                if (kk == 0) {
                    wk = nw;
                    gk = ng;
                    lk = nl;
                }
                if (on) {
                    lrow[kk] = wipe ? -1.0f : wk;
                    lrow[H + kk] = wipe ? -1.0f : lk;
                    lrow[2 * H + kk] = wipe ? -1.0f : gk;
                }
            }
#pragma unroll
            for (int j = 0; j < H; ++j)
                if (j == aslot) {
                    og_v[j] = ng;
                    ow_v[j] = nw;
                    ol_v[j] = nl;
                }
            if (wipe) {
#pragma unroll
                for (int j = 0; j < H; ++j) {
                    og_v[j] = -1.0f;
                    ow_v[j] = -1.0f;
                    ol_v[j] = -1.0f;
                }
            }
            // the wave's own rows (in-order LDS within a wave), copied out in
            // line order
            __builtin_amdgcn_wave_barrier();
            {
                const float *lds = stage;
                float *out = reinterpret_cast<float *>(reinterpret_cast<char *>(a.obs) + ro) + e_first * P * row;
                constexpr int kV = (span / 4 + 63) / 64;
                if ((nblk & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
                    const float4 *src = reinterpret_cast<const float4 *>(lds);
                    float4 *dst4 = reinterpret_cast<float4 *>(out);
                    const int n4 = nblk >> 2;
                    float4 v[kV];
#pragma unroll
                    for (int u = 0; u < kV; ++u) {
                        const int q = lane + 64 * u;
                        v[u] = src[q < n4 ? q : n4 - 1];
                    }
#pragma unroll
                    for (int u = 0; u < kV; ++u) {
                        const int q = lane + 64 * u;
                        if (q < n4) dst4[q] = v[u];
                    }
                } else {
                    for (int q = lane; q < nblk; q += 64) out[q] = lds[q];
                }
            }
            __builtin_amdgcn_wave_barrier();                // rows read before the next step rewrites them
        }
        if (on) {
#pragma unroll
            for (int j = 0; j < H; ++j) {
                at32(a.og, j * Eu * P + ep) = og_v[j];
                at32(a.ow, j * Eu * P + ep) = ow_v[j];
                if (i == 0) at32(a.ol, j * Eu + eu) = ol_v[j];
            }
        }
    } else {
        // ===================== info wave =====================
        // the |.| sums ring, the fourteen info values, reward / done / length
        double sa_v[H];
#pragma unroll
        for (int j = 0; j < H; ++j) sa_v[j] = at32(a.sa, j * Eu * P + ep);
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // step t's results handed over
            const long long ro = t * out_step;
            const MultiXch xi = xch[buf][lane];
            if (CE_MP2_DIAG & 1) continue;
            const int s = xi.s;
            const bool terminal = xi.terminal != 0;
            const bool wipe = terminal && a.auto_reset;
            const int aslot = (s - 1) % H;
            double st_abs = 0.0;
            const int k0 = aslot;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int kk = k0 - j >= 0 ? k0 - j : k0 - j + H;
                st_abs += kk == 0 ? xi.nsum : sa_v[j];
            }
#pragma unroll
            for (int j = 0; j < H; ++j)
                if (j == aslot) sa_v[j] = xi.nsum;
            if (wipe) {
#pragma unroll
                for (int j = 0; j < H; ++j) sa_v[j] = 0.0;
            }
            const double thn = xi.thn, lr = xi.lr;
            auto mine = [&](double v) { return on ? v : 0.0; };
            const double wsum = group_sum<G>(mine(fabs(thn)));
            const double amean = group_sum<G>(mine(lr)) / P;
            const double dev = lr - amean;
            const double avar = group_sum<G>(mine(dev * dev)) / P;
            const double adjg = group_sum<G>(mine(fabs(xi.adj_g))) / P;
            const double gdiff = group_sum<G>(mine(fabs(static_cast<double>(xi.g) - static_cast<double>(xi.gp)))) / P;
            const double gsum_all = group_sum<G>(mine(xi.gsum));
            const double st_all = group_sum<G>(mine(st_abs));
            if (on) {
                if (i == 0) {
                    float *info = reinterpret_cast<float *>(reinterpret_cast<char *>(a.info) + ro) + eu * kMultiInfo;
                    info[0] = terminal ? xi.loss : __builtin_nanf("");
                    info[1] = xi.loss;
                    info[2] = static_cast<float>(wsum / P);
                    info[3] = static_cast<float>(wsum);
                    info[4] = static_cast<float>(amean);
                    info[5] = static_cast<float>(sqrt(avar));
                    info[6] = static_cast<float>(st_all / (P * row));
                    info[7] = static_cast<float>(st_all);
                    info[8] = static_cast<float>(gsum_all / (kRawHist * P));
                    info[9] = static_cast<float>(gsum_all);
                    info[10] = static_cast<float>(xi.lsum / kRawHist);
                    info[11] = static_cast<float>(xi.adj_l);
                    info[12] = static_cast<float>(adjg);
                    info[13] = static_cast<float>(gdiff);
                    at32(reinterpret_cast<int32_t *>(reinterpret_cast<char *>(a.episode_len) + ro), eu) = xi.s;
                }
                at32(reinterpret_cast<float *>(reinterpret_cast<char *>(a.reward) + ro), eu * P + r) =
                    static_cast<float>(xi.reward);
                at32(reinterpret_cast<uint8_t *>(a.done) + ro, eu * P + r) = terminal ? 1 : 0;
            }
        }
        if (on) {
#pragma unroll
            for (int j = 0; j < H; ++j) at32(a.sa, j * Eu * P + ep) = sa_v[j];
        }
    }
}


// The four-wave form (multi_persist4_kernel): multi_persist2_kernel's state
// wave issued ≈380 instructions per step and bounded the step (its outputs'
// work: the three ratios, reward, sums).  Here a fourth wave, on the fourth
// SIMD, takes the ratios, the reward, the |.| sum and the info values of its
// own operands (two of the seven group sums); the state wave keeps the
// loop-carried chain (the update, the Rosenbrock pair), the raw history, its
// sums' info values and the exp10 of the next step's action, which fill its
// chain's latency.  The rows wave holds its rings newest first (a shift
// register), so the rows are written at constant LDS offsets.  One
// 256-thread barrier per step; every hand-over is double-buffered by step
// parity:
//   state  (W0) step t between barriers t-1 and t: raw[t] out
//   ratio  (W3) step t between barriers t and t+1: raw[t] in, xch[t] out
//   rows / info (W1, W2) step t between barriers t+1 and t+2: xch[t] in
// The arithmetic and its order are multi_persist_kernel's: bit-identical
// outputs.
struct MultiXch4 {       // what the rows and info waves take from the ratio wave
    double nsum;
    float thn, lr, loss, reward, nw, nl, ng;
    float info8, info9, info10, info11, info12, info13;
    int s, terminal;
};
struct MultiRaw {
    float thn, g, loss, lr, gp, wp, lp;
    float info8, info9, info10;
    int s, terminal;
};

template <int P, int HC>
__global__ __launch_bounds__(256) void multi_persist4_kernel(MultiArgs a, int K, long long act_stride,
                                                            long long out_step) {
#pragma clang fp contract(off)
    constexpr int G = Group<P>::G;
    constexpr int H = HC;
    constexpr int row = 3 * H;
    static_assert(HC > 0 && HC <= kMultiStageH, "compile-time history");
    constexpr int span = 64 / G * P * row;
    __shared__ __attribute__((aligned(16))) float stage[span];
    __shared__ MultiXch4 xch[2][64];
    __shared__ MultiRaw raw[2][64];
    // (the wave index made wave-uniform by readfirstlane measured 2 % slower)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t gt = static_cast<size_t>(blockIdx.x) * 64 + lane;
    const size_t e = gt / G;
    const int i = static_cast<int>(gt % G);
    const size_t E = a.E;
    const bool env_ok = e < E;
    const bool on = env_ok && i < P;
    const size_t ec = env_ok ? e : 0;
    const int ic = i < P ? i : 0;
    const int r = P <= 10 ? ic : a.agent_row[ic];
    const unsigned Eu = static_cast<unsigned>(E), eu = static_cast<unsigned>(ec);
    const unsigned ep = eu * P + ic;
    const size_t e_first = static_cast<size_t>(blockIdx.x) * 64 / G;
    const size_t envs = e_first < E ? (E - e_first < static_cast<size_t>(64 / G) ? E - e_first
                                                                                  : static_cast<size_t>(64 / G))
                                    : 0;
    const int nblk = static_cast<int>(envs) * P * row;

    if (wave == 0) {
        // ======================= state wave =======================
        int s_prev = at32(a.step, eu);
        const float th_init = i < P ? a.init[i] : 0.0f;
        const float g_init = i < P ? a.init_g[i] : 0.0f, l_init = a.init_l;
        float th = at32(a.theta, ep);
        float gc = at32(a.grad, ep);
        float hl_v[kRawHist], hg_v[kRawHist], hw_v[kRawHist];
#pragma unroll
        for (int k = 0; k < kRawHist; ++k) {
            hl_v[k] = at32(a.hl, k * Eu + eu);
            hg_v[k] = at32(a.hg, k * Eu * P + ep);
            hw_v[k] = at32(a.hw, k * Eu * P + ep);
        }
        // lr = 10^(a - 4) (multioptlrs.py:81-87): an action's lr depends on
        // the action alone, so step t + 1's is formed during step t
        float lr = static_cast<float>(exp10(static_cast<double>(at32(a.act, eu * P + r) - 4.0f)));
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            const float act_next = at32(a.act + (t + 1 < K ? (t + 1) * act_stride : 0), eu * P + r);
            const int s = s_prev + 1;
            const float thn = th - gc * lr;
            float g, loss;
            rosenbrock_lane<P>(thn, i, g, loss);
            bool terminal = s >= a.max_batches;
            if (!terminal && loss > 1e4f) terminal = true;
            const int slot = s % kRawHist, prev = (s - 1) % kRawHist;
            float lp = 0.0f, gp = 0.0f, wp = 0.0f;
            double lsum = loss, gsum = g;
#pragma unroll
            for (int k = 0; k < kRawHist; ++k) {
                if (k == prev) {
                    lp = hl_v[k];
                    gp = hg_v[k];
                    wp = hw_v[k];
                }
                if (k != slot) {
                    lsum += hl_v[k];
                    gsum += hg_v[k];
                }
            }
            // the raw sums' info values (the state wave has the slack)
            const double gsum_all = group_sum<G>(on ? gsum : 0.0);
            MultiRaw &ro = raw[buf][lane];
            ro.info8 = static_cast<float>(gsum_all / (kRawHist * P));
            ro.info9 = static_cast<float>(gsum_all);
            ro.info10 = static_cast<float>(lsum / kRawHist);
            ro.thn = thn;
            ro.g = g;
            ro.loss = loss;
            ro.lr = lr;
            ro.gp = gp;
            ro.wp = wp;
            ro.lp = lp;
            ro.s = s;
            ro.terminal = terminal ? 1 : 0;
#pragma unroll
            for (int k = 0; k < kRawHist; ++k)
                if (k == slot) {
                    hg_v[k] = g;
                    hw_v[k] = thn;
                    hl_v[k] = loss;
                }
            if (terminal && a.auto_reset) {
#pragma unroll
                for (int k = 0; k < kRawHist; ++k) {
                    hg_v[k] = k == 0 ? g_init : 0.0f;
                    hw_v[k] = k == 0 ? th_init : 0.0f;
                    hl_v[k] = k == 0 ? l_init : 0.0f;
                }
                th = th_init;
                gc = g_init;
                s_prev = 0;
            } else {
                th = thn;
                gc = g;
                s_prev = s;
            }
            lr = static_cast<float>(exp10(static_cast<double>(act_next - 4.0f)));
            __syncthreads();                                // barrier t: raw[t] out
        }
        __syncthreads();                                    // barrier K
        if (on) {
            at32(a.theta, ep) = th;
            at32(a.grad, ep) = gc;
#pragma unroll
            for (int k = 0; k < kRawHist; ++k) {
                at32(a.hg, k * Eu * P + ep) = hg_v[k];
                at32(a.hw, k * Eu * P + ep) = hw_v[k];
                if (i == 0) at32(a.hl, k * Eu + eu) = hl_v[k];
            }
            if (i == 0) at32(a.step, eu) = s_prev;
        }
    } else if (wave == 3) {
        // ======================= ratio wave =======================
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // barrier t: raw[t] in
            if (CE_MP2_DIAG & 8) continue;
            const MultiRaw ri = raw[buf][lane];
            const int s = ri.s;
            const double adj_l = ratio_fast(ri.loss, ri.lp);
            const double adj_g = ratio_fast(ri.g, ri.gp);
            const double adj_w = ratio_fast(ri.thn, ri.wp);
            double reward = 1.0 - adj_l;
            reward = reward < -100.0 ? -100.0 : (reward > 100.0 ? 100.0 : reward);
            if (!(s >= a.max_batches) && ri.loss > 1e4f) reward -= static_cast<double>(a.max_batches - s);
            // the info values of the ratio wave's own operands (the group sums
            // of multi_persist_kernel, same butterfly)
            auto mine = [&](double v) { return on ? v : 0.0; };
            const double adjg = group_sum<G>(mine(fabs(adj_g))) / P;
            const double gdiff = group_sum<G>(mine(fabs(static_cast<double>(ri.g) - static_cast<double>(ri.gp)))) / P;
            MultiXch4 &xo = xch[buf][lane];
            xo.nsum = fabs(adj_w) + fabs(adj_g) + fabs(adj_l);
            xo.thn = ri.thn;
            xo.lr = ri.lr;
            xo.loss = ri.loss;
            xo.reward = static_cast<float>(reward);
            xo.nw = static_cast<float>(clip100(adj_w) - 1.0);
            xo.nl = static_cast<float>(clip100(adj_l) - 1.0);
            xo.ng = static_cast<float>(clip100(adj_g) - 1.0);
            xo.info8 = ri.info8;
            xo.info9 = ri.info9;
            xo.info10 = ri.info10;
            xo.info11 = static_cast<float>(adj_l);
            xo.info12 = static_cast<float>(adjg);
            xo.info13 = static_cast<float>(gdiff);
            xo.s = s;
            xo.terminal = ri.terminal;
        }
        __syncthreads();                                    // barrier K
    } else if (wave == 1) {
        // ======================= rows wave =======================
        // The adjusted rings' observation columns, held newest first (a
        // shift register: the row is the ring as it stands, written at
        // constant LDS offsets).  In HBM they stay in slot order, slot
        // (s - 1) % H the newest, as the one-step kernel keeps them.
        const int s0 = at32(a.step, eu);
        const int new0 = ((s0 - 1) % H + H) % H;
        float ol_v[H], og_v[H], ow_v[H];
#pragma unroll
        for (int q = 0; q < H; ++q) {
            const int j = (new0 - q + H) % H;
            ol_v[q] = at32(a.ol, j * Eu + eu);
            og_v[q] = at32(a.og, j * Eu * P + ep);
            ow_v[q] = at32(a.ow, j * Eu * P + ep);
        }
        float *const lrow = stage + ((lane / G) * P + r) * row;
        int s_end = s0;
        __syncthreads();                                    // barrier 0
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // barrier t + 1: xch[t] in
            const long long ro = t * out_step;
            const MultiXch4 &xi = xch[buf][lane];
            if (CE_MP2_DIAG & 2) continue;
            const bool wipe = xi.terminal != 0 && a.auto_reset;
            const float nw = xi.nw, ng = xi.ng, nl = xi.nl;
            s_end = wipe ? 0 : xi.s;
#pragma unroll
            for (int q = H - 1; q > 0; --q) {
                og_v[q] = og_v[q - 1];
                ow_v[q] = ow_v[q - 1];
                ol_v[q] = ol_v[q - 1];
            }
            og_v[0] = ng;
            ow_v[0] = nw;
            ol_v[0] = nl;
            if (wipe) {
#pragma unroll
                for (int q = 0; q < H; ++q) {
                    og_v[q] = -1.0f;
                    ow_v[q] = -1.0f;
                    ol_v[q] = -1.0f;
                }
            }
            if (on) {
#pragma unroll
                for (int q = 0; q < H; ++q) {
                    lrow[q] = ow_v[q];
                    lrow[H + q] = ol_v[q];
                    lrow[2 * H + q] = og_v[q];
                }
            }
            __builtin_amdgcn_wave_barrier();
            {
                const float *lds = stage;
                float *out = reinterpret_cast<float *>(reinterpret_cast<char *>(a.obs) + ro) + e_first * P * row;
                constexpr int kV = (span / 4 + 63) / 64;
                if ((nblk & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
                    const float4 *src = reinterpret_cast<const float4 *>(lds);
                    float4 *dst4 = reinterpret_cast<float4 *>(out);
                    const int n4 = nblk >> 2;
                    float4 v[kV];
#pragma unroll
                    for (int u = 0; u < kV; ++u) {
                        const int q = lane + 64 * u;
                        v[u] = src[q < n4 ? q : n4 - 1];
                    }
#pragma unroll
                    for (int u = 0; u < kV; ++u) {
                        const int q = lane + 64 * u;
                        if (q < n4) dst4[q] = v[u];
                    }
                } else {
                    for (int q = lane; q < nblk; q += 64) out[q] = lds[q];
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (on) {
            const int new_end = ((s_end - 1) % H + H) % H;
#pragma unroll
            for (int q = 0; q < H; ++q) {
                const int j = (new_end - q + H) % H;
                at32(a.og, j * Eu * P + ep) = og_v[q];
                at32(a.ow, j * Eu * P + ep) = ow_v[q];
                if (i == 0) at32(a.ol, j * Eu + eu) = ol_v[q];
            }
        }
    } else {
        // ======================= info wave =======================
        double sa_v[H];
#pragma unroll
        for (int j = 0; j < H; ++j) sa_v[j] = at32(a.sa, j * Eu * P + ep);
        __syncthreads();                                    // barrier 0
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // barrier t + 1: xch[t] in
            const long long ro = t * out_step;
            const MultiXch4 xi = xch[buf][lane];
            if (CE_MP2_DIAG & 1) continue;
            const int s = xi.s;
            const bool terminal = xi.terminal != 0;
            const bool wipe = terminal && a.auto_reset;
            const int aslot = (s - 1) % H;
            double st_abs = 0.0;
            const int k0 = aslot;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int kk = k0 - j >= 0 ? k0 - j : k0 - j + H;
                st_abs += kk == 0 ? xi.nsum : sa_v[j];
            }
#pragma unroll
            for (int j = 0; j < H; ++j)
                if (j == aslot) sa_v[j] = xi.nsum;
            if (wipe) {
#pragma unroll
                for (int j = 0; j < H; ++j) sa_v[j] = 0.0;
            }
            const double lr = xi.lr;
            auto mine = [&](double v) { return on ? v : 0.0; };
            const double wsum = group_sum<G>(mine(fabs(static_cast<double>(xi.thn))));
            const double amean = group_sum<G>(mine(lr)) / P;
            const double dev = lr - amean;
            const double avar = group_sum<G>(mine(dev * dev)) / P;
            const double st_all = group_sum<G>(mine(st_abs));
            if (on) {
                if (i == 0) {
                    float *info = reinterpret_cast<float *>(reinterpret_cast<char *>(a.info) + ro) + eu * kMultiInfo;
                    info[0] = terminal ? xi.loss : __builtin_nanf("");
                    info[1] = xi.loss;
                    info[2] = static_cast<float>(wsum / P);
                    info[3] = static_cast<float>(wsum);
                    at32(reinterpret_cast<int32_t *>(reinterpret_cast<char *>(a.episode_len) + ro), eu) = xi.s;
                    info[4] = static_cast<float>(amean);
                    info[5] = static_cast<float>(sqrt(avar));
                    info[6] = static_cast<float>(st_all / (P * row));
                    info[7] = static_cast<float>(st_all);
                    info[8] = xi.info8;
                    info[9] = xi.info9;
                    info[10] = xi.info10;
                    info[11] = xi.info11;
                    info[12] = xi.info12;
                    info[13] = xi.info13;
                }
                at32(reinterpret_cast<float *>(reinterpret_cast<char *>(a.reward) + ro), eu * P + r) = xi.reward;
                at32(reinterpret_cast<uint8_t *>(a.done) + ro, eu * P + r) = terminal ? 1 : 0;
            }
        }
        if (on) {
#pragma unroll
            for (int j = 0; j < H; ++j) at32(a.sa, j * Eu * P + ep) = sa_v[j];
        }
    }
}

// The five-wave form (multi_persist5_kernel, the default; CE_MULTI_FORM=four
// runs the four-wave form): the four-wave state wave's raw history and sums
// move to a fifth wave (sharing SIMD 0 with the state wave), so the state
// wave issues only its chain (≈80 instructions per step): the update, the
// Rosenbrock pair, the terminal test and the next lr.  One more pipeline
// stage: state step t between barriers t-1 and t, sums between t and t+1,
// ratio between t+1 and t+2, rows / info between t+2 and t+3; K + 2
// barriers per launch.  Measured 0.59 -> 0.525 us per 1024-env step long
// run, 1.38 -> 1.30-1.32 in the driver form (profiles/r06q_*).
// The sums wave is wave 4 (with the state wave's SIMD if waves pair round
// robin); the rows wave there instead measured 0.530 against 0.525 us per
// step (profiles/r06s_*)
constexpr int kSumsWave = 4;
constexpr int kRowsWave = 1;
struct MultiRaw0 {       // what the sums wave takes from the state wave
    float thn, g, loss, lr;
    int s, terminal;
};

template <int P, int HC>
__global__ __launch_bounds__(320) void multi_persist5_kernel(MultiArgs a, int K, long long act_stride,
                                                            long long out_step) {
#pragma clang fp contract(off)
    constexpr int G = Group<P>::G;
    constexpr int H = HC;
    constexpr int row = 3 * H;
    static_assert(HC > 0 && HC <= kMultiStageH, "compile-time history");
    constexpr int span = 64 / G * P * row;
    __shared__ __attribute__((aligned(16))) float stage[span];
    __shared__ MultiXch4 xch[2][64];
    __shared__ MultiRaw raw[2][64];         // sums wave -> ratio wave
    __shared__ MultiRaw0 raw0[2][64];       // state wave -> sums wave
    // (the wave index made wave-uniform by readfirstlane measured 2 % slower)
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const size_t gt = static_cast<size_t>(blockIdx.x) * 64 + lane;
    const size_t e = gt / G;
    const int i = static_cast<int>(gt % G);
    const size_t E = a.E;
    const bool env_ok = e < E;
    const bool on = env_ok && i < P;
    const size_t ec = env_ok ? e : 0;
    const int ic = i < P ? i : 0;
    const int r = P <= 10 ? ic : a.agent_row[ic];
    const unsigned Eu = static_cast<unsigned>(E), eu = static_cast<unsigned>(ec);
    const unsigned ep = eu * P + ic;
    const size_t e_first = static_cast<size_t>(blockIdx.x) * 64 / G;
    const size_t envs = e_first < E ? (E - e_first < static_cast<size_t>(64 / G) ? E - e_first
                                                                                  : static_cast<size_t>(64 / G))
                                    : 0;
    const int nblk = static_cast<int>(envs) * P * row;

    if (wave == 0) {
        // ======================= state wave =======================
        // the loop-carried chain only: the update, the Rosenbrock pair, the
        // terminal test; lr of the next step's action beside it
        int s_prev = at32(a.step, eu);
        const float th_init = i < P ? a.init[i] : 0.0f;
        const float g_init = i < P ? a.init_g[i] : 0.0f;
        float th = at32(a.theta, ep);
        float gc = at32(a.grad, ep);
        float lr = static_cast<float>(exp10(static_cast<double>(at32(a.act, eu * P + r) - 4.0f)));
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            const float act_next = at32(a.act + (t + 1 < K ? (t + 1) * act_stride : 0), eu * P + r);
            const int s = s_prev + 1;
            const float thn = th - gc * lr;
            float g, loss;
            rosenbrock_lane<P>(thn, i, g, loss);
            bool terminal = s >= a.max_batches;
            if (!terminal && loss > 1e4f) terminal = true;
            MultiRaw0 &ro = raw0[buf][lane];
            ro.thn = thn;
            ro.g = g;
            ro.loss = loss;
            ro.lr = lr;
            ro.s = s;
            ro.terminal = terminal ? 1 : 0;
            if (terminal && a.auto_reset) {
                th = th_init;
                gc = g_init;
                s_prev = 0;
            } else {
                th = thn;
                gc = g;
                s_prev = s;
            }
            lr = static_cast<float>(exp10(static_cast<double>(act_next - 4.0f)));
            __syncthreads();                                // barrier t: raw0[t] out
        }
        __syncthreads();                                    // barrier K
        __syncthreads();                                    // barrier K + 1
        if (on) {
            at32(a.theta, ep) = th;
            at32(a.grad, ep) = gc;
            if (i == 0) at32(a.step, eu) = s_prev;
        }
    } else if (wave == kSumsWave) {
        // ======================= sums wave =======================
        // the raw history, the previous entries and the raw sums' info values
        const float th_init = i < P ? a.init[i] : 0.0f;
        const float g_init = i < P ? a.init_g[i] : 0.0f, l_init = a.init_l;
        float hl_v[kRawHist], hg_v[kRawHist], hw_v[kRawHist];
#pragma unroll
        for (int k = 0; k < kRawHist; ++k) {
            hl_v[k] = at32(a.hl, k * Eu + eu);
            hg_v[k] = at32(a.hg, k * Eu * P + ep);
            hw_v[k] = at32(a.hw, k * Eu * P + ep);
        }
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // barrier t: raw0[t] in
            const MultiRaw0 ri = raw0[buf][lane];
            const int s = ri.s;
            const float thn = ri.thn, g = ri.g, loss = ri.loss;
            const int slot = s % kRawHist, prev = (s - 1) % kRawHist;
            float lp = 0.0f, gp = 0.0f, wp = 0.0f;
            double lsum = loss, gsum = g;
#pragma unroll
            for (int k = 0; k < kRawHist; ++k) {
                if (k == prev) {
                    lp = hl_v[k];
                    gp = hg_v[k];
                    wp = hw_v[k];
                }
                if (k != slot) {
                    lsum += hl_v[k];
                    gsum += hg_v[k];
                }
            }
            const double gsum_all = group_sum<G>(on ? gsum : 0.0);
            MultiRaw &ro = raw[buf][lane];
            ro.info8 = static_cast<float>(gsum_all / (kRawHist * P));
            ro.info9 = static_cast<float>(gsum_all);
            ro.info10 = static_cast<float>(lsum / kRawHist);
            ro.thn = thn;
            ro.g = g;
            ro.loss = loss;
            ro.lr = ri.lr;
            ro.gp = gp;
            ro.wp = wp;
            ro.lp = lp;
            ro.s = s;
            ro.terminal = ri.terminal;
#pragma unroll
            for (int k = 0; k < kRawHist; ++k)
                if (k == slot) {
                    hg_v[k] = g;
                    hw_v[k] = thn;
                    hl_v[k] = loss;
                }
            if (ri.terminal && a.auto_reset) {
#pragma unroll
                for (int k = 0; k < kRawHist; ++k) {
                    hg_v[k] = k == 0 ? g_init : 0.0f;
                    hw_v[k] = k == 0 ? th_init : 0.0f;
                    hl_v[k] = k == 0 ? l_init : 0.0f;
                }
            }
        }
        __syncthreads();                                    // barrier K
        __syncthreads();                                    // barrier K + 1
        if (on) {
#pragma unroll
            for (int k = 0; k < kRawHist; ++k) {
                at32(a.hg, k * Eu * P + ep) = hg_v[k];
                at32(a.hw, k * Eu * P + ep) = hw_v[k];
                if (i == 0) at32(a.hl, k * Eu + eu) = hl_v[k];
            }
        }
    } else if (wave == 3) {
        // ======================= ratio wave =======================
        __syncthreads();                                    // barrier 0
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // barrier t + 1: raw[t] in
            if (CE_MP2_DIAG & 8) continue;
            const MultiRaw ri = raw[buf][lane];
            const int s = ri.s;
            const double adj_l = ratio_fast(ri.loss, ri.lp);
            const double adj_g = ratio_fast(ri.g, ri.gp);
            const double adj_w = ratio_fast(ri.thn, ri.wp);
            double reward = 1.0 - adj_l;
            reward = reward < -100.0 ? -100.0 : (reward > 100.0 ? 100.0 : reward);
            if (!(s >= a.max_batches) && ri.loss > 1e4f) reward -= static_cast<double>(a.max_batches - s);
            // the info values of the ratio wave's own operands (the group sums
            // of multi_persist_kernel, same butterfly)
            auto mine = [&](double v) { return on ? v : 0.0; };
            const double adjg = group_sum<G>(mine(fabs(adj_g))) / P;
            const double gdiff = group_sum<G>(mine(fabs(static_cast<double>(ri.g) - static_cast<double>(ri.gp)))) / P;
            MultiXch4 &xo = xch[buf][lane];
            xo.nsum = fabs(adj_w) + fabs(adj_g) + fabs(adj_l);
            xo.thn = ri.thn;
            xo.lr = ri.lr;
            xo.loss = ri.loss;
            xo.reward = static_cast<float>(reward);
            xo.nw = static_cast<float>(clip100(adj_w) - 1.0);
            xo.nl = static_cast<float>(clip100(adj_l) - 1.0);
            xo.ng = static_cast<float>(clip100(adj_g) - 1.0);
            xo.info8 = ri.info8;
            xo.info9 = ri.info9;
            xo.info10 = ri.info10;
            xo.info11 = static_cast<float>(adj_l);
            xo.info12 = static_cast<float>(adjg);
            xo.info13 = static_cast<float>(gdiff);
            xo.s = s;
            xo.terminal = ri.terminal;
        }
        __syncthreads();                                    // barrier K + 1
    } else if (wave == kRowsWave) {
        // ======================= rows wave =======================
        // The adjusted rings' observation columns, held newest first (a
        // shift register: the row is the ring as it stands, written at
        // constant LDS offsets).  In HBM they stay in slot order, slot
        // (s - 1) % H the newest, as the one-step kernel keeps them.
        const int s0 = at32(a.step, eu);
        const int new0 = ((s0 - 1) % H + H) % H;
        float ol_v[H], og_v[H], ow_v[H];
#pragma unroll
        for (int q = 0; q < H; ++q) {
            const int j = (new0 - q + H) % H;
            ol_v[q] = at32(a.ol, j * Eu + eu);
            og_v[q] = at32(a.og, j * Eu * P + ep);
            ow_v[q] = at32(a.ow, j * Eu * P + ep);
        }
        float *const lrow = stage + ((lane / G) * P + r) * row;
        int s_end = s0;
        __syncthreads();                                    // barrier 0
        __syncthreads();                                    // barrier 1
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // barrier t + 2: xch[t] in
            const long long ro = t * out_step;
            const MultiXch4 &xi = xch[buf][lane];
            if (CE_MP2_DIAG & 2) continue;
            const bool wipe = xi.terminal != 0 && a.auto_reset;
            const float nw = xi.nw, ng = xi.ng, nl = xi.nl;
            s_end = wipe ? 0 : xi.s;
#pragma unroll
            for (int q = H - 1; q > 0; --q) {
                og_v[q] = og_v[q - 1];
                ow_v[q] = ow_v[q - 1];
                ol_v[q] = ol_v[q - 1];
            }
            og_v[0] = ng;
            ow_v[0] = nw;
            ol_v[0] = nl;
            if (wipe) {
#pragma unroll
                for (int q = 0; q < H; ++q) {
                    og_v[q] = -1.0f;
                    ow_v[q] = -1.0f;
                    ol_v[q] = -1.0f;
                }
            }
            if (on) {
#pragma unroll
                for (int q = 0; q < H; ++q) {
                    lrow[q] = ow_v[q];
                    lrow[H + q] = ol_v[q];
                    lrow[2 * H + q] = og_v[q];
                }
            }
            __builtin_amdgcn_wave_barrier();
            {
                const float *lds = stage;
                float *out = reinterpret_cast<float *>(reinterpret_cast<char *>(a.obs) + ro) + e_first * P * row;
                constexpr int kV = (span / 4 + 63) / 64;
                if ((nblk & 3) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0) {
                    const float4 *src = reinterpret_cast<const float4 *>(lds);
                    float4 *dst4 = reinterpret_cast<float4 *>(out);
                    const int n4 = nblk >> 2;
                    float4 v[kV];
#pragma unroll
                    for (int u = 0; u < kV; ++u) {
                        const int q = lane + 64 * u;
                        v[u] = src[q < n4 ? q : n4 - 1];
                    }
#pragma unroll
                    for (int u = 0; u < kV; ++u) {
                        const int q = lane + 64 * u;
                        if (q < n4) dst4[q] = v[u];
                    }
                } else {
                    for (int q = lane; q < nblk; q += 64) out[q] = lds[q];
                }
            }
            __builtin_amdgcn_wave_barrier();
        }
        if (on) {
            const int new_end = ((s_end - 1) % H + H) % H;
#pragma unroll
            for (int q = 0; q < H; ++q) {
                const int j = (new_end - q + H) % H;
                at32(a.og, j * Eu * P + ep) = og_v[q];
                at32(a.ow, j * Eu * P + ep) = ow_v[q];
                if (i == 0) at32(a.ol, j * Eu + eu) = ol_v[q];
            }
        }
    } else {
        // ======================= info wave =======================
        double sa_v[H];
#pragma unroll
        for (int j = 0; j < H; ++j) sa_v[j] = at32(a.sa, j * Eu * P + ep);
        __syncthreads();                                    // barrier 0
        __syncthreads();                                    // barrier 1
        for (int t = 0; t < K; ++t) {
            const int buf = t & 1;
            __syncthreads();                                // barrier t + 2: xch[t] in
            const long long ro = t * out_step;
            const MultiXch4 xi = xch[buf][lane];
            if (CE_MP2_DIAG & 1) continue;
            const int s = xi.s;
            const bool terminal = xi.terminal != 0;
            const bool wipe = terminal && a.auto_reset;
            const int aslot = (s - 1) % H;
            double st_abs = 0.0;
            const int k0 = aslot;
#pragma unroll
            for (int j = 0; j < H; ++j) {
                const int kk = k0 - j >= 0 ? k0 - j : k0 - j + H;
                st_abs += kk == 0 ? xi.nsum : sa_v[j];
            }
#pragma unroll
            for (int j = 0; j < H; ++j)
                if (j == aslot) sa_v[j] = xi.nsum;
            if (wipe) {
#pragma unroll
                for (int j = 0; j < H; ++j) sa_v[j] = 0.0;
            }
            const double lr = xi.lr;
            auto mine = [&](double v) { return on ? v : 0.0; };
            const double wsum = group_sum<G>(mine(fabs(static_cast<double>(xi.thn))));
            const double amean = group_sum<G>(mine(lr)) / P;
            const double dev = lr - amean;
            const double avar = group_sum<G>(mine(dev * dev)) / P;
            const double st_all = group_sum<G>(mine(st_abs));
            if (on) {
                if (i == 0) {
                    float *info = reinterpret_cast<float *>(reinterpret_cast<char *>(a.info) + ro) + eu * kMultiInfo;
                    info[0] = terminal ? xi.loss : __builtin_nanf("");
                    info[1] = xi.loss;
                    info[2] = static_cast<float>(wsum / P);
                    info[3] = static_cast<float>(wsum);
                    at32(reinterpret_cast<int32_t *>(reinterpret_cast<char *>(a.episode_len) + ro), eu) = xi.s;
                    info[4] = static_cast<float>(amean);
                    info[5] = static_cast<float>(sqrt(avar));
                    info[6] = static_cast<float>(st_all / (P * row));
                    info[7] = static_cast<float>(st_all);
                    info[8] = xi.info8;
                    info[9] = xi.info9;
                    info[10] = xi.info10;
                    info[11] = xi.info11;
                    info[12] = xi.info12;
                    info[13] = xi.info13;
                }
                at32(reinterpret_cast<float *>(reinterpret_cast<char *>(a.reward) + ro), eu * P + r) = xi.reward;
                at32(reinterpret_cast<uint8_t *>(a.done) + ro, eu * P + r) = terminal ? 1 : 0;
            }
        }
        if (on) {
#pragma unroll
            for (int j = 0; j < H; ++j) at32(a.sa, j * Eu * P + ep) = sa_v[j];
        }
    }
}

}  // namespace ce
