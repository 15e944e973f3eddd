// Fused Optimize-v0 step for gfx950, two environments per wavefront.
//
// Same computation as ce::optimize_step_kernel (optimize_kernels.h, which
// cites the reference lines it follows) for the two-class shapes with
// F <= 14 (P = 2F <= 28): lanes 0-31 of a wave run env 2w and lanes 32-63
// env 2w+1.  Why:
//   - the per-env fixed work of a step (state loads, the reduction of the
//     gradient / loss / hit partials, the recurrences, divisions and stores)
//     is done by one wave instruction for both envs, so it costs half;
//   - 4096 envs are 2048 waves, 2 per SIMD, each carrying U independent row
//     chains (registers are not the limit at 2 waves per SIMD), instead of 4
//     waves with one chain each.
// Row i of an env's minibatch lives on lane (i mod 32) of its half; both
// halves walk the same rows, each with its own weights.  The weight margin
// w0 - w1 of each half is handed over through a per-wave LDS slot and held
// in VGPRs (SGPRs cannot hold two envs' weights).
#pragma once

#include "optimize_kernels.h"

namespace ce {

constexpr int kHalf = 32;
constexpr int kPairWavesPerBlock = 8;                  // 16 envs per block
constexpr int kPairBlock = kWave * kPairWavesPerBlock;
constexpr int kPairEnvsPerBlock = 2 * kPairWavesPerBlock;

__host__ __device__ constexpr bool pair_shape(int F, int K) { return K == 2 && F <= 14; }

// Bytes of the per-wave w0 - w1 hand-over area that follows the dataset stage.
template <typename T>
__host__ __device__ constexpr size_t pair_scratch_bytes(int F) {
    return static_cast<size_t>(kPairWavesPerBlock) * 2 * ((F + 1) / 2 * 2) * sizeof(T);
}

// W <- W0, histories <- 0, current_step <- 0, order <- order[perm] for the
// env of this half (optimize.py:58-67); sl = lane within the half.
template <typename T, int P>
__device__ __forceinline__ void reset_env_half(const StepArgs<T> &a, int e, int sl) {
    const size_t base = static_cast<size_t>(e) * P;
    if (sl < P) {
        a.W[base + sl] = a.W0[base + sl];
        a.G[base + sl] = T(0);
    }
    if (sl == 0) {
        a.L[e] = 0.0;
        a.step[e] = 0;
    }
    if (a.order != nullptr) {
        const int sel = a.order_sel[e];
        const size_t stride = static_cast<size_t>(a.E) * a.N;
        const int32_t *cur = a.order + sel * stride + static_cast<size_t>(e) * a.N;
        int32_t *nxt = a.order + (1 - sel) * stride + static_cast<size_t>(e) * a.N;
        const int32_t *pm = a.perm + static_cast<size_t>(e) * a.N;
        for (int i = sl; i < a.N; i += kHalf) nxt[i] = cur[pm[i]];
        if (sl == 0) a.order_sel[e] = 1 - sel;
    }
}

// UU rows of each half: minibatch rows i, i + 32, ..., i + 32 (UU - 1).
template <typename Model, typename T, int F, bool MASKED, bool ORDERED, bool FIX, int UU, int NA>
__device__ __forceinline__ void pair_rows(const T *xs, const int32_t *ys, const int32_t *order,
                                          int i, int B, const T (&w)[Model::NB], T (&acc)[NA],
                                          T &loss, T &prod, int &hits,
                                          typename Model::Watch &wt) {
    T x[UU][F];
    int r[UU];
    bool valid[UU];
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        const int iu = i + u * kHalf;
        valid[u] = !MASKED || iu < B;
        r[u] = valid[u] ? (ORDERED ? order[iu] : iu) : 0;
        load_row<T, F>(xs, r[u], x[u]);
    }
    if constexpr (!FIX && Model::kProd) {
        Model::template rows_multi<MASKED, UU>(x, w, valid, acc, prod, hits, wt);
        return;
    }
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        if constexpr (FIX)
            Model::template fixup<MASKED>(x[u], w, ys, r[u], valid[u], loss, hits);
        else
            Model::template row<true, MASKED>(x[u], w, ys, r[u], valid[u], acc, loss, prod, hits,
                                              wt);
    }
}

template <typename Model, typename T, int F, bool ORDERED, int U, int NA>
__device__ __forceinline__ void pair_minibatch(const T *xs, const int32_t *ys,
                                               const int32_t *order, int sl, int B,
                                               const T (&w)[Model::NB], T (&acc)[NA], T &loss,
                                               int &hits) {
    T prod = T(1);
    int since = 0;
    typename Model::Watch wt;
    const int full = B / (kHalf * U) * (kHalf * U);
    for (int i0 = 0; i0 < full; i0 += kHalf * U) {
        pair_rows<Model, T, F, false, ORDERED, false, U>(xs, ys, order, i0 + sl, B, w, acc, loss,
                                                         prod, hits, wt);
        if (Model::kProd && (since += U) >= kProdFold) {
            loss -= log_pos(prod);
            prod = T(1);
            since = 0;
        }
    }
    for (int i0 = full; i0 < B; i0 += kHalf)
        pair_rows<Model, T, F, true, ORDERED, false, 1>(xs, ys, order, i0 + sl, B, w, acc, loss,
                                                        prod, hits, wt);
    if (Model::kProd) loss -= log_pos(prod);
    if (__any(wt.flagged())) {
        for (int i0 = 0; i0 < B; i0 += kHalf)
            pair_rows<Model, T, F, true, ORDERED, true, 1>(xs, ys, order, i0 + sl, B, w, acc,
                                                           loss, prod, hits, wt);
    }
}

template <typename T, int F, int U>
__global__ __launch_bounds__(kPairBlock) void optimize_pair_kernel(StepArgs<T> a) {
    using Model = TwoClassModel<T, F>;
    constexpr int P = 2 * F;
    constexpr int OBS = 2 * P + 1;
    constexpr int NE = Model::NE;
    constexpr int NP = next_pow2(NE + 2);
    static_assert(NP <= kHalf / 2, "pair path needs two lanes per reduced element");
    constexpr int S = 5 - Log2<NP>::value;               // element of lane sl: sl >> S

#ifdef CE_DIAG
    unsigned long long stamps[kStamps] = {0};
    stamps[6] = __builtin_amdgcn_s_memrealtime();
#endif
    CE_STAMP(0);
    const int lane = threadIdx.x & (kWave - 1);
    const int half = lane >> 5;
    const int sl = lane & (kHalf - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int e = (blockIdx.x * kPairWavesPerBlock + wave) * 2 + half;
    const bool active = e < a.E;                         // uniform per half
    const int eidx = active ? e : 0;
    const size_t pbase = static_cast<size_t>(eidx) * P;
    const int N = a.N;

    // ---- state loads (unconditional, clamped): overlap the staging copy.
    int j_own;
    T sign_own;
    const bool owner = Model::param_of(sl >> S, sl & ((1 << S) - 1), j_own, sign_own);
    const int pl = sl < P ? sl : P - 1;
    const T w_raw = a.W[pbase + pl];
    const float a_raw = a.act[pbase + pl];
    const T g_raw = a.G[pbase + (owner ? j_own : 0)];
    const double lprev = a.L[eidx];
    const int step_prev = a.step[eidx];

    // ---- dataset -> LDS by LDS-DMA (1 KiB per wave-instruction), rotated
    // per block; then the per-wave w0 - w1 slots after it.
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int RS = row_stride(F, sizeof(T));
    const size_t xbytes = align16_dev(sizeof(T) * RS * static_cast<size_t>(N));
    const size_t sbytes = align16_dev(xbytes + 4 * static_cast<size_t>(N));
    {
        const int nvec = static_cast<int>(sbytes / 16);
        const int nch = (nvec + kWave - 1) / kWave;
        const int rot = static_cast<int>((blockIdx.x * 5u) % static_cast<unsigned>(nch));
        for (int c0 = wave; c0 < nch; c0 += kPairWavesPerBlock) {
            const int c = c0 + rot < nch ? c0 + rot : c0 + rot - nch;   // wave-uniform
            const int v = c * kWave + lane;
            if (v < nvec)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) void *)(a.data + static_cast<size_t>(v) * 16),
                    (__attribute__((address_space(3))) void *)(smem + c * kWave * 16), 16, 0, 0);
        }
    }
    __syncthreads();
    CE_STAMP(1);
    const T *xs = reinterpret_cast<const T *>(smem);
    const int32_t *ys = reinterpret_cast<const int32_t *>(smem + xbytes);
    if (!__any(active)) return;                          // both halves past E

    // ---- W <- W - a (optimize.py:74-75); lane sl of a half owns parameter sl.
    const T gprev = owner ? g_raw : T(0);
    const T wl = sl < P ? w_raw - static_cast<T>(a_raw) : T(0);
    // w0 - w1 per feature: lane 2f of a half forms it, the half reads it back
    // as broadcast LDS reads (identical addresses within a half).
    constexpr int FS = (F + 1) / 2 * 2;
    T *slot = reinterpret_cast<T *>(smem + sbytes) + (wave * 2 + half) * FS;
    const T d = wl - __shfl_down(wl, 1);
    if (sl < 2 * F && (sl & 1) == 0) slot[sl >> 1] = d;
    __builtin_amdgcn_wave_barrier();
    T wd[F];
#pragma unroll
    for (int f = 0; f < F; ++f) wd[f] = slot[f];
    const int cur_step = step_prev + 1;
    CE_STAMP(2);

    // ---- minibatch rows of each half's env.
    const int32_t *order = nullptr;
    if (a.order != nullptr) {
        const int sel = a.order_sel[eidx];
        order = a.order + sel * static_cast<size_t>(a.E) * N + static_cast<size_t>(eidx) * N;
    }
    T acc[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) acc[j] = T(0);
    T loss_l = T(0);
    int hits_l = 0;
    if (a.order != nullptr)
        pair_minibatch<Model, T, F, true, U>(xs, ys, order, sl, a.B, wd, acc, loss_l, hits_l);
    else
        pair_minibatch<Model, T, F, false, U>(xs, ys, nullptr, sl, a.B, wd, acc, loss_l, hits_l);
    acc[NE] = loss_l;
    acc[NE + 1] = static_cast<T>(hits_l);
    CE_STAMP(3);
    ReduceScatter<T, NP, 16>::run(acc, lane);            // within each 32-lane half
    const int hb = half * kHalf;
    const T tot_loss = __shfl(acc[0], hb + (NE << S));
    const T tot_hit = __shfl(acc[0], hb + ((NE + 1) << S));
    const double loss = static_cast<double>(tot_loss) / a.B;
    double objective = loss, accuracy = static_cast<double>(tot_hit) / a.B;

    // ---- info pass over the full dataset (optimize.py:94-97), B < N only.
    if (a.B != N) {
        T fl = T(0), fprod = T(1);
        int fh = 0, since = 0;
        T none[1];
        typename Model::Watch wt;
        for (int i0 = 0; i0 < N; i0 += kHalf) {
            const int r = i0 + sl;
            const bool valid = r < N;
            const int rr = valid ? r : 0;
            T x[F];
            load_row<T, F>(xs, rr, x);
            Model::template row<false, true>(x, wd, ys, rr, valid, none, fl, fprod, fh, wt);
            if (Model::kProd && ++since >= kProdFold) {
                fl -= log_pos(fprod);
                fprod = T(1);
                since = 0;
            }
        }
        if (Model::kProd) fl -= log_pos(fprod);
        if (__any(wt.flagged())) {
            for (int i0 = 0; i0 < N; i0 += kHalf) {
                const int r = i0 + sl;
                const bool valid = r < N;
                const int rr = valid ? r : 0;
                T x[F];
                load_row<T, F>(xs, rr, x);
                Model::template fixup<true>(x, wd, ys, rr, valid, fl, fh);
            }
        }
        objective = static_cast<double>(lane_sum<T, 16>(fl)) / N;
        accuracy = static_cast<double>(lane_sum<T, 16>(static_cast<T>(fh))) / N;
    }

    CE_STAMP(4);
    // ---- recurrences (optimize.py:80-86) and outputs, per half.
    const double lnew = (loss - lprev) / (lprev + 0.1);
    const bool done = cur_step >= a.max_steps;
    const bool wipe = done && a.auto_reset;              // VecEnv auto-reset this step
    float gnew_f = 0.0f;
    if (owner) {
        const T g = sign_own * acc[0] / static_cast<T>(a.B);
        const T gnew = g / (fabs(gprev) + T(1));
        if (active && !wipe) a.G[pbase + j_own] = gnew;
        gnew_f = static_cast<float>(gnew);
    }
    if (active && sl < P && !wipe) a.W[pbase + sl] = wl;
    // obs row = [0 (P) | L' | G' (P)] (zeros on auto-reset): 32 entries per
    // half per store instruction, G' gathered from its owner lanes.
    float *obs = a.obs + static_cast<size_t>(eidx) * OBS;
#pragma unroll
    for (int i0 = 0; i0 < OBS; i0 += kHalf) {
        const int i = i0 + sl;
        const int src = hb + ((i > P && i < OBS) ? Model::owner_lane(i - P - 1, S) : 0);
        const float gv = __shfl(gnew_f, src);
        float v = i < P ? 0.0f : (i == P ? static_cast<float>(lnew) : gv);
        if (wipe) v = 0.0f;
        if (active && i < OBS) obs[i] = v;
    }
    if (active && sl == 0) {
        a.reward[e] = static_cast<float>(-loss);
        a.done[e] = done ? 1 : 0;
        a.objective[e] = static_cast<float>(objective);
        a.accuracy[e] = static_cast<float>(accuracy);
        a.episode_len[e] = cur_step;
        if (!wipe) {
            a.L[e] = lnew;
            a.step[e] = cur_step;
        }
    }
    if (active && wipe) reset_env_half<T, P>(a, e, sl);
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CE_STAMP(5);
    stamps[7] = __builtin_amdgcn_s_memrealtime();
    if (active && sl < kStamps) a.diag[static_cast<size_t>(e) * kStamps + sl] = stamps[sl];
#endif
}

}  // namespace ce
