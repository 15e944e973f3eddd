// Fused Optimize-v0 step for gfx950: one 64-lane wavefront per environment.
//
// One launch advances every env of the engine by one VecEnv.step, i.e. the
// whole chain
//   _worker 'step' + auto-reset     custom_envs/utils/utils_venv.py:24-56 (:31)
//   BaseEnvironment.step            custom_envs/envs/baseenvironment.py:30-41
//   Optimize.base_step              custom_envs/envs/optimize.py:69-100
//   ModelNumpy.compute_backprop     (build-defined)
//   softmax / cross_entropy         custom_envs/utils/utils_math.py:51-63,25-34
// for E envs at once.  Per env and step:
//   W   <- W - a                                        (optimize.py:74-75)
//   P    = softmax(X_b W); loss = mean CE; acc           (A7)
//   g    = X_b^T (P - Y) / B                             (optimize.py:76-78)
//   L'   = (loss - L) / (L + 0.1)                        (optimize.py:80-81)
//   G'   = g / (|G| + 1)                                 (optimize.py:82-83)
//   obs  = [0 (P), L', G' (P)]   (wght_hist is identically 0: optimize.py:84-86)
//   reward = -loss, done = step >= max_steps, info = full-data (loss, acc)
//   done -> W <- W0, G <- 0, L <- 0, step <- 0, order <- order[perm]
//
// Lane mapping: minibatch row i of an env lives on lane i % 64 (chunks of
// 64 rows).  W is broadcast from lanes 0..P-1 into scalar registers with
// v_readlane, so the row loop is VGPR(x) x SGPR(w) FMAs.  The P gradient
// partials, the loss and the hit count are combined by a recursive-halving
// reduce-scatter over the wave (log2(NP) xor-shuffle levels moving NP-1
// values instead of NP*6), after which lane l owns element l >> S.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ce {

constexpr int kWave = 64;
constexpr int kWavesPerBlock = 4;
constexpr int kBlock = kWave * kWavesPerBlock;

template <typename T>
struct StepArgs {
    int E, N, B, max_steps, auto_reset;
    const T *X;            // [N][F] row-major dataset (device copy, type T)
    const int32_t *label;  // [N] class index (one-hot targets)
    T *W;                  // [E][P] model.weights
    T *G;                  // [E][P] grad_hist[idx] of the last step
    double *L;             // [E]    loss_hist[idx] of the last step
    int32_t *step;         // [E]    current_step
    const T *W0;           // [E][P] weights every reset restores
    const int32_t *perm;   // [E][N] reset permutation (B < N only)
    int32_t *order;        // [2][E][N] row-order ping-pong (B < N only)
    int32_t *order_sel;    // [E]
    const float *act;      // [E][P] actions (float32, the Box dtype)
    float *obs;            // [E][2P+1]
    float *reward;
    uint8_t *done;
    float *objective;
    float *accuracy;
    int32_t *episode_len;
};

__device__ __forceinline__ double readlane(double v, int l) {
    const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(v));
    const int lo = __builtin_amdgcn_readlane(static_cast<int>(bits & 0xffffffffull), l);
    const int hi = __builtin_amdgcn_readlane(static_cast<int>(bits >> 32), l);
    return __longlong_as_double(static_cast<long long>(
        (static_cast<unsigned long long>(static_cast<unsigned>(hi)) << 32) |
        static_cast<unsigned>(lo)));
}

__device__ __forceinline__ float readlane(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

__device__ __forceinline__ double exp_t(double v) { return exp(v); }
__device__ __forceinline__ float exp_t(float v) { return expf(v); }
__device__ __forceinline__ double log_t(double v) { return log(v); }
__device__ __forceinline__ float log_t(float v) { return logf(v); }

template <int N>
struct Log2 { static constexpr int value = 1 + Log2<N / 2>::value; };
template <>
struct Log2<1> { static constexpr int value = 0; };

constexpr int next_pow2(int v) {
    int p = 1;
    while (p < v) p <<= 1;
    return p;
}

// Recursive-halving reduce-scatter over the 64 lanes of a wave.  On entry
// acc[0..NP) holds per-lane partials; on exit acc[0] of lane l holds the
// wave total of element (l >> (6 - log2 NP)).
template <typename T, int NP, int OFF>
struct ReduceScatter {
    static __device__ __forceinline__ void run(T (&acc)[NP], int lane) {
        constexpr int half = NP / 2;
        static_assert(NP >= 2, "");
        const bool hi = (lane & OFF) != 0;
#pragma unroll
        for (int j = 0; j < half; ++j) {
            const T keep = hi ? acc[j + half] : acc[j];
            const T send = hi ? acc[j] : acc[j + half];
            acc[j] = keep + __shfl_xor(send, OFF);
        }
        T (&next)[half] = *reinterpret_cast<T(*)[half]>(&acc[0]);
        ReduceScatter<T, half, OFF / 2>::run(next, lane);
    }
};
template <typename T, int OFF>
struct ReduceScatter<T, 1, OFF> {
    static __device__ __forceinline__ void run(T (&acc)[1], int) {
#pragma unroll
        for (int off = OFF; off >= 1; off >>= 1) acc[0] += __shfl_xor(acc[0], off);
    }
};
template <typename T, int NP>
struct ReduceScatter<T, NP, 0> {
    static __device__ __forceinline__ void run(T (&)[NP], int) {}
};
template <typename T>
struct ReduceScatter<T, 1, 0> {
    static __device__ __forceinline__ void run(T (&)[1], int) {}
};

template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off);
    return v;
}

// Forward pass of one row: softmax probabilities, loss term, hit.
template <typename T, int F, int K>
__device__ __forceinline__ void row_forward(const T (&x)[F], const T (&w)[F * K], int y,
                                            T (&p)[K], T &loss_term, int &hit) {
    T logit[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        T s = x[0] * w[k];
#pragma unroll
        for (int f = 1; f < F; ++f) s = fma(x[f], w[f * K + k], s);
        logit[k] = s;
    }
    T m = logit[0];
#pragma unroll
    for (int k = 1; k < K; ++k) m = logit[k] > m ? logit[k] : m;
    T denom = T(0);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        p[k] = exp_t(logit[k] - m);
        denom += p[k];
    }
    int best = 0;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        p[k] = p[k] / denom;
        if (k > 0 && p[k] > p[best]) best = k;   // np.argmax: first maximum
    }
    T py = p[0];
#pragma unroll
    for (int k = 1; k < K; ++k) py = (k == y) ? p[k] : py;
    loss_term = -log_t(py + T(1e-16));
    hit = (best == y) ? 1 : 0;
}

template <typename T, int F>
__device__ __forceinline__ void load_row(const T *X, int r, T (&x)[F]) {
    const T *src = X + static_cast<size_t>(r) * F;
#pragma unroll
    for (int f = 0; f < F; ++f) x[f] = src[f];
}

// Restore the env to what Optimize.base_reset leaves (optimize.py:58-67):
// W <- W0, histories <- 0, current_step <- 0, dataset order <- order[perm].
template <typename T, int P>
__device__ __forceinline__ void reset_env(const StepArgs<T> &a, int e, int lane) {
    const size_t base = static_cast<size_t>(e) * P;
    if (lane < P) {
        a.W[base + lane] = a.W0[base + lane];
        a.G[base + lane] = T(0);
    }
    if (lane == 0) {
        a.L[e] = 0.0;
        a.step[e] = 0;
    }
    if (a.order != nullptr) {
        const int sel = a.order_sel[e];
        const size_t stride = static_cast<size_t>(a.E) * a.N;
        const int32_t *cur = a.order + sel * stride + static_cast<size_t>(e) * a.N;
        int32_t *nxt = a.order + (1 - sel) * stride + static_cast<size_t>(e) * a.N;
        const int32_t *pm = a.perm + static_cast<size_t>(e) * a.N;
        for (int i = lane; i < a.N; i += kWave) nxt[i] = cur[pm[i]];
        if (lane == 0) a.order_sel[e] = 1 - sel;
    }
}

template <typename T, int F, int K>
__global__ __launch_bounds__(kBlock) void optimize_reset_kernel(StepArgs<T> a) {
    constexpr int P = F * K;
    constexpr int OBS = 2 * P + 1;
    const int lane = threadIdx.x & (kWave - 1);
    const int e = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (e >= a.E) return;
    reset_env<T, P>(a, e, lane);
    for (int i = lane; i < OBS; i += kWave) a.obs[static_cast<size_t>(e) * OBS + i] = 0.0f;
}

template <typename T, int F, int K>
__global__ __launch_bounds__(kBlock) void optimize_step_kernel(StepArgs<T> a) {
    constexpr int P = F * K;
    constexpr int OBS = 2 * P + 1;
    constexpr int NP = next_pow2(P + 2);
    static_assert(NP <= kWave, "register path needs F*K + 2 <= 64");
    constexpr int SHIFT = 6 - Log2<NP>::value;

    const int lane = threadIdx.x & (kWave - 1);
    const int e = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    if (e >= a.E) return;   // wave-uniform
    const size_t pbase = static_cast<size_t>(e) * P;

    // ---- W <- W - a (optimize.py:74-75); lane j owns parameter j.
    T wl = T(0);
    if (lane < P) wl = a.W[pbase + lane] - static_cast<T>(a.act[pbase + lane]);
    T w[P];
#pragma unroll
    for (int j = 0; j < P; ++j) w[j] = readlane(wl, j);
    const int cur_step = __builtin_amdgcn_readfirstlane(a.step[e]) + 1;

    // ---- minibatch rows: sequence[0] = rows [0, B) of the current order.
    const int32_t *order = nullptr;
    if (a.order != nullptr) {
        const int sel = __builtin_amdgcn_readfirstlane(a.order_sel[e]);
        order = a.order + sel * static_cast<size_t>(a.E) * a.N + static_cast<size_t>(e) * a.N;
    }
    T acc[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) acc[j] = T(0);
    for (int i0 = 0; i0 < a.B; i0 += kWave) {
        const int i = i0 + lane;
        if (i < a.B) {
            const int r = order ? order[i] : i;
            T x[F];
            load_row<T, F>(a.X, r, x);
            const int y = a.label[r];
            T p[K], lt;
            int hit;
            row_forward<T, F, K>(x, w, y, p, lt, hit);
#pragma unroll
            for (int k = 0; k < K; ++k) {
                const T d = p[k] - (k == y ? T(1) : T(0));
#pragma unroll
                for (int f = 0; f < F; ++f) acc[f * K + k] = fma(x[f], d, acc[f * K + k]);
            }
            acc[P] += lt;
            acc[P + 1] += static_cast<T>(hit);
        }
    }
    ReduceScatter<T, NP, 32>::run(acc, lane);
    const int mine = lane >> SHIFT;              // element this lane now owns
    const bool owner = (lane & ((1 << SHIFT) - 1)) == 0;
    const T tot_loss = readlane(acc[0], P << SHIFT);
    const T tot_hit = readlane(acc[0], (P + 1) << SHIFT);
    const double loss = static_cast<double>(tot_loss) / a.B;
    const double acc_mb = static_cast<double>(tot_hit) / a.B;

    // ---- info pass over the full dataset (optimize.py:94-97); with B == N
    // the minibatch *is* the dataset and the reference computes the same
    // numbers twice, so they are reused.
    double objective = loss, accuracy = acc_mb;
    if (a.B != a.N) {
        T fl = T(0), fh = T(0);
        for (int i0 = 0; i0 < a.N; i0 += kWave) {
            const int r = i0 + lane;
            if (r < a.N) {
                T x[F];
                load_row<T, F>(a.X, r, x);
                T p[K], lt;
                int hit;
                row_forward<T, F, K>(x, w, a.label[r], p, lt, hit);
                fl += lt;
                fh += static_cast<T>(hit);
            }
        }
        fl = wave_sum(fl);
        fh = wave_sum(fh);
        objective = static_cast<double>(fl) / a.N;
        accuracy = static_cast<double>(fh) / a.N;
    }

    // ---- recurrences (optimize.py:80-86) and outputs.
    const double lprev = a.L[e];
    const double lnew = (loss - lprev) / (lprev + 0.1);
    const bool done = cur_step >= a.max_steps;
    const bool wipe = done && a.auto_reset;   // VecEnv auto-reset this step
    float *obs = a.obs + static_cast<size_t>(e) * OBS;
    if (owner && mine < P) {
        const T g = static_cast<T>(static_cast<double>(acc[0]) / a.B);
        const T gprev = a.G[pbase + mine];
        const T gnew = g / (fabs(gprev) + T(1));
        if (!wipe) {
            a.G[pbase + mine] = gnew;
            obs[P + 1 + mine] = static_cast<float>(gnew);
        }
    }
    if (lane < P) {
        obs[lane] = 0.0f;
        if (!wipe) a.W[pbase + lane] = wl;
    }
    if (lane == 0) {
        a.reward[e] = static_cast<float>(-loss);
        a.done[e] = done ? 1 : 0;
        a.objective[e] = static_cast<float>(objective);
        a.accuracy[e] = static_cast<float>(accuracy);
        a.episode_len[e] = cur_step;
        if (!wipe) {
            a.L[e] = lnew;
            a.step[e] = cur_step;
            obs[P] = static_cast<float>(lnew);
        }
    }
    if (wipe) {   // the returned obs is the reset obs (zeros)
        reset_env<T, P>(a, e, lane);
        for (int i = lane; i < OBS; i += kWave) obs[i] = 0.0f;
    }
}

}  // namespace ce
