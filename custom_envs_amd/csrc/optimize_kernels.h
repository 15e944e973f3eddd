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
// Layout and mapping
//   - The dataset is stored row-major with rows padded to an odd number of
//     16-byte units (row_stride) and staged once per workgroup into LDS (16
//     envs share one copy): a row is F/2 conflict-free ds_read_b128 at
//     immediate offsets.
//   - Minibatch row i of an env lives on lane i % 64 (chunks of 64 rows).
//   - W is broadcast from lanes 0..P-1 into scalar registers (v_readlane):
//     the row loop is VGPR(x) x SGPR(w) FMAs.
//   - K = 2 uses the two-class form of the same softmax (TwoClassModel):
//     z = x.(w0 - w1), t = exp(-|z|), p_max = 1/(1+t), p_min = t/(1+t): one
//     exp and one reciprocal per row, the cross-entropy as the log of a
//     per-lane product, and column 1 of X^T(P-Y) is exactly minus column 0.
//     The benchmark shape runs the two-envs-per-wave variant of this kernel
//     (optimize_pair_kernel.h); this one-env-per-wave kernel covers the rest.
//   - p_y - 1 is formed as -(sum of the other classes' p), which is the
//     same number without the cancellation.
//   - Gradient partials, the loss and the hit count are combined by a
//     recursive-halving reduce-scatter over the wave (log2(NP) xor-shuffle
//     levels moving NP-1 values instead of NP*6), after which lane l owns
//     element l >> S.
#pragma once

#include "exp2_table.h"

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace ce {

// A store of a 4- or 8-byte value, write-through (sc1: an agent-scope relaxed
// atomic store) when WT: the L2 line is written back as the store lands, so a
// launch ends with little dirty L2 for the kernel boundary to write back
// (MI355X_MICROARCH.md, kernel boundaries).  Other sizes store plainly.
template <bool WT, typename T>
__device__ __forceinline__ void wt_store(T *p, T v) {
    if constexpr (WT && sizeof(T) == 8) {
        __hip_atomic_store((__attribute__((address_space(1))) unsigned long long *)(p),
                           __builtin_bit_cast(unsigned long long, v), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    } else if constexpr (WT && sizeof(T) == 4) {
        __hip_atomic_store((__attribute__((address_space(1))) unsigned *)(p),
                           __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *p = v;
    }
}


constexpr int kWave = 64;
constexpr int kWavesPerBlock = 16;
constexpr int kBlock = kWave * kWavesPerBlock;
constexpr size_t kStageLimit = 64 * 1024;   // LDS bytes a block may stage

// Near-minimax (Chebyshev-fitted) polynomial for the two-class fast path:
//   exp(r),  |r| <= ln2/2 : degree 10, rel. err 6.7e-16 (c0 = 1 exactly, so
//                           exp(0) == 1 as in libm)
// (fit: scripts/fit_poly.py).  Horner order is from the top coefficient.
constexpr int kExpTerms = 11;
constexpr double kExpCoef[kExpTerms] = {
    1.0, 1.000000000000006, 0.49999999999997946, 0.16666666666560392,
    0.041666666667466275, 0.008333333384270189, 0.0013888888768614806,
    0.00019841171680137992, 2.4801650828121558e-05, 2.7639677785365415e-06,
    2.7575738554394086e-07};
constexpr double kLn2Hi = 6.93147180369123816490e-01;
constexpr double kLn2Lo = 1.90821492927058770002e-10;
constexpr double kLog2e = 1.44269504088896338700e+00;

// e^-x for Q arguments x in [-700, 750] through a table of 2^(j/2048)
// (CE_LR_TEXP): m = rint(-2048 x log2e) by the shifter, r = -x - m ln2/2048
// in [-ln2/4096, ln2/4096], e^r - 1 = r + r^2/2 + r^3/6 (truncation r^4/24 <
// 3.5e-17 relative), e^-x = 2^(m >> 11) (T[m & 2047] + T[m & 2047] (e^r - 1)).
// 9 f64 operations per value against exp_neg_q's 15; the table entry is an
// LDS read under the polynomial.  T[j] is 2^(j/2048) rounded to float64
// (exp2_table.h, scripts/gen_exp2_table.py); the result is within 1.3 ulp
// (tests/test_exp_table.py; the degree-10 polynomial: 3 ulp).  The 256-entry
// table with a degree-4 polynomial it replaces measured 2 % slower on the
// benchmark kernel (profiles/r05af_*).
constexpr int kLrExpTab = CE_EXP2_TAB_SIZE;
#ifndef CE_TEXP_PIN
#define CE_TEXP_PIN 1
#endif
constexpr int kLrExpBits = 11;
static_assert(kLrExpTab == 1 << kLrExpBits, "exp2_table.h size");
template <int Q>
__device__ __forceinline__ void exp_neg_tab(double (&a)[Q], const double *tab) {
    constexpr double kShift = 0x1.8p52;
    constexpr double kC = kLog2e * kLrExpTab;           // exact: power-of-two scale
    constexpr double kH = kLn2Hi / kLrExpTab, kL = kLn2Lo / kLrExpTab;
    double big[Q], r[Q], p[Q], t[Q];
    int n[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
        big[i] = fma(a[i], -kC, kShift);
        const double m = big[i] - kShift;
        // the inner fma is exact: m kH is exact inside it, and -x - m kH,
        // below 2^-12 in magnitude, has no bit under min(ulp(x), 2^-43)
        r[i] = fma(m, -kL, fma(m, -kH, -a[i]));
        const int lo = static_cast<int>(static_cast<unsigned>(__double_as_longlong(big[i])));
        t[i] = tab[lo & (kLrExpTab - 1)];
        n[i] = lo >> kLrExpBits;                        // floor(m / 2048)
    }
#if CE_TEXP_PIN
    // the table reads stay here, ahead of the polynomial that hides their
    // latency (left alone the scheduler sinks them to their use)
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int i = 0; i < Q; ++i) p[i] = fma(r[i], 1.0 / 6.0, 0.5);
#pragma unroll
    for (int i = 0; i < Q; ++i) p[i] = fma(p[i], r[i], 1.0);
#pragma unroll
    for (int i = 0; i < Q; ++i) p[i] *= r[i];
#pragma unroll
    for (int i = 0; i < Q; ++i) a[i] = ldexp(fma(t[i], p[i], t[i]), n[i]);
}

// The workgroup's LDS copy of the table, entries tid + NTHR i, loaded by its
// NTHR threads (16 KB: one copy per workgroup, not per wave).  The loads are
// issued first in the prologue, so the store waits on them alone (vmcnt
// retires in order); the caller orders the store before the first lookup with
// a workgroup barrier.
template <int NTHR>
struct LrExpSlice {
    static_assert(kLrExpTab % NTHR == 0, "table split");
    double v[kLrExpTab / NTHR];
    __device__ __forceinline__ void load(const double *src, int tid) {
#pragma unroll
        for (int i = 0; i < kLrExpTab / NTHR; ++i) v[i] = src[tid + NTHR * i];
    }
    __device__ __forceinline__ void store(double *tab, int tid) const {
#pragma unroll
        for (int i = 0; i < kLrExpTab / NTHR; ++i) tab[tid + NTHR * i] = v[i];
    }
};

template <typename T>
struct MathConsts {};

template <typename T>
struct StepArgs {
    int E, N, B, max_steps, auto_reset;
    int F, K;                   // features, classes (the runtime-shape kernel reads them)
    const unsigned char *data;  // [N][RS] rows (padded, row_stride) then [N] int32 labels
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
    unsigned long long *diag;   // [E][kStamps] (CE_DIAG builds only)
    double inv_B;               // 1 / B, correctly rounded (host)
    int p_mul;                  // ceil(65536 / P): j = (t p_mul) >> 16 = t / P for t < 2^9
    int lr_waves;               // two-class MFMA kernel: 0 = pick per launch, 4 / 8 = forced
    int gen_tail;               // runtime-shape MFMA kernel: last feature on the VALU when F % 16 == 1
    int gen_cat;                // full batch: the class-concatenated kernel where it is compiled
    int lr_mode_cap;            // two-class MFMA kernel: cap on the row-loop mode (3 = none)
    int obs_stride;             // floats per obs row: 2P + 1, or P + 1 in the compact form
    int obs_lo;                 // first obs entry stored: 0, or P (compact: the wght_hist
                                // block is identically 0 and not stored; done may be null)
};

// Diagnostic builds (-DCE_DIAG) stamp s_memtime at phase boundaries into a
// per-wave record; product builds compile the stamps away.
#ifdef CE_DIAG
#define CE_STAMP(k)                                                              \
    do {                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                       \
        unsigned long long t_;                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory"); \
        __builtin_amdgcn_sched_barrier(0);                                       \
        stamps[k] = t_;                                                          \
    } while (0)
constexpr int kStamps = 8;
#else
#define CE_STAMP(k) \
    do {            \
    } while (0)
#endif

__host__ __device__ constexpr size_t align16_dev(size_t v) { return (v + 15) & ~size_t(15); }

// Row-major dataset rows padded to an odd number of 16-byte units: one row
// is F/2 (double) or F/4 (float) 16-byte loads at immediate offsets, and the
// 16 lanes a ds_read_b128 services together hit 16 disjoint 4-bank groups.
__host__ __device__ constexpr int row_stride(int F, int tsize) {
    const int units = (F * tsize + 15) / 16;
    return (units % 2 ? units : units + 1) * 16 / tsize;
}

// Bytes of the [rows | labels] dataset image (device buffer and LDS stage).
__host__ __device__ constexpr size_t stage_bytes_total(int F, int N, int tsize) {
    return align16_dev(align16_dev(static_cast<size_t>(row_stride(F, tsize)) * N * tsize) +
                   static_cast<size_t>(N) * 4);
}

template <typename T>
struct Vec16;
template <>
struct Vec16<double> { using type = double2; static constexpr int n = 2; };
template <>
struct Vec16<float> { using type = float4; static constexpr int n = 4; };

template <typename T, int F>
__device__ __forceinline__ void load_row(const T *base, int r, T (&x)[F]) {
    using V = typename Vec16<T>::type;
    constexpr int NV = (F + Vec16<T>::n - 1) / Vec16<T>::n;
    constexpr int RS = row_stride(F, sizeof(T));
    const V *src = reinterpret_cast<const V *>(base + static_cast<size_t>(r) * RS);
#pragma unroll
    for (int v = 0; v < NV; ++v) {
        const V q = src[v];
        const T *qe = reinterpret_cast<const T *>(&q);
#pragma unroll
        for (int c = 0; c < Vec16<T>::n; ++c)
            if (v * Vec16<T>::n + c < F) x[v * Vec16<T>::n + c] = qe[c];
    }
}

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

// Cross-lane exchange primitives (gfx950).  xchg<OFF> returns the value of
// lane (l ^ OFF) for OFF < 16 (DPP quad_perm / row_ror:8, ds_swizzle for 4);
// the 16- and 32-lane levels use v_permlane16/32_swap, which exchange whole
// register halves between two VGPRs in one instruction.
template <int OFF>
__device__ __forceinline__ unsigned xchg_u32(unsigned v) {
    if constexpr (OFF == 1)
        return __builtin_amdgcn_update_dpp(0u, v, 0xB1, 0xf, 0xf, false);   // quad_perm [1,0,3,2]
    else if constexpr (OFF == 2)
        return __builtin_amdgcn_update_dpp(0u, v, 0x4E, 0xf, 0xf, false);   // quad_perm [2,3,0,1]
    else if constexpr (OFF == 4)
        return __builtin_amdgcn_ds_swizzle(v, 0x101f);                      // xor 4 (bitmask mode)
    else if constexpr (OFF == 8)
        return __builtin_amdgcn_update_dpp(0u, v, 0x128, 0xf, 0xf, false);  // row_ror:8 = xor 8
    else                                                                     // 16, 32: ds_bpermute
        return static_cast<unsigned>(__shfl_xor(static_cast<int>(v), OFF));
}

template <int OFF>
__device__ __forceinline__ double xchg(double v) {
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
    const unsigned lo = xchg_u32<OFF>(static_cast<unsigned>(b));
    const unsigned hi = xchg_u32<OFF>(static_cast<unsigned>(b >> 32));
    return __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo));
}
template <int OFF>
__device__ __forceinline__ float xchg(float v) { return __uint_as_float(xchg_u32<OFF>(__float_as_uint(v))); }

// (a, b) -> (a', b') with a' + b' = [A totals | B totals]: for OFF = 32 the
// lanes with bit 5 clear end up with a_l + a_{l^32}, the others with
// b_l + b_{l^32}; OFF = 16 likewise on 16-lane rows.
template <int OFF>
__device__ __forceinline__ void swap_halves_u32(unsigned &a, unsigned &b) {
    if constexpr (OFF == 32) {
        const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    } else {
        const auto r = __builtin_amdgcn_permlane16_swap(a, b, false, false);
        a = r[0];
        b = r[1];
    }
}
template <int OFF>
__device__ __forceinline__ double fold_pair(double a, double b) {
    unsigned long long ab = static_cast<unsigned long long>(__double_as_longlong(a));
    unsigned long long bb = static_cast<unsigned long long>(__double_as_longlong(b));
    unsigned alo = static_cast<unsigned>(ab), ahi = static_cast<unsigned>(ab >> 32);
    unsigned blo = static_cast<unsigned>(bb), bhi = static_cast<unsigned>(bb >> 32);
    swap_halves_u32<OFF>(alo, blo);
    swap_halves_u32<OFF>(ahi, bhi);
    const double a2 = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(ahi) << 32) | alo));
    const double b2 = __longlong_as_double(static_cast<long long>((static_cast<unsigned long long>(bhi) << 32) | blo));
    return a2 + b2;
}
template <int OFF>
__device__ __forceinline__ float fold_pair(float a, float b) {
    unsigned au = __float_as_uint(a), bu = __float_as_uint(b);
    swap_halves_u32<OFF>(au, bu);
    return __uint_as_float(au) + __uint_as_float(bu);
}

// Recursive-halving reduce-scatter over the 64 lanes of a wave.  On entry
// acc[0..NP) holds per-lane partials; on exit acc[0] of lane l holds the
// wave total of element (l >> (6 - log2 NP)).  Levels 32 and 16 are
// select-free permlane swaps; lower levels exchange the half a lane gives up.
template <typename T, int NP, int OFF>
struct ReduceScatter {
    static __device__ __forceinline__ void run(T (&acc)[NP], int lane) {
        constexpr int half = NP / 2;
        if constexpr (OFF >= 16) {
#pragma unroll
            for (int j = 0; j < half; ++j) acc[j] = fold_pair<OFF>(acc[j], acc[j + half]);
        } else {
            const bool hi = (lane & OFF) != 0;
#pragma unroll
            for (int j = 0; j < half; ++j) {
                const T keep = hi ? acc[j + half] : acc[j];
                const T send = hi ? acc[j] : acc[j + half];
                acc[j] = keep + xchg<OFF>(send);
            }
        }
        T (&next)[half] = *reinterpret_cast<T(*)[half]>(&acc[0]);
        ReduceScatter<T, half, OFF / 2>::run(next, lane);
    }
};

// Sum of v over the lanes that differ in bits OFF, OFF/2, ..., 1.
template <typename T, int OFF>
__device__ __forceinline__ T lane_sum(T v) {
    if constexpr (OFF == 0) {
        return v;
    } else {
        if constexpr (OFF >= 16) v = fold_pair<OFF>(v, v);
        else v = v + xchg<OFF>(v);
        return lane_sum<T, OFF / 2>(v);
    }
}

template <typename T, int OFF>
struct ReduceScatter<T, 1, OFF> {
    static __device__ __forceinline__ void run(T (&acc)[1], int) { acc[0] = lane_sum<T, OFF>(acc[0]); }
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
__device__ __forceinline__ T wave_sum(T v) { return lane_sum<T, 32>(v); }

// ---------------------------------------------------------------------------
// Problem kernels.  Each "Model" describes the per-row math, how many values
// a lane accumulates (NE gradient elements, then the loss and the hit count),
// and how a reduced element maps back to parameters.  A row call adds the
// row's gradient terms to g[0..NE), its loss term to `loss`, a factor to
// `prod` (models with kProd: sum log(1 + t) is taken as log of a product)
// and its argmax hit to `hits`.
//
// General K: the softmax classifier exactly as written in the reference.
template <typename T, int F, int K>
struct SoftmaxModel {
    static constexpr int P = F * K;
    static constexpr int NE = P;           // reduced gradient elements
    static constexpr int NB = F * K;       // broadcast weight values
    static constexpr bool kProd = false;

    static __device__ __forceinline__ void broadcast(T wl, T (&w)[NB]) {
#pragma unroll
        for (int j = 0; j < NB; ++j) w[j] = readlane(wl, j);
    }

    static constexpr bool kFixup = false;
    struct Watch {
        __device__ __forceinline__ bool flagged() const { return false; }
    };
    template <bool MASKED>
    static __device__ __forceinline__ void fixup(const T (&)[F], const T (&)[NB],
                                                 const int32_t *, int, bool, T &, int &) {}

    template <bool GRAD, bool MASKED, int NA>
    static __device__ __forceinline__ void row(const T (&x)[F], const T (&w)[NB],
                                               const int32_t *ys, int r, bool valid,
                                               T (&acc)[NA], T &loss, T &, int &hits, Watch &) {
        const int y = ys[r];
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
        T p[K], denom = T(0);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            p[k] = exp_t(logit[k] - m);
            denom += p[k];
        }
        int best = 0;
        T py = T(0), rest = T(0);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            p[k] = p[k] / denom;
            if (k > 0 && p[k] > p[best]) best = k;   // np.argmax: first maximum
            if (k == y) py = p[k]; else rest += p[k];
        }
        valid = valid || !MASKED;
        loss += valid ? -log_t(py + T(1e-16)) : T(0);
        hits += (valid && best == y) ? 1 : 0;
        if (GRAD) {
#pragma unroll
            for (int k = 0; k < K; ++k) {
                T d = (k == y) ? -rest : p[k];         // p_k - y_k
                d = valid ? d : T(0);
#pragma unroll
                for (int f = 0; f < F; ++f) acc[f * K + k] = fma(x[f], d, acc[f * K + k]);
            }
        }
    }

    // Parameter index and sign of the value this lane owns after the reduction.
    static __device__ __forceinline__ bool param_of(int m, int sub, int &j, T &sign) {
        j = m;
        sign = T(1);
        return sub == 0 && m < P;
    }
    // A lane that owns parameter j after a reduction with the given shift.
    static __device__ __forceinline__ int owner_lane(int j, int shift) { return j << shift; }
};

// 1/d for d in [1, 4]: hardware reciprocal + two Newton steps (no scaling
// or special cases needed on that range).  Measured on gfx950 over 4M d
// (profiles/r01_rcp_accuracy.json): v_rcp_f64 alone is ~2^-24 relative, one
// Newton step leaves up to 11 ulp, two give the correctly rounded 1/d.
__device__ __forceinline__ double rcp_unit(double d) {
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}
__device__ __forceinline__ float rcp_unit(float d) { return __builtin_amdgcn_rcpf(d); }

// exp(-a) for a >= 0:  m = rint(-a log2e),  r = -a - m ln2 in [-ln2/2, ln2/2],
// exp(-a) = 2^m exp(r) (m is formed negative so no integer negate is needed).  a is clamped at 750, past which exp(-a) is 0 in
// float64 (ldexp underflows), so huge |z| cannot push r out of range.
template <typename T>
__device__ __forceinline__ T exp_neg(T a, const MathConsts<T> &) {
    a = fmin(a, T(750));
    const T m = rint(a * -kLog2e);
    const T r = fma(m, -kLn2Lo, fma(m, -kLn2Hi, -a));
    T q = kExpCoef[kExpTerms - 1];
#pragma unroll
    for (int k = kExpTerms - 2; k >= 0; --k) q = fma(q, r, kExpCoef[k]);
    return ldexp(q, static_cast<int>(m));
}

// The same exp(-a) for Q independent arguments, the Q Horner chains
// interleaved step by step (Q dependent chains hide each other's latency)
// and forced to three-operand v_fma_f64: left to itself the compiler keeps
// the coefficients in VGPRs and emits a v_mov_b64 copy before every
// two-operand v_fmac_f64 (10 extra instructions per exp).
// exp_neg_multi_clamped takes arguments already in [0, 750].
template <int Q>
__device__ __forceinline__ void exp_neg_multi_clamped(double (&a)[Q]) {
    double m[Q], r[Q], q[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
        const double x = a[i];
        m[i] = rint(x * -kLog2e);
        r[i] = fma(m[i], -kLn2Lo, fma(m[i], -kLn2Hi, -x));
        q[i] = kExpCoef[kExpTerms - 1];
    }
#pragma unroll
    for (int k = kExpTerms - 2; k >= 0; --k) {
        const double ck = kExpCoef[k];
#pragma unroll
        for (int i = 0; i < Q; ++i)
            asm("v_fma_f64 %0, %1, %2, %3" : "=v"(q[i]) : "v"(q[i]), "v"(r[i]), "v"(ck));
    }
#pragma unroll
    for (int i = 0; i < Q; ++i) a[i] = ldexp(q[i], static_cast<int>(m[i]));
}
template <int Q>
__device__ __forceinline__ void exp_neg_multi(double (&a)[Q]) {
#pragma unroll
    for (int i = 0; i < Q; ++i) a[i] = fmin(a[i], 750.0);
    exp_neg_multi_clamped<Q>(a);
}
// min(|u|, 750) in one v_min_f64 (fmin(fabs(u), 750) of an MFMA result gets a
// canonicalising v_max_f64 first)
__device__ __forceinline__ double abs_clamp750(double u) {
    double r;
    asm("v_min_f64 %0, |%1|, %2" : "=v"(r) : "v"(u), "v"(750.0));
    return r;
}

// float32 engine: hardware v_exp_f32 (about 1 ulp of float).
__device__ __forceinline__ float exp_neg(float a, const MathConsts<float> &) {
    return __expf(-a);
}

// log(q) for any positive normal q, inline: q = 2^ex m, m in [1/2, 1).
// y0 = log(m) from v_log_f32 (~1e-7 relative) is refined with the float64
// exp already used by the row loop:  d = m exp(-y0) - 1 (|d| ~ 1e-7),
// log(m) = y0 + log1p(d) = y0 + d - d^2/2 + d^3/3 (+ O(d^4) ~ 1e-28).
// No logarithm coefficient table, so nothing beyond the exp constants has
// to stay resident in registers across the row loop.
__device__ __forceinline__ double log_pos(double q) {
    const int ex = __builtin_amdgcn_frexp_exp(q);       // q = 2^ex * m, m in [1/2, 1)
    const double m = __builtin_amdgcn_frexp_mant(q);
    const double y0 = static_cast<double>(__logf(static_cast<float>(m)));
    const double d = fma(m, exp_neg(y0, MathConsts<double>()), -1.0);
    const double lm = fma(d * d, fma(d, 1.0 / 3.0, -0.5), d) + y0;
    return fma(static_cast<double>(ex), kLn2Hi, fma(static_cast<double>(ex), kLn2Lo, lm));
}
__device__ __forceinline__ float log_pos(float q) { return __logf(q); }

// Two-class rows are stored pre-multiplied by s_y = +1 (y = 0) or -1 (y = 1)
// (engine.hip builds the image), so one dot product gives u = s_y z with
// z = x.(w0 - w1) the logit margin of class 0.  Negating an FMA chain's
// inputs negates its result exactly, so |u| = |z| bit for bit.
__host__ __device__ constexpr bool signed_rows(int F, int K) { return K == 2 && F + 2 <= 32; }

// K = 2: the same softmax in its two-class form.  With t = exp(-|z|):
//   p_max = 1/(1+t), p_min = t/(1+t)   (u < 0: y is the smaller-logit class)
//   q     = 1 - p_y = (u < 0 ? p_max : p_min)   (probability of the other class)
//   CE    = -log(p_y + 1e-16)                  (utils_math.py:25-34, literally)
//   p_0 - y_0 = -s_y q, so x (p_0 - y_0) = -(s_y x) q: the gradient column 0
//                        is minus the sum of x~ q, column 1 is plus it.
//   argmax hit = u > 0, exact unless t == 1 (p_max == p_min, a tie: the
//                        reference's np.argmax then picks class 0).
// In float64 the row loop carries no logarithm: sum_i -log(p_y,i + 1e-16) is
// taken as -log of the lane's product of the (p_y + 1e-16) factors, each in
// (1e-16, 1], folded into the sum every kProdFold rows so it cannot
// underflow.  The loop is branch-free; it tracks max(t) per lane, and rows
// with t == 1 get the exact tie argmax from `fixup`, in a second pass a wave
// takes only if one of its lanes saw a tie (practically never: |z| < 2^-53).
template <typename T, int F>
struct TwoClassModel {
    static constexpr int K = 2;
    static constexpr int P = F * 2;
    static constexpr int NE = F;           // column 1 of the gradient = -column 0
    static constexpr int NB = F;           // broadcast w0 - w1
    static constexpr bool kProd = std::is_same<T, double>::value;
    static constexpr bool kFixup = true;

    static __device__ __forceinline__ void broadcast(T wl, T (&wd)[NB]) {
        const T d = wl - __shfl_down(wl, 1);       // lane 2f: w[f][0] - w[f][1]
#pragma unroll
        for (int f = 0; f < F; ++f) wd[f] = readlane(d, 2 * f);
    }

    static __device__ __forceinline__ T margin(const T (&x)[F], const T (&wd)[NB]) {
        T u = x[0] * wd[0];
#pragma unroll
        for (int f = 1; f < F; ++f) u = fma(x[f], wd[f], u);
        return u;
    }

    // Per lane: tmax = max t over the lane's rows (t == 1 marks a tie).
    struct Watch {
        T tmax = T(0);
        __device__ __forceinline__ bool flagged() const { return tmax == T(1); }
    };

    template <bool GRAD, bool MASKED, int NA>
    static __device__ __forceinline__ void row(const T (&x)[F], const T (&wd)[NB],
                                               const int32_t *, int, bool valid,
                                               T (&acc)[NA], T &loss, T &prod, int &hits,
                                               Watch &wt) {
        const T u = margin(x, wd);
        const T t = exp_neg(fabs(u), MathConsts<T>());
        const T inv = rcp_unit(T(1) + t);            // p of the larger-logit class
        const T lo = t * inv;                        // p of the other class
        const bool neg = u < T(0);
        T q = neg ? inv : lo;
        T py = (neg ? lo : inv) + T(1e-16);
        bool hit = u > T(0);
        if (MASKED && !valid) {
            q = T(0);
            py = T(1);
            hit = false;
        }
        wt.tmax = fmax(wt.tmax, (MASKED && !valid) ? T(0) : t);
        if constexpr (kProd)
            prod *= py;
        else
            loss -= log_pos(py);
        hits += hit ? 1 : 0;
        if (GRAD) {
#pragma unroll
            for (int f = 0; f < F; ++f) acc[f] = fma(x[f], q, acc[f]);
        }
    }

    // `row` for UU rows at once, float64, every stage of the UU rows issued
    // side by side (margins, exp chains, reciprocals, then the gradient
    // FMAs): one row's ~30-deep dependent chain is otherwise issued back to
    // back, each f64 step waiting out the ~10-cycle dependent latency.
    template <bool MASKED, int UU, int NA>
    static __device__ __forceinline__ void rows_multi(const T (&x)[UU][F], const T (&wd)[NB],
                                                      const bool (&valid)[UU], T (&acc)[NA],
                                                      T &prod, int &hits, Watch &wt) {
        static_assert(std::is_same<T, double>::value, "float64 rows only");
        double u[UU], t[UU];
#pragma unroll
        for (int i = 0; i < UU; ++i) u[i] = x[i][0] * wd[0];
#pragma unroll
        for (int f = 1; f < F; ++f)
#pragma unroll
            for (int i = 0; i < UU; ++i) u[i] = fma(x[i][f], wd[f], u[i]);
#pragma unroll
        for (int i = 0; i < UU; ++i) t[i] = fabs(u[i]);
        exp_neg_multi<UU>(t);
        double d[UU], r[UU], e[UU];
#pragma unroll
        for (int i = 0; i < UU; ++i) {
            d[i] = 1.0 + t[i];
            r[i] = __builtin_amdgcn_rcp(d[i]);
        }
#pragma unroll
        for (int n = 0; n < 2; ++n) {                    // two Newton steps: <= 1 ulp
#pragma unroll
            for (int i = 0; i < UU; ++i) e[i] = fma(-d[i], r[i], 1.0);
#pragma unroll
            for (int i = 0; i < UU; ++i) r[i] = fma(r[i], e[i], r[i]);
        }
        double q[UU];
#pragma unroll
        for (int i = 0; i < UU; ++i) {
            const double inv = r[i];                     // p of the larger-logit class
            const double lo = t[i] * inv;                // p of the other class
            const bool neg = u[i] < 0.0;
            const bool ok = !MASKED || valid[i];
            q[i] = ok ? (neg ? inv : lo) : 0.0;
            prod *= ok ? (neg ? lo : inv) + 1e-16 : 1.0;
            wt.tmax = fmax(wt.tmax, ok ? t[i] : 0.0);
            hits += (ok && u[i] > 0.0) ? 1 : 0;
        }
#pragma unroll
        for (int i = 0; i < UU; ++i)
#pragma unroll
            for (int f = 0; f < F; ++f) acc[f] = fma(x[i][f], q[i], acc[f]);
    }

    // The first-maximum argmax of a tied row (t == 1): hit iff y == 0.
    template <bool MASKED>
    static __device__ __forceinline__ void fixup(const T (&x)[F], const T (&wd)[NB],
                                                 const int32_t *ys, int r, bool valid, T &,
                                                 int &hits) {
        const T u = margin(x, wd);
        const T t = exp_neg(fabs(u), MathConsts<T>());
        if ((MASKED && !valid) || !(t == T(1))) return;
        hits += (ys[r] == 0 ? 1 : 0) - (u > T(0) ? 1 : 0);
    }

    static __device__ __forceinline__ bool param_of(int m, int sub, int &j, T &sign) {
        j = 2 * m + sub;
        sign = sub == 0 ? T(-1) : T(1);
        return sub < 2 && m < F;
    }
    static __device__ __forceinline__ int owner_lane(int j, int shift) {
        return ((j >> 1) << shift) | (j & 1);
    }
};

template <int F, int K>
struct UseTwoClass { static constexpr bool value = signed_rows(F, K); };

// Rows of one lane between log folds of `prod` (factors in (1e-16, 1]:
// 16 of them stay above 1e-256).
constexpr int kProdFold = 16;

// UU chunks of 64 minibatch rows: minibatch row i -> dataset row order[i]
// (ORDERED) or row i.  FIX runs Model::fixup on them instead of Model::row.
template <typename Model, typename T, int F, bool MASKED, bool ORDERED, bool FIX, int UU, int NA>
__device__ __forceinline__ void rows_block(const T *xs, const int32_t *ys, const int32_t *order,
                                           int i, int B, const T (&w)[Model::NB], T (&acc)[NA],
                                           T &loss, T &prod, int &hits,
                                           typename Model::Watch &wt) {
    T x[UU][F];
    int r[UU];
    bool valid[UU];
#pragma unroll
    for (int u = 0; u < UU; ++u) {
        const int iu = i + u * kWave;
        valid[u] = !MASKED || iu < B;
        r[u] = valid[u] ? (ORDERED ? order[iu] : iu) : 0;
        load_row<T, F>(xs, r[u], x[u]);
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

// The minibatch pass: full groups of U chunks (64 rows each) run unmasked
// with U independent dependency chains in flight; a ragged tail runs one
// masked chunk at a time.  Then, only if some lane flagged a row, the
// exact fix-up pass over the same rows.
template <typename Model, typename T, int F, bool ORDERED, int NA>
__device__ __forceinline__ void minibatch_pass(const T *xs, const int32_t *ys,
                                               const int32_t *order, int lane, int B,
                                               const T (&w)[Model::NB], T (&acc)[NA],
                                               T &loss, int &hits) {
    constexpr int U = sizeof(T) == 8 ? 1 : 4;
    T prod = T(1);
    int since = 0;
    typename Model::Watch wt;
    const int full = B / (kWave * U) * (kWave * U);
    for (int i0 = 0; i0 < full; i0 += kWave * U) {
        rows_block<Model, T, F, false, ORDERED, false, U>(xs, ys, order, i0 + lane, B, w, acc,
                                                          loss, prod, hits, wt);
        if (Model::kProd && (since += U) >= kProdFold) {
            loss -= log_pos(prod);
            prod = T(1);
            since = 0;
        }
    }
    for (int i0 = full; i0 < B; i0 += kWave)
        rows_block<Model, T, F, true, ORDERED, false, 1>(xs, ys, order, i0 + lane, B, w, acc,
                                                         loss, prod, hits, wt);
    if (Model::kProd) loss -= log_pos(prod);
    if (Model::kFixup && __any(wt.flagged())) {
        for (int i0 = 0; i0 < B; i0 += kWave)
            rows_block<Model, T, F, true, ORDERED, true, 1>(xs, ys, order, i0 + lane, B, w, acc,
                                                            loss, prod, hits, wt);
    }
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

template <typename T, int F, int K, bool STAGED>
__global__ __launch_bounds__(kBlock) void optimize_step_kernel(StepArgs<T> a) {
    using Model = typename std::conditional<UseTwoClass<F, K>::value, TwoClassModel<T, F>,
                                            SoftmaxModel<T, F, K>>::type;
    constexpr int P = F * K;
    constexpr int OBS = 2 * P + 1;
    constexpr int NE = Model::NE;
    constexpr int NP = next_pow2(NE + 2);
    static_assert(NP <= kWave, "register path needs the reduced set to fit one wave");
    constexpr int SHIFT = 6 - Log2<NP>::value;

#ifdef CE_DIAG
    unsigned long long stamps[kStamps] = {0};
    stamps[6] = __builtin_amdgcn_s_memrealtime();   // 100 MHz, chip-wide
#endif
    CE_STAMP(0);
    const int lane = threadIdx.x & (kWave - 1);
    const int e = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const bool active = e < a.E;   // wave-uniform
    const size_t pbase = static_cast<size_t>(active ? e : 0) * P;
    const int N = a.N;

    // ---- per-env state loads first: their latency overlaps the staging copy.
    // Unconditional loads from clamped indices (inactive lanes and waves
    // read a valid element and discard it), so no branch separates a load
    // from its use and nothing waits on them before the staging barrier.
    int j_own;
    T sign_own;
    const bool owner = Model::param_of(lane >> SHIFT, lane & ((1 << SHIFT) - 1), j_own, sign_own);
    const int eidx = active ? e : 0;
    const int pl = lane < P ? lane : P - 1;
    const T w_raw = a.W[pbase + pl];
    const float a_raw = a.act[pbase + pl];
    const T g_raw = a.G[pbase + (owner ? j_own : 0)];
    const double lprev = a.L[eidx];
    const int step_prev = a.step[eidx];

    // ---- dataset: [rows | labels] staged into LDS once per block (16-byte copies).
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int RS = row_stride(F, sizeof(T));
    const size_t xbytes = align16_dev(sizeof(T) * RS * static_cast<size_t>(N));
    const T *xs;
    const int32_t *ys;
    if constexpr (STAGED) {
        // LDS-DMA (global_load_lds_dwordx4): each wave-instruction copies one
        // 1 KiB chunk straight into LDS (destination = chunk base + lane*16),
        // with no VGPR round trip; all of a wave's chunks are in flight at
        // once.  Every block reads the same few KB, so each block starts at
        // a rotated chunk to spread the 32 CUs of an XCD over the L2 lines.
        const int nvec = static_cast<int>(align16_dev(xbytes + 4 * static_cast<size_t>(N)) / 16);
        const int nch = (nvec + kWave - 1) / kWave;
        const int rot = static_cast<int>((blockIdx.x * 5u) % static_cast<unsigned>(nch));
        const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
        for (int c0 = wave; c0 < nch; c0 += kWavesPerBlock) {
            const int c = c0 + rot < nch ? c0 + rot : c0 + rot - nch;   // wave-uniform
            const int v = c * kWave + lane;
            if (v < nvec)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) void *)(a.data + static_cast<size_t>(v) * 16),
                    (__attribute__((address_space(3))) void *)(smem + c * kWave * 16), 16, 0, 0);
        }
        __syncthreads();
        CE_STAMP(1);
        xs = reinterpret_cast<const T *>(smem);
        ys = reinterpret_cast<const int32_t *>(smem + xbytes);
    } else {
        xs = reinterpret_cast<const T *>(a.data);
        ys = reinterpret_cast<const int32_t *>(a.data + xbytes);
    }
    if (!active) return;

    // ---- W <- W - a (optimize.py:74-75); lane j owns parameter j.
    const T gprev = owner ? g_raw : T(0);
    T wl = lane < P ? w_raw - static_cast<T>(a_raw) : T(0);
    T w[Model::NB];
    Model::broadcast(wl, w);
    const int cur_step = __builtin_amdgcn_readfirstlane(step_prev) + 1;
    CE_STAMP(2);

    // ---- minibatch rows: sequence[0] = rows [0, B) of the current order.
    const int32_t *order = nullptr;
    if (a.order != nullptr) {
        const int sel = __builtin_amdgcn_readfirstlane(a.order_sel[e]);
        order = a.order + sel * static_cast<size_t>(a.E) * N + static_cast<size_t>(e) * N;
    }
    T acc[NP];
#pragma unroll
    for (int j = 0; j < NP; ++j) acc[j] = T(0);
    T loss_l = T(0);
    int hits_l = 0;
    if (order)
        minibatch_pass<Model, T, F, true>(xs, ys, order, lane, a.B, w, acc, loss_l, hits_l);
    else
        minibatch_pass<Model, T, F, false>(xs, ys, nullptr, lane, a.B, w, acc, loss_l, hits_l);
    acc[NE] = loss_l;
    acc[NE + 1] = static_cast<T>(hits_l);
    CE_STAMP(3);
    ReduceScatter<T, NP, 32>::run(acc, lane);
    const T tot_loss = readlane(acc[0], NE << SHIFT);
    const T tot_hit = readlane(acc[0], (NE + 1) << SHIFT);
    const double loss = static_cast<double>(tot_loss) / a.B;
    double objective = loss, accuracy = static_cast<double>(tot_hit) / a.B;

    // ---- info pass over the full dataset (optimize.py:94-97); with B == N
    // the minibatch *is* the dataset and the reference computes the same
    // numbers twice, so they are reused.
    if (a.B != N) {
        T fl = T(0), fprod = T(1);
        int fh = 0, since = 0;
        T none[1];
        typename Model::Watch wt;
        for (int i0 = 0; i0 < N; i0 += kWave) {
            const int r = i0 + lane;
            const bool valid = r < N;
            const int rr = valid ? r : 0;
            T x[F];
            load_row<T, F>(xs, rr, x);
            Model::template row<false, true>(x, w, ys, rr, valid, none, fl, fprod, fh, wt);
            if (Model::kProd && ++since >= kProdFold) {
                fl -= log_pos(fprod);
                fprod = T(1);
                since = 0;
            }
        }
        if (Model::kProd) fl -= log_pos(fprod);
        if (Model::kFixup && __any(wt.flagged())) {
            for (int i0 = 0; i0 < N; i0 += kWave) {
                const int r = i0 + lane;
                const bool valid = r < N;
                const int rr = valid ? r : 0;
                T x[F];
                load_row<T, F>(xs, rr, x);
                Model::template fixup<true>(x, w, ys, rr, valid, fl, fh);
            }
        }
        objective = static_cast<double>(wave_sum(fl)) / N;
        accuracy = static_cast<double>(wave_sum(static_cast<T>(fh))) / N;
    }

    CE_STAMP(4);
    // ---- recurrences (optimize.py:80-86) and outputs.
    const double lnew = (loss - lprev) / (lprev + 0.1);
    const bool done = cur_step >= a.max_steps;
    const bool wipe = done && a.auto_reset;   // VecEnv auto-reset this step
    float *obs = a.obs + static_cast<size_t>(e) * OBS;
    float gnew_f = 0.0f;
    if (owner) {
        const T g = sign_own * acc[0] / static_cast<T>(a.B);
        const T gnew = g / (fabs(gprev) + T(1));
        if (!wipe) a.G[pbase + j_own] = gnew;
        gnew_f = static_cast<float>(gnew);
    }
    if (lane < P && !wipe) a.W[pbase + lane] = wl;
    // obs row = [0 (P) | L' | G' (P)], or the zero reset obs: one coalesced
    // store per 64 entries, G' gathered from its owner lanes.
#pragma unroll
    for (int i0 = 0; i0 < OBS; i0 += kWave) {
        const int i = i0 + lane;
        const int src = (i > P && i < OBS) ? Model::owner_lane(i - P - 1, SHIFT) : 0;
        const float gv = __shfl(gnew_f, src);
        float v = i < P ? 0.0f : (i == P ? static_cast<float>(lnew) : gv);
        if (wipe) v = 0.0f;
        if (i < OBS) obs[i] = v;
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
        }
    }
    if (wipe) reset_env<T, P>(a, e, lane);   // the returned obs was the reset obs (zeros)
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CE_STAMP(5);
    stamps[7] = __builtin_amdgcn_s_memrealtime();
    if (lane < kStamps) a.diag[static_cast<size_t>(e) * kStamps + lane] = stamps[lane];
#endif
}

}  // namespace ce
