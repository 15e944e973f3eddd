// Two-class Optimize-v0 step on the f64 matrix cores, envs along the MFMA
// N dimension (gfx950).  The benchmarked shape: load_data-style
// logistic regression, K = 2, full batch (batch_size=None, optimize.py:40),
// F <= 16 features.
//
// With B == N every env of the engine multiplies the SAME rows: the logit
// margins of 16 envs are one GEMM, U (rows x 16 envs) = X~ (rows x F) .
// Wd (F x 16 envs), and their gradients another, S (F x 16 envs) =
// X~^T (F x rows) . Q (rows x 16 envs).  X~ = s_y x (the sign-folded rows of
// TwoClassModel, optimize_kernels.h) gives u = s_y z directly; q is the
// probability of the other class, and column 0 of X^T (P - Y) is -S,
// column 1 is +S (optimize.py:74-78 with the A7 model).  So per 16 rows and
// 16 envs: ceil(F/4) forward MFMAs, the per-(row, env) two-class softmax on
// the VALU (one exp, one reciprocal), and 4 gradient MFMAs whose B operand
// is the forward's C registers as they stand: f64 C register q of lane l is
// row (l>>4) + 4q, env l&15 -- the B operand of k-step q.
//
// Mapping: a workgroup owns 16 envs; its W waves split the rows (16-row
// tiles t = wave, wave + W, ...).  Forward operands come from
// a fragment-ordered image built once at ce_create (one coalesced 8-byte
// load per lane per k-step, no LDS staging and no barrier before the math);
// the gradient's A operand is the same 16 x 16 tile transposed, so each
// wave turns its forward operands around through its own LDS tile instead
// of loading a second copy (the tile loads fell from 7 to 3 per 16 rows).
// Each wave's partial sums (gradient; log-loss and hits already folded over
// an env's 4 lane groups) meet in LDS behind the workgroup's ONE barrier;
// then a "scalar" thread per env (loss, accuracy, L', reward, done) and a
// "parameter" thread per (env, parameter) (G', W', obs) run side by side
// (optimize.py:80-100, utils_venv.py:31 auto-reset).  Loaded state is
// consumed before any store is issued (vmcnt counts stores too), the
// epilogue's divisors are known at the start, so their reciprocals are
// formed there and each quotient is 3 dependent FMAs (div_rcp).
// Measured anatomy: 1.7 us launch floor, ~1.0 us state
// round trip, ~2.5 us row work (softmax VALU ~1.4, f64 MFMA ~1.2: the f64
// matrix rate equals the f64 vector rate on gfx950), ~0.7 us epilogue.
#pragma once

#include <type_traits>

#include "optimize_kernels.h"

namespace ce {

typedef double lr_d4 __attribute__((ext_vector_type(4)));

// Round-3 levers (each a build switch for A/B runs; the defaults are the
// measured winners):
//  CE_LR_W0_LAZY  the reset weights W0 are loaded only for envs whose step
//                 wipes (1 step in 40), after the step counter has arrived
//  CE_LR_RCP1     1/(1 + t) from v_rcp_f64 plus ONE Newton step (<= 11 ulp,
//                 profiles/r01_rcp_accuracy.json) instead of two
//  CE_LR_NOCLAMP  a workgroup whose |u| bound (sum_f |w'_f0 - w'_f1| max_r
//                 |x_rf|, host-computed column maxima) stays below 650 runs
//                 the row loop without the exp argument clamp
#ifndef CE_LR_W0_LAZY
#define CE_LR_W0_LAZY 1
#endif
#ifndef CE_LR_RCP1
#define CE_LR_RCP1 1
#endif
#ifndef CE_LR_NOCLAMP
#define CE_LR_NOCLAMP 1
#endif
//  CE_LR_WT       the outputs and state are stored write-through (sc1: an
//                 agent-scope relaxed atomic store), so the launch ends with
//                 less dirty L2 for the kernel boundary to write back
//                 (rocprof average 6.29 -> 6.10 us per 4096-env launch)
#ifndef CE_LR_WT
#define CE_LR_WT 1
#endif
//  CE_LR_OBS_STAGE the workgroup's observation block (16 envs x obs_stride
//                 floats: line-aligned, whole lines) is assembled in LDS and
//                 stored 16 B per lane in line order, instead of the zero,
//                 L' and G' pieces each storing a part of every line.  PMC
//                 (4096 envs, profiles/r04_lr_writes.txt): writes 2.515 ->
//                 2.105 MB per launch (algorithmic 2.10), reads 2.11 -> 2.10;
//                 5.93-5.99 -> 6.00-6.03 us
#ifndef CE_LR_OBS_STAGE
#define CE_LR_OBS_STAGE 1
#endif
//  CE_LR_TEXP     e^-u through a 2048-entry table of 2^(j/2048) and a
//                 degree-3 polynomial (exp_neg_tab, 9 f64 operations per
//                 value) instead of the degree-10 polynomial over
//                 [-ln2/2, ln2/2] (exp_neg_q, 15): the row work is f64-pipe bound
#ifndef CE_LR_TEXP
#define CE_LR_TEXP 1
#endif
//  CE_LR_TGLOBAL  the one-step kernel reads the table entries straight from
//                 the image in global memory (L1 / L2) instead of copying the
//                 16 KB into LDS behind a barrier first (the K-step kernels
//                 keep their LDS copy: they pay for it once per K steps)
#ifndef CE_LR_TGLOBAL
#define CE_LR_TGLOBAL 1
#endif

constexpr int kLrEnvs = 16;                    // envs per workgroup (MFMA N)

// plain or write-through (CE_LR_WT) stores of 4- and 8-byte values
template <typename T>
__device__ __forceinline__ void lr_store(T *p, T v) {
    wt_store<CE_LR_WT != 0>(p, v);
}
constexpr int kLrMaxF = 16;
// Waves per workgroup W (the row split) is a template parameter: 8 waves
// (2 per SIMD, 2 tiles each) or 4 waves (1 per SIMD, 4 tiles per group,
// software-pipelined); lr_waves picks per launch (optimize_mfma.hip).
template <int W>
struct LrShape {
    static constexpr int kBlock = kWave * W;
    static constexpr int kParamSlots = (kLrEnvs * 2 * kLrMaxF + kBlock - 1) / kBlock;   // (env, parameter) roles per thread
};

__host__ __device__ constexpr bool lr_mfma_shape(int F, int K) { return K == 2 && F <= kLrMaxF; }
__host__ __device__ constexpr int lr_nkf(int F) { return (F + 3) / 4; }
// float64 operands per lane per 16-row tile: nkf forward A + 4 gradient A,
// then 4 int32 labels (-1 = padding row) as 2 float64 slots.
__host__ __device__ constexpr int lr_tile_doubles(int nkf) { return (nkf + 4 + 2) * kWave; }

// Image of tile t (rows 16t .. 16t + 15), lane l:
//   [k]        forward A  X~[16t + (l&15)][4k + (l>>4)]           k < nkf
//   [nkf + q]  gradient A X~[16t + (l>>4) + 4q][l&15]             q < 4
//   [nkf + 4]  int32 pair: labels of rows 16t + (l>>4) + 4q, q = 0, 1
//   [nkf + 5]  int32 pair: q = 2, 3
// (layout [tile][slot][lane]; built by the engine at ce_create), then
// kLrMaxF doubles: max over rows of |x[r][f]| (0 past F), the column maxima
// of the |u| bound (CE_LR_NOCLAMP), then the kLrExpTab entries 2^(j/2048) of
// exp_neg_tab

// MODE (lr_mode): 0 = one tile at a time, padding rows (label -1) masked
// out of every statistic; 1 = N a multiple of 16 and every wave owning the
// same number of tiles, so the row loop reads no labels (the sign-folded
// rows carry y); 2 / 3 = as 1 with the wave's tiles taken 2 / 4 at a time:
// all forward MFMA chains of the group first, then per tile softmax and
// gradient MFMAs, so the matrix pipe works through one tile's MFMAs while
// the VALU does another's softmax (f64 MFMA and f64 VALU have the same rate
// on gfx950; only the overlap gains).
__host__ __device__ constexpr int lr_mode(int N, int W) {
    return N % 16 != 0 || ((N + 15) / 16) % W != 0 ? 0
           : ((N + 15) / 16) % (4 * W) == 0 && W <= 4 ? 3
           : ((N + 15) / 16) % (2 * W) == 0           ? 2
                                                      : 1;
}

// exp argument range of the signed two-class form: t = e^-u for u clamped
// to [-700, 750] (e^700 < DBL_MAX; past either end p_y + 1e-16 and q are
// the same float64 numbers as unclamped)
__device__ __forceinline__ double clamp_u(double u) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(u), "v"(-700.0));
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(r), "v"(750.0));
    return r;
}

// 1/d for d in [1, 2^1010]: hardware reciprocal (~2^-24) + one Newton step,
// within 11 ulp (profiles/r01_rcp_accuracy.json); p_y and q feed sums whose
// float32 outputs are compared at 1e-6
__device__ __forceinline__ double rcp_newton1(double d) {
    const double r = __builtin_amdgcn_rcp(d);
    return fma(r, fma(-d, r, 1.0), r);
}

// 1/d for any normal finite d != 0: hardware reciprocal + two Newton steps
// (within an ulp; the residual step of div_rcp absorbs it)
__device__ __forceinline__ double rcp_newton2(double d) {
    double r = __builtin_amdgcn_rcp(d);
    r = fma(r, fma(-d, r, 1.0), r);
    return fma(r, fma(-d, r, 1.0), r);
}

// a / b from rb ~ 1/b (formed off the critical path):
// q0 = a rb, then one residual correction (Markstein) gives the correctly
// rounded quotient, as IEEE division does, in 3 dependent operations
__device__ __forceinline__ double div_rcp(double a, double b, double rb) {
    const double q0 = a * rb;
    return fma(fma(-q0, b, a), rb, q0);
}

// e^-x for Q arguments x in [-700, 750], the Q chains interleaved:
// m = rint(-x log2e) by the 1.5 2^52 shifter (the integer lands in the low
// word: no conversion instruction), r = -x - m ln2 in [-ln2/2, ln2/2],
// Horner on kExpCoef (three-operand FMAs, as exp_neg_multi_clamped), 2^m by
// ldexp
template <int Q>
__device__ __forceinline__ void exp_neg_q(double (&a)[Q]) {
    constexpr double kShift = 0x1.8p52;
    double big[Q], r[Q], q[Q];
#pragma unroll
    for (int i = 0; i < Q; ++i) {
        big[i] = fma(a[i], -kLog2e, kShift);
        const double m = big[i] - kShift;
        r[i] = fma(m, -kLn2Lo, fma(m, -kLn2Hi, -a[i]));
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
    for (int i = 0; i < Q; ++i)
        a[i] = ldexp(q[i], static_cast<int>(static_cast<unsigned long long>(__double_as_longlong(big[i]))));
}

// the row loops' exponential: the table form, or exp_neg_q (CE_LR_TEXP=0)
template <int Q>
__device__ __forceinline__ void lr_exp_neg(double (&a)[Q], const double *tab) {
#if CE_LR_TEXP
    exp_neg_tab<Q>(a, tab);
#else
    (void)tab;
    exp_neg_q<Q>(a);
#endif
}

// The argmax hit of a row by the sign bit of u (two integer operations per
// row instead of an f64 compare and a carry add): u > 0 and "sign clear"
// differ only at u = +0, a tie (|u| < 2^-52) that the exact re-walk after the
// row loop settles with lr_hit, the same test.  lr_miss is 1 for a row that
// is not a hit or not a real row (a padding row); hits = rows - misses.
__device__ __forceinline__ unsigned lr_miss(double u, bool valid) {
    const unsigned hi = static_cast<unsigned>(static_cast<unsigned long long>(__double_as_longlong(u)) >> 32);
    return valid ? hi >> 31 : 1u;
}
__device__ __forceinline__ int lr_hit(double u) { return __double_as_longlong(u) >= 0 ? 1 : 0; }

// sum of an int over lanes l, l^16, l^32, l^48 (permlane swaps)
__device__ __forceinline__ int fold_env_lanes(int v) {
    unsigned x = static_cast<unsigned>(v), y = x;
    swap_halves_u32<16>(x, y);
    x += y;
    y = x;
    swap_halves_u32<32>(x, y);
    return static_cast<int>(x + y);
}

// Everything the prologue's load addresses need -- the weights, actions,
// data-set image, G, step and L arrays, E | F << 24 and N -- comes as leading
// scalar arguments as well as in `a`: built with
// -amdgpu-kernarg-preload-count=14 (build.py) they arrive in SGPRs at wave
// launch, so every state and tile load issues without waiting for the
// kernel-argument load (~530 cycles)
template <int NKF, int MODE, int W>
__global__ __launch_bounds__(LrShape<W>::kBlock) void optimize_lr_mfma_kernel(
    double *Wp, const float *actp, const unsigned char *datap, double *Gp, int32_t *stepp, double *Lp,
    unsigned efp, int Np, StepArgs<double> a) {
    const int Ep = static_cast<int>(efp & 0xffffffu), Fp = static_cast<int>(efp >> 24);
    constexpr int kLrWaves = W;
    constexpr int kLrBlock = LrShape<W>::kBlock;
    constexpr int P_MAX = 2 * kLrMaxF;
    constexpr int TD = lr_tile_doubles(NKF);
    constexpr int NT = MODE == 3 ? 4 : MODE == 2 ? 2 : 1;   // row tiles per group
    constexpr int PR = LrShape<W>::kParamSlots;
    constexpr int XS = 17;                              // transpose row stride (doubles)
    __shared__ double xt[kLrWaves][NT][16 * XS];        // per-wave X~ tile transposes
    __shared__ double red_s[kLrWaves][4][kWave];        // per-wave gradient partials
    __shared__ double red_l[kLrWaves][kLrEnvs];         // per-wave -log CE partials
    __shared__ double red_h[kLrWaves][kLrEnvs];         // per-wave hit counts
    __shared__ __attribute__((aligned(16))) double wsh[kLrEnvs][P_MAX];   // W' of the group's envs
#if CE_LR_OBS_STAGE
    __shared__ __attribute__((aligned(16))) float obs_s[kLrEnvs * (2 * P_MAX + 4)];
#endif
    // the exp table, one copy per workgroup (one per wave at 4 waves, with no
    // barrier before the first lookup, measured 6.5e8 -> 5.9-6.1e8 env-steps/s
    // per-step launch, profiles/r05ai_*)
    constexpr bool TLDS = CE_LR_TEXP && !CE_LR_TGLOBAL;  // the table copied into LDS
    __shared__ double tab_s[TLDS ? kLrExpTab : 1];
#ifdef CE_DIAG
    unsigned long long stamps[kStamps] = {0};
    stamps[6] = __builtin_amdgcn_s_memrealtime();
#endif
    CE_STAMP(0);
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, h = lane >> 4;
    const int F = Fp, P = 2 * F, N = Np, B = a.B;
    // observation rows: obs_stride floats per env from entry obs_lo on (the
    // compact form, obs_lo = P, leaves out the identically-zero weight block)
    const int OS = a.obs_stride, OL = a.obs_lo;
    const int e0 = blockIdx.x * kLrEnvs;
    const int e = e0 + c;                               // this lane's env (columns)
    const bool env_ok = e < Ep;
    // 32-bit element offsets throughout: every load / store is a uniform
    // base (SGPRs) + a VGPR offset, no 64-bit address arithmetic
    const unsigned pbase = static_cast<unsigned>(env_ok ? e : 0) * P;
    const double *img = reinterpret_cast<const double *>(datap);
    const int ntiles = (N + 15) / 16;

    // ---- every load of the step issued before any is used (one memory
    // round trip), in the order they are needed (vmcnt retires in order):
    //  - W and the action of features 4k + h of env c (forward B operand);
    //  - the first group's row tiles (forward A operands);
    //  - role "parameter" (index i = j P + p < 16 P, i = tid + r kLrBlock):
    //    G and W0 of parameter p of env e0 + j and that env's step counter;
    //  - role "scalar" (the last 16 threads, one per env of the group): L
    //    and the step counter.
    // the exp table behind the image's column maxima
    const double *tab_g = img + static_cast<unsigned>(ntiles) * TD + kLrMaxF;
#if CE_LR_TEXP && !CE_LR_TGLOBAL
    // its LDS copy: the first loads issued
    LrExpSlice<kLrBlock> tslice;
    tslice.load(tab_g, tid);
#endif
    double2 wv[NKF];
    float2 av[NKF];
#if CE_LR_NOCLAMP
    double xm[NKF];                                     // max_r |x[r][4k + h]|
    const double *colmax = img + static_cast<unsigned>(ntiles) * TD;
#endif
#pragma unroll
    for (int k = 0; k < NKF; ++k) {
        const int f = 4 * k + h;
        const unsigned i0 = pbase + (f < F ? 2 * f : 0);
        wv[k] = *reinterpret_cast<const double2 *>(Wp + i0);   // 16-B aligned: P even
        av[k] = *reinterpret_cast<const float2 *>(actp + i0);  // 8-B aligned
#if CE_LR_NOCLAMP
        xm[k] = colmax[f];
#endif
    }
    // the wave's row tiles, each group's forward operands loaded a group ahead
    constexpr bool PAD = MODE == 0;
    // forward A of tile t: X~[16t + c][4k + h]; labels of rows 16t + h + 4q
    auto operands = [&](int t, double (&fv)[NKF], int (&yv)[4], bool labels) {
        const double *ti = img + static_cast<unsigned>(t) * TD;
#pragma unroll
        for (int k = 0; k < NKF; ++k) fv[k] = ti[k * kWave + lane];
        if (labels) {
            const int2 ya = reinterpret_cast<const int2 *>(ti + (NKF + 4) * kWave)[lane];
            const int2 yb = reinterpret_cast<const int2 *>(ti + (NKF + 5) * kWave)[lane];
            yv[0] = ya.x;
            yv[1] = ya.y;
            yv[2] = yb.x;
            yv[3] = yb.y;
        }
    };
    double xf[NT][NKF];
    int yl[NT][4] = {};
    auto load_group = [&](int t) {                      // tiles t, t + kLrWaves, ...
#pragma unroll
        for (int i = 0; i < NT; ++i) operands(t + i * kLrWaves, xf[i], yl[i], PAD && i == 0);
    };
    // the first group's tile loads right behind W and the action: the
    // G / step / L loads below are the epilogue's and may wait
    load_group(wave < ntiles ? wave : 0);              // unconditional: no merge-point vmcnt(0)
    const int np_ = kLrEnvs * P;
    const int pmul = (65536 + P - 1) / P;              // a.p_mul, formed here (uniform)
    int pj[PR], pp[PR], step_p[PR];
    bool prole[PR];
    unsigned gi[PR];
    double g_prev[PR], w_init[PR];
#pragma unroll
    for (int r = 0; r < PR; ++r) {
        const int i = tid + r * kLrBlock;
        pj[r] = (i * pmul) >> 16;                     // i / P, exact for i < 2^9
        pp[r] = i - pj[r] * P;
        prole[r] = i < np_ && e0 + pj[r] < Ep;
        gi[r] = static_cast<unsigned>(prole[r] ? e0 + pj[r] : 0) * P + (prole[r] ? pp[r] : 0);
        g_prev[r] = Gp[gi[r]];
#if CE_LR_W0_LAZY
        w_init[r] = 0.0;                                // loaded below, wiping envs only
#else
        w_init[r] = a.W0[gi[r]];
#endif
        step_p[r] = stepp[prole[r] ? e0 + pj[r] : 0];
    }
    const int sj = tid - (kLrBlock - kLrEnvs);
    const bool srole = sj >= 0 && e0 + sj < Ep;
    const unsigned es = srole ? e0 + sj : 0;
    const double lprev = Lp[es];
    const int step_prev = stepp[es];
#if CE_LR_TEXP && !CE_LR_TGLOBAL
    tslice.store(tab_s, tid);                           // waits on the table loads only
#endif


    // ---- W' = W - a (optimize.py:74-75); forward B operand: the margin
    // w'_f0 - w'_f1 of feature 4k + h for env c
    // (every wave loads the W / action pairs it needs itself: forming W'
    // once per workgroup in LDS behind a barrier measured slower at 4, 8
    // and 16 waves, 6.16 / 6.33 / 6.97 against 5.98 / 6.04 / 6.99 us)
    double wd[NKF];
#pragma unroll
    for (int k = 0; k < NKF; ++k) {
        const int f = 4 * k + h;
        const bool own = f < F;
        const double w0 = wv[k].x - static_cast<double>(av[k].x);
        const double w1 = wv[k].y - static_cast<double>(av[k].y);
        wd[k] = own ? w0 - w1 : 0.0;
        if (wave == 0 && own) {                         // kept for the epilogue
            wsh[c][2 * f] = w0;
            wsh[c][2 * f + 1] = w1;
        }
    }
#if CE_LR_NOCLAMP
    // |u| <= sum_f |x_f| |w'_f0 - w'_f1| <= sum_f max_r |x_rf| |wd_f| (the
    // rounding of u and of this sum is ~1e-15 relative): below 650, no u can
    // leave the exp's [-700, 750] argument range, so the row loop runs
    // without the clamp.  Every wave forms the same wd, so the choice is
    // uniform over the workgroup.
    double ub = 0.0;
#pragma unroll
    for (int k = 0; k < NKF; ++k) ub = fma(fabs(wd[k]), xm[k], ub);
    // the lane's partial covers features 4k + h of env c: four partials
    // below 162.5 bound the sum below 650 (sufficient, no cross-lane fold)
    const bool bounded = __all(ub < 162.5);
#else
    const bool bounded = false;
#endif
    const int cur = step_prev + 1;
    // the epilogue's divisors are known now: their reciprocals leave the
    // critical path (div_rcp)
    const double dB = static_cast<double>(B), dL = lprev + 0.1;
    double rB = a.inv_B, rL = rcp_newton2(dL);
    double rG[PR];
#pragma unroll
    for (int r = 0; r < PR; ++r) {
        rG[r] = rcp_newton2(fabs(g_prev[r]) + 1.0);
        // Pin the state values and the reciprocals in registers here.  vmcnt
        // counts stores too, so a first use of a loaded value in the
        // epilogue would wait for the completion of every store issued
        // before it; and left alone the compiler sinks the reciprocals into
        // the epilogue.
#if CE_LR_W0_LAZY
        asm volatile("" : "+v"(rG[r]) : "v"(step_p[r]));
#else
        asm volatile("" : "+v"(rG[r]) : "v"(w_init[r]), "v"(step_p[r]));
#endif
    }
    asm volatile("" : "+v"(rB), "+v"(rL));
#if CE_LR_W0_LAZY
    // W0 only where this step wipes (the auto-reset, utils_venv.py:31): one
    // step in 40; the load runs under the row work and is pinned after it
#pragma unroll
    for (int r = 0; r < PR; ++r)
        if (prole[r] && step_p[r] + 1 >= a.max_steps && a.auto_reset) w_init[r] = a.W0[gi[r]];
#endif
#if CE_LR_TEXP && !CE_LR_TGLOBAL
    __syncthreads();                                    // the table, before the first lookup
#endif
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    CE_STAMP(1);

    // ONE gradient accumulator chain over the wave's tiles in tile order (the
    // K-step kernels' order): each tile's MFMAs wait on the previous tile's
    // behind its softmax anyway, and no per-tile sums are left to add
    lr_d4 sacc = {0.0, 0.0, 0.0, 0.0};
    double prod = 1.0, nlog = 0.0, umin = 1.0;
    unsigned miss = 0;
    int rows_seen = 0;
    int since = 0;
    // two-class softmax of TwoClassModel per (row, env) in its signed form:
    // u = s_y z, t = e^-u, p_y = 1/(1+t), q = 1 - p_y = t p_y (the gradient
    // weight) -- no per-row selects.  Argmax hit = u > 0 except on a tie
    // (e^-|u| == 1, so |u| < 2^-52), which min |u| flags for the exact pass
    // after the loop.
    // QC exp chains at a time: 4 with 1-2 waves per SIMD (the wave's own
    // chains cover the f64 latency), 2 at 4 waves per SIMD (the other waves
    // cover it, and the 128-register budget has no room for 4)
    constexpr int QC = W >= 16 ? 2 : 4;
    // per (row, env) after the exp: p_y, q, the loss factor, min |u|, hit
    auto post = [&](double uq, double t, int y, double &qo) {
#if CE_LR_RCP1
        const double inv = rcp_newton1(1.0 + t);        // p_y
#else
        const double inv = rcp_unit(1.0 + t);           // p_y
#endif
        const bool valid = !PAD || y >= 0;
        qo = valid ? t * inv : 0.0;
        prod *= valid ? inv + 1e-16 : 1.0;
        // min(umin, |u|) as one v_min_f64 with the abs modifier (fmin of an
        // MFMA result gets a canonicalising v_max_f64 first)
        {
            const double au = valid ? uq : 1.0;
            asm("v_min_f64 %0, %1, |%2|" : "=v"(umin) : "v"(umin), "v"(au));
        }
        miss += lr_miss(uq, valid);
    };
    auto softmax = [&](auto clamp_c, const lr_d4 &u, const int (&ys)[4], double (&qv)[4]) {
#pragma unroll
        for (int q0 = 0; q0 < 4; q0 += QC) {
            double tx[QC];
#pragma unroll
            for (int i = 0; i < QC; ++i) {
                if constexpr (decltype(clamp_c)::value) tx[i] = clamp_u(u[q0 + i]);
                else tx[i] = u[q0 + i];
            }
            lr_exp_neg<QC>(tx, TLDS ? tab_s : tab_g);   // t = e^-u
#pragma unroll
            for (int i = 0; i < QC; ++i) post(u[q0 + i], tx[i], ys[q0 + i], qv[q0 + i]);
        }
    };
    auto forward = [&](const double (&xv)[NKF]) {
        lr_d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < NKF; ++k) u = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[k], wd[k], u, 0, 0, 0);
        return u;
    };
    // gradient A operand X~[16t + h + 4q][c] is the forward operand's tile
    // transposed: through the wave's own LDS tile (in-order LDS within a
    // wave; no barrier).  Feature rows c >= 4 NKF read a finite stand-in:
    // rows of S past F are never used.
    auto put = [&](int slot, const double (&fv)[NKF]) {
        double *x = &xt[wave][slot][0];
#pragma unroll
        for (int k = 0; k < NKF; ++k) x[c * XS + 4 * k + h] = fv[k];
        __builtin_amdgcn_wave_barrier();
    };
    auto gradient = [&](int slot, const double (&qv)[4]) {
        const double *x = &xt[wave][slot][0];
        const int cc = c < 4 * NKF ? c : 0;
        double gv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) gv[q] = x[(h + 4 * q) * XS + cc];
#pragma unroll
        for (int q = 0; q < 4; ++q) sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(gv[q], qv[q], sacc, 0, 0, 0);
        __builtin_amdgcn_wave_barrier();
    };
    // With two waves per SIMD, waves kLrWaves/2.. share SIMDs with the
    // older half and lose every VALU / matrix issue arbitration; one static
    // priority raise for the row work (6.17 -> 6.05 us per 4096-env launch
    // at 8 waves; a stagger of their tile order instead measured 6.30,
    // MI355X_MICROARCH.md "Two waves per SIMD" items 4 and 9)
    if (kLrWaves == 8 && wave >= kLrWaves / 2) __builtin_amdgcn_s_setprio(1);
#if defined(CE_LR_EXP) && (CE_LR_EXP == 1 || CE_LR_EXP == 3)
    const int t_first = ntiles;                         // experiment: no row work
#else
    const int t_first = wave;
#endif
    const int none[4] = {0, 0, 0, 0};
    auto row_loop = [&](auto clamp_c) {
    for (int t = t_first; t < ntiles; t += NT * kLrWaves) {
        since += NT;
        rows_seen += 4 * NT;
        if (since > 4) {                                // 16 factors in (1e-16, 1]: fold
            nlog -= log_pos(prod);
            prod = 1.0;
            since = NT;
        }
        // 1-2 waves per SIMD: the next group's operands load while this
        // one computes; 4 waves per SIMD: the other waves cover the load,
        // and the registers of a second copy are not there
        if constexpr (W >= 16)
            if (t != t_first) load_group(t);
        double cf[NT][NKF];
        int ys[NT][4];
#pragma unroll
        for (int i = 0; i < NT; ++i) {
#pragma unroll
            for (int k = 0; k < NKF; ++k) cf[i][k] = xf[i][k];
#pragma unroll
            for (int q = 0; q < 4; ++q) ys[i][q] = yl[i][q];
        }
        if constexpr (W < 16)
            if (t + NT * kLrWaves < ntiles) load_group(t + NT * kLrWaves);
        lr_d4 u[NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) u[i] = forward(cf[i]);
#pragma unroll
        for (int i = 0; i < NT; ++i) put(i, cf[i]);
#pragma unroll
        for (int i = 0; i < NT; ++i) {
            double qv[4];
            softmax(clamp_c, u[i], PAD ? ys[i] : none, qv);
            gradient(i, qv);
        }
    }
    };
    if (bounded) row_loop(std::false_type{});
    else row_loop(std::true_type{});
    // a tie (p0 == p1) is np.argmax's class 0: hit iff y == 0.  Only a wave
    // that saw |u| < 2^-52 re-walks its tiles with the exact test e^-|u| == 1
    // (practically never).
    int hits = rows_seen - static_cast<int>(miss);
    if (__any(umin < 0x1p-52)) {
        for (int t = wave; t < ntiles; t += kLrWaves) {
            double fv[NKF];
            int yv[4];
            operands(t, fv, yv, true);
            const lr_d4 uu = forward(fv);
            double tx[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) tx[q] = abs_clamp750(uu[q]);
            exp_neg_multi_clamped<4>(tx);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (yv[q] >= 0 && tx[q] == 1.0) hits += (yv[q] == 0 ? 1 : 0) - lr_hit(uu[q]);
        }
    }
#if CE_LR_W0_LAZY
#pragma unroll
    for (int r = 0; r < PR; ++r) asm volatile("" : "+v"(w_init[r]));
#endif
    // outputs nothing reads back in this launch, issued once the row loop
    // has consumed its loads (vmcnt counts stores as well): the
    // observation's weight part (wght_hist is identically 0), done and the
    // episode length
#if CE_LR_OBS_STAGE
#pragma unroll
    for (int r = 0; r < PR; ++r)
        if (prole[r] && OL == 0) obs_s[pj[r] * OS + pp[r]] = 0.0f;
#else
#pragma unroll
    for (int r = 0; r < PR; ++r)
        if (prole[r] && OL == 0) lr_store(&a.obs[static_cast<unsigned>(e0 + pj[r]) * OS + pp[r]], 0.0f);
#endif
    if (srole) {
        if (a.done) a.done[es] = cur >= a.max_steps ? 1 : 0;
        lr_store(&a.episode_len[es], cur);
    }
    // partials of this wave: s (features h + 4r of env c); -log of the
    // cross-entropy factors and the hits summed over the env's 4 lane groups
    double lsum = nlog - log_pos(prod);
    lsum = fold_pair<16>(lsum, lsum);
    lsum = fold_pair<32>(lsum, lsum);
    const double hsum = static_cast<double>(fold_env_lanes(hits));
#pragma unroll
    for (int r = 0; r < 4; ++r) red_s[wave][r][lane] = sacc[r];
    if (lane < kLrEnvs) {
        red_l[wave][lane] = lsum;
        red_h[wave][lane] = hsum;
    }
    CE_STAMP(2);
    __syncthreads();                                    // the one workgroup barrier
    CE_STAMP(3);

    // ---- epilogue: the scalar and the parameter roles run side by side
#if defined(CE_LR_EXP) && (CE_LR_EXP == 2 || CE_LR_EXP == 3)
    if (srole && a.reward) a.reward[es] = static_cast<float>(red_l[0][sj]);
    return;                                             // experiment: no epilogue
#endif
    if (srole) {
        double lt = 0.0, ht = 0.0;
#pragma unroll
        for (int w = 0; w < kLrWaves; ++w) {
            lt += red_l[w][sj];
            ht += red_h[w][sj];
        }
        const double loss = div_rcp(lt, dB, rB);
        const double acc = div_rcp(ht, dB, rB);
        const double lnew = div_rcp(loss - lprev, dL, rL);
        const bool wipe = cur >= a.max_steps && a.auto_reset;
        if (a.reward) lr_store(&a.reward[es], static_cast<float>(-loss));   // compact: -objective
        lr_store(&a.objective[es], static_cast<float>(loss));   // B == N: the same numbers
        lr_store(&a.accuracy[es], static_cast<float>(acc));
#if CE_LR_OBS_STAGE
        obs_s[sj * OS + P - OL] = wipe ? 0.0f : static_cast<float>(lnew);
#else
        lr_store(&a.obs[es * OS + P - OL], wipe ? 0.0f : static_cast<float>(lnew));
#endif
        lr_store(&Lp[es], wipe ? 0.0 : lnew);
        lr_store(&stepp[es], wipe ? 0 : cur);
    }
    // per (env, parameter): W', G', obs, or the auto-reset's W0 / zeros
#pragma unroll
    for (int r = 0; r < PR; ++r) {
        if (!prole[r]) continue;
        const bool wipe = step_p[r] + 1 >= a.max_steps && a.auto_reset;
        const int f = pp[r] >> 1;                       // parameter p = 2f + col
        // S[f][env j] sits on lane j + 16 (f & 3), register f >> 2
        double sf = 0.0;
#pragma unroll
        for (int w = 0; w < kLrWaves; ++w) sf += red_s[w][f >> 2][pj[r] + 16 * (f & 3)];
        const double g = div_rcp((pp[r] & 1) ? sf : -sf, dB, rB);
        const double gnew = div_rcp(g, fabs(g_prev[r]) + 1.0, rG[r]);
#if CE_LR_OBS_STAGE
        obs_s[pj[r] * OS + P + 1 + pp[r] - OL] = wipe ? 0.0f : static_cast<float>(gnew);
#else
        lr_store(&a.obs[static_cast<unsigned>(e0 + pj[r]) * OS + P + 1 + pp[r] - OL],
                 wipe ? 0.0f : static_cast<float>(gnew));
#endif
        lr_store(&Wp[gi[r]], wipe ? w_init[r] : wsh[pj[r]][pp[r]]);
        lr_store(&Gp[gi[r]], wipe ? 0.0 : gnew);
    }
#if CE_LR_OBS_STAGE
    __syncthreads();
    {   // the block [e0 OS, (e0 + nenv) OS) floats: 64-B aligned (16 OS floats per full group)
        const int nenv = Ep - e0 < kLrEnvs ? Ep - e0 : kLrEnvs;
        const int nfl = nenv * OS, n4 = nfl >> 2;
        float *ob = a.obs + static_cast<unsigned>(e0) * OS;
        for (int i = tid; i < n4; i += kLrBlock) {
            typedef float lr_f4 __attribute__((ext_vector_type(4)));
            const lr_f4 v = *reinterpret_cast<const lr_f4 *>(&obs_s[4 * i]);
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(ob + 4 * i), "v"(v) : "memory");
        }
        for (int i = 4 * n4 + tid; i < nfl; i += kLrBlock) lr_store(&ob[i], obs_s[i]);
    }
#endif
    CE_STAMP(4);
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CE_STAMP(5);
    stamps[7] = __builtin_amdgcn_s_memrealtime();
    const int row = blockIdx.x * kLrWaves + wave;
    if (row < Ep && lane < kStamps) a.diag[static_cast<size_t>(row) * kStamps + lane] = stamps[lane];
#endif
}

}  // namespace ce
