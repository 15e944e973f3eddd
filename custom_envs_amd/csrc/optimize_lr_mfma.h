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
// Mapping: a workgroup owns 16 envs; its kLrWaves waves split the rows
// (16-row tiles t = wave, wave + kLrWaves, ...).  Rows come from a
// fragment-ordered image built once at ce_create (every MFMA operand one
// coalesced 8-byte load per lane, no LDS staging and no barrier before the
// math; staging the rows row-major into LDS by LDS-DMA and reading the
// operands from there was measured slower), the W' operands
// from the envs' state.  Each wave's partial sums
// (gradient, log-loss, hits) meet in LDS; the epilogue -- recurrences,
// observation, state, auto-reset (optimize.py:80-100, utils_venv.py:31) --
// is spread over the workgroup's threads.
#pragma once

#include "optimize_kernels.h"

namespace ce {

typedef double lr_d4 __attribute__((ext_vector_type(4)));

constexpr int kLrEnvs = 16;                    // envs per workgroup (MFMA N)
#ifndef CE_LR_WAVES
#define CE_LR_WAVES 8
#endif
constexpr int kLrWaves = CE_LR_WAVES;          // waves per workgroup (row split)
constexpr int kLrBlock = kWave * kLrWaves;
constexpr int kLrMaxF = 16;

static_assert(kLrEnvs * 2 * kLrMaxF <= kLrBlock, "one epilogue thread per (env, parameter)");

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
// (layout [tile][slot][lane]; built by the engine at ce_create)

// MODE (lr_mode): 0 = one tile at a time, padding rows (label -1) masked
// out of every statistic; 1 = N a multiple of 16 and every wave owning the
// same number of tiles, so the row loop reads no labels (the sign-folded
// rows carry y); 2 = as 1 with an even number of tiles per wave, run two at
// a time: both forward MFMA chains first, then softmax A, gradient MFMAs A,
// softmax B, gradient MFMAs B, so the matrix pipe works through one tile's
// MFMAs while the VALU does the other's softmax (f64 MFMA and f64 VALU have
// the same rate on gfx950; only the overlap gains).
__host__ __device__ constexpr int lr_mode(int N) {
    return N % 16 != 0 || ((N + 15) / 16) % kLrWaves != 0 ? 0
           : ((N + 15) / 16) % (2 * kLrWaves) == 0      ? 2
                                                          : 1;
}

template <int NKF, int MODE>
__global__ __launch_bounds__(kLrBlock) void optimize_lr_mfma_kernel(StepArgs<double> a) {
    constexpr int P_MAX = 2 * kLrMaxF;
    constexpr int TD = lr_tile_doubles(NKF);
    __shared__ double red[kLrWaves][6][kWave];          // per-wave partials
    __shared__ double tot[6][kWave];                    // workgroup totals
    __shared__ double wsh[kLrEnvs][P_MAX];              // W' of the group's envs
    __shared__ int wipe_sh[kLrEnvs];                    // auto-reset this step
#ifdef CE_DIAG
    unsigned long long stamps[kStamps] = {0};
    stamps[6] = __builtin_amdgcn_s_memrealtime();
#endif
    CE_STAMP(0);
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = lane & 15, h = lane >> 4;
    const int F = a.F, P = 2 * F, N = a.N;
    const int e0 = blockIdx.x * kLrEnvs;
    const int e = e0 + c;                               // this lane's env (columns)
    const bool env_ok = e < a.E;
    const size_t pbase = static_cast<size_t>(env_ok ? e : 0) * P;
    const double *img = reinterpret_cast<const double *>(a.data);
    const int ntiles = (N + 15) / 16;

    // ---- every state load of the step issued before any is used (one
    // memory round trip): W and the action of features 4k + h of env c
    // (forward B operand), then the epilogue's per (env, parameter) G and
    // W0 and per env L and the step counter
    double2 wv[NKF];
    float av0[NKF], av1[NKF];
#pragma unroll
    for (int k = 0; k < NKF; ++k) {
        const int f = 4 * k + h;
        const size_t i0 = pbase + (f < F ? 2 * f : 0);
        wv[k] = *reinterpret_cast<const double2 *>(a.W + i0);   // 16-B aligned: P even
        av0[k] = a.act[i0];
        av1[k] = a.act[i0 + 1];
    }
    const int tid = threadIdx.x;
    const int B = a.B;
    const int np_ = kLrEnvs * P;
    double g_prev = 0.0, w_init = 0.0;
    {
        const int j = tid / P;
        const int ee = e0 + (tid < np_ ? j : 0);
        const size_t gi = static_cast<size_t>(ee < a.E ? ee : 0) * P + (tid < np_ ? tid - j * P : 0);
        g_prev = a.G[gi];
        w_init = a.W0[gi];
    }
    const int es = e0 + (tid < kLrEnvs ? tid : 0);
    const double lprev = a.L[es < a.E ? es : 0];
    const int step_prev = a.step[es < a.E ? es : 0];

    // the wave's row tiles, each one's operands loaded a tile ahead
    constexpr bool PAD = MODE == 0;
    constexpr bool FULL = MODE == 2;
    // MFMA operands of tile t: forward A X~[16t + c][4k + h], gradient A
    // X~[16t + h + 4q][c], labels of rows 16t + h + 4q
    auto operands = [&](int t, double (&fv)[NKF], double (&gv)[4], int (&yv)[4], bool grad,
                        bool labels) {
        const double *ti = img + static_cast<size_t>(t) * TD;
#pragma unroll
        for (int k = 0; k < NKF; ++k) fv[k] = ti[k * kWave + lane];
        if (grad)
#pragma unroll
            for (int q = 0; q < 4; ++q) gv[q] = ti[(NKF + q) * kWave + lane];
        if (labels) {
            const int2 ya = reinterpret_cast<const int2 *>(ti + (NKF + 4) * kWave)[lane];
            const int2 yb = reinterpret_cast<const int2 *>(ti + (NKF + 5) * kWave)[lane];
            yv[0] = ya.x;
            yv[1] = ya.y;
            yv[2] = yb.x;
            yv[3] = yb.y;
        }
    };
    double xf[NKF], xg[4], xf2[NKF], xg2[4];
    int yl[4] = {0, 0, 0, 0}, yl2[4];
    auto load_tile = [&](int t) {
        operands(t, xf, xg, yl, true, PAD);
        if constexpr (FULL) operands(t + kLrWaves, xf2, xg2, yl2, true, false);   // the pair's second tile
    };
    if (wave < ntiles) load_tile(wave);

    // ---- W' = W - a (optimize.py:74-75); forward B operand: the margin
    // w'_f0 - w'_f1 of feature 4k + h for env c
    double wd[NKF];
#pragma unroll
    for (int k = 0; k < NKF; ++k) {
        const int f = 4 * k + h;
        const bool own = f < F;
        const double w0 = wv[k].x - static_cast<double>(av0[k]);
        const double w1 = wv[k].y - static_cast<double>(av1[k]);
        wd[k] = own ? w0 - w1 : 0.0;
        if (wave == 0 && own) {                         // kept for the epilogue
            wsh[c][2 * f] = w0;
            wsh[c][2 * f + 1] = w1;
        }
    }
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    CE_STAMP(1);

    lr_d4 s = {0.0, 0.0, 0.0, 0.0};
    double prod = 1.0, nlog = 0.0, tmax = 0.0;
    int hits = 0;
    int since = 0;
    // two-class softmax of TwoClassModel per (row, env): t = e^-|u|, p of
    // the larger logit 1/(1+t); q = 1 - p_y (the gradient weight).  Argmax
    // hit = u > 0 except on a tie (t == 1), which max(t) flags for the exact
    // pass after the loop.
    auto softmax = [&](const lr_d4 &u, const int (&ys)[4], double (&qv)[4]) {
        double tx[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) tx[q] = abs_clamp750(u[q]);
        exp_neg_multi_clamped<4>(tx);                   // t = e^-|u|, 4 chains interleaved
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const double uq = u[q];
            const double tq = tx[q];
            const double inv = rcp_unit(1.0 + tq);
            const double lo = tq * inv;
            const bool neg = uq < 0.0;
            const bool valid = !PAD || ys[q] >= 0;
            qv[q] = valid ? (neg ? inv : lo) : 0.0;
            prod *= valid ? (neg ? lo : inv) + 1e-16 : 1.0;
            tmax = fmax(tmax, valid ? tq : 0.0);
            hits += (valid && uq > 0.0) ? 1 : 0;
        }
    };
    auto forward = [&](const double (&xv)[NKF]) {
        lr_d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < NKF; ++k) u = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[k], wd[k], u, 0, 0, 0);
        return u;
    };
    auto gradient = [&](const double (&xv)[4], const double (&qv)[4]) {
#pragma unroll
        for (int q = 0; q < 4; ++q) s = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[q], qv[q], s, 0, 0, 0);
    };
#if defined(CE_LR_EXP) && (CE_LR_EXP == 1 || CE_LR_EXP == 3)
    const int t_first = ntiles;                         // experiment: no row work
#else
    const int t_first = wave;
#endif
    if constexpr (FULL) {
        const int none[4] = {0, 0, 0, 0};
        for (int t = t_first; t < ntiles; t += 2 * kLrWaves) {
            if (++since > 2) {                          // 16 factors in (1e-16, 1]: fold
                nlog -= log_pos(prod);
                prod = 1.0;
                since = 1;
            }
            double cf[NKF], cg[4], cf2[NKF], cg2[4];
#pragma unroll
            for (int k = 0; k < NKF; ++k) {
                cf[k] = xf[k];
                cf2[k] = xf2[k];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                cg[q] = xg[q];
                cg2[q] = xg2[q];
            }
            if (t + 2 * kLrWaves < ntiles) load_tile(t + 2 * kLrWaves);
            const lr_d4 ua = forward(cf);
            const lr_d4 ub = forward(cf2);
            double qa[4], qb[4];
            softmax(ua, none, qa);
            gradient(cg, qa);
            softmax(ub, none, qb);
            gradient(cg2, qb);
        }
    } else {
        const int none[4] = {0, 0, 0, 0};
        for (int t = t_first; t < ntiles; t += kLrWaves) {
            if (++since > 4) {                          // 16 factors in (1e-16, 1]: fold
                nlog -= log_pos(prod);
                prod = 1.0;
                since = 1;
            }
            double cf[NKF], cg[4];
#pragma unroll
            for (int k = 0; k < NKF; ++k) cf[k] = xf[k];
#pragma unroll
            for (int q = 0; q < 4; ++q) cg[q] = xg[q];
            const int ys[4] = {yl[0], yl[1], yl[2], yl[3]};
            if (t + kLrWaves < ntiles) load_tile(t + kLrWaves);
            double qv[4];
            softmax(forward(cf), PAD ? ys : none, qv);
            gradient(cg, qv);
        }
    }
    // a tie (p0 == p1) is np.argmax's class 0: hit iff y == 0.  Only a wave
    // that saw t == 1 re-walks its tiles (practically never: |z| < 2^-53).
    if (__any(tmax == 1.0)) {
        for (int t = wave; t < ntiles; t += kLrWaves) {
            double fv[NKF], gv[4];
            int ys[4];
            operands(t, fv, gv, ys, false, true);
            const lr_d4 u = forward(fv);
            double tx[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) tx[q] = abs_clamp750(u[q]);
            exp_neg_multi_clamped<4>(tx);
#pragma unroll
            for (int q = 0; q < 4; ++q)
                if (ys[q] >= 0 && tx[q] == 1.0) hits += (ys[q] == 0 ? 1 : 0) - (u[q] > 0.0 ? 1 : 0);
        }
    }
    // partials of this wave: s (features h + 4r of env c), -log of the
    // cross-entropy factors, hits
    red[wave][0][lane] = s[0];
    red[wave][1][lane] = s[1];
    red[wave][2][lane] = s[2];
    red[wave][3][lane] = s[3];
    red[wave][4][lane] = nlog - log_pos(prod);
    red[wave][5][lane] = static_cast<double>(hits);
    CE_STAMP(2);
    __syncthreads();
    if (wave < 6) {                                     // wave v sums value v over waves
        double acc = 0.0;
#pragma unroll
        for (int w = 0; w < kLrWaves; ++w) acc += red[w][wave][lane];
        if (wave >= 4) {                                // loss, hits: + lanes of the same env
            acc = fold_pair<16>(acc, acc);
            acc = fold_pair<32>(acc, acc);
        }
        tot[wave][lane] = acc;
    }
    __syncthreads();
    CE_STAMP(3);

    // ---- epilogue over the group's 16 envs, spread over the threads
#if defined(CE_LR_EXP) && (CE_LR_EXP == 2 || CE_LR_EXP == 3)
    if (tid < kLrEnvs && e0 + tid < a.E) a.reward[e0 + tid] = static_cast<float>(tot[4][tid]);
    return;                                             // experiment: no epilogue
#endif
    // per env scalars: thread j < 16 handles env e0 + j
    const int OBS = 2 * P + 1;
    if (tid < kLrEnvs && e0 + tid < a.E) {
        const int ee = e0 + tid;
        const double loss = tot[4][tid] / B;            // lane tid holds env tid, h = 0
        const double acc = tot[5][tid] / B;
        const int cur = step_prev + 1;
        const double lnew = (loss - lprev) / (lprev + 0.1);
        const bool done = cur >= a.max_steps;
        const bool wipe = done && a.auto_reset;
        a.reward[ee] = static_cast<float>(-loss);
        a.done[ee] = done ? 1 : 0;
        a.objective[ee] = static_cast<float>(loss);     // B == N: the same numbers
        a.accuracy[ee] = static_cast<float>(acc);
        a.episode_len[ee] = cur;
        a.obs[static_cast<size_t>(ee) * OBS + P] = wipe ? 0.0f : static_cast<float>(lnew);
        a.L[ee] = wipe ? 0.0 : lnew;
        a.step[ee] = wipe ? 0 : cur;
        wipe_sh[tid] = wipe ? 1 : 0;
    }
    __syncthreads();
    CE_STAMP(4);
    // per (env, parameter): W', G', obs, or the auto-reset's W0 / zeros
    if (tid < np_) {
        const int j = tid / P, p = tid - j * P;         // env e0 + j, parameter p = 2f + col
        const int ee = e0 + j;
        if (ee < a.E) {
            const bool wipe = wipe_sh[j] != 0;
            const size_t gi = static_cast<size_t>(ee) * P + p;
            const int f = p >> 1;
            // S[f][env j] sits on lane j + 16 (f & 3), register f >> 2
            const double sf = tot[f >> 2][j + 16 * (f & 3)];
            const double g = ((p & 1) ? sf : -sf) / B;
            const double gnew = g / (fabs(g_prev) + 1.0);
            float *obs = a.obs + static_cast<size_t>(ee) * OBS;
            obs[p] = 0.0f;                               // wght_hist is identically 0
            obs[P + 1 + p] = wipe ? 0.0f : static_cast<float>(gnew);
            a.W[gi] = wipe ? w_init : wsh[j][p];
            a.G[gi] = wipe ? 0.0 : gnew;
        }
    }
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    CE_STAMP(5);
    stamps[7] = __builtin_amdgcn_s_memrealtime();
    const int row = blockIdx.x * kLrWaves + wave;
    if (row < a.E && lane < kStamps) a.diag[static_cast<size_t>(row) * kStamps + lane] = stamps[lane];
#endif
}

}  // namespace ce
