// K consecutive Optimize-v0 steps in ONE launch: the two-class full-batch
// float64 step of optimize_lr_mfma.h (the benchmark shape), made persistent.
//
// What a step of the reference does (optimize.py:69-100 under the VecEnv
// auto-reset of utils_venv.py:31, K times in a row for
// concurrentvecenv.py:94-104's step_async / step_wait) only ever reads an
// env's own state, so a workgroup that owns 16 envs can run K steps back to
// back with no grid synchronisation.  Everything that is per-launch cost in
// the one-step kernel is paid once per K steps here:
//   - the state (W, W0, G, L, step counter) is loaded once, lives in VGPRs
//     across the K steps and is stored once at the end;
//   - the data set never leaves registers: a wave's row tiles (forward A
//     operand and the transposed gradient A operand, both in the
//     fragment-ordered image of ce_create) are loaded once, so a step issues
//     no tile loads and no LDS transposes;
//   - step t + 1's actions are loaded at the top of step t and consumed after
//     its row work (the load is hidden under ~2 us of f64 work);
//   - the launch boundary (~1.7 us) and the state round trip (~1 us,
//     DESIGN.md 3.9) are paid once per launch instead of once per step.
// Per step a wave issues only its f64 MFMA + softmax work, one s_barrier
// (its partial sums meet the other waves' in LDS, double-buffered by step
// parity so the next step's row work never waits for this step's
// epilogue), and the step's outputs: written through to the output record of
// step t, `out_step` bytes after step t - 1's (0: every step overwrites the
// same record, ce_step_many's contract).
//
// The arithmetic is the one-step kernel's, operation for operation (the same
// tile -> wave assignment and summation order, the same exp / reciprocal /
// log forms), so K steps here leave the state bit-identical to K one-step
// launches (tests/test_gpu_persist.py).
#pragma once

#include "optimize_lr_mfma.h"

namespace ce {

// The K-step launch's own arguments (beside StepArgs).
struct ManyArgs {
    int k;                 // steps in this launch
    long long act_stride;  // floats between consecutive steps' [E][P] action blocks
    long long out_step;    // bytes between consecutive steps' output records (0: overwrite)
};

constexpr int kLpWaves = 4;                   // default: one wave per SIMD (the one-step kernel's W = 4)
constexpr int kLpMaxTpw = 8;                  // row tiles a wave keeps in registers

// The gradient on v_mfma_f64_4x4x4f64 (4 blocks of 4x4x4: feature groups of
// 4 instead of 16 rows of M, 10 features in 12 instead of 16) where the
// feature groups are at most 3: 4 NKF of its ~0.26-time MFMAs per 4 rows
// against one 16x16x4 (CE_LP_G4=0 keeps the 16x16x4 form)
#ifndef CE_LP_G4
#define CE_LP_G4 1
#endif
// the 4x4x4 gradient's A operands transposed in-kernel from the forward
// operands (CE_LP_G4_XF=1) or loaded from the image's gradient slots (0)
#ifndef CE_LP_G4_XF
#define CE_LP_G4_XF 1
#endif
#ifndef CE_LP_EPI_SLEEP
#define CE_LP_EPI_SLEEP 0
#endif
#ifndef CE_LP_ROW_PRIO
#define CE_LP_ROW_PRIO 3
#endif
__host__ __device__ constexpr bool lp_g4(int nkf) { return CE_LP_G4 && nkf <= 3; }

// Row tiles per wave for N rows over W waves: the smallest of 1, 2, 4, 8
// covering the tiles; 0 when N needs more (the caller then launches step by
// step).
__host__ __device__ constexpr int lp_tpw(int N, int W = kLpWaves) {
    const int per = ((N + 15) / 16 + W - 1) / W;
    return per <= 1 ? 1 : per <= 2 ? 2 : per <= 4 ? 4 : per <= 8 ? 8 : 0;
}
// Padding rows or tiles present: the softmax masks them out of every statistic.
__host__ __device__ constexpr bool lp_pad(int N, int W = kLpWaves) {
    return N % 16 != 0 || (N + 15) / 16 != W * lp_tpw(N, W);
}

// Diagnostic builds (-DCE_DIAG): s_memrealtime (100 MHz, chip-wide) per wave
// at entry, prologue loaded, steps 0 / 1 / K-1 done (after the barrier),
// loop exit, final stores drained; row blockIdx W + wave of a.diag.
#ifdef CE_DIAG
#define LP_STAMP(k)                                                   \
    do {                                                              \
        __builtin_amdgcn_sched_barrier(0);                            \
        lp_st[k] = __builtin_amdgcn_s_memrealtime();                  \
        __builtin_amdgcn_sched_barrier(0);                            \
    } while (0)
#else
#define LP_STAMP(k) \
    do {            \
    } while (0)
#endif

template <int NKF, int TPW, bool PAD, int W>
__global__ __launch_bounds__(kWave * W) void optimize_lr_persist_kernel(StepArgs<double> a, ManyArgs m) {
    constexpr int BLK = kWave * W;
    constexpr int P_MAX = 2 * kLrMaxF;
    constexpr int TD = lr_tile_doubles(NKF);
    constexpr int PR = (kLrEnvs * P_MAX + BLK - 1) / BLK;   // (env, parameter) roles per thread
    constexpr int OSM = 2 * P_MAX + 4;                      // obs floats per env, padded
    constexpr int NG = TPW < 4 ? TPW : 4;                   // tiles per software-pipelined group
    __shared__ double red_s[2][W][4][kWave];                // per-wave gradient partials, by step parity
    __shared__ double red_l[2][W][kLrEnvs];                 // per-wave -log CE partials
    __shared__ double red_h[2][W][kLrEnvs];                 // per-wave hit counts
    __shared__ __attribute__((aligned(16))) float obs_s[2][kLrEnvs * OSM];
    __shared__ double tab_s[CE_LR_TEXP ? kLrExpTab : 1];   // the workgroup's exp table

#ifdef CE_DIAG
    unsigned long long lp_st[8] = {0};
#endif
    LP_STAMP(0);
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, h = lane >> 4;
    const int E = a.E, F = a.F, P = 2 * F, N = a.N, B = a.B;
    const int OS = a.obs_stride, OL = a.obs_lo;
    const int e0 = blockIdx.x * kLrEnvs;
    const int e = e0 + c;                                   // this lane's env (MFMA columns)
    const bool env_ok = e < E;
    const unsigned pbase = static_cast<unsigned>(env_ok ? e : 0) * P;
    const double *img = reinterpret_cast<const double *>(a.data);
    const int ntiles = (N + 15) / 16;

    // ---- once per launch: the state and the wave's row tiles into registers
#if CE_LR_TEXP
    // the exp table behind the image's column maxima, the first loads issued
    LrExpSlice<BLK> tslice;
    tslice.load(img + static_cast<unsigned>(ntiles) * TD + kLrMaxF, tid);
#endif
    unsigned ioff[NKF];                                     // element offset of (env c, feature 4k + h)
    double2 wv[NKF], w0v[NKF];
    float2 av[NKF];
#if CE_LR_NOCLAMP
    double xm[NKF];                                         // max_r |x[r][4k + h]|
    const double *colmax = img + static_cast<unsigned>(ntiles) * TD;
#endif
#pragma unroll
    for (int k = 0; k < NKF; ++k) {
        const int f = 4 * k + h;
        ioff[k] = pbase + (f < F ? 2 * f : 0);
        wv[k] = *reinterpret_cast<const double2 *>(a.W + ioff[k]);
        w0v[k] = *reinterpret_cast<const double2 *>(a.W0 + ioff[k]);
        av[k] = *reinterpret_cast<const float2 *>(a.act + ioff[k]);
#if CE_LR_NOCLAMP
        xm[k] = colmax[f];
#endif
    }
    // tile wave + W i: forward A X~[16t + c][4k + h], gradient A X~[16t + h + 4q][c]
    double xf[TPW][NKF], xg[TPW][4];
    unsigned vmask = 0;                                     // PAD: bit 4i + q = row 16t + h + 4q is real
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
        const int t = wave + W * i;
        const bool live = !PAD || t < ntiles;           // without padding every tile is real
        const double *ti = img + static_cast<unsigned>(live ? t : 0) * TD;
#pragma unroll
        for (int k = 0; k < NKF; ++k) xf[i][k] = live ? ti[k * kWave + lane] : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) xg[i][q] = live ? ti[(NKF + q) * kWave + lane] : 0.0;
        if constexpr (PAD) {
            const int2 ya = reinterpret_cast<const int2 *>(ti + (NKF + 4) * kWave)[lane];
            const int2 yb = reinterpret_cast<const int2 *>(ti + (NKF + 5) * kWave)[lane];
            const int ys[4] = {ya.x, ya.y, yb.x, yb.y};
#pragma unroll
            for (int q = 0; q < 4; ++q) vmask |= (live && ys[q] >= 0 ? 1u : 0u) << (4 * i + q);
        }
    }
    int step_c = a.step[env_ok ? e : 0];                    // env c's counter (the wipe of wv)
    // role "parameter": index i = j P + p < 16 P, i = tid + r BLK
    const int np_ = kLrEnvs * P;
    const int pmul = (65536 + P - 1) / P;
    int pj[PR], pp[PR], step_p[PR];
    bool prole[PR];
    unsigned gi[PR];
    double g_prev[PR], rG[PR];
#pragma unroll
    for (int r = 0; r < PR; ++r) {
        const int i = tid + r * BLK;
        pj[r] = (i * pmul) >> 16;
        pp[r] = i - pj[r] * P;
        prole[r] = i < np_ && e0 + pj[r] < E;
        gi[r] = static_cast<unsigned>(prole[r] ? e0 + pj[r] : 0) * P + (prole[r] ? pp[r] : 0);
        g_prev[r] = a.G[gi[r]];
        step_p[r] = a.step[prole[r] ? e0 + pj[r] : 0];
    }
    // role "scalar": the last 16 threads, one per env of the group
    const int sj = tid - (BLK - kLrEnvs);
    const bool srole = sj >= 0 && e0 + sj < E;
    const unsigned es = srole ? e0 + sj : 0;
    double lprev = a.L[es];
    int step_s = a.step[es];
#if CE_LR_TEXP
    tslice.store(tab_s, tid);                               // waits on the table loads only
    __syncthreads();
#endif
    const double dB = static_cast<double>(B), rB = a.inv_B;
    double rL = rcp_newton2(lprev + 0.1);
#pragma unroll
    for (int r = 0; r < PR; ++r) rG[r] = rcp_newton2(fabs(g_prev[r]) + 1.0);
    // the observation's weight block (wght_hist is identically 0,
    // optimize.py:84-86) is the same zeros every step: written into both
    // staging buffers once
    if (OL == 0)
        for (int i = tid; i < kLrEnvs * OS; i += BLK) {
            const int j = i / OS, p = i - j * OS;
            if (p < P) obs_s[0][i] = obs_s[1][i] = 0.0f;
        }

    // W' = W - a (optimize.py:74-75) and the forward B operand: the margin
    // w'_f0 - w'_f1 of feature 4k + h for env c
    double wd[NKF];
    auto margins = [&]() {
#pragma unroll
        for (int k = 0; k < NKF; ++k) {
            const int f = 4 * k + h;
            const double w0 = wv[k].x - static_cast<double>(av[k].x);
            const double w1 = wv[k].y - static_cast<double>(av[k].y);
            wv[k] = double2{w0, w1};
            wd[k] = f < F ? w0 - w1 : 0.0;
        }
    };
    margins();
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
    LP_STAMP(1);

    constexpr int QC = 4;                                   // exp chains in flight
    auto forward = [&](const double (&xv)[NKF]) {
        lr_d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < NKF; ++k) u = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[k], wd[k], u, 0, 0, 0);
        return u;
    };
    const int nenv = E - e0 < kLrEnvs ? E - e0 : kLrEnvs;
    // the staged observation block of one step: [e0 OS, (e0 + nenv) OS)
    // floats of that step's record, whole 16-B units in line order
    auto flush_obs = [&](int t) {
        float *ob = reinterpret_cast<float *>(reinterpret_cast<char *>(a.obs) + t * m.out_step) +
                    static_cast<unsigned>(e0) * OS;
        const float *src = obs_s[t & 1];
        const int nfl = nenv * OS, n4 = nfl >> 2;
        for (int i = tid; i < n4; i += BLK) {
            typedef float lp_f4 __attribute__((ext_vector_type(4)));
            const lp_f4 v = *reinterpret_cast<const lp_f4 *>(&src[4 * i]);
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(ob + 4 * i), "v"(v) : "memory");
        }
        for (int i = 4 * n4 + tid; i < nfl; i += BLK) lr_store(&ob[i], src[i]);
    };

    for (int t = 0; t < m.k; ++t) {
        const int buf = t & 1;
        // step t + 1's actions, consumed after this step's row work
        float2 an[NKF];
        {
            const float *actn = a.act + (t + 1 < m.k ? (t + 1) * m.act_stride : 0);
#pragma unroll
            for (int k = 0; k < NKF; ++k) an[k] = *reinterpret_cast<const float2 *>(actn + ioff[k]);
        }
#if CE_LR_NOCLAMP
        // |u| <= sum_f max_r |x_rf| |wd_f| < 650: no exp argument can leave
        // [-700, 750], the row work runs without the clamp (uniform choice)
        double ub = 0.0;
#pragma unroll
        for (int k = 0; k < NKF; ++k) ub = fma(fabs(wd[k]), xm[k], ub);
        // the lane's partial covers features 4k + h of env c: four partials
        // below 162.5 bound the sum below 650 (sufficient, no cross-lane fold)
        const bool bounded = __all(ub < 162.5);
#else
        const bool bounded = false;
#endif
        // ---- the row work: per group of NG tiles every forward chain, then
        // per tile the signed two-class softmax and its 4 gradient MFMAs
        lr_d4 sacc = {0.0, 0.0, 0.0, 0.0};                 // one gradient chain, tile order
        double prod = 1.0, nlog = 0.0, umin = 1.0;
        unsigned miss = 0;
        auto post = [&](double uq, double tq, bool valid, double &qo) {
#if CE_LR_RCP1
            const double inv = rcp_newton1(1.0 + tq);       // p_y
#else
            const double inv = rcp_unit(1.0 + tq);
#endif
            qo = valid ? tq * inv : 0.0;
            prod *= valid ? inv + 1e-16 : 1.0;
            {
                const double au = valid ? uq : 1.0;
                asm("v_min_f64 %0, %1, |%2|" : "=v"(umin) : "v"(umin), "v"(au));
            }
            miss += lr_miss(uq, valid);
        };
        auto rows = [&](auto clamp_c) {
#pragma unroll
            for (int g0 = 0; g0 < TPW; g0 += NG) {
                if (g0 > 0) {                               // 16 factors in (1e-16, 1]: fold
                    nlog -= log_pos(prod);
                    prod = 1.0;
                }
                lr_d4 u[NG];
#pragma unroll
                for (int i = 0; i < NG; ++i) u[i] = forward(xf[g0 + i]);
#pragma unroll
                for (int i = 0; i < NG; ++i) {
                    double qv[4];
#pragma unroll
                    for (int q0 = 0; q0 < 4; q0 += QC) {
                        double tx[QC];
#pragma unroll
                        for (int j = 0; j < QC; ++j) {
                            if constexpr (decltype(clamp_c)::value) tx[j] = clamp_u(u[i][q0 + j]);
                            else tx[j] = u[i][q0 + j];
                        }
                        lr_exp_neg<QC>(tx, tab_s);                  // t = e^-u
#pragma unroll
                        for (int j = 0; j < QC; ++j) {
                            const bool valid = !PAD || ((vmask >> (4 * (g0 + i) + q0 + j)) & 1u);
                            post(u[i][q0 + j], tx[j], valid, qv[q0 + j]);
                        }
                    }
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(xg[g0 + i][q], qv[q], sacc, 0, 0, 0);
                }
            }
        };
        if (bounded) rows(std::false_type{});
        else rows(std::true_type{});
        // a tie (p0 == p1, |u| < 2^-52) is np.argmax's class 0: hit iff y == 0;
        // only a wave that saw one re-walks its tiles exactly (practically never)
        int hits = 4 * TPW - static_cast<int>(miss);
        if (__any(umin < 0x1p-52)) {
#pragma unroll
            for (int i = 0; i < TPW; ++i) {
                const int tt = wave + W * i;
                if (tt >= ntiles) continue;
                const double *ti = img + static_cast<unsigned>(tt) * TD;
                const int2 ya = reinterpret_cast<const int2 *>(ti + (NKF + 4) * kWave)[lane];
                const int2 yb = reinterpret_cast<const int2 *>(ti + (NKF + 5) * kWave)[lane];
                const int yv[4] = {ya.x, ya.y, yb.x, yb.y};
                const lr_d4 uu = forward(xf[i]);
                double tx[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) tx[q] = abs_clamp750(uu[q]);
                exp_neg_multi_clamped<4>(tx);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (yv[q] >= 0 && tx[q] == 1.0) hits += (yv[q] == 0 ? 1 : 0) - lr_hit(uu[q]);
            }
        }
        // this wave's partials: s (features h + 4r of env c); -log of the
        // cross-entropy factors and the hits over the env's 4 lane groups
        double lsum = nlog - log_pos(prod);
        lsum = fold_pair<16>(lsum, lsum);
        lsum = fold_pair<32>(lsum, lsum);
        const double hsum = static_cast<double>(fold_env_lanes(hits));
#pragma unroll
        for (int r = 0; r < 4; ++r) red_s[buf][wave][r][lane] = sacc[r];
        if (lane < kLrEnvs) {
            red_l[buf][wave][lane] = lsum;
            red_h[buf][wave][lane] = hsum;
        }
        // the next step's weights: the auto-reset's W0 (utils_venv.py:31) or
        // W', then W'' = that - a_{t+1}
        {
            const bool wipe = step_c + 1 >= a.max_steps && a.auto_reset;
            step_c = wipe ? 0 : step_c + 1;
#pragma unroll
            for (int k = 0; k < NKF; ++k)
                if (wipe) wv[k] = w0v[k];
            if (t + 1 < m.k) {
#pragma unroll
                for (int k = 0; k < NKF; ++k) av[k] = an[k];
                margins();
            }
        }
        __syncthreads();                                    // the step's one workgroup barrier
#ifdef CE_DIAG
        if (t == 0) LP_STAMP(2);
        if (t == 1) LP_STAMP(3);
        if (t == m.k - 1) LP_STAMP(4);
#endif
        if (t > 0) flush_obs(t - 1);                        // staged behind this barrier

        // ---- epilogue of step t: the scalar and the parameter roles
        const long long ro = t * m.out_step;                // this step's record, bytes past step 0's
        if (srole) {
            double lt = 0.0, ht = 0.0;
#pragma unroll
            for (int w = 0; w < W; ++w) {
                lt += red_l[buf][w][sj];
                ht += red_h[buf][w][sj];
            }
            const double loss = div_rcp(lt, dB, rB);
            const double acc = div_rcp(ht, dB, rB);
            const double lnew = div_rcp(loss - lprev, lprev + 0.1, rL);
            const int cur = step_s + 1;
            const bool wipe = cur >= a.max_steps && a.auto_reset;
            if (a.reward) lr_store(reinterpret_cast<float *>(reinterpret_cast<char *>(a.reward) + ro) + es,
                                   static_cast<float>(-loss));
            lr_store(reinterpret_cast<float *>(reinterpret_cast<char *>(a.objective) + ro) + es,
                     static_cast<float>(loss));
            lr_store(reinterpret_cast<float *>(reinterpret_cast<char *>(a.accuracy) + ro) + es,
                     static_cast<float>(acc));
            if (a.done) (reinterpret_cast<uint8_t *>(a.done) + ro)[es] = cur >= a.max_steps ? 1 : 0;
            lr_store(reinterpret_cast<int32_t *>(reinterpret_cast<char *>(a.episode_len) + ro) + es, cur);
            obs_s[buf][sj * OS + P - OL] = wipe ? 0.0f : static_cast<float>(lnew);
            lprev = wipe ? 0.0 : lnew;
            step_s = wipe ? 0 : cur;
            rL = rcp_newton2(lprev + 0.1);
        }
#pragma unroll
        for (int r = 0; r < PR; ++r) {
            if (!prole[r]) continue;
            const bool wipe = step_p[r] + 1 >= a.max_steps && a.auto_reset;
            const int f = pp[r] >> 1;                       // parameter p = 2f + col
            double sf = 0.0;
#pragma unroll
            for (int w = 0; w < W; ++w) sf += red_s[buf][w][f >> 2][pj[r] + 16 * (f & 3)];
            const double g = div_rcp((pp[r] & 1) ? sf : -sf, dB, rB);
            const double gnew = div_rcp(g, fabs(g_prev[r]) + 1.0, rG[r]);
            obs_s[buf][pj[r] * OS + P + 1 + pp[r] - OL] = wipe ? 0.0f : static_cast<float>(gnew);
            g_prev[r] = wipe ? 0.0 : gnew;
            step_p[r] = wipe ? 0 : step_p[r] + 1;
            rG[r] = rcp_newton2(fabs(g_prev[r]) + 1.0);
        }
    }
    LP_STAMP(5);
    __syncthreads();
    if (m.k > 0) flush_obs(m.k - 1);
    // ---- the state after K steps, once
    if (wave == 0 && env_ok) {
#pragma unroll
        for (int k = 0; k < NKF; ++k)
            if (4 * k + h < F) {
                lr_store(a.W + ioff[k], wv[k].x);
                lr_store(a.W + ioff[k] + 1, wv[k].y);
            }
    }
#pragma unroll
    for (int r = 0; r < PR; ++r)
        if (prole[r]) lr_store(&a.G[gi[r]], g_prev[r]);
    if (srole) {
        lr_store(&a.L[es], lprev);
        lr_store(&a.step[es], step_s);
    }
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LP_STAMP(6);
    const int row = blockIdx.x * W + wave;
    if (row < E && lane < 8) a.diag[static_cast<size_t>(row) * 8 + lane] = lp_st[lane];
#endif
}


// The wave-specialised form: 4 ROW waves (one per SIMD, the row work of the
// kernel above, tile for tile) and 4 EPILOGUE waves (the scalar / parameter
// roles and the output stores) in one 512-thread workgroup.  Above, every
// wave runs the epilogue after the step's barrier, so its dependent f64
// chains (~0.6 us per step, the stamps of scripts/diag_persist.py) sit
// between two steps' row work.  Here the row waves go straight from the
// barrier into the next step's rows while the epilogue waves -- the younger,
// lower-priority wave of each SIMD -- turn the partials of the step just
// finished into its outputs, in the issue slots the row wave leaves; the
// next barrier finds them done.  The LDS partials and staged observation
// blocks are double-buffered by step parity, as above, so one barrier per
// step orders both (row waves: rows t, partials t -> buf, barrier t;
// epilogue waves: barrier t, flush obs t - 1, epilogue t from buf).  To fit
// two waves per SIMD (256 registers each) the gradient A operands live in
// the row wave's own LDS tiles instead of registers.  Same arithmetic, same summation
// order as optimize_lr_persist_kernel<NKF, TPW, PAD, 4>: bit-identical.
template <int NKF, int TPW, bool PAD>
__global__ __launch_bounds__(512) void optimize_lr_persist_ws_kernel(
    double *Wp, const float *actp, const unsigned char *datap, double *Gp, int32_t *stepp, double *Lp,
    unsigned efp, int Np, StepArgs<double> a, ManyArgs m) {
    constexpr int W = 4;                                    // row waves
    constexpr int BLK = 512;
    constexpr int EB = BLK - kWave * W;                     // epilogue threads
    constexpr int P_MAX = 2 * kLrMaxF;
    constexpr int TD = lr_tile_doubles(NKF);
    constexpr int PR = (kLrEnvs * P_MAX + EB - 1) / EB;
    constexpr int OSM = 2 * P_MAX + 4;
    constexpr int NG = TPW < 4 ? TPW : 4;
    __shared__ double red_s[2][W][4][kWave];
    __shared__ double red_l[2][W][kLrEnvs];
    __shared__ double red_h[2][W][kLrEnvs];
    __shared__ __attribute__((aligned(16))) float obs_s[2][kLrEnvs * OSM];
    // gradient A operands: the 16x16x4 form's tile slots, or for the 4x4x4
    // form (G4) X~[16t + 4j + k][4g + m] at [wave][tile][4k + m][j NKF + g],
    // a 14-double row stride per (k, m) so a row's ds_read_b128s meet no bank
    // twice
    constexpr bool G4 = lp_g4(NKF);
    constexpr int G4S = 14;
    __shared__ __attribute__((aligned(16))) double xgs[G4 ? 1 : W][G4 ? 1 : TPW][4][kWave];
    __shared__ __attribute__((aligned(16))) double xga[G4 ? W : 1][G4 ? TPW : 1][16][G4S];
    __shared__ double tab_s[CE_LR_TEXP ? kLrExpTab : 1];   // the row waves' exp table

#ifdef CE_DIAG
    unsigned long long lp_st[8] = {0};
#endif
    LP_STAMP(0);
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int c = lane & 15, h = lane >> 4;
    // the prologue's pointers and sizes as leading scalar arguments: built
    // with -amdgpu-kernarg-preload-count=14 (build.py) they arrive in SGPRs at
    // wave launch and the first loads need no kernel-argument load
    const int E = static_cast<int>(efp & 0xffffffu), F = static_cast<int>(efp >> 24), P = 2 * F, N = Np, B = a.B;
    const int OS = a.obs_stride, OL = a.obs_lo;
    const int e0 = blockIdx.x * kLrEnvs;
    const double *img = reinterpret_cast<const double *>(datap);
    const int ntiles = (N + 15) / 16;
    const int nenv = E - e0 < kLrEnvs ? E - e0 : kLrEnvs;

    // One workgroup barrier before the first step, for the shared exp table
    // (CE_LR_TEXP): a row wave's LDS tiles are its own (in-order within the
    // wave), W0 is in its registers, and the staging buffers are the
    // epilogue waves' alone.
#if CE_LR_TEXP
    // the exp table behind the image's column maxima, the first loads issued:
    // entries tid + 512 i, split over the row and the epilogue waves, one
    // workgroup barrier (the epilogue waves' first) before the first lookup
    LrExpSlice<BLK> tslice;
    tslice.load(img + static_cast<unsigned>(ntiles) * TD + kLrMaxF, tid);
#endif
    if (wave < W) {
        // ======================= row waves =======================
#if CE_LP_ROW_PRIO > 0
        __builtin_amdgcn_s_setprio(CE_LP_ROW_PRIO);      // experiment: row waves win arbitration
#endif
        const int e = e0 + c;
        const bool env_ok = e < E;
        const unsigned pbase = static_cast<unsigned>(env_ok ? e : 0) * P;
        unsigned ioff[NKF];
        double2 wv[NKF], w0v[NKF];
        float2 av[NKF];
#if CE_LR_NOCLAMP
        double xm[NKF];
        const double *colmax = img + static_cast<unsigned>(ntiles) * TD;
#endif
#pragma unroll
        for (int k = 0; k < NKF; ++k) {
            const int f = 4 * k + h;
            ioff[k] = pbase + (f < F ? 2 * f : 0);
            wv[k] = *reinterpret_cast<const double2 *>(Wp + ioff[k]);
            av[k] = *reinterpret_cast<const float2 *>(actp + ioff[k]);
#if CE_LR_NOCLAMP
            xm[k] = colmax[f];
#endif
        }
        double xf[TPW][NKF];
        // W0 (the auto-reset's weights) after the first step's operands: its
        // loads are not on the way to the first step's row work
#pragma unroll
        for (int k = 0; k < NKF; ++k) w0v[k] = *reinterpret_cast<const double2 *>(a.W0 + ioff[k]);
        unsigned vmask = 0;
#pragma unroll
        for (int i = 0; i < TPW; ++i) {
            const int t = wave + W * i;
            const bool live = !PAD || t < ntiles;
            const double *ti = img + static_cast<unsigned>(live ? t : 0) * TD;
#pragma unroll
            for (int k = 0; k < NKF; ++k) xf[i][k] = live ? ti[k * kWave + lane] : 0.0;
            if constexpr (G4) {
#if CE_LP_G4_XF
                // from the forward operands already in registers (no second
                // copy of the tile read from L2 in the prologue): lane (h, c)
                // holds X~[16t + c][4g + h] = xf[i][g], the A value of slot
                // (k = c & 3, m = h), column j = c >> 2, group g
                const int km = 4 * (c & 3) + h, j4 = c >> 2;
#pragma unroll
                for (int g = 0; g < NKF; ++g) xga[wave][i][km][j4 * NKF + g] = xf[i][g];
#else
                // lane (k, b, m) keeps feature group g = b: its own lane of the
                // tile's gradient slot j is X~[16t + 4j + k][4b + m]
                const int b4 = (lane >> 2) & 3, km = 4 * (lane >> 4) + (lane & 3);
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (b4 < NKF) xga[wave][i][km][q * NKF + b4] = live ? ti[(NKF + q) * kWave + lane] : 0.0;
#endif
            } else {
#pragma unroll
                for (int q = 0; q < 4; ++q) xgs[wave][i][q][lane] = live ? ti[(NKF + q) * kWave + lane] : 0.0;
            }
            if constexpr (PAD) {
                const int2 ya = reinterpret_cast<const int2 *>(ti + (NKF + 4) * kWave)[lane];
                const int2 yb = reinterpret_cast<const int2 *>(ti + (NKF + 5) * kWave)[lane];
                const int ys[4] = {ya.x, ya.y, yb.x, yb.y};
#pragma unroll
                for (int q = 0; q < 4; ++q) vmask |= (live && ys[q] >= 0 ? 1u : 0u) << (4 * i + q);
            }
        }
        int step_c = stepp[env_ok ? e : 0];
#if CE_LR_TEXP
        tslice.store(tab_s, tid);                           // waits on the table loads only
        __syncthreads();
#endif
        double wd[NKF];
        auto margins = [&]() {
#pragma unroll
            for (int k = 0; k < NKF; ++k) {
                const int f = 4 * k + h;
                const double w0 = wv[k].x - static_cast<double>(av[k].x);
                const double w1 = wv[k].y - static_cast<double>(av[k].y);
                wv[k] = double2{w0, w1};
                wd[k] = f < F ? w0 - w1 : 0.0;
            }
        };
        margins();
#ifdef CE_DIAG
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
        LP_STAMP(1);
        constexpr int QC = 4;
        auto forward = [&](const double (&xv)[NKF]) {
            lr_d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int k = 0; k < NKF; ++k) u = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[k], wd[k], u, 0, 0, 0);
            return u;
        };
        for (int t = 0; t < m.k; ++t) {
            const int buf = t & 1;
            float2 an[NKF];
            {
                const float *actn = actp + (t + 1 < m.k ? (t + 1) * m.act_stride : 0);
#pragma unroll
                for (int k = 0; k < NKF; ++k) an[k] = *reinterpret_cast<const float2 *>(actn + ioff[k]);
            }
#if CE_LR_NOCLAMP
            double ub = 0.0;
#pragma unroll
            for (int k = 0; k < NKF; ++k) ub = fma(fabs(wd[k]), xm[k], ub);
            // the lane's partial covers features 4k + h of env c: four partials
            // below 162.5 bound the sum below 650 (sufficient, no cross-lane fold)
            const bool bounded = __all(ub < 162.5);
#else
            const bool bounded = false;
#endif
            lr_d4 sacc = {0.0, 0.0, 0.0, 0.0};             // one gradient chain, tile order
            double gacc[NKF];                               // G4: one chain per feature group
#pragma unroll
            for (int g = 0; g < NKF; ++g) gacc[g] = 0.0;
            double prod = 1.0, nlog = 0.0, umin = 1.0;
            unsigned miss = 0;
            auto post = [&](double uq, double tq, bool valid, double &qo) {
#if CE_LR_RCP1
                const double inv = rcp_newton1(1.0 + tq);
#else
                const double inv = rcp_unit(1.0 + tq);
#endif
                qo = valid ? tq * inv : 0.0;
                prod *= valid ? inv + 1e-16 : 1.0;
                {
                    const double au = valid ? uq : 1.0;
                    asm("v_min_f64 %0, %1, |%2|" : "=v"(umin) : "v"(umin), "v"(au));
                }
                miss += lr_miss(uq, valid);
            };
            auto rows = [&](auto clamp_c) {
#pragma unroll
                for (int g0 = 0; g0 < TPW; g0 += NG) {
                    if (g0 > 0) {
                        nlog -= log_pos(prod);
                        prod = 1.0;
                    }
                    lr_d4 u[NG];
#pragma unroll
                    for (int i = 0; i < NG; ++i) u[i] = forward(xf[g0 + i]);
#pragma unroll
                    for (int i = 0; i < NG; ++i) {
                        double gv[G4 ? 4 * NKF : 4];
                        if constexpr (G4) {
                            typedef double lp_d2 __attribute__((ext_vector_type(2)));
                            const lp_d2 *src = reinterpret_cast<const lp_d2 *>(
                                &xga[wave][g0 + i][4 * (lane >> 4) + (lane & 3)][0]);
#pragma unroll
                            for (int p2 = 0; p2 < 2 * NKF; ++p2) {
                                const lp_d2 v = src[p2];
                                gv[2 * p2] = v.x;
                                gv[2 * p2 + 1] = v.y;
                            }
                        } else {
#pragma unroll
                            for (int q = 0; q < 4; ++q) gv[q] = xgs[wave][g0 + i][q][lane];
                        }
                        double qv[4];
#pragma unroll
                        for (int q0 = 0; q0 < 4; q0 += QC) {
                            double tx[QC];
#pragma unroll
                            for (int j = 0; j < QC; ++j) {
                                if constexpr (decltype(clamp_c)::value) tx[j] = clamp_u(u[i][q0 + j]);
                                else tx[j] = u[i][q0 + j];
                            }
                            lr_exp_neg<QC>(tx, tab_s);
#pragma unroll
                            for (int j = 0; j < QC; ++j) {
                                const bool valid = !PAD || ((vmask >> (4 * (g0 + i) + q0 + j)) & 1u);
                                post(u[i][q0 + j], tx[j], valid, qv[q0 + j]);
                            }
                        }
                        if constexpr (G4) {
                            // S[4g + m][4b + n] += X~[4q + k][4g + m] q[4q + k][4b + n]:
                            // the forward's C register q is the B operand as it stands
#pragma unroll
                            for (int q = 0; q < 4; ++q)
#pragma unroll
                                for (int g = 0; g < NKF; ++g)
                                    gacc[g] = __builtin_amdgcn_mfma_f64_4x4x4f64(gv[q * NKF + g], qv[q], gacc[g], 0, 0, 0);
                        } else {
#pragma unroll
                            for (int q = 0; q < 4; ++q)
                                sacc = __builtin_amdgcn_mfma_f64_16x16x4f64(gv[q], qv[q], sacc, 0, 0, 0);
                        }
                    }
                }
            };
            if (bounded) rows(std::false_type{});
            else rows(std::true_type{});
            int hits = 4 * TPW - static_cast<int>(miss);
            if (__any(umin < 0x1p-52)) {
#pragma unroll
                for (int i = 0; i < TPW; ++i) {
                    const int tt = wave + W * i;
                    if (tt >= ntiles) continue;
                    const double *ti = img + static_cast<unsigned>(tt) * TD;
                    const int2 ya = reinterpret_cast<const int2 *>(ti + (NKF + 4) * kWave)[lane];
                    const int2 yb = reinterpret_cast<const int2 *>(ti + (NKF + 5) * kWave)[lane];
                    const int yv[4] = {ya.x, ya.y, yb.x, yb.y};
                    const lr_d4 uu = forward(xf[i]);
                    double tx[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) tx[q] = abs_clamp750(uu[q]);
                    exp_neg_multi_clamped<4>(tx);
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        if (yv[q] >= 0 && tx[q] == 1.0) hits += (yv[q] == 0 ? 1 : 0) - lr_hit(uu[q]);
                }
            }
            double lsum = nlog - log_pos(prod);
            lsum = fold_pair<16>(lsum, lsum);
            lsum = fold_pair<32>(lsum, lsum);
            const double hsum = static_cast<double>(fold_env_lanes(hits));
            // S[f][env] at [f >> 2][16 (f & 3) + env] in both forms (rows past F unread)
            if constexpr (G4) {
#pragma unroll
                for (int g = 0; g < NKF; ++g) red_s[buf][wave][g][lane] = gacc[g];
            } else {
#pragma unroll
                for (int r = 0; r < 4; ++r) red_s[buf][wave][r][lane] = sacc[r];
            }
            if (lane < kLrEnvs) {
                red_l[buf][wave][lane] = lsum;
                red_h[buf][wave][lane] = hsum;
            }
            {
                const bool wipe = step_c + 1 >= a.max_steps && a.auto_reset;
                step_c = wipe ? 0 : step_c + 1;
                // one step in max_steps wipes: the selects behind a uniform branch
                if (__any(wipe)) {
#pragma unroll
                    for (int k = 0; k < NKF; ++k)
                        if (wipe) wv[k] = w0v[k];
                }
                if (t + 1 < m.k) {
#pragma unroll
                    for (int k = 0; k < NKF; ++k) av[k] = an[k];
                    margins();
                }
            }
#ifdef CE_DIAG
            if (t == 1) LP_STAMP(7);                        // step 1's row work done
#endif
            __syncthreads();                                // partials t -> the epilogue waves
#ifdef CE_DIAG
            if (t == 0) LP_STAMP(2);
            if (t == 1) LP_STAMP(3);
            if (t == m.k - 1) LP_STAMP(4);
#endif
        }
        LP_STAMP(5);
        __syncthreads();                                    // the epilogue's last obs block
        if (wave == 0 && env_ok) {
#pragma unroll
            for (int k = 0; k < NKF; ++k)
                if (4 * k + h < F) {
                    lr_store(Wp + ioff[k], wv[k].x);
                    lr_store(Wp + ioff[k] + 1, wv[k].y);
                }
        }
    } else {
        // ==================== epilogue waves ====================
        const int te = tid - kWave * W;                     // 0 .. EB - 1
        const int np_ = kLrEnvs * P;
        const int pmul = (65536 + P - 1) / P;
        int pj[PR], pp[PR], step_p[PR];
        bool prole[PR];
        unsigned gi[PR];
        double g_prev[PR], rG[PR];
#pragma unroll
        for (int r = 0; r < PR; ++r) {
            const int i = te + r * EB;
            pj[r] = (i * pmul) >> 16;
            pp[r] = i - pj[r] * P;
            prole[r] = i < np_ && e0 + pj[r] < E;
            gi[r] = static_cast<unsigned>(prole[r] ? e0 + pj[r] : 0) * P + (prole[r] ? pp[r] : 0);
            g_prev[r] = Gp[gi[r]];
            step_p[r] = stepp[prole[r] ? e0 + pj[r] : 0];
        }
        const int sj = te - (EB - kLrEnvs);
        const bool srole = sj >= 0 && e0 + sj < E;
        const unsigned es = srole ? e0 + sj : 0;
        double lprev = Lp[es];
        int step_s = stepp[es];
#if CE_LR_TEXP
        tslice.store(tab_s, tid);
#endif
        const double dB = static_cast<double>(B), rB = a.inv_B;
        double rL = rcp_newton2(lprev + 0.1);
#pragma unroll
        for (int r = 0; r < PR; ++r) rG[r] = rcp_newton2(fabs(g_prev[r]) + 1.0);
#if CE_LR_TEXP
        __syncthreads();                                    // the row waves' table barrier
#endif
        auto flush_obs = [&](int t) {
            float *ob = reinterpret_cast<float *>(reinterpret_cast<char *>(a.obs) + t * m.out_step) +
                        static_cast<unsigned>(e0) * OS;
            const float *src = obs_s[t & 1];
            const int nfl = nenv * OS, n4 = nfl >> 2;
            for (int i = te; i < n4; i += EB) {
                typedef float lp_f4 __attribute__((ext_vector_type(4)));
                const lp_f4 v = *reinterpret_cast<const lp_f4 *>(&src[4 * i]);
                asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(ob + 4 * i), "v"(v) : "memory");
            }
            for (int i = 4 * n4 + te; i < nfl; i += EB) lr_store(&ob[i], src[i]);
        };
        if (OL == 0)                                        // the weight block of both buffers
            for (int i = te; i < kLrEnvs * OS; i += EB) {
                const int j = i / OS, p = i - j * OS;
                if (p < P) obs_s[0][i] = obs_s[1][i] = 0.0f;
            }
        // x / B: with a power-of-two B, x rB is the exact quotient that
        // div_rcp's correction step would return (two operations fewer per
        // division; the epilogue's f64 work shares the row waves' pipe)
        auto epi_steps = [&](auto pow2_c) {
            auto divB = [&](double x) {
                if constexpr (decltype(pow2_c)::value) return x * rB;
                else return div_rcp(x, dB, rB);
            };
            for (int t = 0; t < m.k; ++t) {
                const int buf = t & 1;
                __syncthreads();                                // the row waves' partials of step t
#if CE_LP_EPI_SLEEP > 0
                // experiment: leave the row wave's forward MFMA block alone
                // (another wave's VALU between back-to-back f64 MFMAs stalls
                // them, profiles/r06_mfma_overlap.jsonl)
                __builtin_amdgcn_s_sleep(CE_LP_EPI_SLEEP);
#endif
    #ifdef CE_DIAG
                if (t == 1) LP_STAMP(2);                        // epilogue waves: step 1 starts
    #endif
                if (t > 0) flush_obs(t - 1);
                const long long ro = t * m.out_step;
                if (srole) {
                    double lt = 0.0, ht = 0.0;
    #pragma unroll
                    for (int w = 0; w < W; ++w) {
                        lt += red_l[buf][w][sj];
                        ht += red_h[buf][w][sj];
                    }
                    const double loss = divB(lt);
                    const double acc = divB(ht);
                    const double lnew = div_rcp(loss - lprev, lprev + 0.1, rL);
                    const int cur = step_s + 1;
                    const bool wipe = cur >= a.max_steps && a.auto_reset;
                    if (a.reward) lr_store(reinterpret_cast<float *>(reinterpret_cast<char *>(a.reward) + ro) + es,
                                           static_cast<float>(-loss));
                    lr_store(reinterpret_cast<float *>(reinterpret_cast<char *>(a.objective) + ro) + es,
                             static_cast<float>(loss));
                    lr_store(reinterpret_cast<float *>(reinterpret_cast<char *>(a.accuracy) + ro) + es,
                             static_cast<float>(acc));
                    if (a.done) (reinterpret_cast<uint8_t *>(a.done) + ro)[es] = cur >= a.max_steps ? 1 : 0;
                    lr_store(reinterpret_cast<int32_t *>(reinterpret_cast<char *>(a.episode_len) + ro) + es, cur);
                    float ol = static_cast<float>(lnew);
                    lprev = lnew;
                    step_s = cur;
                    if (__any(wipe)) {                          // the auto-reset's zeros
                        if (wipe) {
                            ol = 0.0f;
                            lprev = 0.0;
                            step_s = 0;
                        }
                    }
                    obs_s[buf][sj * OS + P - OL] = ol;
                    rL = rcp_newton2(lprev + 0.1);
                }
    #pragma unroll
                for (int r = 0; r < PR; ++r) {
                    if (!prole[r]) continue;
                    const bool wipe = step_p[r] + 1 >= a.max_steps && a.auto_reset;
                    const int f = pp[r] >> 1;
                    double sf = 0.0;
    #pragma unroll
                    for (int w = 0; w < W; ++w) sf += red_s[buf][w][f >> 2][pj[r] + 16 * (f & 3)];
                    const double g = divB((pp[r] & 1) ? sf : -sf);
                    const double gnew = div_rcp(g, fabs(g_prev[r]) + 1.0, rG[r]);
                    float og = static_cast<float>(gnew);
                    g_prev[r] = gnew;
                    step_p[r] = step_p[r] + 1;
                    if (__any(wipe)) {                          // the auto-reset's zeros
                        if (wipe) {
                            og = 0.0f;
                            g_prev[r] = 0.0;
                            step_p[r] = 0;
                        }
                    }
                    obs_s[buf][pj[r] * OS + P + 1 + pp[r] - OL] = og;
                    rG[r] = rcp_newton2(fabs(g_prev[r]) + 1.0);
                }
    #ifdef CE_DIAG
                if (t == 1) {                                   // step 1's epilogue issued and drained
                    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
                    LP_STAMP(7);
                }
    #endif
            }
        };
        if ((B & (B - 1)) == 0) epi_steps(std::true_type{});
        else epi_steps(std::false_type{});
        __syncthreads();                                    // the last step's obs block staged
        if (m.k > 0) flush_obs(m.k - 1);
#pragma unroll
        for (int r = 0; r < PR; ++r)
            if (prole[r]) lr_store(&Gp[gi[r]], g_prev[r]);
        if (srole) {
            lr_store(&Lp[es], lprev);
            lr_store(&stepp[es], step_s);
        }
    }
#ifdef CE_DIAG
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    LP_STAMP(6);
    const int row = blockIdx.x * 8 + wave;                  // 8 stamp rows per workgroup
    if (row < E && lane < 8) a.diag[static_cast<size_t>(row) * 8 + lane] = lp_st[lane];
#endif
}

}  // namespace ce
