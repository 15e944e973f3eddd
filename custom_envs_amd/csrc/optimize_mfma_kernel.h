// Optimize-v0 step for any data-set shape on the f64 matrix cores (gfx950).
//
// The register-path kernels (optimize_kernels.h, optimize_pair_kernel.h)
// are compiled per (F, K) and keep a whole dataset in one workgroup's LDS.
// The reference's default data sets do not fit that: load_data('mnist' |
// 'fashion' | 'emnist-digits') is 60,000 rows of 7x7 = 49 features and 10
// classes (custom_envs/data/load_data.py:65-97; Optimize.__init__ defaults
// to data_set='mnist', batch_size=None, custom_envs/envs/optimize.py:40), so
// one step of one env is X_b W (N x 49 x 10), a softmax, and X_b^T (P - Y)
// (optimize.py:74-78, the build-defined ModelNumpy): two dense
// GEMMs.  This kernel runs them on v_mfma_f64_16x16x4_f64 for any F <= 64,
// K <= 16, N and B, in float64 (the reference's dtype).
//
// Mapping: one wave per env, kGenWaves envs per workgroup.  The dataset
// streams through LDS in blocks of 64 rows (LDS-DMA, double-buffered), so
// one HBM/L2 read of a block serves the workgroup's 8 envs.  Per 16-row
// sub-block and env:
//   forward   Z^T (16 classes x 16 rows) = W'^T (16 x 4nk) . X^T (4nk x 16):
//             nk = ceil(F/4) MFMAs; A = W'[4k + l>>4][l&15], held in
//             registers for the whole step, B = X[row l&15][4k + l>>4] from
//             LDS.
//   softmax   f64 MFMA C layout: lane l holds row l&15, classes (l>>4) + 4q,
//             q = 0..3: a row's 16 classes are 4 registers of 4 lanes
//             (l, l^16, l^32, l^48), so max / sum / first-argmax are an
//             in-register step plus two permlane-swap levels.
//   gradient  G (16 features x 16 classes) += X^T (16 x 4 rows) . D (4 rows
//             x 16 classes) per feature tile, D = P - Y transposed through a
//             2 KB per-wave LDS tile: A = X[row 4r + (l>>4)][16 ft + (l&15)],
//             B = D[row 4r + (l>>4)][class l&15]; 4 * ceil(F/16) MFMAs, no
//             cross-lane reduction (the row sum is the MFMA's k).
// Minibatches (B < N) gather their B rows per env through the env's row
// order straight from HBM/L2; the full-data info pass (optimize.py:94-97)
// is then the LDS stream without the gradient.  With B == N the reference
// computes the same numbers twice; they are reused.
// Cross-entropy is -log(p_y + 1e-16) per row (utils_math.py:25-34), taken
// as -log of per-lane products folded once per block; the argmax is
// np.argmax's first maximum of P.
#pragma once

#include "optimize_kernels.h"

namespace ce {

typedef double gen_d4 __attribute__((ext_vector_type(4)));

constexpr int kGenWaves = 8;                   // envs per workgroup, one wave each
constexpr int kGenBlock = kWave * kGenWaves;
constexpr int kGenRows = 64;                   // dataset rows per LDS block
constexpr int kGenMaxFT = 4;                   // feature tiles of 16: F <= 64
constexpr int kGenMaxNK = 16;                  // forward k-steps of 4 features
constexpr int kGenMaxK = 16;                   // classes: one 16-wide tile
constexpr int kGenResetWaves = 16;

__host__ __device__ constexpr int gen_ft(int F) { return (F + 15) / 16; }
// float64 per stored row: 16 FT features (zero-padded), one pad, the label
// (as a double; -1 marks the rows that pad N up to a whole block).  An odd
// number of 16-byte units keeps the forward's A reads conflict-free.
__host__ __device__ constexpr int gen_stride(int ft) { return 16 * ft + 2; }
__host__ __device__ constexpr size_t gen_block_bytes(int ft) {
    return static_cast<size_t>(kGenRows) * gen_stride(ft) * sizeof(double);
}
__host__ __device__ constexpr size_t gen_lds_bytes(int ft) {
    return 2 * gen_block_bytes(ft) + kGenWaves * 16 * 17 * sizeof(double);
}
__host__ __device__ constexpr int gen_rows_padded(int N) {
    return (N + kGenRows - 1) / kGenRows * kGenRows;
}

// max / min / sum with the lane l ^ OFF (OFF = 16, 32): one permlane swap
// per 32-bit half leaves {own, partner} in the two registers.
template <int OFF>
__device__ __forceinline__ double lane_max(double v) {
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
    unsigned lo = static_cast<unsigned>(b), hi = static_cast<unsigned>(b >> 32);
    unsigned lo2 = lo, hi2 = hi;
    swap_halves_u32<OFF>(lo, lo2);
    swap_halves_u32<OFF>(hi, hi2);
    const double x = __longlong_as_double(static_cast<long long>(
        (static_cast<unsigned long long>(hi) << 32) | lo));
    const double y = __longlong_as_double(static_cast<long long>(
        (static_cast<unsigned long long>(hi2) << 32) | lo2));
    return fmax(x, y);
}
template <int OFF>
__device__ __forceinline__ int lane_min(int v) {
    unsigned a = static_cast<unsigned>(v), b = a;
    swap_halves_u32<OFF>(a, b);
    return min(static_cast<int>(a), static_cast<int>(b));
}

// The softmax classifier on one row (utils_math.py:51-63, 25-34 and the A7
// model), spread over 4 lanes x 4 registers: z[q] is class h + 4q of the
// row.  Writes P - Y to d[q] (0 for padded rows / classes), multiplies the
// row's cross-entropy factor p_y + 1e-16 into `prod` and adds the argmax
// hit, both on the lane holding the label class.
//   Branch-free: padded classes are selected out, never branched around.
__device__ __forceinline__ void gen_softmax(const gen_d4 &z, int h, int K, int y, double (&d)[4],
                                            double &prod, int &hits) {
    const bool valid = y >= 0;
    bool cls[4];
    double m = -INFINITY;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        cls[q] = h + 4 * q < K;
        m = cls[q] ? fmax(m, z[q]) : m;
    }
    m = lane_max<32>(lane_max<16>(m));
    // exp(z - max), branch-free over the 3 (K <= 12) or 4 class registers
    double ex[4], s = 0.0;
    if (K <= 12) {
        double x[3];
#pragma unroll
        for (int q = 0; q < 3; ++q) x[q] = cls[q] ? m - z[q] : 750.0;
        exp_neg_multi<3>(x);
#pragma unroll
        for (int q = 0; q < 3; ++q) ex[q] = cls[q] ? x[q] : 0.0;
        ex[3] = 0.0;
    } else {
        double x[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = cls[q] ? m - z[q] : 750.0;
        exp_neg_multi<4>(x);
#pragma unroll
        for (int q = 0; q < 4; ++q) ex[q] = cls[q] ? x[q] : 0.0;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) s += ex[q];
    s = fold_pair<16>(s, s);                     // + lane l^16, then l^32: the row's 4 lanes
    s = fold_pair<32>(s, s);
    const double inv = 1.0 / s;
    // P = ex * (1/s): the row-max classes have ex = exp_neg(0) = 1 exactly,
    // so max(P) = inv and argmax(P) = the first class whose p equals it
    // (np.argmax's first maximum, on this P; the reference's p_exp / p_sum
    // differs from it by at most an ulp)
    int first = 99;
    double p[4];
#pragma unroll
    for (int q = 3; q >= 0; --q) {
        p[q] = ex[q] * inv;
        first = (cls[q] && p[q] == inv) ? h + 4 * q : first;
    }
    first = lane_min<32>(lane_min<16>(first));
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const bool own = valid && h + 4 * q == y;
        hits += (own && first == y) ? 1 : 0;
        prod *= own ? p[q] + 1e-16 : 1.0;
        d[q] = (valid && cls[q]) ? p[q] - (own ? 1.0 : 0.0) : 0.0;
    }
}

// -log of a lane's product of cross-entropy factors, folded once per LDS
// block: at most 16 factors per lane per block, each in (1e-16, 1], so the
// product stays above 1e-256 (no underflow, no branch).
__device__ __forceinline__ void gen_fold(double &loss, double &prod) {
    loss -= log_pos(prod);
    prod = 1.0;
}

// Per-wave 16 x 16 tile that turns D from the softmax layout (lane = row)
// into the gradient's B operand layout (lane = class): row stride 17
// doubles keeps the 8-byte stores and loads conflict-free.
constexpr int kGenDStride = 17;
constexpr size_t kGenDBytes = 16 * kGenDStride * sizeof(double);

__device__ __forceinline__ void gen_grad(const double (&d)[4], double *dsh, int c, int h,
                                         double (&bd)[4]) {
#pragma unroll
    for (int q = 0; q < 4; ++q) dsh[c * kGenDStride + h + 4 * q] = d[q];   // row c, class h + 4q
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 0; r < 4; ++r) bd[r] = dsh[(4 * r + h) * kGenDStride + c];  // row 4r + h, class c
    __builtin_amdgcn_wave_barrier();
}

// W <- W0, histories <- 0, current_step <- 0, order <- order[perm]
// (optimize.py:58-67) for a runtime parameter count.
__device__ __forceinline__ void reset_env_rt(const StepArgs<double> &a, int e, int lane, int P) {
    const size_t base = static_cast<size_t>(e) * P;
    for (int i = lane; i < P; i += kWave) {
        a.W[base + i] = a.W0[base + i];
        a.G[base + i] = 0.0;
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

__global__ __launch_bounds__(kWave *kGenResetWaves) void optimize_reset_rt_kernel(
    StepArgs<double> a) {
    const int lane = threadIdx.x & (kWave - 1);
    const int e = blockIdx.x * kGenResetWaves + (threadIdx.x >> 6);
    if (e >= a.E) return;
    const int P = a.F * a.K;
    reset_env_rt(a, e, lane, P);
    (void)P;
    float *obs = a.obs + static_cast<size_t>(e) * a.obs_stride;   // full or compact row
    for (int i = lane; i < a.obs_stride; i += kWave) obs[i] = 0.0f;
}

// Z^T = sum over k of W'^T_k X^T_k as kGenChains accumulator chains, added
// at the end.  One chain: the class-concatenated kernel
// (optimize_cat_kernel.h) sums its forward in one chain too, and the two
// kernels' results agree bit for bit (test_class_concatenated_agrees_with_
// per_env_kernel); CE_GEN_CHAINS=2 builds the two-chain A/B arm.
#ifdef CE_GEN_CHAINS
constexpr int kGenChains = CE_GEN_CHAINS;
#else
constexpr int kGenChains = 1;
#endif
template <int NK>
__device__ __forceinline__ gen_d4 gen_forward(const double (&wb)[NK], const double (&av)[NK]) {
    gen_d4 z[kGenChains];
#pragma unroll
    for (int i = 0; i < kGenChains; ++i) z[i] = gen_d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < NK; ++k)
        z[k % kGenChains] = __builtin_amdgcn_mfma_f64_16x16x4f64(wb[k], av[k], z[k % kGenChains],
                                                                 0, 0, 0);
#pragma unroll
    for (int i = 1; i < kGenChains; ++i) z[0] += z[i];
    return z[0];
}

// NK = ceil(F / 4) forward k-steps (a compile-time count, so the MFMA
// chains are straight-line code with their LDS reads issued together),
// FT = ceil(F / 16) gradient feature tiles.
// TAIL (F = 16 (FT - 1) + 1: F = 17, 33, 49 -- the 7x7 image sets): in the
// full-data LDS stream the last feature is done on the VALU instead of by a
// whole padded MFMA k-step (forward: 4 FMAs per lane per sub-block in place
// of 1 MFMA) and a whole padded 16-feature gradient tile (4 FMAs in place of
// 4 MFMAs), 29 -> 24 f64 MFMAs per 16 rows at F = 49.
template <int NK, bool TAIL>
__global__ __launch_bounds__(kGenBlock) void optimize_mfma_kernel(StepArgs<double> a) {
    constexpr int FT = (NK + 3) / 4;
    static_assert(!TAIL || (NK % 4 == 1 && NK > 1), "TAIL: the last k-step and the last tile hold one feature");
    constexpr int RS = gen_stride(FT);
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int e = blockIdx.x * kGenWaves + wave;
    const bool active = e < a.E;                     // wave-uniform
    const int eidx = active ? e : 0;
    const int F = a.F, K = a.K, P = F * K, N = a.N, B = a.B;
    const int c = lane & 15, h = lane >> 4;
    const double *X = reinterpret_cast<const double *>(a.data);
    const size_t pbase = static_cast<size_t>(eidx) * P;
    double *dsh = reinterpret_cast<double *>(smem + 2 * gen_block_bytes(FT) + wave * kGenDBytes);

    // ---- state: W' = W - a (optimize.py:74-75) as the forward's A operands
    const int step_prev = a.step[eidx];
    const double lprev = a.L[eidx];
    double wb[NK];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
        const int f = 4 * k + h;
        const bool own = f < F && c < K;
        const int idx = own ? f * K + c : 0;
        const double w = a.W[pbase + idx] - static_cast<double>(a.act[pbase + idx]);
        wb[k] = own ? w : 0.0;
    }

    // TAIL: W'[fl][class h + 4q] of the last feature fl = F - 1 (forward C
    // layout), and the lane's running sum of x[row][fl] D[row][class c]
    constexpr int FL = 4 * (NK - 1);
    double wt[4] = {0.0, 0.0, 0.0, 0.0};
    double gtail = 0.0;
    if constexpr (TAIL) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int k = h + 4 * q;
            const int idx = k < K ? FL * K + k : 0;
            const double w = a.W[pbase + idx] - static_cast<double>(a.act[pbase + idx]);
            wt[q] = k < K ? w : 0.0;
        }
    }

    gen_d4 g[FT];
#pragma unroll
    for (int t = 0; t < FT; ++t) g[t] = gen_d4{0.0, 0.0, 0.0, 0.0};
    double loss = 0.0, prod = 1.0;       // minibatch cross-entropy partials
    int hits = 0;
    double floss = 0.0, fprod = 1.0;     // info pass (B < N)
    int fhits = 0;
    const bool full = B == N;

    // ---- minibatch B < N: sequence[0] = rows [0, B) of the env's order
    if (!full && active) {
        const int sel = a.order_sel[e];
        const int32_t *order = a.order + sel * static_cast<size_t>(a.E) * N +
                               static_cast<size_t>(e) * N;
        for (int i0 = 0; i0 < B; i0 += 16) {
            const int ia = i0 + c;                           // this lane's row of Z^T
            const double *xa = X + static_cast<size_t>(order[ia < B ? ia : 0]) * RS;
            double av[NK];
#pragma unroll
            for (int k = 0; k < NK; ++k) av[k] = ia < B ? xa[4 * k + h] : 0.0;
            const int y = ia < B ? static_cast<int>(xa[RS - 1]) : -1;
            const gen_d4 z = gen_forward<NK>(wb, av);
            double d[4], bd[4];
            gen_softmax(z, h, K, y, d, prod, hits);
            gen_grad(d, dsh, c, h, bd);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int ir = i0 + 4 * r + h;
                const double *xr = X + static_cast<size_t>(order[ir < B ? ir : 0]) * RS;
#pragma unroll
                for (int t = 0; t < FT; ++t)
                    g[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(ir < B ? xr[16 * t + c] : 0.0, bd[r],
                                                                g[t], 0, 0, 0);
            }
            if ((i0 & 48) == 48) gen_fold(loss, prod);
        }
    }

    // ---- every row, streamed through LDS (forward [+ gradient when B == N])
    const int nblk = gen_rows_padded(N) / kGenRows;
    constexpr size_t kBlk = gen_block_bytes(FT);
    constexpr int kVec = static_cast<int>(kBlk / 16);
    constexpr int kChunks = (kVec + kWave - 1) / kWave;
    auto stage = [&](int j, int buf) {
        // LDS-DMA: one wave instruction moves 1 KiB straight into LDS
        const unsigned char *src = a.data + static_cast<size_t>(j) * kBlk;
        unsigned char *dst = smem + buf * kBlk;
        for (int ch = wave; ch < kChunks; ch += kGenWaves) {
            const int v = ch * kWave + lane;
            if (v < kVec)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) void *)(src + static_cast<size_t>(v) * 16),
                    (__attribute__((address_space(3))) void *)(dst + ch * kWave * 16), 16, 0, 0);
        }
    };
    stage(0, 0);
    for (int j = 0; j < nblk; ++j) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's part of block j
        __syncthreads();                                   // everyone's; block j-1 consumed
        if (j + 1 < nblk) stage(j + 1, (j + 1) & 1);
        if (active) {
            const double *xb = reinterpret_cast<const double *>(smem + (j & 1) * kBlk);
            // software-pipelined over the block's 4 sub-blocks: the forward
            // MFMAs of sub-block sb + 1 are issued before the softmax of sb,
            // so the matrix pipe runs while this wave does its VALU work
            auto forward = [&](int sb) {
                const double *xs = xb + sb * 16 * RS;
                if constexpr (TAIL) {
                    double av[NK - 1], wv[NK - 1];
#pragma unroll
                    for (int k = 0; k < NK - 1; ++k) {
                        av[k] = xs[c * RS + 4 * k + h];
                        wv[k] = wb[k];
                    }
                    gen_d4 z = gen_forward<NK - 1>(wv, av);
                    const double xl = xs[c * RS + FL];          // row c, the last feature
#pragma unroll
                    for (int q = 0; q < 4; ++q) z[q] = fma(wt[q], xl, z[q]);
                    return z;
                }
                double av[NK];
#pragma unroll
                for (int k = 0; k < NK; ++k) av[k] = xs[c * RS + 4 * k + h];
                return gen_forward<NK>(wb, av);
            };
            gen_d4 z = forward(0);
#pragma unroll
            for (int sb = 0; sb < kGenRows / 16; ++sb) {
                const double *xs = xb + sb * 16 * RS;
                const int y = static_cast<int>(xs[c * RS + RS - 1]);
                gen_d4 zn = z;
                if (sb + 1 < kGenRows / 16) zn = forward(sb + 1);
                double d[4];
                if (full) {
                    double bd[4];
                    gen_softmax(z, h, K, y, d, prod, hits);
                    gen_grad(d, dsh, c, h, bd);
                    constexpr int FTM = TAIL ? FT - 1 : FT;     // tiles on the matrix pipe
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
#pragma unroll
                        for (int t = 0; t < FTM; ++t)
                            g[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(
                                xs[(4 * r + h) * RS + 16 * t + c], bd[r], g[t], 0, 0, 0);
                        if constexpr (TAIL) gtail = fma(xs[(4 * r + h) * RS + FL], bd[r], gtail);
                    }
                } else {
                    gen_softmax(z, h, K, y, d, fprod, fhits);
                }
                z = zn;
            }
            if (full)
                gen_fold(loss, prod);
            else
                gen_fold(floss, fprod);
        }
    }
    if (!active) return;

    // ---- totals
    loss -= log_pos(prod);
    const double mb_loss = wave_sum(loss) / B;
    const double mb_acc = wave_sum(static_cast<double>(hits)) / B;
    double objective = mb_loss, accuracy = mb_acc;
    if (!full) {
        floss -= log_pos(fprod);
        objective = wave_sum(floss) / N;
        accuracy = wave_sum(static_cast<double>(fhits)) / N;
    }

    // TAIL: G[fl][class c] = the lane sums over the 4 row groups h; it is
    // register 0 of the last tile on the h = 0 lanes (full data only; a
    // minibatch ran the last tile on the matrix pipe)
    if constexpr (TAIL) {
        gtail = fold_pair<16>(gtail, gtail);
        gtail = fold_pair<32>(gtail, gtail);
        if (full) g[FT - 1][0] = gtail;
    }

    // ---- recurrences (optimize.py:78-92) and outputs
    const int cur_step = step_prev + 1;
    const double lnew = (mb_loss - lprev) / (lprev + 0.1);
    const bool done = cur_step >= a.max_steps;
    const bool wipe = done && a.auto_reset;
    const int OBS = 2 * P + 1;
    float *obs = a.obs + static_cast<size_t>(e) * OBS;
#pragma unroll
    for (int t = 0; t < FT; ++t)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int f = 16 * t + h + 4 * q;       // C row of register q
            if (f < F && c < K) {
                const int idx = f * K + c;
                const double gp = a.G[pbase + idx];
                const double gn = (g[t][q] / B) / (fabs(gp) + 1.0);
                if (!wipe) a.G[pbase + idx] = gn;
                obs[P + 1 + idx] = wipe ? 0.0f : static_cast<float>(gn);
            }
        }
    if (!wipe) {
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const int f = 4 * k + h;
            if (f < F && c < K) a.W[pbase + f * K + c] = wb[k];
        }
    }
    for (int i = lane; i < P; i += kWave) obs[i] = 0.0f;   // wght_hist is identically 0
    if (lane == 0) {
        obs[P] = wipe ? 0.0f : static_cast<float>(lnew);
        a.reward[e] = static_cast<float>(-mb_loss);
        a.done[e] = done ? 1 : 0;
        a.objective[e] = static_cast<float>(objective);
        a.accuracy[e] = static_cast<float>(accuracy);
        a.episode_len[e] = cur_step;
        if (!wipe) {
            a.L[e] = lnew;
            a.step[e] = cur_step;
        }
    }
    if (wipe) reset_env_rt(a, e, lane, P);
}

}  // namespace ce
