// Optimize-v0 with the full batch (batch_size=None, optimize.py:40) for any
// float64 shape, the classes of a workgroup's envs concatenated along the
// MFMA dimension (gfx950).  The reference's default data set,
// load_data('mnist'): 60,000 rows of 7x7 = 49 features and 10 classes
// (custom_envs/data/load_data.py:65-97): with B == N every env multiplies
// the SAME rows, so the 8 envs of a workgroup are one GEMM of 8 K columns
// (80 class-pairs for K = 10: 5 tiles of 16, no padding), where one env per
// 16-wide tile (optimize_mfma_kernel.h) pads 10 classes to 16 in both GEMMs.
//
// Per 64-row block of the LDS-DMA stream (double-buffered; the same row
// layout as optimize_mfma_kernel.h), three phases behind workgroup barriers:
//   forward   Z^T (class-pairs x rows) = W'cat^T . X^T: 4 MT units of
//             (16-class-pair tile, 16-row sub-block), round-robin over the
//             8 waves; A = W' of the tile's class-pairs (registers, all
//             step), B = X from LDS; C -> LDS Z (class-pair-major)
//   softmax   wave e = env e, lane = row: its K logits from Z, the literal
//             softmax (utils_math.py:51-63), -log(p_y + 1e-16) (:25-34),
//             np.argmax's first maximum, D = P - Y written back into Z
//   gradient  G (features x class-pairs) += X^T . D: FTM x MT (feature tile,
//             class-pair tile) accumulators round-robin over the waves, K of
//             each MFMA = 4 rows; A = X from LDS, B = D from LDS
// TAIL (F = 16 (FT - 1) + 1, the image sets' 49): the last feature runs on
// the VALU in both GEMMs (forward: 4 FMAs per unit lane; gradient: the
// softmax lane's K FMAs into per-lane sums).
// Epilogue: the accumulators meet in LDS; wave e finishes env e as the
// runtime-shape kernel does (optimize.py:78-100, the auto-reset).
#pragma once

#include "optimize_mfma_kernel.h"

namespace ce {

constexpr int kCatEnvs = 8;                    // envs per workgroup, one softmax wave each
constexpr int kCatWaves = 8;
constexpr int kCatBlock = kWave * kCatWaves;
constexpr int kCatRows = 64;                   // dataset rows per LDS block (= lanes)
constexpr int kCatZS = kCatRows + 2;           // Z row stride: 33 16-byte units (odd)

__host__ __device__ constexpr int cat_mt(int K) { return (kCatEnvs * K + 15) / 16; }
// Z: 16 MT class-pair rows of kCatZS doubles; the epilogue's G [64][16 MT + 2]
// reuses it
__host__ __device__ constexpr size_t cat_z_bytes(int mt) {
    return (static_cast<size_t>(16 * mt) * kCatZS > static_cast<size_t>(64) * (16 * mt + 2)
                ? static_cast<size_t>(16 * mt) * kCatZS
                : static_cast<size_t>(64) * (16 * mt + 2)) * sizeof(double);
}
// LDS: two row blocks, then Z (which the epilogue reuses for G: 64 features x
// 16 MT class-pairs fits in 16 MT rows of kCatZS >= 64 doubles)
__host__ __device__ constexpr size_t cat_lds_bytes(int ft, int mt) {
    return 2 * gen_block_bytes(ft) + cat_z_bytes(mt);
}

// v_max_f64 of two MFMA / LDS values without fmax's canonicalising
// v_max_f64 x, x, x on each operand (neither can be a signalling NaN)
__device__ __forceinline__ double cat_max(double x, double y) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
    return r;
}

// Diagnostic builds (-DCE_DIAG): per wave, shader-clock sums of the phases
// of every 64-row block (the stamp's own lgkmcnt(0) wait included, so these
// are shares, not speeds): 0 top wait (own LDS-DMA + barrier 1), 1 forward,
// 2 barrier 2, 3 softmax, 4 barrier 3, 5 gradient issue; 6 / 7 = the wave's
// start / end s_memtime (end after its stores drain).
#ifdef CE_DIAG
#define CAT_MARK(k)                                                                  \
    do {                                                                             \
        __builtin_amdgcn_sched_barrier(0);                                           \
        unsigned long long t_;                                                       \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");    \
        __builtin_amdgcn_sched_barrier(0);                                           \
        cat_acc[k] += t_ - cat_t;                                                    \
        cat_t = t_;                                                                  \
    } while (0)
#else
#define CAT_MARK(k) \
    do {            \
    } while (0)
#endif

// Instances per (NK, TAIL, K): the class count is compile-time so every
// per-wave array is sized to the units, pairs and classes it holds.
template <int NK, bool TAIL, int K>
__global__ __launch_bounds__(kCatBlock) void optimize_cat_kernel(StepArgs<double> a) {
    static_assert(K >= 2 && K <= kGenMaxK, "K classes");
    constexpr int FT = (NK + 3) / 4;
    constexpr int FTM = TAIL ? FT - 1 : FT;              // feature tiles on the matrix pipe
    constexpr int NKM = TAIL ? NK - 1 : NK;              // forward k-steps on the matrix pipe
    constexpr int FL = 4 * (NK - 1);                     // TAIL: the last feature
    constexpr int RS = gen_stride(FT);
    constexpr int MT = cat_mt(K), CP = kCatEnvs * K;
    constexpr int kUnitsMax = (4 * MT + kCatWaves - 1) / kCatWaves;       // forward units per wave
    constexpr int kPairsMax = (FTM * MT + kCatWaves - 1) / kCatWaves;    // gradient pairs per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = lane & 15, h = lane >> 4;
    const int F = a.F, P = F * K, N = a.N;
    const int e0 = blockIdx.x * kCatEnvs;
    double *zb = reinterpret_cast<double *>(smem + 2 * gen_block_bytes(FT));

    // ---- W' = W - a (optimize.py:74-75) of the class-pairs this wave's
    // forward units use: A[m = class-pair 16 mt + c][k = feature 4 s + h]
    const int n_units = 4 * MT;
    double wa[kUnitsMax][NKM > 0 ? NKM : 1];
    double wt[kUnitsMax][4];                             // TAIL: W'[FL][cp (l>>4) + 4q]
    auto w_prime = [&](int cp, int f) -> double {        // 0 past the real shape / envs
        const int e = e0 + cp / K, k = cp - (cp / K) * K;
        if (cp >= CP || f >= F || e >= a.E) return 0.0;
        const size_t i = static_cast<size_t>(e) * P + static_cast<size_t>(f) * K + k;
        return a.W[i] - static_cast<double>(a.act[i]);
    };
#pragma unroll
    for (int j = 0; j < kUnitsMax; ++j) {
        const int u = wave + j * kCatWaves;
        const int mt = u < n_units ? u / 4 : 0;
#pragma unroll
        for (int s = 0; s < NKM; ++s) wa[j][s] = u < n_units ? w_prime(16 * mt + c, 4 * s + h) : 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) wt[j][q] = TAIL && u < n_units ? w_prime(16 * mt + h + 4 * q, FL) : 0.0;
    }

    // per-wave gradient accumulators: pairs (ft, ct), p = wave + j kCatWaves
    const int n_pairs = FTM * MT;
    gen_d4 g[kPairsMax];
#pragma unroll
    for (int j = 0; j < kPairsMax; ++j) g[j] = gen_d4{0.0, 0.0, 0.0, 0.0};

    // softmax lane state: env e = e0 + wave, row = lane of the block
    const int me = e0 + wave;
    const bool env_ok = me < a.E;
    double prod = 1.0, loss = 0.0;
    int hits = 0, since = 0;
    double gtail[K];
#pragma unroll
    for (int k = 0; k < K; ++k) gtail[k] = 0.0;

    const int nblk = gen_rows_padded(N) / kCatRows;
    constexpr size_t kBlk = gen_block_bytes(FT);
    constexpr int kVec = static_cast<int>(kBlk / 16);
    constexpr int kChunks = (kVec + kWave - 1) / kWave;
    auto stage = [&](int j, int buf) {                   // LDS-DMA of row block j
        const unsigned char *src = a.data + static_cast<size_t>(j) * kBlk;
        unsigned char *dst = smem + buf * kBlk;
        for (int ch = wave; ch < kChunks; ch += kCatWaves) {
            const int v = ch * kWave + lane;
            if (v < kVec)
                __builtin_amdgcn_global_load_lds(
                    (__attribute__((address_space(1))) void *)(src + static_cast<size_t>(v) * 16),
                    (__attribute__((address_space(3))) void *)(dst + ch * kWave * 16), 16, 0, 0);
        }
    };
#ifdef CE_DIAG
    unsigned long long cat_acc[6] = {0, 0, 0, 0, 0, 0}, cat_t0, cat_t;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(cat_t0)::"memory");
    cat_t = cat_t0;
#endif
    stage(0, 0);
    for (int jb = 0; jb < nblk; ++jb) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's part of block jb
        __syncthreads();                                   // all of it; block jb-1 consumed
        CAT_MARK(0);
        if (jb + 1 < nblk) stage(jb + 1, (jb + 1) & 1);
        const double *xb = reinterpret_cast<const double *>(smem + (jb & 1) * kBlk);

        // ---- forward: units u = 4 mt + sb
#pragma unroll
        for (int j = 0; j < kUnitsMax; ++j) {
            const int u = wave + j * kCatWaves;
            if (u < n_units) {                            // wave-uniform
                const int mt = u >> 2, sb = u & 3;
                const double *xs = xb + sb * 16 * RS;
                double av[NKM > 0 ? NKM : 1];
#pragma unroll
                for (int s = 0; s < NKM; ++s) av[s] = xs[c * RS + 4 * s + h];
                const double xl = TAIL ? xs[c * RS + FL] : 0.0;  // row c's last feature
                // one accumulator chain (the SIMD's other wave fills the
                // dependent MFMAs' gaps; two chains measured 10.61 against
                // 10.45 ms at the image shape) -- the per-env kernel sums in
                // the same single chain (kGenChains), so the two agree bit
                // for bit
                gen_d4 z[1] = {gen_d4{0.0, 0.0, 0.0, 0.0}};
#pragma unroll
                for (int s = 0; s < NKM; ++s)
                    z[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(wa[j][s], av[s], z[0], 0, 0, 0);
                if constexpr (TAIL) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) z[0][q] = fma(wt[j][q], xl, z[0][q]);
                }
                // C register q of lane l: class-pair 16 mt + h + 4q, row 16 sb + c
#pragma unroll
                for (int q = 0; q < 4; ++q) zb[(16 * mt + h + 4 * q) * kCatZS + 16 * sb + c] = z[0][q];
            }
        }
        CAT_MARK(1);
        __syncthreads();
        CAT_MARK(2);

        // ---- softmax: wave = env, lane = row
        {
            const double *xr = xb + lane * RS;
            double zk[K];
#pragma unroll
            for (int k = 0; k < K; ++k) zk[k] = zb[(wave * K + k) * kCatZS + lane];
            const double yl = xr[RS - 1], xl = TAIL ? xr[FL] : 0.0;
            const int y = static_cast<int>(yl);           // -1: rows padding N to the block
            const bool valid = y >= 0 && env_ok;
            double m = zk[0];
#pragma unroll
            for (int k = 1; k < K; ++k) m = cat_max(m, zk[k]);
            double ex[K];
#pragma unroll
            for (int k = 0; k < K; ++k) ex[k] = abs_clamp750(m - zk[k]);
            exp_neg_multi_clamped<K>(ex);                 // K interleaved Horner chains
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < K; ++k) s += ex[k];
            const double inv = 1.0 / s;
            // P = ex * (1/s): the row-max classes have ex = 1 exactly, so
            // max(P) = inv and argmax(P) = the first class whose p equals it
            int first = 99;
            double py = 1.0;
#pragma unroll
            for (int k = K - 1; k >= 0; --k) {
                const double p = ex[k] * inv;
                first = p == inv ? k : first;
                py = k == y ? p : py;
                const double d = valid ? p - (k == y ? 1.0 : 0.0) : 0.0;
                zb[(wave * K + k) * kCatZS + lane] = d;
                if constexpr (TAIL) gtail[k] = fma(xl, d, gtail[k]);
            }
            hits += (valid && first == y) ? 1 : 0;
            prod *= valid ? py + 1e-16 : 1.0;
            if (++since == 16) {                          // 16 factors in (1e-16, 1]: fold
                loss -= log_pos(prod);
                prod = 1.0;
                since = 0;
            }
        }
        CAT_MARK(3);
        __syncthreads();
        CAT_MARK(4);

        // ---- gradient: pairs p = FTM-major (ft = p / MT, ct = p % MT)
#pragma unroll
        for (int j = 0; j < kPairsMax; ++j) {
            const int p = wave + j * kCatWaves;
            if (p < n_pairs) {                            // wave-uniform
                const int ft = p / MT, ct = p - ft * MT;
#pragma unroll
                for (int s = 0; s < kCatRows / 4; ++s) {
                    const double xa = xb[(4 * s + h) * RS + 16 * ft + c];
                    const double db = zb[(16 * ct + c) * kCatZS + 4 * s + h];
                    g[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(xa, db, g[j], 0, 0, 0);
                }
            }
        }
        CAT_MARK(5);
    }
    __syncthreads();                                      // every wave done with Z

    // ---- the accumulators meet in LDS: gb[f][cp] (row stride kCatZS... as
    // [f][16 MT] with stride 16 MT + 2)
    const int GS = 16 * MT + 2;
    double *gb = zb;
#pragma unroll
    for (int j = 0; j < kPairsMax; ++j) {
        const int p = wave + j * kCatWaves;
        if (p < n_pairs) {
            const int ft = p / MT, ct = p - ft * MT;
#pragma unroll
            for (int q = 0; q < 4; ++q) gb[(16 * ft + h + 4 * q) * GS + 16 * ct + c] = g[j][q];
        }
    }
    // TAIL: G[FL][class k] of this wave's env = the sum of its lanes' partials
    if constexpr (TAIL) {
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const double v = wave_sum(gtail[k]);
            if (lane == 0) gb[FL * GS + wave * K + k] = v;
        }
    }
    __syncthreads();
#ifdef CE_DIAG
    const auto cat_diag = [&]() {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned long long t_;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");
        const int row = blockIdx.x * kCatWaves + wave;
        if (row < a.E && lane < 8)
            a.diag[static_cast<size_t>(row) * 8 + lane] =
                lane < 6 ? cat_acc[lane] : lane == 6 ? cat_t0 : t_;
    };
    if (!env_ok) {
        cat_diag();
        return;
    }
#else
    if (!env_ok) return;
#endif

    // ---- env e = me: totals, recurrences (optimize.py:78-92), outputs
    const int e = me;
    const size_t pbase = static_cast<size_t>(e) * P;
    loss -= log_pos(prod);
    const double mb_loss = wave_sum(loss) / N;
    const double mb_acc = wave_sum(static_cast<double>(hits)) / N;
    const int step_prev = a.step[e];
    const double lprev = a.L[e];
    const int cur_step = step_prev + 1;
    const double lnew = (mb_loss - lprev) / (lprev + 0.1);
    const bool done = cur_step >= a.max_steps;
    const bool wipe = done && a.auto_reset;
    const size_t OS = a.obs_stride;
    float *obs = a.obs + static_cast<size_t>(e) * OS;
    for (int i = lane; i < P; i += kWave) {
        const int f = i / K, k = i - f * K;
        const double gp = a.G[pbase + i];
        const double gn = (gb[f * GS + wave * K + k] / N) / (fabs(gp) + 1.0);
        const double w = a.W[pbase + i] - static_cast<double>(a.act[pbase + i]);
        obs[P + 1 + i] = wipe ? 0.0f : static_cast<float>(gn);
        obs[i] = 0.0f;                                    // wght_hist is identically 0
        if (!wipe) {
            a.G[pbase + i] = gn;
            a.W[pbase + i] = w;
        }
    }
    if (lane == 0) {
        obs[P] = wipe ? 0.0f : static_cast<float>(lnew);
        a.reward[e] = static_cast<float>(-mb_loss);
        if (a.done) a.done[e] = done ? 1 : 0;
        a.objective[e] = static_cast<float>(mb_loss);     // B == N: the same numbers
        a.accuracy[e] = static_cast<float>(mb_acc);
        a.episode_len[e] = cur_step;
        if (!wipe) {
            a.L[e] = lnew;
            a.step[e] = cur_step;
        }
    }
    if (wipe) reset_env_rt(a, e, lane, P);
#ifdef CE_DIAG
    cat_diag();
#endif
}

}  // namespace ce
