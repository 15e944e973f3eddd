// Optimize-v0 over the config-3 MLP problem for gfx950.
//
// One VecEnv.step of E envs is two launches on one stream, each a 256-thread
// workgroup per env:
//   mlp_train_kernel:
//     Optimize.base_step        custom_envs/envs/optimize.py:69-93
//       W <- W - a              (:74-75), fused into the forward's operand loads
//       minibatch forward/backward of the F -> 64 (relu) -> K softmax MLP
//       (problems/optimize_nn.py:35-52; gradient = d(sum_i CE_i)/dtheta), the
//       flat parameter order [W1 | b1 | W2 | b2] (utils_common.py:199-207)
//       g / B, L' = (loss - L)/(L + 0.1), G' = g/(|G| + 1)   (:78-83)
//       obs = [0 (P) | L' | G' (P)], reward = -loss, done = step >= 40
//   mlp_info_kernel:
//       info objective/accuracy over the full dataset     (optimize.py:94-97)
//       auto-reset of finished envs (utils_venv.py:31): W <- W0, histories 0,
//       row order composed with the reset permutation (inmemorydataset
//       on_epoch_end under use_random_state, optimize.py:58-67)
//
// Matrix work runs on the f32-input MFMA v_mfma_f32_32x32x2_f32 (exact f32
// products, k-ordered fma chain): lane l supplies A[i = l&31][k = l>>5] and
// B[k = l>>5][j = l&31]; the 32x32 result has column j = l&31 on the lane and
// rows (r&3) + 8(r>>2) + 4(l>>5) in accumulator register r.
//   * forward: H^T (hidden x samples) = W1^T . X_b^T.  A chunk of 8 k's is
//     one float4 of a sample row per lane half (k = 8c + 4h + jj); the
//     matching W1 rows are lane-contiguous 128-B segments;
//   * logits^T (classes x samples) = W2^T . H^T takes the H^T accumulator
//     as its B operand register by register (no LDS round trip);
//   * dW1 (features x hidden) = X_b^T . dz1, K = 32 samples, one tile per
//     32x32 output block, G' and obs written from the accumulator.
// Shapes: hidden = 64, minibatch B = 32, F % 8 == 0, K <= 16, N % 64 == 0.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ce {

constexpr int kMlpHidden = 64;
constexpr int kMlpBatch = 32;
constexpr int kMlpMaxK = 16;
constexpr int kMlpBlock = 256;   // 4 waves
constexpr int kInfoTiles = 8;    // 32-sample tiles per wave per info pass

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct MlpArgs {
    int E, N, F, K, P, max_steps, auto_reset;
    const float *X;          // [N][F] dataset rows (dataset order)
    const float *Xs;         // the same rows in MFMA operand order:
                             // [N/32 tiles][F/8 chunks][64 lanes][4], element j of
                             // lane l = X[32 t + (l & 31)][8 c + 4 (l >> 5) + j]
    const int32_t *label;    // [N]
    float *W;                // [E][P]
    const float *W0;         // [E][P]
    double *G;               // [E][P] grad_hist[idx] (float64, np.zeros)
    double *L;               // [E]
    int32_t *step;           // [E]
    const int32_t *perm;     // [E][N] reset permutation
    int32_t *order;          // [2][E][N] current row order (ping-pong)
    int32_t *order_sel;      // [E]
    const float *act;        // [E][P]
    float *obs;              // [E][2P+1]
    float *reward;
    uint8_t *done;
    float *objective;
    float *accuracy;
    int32_t *episode_len;
};

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// row of accumulator register r for lane half h (32x32 C/D map)
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ void mlp_offsets(const MlpArgs &a, int &ob1, int &oW2, int &ob2) {
    ob1 = a.F * kMlpHidden;
    oW2 = ob1 + kMlpHidden;
    ob2 = oW2 + kMlpHidden * a.K;
}

// G' = g / (|G| + 1) in float64 (optimize.py:82-83 with grad_hist float64);
// obs carries it as float32 after the P zero weight-history entries and L'.
__device__ __forceinline__ void write_grad(const MlpArgs &a, size_t e, int idx, float g) {
    const size_t gi = e * a.P + idx;
    const double gn = static_cast<double>(g) / (fabs(a.G[gi]) + 1.0);
    a.G[gi] = gn;
    a.obs[e * (2 * static_cast<size_t>(a.P) + 1) + a.P + 1 + idx] = static_cast<float>(gn);
}

__device__ __forceinline__ void mlp_train_body(const MlpArgs &a, const size_t e) {
    __shared__ float part[4][kMlpHidden][kMlpBatch];     // per-wave partial H^T
    __shared__ float hs[kMlpBatch][kMlpHidden + 1];      // H, then dz1 (sample-major)
    __shared__ float w2s[kMlpHidden][kMlpMaxK];
    __shared__ float b1s[kMlpHidden], b2s[kMlpMaxK];
    __shared__ float dz2[kMlpBatch][kMlpMaxK];
    __shared__ float ce[kMlpBatch];
    __shared__ int rows[kMlpBatch];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, h = lane >> 5;
    const int F = a.F, K = a.K, P = a.P;
    int ob1, oW2, ob2;
    mlp_offsets(a, ob1, oW2, ob2);
    float *W = a.W + e * P;
    const float *act = a.act + e * P;
    float *obs = a.obs + e * (2 * static_cast<size_t>(P) + 1);

    if (tid < kMlpBatch) {
        const int sel = a.order_sel[e];
        rows[tid] = a.order[(static_cast<size_t>(sel) * a.E + e) * a.N + tid];
    }
    // small parameters: b1, W2, b2 updated (W <- W - a) and staged
    for (int i = tid; i < P - ob1; i += kMlpBlock) {
        const int idx = ob1 + i;
        const float w = W[idx] - act[idx];
        W[idx] = w;
        if (idx < oW2) b1s[idx - ob1] = w;
        else if (idx < ob2) w2s[(idx - oW2) / K][(idx - oW2) % K] = w;
        else b2s[idx - ob2] = w;
    }
    // obs[0:P] = wght_hist[idx] == 0 (optimize.py:84-86 never leaves zero)
    for (int i = tid; i < P; i += kMlpBlock) obs[i] = 0.0f;
    __syncthreads();

    // ---- forward H^T = W1'^T X_b^T, k split over the 4 waves; W1 <- W1 - a
    {
        const int chunks = F / 8;
        const int c0 = wave * chunks / 4, c1 = (wave + 1) * chunks / 4;
        f32x16 acc0 = {}, acc1 = {};
        const float *xrow = a.X + static_cast<size_t>(rows[li]) * F + 4 * h;
        // operands of chunk c + 1 are loaded while chunk c is on the MFMA pipe
        float4 xn = *reinterpret_cast<const float4 *>(xrow + 8 * c0);
        float wn[8], an[8];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int base = (8 * c0 + 4 * h + jj) * kMlpHidden + li;
            wn[2 * jj] = W[base];
            wn[2 * jj + 1] = W[base + 32];
            an[2 * jj] = act[base];
            an[2 * jj + 1] = act[base + 32];
        }
        for (int c = c0; c < c1; ++c) {
            const float xs[4] = {xn.x, xn.y, xn.z, xn.w};
            float wc[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) wc[q] = wn[q] - an[q];
            if (c + 1 < c1) {
                xn = *reinterpret_cast<const float4 *>(xrow + 8 * (c + 1));
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int base = (8 * (c + 1) + 4 * h + jj) * kMlpHidden + li;
                    wn[2 * jj] = W[base];
                    wn[2 * jj + 1] = W[base + 32];
                    an[2 * jj] = act[base];
                    an[2 * jj + 1] = act[base + 32];
                }
            }
#pragma unroll
            for (int jj = 0; jj < 4; ++jj) {
                const int base = (8 * c + 4 * h + jj) * kMlpHidden + li;
                W[base] = wc[2 * jj];
                W[base + 32] = wc[2 * jj + 1];
                acc0 = mfma32(wc[2 * jj], xs[jj], acc0);
                acc1 = mfma32(wc[2 * jj + 1], xs[jj], acc1);
            }
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
            part[wave][acc_row(r, h)][li] = acc0[r];
            part[wave][32 + acc_row(r, h)][li] = acc1[r];
        }
    }
    __syncthreads();
    for (int i = tid; i < kMlpHidden * kMlpBatch; i += kMlpBlock) {
        const int j = i / kMlpBatch, s = i % kMlpBatch;
        const float z = ((part[0][j][s] + part[1][j][s]) + (part[2][j][s] + part[3][j][s])) + b1s[j];
        hs[s][j] = z > 0.0f ? z : 0.0f;
    }
    __syncthreads();

    // ---- logits, softmax, cross-entropy (utils_math.py:25-34,51-63), P - Y
    if (tid < kMlpBatch) {
        const int s = tid;
        float z[kMlpMaxK];
        float m = -INFINITY;
        for (int k = 0; k < K; ++k) {
            float acc = b2s[k];
            for (int j = 0; j < kMlpHidden; ++j) acc = fmaf(hs[s][j], w2s[j][k], acc);
            z[k] = acc;
            m = fmaxf(m, acc);
        }
        float sum = 0.0f;
        for (int k = 0; k < K; ++k) {
            z[k] = expf(z[k] - m);
            sum += z[k];
        }
        const int y = a.label[rows[s]];
        for (int k = 0; k < K; ++k) {
            const float p = z[k] / sum;
            dz2[s][k] = p - (k == y ? 1.0f : 0.0f);
            if (k == y) ce[s] = -logf(p + 1e-16f);
        }
    }
    __syncthreads();

    // ---- small gradients: dW2, db2, dz1 = (dz2 W2^T) * (H > 0), db1
    const float inv_b = 1.0f / kMlpBatch;
    for (int i = tid; i < kMlpHidden * K; i += kMlpBlock) {
        const int j = i / K, k = i % K;
        float acc = 0.0f;
        for (int s = 0; s < kMlpBatch; ++s) acc = fmaf(hs[s][j], dz2[s][k], acc);
        write_grad(a, e, oW2 + i, acc * inv_b);
    }
    if (tid < K) {
        float acc = 0.0f;
        for (int s = 0; s < kMlpBatch; ++s) acc += dz2[s][tid];
        write_grad(a, e, ob2 + tid, acc * inv_b);
    }
    float dz1v[kMlpHidden * kMlpBatch / kMlpBlock];
#pragma unroll
    for (int q = 0; q < kMlpHidden * kMlpBatch / kMlpBlock; ++q) {
        const int i = tid + q * kMlpBlock;
        const int s = i / kMlpHidden, j = i % kMlpHidden;
        float acc = 0.0f;
        for (int k = 0; k < K; ++k) acc = fmaf(dz2[s][k], w2s[j][k], acc);
        dz1v[q] = hs[s][j] > 0.0f ? acc : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kMlpHidden * kMlpBatch / kMlpBlock; ++q) {
        const int i = tid + q * kMlpBlock;
        hs[i / kMlpHidden][i % kMlpHidden] = dz1v[q];
    }
    __syncthreads();
    if (tid < kMlpHidden) {
        float acc = 0.0f;
        for (int s = 0; s < kMlpBatch; ++s) acc += hs[s][tid];
        write_grad(a, e, ob1 + tid, acc * inv_b);
    }

    // ---- dW1 = X_b^T dz1 on MFMA: 32 features x 64 hidden per tile (two
    // accumulators sharing the X operand), K = 32 samples; G' and obs from the
    // accumulators, each feature row's 64 values written as one 512-B run
    {
        const int ftiles = (F + 31) / 32;
        for (int ft = wave; ft < ftiles; ft += 4) {
            const int f = ft * 32 + li;
            f32x16 acc0 = {}, acc1 = {};
#pragma unroll 4
            for (int ks = 0; ks < kMlpBatch / 2; ++ks) {
                const int s = 2 * ks + h;
                const float xa = f < F ? a.X[static_cast<size_t>(rows[s]) * F + f] : 0.0f;
                acc0 = mfma32(xa, hs[s][li], acc0);
                acc1 = mfma32(xa, hs[s][32 + li], acc1);
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int fr = ft * 32 + acc_row(r, h);
                if (fr < F) {
                    write_grad(a, e, fr * kMlpHidden + li, acc0[r] * inv_b);
                    write_grad(a, e, fr * kMlpHidden + 32 + li, acc1[r] * inv_b);
                }
            }
        }
    }

    // ---- loss recurrence, reward, done (optimize.py:80-81,90-91,102-103)
    if (tid == 0) {
        float loss = 0.0f;
        for (int s = 0; s < kMlpBatch; ++s) loss += ce[s];
        loss /= static_cast<float>(kMlpBatch);
        const double lp = a.L[e];
        const double ln = (static_cast<double>(loss) - lp) / (lp + 0.1);
        a.L[e] = ln;
        obs[P] = static_cast<float>(ln);
        const int s = a.step[e] + 1;
        a.step[e] = s;
        a.reward[e] = -loss;
        a.done[e] = s >= a.max_steps ? 1 : 0;
        a.episode_len[e] = s;
    }
}

// Reset one env (block-wide): W <- W0, histories zero, order composed with
// the reset permutation, reset observation = zeros (optimize.py:58-67).
__device__ void mlp_reset_env(const MlpArgs &a, size_t e, bool write_obs) {
    const int tid = threadIdx.x, P = a.P;
    for (int i = tid; i < P; i += kMlpBlock) {
        a.W[e * P + i] = a.W0[e * P + i];
        a.G[e * P + i] = 0.0;
    }
    if (write_obs) {
        float *obs = a.obs + e * (2 * static_cast<size_t>(P) + 1);
        for (int i = tid; i < 2 * P + 1; i += kMlpBlock) obs[i] = 0.0f;
    }
    const int sel = a.order_sel[e];
    const int32_t *cur = a.order + (static_cast<size_t>(sel) * a.E + e) * a.N;
    int32_t *nxt = a.order + (static_cast<size_t>(1 - sel) * a.E + e) * a.N;
    const int32_t *perm = a.perm + e * a.N;
    for (int i = tid; i < a.N; i += kMlpBlock) nxt[i] = cur[perm[i]];
    __syncthreads();
    if (tid == 0) {
        a.order_sel[e] = 1 - sel;
        a.L[e] = 0.0;
        a.step[e] = 0;
    }
}

__global__ __launch_bounds__(kMlpBlock) void mlp_reset_kernel(MlpArgs a) {
    mlp_reset_env(a, blockIdx.x, true);
}

// Full-dataset forward for info['objective'] / info['accuracy'] with the
// updated weights, then the auto-reset of envs that just finished.
__device__ __forceinline__ void mlp_info_body(const MlpArgs &a, const size_t e) {
    __shared__ float w2s[kMlpHidden][kMlpMaxK];
    __shared__ float b1s[kMlpHidden], b2s[kMlpMaxK];
    __shared__ float red_loss[4];
    __shared__ int red_hits[4];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, h = lane >> 5;
    const int F = a.F, K = a.K, P = a.P;
    int ob1, oW2, ob2;
    mlp_offsets(a, ob1, oW2, ob2);
    const float *W = a.W + e * P;
    for (int i = tid; i < P - ob1; i += kMlpBlock) {
        const int idx = ob1 + i;
        const float w = W[idx];
        if (idx < oW2) b1s[idx - ob1] = w;
        else if (idx < ob2) w2s[(idx - oW2) / K][(idx - oW2) % K] = w;
        else b2s[idx - ob2] = w;
    }
    __syncthreads();

    float loss_acc = 0.0f;
    int hits = 0;
    const int tiles = a.N / 32;
    const int chunks = F / 8;
    const size_t tstride = static_cast<size_t>(chunks) * 64 * 4;   // floats per swizzled tile
    // A pass gives each wave kInfoTiles consecutive 32-sample tiles: 2 x kInfoTiles
    // accumulators live across one sweep over K, so every W1 fragment a wave
    // loads feeds 2 kInfoTiles MFMAs and W1 is read once per wave per pass.
    for (int t0 = wave * kInfoTiles; t0 < tiles; t0 += 4 * kInfoTiles) {
        const int nt = tiles - t0 < kInfoTiles ? tiles - t0 : kInfoTiles;   // wave-uniform
        f32x16 acc[kInfoTiles][2];
#pragma unroll
        for (int q = 0; q < kInfoTiles; ++q) acc[q][0] = acc[q][1] = f32x16{};
        const float *xb = a.Xs + (static_cast<size_t>(t0) * chunks * 64 + lane) * 4;
        // operands of chunk c + 1 are loaded while chunk c is on the MFMA pipe
        float4 xn[kInfoTiles];
        float wn[8];
        // tiles past the end of a partial pass read tile 0 (valid memory); their
        // accumulators are never used, so the MFMA loop stays branch-free
        size_t toff[kInfoTiles];
#pragma unroll
        for (int q = 0; q < kInfoTiles; ++q) {
            toff[q] = (q < nt ? q : 0) * tstride;
            xn[q] = *reinterpret_cast<const float4 *>(xb + toff[q]);
        }
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
            const int base = (4 * h + jj) * kMlpHidden + li;
            wn[2 * jj] = W[base];
            wn[2 * jj + 1] = W[base + 32];
        }
        for (int c = 0; c < chunks; ++c) {
            float wc[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) wc[q] = wn[q];
            if (c + 1 < chunks) {
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    const int base = (8 * (c + 1) + 4 * h + jj) * kMlpHidden + li;
                    wn[2 * jj] = W[base];
                    wn[2 * jj + 1] = W[base + 32];
                }
            }
            // tile-major: tile q's X register is reloaded for chunk c + 1 as
            // soon as its 8 MFMAs of chunk c have issued
#pragma unroll
            for (int q = 0; q < kInfoTiles; ++q) {
                const float xs[4] = {xn[q].x, xn[q].y, xn[q].z, xn[q].w};
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    acc[q][0] = mfma32(wc[2 * jj], xs[jj], acc[q][0]);
                    acc[q][1] = mfma32(wc[2 * jj + 1], xs[jj], acc[q][1]);
                }
                if (c + 1 < chunks)
                    xn[q] = *reinterpret_cast<const float4 *>(xb + toff[q] + 256 * (c + 1));
            }
        }
#pragma unroll
        for (int q = 0; q < kInfoTiles; ++q) {
            if (q >= nt) continue;
            // bias + relu on H^T, then logits^T = W2^T H^T with H^T as the B operand
            f32x16 lg = {};
#pragma unroll
            for (int ht = 0; ht < 2; ++ht) {
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int hid = ht * 32 + acc_row(r, h);
                    const float z = acc[q][ht][r] + b1s[hid];
                    const float hv = z > 0.0f ? z : 0.0f;
                    const float wa = li < K ? w2s[hid][li] : 0.0f;
                    lg = mfma32(wa, hv, lg);
                }
            }
            // lane (sample li, half h) holds classes acc_row(r, h) of its sample
            float m = -INFINITY, best = -INFINITY;
            int arg = 0;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int k = acc_row(r, h);
                if (k < K) {
                    const float z = lg[r] + b2s[k];
                    lg[r] = z;
                    m = fmaxf(m, z);
                }
            }
            m = fmaxf(m, __shfl_xor(m, 32));
            float sum = 0.0f;
            const int row = (t0 + q) * 32 + li;
            const int y = a.label[row];
            float zy = 0.0f;
#pragma unroll
            for (int r = 0; r < 8; ++r) {
                const int k = acc_row(r, h);
                if (k < K) {
                    sum += expf(lg[r] - m);
                    if (k == y) zy = lg[r];
                    if (lg[r] > best || (lg[r] == best && k < arg)) {
                        best = lg[r];
                        arg = k;
                    }
                }
            }
            sum += __shfl_xor(sum, 32);
            zy += __shfl_xor(zy, 32);            // exactly one half owns class y
            const float best_o = __shfl_xor(best, 32);
            const int arg_o = __shfl_xor(arg, 32);
            if (best_o > best || (best_o == best && arg_o < arg)) arg = arg_o;
            if (h == 0) {
                const float p = expf(zy - m) / sum;
                loss_acc += -logf(p + 1e-16f);
                hits += arg == y ? 1 : 0;
            }
        }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        loss_acc += __shfl_xor(loss_acc, off);
        hits += __shfl_xor(hits, off);
    }
    if (lane == 0) {
        red_loss[wave] = loss_acc;
        red_hits[wave] = hits;
    }
    __syncthreads();
    if (tid == 0) {
        const float tot = (red_loss[0] + red_loss[1]) + (red_loss[2] + red_loss[3]);
        a.objective[e] = tot / static_cast<float>(a.N);
        a.accuracy[e] = static_cast<float>(red_hits[0] + red_hits[1] + red_hits[2] + red_hits[3]) /
                        static_cast<float>(a.N);
    }
    const bool wipe = a.auto_reset && a.step[e] >= a.max_steps;
    __syncthreads();
    if (wipe) mlp_reset_env(a, e, true);
}

// The two phases of a step, launched back to back on one stream.  The train
// phase streams state (HBM-bound) at 2 waves per SIMD; the info phase holds
// 16 32x32 accumulators per wave (one wave per SIMD, 512 registers).
__global__ __launch_bounds__(kMlpBlock) void mlp_train_kernel(MlpArgs a) {
    mlp_train_body(a, blockIdx.x);
}

__global__ __launch_bounds__(kMlpBlock) void mlp_info_kernel(MlpArgs a) {
    mlp_info_body(a, blockIdx.x);
}

}  // namespace ce
