// MultiOptLRs-v0 over the OptimizeNN problem for gfx950.
//
// One OptVecEnv.step of E envs = two launches, one 512-thread workgroup per
// env in each:
//   nn_grad_kernel   MultiOptLRs.base_step up to the update
//                    (custom_envs/envs/multioptlrs.py:81-87):
//                      grad = model.get_gradient()   forward + backward of the
//                        F -> hidden... (relu) -> K softmax network on the
//                        current batch (problems/optimize_nn.py:35-52,122-126)
//                      lr = 10^(a - 4)                (utils/utils_env.py:113-114)
//                      theta' = theta - grad * lr     -> theta_n
//                    and, for an env that was just reset, the reset's
//                    model.get() (multioptlrs.py:70-71): same weights, same
//                    batch, so the same gradient seeds the raw history.
//   nn_step_kernel   the rest of base_step (multioptlrs.py:88-129):
//                      grad, loss = model.get()       at theta' on the same batch
//                      History append, observation v3 ratios, adjusted
//                      history, obs = clip(nan_to_num(.), +-100) - 1,
//                      reward v6, early stop, the 14 info values
//                      model.next()                   (optimize_nn.py:102-112)
//                    then OptVecEnv's auto-reset (concurrentvecenv.py:37).
//
// Matrices run on v_mfma_f32_32x32x2_f32.  Every activation lives in LDS
// sample-major ([32 samples][width + 4]); each GEMM picks the operand roles
// that keep both operands' reads contiguous:
//   forward   Z^T (units x samples) = W^T . H^T : A = W columns (global, lanes
//             contiguous along the output units), B = H rows (ds_read_b128,
//             k = 8c + 4h + m); the C tile holds 4 consecutive units per
//             register group, stored back sample-major as float4.
//   dH^T      (in units x samples) = W . dZ^T : A = W rows (one float4 per
//             lane per 4 MFMAs), B = dZ rows (ds_read_b128).
//   dW        (in units x out units) = H^T . dZ : reduction over the 32
//             samples, s = 2c + h; element (i, j) of the C tile is flat
//             parameter off + i * w_out + j, lanes contiguous along j.
// The output layer (K <= 32 classes) is VALU work.  Each gradient element is
// handed to the kernel's per-element epilogue straight from the accumulator
// registers, so the gradient never makes an HBM round trip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "multiopt_kernels.h"     // ratio, clip100, kRawHist, kMultiInfo

namespace ce {

typedef float nn_f32x16 __attribute__((ext_vector_type(16)));

// v_mfma_f32_32x32x2_f32: lane l supplies A[l & 31][l >> 5], B[l >> 5][l & 31]
__device__ __forceinline__ nn_f32x16 nn_mfma(float a, float b, nn_f32x16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// row of accumulator register r for lane half h (32x32 C/D map); the column
// is l & 31
__device__ __forceinline__ int nn_acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

constexpr int kNnBlock = 512;      // 8 waves
constexpr int kNnWaves = kNnBlock / 64;
constexpr int kNnBatch = 32;       // samples per minibatch tile (B <= 32)
constexpr int kNnMaxHidden = 4;    // hidden layers
constexpr int kNnMaxWidth = 512;   // hidden units per layer (multiple of 32)
constexpr int kNnMaxK = 32;        // classes
constexpr int kNnMaxH = 16;        // adjusted-history length
constexpr int kNnPad = 4;          // LDS row padding (floats)

struct NnArgs {
    int E, N, F, K, L, B, nb, H, max_batches, auto_reset;
    int P;                         // parameters (= agents) per env
    int Ps;                        // per-env stride of [E][P] state (P rounded up)
    int dims[kNnMaxHidden + 2];    // F, hidden..., K
    int off_w[kNnMaxHidden + 1];   // flat offset of layer l's kernel [dims[l]][dims[l+1]]
    int off_b[kNnMaxHidden + 1];   // flat offset of layer l's bias
    int lds_x, lds_h[kNnMaxHidden], lds_z, lds_part, lds_bytes;   // float offsets
    int split;                     // 1: some hidden forward needs the split-k scratch
    const float *X;                // [N][F] dataset rows (dataset order)
    const int32_t *label;          // [N]
    float *theta;                  // [E][Ps] current parameters
    float *theta_n;                // [E][Ps] parameters after this step's update
    const float *theta0;           // [E][Ps] reset parameters
    float *gprev;                  // [E][Ps] newest raw-history gradient
    float *rw, *rg;                // [H][E][Ps] adjusted w~ / g~ entries, obs form
    double *al;                    // [H][E] adjusted loss entries (raw)
    double *sw, *sg;               // [H][E] sum |w~|, sum |g~| of each entry
    float *hl;                     // [5][E] raw-history losses
    double *hsg;                   // [5][E] raw-history gradient sums
    double *lr_stats;              // [E][2] sum lr, sum lr^2 of this step
    int32_t *step;                 // [E]
    int32_t *cursor;               // [E] current batch index within the epoch
    int32_t *order;                // [2][E][N] row order (ping-pong)
    int32_t *order_sel;            // [E]
    const int32_t *reset_perm;     // [E][N] the shuffle every reset draws
    const int32_t *epoch_perm;     // [E][N] the shuffle every epoch end draws
    const int32_t *agent_row;      // [P] OptVecEnv row of agent p (sorted names)
    const float *act;              // [E][P] rows
    float *obs;                    // [E][P][3H] rows
    float *reward;                 // [E][P] rows
    uint8_t *done;                 // [E][P] rows
    float *info;                   // [E][14]
    int32_t *episode_len;          // [E]
};

__device__ __forceinline__ int nn_ld(int w) { return ((w + 31) & ~31) + kNnPad; }

// ---------------------------------------------------------------- LDS staging
// Batch rows of env e: order[sel][e][cursor * B + s], s < nrows; X rows
// zero-padded to the 32-column tile and zero for s >= nrows.
__device__ __forceinline__ int nn_stage_batch(const NnArgs &a, size_t e, float *lds, int *rows) {
    const int tid = threadIdx.x;
    const int cur = a.cursor[e];
    const int first = cur * a.B;
    const int nrows = a.N - first < a.B ? a.N - first : a.B;
    if (tid < kNnBatch) {
        const int sel = a.order_sel[e];
        rows[tid] = tid < nrows ? a.order[(static_cast<size_t>(sel) * a.E + e) * a.N + first + tid]
                                : -1;
    }
    __syncthreads();
    const int ldx = nn_ld(a.F), wpad = (a.F + 31) & ~31;
    float *xb = lds + a.lds_x;
    for (int i = tid; i < kNnBatch * wpad; i += kNnBlock) {
        const int s = i / wpad, f = i % wpad;
        const int r = rows[s];
        xb[s * ldx + f] = (r >= 0 && f < a.F) ? a.X[static_cast<size_t>(r) * a.F + f] : 0.0f;
    }
    return nrows;
}

// ------------------------------------------------------------------- forward
// out[s][j] = relu(b[j] + sum_k in[s][k] W[k][j]) for one hidden layer.
__device__ void nn_forward_hidden(const float *W, const float *bias, int w_in, int w_out,
                                  const float *in, int ld_in, float *out, int ld_out,
                                  float *part) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int li = lane & 31, h = lane >> 5;
    const int tiles = w_out / 32;
    const int S = tiles >= kNnWaves ? 1 : kNnWaves / tiles;     // k split
    const int chunks = (w_in + 7) / 8;
    for (int item = wave; item < tiles * S; item += kNnWaves) {
        const int tile = item % tiles, sp = item / tiles;
        const int c0 = sp * chunks / S, c1 = (sp + 1) * chunks / S;
        const int j = tile * 32 + li;
        nn_f32x16 acc = {};
        const float *xrow = in + li * ld_in + 4 * h;
        float wn[4];
        float4 xn = {};
        auto load = [&](int c) {
            xn = *reinterpret_cast<const float4 *>(xrow + 8 * c);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int k = 8 * c + 4 * h + m;
                wn[m] = k < w_in ? W[static_cast<size_t>(k) * w_out + j] : 0.0f;
            }
        };
        if (c0 < c1) load(c0);
        for (int c = c0; c < c1; ++c) {
            const float xs[4] = {xn.x, xn.y, xn.z, xn.w};
            const float wc[4] = {wn[0], wn[1], wn[2], wn[3]};
            if (c + 1 < c1) load(c + 1);
#pragma unroll
            for (int m = 0; m < 4; ++m) acc = nn_mfma(wc[m], xs[m], acc);
        }
        // lane holds sample li, units tile*32 + nn_acc_row(r, h): r = 4g..4g+3
        // are 4 consecutive units
        if (S == 1) {
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int u = tile * 32 + 8 * g + 4 * h;
                float4 v;
                v.x = fmaxf(acc[4 * g + 0] + bias[u + 0], 0.0f);
                v.y = fmaxf(acc[4 * g + 1] + bias[u + 1], 0.0f);
                v.z = fmaxf(acc[4 * g + 2] + bias[u + 2], 0.0f);
                v.w = fmaxf(acc[4 * g + 3] + bias[u + 3], 0.0f);
                *reinterpret_cast<float4 *>(out + li * ld_out + u) = v;
            }
        } else {
            // partial sums [sp][sample][unit]: S * 32 * w_out <= 8 * 32 * 32 floats
            float *pp = part + (static_cast<size_t>(sp) * kNnBatch + li) * w_out;
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int u = tile * 32 + 8 * g + 4 * h;
                *reinterpret_cast<float4 *>(pp + u) =
                    float4{acc[4 * g], acc[4 * g + 1], acc[4 * g + 2], acc[4 * g + 3]};
            }
        }
    }
    if (S > 1) {
        __syncthreads();
        for (int i = threadIdx.x; i < kNnBatch * w_out; i += kNnBlock) {
            const int s = i / w_out, u = i % w_out;
            float z = 0.0f;
            for (int q = 0; q < S; ++q) z += part[(static_cast<size_t>(q) * kNnBatch + s) * w_out + u];
            out[s * ld_out + u] = fmaxf(z + bias[u], 0.0f);
        }
    }
}

// logits[s][k] = b[k] + sum_j in[s][j] W[j][k] (K <= 32) on the VALU: thread
// (sample s = t / 16, chunk t % 16) sums its w/16 units, then a 16-lane
// butterfly.  Rows s >= nrows are computed and ignored.
__device__ void nn_forward_logits(const float *W, const float *bias, int w_in, int K,
                                  const float *in, int ld_in, float *z, int ld_z) {
    const int t = threadIdx.x;
    const int s = t >> 4, ch = t & 15;
    const int per = w_in / 16;
    float acc[kNnMaxK];
#pragma unroll
    for (int k = 0; k < kNnMaxK; ++k) acc[k] = 0.0f;
    for (int q = 0; q < per; ++q) {
        const int j = ch * per + q;
        const float hv = in[s * ld_in + j];
        const float *wr = W + static_cast<size_t>(j) * K;
#pragma unroll
        for (int k = 0; k < kNnMaxK; ++k)
            if (k < K) acc[k] = fmaf(hv, wr[k], acc[k]);
    }
#pragma unroll
    for (int k = 0; k < kNnMaxK; ++k) {
        if (k < K) {
            float v = acc[k];
            v += __shfl_xor(v, 8, 16);
            v += __shfl_xor(v, 4, 16);
            v += __shfl_xor(v, 2, 16);
            v += __shfl_xor(v, 1, 16);
            acc[k] = v;
        }
    }
    if (ch == 0) {
#pragma unroll
        for (int k = 0; k < kNnMaxK; ++k)
            if (k < K) z[s * ld_z + k] = acc[k] + bias[k];
    }
}

// softmax cross-entropy on the logits (tf.nn.softmax_cross_entropy_with_logits,
// the tf.keras route for a Softmax output): CE = log(sum exp(z - m)) - (z_y - m),
// dZ = softmax - y for valid rows, 0 for padding rows.  Returns the mean CE
// over the nrows valid rows (every thread).
__device__ float nn_softmax_ce(const NnArgs &a, const int *rows, int nrows, float *z, int ld_z,
                               float *red) {
    const int t = threadIdx.x;
    float ce = 0.0f;
    if (t < kNnBatch) {
        const int s = t, K = a.K;
        float *zr = z + s * ld_z;
        if (s < nrows) {
            float m = -INFINITY;
            for (int k = 0; k < K; ++k) m = fmaxf(m, zr[k]);
            float se = 0.0f;
            for (int k = 0; k < K; ++k) se += expf(zr[k] - m);
            const int y = a.label[rows[s]];
            ce = logf(se) - (zr[y] - m);
            for (int k = 0; k < K; ++k) zr[k] = expf(zr[k] - m) / se - (k == y ? 1.0f : 0.0f);
        } else {
            for (int k = 0; k < K; ++k) zr[k] = 0.0f;
        }
    }
    if (t < 64) {
        // samples 0..31 are lanes 0..31 of wave 0, in order
        float v = ce;
        for (int off = 1; off < 32; off <<= 1) v += __shfl_xor(v, off, 32);
        if (t == 0) red[0] = v / static_cast<float>(nrows);
    }
    __syncthreads();
    return red[0];
}

// ------------------------------------------------------------------ backward
// Calls emit(p, g) once per flat parameter p with g = d(sum_i CE_i)/dtheta_p.
// Leaves the LDS activations overwritten by the dZ's.
template <typename Emit>
__device__ __forceinline__ void nn_backward(const NnArgs &a, const float *theta, float *lds, Emit &emit) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int li = lane & 31, h = lane >> 5;
    const int L = a.L, K = a.K;
    float *zb = lds + a.lds_z;
    const int ldz = nn_ld(K);

    // ---- output layer: dW_out = H_L^T dZ, db_out = sum_s dZ, dH_L
    {
        const int w = a.dims[L];
        const float *hb = lds + (L ? a.lds_h[L - 1] : a.lds_x);
        const int ldh = nn_ld(w);
        const int ow = a.off_w[L], ob = a.off_b[L];
        for (int i = tid; i < w * K; i += kNnBlock) {
            const int j = i / K, k = i % K;
            float g = 0.0f;
            for (int s = 0; s < kNnBatch; ++s) g = fmaf(hb[s * ldh + j], zb[s * ldz + k], g);
            emit(ow + i, g);
        }
        if (tid < K) {
            float g = 0.0f;
            for (int s = 0; s < kNnBatch; ++s) g += zb[s * ldz + tid];
            emit(ob + tid, g);
        }
        if (L == 0) return;
        // dH_L[s][j] = sum_k dZ[s][k] W_out[j][k], masked by H_L > 0: 32 x w
        // values, w / 16 per thread, written back after every read of H_L
        const float *Wo = theta + ow;
        constexpr int kPer = kNnMaxWidth * kNnBatch / kNnBlock;
        float dh[kPer];
        const int per = w * kNnBatch / kNnBlock;
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            if (q < per) {
                const int i = tid + q * kNnBlock;
                const int s = i / w, j = i % w;
                float v = 0.0f;
                for (int k = 0; k < K; ++k)
                    v = fmaf(zb[s * ldz + k], Wo[static_cast<size_t>(j) * K + k], v);
                dh[q] = hb[s * ldh + j] > 0.0f ? v : 0.0f;
            }
        }
        __syncthreads();
        float *hw = lds + a.lds_h[L - 1];
#pragma unroll
        for (int q = 0; q < kPer; ++q) {
            if (q < per) {
                const int i = tid + q * kNnBlock;
                hw[(i / w) * ldh + i % w] = dh[q];
            }
        }
        __syncthreads();
    }

    // ---- hidden layers l = L-1 .. 0 (layer l maps dims[l] -> dims[l+1]);
    // dZ of its output sits in buffer h[l]
    for (int l = L - 1; l >= 0; --l) {
        const int w_in = a.dims[l], w_out = a.dims[l + 1];
        const float *dz = lds + a.lds_h[l];
        const int ldo = nn_ld(w_out);
        float *hin = lds + (l ? a.lds_h[l - 1] : a.lds_x);
        const int ldi = nn_ld(w_in);
        const float *W = theta + a.off_w[l];

        // db_l
        for (int j = tid; j < w_out; j += kNnBlock) {
            float g = 0.0f;
            for (int s = 0; s < kNnBatch; ++s) g += dz[s * ldo + j];
            emit(a.off_b[l] + j, g);
        }

        // dH_{l}^T tiles (input units x samples) = W . dZ^T, kept in registers
        const int tin = w_in / 32;          // l > 0: w_in is a multiple of 32
        nn_f32x16 dht[kNnMaxWidth / 32 / kNnWaves];
        if (l > 0) {
            const int chunks = w_out / 8;
#pragma unroll
            for (int q = 0; q < kNnMaxWidth / 32 / kNnWaves; ++q) {
                const int tile = wave + q * kNnWaves;
                nn_f32x16 acc = {};
                if (tile < tin) {
                    const float *wrow = W + static_cast<size_t>(tile * 32 + li) * w_out + 4 * h;
                    const float *zrow = dz + li * ldo + 4 * h;
                    for (int c = 0; c < chunks; ++c) {
                        const float4 wa = *reinterpret_cast<const float4 *>(wrow + 8 * c);
                        const float4 zv = *reinterpret_cast<const float4 *>(zrow + 8 * c);
                        acc = nn_mfma(wa.x, zv.x, acc);
                        acc = nn_mfma(wa.y, zv.y, acc);
                        acc = nn_mfma(wa.z, zv.z, acc);
                        acc = nn_mfma(wa.w, zv.w, acc);
                    }
                }
                dht[q] = acc;
            }
        }

        // dW_l = H_l^T dZ: tiles of 32 input units x 32 output units
        const int tr = (w_in + 31) / 32, tc = w_out / 32;
        for (int q = wave; q < tr * tc; q += kNnWaves) {
            const int ti = q / tc, tj = q % tc;
            const int i0 = ti * 32, j0 = tj * 32;
            nn_f32x16 acc = {};
#pragma unroll 4
            for (int c = 0; c < kNnBatch / 2; ++c) {
                const int s = 2 * c + h;
                acc = nn_mfma(hin[s * ldi + i0 + li], dz[s * ldo + j0 + li], acc);
            }
            const int base = a.off_w[l] + j0 + li;
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int i = i0 + nn_acc_row(r, h);
                if (i < w_in) emit(base + i * w_out, acc[r]);
            }
        }

        if (l > 0) {
            // every read of H_l (dW) is done: dZ_{l-1} = dH masked by H_l > 0,
            // written in place (sample li, units tile*32 + 8g + 4h + 0..3)
            __syncthreads();
#pragma unroll
            for (int q = 0; q < kNnMaxWidth / 32 / kNnWaves; ++q) {
                const int tile = wave + q * kNnWaves;
                if (tile < tin) {
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        float *p = hin + li * ldi + tile * 32 + 8 * g + 4 * h;
                        float4 hv = *reinterpret_cast<float4 *>(p);
                        hv.x = hv.x > 0.0f ? dht[q][4 * g + 0] : 0.0f;
                        hv.y = hv.y > 0.0f ? dht[q][4 * g + 1] : 0.0f;
                        hv.z = hv.z > 0.0f ? dht[q][4 * g + 2] : 0.0f;
                        hv.w = hv.w > 0.0f ? dht[q][4 * g + 3] : 0.0f;
                        *reinterpret_cast<float4 *>(p) = hv;
                    }
                }
            }
            __syncthreads();
        }
    }
}

// forward of the whole network at `theta`; returns the minibatch mean CE and
// leaves dZ_out in the logits buffer, the hidden activations in h[l].
__device__ float nn_forward(const NnArgs &a, const float *theta, float *lds, const int *rows,
                            int nrows, float *red) {
    const int L = a.L;
    for (int l = 0; l < L; ++l) {
        const float *in = lds + (l ? a.lds_h[l - 1] : a.lds_x);
        nn_forward_hidden(theta + a.off_w[l], theta + a.off_b[l], a.dims[l], a.dims[l + 1], in,
                          nn_ld(a.dims[l]), lds + a.lds_h[l], nn_ld(a.dims[l + 1]),
                          lds + a.lds_part);
        __syncthreads();
    }
    const float *hl = lds + (L ? a.lds_h[L - 1] : a.lds_x);
    nn_forward_logits(theta + a.off_w[L], theta + a.off_b[L], a.dims[L], a.K, hl,
                      nn_ld(a.dims[L]), lds + a.lds_z, nn_ld(a.K));
    __syncthreads();
    return nn_softmax_ce(a, rows, nrows, lds + a.lds_z, nn_ld(a.K), red);
}

// block-wide float64 sums of NV values per thread (wave butterfly + LDS)
template <int NV>
__device__ __forceinline__ void nn_block_sum(double (&v)[NV], double *red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
    for (int k = 0; k < NV; ++k)
        for (int off = 32; off >= 1; off >>= 1) v[k] += __shfl_xor(v[k], off);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < NV; ++k) red[wave * NV + k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
        double s = 0.0;
        for (int w = 0; w < kNnWaves; ++w) s += red[w * NV + k];
        v[k] = s;
    }
    __syncthreads();
}

__device__ __forceinline__ float nn_lr(float act) {
    return static_cast<float>(exp10(static_cast<double>(act - 4.0f)));
}

// ------------------------------------------------------------------ kernels
struct NnGradEmit {
    const float *theta, *act;
    float *theta_n, *gprev;
    const int32_t *agent_row;
    bool fresh;
    double lr_sum = 0.0, lr_sq = 0.0, g_sum = 0.0;
    __device__ __forceinline__ void operator()(int p, float g) {
        const float lr = nn_lr(act[agent_row[p]]);
        theta_n[p] = theta[p] - g * lr;
        lr_sum += lr;
        lr_sq += static_cast<double>(lr) * lr;
        if (fresh) {
            gprev[p] = g;
            g_sum += g;
        }
    }
};

__global__ __launch_bounds__(kNnBlock, 2) void nn_grad_kernel(NnArgs a) {
#pragma clang fp contract(off)
    extern __shared__ float lds[];
    __shared__ int rows[kNnBatch];
    __shared__ double red[kNnWaves * 4];
    const size_t e = blockIdx.x;
    const size_t ps = a.Ps;
    const int nrows = nn_stage_batch(a, e, lds, rows);
    __syncthreads();
    const float *theta = a.theta + e * ps;
    const float loss = nn_forward(a, theta, lds, rows, nrows, reinterpret_cast<float *>(red));
    const bool fresh = a.step[e] == 0;
    NnGradEmit em{theta, a.act + e * a.P, a.theta_n + e * ps, a.gprev + e * ps, a.agent_row,
                  fresh};
    nn_backward(a, theta, lds, em);
    double v[3] = {em.lr_sum, em.lr_sq, em.g_sum};
    nn_block_sum<3>(v, red);
    if (threadIdx.x == 0) {
        a.lr_stats[2 * e] = v[0];
        a.lr_stats[2 * e + 1] = v[1];
        if (fresh) {
            // the reset's History: [entry of model.get() at theta0, 0, 0, 0, 0]
            for (int k = 0; k < kRawHist; ++k) {
                a.hl[k * a.E + e] = k == 0 ? loss : 0.0f;
                a.hsg[k * a.E + e] = k == 0 ? v[2] : 0.0;
            }
        }
    }
}

struct NnStepEmit {
    // copies of the argument fields used per element (a pointer to the
    // kernel argument block would force it into scratch)
    float *theta, *gprev, *rw, *rg, *obs;
    const float *theta_n, *theta0;
    const int32_t *agent_row;
    size_t plane;                  // E * Ps: stride between ring slots
    size_t obs_base;               // e * P
    int s, H, slot;                // step, history length, adjusted slot of this step
    bool wipe;
    const float *lobs;             // [H] l~ entries in obs form, age order (LDS)
    double sum_w = 0.0, sum_aw = 0.0, sum_ag = 0.0, sum_g = 0.0, sum_gd = 0.0;
    __device__ __forceinline__ void operator()(int p, float g) {
        const float th_old = theta[p];
        const float th_new = theta_n[p];
        const float gp = gprev[p];
        const double adj_w = ratio(th_new, th_old);
        const double adj_g = ratio(g, gp);
        sum_w += fabs(static_cast<double>(th_new));
        sum_aw += fabs(adj_w);
        sum_ag += fabs(adj_g);
        sum_g += g;
        sum_gd += fabs(static_cast<double>(g) - static_cast<double>(gp));
        const float ow = static_cast<float>(clip100(adj_w) - 1.0);
        const float og = static_cast<float>(clip100(adj_g) - 1.0);
        float *dst = obs + (obs_base + agent_row[p]) * (3 * static_cast<size_t>(H));
        for (int k = 0; k < H; ++k) {
            float wk, gk, lk;
            if (wipe) {
                wk = gk = lk = -1.0f;
            } else if (k == 0) {
                wk = ow;
                gk = og;
                lk = lobs[0];
            } else if (k < s) {
                const int sl = ((slot - k) % H + H) % H;
                wk = rw[sl * plane + p];
                gk = rg[sl * plane + p];
                lk = lobs[k];
            } else {
                wk = gk = lk = -1.0f;          // clip(0) - 1: the reset zeros
            }
            dst[k] = wk;
            dst[H + k] = lk;
            dst[2 * H + k] = gk;
        }
        rw[slot * plane + p] = ow;
        rg[slot * plane + p] = og;
        gprev[p] = g;
        theta[p] = wipe ? theta0[p] : th_new;
    }
};

__global__ __launch_bounds__(kNnBlock, 2) void nn_step_kernel(NnArgs a) {
#pragma clang fp contract(off)
    extern __shared__ float lds[];
    __shared__ int rows[kNnBatch];
    __shared__ double red[kNnWaves * 5];
    __shared__ int32_t comp[1];
    __shared__ float lobs[kNnMaxH];
    const size_t e = blockIdx.x;
    const size_t ps = a.Ps, E = a.E;
    const int tid = threadIdx.x, H = a.H;
    const int nrows = nn_stage_batch(a, e, lds, rows);
    __syncthreads();
    const float *theta_n = a.theta_n + e * ps;
    const float loss = nn_forward(a, theta_n, lds, rows, nrows, reinterpret_cast<float *>(red));

    // History append (raw, 5 entries) and observation v3 of the loss
    const int s = a.step[e] + 1;
    const int slot5 = s % kRawHist, prev5 = (s - 1) % kRawHist;
    const float l_prev = a.hl[prev5 * E + e];
    const double adj_l = ratio(loss, l_prev);
    const int slot = (s - 1) % H;
    double reward = 1.0 - adj_l;
    reward = reward < -100.0 ? -100.0 : (reward > 100.0 ? 100.0 : reward);
    bool terminal = s >= a.max_batches;
    if (!terminal && loss > 1e4f) {
        terminal = true;
        reward -= static_cast<double>(a.max_batches - s);
    }
    const bool wipe = terminal && a.auto_reset;

    NnStepEmit em;
    em.theta = a.theta + e * ps;
    em.gprev = a.gprev + e * ps;
    em.rw = a.rw + e * ps;
    em.rg = a.rg + e * ps;
    em.obs = a.obs;
    em.theta_n = theta_n;
    em.theta0 = a.theta0 + e * ps;
    em.agent_row = a.agent_row;
    em.plane = E * ps;
    em.obs_base = e * a.P;
    em.s = s;
    em.H = H;
    em.slot = slot;
    em.wipe = wipe;
    if (tid < H) {
        const int k = tid;
        double lk = 0.0;
        if (k == 0) lk = adj_l;
        else if (k < s) lk = a.al[(((slot - k) % H + H) % H) * E + e];
        lobs[k] = static_cast<float>(clip100(lk) - 1.0);
    }
    em.lobs = lobs;
    __syncthreads();
    nn_backward(a, theta_n, lds, em);
    double v[5] = {em.sum_w, em.sum_aw, em.sum_ag, em.sum_g, em.sum_gd};
    nn_block_sum<5>(v, red);

    const int P = a.P;
    if (tid == 0) {
        // rings: this step's entries, then the info sums over them
        a.al[slot * E + e] = adj_l;
        a.sw[slot * E + e] = v[1];
        a.sg[slot * E + e] = v[2];
        a.hl[slot5 * E + e] = loss;
        a.hsg[slot5 * E + e] = v[3];
        double lsum = 0.0, gsum = 0.0, st = 0.0;
        for (int k = 0; k < kRawHist; ++k) {
            lsum += a.hl[k * E + e];
            gsum += a.hsg[k * E + e];
        }
        for (int k = 0; k < H && k < s; ++k) {
            const int sl = ((slot - k) % H + H) % H;
            st += a.sw[sl * E + e] + a.sg[sl * E + e] + P * fabs(a.al[sl * E + e]);
        }
        const double n = P;
        const double amean = a.lr_stats[2 * e] / n;
        const double avar = fmax(a.lr_stats[2 * e + 1] / n - amean * amean, 0.0);
        float *info = a.info + e * kMultiInfo;
        info[0] = terminal ? loss : __builtin_nanf("");
        info[1] = loss;
        info[2] = static_cast<float>(v[0] / n);
        info[3] = static_cast<float>(v[0]);
        info[4] = static_cast<float>(amean);
        info[5] = static_cast<float>(sqrt(avar));
        info[6] = static_cast<float>(st / (n * 3 * H));
        info[7] = static_cast<float>(st);
        info[8] = static_cast<float>(gsum / (kRawHist * n));
        info[9] = static_cast<float>(gsum);
        info[10] = static_cast<float>(lsum / kRawHist);
        info[11] = static_cast<float>(adj_l);
        info[12] = static_cast<float>(v[2] / n);
        info[13] = static_cast<float>(v[4] / n);
        a.episode_len[e] = s;
        a.step[e] = wipe ? 0 : s;
        // model.next() (optimize_nn.py:102-112), then the reset's
        // on_epoch_end when the env restarts; both compose the row order
        const int cur = a.cursor[e] + 1;
        const bool wrap = cur >= a.nb;
        a.cursor[e] = wipe || wrap ? 0 : cur;
        comp[0] = (wrap ? 1 : 0) | (wipe ? 2 : 0);
    }
    // reward / done rows (replicated per agent, optvecenv.py:43-45)
    const float rw = static_cast<float>(reward);
    for (int r = tid; r < P; r += kNnBlock) {
        a.reward[e * P + r] = rw;
        a.done[e * P + r] = terminal ? 1 : 0;
    }
    __syncthreads();
    const int c = comp[0];
    if (c) {
        const int sel = a.order_sel[e];
        const int32_t *cur = a.order + (static_cast<size_t>(sel) * E + e) * a.N;
        int32_t *nxt = a.order + (static_cast<size_t>(1 - sel) * E + e) * a.N;
        const int32_t *pi = a.epoch_perm + e * a.N, *rho = a.reset_perm + e * a.N;
        for (int i = tid; i < a.N; i += kNnBlock) {
            int j = (c & 2) ? rho[i] : i;
            if (c & 1) j = pi[j];
            nxt[i] = cur[j];
        }
        __syncthreads();
        if (tid == 0) a.order_sel[e] = 1 - sel;
    }
}

// MultiOptLRs.base_reset (multioptlrs.py:66-78) of every env: the problem at
// its initial weights, the row order composed with the reset shuffle, batch
// 0 current, obs = clip(nan_to_num(0)) - 1 = -1.  The reset's model.get()
// runs in the next step's nn_grad_kernel (step == 0).
__global__ __launch_bounds__(kNnBlock) void nn_reset_kernel(NnArgs a) {
    const size_t e = blockIdx.x;
    const size_t ps = a.Ps, E = a.E;
    const int tid = threadIdx.x;
    for (int p = tid; p < a.P; p += kNnBlock) a.theta[e * ps + p] = a.theta0[e * ps + p];
    const size_t row = 3 * static_cast<size_t>(a.H);
    float *o = a.obs + e * a.P * row;
    for (size_t i = tid; i < a.P * row; i += kNnBlock) o[i] = -1.0f;
    const int sel = a.order_sel[e];
    const int32_t *cur = a.order + (static_cast<size_t>(sel) * E + e) * a.N;
    int32_t *nxt = a.order + (static_cast<size_t>(1 - sel) * E + e) * a.N;
    const int32_t *rho = a.reset_perm + e * a.N;
    for (int i = tid; i < a.N; i += kNnBlock) nxt[i] = cur[rho[i]];
    __syncthreads();
    if (tid == 0) {
        a.order_sel[e] = 1 - sel;
        a.cursor[e] = 0;
        a.step[e] = 0;
    }
}

}  // namespace ce
