// MultiOptLRs-v0 over the OptimizeNN problem for gfx950.
//
// One OptVecEnv.step of E envs is five launches on one stream:
//   nn_grad_kernel      (one 512-thread workgroup per env) grad =
//                       model.get_gradient(): forward + backward of the
//                       F -> hidden... (relu) -> K softmax network on the
//                       current batch (multioptlrs.py:85, optimize_nn.py:
//                       35-52,122-126); for an env just reset this is also the
//                       reset's model.get() (multioptlrs.py:70-71)
//   nn_update_kernel    (four agents per thread) lr = 10^(a - 4)
//                       (utils_env.py:113-114), theta' = theta - grad * lr
//   nn_step_kernel      (per env) grad, loss = model.get() at theta'
//                       (multioptlrs.py:88)
//   nn_agent_rows_kernel (per observation row) History append, obs v3 ratios,
//                       adjusted history, obs = clip(nan_to_num(.), +-100) - 1
//                       (multioptlrs.py:89-101, utils_env.py:155-161)
//   nn_finalize_kernel  (per env) reward v6, early stop, the 14 info values
//                       (multioptlrs.py:102-127), model.next() (optimize_nn.py:
//                       102-112) and OptVecEnv's auto-reset (concurrentvecenv.py:37)
// The per-env kernels are MFMA work with the whole network state of one env
// in LDS; the per-agent kernels stream the HBM state with every load of an
// agent issued before its stores, on a grid of env x (P / 256) blocks.
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
// The output layer (K <= 32 classes) is VALU work.  Gradients leave the
// accumulator registers as one coalesced store per element.
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
constexpr int kNnChunk = 256;      // threads per block of the update / finalize kernels
#ifndef CE_NN_ROWS
#define CE_NN_ROWS 256
#endif
constexpr int kNnRows = CE_NN_ROWS;  // threads (and observation rows) per block of nn_agent_rows_kernel
constexpr int kNnUpdPer = 4;       // agents per thread of nn_update_kernel
constexpr int kNnPrefetch = 8;     // 8-float k-chunks of W in flight per lane

struct NnArgs {
    int E, N, F, K, L, B, nb, H, max_batches, auto_reset;
    int P;                         // parameters (= agents) per env
    int Ps;                        // per-env stride of [E][P] state (P rounded up)
    int dims[kNnMaxHidden + 2];    // F, hidden..., K
    int off_w[kNnMaxHidden + 1];   // flat offset of layer l's kernel [dims[l]][dims[l+1]]
    int off_b[kNnMaxHidden + 1];   // flat offset of layer l's bias
    int lds_x, lds_h[kNnMaxHidden], lds_z, lds_wo, lds_part, lds_bytes;   // float offsets
    int split;                     // 1: some hidden forward needs the split-k scratch
    const float *X;                // [N][F] dataset rows (dataset order)
    const int32_t *label;          // [N]
    // theta/theta_n and gprev/gN are two ping-pong pairs: the engine swaps
    // them every step, so theta' and the new gradient become current
    // without a copy
    float *theta;                  // [E][Ps] current parameters
    float *theta_n;                // [E][Ps] parameters after this step's update
    const float *theta0;           // [E][Ps] reset parameters
    float *gprev;                  // [E][Ps] newest raw-history gradient
    float *gN;                     // [E][Ps] gradient at theta' (this step's entry)
    float *gU;                     // [E][Ps] gradient at theta (the update's)
    float *loss_b;                 // [E] minibatch loss at theta'
    double *part_u;                // [E][nchunk_u][3] update sums (lr, lr^2, reset gradient)
    double *part_c;                // [E][nchunk][5] agent sums (|theta'|, |w~|, |g~|, g, |dg|)
    int nchunk;                    // nn_agent_rows_kernel blocks per env (kNnRows rows each)
    int nchunk_u;                  // nn_update_kernel blocks per env
    float *rw, *rg;                // [H][E][Ps] adjusted w~ / g~ entries, obs form
    double *al;                    // [H][E] adjusted loss entries (raw)
    double *sw, *sg;               // [H][E] sum |w~|, sum |g~| of each entry
    float *hl;                     // [5][E] raw-history losses
    double *hsg;                   // [5][E] raw-history gradient sums
    int32_t *step;                 // [E]
    int32_t *cursor;               // [E] current batch index within the epoch
    int32_t *order;                // [2][E][N] row order (ping-pong)
    int32_t *order_sel;            // [E]
    const int32_t *reset_perm;     // [E][N] the shuffle every reset draws
    const int32_t *epoch_perm;     // [E][N] the shuffle every epoch end draws
    const int32_t *agent_row;      // [P] OptVecEnv row of agent p (sorted names)
    const int32_t *row_agent;      // [P] agent of OptVecEnv row r (the inverse)
    const float *act;              // [E][P] rows
    float *obs;                    // [E][P][3H] rows
    float *reward;                 // [E][P] rows
    uint8_t *done;                 // [E][P] rows
    float *info;                   // [E][14]
    int32_t *episode_len;          // [E]
    unsigned long long *diag;      // [E][kNnStamps] phase stamps (CE_DIAG builds only)
};

// Diagnostic builds (-DCE_DIAG) stamp s_memtime (thread 0 of each eval
// workgroup) at phase boundaries; product builds compile the stamps away.
constexpr int kNnStamps = 10;
#ifdef CE_DIAG
#define NN_STAMP(a, e, k)                                                              \
    do {                                                                               \
        __builtin_amdgcn_sched_barrier(0);                                             \
        unsigned long long t_;                                                         \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");      \
        __builtin_amdgcn_sched_barrier(0);                                             \
        if (threadIdx.x == 0) (a).diag[(e) * kNnStamps + (k)] = t_;                    \
    } while (0)
#define NN_STAMP_RT(a, e, k)                                                           \
    do {                                                                               \
        unsigned long long t_;                                                         \
        asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");  \
        if (threadIdx.x == 0) (a).diag[(e) * kNnStamps + (k)] = t_;                    \
    } while (0)
#else
#define NN_STAMP(a, e, k) \
    do {                  \
    } while (0)
#define NN_STAMP_RT(a, e, k) \
    do {                     \
    } while (0)
#endif

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
        // W fragments stream from HBM kNnPrefetch chunks ahead (a register
        // ring refilled right after use); the X rows come from LDS at use.
        // Loads are branch-free (clamped address, value selected) so the
        // compiler keeps them all in flight instead of fencing each chunk.
        float wb[kNnPrefetch][4];
        const int kmax = w_in - 1, clast = c1 - 1;
        auto loadw = [&](int c, float (&w)[4]) {
            const int cc = c < clast ? c : clast;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int k = 8 * cc + 4 * h + m;
                const float v = W[static_cast<size_t>(k < kmax ? k : kmax) * w_out + j];
                w[m] = k <= kmax ? v : 0.0f;
            }
        };
        if (c0 < c1) {
#pragma unroll
            for (int d = 0; d < kNnPrefetch; ++d) loadw(c0 + d, wb[d]);
        }
        for (int c = c0; c < c1; c += kNnPrefetch) {
#pragma unroll
            for (int d = 0; d < kNnPrefetch; ++d) {
                if (c + d < c1) {                   // uniform
                    const float4 x = *reinterpret_cast<const float4 *>(xrow + 8 * (c + d));
                    acc = nn_mfma(wb[d][0], x.x, acc);
                    acc = nn_mfma(wb[d][1], x.y, acc);
                    acc = nn_mfma(wb[d][2], x.z, acc);
                    acc = nn_mfma(wb[d][3], x.w, acc);
                }
                loadw(c + kNnPrefetch + d, wb[d]);
            }
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
// butterfly.  Rows s >= nrows are computed and ignored.  Up to 4 classes
// (the reference's iris-shaped default) take a 4-accumulator instance: the k
// loops then run to 4, not to 32 with most of their work predicated off.
template <int KM>
__device__ void nn_logits_k(const float *W, const float *bias, int w_in, int K, const float *in,
                            int ld_in, float *z, int ld_z) {
    const int t = threadIdx.x;
    const int s = t >> 4, ch = t & 15;
    const int per = w_in / 16;
    float acc[KM];
#pragma unroll
    for (int k = 0; k < KM; ++k) acc[k] = 0.0f;
    for (int q = 0; q < per; ++q) {
        const int j = ch * per + q;
        const float hv = in[s * ld_in + j];
        const float *wr = W + static_cast<size_t>(j) * K;
#pragma unroll
        for (int k = 0; k < KM; ++k)
            if (k < K) acc[k] = fmaf(hv, wr[k], acc[k]);
    }
#pragma unroll
    for (int k = 0; k < KM; ++k) {
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
        for (int k = 0; k < KM; ++k)
            if (k < K) z[s * ld_z + k] = acc[k] + bias[k];
    }
}
__device__ void nn_forward_logits(const float *W, const float *bias, int w_in, int K,
                                  const float *in, int ld_in, float *z, int ld_z) {
    if (K <= 4) nn_logits_k<4>(W, bias, w_in, K, in, ld_in, z, ld_z);
    else nn_logits_k<kNnMaxK>(W, bias, w_in, K, in, ld_in, z, ld_z);
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
        const float *Wo = lds + a.lds_wo;          // staged by nn_forward
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

    NN_STAMP(a, blockIdx.x, 5);
    // ---- hidden layers l = L-1 .. 0 (layer l maps dims[l] -> dims[l+1]);
    // dZ of its output sits in buffer h[l]
    for (int l = L - 1; l >= 0; --l) {
        const int w_in = a.dims[l], w_out = a.dims[l + 1];
        const float *dz = lds + a.lds_h[l];
        const int ldo = nn_ld(w_out);
        float *hin = lds + (l ? a.lds_h[l - 1] : a.lds_x);
        const int ldi = nn_ld(w_in);
        const float *W = theta + a.off_w[l];
        if (l == 0 && L > 1) NN_STAMP(a, blockIdx.x, 6);

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
                    // float4 W rows kNnPrefetch chunks ahead, branch-free
                    // (clamped addresses) so every load stays in flight
                    float4 wb[kNnPrefetch];
                    const int clast = chunks - 1;
#pragma unroll
                    for (int d = 0; d < kNnPrefetch; ++d)
                        wb[d] = *reinterpret_cast<const float4 *>(wrow + 8 * (d < clast ? d : clast));
                    for (int c = 0; c < chunks; c += kNnPrefetch) {
#pragma unroll
                        for (int d = 0; d < kNnPrefetch; ++d) {
                            if (c + d < chunks) {       // uniform
                                const float4 zv =
                                    *reinterpret_cast<const float4 *>(zrow + 8 * (c + d));
                                acc = nn_mfma(wb[d].x, zv.x, acc);
                                acc = nn_mfma(wb[d].y, zv.y, acc);
                                acc = nn_mfma(wb[d].z, zv.z, acc);
                                acc = nn_mfma(wb[d].w, zv.w, acc);
                            }
                            const int cn = c + kNnPrefetch + d;
                            wb[d] = *reinterpret_cast<const float4 *>(wrow + 8 * (cn < clast ? cn : clast));
                        }
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
    // the output layer's kernel [dims[L]][K] (a few KB) is read by every
    // thread of the logits and dH_L passes: stage it once
    for (int i = threadIdx.x; i < a.dims[L] * a.K; i += kNnBlock)
        lds[a.lds_wo + i] = theta[a.off_w[L] + i];
    for (int l = 0; l < L; ++l) {
        const float *in = lds + (l ? a.lds_h[l - 1] : a.lds_x);
        if (l == 1) NN_STAMP(a, blockIdx.x, 2);
        nn_forward_hidden(theta + a.off_w[l], theta + a.off_b[l], a.dims[l], a.dims[l + 1], in,
                          nn_ld(a.dims[l]), lds + a.lds_h[l], nn_ld(a.dims[l + 1]),
                          lds + a.lds_part);
        __syncthreads();
    }
    NN_STAMP(a, blockIdx.x, 3);
    const float *hl = lds + (L ? a.lds_h[L - 1] : a.lds_x);
    nn_forward_logits(lds + a.lds_wo, theta + a.off_b[L], a.dims[L], a.K, hl,
                      nn_ld(a.dims[L]), lds + a.lds_z, nn_ld(a.K));
    __syncthreads();
    return nn_softmax_ce(a, rows, nrows, lds + a.lds_z, nn_ld(a.K), red);
}

// block-wide float64 sums of NV values per thread (wave butterfly + LDS)
template <int NV, int BLOCK>
__device__ __forceinline__ void nn_block_sum(double (&v)[NV], double *red) {
    constexpr int kW = BLOCK / 64;
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
        for (int w = 0; w < kW; ++w) s += red[w * NV + k];
        v[k] = s;
    }
    __syncthreads();
}

__device__ __forceinline__ float nn_lr(float act) {
    return static_cast<float>(exp10(static_cast<double>(act - 4.0f)));
}

// ------------------------------------------------------------- eval kernels
// The gradient of one forward+backward goes to an [E][Ps] buffer with one
// coalesced store per element (32 lanes x 4 B per accumulator register).
struct NnStore {
    float *g;
    __device__ __forceinline__ void operator()(int p, float v) const { g[p] = v; }
};

__device__ __forceinline__ float nn_eval(const NnArgs &a, size_t e, const float *theta, float *g,
                                         float *lds, int *rows, float *red) {
    NN_STAMP_RT(a, e, 8);
    NN_STAMP(a, e, 0);
    const int nrows = nn_stage_batch(a, e, lds, rows);
    __syncthreads();
    NN_STAMP(a, e, 1);
    const float loss = nn_forward(a, theta, lds, rows, nrows, red);
    NN_STAMP(a, e, 4);
    NnStore st{g};
    nn_backward(a, theta, lds, st);
    NN_STAMP(a, e, 7);
    NN_STAMP_RT(a, e, 9);
    return loss;
}

// model.get_gradient() at theta (multioptlrs.py:85); for an env that was
// just reset it is also the reset's model.get() (multioptlrs.py:70-71):
// same weights, same batch, so it seeds the raw history [l0, 0, 0, 0, 0].
__global__ __launch_bounds__(kNnBlock, 4) void nn_grad_kernel(NnArgs a) {
    extern __shared__ float lds[];
    __shared__ int rows[kNnBatch];
    __shared__ float red[4];
    const size_t e = blockIdx.x, ps = a.Ps;
    const float loss = nn_eval(a, e, a.theta + e * ps, a.gU + e * ps, lds, rows, red);
    if (threadIdx.x == 0 && a.step[e] == 0)
        for (int k = 0; k < kRawHist; ++k) a.hl[k * a.E + e] = k == 0 ? loss : 0.0f;
}

// model.get() at theta' on the same batch (multioptlrs.py:88)
__global__ __launch_bounds__(kNnBlock, 4) void nn_step_kernel(NnArgs a) {
    extern __shared__ float lds[];
    __shared__ int rows[kNnBatch];
    __shared__ float red[4];
    const size_t e = blockIdx.x, ps = a.Ps;
    NnArgs b = a;
#ifdef CE_DIAG
    b.diag = a.diag + static_cast<size_t>(a.E) * kNnStamps;   // the step kernel's own record
#endif
    const float loss = nn_eval(b, e, a.theta_n + e * ps, a.gN + e * ps, lds, rows, red);
    if (threadIdx.x == 0) a.loss_b[e] = loss;
}

// ------------------------------------------------------- elementwise kernels
// One thread per (env, agent); blocks of kNnChunk consecutive agents of one
// env (blockIdx.x = chunk, blockIdx.y = env), every load issued before any
// store so a wave keeps all its memory traffic in flight at once.

// the update (multioptlrs.py:86-87): lr = 10^(a - 4), theta' = theta - g lr;
// per-chunk sums of lr, lr^2 (actions_mean/std) and, after a reset, of the
// reset gradient (the raw history's first entry).  kNnUpdPer agents per
// thread, strided by the block so every load stays coalesced: the action
// gather (through the sorted-name row table) is the second round trip, and
// four agents' worth of it is in flight at once.
__global__ __launch_bounds__(kNnChunk) void nn_update_kernel(NnArgs a) {
#pragma clang fp contract(off)
    __shared__ double red[(kNnChunk / 64) * 3];
    const size_t e = blockIdx.y, ps = a.Ps;
    const int chunk = blockIdx.x;
    const int base = chunk * kNnChunk * kNnUpdPer + threadIdx.x;
    const bool fresh = a.step[e] == 0;
    const float *act = a.act + e * a.P;
    const float *gu = a.gU + e * ps, *th = a.theta + e * ps;
    float g[kNnUpdPer], t[kNnUpdPer], av[kNnUpdPer];
    int row[kNnUpdPer];
#pragma unroll
    for (int q = 0; q < kNnUpdPer; ++q) {
        const int p = base + q * kNnChunk;
        const int pc = p < a.P ? p : 0;
        g[q] = gu[pc];
        t[q] = th[pc];
        row[q] = a.agent_row[pc];
    }
#pragma unroll
    for (int q = 0; q < kNnUpdPer; ++q) av[q] = act[row[q]];
    double v[3] = {0.0, 0.0, 0.0};
    float *tn = a.theta_n + e * ps, *gp = a.gprev + e * ps;
#pragma unroll
    for (int q = 0; q < kNnUpdPer; ++q) {
        const int p = base + q * kNnChunk;
        if (p < a.P) {
            const float lr = nn_lr(av[q]);
            tn[p] = t[q] - g[q] * lr;
            v[0] += lr;
            v[1] += static_cast<double>(lr) * lr;
            if (fresh) {
                gp[p] = g[q];
                v[2] += g[q];
            }
        }
    }
    nn_block_sum<3, kNnChunk>(v, red);
    if (threadIdx.x == 0) {
        double *o = a.part_u + (e * a.nchunk_u + chunk) * 3;
        o[0] = v[0];
        o[1] = v[1];
        o[2] = v[2];
    }
}

// per-env scalars every agent of a step shares (multioptlrs.py:88-107)
struct NnStepScalars {
    int s, slot, slot5;
    float loss;
    double adj_l, reward;
    bool terminal, wipe;
};

__device__ __forceinline__ NnStepScalars nn_step_scalars(const NnArgs &a, size_t e) {
    NnStepScalars r;
    const size_t E = a.E;
    r.s = a.step[e] + 1;
    r.slot = (r.s - 1) % a.H;
    r.slot5 = r.s % kRawHist;
    r.loss = a.loss_b[e];
    const float l_prev = a.hl[((r.s - 1) % kRawHist) * E + e];
    r.adj_l = ratio(r.loss, l_prev);
    double reward = 1.0 - r.adj_l;
    reward = reward < -100.0 ? -100.0 : (reward > 100.0 ? 100.0 : reward);
    r.terminal = r.s >= a.max_batches;
    if (!r.terminal && r.loss > 1e4f) {
        r.terminal = true;
        reward -= static_cast<double>(a.max_batches - r.s);
    }
    r.reward = reward;
    r.wipe = r.terminal && a.auto_reset;
    return r;
}

// History append + observation v3 + adjusted history + obs rows
// (multioptlrs.py:89-101; on auto-reset theta_n <- theta0), in OBSERVATION-ROW
// order: block = kNnChunk consecutive obs rows of one env, thread = row r,
// agent p = row_agent[r].  (An agent-order form measured 1.87-1.94 ms at
// 1024 envs against 1.44 ms for this one)
//   - The block's observation rows are one contiguous run of kNnChunk * 3H
//     floats: staged in LDS at the run's 16-byte phase, then written as
//     float4s (plus at most 3 head and 3 tail floats) instead of 4-byte
//     stores around the holes the other agents' rows leave in agent order.
//   - The adjusted rings are kept in row order, so their reads and writes
//     stay contiguous; theta, theta' and the gradients are gathered through
//     row_agent, which in sorted-name order is runs of consecutive agents.
//   - The per-block sums (|theta'|, |w~|, |g~|, g, |dg|) are sums over the
//     same agents in another order.
__global__ __launch_bounds__(kNnRows) void nn_agent_rows_kernel(NnArgs a) {
#pragma clang fp contract(off)
    extern __shared__ float4 stage4[];             // [kNnRows * 3H + 4] rows at the run's phase
    float *stage = reinterpret_cast<float *>(stage4);
    __shared__ float lobs[kNnMaxH];
    __shared__ double red[(kNnRows / 64) * 5];
    const size_t e = blockIdx.y, ps = a.Ps, E = a.E;
    const int chunk = blockIdx.x, tid = threadIdx.x, H = a.H, W = 3 * H;
    const int r0 = chunk * kNnRows;
    const int r = r0 + tid;
    const bool on = r < a.P;
    const int rc = on ? r : r0;
    const NnStepScalars sc = nn_step_scalars(a, e);
    const int s = sc.s, slot = sc.slot;
    const size_t plane = E * ps;
    const size_t eb = e * ps;

    // ---- every load up front: the agent, its four values, its ring ages
    const int p = a.row_agent[rc];
    const float to = a.theta[eb + p], tn = a.theta_n[eb + p];
    const float gp = a.gprev[eb + p], g = a.gN[eb + p];
    float rwv[kNnMaxH], rgv[kNnMaxH];
#pragma unroll
    for (int k = 1; k < kNnMaxH; ++k) {
        if (k < H && k < s) {                       // block-uniform
            const size_t sl = ((slot - k) % H + H) % H;
            rwv[k] = a.rw[sl * plane + eb + rc];
            rgv[k] = a.rg[sl * plane + eb + rc];
        } else {
            rwv[k] = rgv[k] = -1.0f;                // clip(0) - 1: the reset zeros
        }
    }
    if (tid < H) {
        const int k = tid;
        double lk = 0.0;
        if (k == 0) lk = sc.adj_l;
        else if (k < s) lk = a.al[(((slot - k) % H + H) % H) * E + e];
        lobs[k] = static_cast<float>(clip100(lk) - 1.0);
    }
    const double adj_w = ratio_fast(tn, to);
    const double adj_g = ratio_fast(g, gp);
    const float ow = static_cast<float>(clip100(adj_w) - 1.0);
    const float og = static_cast<float>(clip100(adj_g) - 1.0);
    double v[5] = {0.0, 0.0, 0.0, 0.0, 0.0};
    if (on) {
        v[0] = fabs(static_cast<double>(tn));
        v[1] = fabs(adj_w);
        v[2] = fabs(adj_g);
        v[3] = g;
        v[4] = fabs(static_cast<double>(g) - static_cast<double>(gp));
        a.rw[slot * plane + eb + r] = ow;
        a.rg[slot * plane + eb + r] = og;
        if (sc.wipe) a.theta_n[eb + p] = a.theta0[eb + p];
    }
    // ---- the block's rows: global floats [g0, g0 + n), staged at LDS
    // position (global index - g0) + off, off = the run's float phase within
    // a 16-byte unit of the ACTUAL address (a caller's obs pointer need only
    // be 4-byte aligned), so 16-byte global chunks are 16-byte LDS chunks
    const size_t g0 = (e * static_cast<size_t>(a.P) + r0) * W;
    const int off = static_cast<int>((reinterpret_cast<uintptr_t>(a.obs + g0) >> 2) & 3);
    __syncthreads();                                // lobs ready
    if (on) {
        float *st = stage + off + tid * W;
#pragma unroll
        for (int k = 0; k < kNnMaxH; ++k) {
            if (k < H) {
                st[k] = sc.wipe ? -1.0f : (k == 0 ? ow : rwv[k]);
                st[H + k] = sc.wipe ? -1.0f : lobs[k];
                st[2 * H + k] = sc.wipe ? -1.0f : (k == 0 ? og : rgv[k]);
            }
        }
    }
    __syncthreads();
    const int n = (a.P - r0 < kNnRows ? a.P - r0 : kNnRows) * W;
    const size_t a0 = g0 + ((4 - off) & 3);             // first 16-byte-aligned float
    const size_t a1 = a0 + ((g0 + n - a0) & ~size_t(3)) * (g0 + n >= a0);   // end of whole units
    float *obs = a.obs;
#ifdef CE_NN_DIAG_NOOBS
    if (n < 0)   // timing diagnostic: no observation stores
#endif
    {
        if (a1 > a0) {
            const int head = static_cast<int>(a0 - g0), tail = static_cast<int>(g0 + n - a1);
            if (tid < head) obs[g0 + tid] = stage[off + tid];
            if (tid < tail) obs[a1 + tid] = stage[off + static_cast<int>(a1 - g0) + tid];
            const int nb = static_cast<int>((a1 - a0) >> 2);
            const float4 *src = reinterpret_cast<const float4 *>(stage + off + head);
            float4 *dst = reinterpret_cast<float4 *>(obs + a0);
            for (int i = tid; i < nb; i += kNnRows) dst[i] = src[i];
        } else {
            for (int i = tid; i < n; i += kNnRows) obs[g0 + i] = stage[off + i];
        }
    }
    nn_block_sum<5, kNnRows>(v, red);
    if (tid == 0) {
        double *o = a.part_c + (e * a.nchunk + chunk) * 5;
        for (int k = 0; k < 5; ++k) o[k] = v[k];
    }
}

// reward, info, rings of per-step sums, step counter, model.next() and the
// auto-reset's row order (multioptlrs.py:102-128, optimize_nn.py:102-120)
__global__ __launch_bounds__(kNnChunk) void nn_finalize_kernel(NnArgs a) {
    __shared__ double red[(kNnChunk / 64) * 8];
    __shared__ int32_t comp[1];
    const size_t e = blockIdx.x, E = a.E;
    const int tid = threadIdx.x, H = a.H, P = a.P;
    double v[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    for (int c = tid; c < a.nchunk_u; c += kNnChunk) {
        const double *u = a.part_u + (e * a.nchunk_u + c) * 3;
        v[0] += u[0];
        v[1] += u[1];
        v[2] += u[2];
    }
    for (int c = tid; c < a.nchunk; c += kNnChunk) {
        const double *q = a.part_c + (e * a.nchunk + c) * 5;
        for (int k = 0; k < 5; ++k) v[3 + k] += q[k];
    }
    nn_block_sum<8, kNnChunk>(v, red);
    const NnStepScalars sc = nn_step_scalars(a, e);
    const int s = sc.s;
    if (tid == 0) {
        if (s == 1) {
            // the reset's raw-history gradient entry (nn_update_kernel sums)
            for (int k = 0; k < kRawHist; ++k) a.hsg[k * E + e] = k == 0 ? v[2] : 0.0;
        }
        a.al[sc.slot * E + e] = sc.adj_l;
        a.sw[sc.slot * E + e] = v[4];
        a.sg[sc.slot * E + e] = v[5];
        a.hl[sc.slot5 * E + e] = sc.loss;
        a.hsg[sc.slot5 * E + e] = v[6];
        double lsum = 0.0, gsum = 0.0, st = 0.0;
        for (int k = 0; k < kRawHist; ++k) {
            lsum += a.hl[k * E + e];
            gsum += a.hsg[k * E + e];
        }
        for (int k = 0; k < H && k < s; ++k) {
            const int sl = ((sc.slot - k) % H + H) % H;
            st += a.sw[sl * E + e] + a.sg[sl * E + e] + P * fabs(a.al[sl * E + e]);
        }
        const double n = P;
        const double amean = v[0] / n;
        const double avar = fmax(v[1] / n - amean * amean, 0.0);
        float *info = a.info + e * kMultiInfo;
        info[0] = sc.terminal ? sc.loss : __builtin_nanf("");
        info[1] = sc.loss;
        info[2] = static_cast<float>(v[3] / n);
        info[3] = static_cast<float>(v[3]);
        info[4] = static_cast<float>(amean);
        info[5] = static_cast<float>(sqrt(avar));
        info[6] = static_cast<float>(st / (n * 3 * H));
        info[7] = static_cast<float>(st);
        info[8] = static_cast<float>(gsum / (kRawHist * n));
        info[9] = static_cast<float>(gsum);
        info[10] = static_cast<float>(lsum / kRawHist);
        info[11] = static_cast<float>(sc.adj_l);
        info[12] = static_cast<float>(v[5] / n);
        info[13] = static_cast<float>(v[7] / n);
        a.episode_len[e] = s;
        a.step[e] = sc.wipe ? 0 : s;
        const int cur = a.cursor[e] + 1;
        const bool wrap = cur >= a.nb;
        a.cursor[e] = sc.wipe || wrap ? 0 : cur;
        comp[0] = (wrap ? 1 : 0) | (sc.wipe ? 2 : 0);
    }
    // reward / done rows (replicated per agent, optvecenv.py:43-45)
    const float rw = static_cast<float>(sc.reward);
    for (int r = tid; r < P; r += kNnChunk) {
        a.reward[e * P + r] = rw;
        a.done[e * P + r] = sc.terminal ? 1 : 0;
    }
    __syncthreads();
    const int c = comp[0];
    if (c) {
        const int sel = a.order_sel[e];
        const int32_t *cur = a.order + (static_cast<size_t>(sel) * E + e) * a.N;
        int32_t *nxt = a.order + (static_cast<size_t>(1 - sel) * E + e) * a.N;
        const int32_t *pi = a.epoch_perm + e * a.N, *rho = a.reset_perm + e * a.N;
        for (int i = tid; i < a.N; i += kNnChunk) {
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
