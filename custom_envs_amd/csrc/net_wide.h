// The wide-layer network path: Optimize-v0 over an OptimizeNN network with
// a hidden layer wider than kNetMaxOp (256) units, which the register-chained
// forward of net_kernels.h cannot hold (create_neural_net, utils_model.py:34
// / utils_tf.py:74-86, accepts any width).  Same step, same outputs, same
// float32 model as the MFMA path, on plain tiled kernels:
//
//   net_wide_update_kernel  W' = W - a into the NATURAL weight image (layer l
//                           rows = its input units in order, op_l columns;
//                           biases in unit order), step += 1
//   net_wide_gemm_kernel    per layer: the minibatch forward H_l = relu(H_{l-1}
//                           W_l + b_l) (layer 0 reads the env's minibatch rows
//                           of the dataset through its row order), the
//                           logits, the info forward over every dataset row,
//                           and the backward dZ_l = (dZ_{l+1} W_{l+1}^T) *
//                           (H_l > 0) -- one 64 x 64 tile of one env per
//                           workgroup, float32 FMAs in k order
//   net_wide_loss_kernel    softmax / -log(p_y + 1e-16) / argmax per row, the
//                           64-row tile partials net_finish_kernel reads, and
//                           dZ = P - Y in place (minibatch)
//   net_grad_kernel         [dW; db] and the float64 epilogue (shared with the
//                           MFMA path: it reads the activations and dZ only)
//   net_finish_kernel       L', reward, done, info, the auto-reset (shared)
//
// All on the caller's stream, in that order.  This is a capability path: the
// benchmark's (256, 256) network and every width <= 256 stay on the MFMA
// kernels.
#pragma once

#include "net_kernels.h"

namespace ce {

// C[e] (M x N) = A[e] (M x K) . B[e] (K x N) [+ bias] [relu] [* (mask > 0)].
// A row m is A + m lda, or, with `order`, dataset row order[sel_e][e][m] of A
// (shared by all envs: a_env = 0).  B(k, n) = B[k ldb + n], or B[n ldb + k]
// with b_trans.
struct WideGemmArgs {
    int E, M, N, K;
    const float *A;
    int64_t a_env;
    int lda;
    const int32_t *order;            // [2][E][n_rows] or nullptr
    const int32_t *order_sel;
    int n_rows;
    const float *B;
    int64_t b_env;
    int ldb, b_trans;
    const float *bias;               // [N] at bias + e bias_env, or nullptr
    int64_t bias_env;
    int relu;
    const float *mask;               // relu' source: C = mask > 0 ? C : 0, or nullptr
    int64_t mask_env;
    int ldm;
    float *C;
    int64_t c_env;
    int ldc;
};

constexpr int kWideTile = 64;
constexpr int kWideK = 16;

__global__ __launch_bounds__(256) void net_wide_gemm_kernel(WideGemmArgs a) {
    const int e = blockIdx.z;
    const int n0 = blockIdx.x * kWideTile, m0 = blockIdx.y * kWideTile;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    __shared__ float As[kWideK][kWideTile + 4];
    __shared__ float Bs[kWideK][kWideTile + 4];
    const int32_t *rows =
        a.order ? a.order + (static_cast<size_t>(a.order_sel[e]) * a.E + e) * a.n_rows : nullptr;
    const float *A = a.A + static_cast<size_t>(e) * a.a_env;
    const float *B = a.B + static_cast<size_t>(e) * a.b_env;
    // this thread's A loads: row ar of the tile, k columns ak .. ak + 3
    const int ar = tid >> 2, ak = (tid & 3) * 4;
    const int am = m0 + ar;
    const float *arow = am < a.M ? A + static_cast<int64_t>(rows ? rows[am] : am) * a.lda : nullptr;
    float acc[4][4] = {};
    for (int k0 = 0; k0 < a.K; k0 += kWideK) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            const int k = k0 + ak + c;
            As[ak + c][ar] = arow && k < a.K ? arow[k] : 0.0f;
        }
        if (!a.b_trans) {
            const int bk = tid >> 4, bn = (tid & 15) * 4, k = k0 + bk;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int n = n0 + bn + c;
                Bs[bk][bn + c] = k < a.K && n < a.N ? B[static_cast<int64_t>(k) * a.ldb + n] : 0.0f;
            }
        } else {
            const int bn = tid >> 2, bk = (tid & 3) * 4, n = n0 + bn;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int k = k0 + bk + c;
                Bs[bk + c][bn] = k < a.K && n < a.N ? B[static_cast<int64_t>(n) * a.ldb + k] : 0.0f;
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < kWideK; ++kk) {
            float av[4], bv[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) av[i] = As[kk][ty * 4 + i];
#pragma unroll
            for (int j = 0; j < 4; ++j) bv[j] = Bs[kk][tx * 4 + j];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j < 4; ++j) acc[i][j] = fmaf(av[i], bv[j], acc[i][j]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int m = m0 + ty * 4 + i;
        if (m >= a.M) continue;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int n = n0 + tx * 4 + j;
            if (n >= a.N) continue;
            float v = acc[i][j];
            if (a.bias) v += a.bias[static_cast<size_t>(e) * a.bias_env + n];
            if (a.relu) v = v > 0.0f ? v : 0.0f;
            if (a.mask)
                v = a.mask[static_cast<size_t>(e) * a.mask_env + static_cast<int64_t>(m) * a.ldm + n] > 0.0f ? v
                                                                                                             : 0.0f;
            a.C[static_cast<size_t>(e) * a.c_env + static_cast<int64_t>(m) * a.ldc + n] = v;
        }
    }
}

// Per row r < R of env e: the softmax of its K logits (utils_math.py:51-63),
// -log(p_y + 1e-16) (utils_math.py:25-34) and np.argmax's first maximum --
// the float32 operations of net_fwd_kernel's epilogue -- summed per 64-row
// tile into part_loss / part_hits [E][T]; with write_dz, dZ = P - Y over the
// logits in place.  One 64-thread workgroup per tile.
struct WideLossArgs {
    int E, R, K, T, write_dz;
    float *Z;                        // logits: row r of env e at Z + e z_env + r ldz
    int64_t z_env;
    int ldz;
    const int32_t *label;            // [n_rows]
    const int32_t *order;            // label of row r: label[order[sel_e][e][r]], or label[r]
    const int32_t *order_sel;
    int n_rows;
    double *part_loss;
    int32_t *part_hits;
};

__global__ __launch_bounds__(64) void net_wide_loss_kernel(WideLossArgs a) {
    const int e = blockIdx.y, tile = blockIdx.x, tid = threadIdx.x;
    const int r = tile * 64 + tid;
    __shared__ double sl[64];
    __shared__ int sh[64];
    double loss_r = 0.0;
    int hit_r = 0;
    if (r < a.R) {
        float *z = a.Z + static_cast<size_t>(e) * a.z_env + static_cast<int64_t>(r) * a.ldz;
        const int32_t *rows =
            a.order ? a.order + (static_cast<size_t>(a.order_sel[e]) * a.E + e) * a.n_rows : nullptr;
        const int yl = a.label[rows ? rows[r] : r];
        const int K = a.K;
        float p[kNetMaxClasses];
        float m = z[0];
#pragma unroll
        for (int k = 0; k < kNetMaxClasses; ++k) {
            p[k] = k < K ? z[k] : 0.0f;
            if (k > 0 && k < K) m = fmaxf(m, p[k]);
        }
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < kNetMaxClasses; ++k)
            if (k < K) {
                p[k] = expf(p[k] - m);
                s += p[k];
            }
        int arg = 0;
        float best = -1.0f, py = 0.0f;
#pragma unroll
        for (int k = 0; k < kNetMaxClasses; ++k)
            if (k < K) {
                p[k] = p[k] / s;
                if (p[k] > best) {
                    best = p[k];
                    arg = k;
                }
                if (k == yl) py = p[k];
            }
        loss_r = static_cast<double>(-logf(py + 1e-16f));
        hit_r = arg == yl ? 1 : 0;
        if (a.write_dz) {
#pragma unroll
            for (int k = 0; k < kNetMaxClasses; ++k)
                if (k < K) z[k] = p[k] - (k == yl ? 1.0f : 0.0f);
        }
    }
    sl[tid] = loss_r;
    sh[tid] = hit_r;
    __syncthreads();
    if (tid == 0) {
        double l = 0.0;
        int h = 0;
        for (int i = 0; i < 64; ++i) {
            l += sl[i];
            h += sh[i];
        }
        a.part_loss[static_cast<size_t>(e) * a.T + tile] = l;
        a.part_hits[static_cast<size_t>(e) * a.T + tile] = h;
    }
}

// W' = W - a (optimize.py:74-75, one float32 subtraction) from the flat
// action into the natural image; current_step += 1 (baseenvironment.py:30-41)
struct WideUpdArgs {
    NetGeom g;
    int E;
    int64_t P;
    float *img;
    const float *act;
    int32_t *step;
};

__global__ __launch_bounds__(256) void net_wide_update_kernel(WideUpdArgs a) {
    const int e = blockIdx.y;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.step[e] += 1;
    float *img = a.img + static_cast<size_t>(e) * a.g.Pimg;
    const float *act = a.act + static_cast<size_t>(e) * a.P;
    for (int64_t p = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; p < a.P;
         p += static_cast<int64_t>(gridDim.x) * 256) {
        int l = 0;
        while (l + 1 < a.g.nl && p >= a.g.flat_w[l + 1]) ++l;
        const int64_t q = p - a.g.flat_w[l];
        const int64_t nw = static_cast<int64_t>(a.g.din[l]) * a.g.dout[l];
        int64_t dst;
        if (q < nw) {
            const int64_t k = q / a.g.dout[l], u = q - k * a.g.dout[l];
            dst = a.g.img_off[l] + k * a.g.op[l] + u;
        } else {
            dst = a.g.bias_base + a.g.bias_rel[l] + (q - nw);
        }
        img[dst] -= act[p];
    }
}

}  // namespace ce
