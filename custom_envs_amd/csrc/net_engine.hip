// Optimize-v0 over a general OptimizeNN network (net_engine.h has the step's
// launch sequence).  The dense products of every layer are plain GEMMs over
// the envs' parameter slabs -- strided-batched f32 GEMMs, batch = envs, the
// dataset operand shared (stride 0) -- and everything around them is
// hand-written: the update and the minibatch gather, the softmax /
// cross-entropy / argmax with its per-env reductions, relu', and the float64
// epilogue.
//
// Bias by augmentation: an env's flat slab [W_l (d_in x d_out) | b_l
// (d_out)] IS the row-major (d_in + 1) x d_out matrix [W_l; b_l], so every
// layer input carries a ones column (activation rows [h_0 .. h_{d-1} | 1 |
// 0 0 0], row stride ld_aug(d)) and one GEMM with K = d_in + 1 gives
// H W + b; its transpose product H_aug^T dZ gives [dW; db] straight into the
// gradient slab.  The hidden layers' relu is the GEMM's epilogue (hipBLASLt
// HIPBLASLT_EPILOGUE_RELU), so no activation makes an extra HBM pass.
#include "net_engine.h"

#include <hipblaslt/hipblaslt.h>
#include <rocblas/rocblas.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>

#include "common.h"

namespace ce {

namespace {

constexpr int kNetBlock = 256;
constexpr int kNetMaxK = 32;

// Row stride of an augmented activation buffer: d values, the ones column,
// rounded up to 16 bytes
__host__ __device__ constexpr int ld_aug(int d) { return (d + 1 + 3) & ~3; }

template <typename T>
int dev_alloc(T **p, size_t count) {
    *p = nullptr;
    if (count == 0) return CE_OK;
    CE_HIP(hipMalloc(reinterpret_cast<void **>(p), count * sizeof(T)));
    return CE_OK;
}

// W' = W - a over every env's parameters (optimize.py:74-75); the step
// counter advances (baseenvironment.py:30-41: current_step += 1 first).
// 16-byte accesses when both arrays allow them (W always does; an action
// block of a ce_step_many stride may sit at 8 bytes), kNetUpd of them per
// array in flight per thread before any store
constexpr int kNetUpd = 4;
__global__ __launch_bounds__(kNetBlock) void net_update_kernel(float *W, const float *act,
                                                             size_t n, int32_t *step, int E) {
    const size_t i0 = static_cast<size_t>(blockIdx.x) * kNetBlock + threadIdx.x;
    const size_t stride = static_cast<size_t>(gridDim.x) * kNetBlock;
    if (i0 < static_cast<size_t>(E)) step[i0] += 1;
    if (((reinterpret_cast<uintptr_t>(W) | reinterpret_cast<uintptr_t>(act)) & 15) == 0) {
        float4 *w4 = reinterpret_cast<float4 *>(W);
        const float4 *a4 = reinterpret_cast<const float4 *>(act);
        const size_t n4 = n >> 2;
        for (size_t i = i0; i < n4; i += kNetUpd * stride) {
            float4 w[kNetUpd], v[kNetUpd];
#pragma unroll
            for (int q = 0; q < kNetUpd; ++q) {
                const size_t j = i + q * stride;
                const size_t jc = j < n4 ? j : i;                 // in range: i < n4
                w[q] = w4[jc];
                v[q] = a4[jc];
            }
#pragma unroll
            for (int q = 0; q < kNetUpd; ++q) {
                const size_t j = i + q * stride;
                if (j < n4) w4[j] = float4{w[q].x - v[q].x, w[q].y - v[q].y, w[q].z - v[q].z,
                                           w[q].w - v[q].w};
            }
        }
        for (size_t i = 4 * n4 + i0; i < n; i += stride) W[i] -= act[i];
    } else {
        float2 *w2 = reinterpret_cast<float2 *>(W);
        const float2 *a2 = reinterpret_cast<const float2 *>(act);
        const size_t n2 = n >> 1;
        for (size_t i = i0; i < n2; i += stride) {
            float2 w = w2[i];
            const float2 v = a2[i];
            w.x -= v.x;
            w.y -= v.y;
            w2[i] = w;
        }
        for (size_t i = 2 * n2 + i0; i < n; i += stride) W[i] -= act[i];
    }
}

// sequence[0]: rows order[0 .. B) of each env's current order
// (inmemorydataset.py:17-28 over the composed reset permutations)
__global__ __launch_bounds__(kNetBlock) void net_gather_kernel(NetArgs a, float *xb, int32_t *yb) {
    const int e = blockIdx.y;
    const int sel = a.order_sel[e];
    const int32_t *order = a.order + (static_cast<size_t>(sel) * a.E + e) * a.N;
    const size_t n = static_cast<size_t>(a.B) * a.F;
    const int ldx = ld_aug(a.F);                        // the ones column is never rewritten
    float *dst = xb + static_cast<size_t>(e) * a.B * ldx;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kNetBlock + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * kNetBlock) {
        const int r = static_cast<int>(i / a.F), f = static_cast<int>(i - static_cast<size_t>(r) * a.F);
        const int row = order[r];
        dst[static_cast<size_t>(r) * ldx + f] = a.X[static_cast<size_t>(row) * a.F + f];
        if (f == 0) yb[static_cast<size_t>(e) * a.B + r] = a.label[row];
    }
}

// rows x ld buffer: column `col` = 1, the columns after it = 0 (the ones
// column of the bias augmentation, written once: no GEMM writes past d);
// with src, columns < col are copied from the src rows (stride col)
__global__ __launch_bounds__(kNetBlock) void net_aug_kernel(float *buf, size_t rows, int ld, int col,
                                                          const float *src) {
    const size_t n = rows * ld;
    for (size_t i = static_cast<size_t>(blockIdx.x) * kNetBlock + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * kNetBlock) {
        const size_t r = i / ld;
        const int c = static_cast<int>(i - r * ld);
        if (c >= col) buf[i] = c == col ? 1.0f : 0.0f;
        else if (src) buf[i] = src[r * col + c];
    }
}

// relu in place over whole augmented buffers (the ones column stays 1, the
// padding 0): the epilogue of a hidden layer when no hipBLASLt solution fits
__global__ __launch_bounds__(kNetBlock) void net_relu_kernel(float *H, size_t n) {
    for (size_t i = static_cast<size_t>(blockIdx.x) * kNetBlock + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * kNetBlock)
        H[i] = fmaxf(H[i], 0.0f);
}

// One env per workgroup, rows strided over its threads: the logits (their
// bias is in the augmented GEMM), the row-max-stabilised softmax (utils_math.py:51-63), -log(p_y + 1e-16)
// (utils_math.py:25-34), np.argmax's first maximum of P, and (when dz is
// set) dZ = P - Y in place.  Per-env sums: the cross-entropy terms in
// float64 and the hits.  Labels: y + e * y_stride (0: the shared labels).
__global__ __launch_bounds__(kNetBlock) void net_softmax_kernel(float *Z, int R, int K,
                                                              const int32_t *y, int64_t y_stride,
                                                              bool dz, double *loss_out,
                                                              int32_t *hits_out) {
    __shared__ double sl[kNetBlock];
    __shared__ int sh[kNetBlock];
    const int e = blockIdx.x;
    float *z = Z + static_cast<size_t>(e) * R * K;
    const int32_t *ye = y + static_cast<size_t>(e) * y_stride;
    double loss = 0.0;
    int hits = 0;
    for (int r = threadIdx.x; r < R; r += kNetBlock) {
        float *zr = z + static_cast<size_t>(r) * K;
        float v[kNetMaxK];
        float m = -INFINITY;
#pragma unroll
        for (int k = 0; k < kNetMaxK; ++k) {
            v[k] = k < K ? zr[k] : -INFINITY;
            m = fmaxf(m, v[k]);
        }
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < kNetMaxK; ++k) {
            v[k] = k < K ? expf(v[k] - m) : 0.0f;
            s += v[k];
        }
        const int yr = ye[r];
        int arg = 0;
        float best = -1.0f;
#pragma unroll
        for (int k = 0; k < kNetMaxK; ++k) {
            if (k < K) {
                v[k] = v[k] / s;                       // P
                if (v[k] > best) {
                    best = v[k];
                    arg = k;
                }
            }
        }
        float py = 0.0f;
#pragma unroll
        for (int k = 0; k < kNetMaxK; ++k) py = k == yr ? v[k] : py;
        loss += static_cast<double>(-logf(py + 1e-16f));
        hits += arg == yr ? 1 : 0;
        if (dz) {
#pragma unroll
            for (int k = 0; k < kNetMaxK; ++k)
                if (k < K) zr[k] = v[k] - (k == yr ? 1.0f : 0.0f);
        }
    }
    sl[threadIdx.x] = loss;
    sh[threadIdx.x] = hits;
    __syncthreads();
    for (int w = kNetBlock / 2; w > 0; w >>= 1) {
        if (threadIdx.x < w) {
            sl[threadIdx.x] += sl[threadIdx.x + w];
            sh[threadIdx.x] += sh[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        loss_out[e] = sl[0];
        hits_out[e] = sh[0];
    }
}

// dZ = dH * relu'(Z), relu'(Z) = (H > 0) on the post-relu activation
__global__ __launch_bounds__(kNetBlock) void net_relu_back_kernel(float *dH, const float *H, size_t n) {
    for (size_t i = static_cast<size_t>(blockIdx.x) * kNetBlock + threadIdx.x; i < n;
         i += static_cast<size_t>(gridDim.x) * kNetBlock)
        if (!(H[i] > 0.0f)) dH[i] = 0.0f;
}

// Per (env, parameter): g = grad / B (float32, as numpy divides the float32
// gradient), G' = g / (|G| + 1) in float64 (optimize.py:78-83, grad_hist
// float64), obs = [0 (P) | L' (written per env) | G' (P)]; the auto-reset
// (utils_venv.py:31) of an env whose step ends its episode: W <- W0, G <- 0,
// obs <- 0 (the reset observation).  step[e] already holds current_step.
// With P even (every shape whose hidden widths are even), two parameters per
// thread: the env's grad / W / W0 slabs then sit at 8-byte and its G slab at
// 16-byte boundaries (float2 / double2 accesses); the observation rows
// (2P + 1 floats) take scalar stores.
__global__ __launch_bounds__(kNetBlock) void net_epilogue_kernel(NetArgs a, const float *grad) {
    const int e = blockIdx.y;
    const int cur = a.step[e];
    const bool wipe = cur >= a.max_steps && a.auto_reset;
    const size_t P = a.P, base = static_cast<size_t>(e) * P;
    float *obs = a.obs + static_cast<size_t>(e) * (2 * P + 1);
    const float fb = static_cast<float>(a.B);
    const size_t t0 = static_cast<size_t>(blockIdx.x) * kNetBlock + threadIdx.x;
    const size_t stride = static_cast<size_t>(gridDim.x) * kNetBlock;
    if ((P & 1) == 0) {
        // kNetEpi parameter pairs per thread, every load before any store
        constexpr int kNetEpi = 2;
        const float2 *g2 = reinterpret_cast<const float2 *>(grad + base);
        double2 *G2 = reinterpret_cast<double2 *>(a.G + base);
        const size_t P2 = P / 2;
        for (size_t q0 = t0; q0 < P2; q0 += kNetEpi * stride) {
            float2 gv[kNetEpi];
            double2 Gv[kNetEpi];
#pragma unroll
            for (int u = 0; u < kNetEpi; ++u) {
                const size_t q = q0 + u * stride;
                const size_t qc = q < P2 ? q : q0;
                gv[u] = g2[qc];
                Gv[u] = G2[qc];
            }
#pragma unroll
            for (int u = 0; u < kNetEpi; ++u) {
                const size_t q = q0 + u * stride;
                if (q >= P2) break;
                const float ga = gv[u].x / fb, gb = gv[u].y / fb;
                const double na = static_cast<double>(ga) / (fabs(Gv[u].x) + 1.0);
                const double nb = static_cast<double>(gb) / (fabs(Gv[u].y) + 1.0);
                const size_t p = 2 * q;
                obs[p] = 0.0f;                            // wght_hist is identically 0
                obs[p + 1] = 0.0f;
                obs[P + 1 + p] = wipe ? 0.0f : static_cast<float>(na);
                obs[P + 2 + p] = wipe ? 0.0f : static_cast<float>(nb);
                G2[q] = wipe ? double2{0.0, 0.0} : double2{na, nb};
                if (wipe)
                    reinterpret_cast<float2 *>(a.W + base)[q] =
                        reinterpret_cast<const float2 *>(a.W0 + base)[q];
            }
        }
        return;
    }
    for (size_t p = t0; p < P; p += stride) {
        const float g = grad[base + p] / fb;
        const double gn = static_cast<double>(g) / (fabs(a.G[base + p]) + 1.0);
        obs[p] = 0.0f;
        obs[P + 1 + p] = wipe ? 0.0f : static_cast<float>(gn);
        a.G[base + p] = wipe ? 0.0 : gn;
        if (wipe) a.W[base + p] = a.W0[base + p];
    }
}

// Per env: L' = (loss - L)/(L + 0.1) (optimize.py:80-81), reward = -loss,
// done = current_step >= max_steps (:102-103), info, episode length; the
// auto-reset's L, step and order <- order[perm] (optimize.py:58-67).
__global__ __launch_bounds__(kNetBlock) void net_finish_kernel(NetArgs a, const double *mb_loss,
                                                             const int32_t *mb_hits,
                                                             const double *inf_loss,
                                                             const int32_t *inf_hits) {
    const int e = blockIdx.x;
    const int cur = a.step[e];
    const bool done = cur >= a.max_steps;
    const bool wipe = done && a.auto_reset;
    __syncthreads();                                      // every thread has read step[e]
    if (threadIdx.x == 0) {
        // the loss is a float32 mean in the reference (TF / numpy float32)
        const float loss = static_cast<float>(mb_loss[e] / a.B);
        const float acc = static_cast<float>(static_cast<double>(mb_hits[e]) / a.B);
        const bool full = a.B == a.N;
        const float obj = full ? loss : static_cast<float>(inf_loss[e] / a.N);
        const float oacc = full ? acc : static_cast<float>(static_cast<double>(inf_hits[e]) / a.N);
        const double lprev = a.L[e];
        const double lnew = (static_cast<double>(loss) - lprev) / (lprev + 0.1);
        const size_t P = a.P;
        a.obs[static_cast<size_t>(e) * (2 * P + 1) + P] = wipe ? 0.0f : static_cast<float>(lnew);
        a.reward[e] = -loss;
        a.done[e] = done ? 1 : 0;
        a.objective[e] = obj;
        a.accuracy[e] = oacc;
        a.episode_len[e] = cur;
        a.L[e] = wipe ? 0.0 : lnew;
        a.step[e] = wipe ? 0 : cur;
    }
    if (wipe && a.order != nullptr) {
        const int sel = a.order_sel[e];
        const int32_t *cur_o = a.order + (static_cast<size_t>(sel) * a.E + e) * a.N;
        int32_t *nxt = a.order + (static_cast<size_t>(1 - sel) * a.E + e) * a.N;
        const int32_t *pm = a.perm + static_cast<size_t>(e) * a.N;
        for (int i = threadIdx.x; i < a.N; i += kNetBlock) nxt[i] = cur_o[pm[i]];
        __syncthreads();
        if (threadIdx.x == 0) a.order_sel[e] = 1 - sel;
    }
}

// Reset (optimize.py:58-67): W <- W0, G <- 0, obs <- 0, then per env L,
// step and order <- order[perm]
__global__ __launch_bounds__(kNetBlock) void net_reset_params_kernel(NetArgs a) {
    const int e = blockIdx.y;
    const size_t P = a.P, base = static_cast<size_t>(e) * P;
    float *obs = a.obs + static_cast<size_t>(e) * (2 * P + 1);
    for (size_t p = static_cast<size_t>(blockIdx.x) * kNetBlock + threadIdx.x; p < 2 * P + 1;
         p += static_cast<size_t>(gridDim.x) * kNetBlock) {
        obs[p] = 0.0f;
        if (p < P) {
            a.W[base + p] = a.W0[base + p];
            a.G[base + p] = 0.0;
        }
    }
}

__global__ __launch_bounds__(kNetBlock) void net_reset_env_kernel(NetArgs a) {
    const int e = blockIdx.x;
    if (threadIdx.x == 0) {
        a.L[e] = 0.0;
        a.step[e] = 0;
    }
    if (a.order != nullptr) {
        const int sel = a.order_sel[e];
        const int32_t *cur_o = a.order + (static_cast<size_t>(sel) * a.E + e) * a.N;
        int32_t *nxt = a.order + (static_cast<size_t>(1 - sel) * a.E + e) * a.N;
        const int32_t *pm = a.perm + static_cast<size_t>(e) * a.N;
        for (int i = threadIdx.x; i < a.N; i += kNetBlock) nxt[i] = cur_o[pm[i]];
        __syncthreads();
        if (threadIdx.x == 0) a.order_sel[e] = 1 - sel;
    }
}

unsigned blocks_for(size_t n, unsigned cap) {
    const size_t b = (n + kNetBlock - 1) / kNetBlock;
    return static_cast<unsigned>(std::max<size_t>(1, std::min<size_t>(b, cap)));
}

}  // namespace

// One forward GEMM of a hidden layer with its relu as the hipBLASLt
// epilogue, descriptors and algorithm fixed at net_create
struct LtGemm {
    hipblasLtMatmulDesc_t op = nullptr;
    hipblasLtMatrixLayout_t la = nullptr, lb = nullptr, ld = nullptr;
    hipblasLtMatmulAlgo_t algo{};
    size_t ws = 0;
    bool ok = false;
};

struct NetPlan {
    rocblas_handle blas = nullptr;
    hipblasLtHandle_t lt = nullptr;
    void *workspace = nullptr, *lt_workspace = nullptr;
    int nl = 0;                             // dense layers (hidden + output)
    int dims[kNetMaxHidden + 2] = {0};      // F, hidden..., K
    int64_t offW[kNetMaxHidden + 1] = {0}, offb[kNetMaxHidden + 1] = {0};
    int dmax = 0;
    float *xaug = nullptr;                  // [N][ld_aug(F)] the dataset rows with the ones column
    float *xb = nullptr;                    // [E][B][ld_aug(F)] gathered minibatch rows (B < N)
    int32_t *yb = nullptr;                  // [E][B]
    float *mb_act[kNetMaxHidden] = {nullptr};   // [E][B][ld_aug(d_l)] hidden activations (post-relu)
    float *mb_out = nullptr;                // [E][B][K] logits, then dZ
    float *dbuf[2] = {nullptr, nullptr};    // [E][B][ld_aug(dmax)] dH / dZ ping-pong
    float *grad = nullptr;                  // [E][P] summed gradient (float32)
    float *inf[kNetMaxHidden] = {nullptr};  // [E][N][ld_aug(d_l)] info activations (B < N)
    float *inf_out = nullptr;               // [E][N][K]
    double *mb_loss = nullptr, *inf_loss = nullptr;
    int32_t *mb_hits = nullptr, *inf_hits = nullptr;
    LtGemm fw_mb[kNetMaxHidden], fw_inf[kNetMaxHidden];   // hidden-layer forwards (relu epilogue)
};

int64_t net_params(int F, int K, int n_hidden, const int *hidden) {
    int64_t P = 0;
    int prev = F;
    for (int l = 0; l <= n_hidden; ++l) {
        const int d = l < n_hidden ? hidden[l] : K;
        P += static_cast<int64_t>(prev) * d + d;
        prev = d;
    }
    return P;
}

namespace {

constexpr size_t kLtWorkspace = 32u << 20;

// Row-major C[M][N] (row stride ldc) = op(A) op(B), op(A) M x K, op(B) K x N,
// batched over envs with element strides (0: shared operand).  rocBLAS is
// column-major: a row-major matrix is its column-major transpose, so the
// call computes C^T = op(B)^T op(A)^T with the operands swapped.
int gemm_rm(rocblas_handle h, bool tA, bool tB, int M, int N, int K, const float *A, int lda,
            int64_t sA, const float *B, int ldb, int64_t sB, float *C, int ldc, int64_t sC,
            int batch) {
    const float one = 1.0f, zero = 0.0f;
    const rocblas_status st = rocblas_sgemm_strided_batched(
        h, tB ? rocblas_operation_transpose : rocblas_operation_none,
        tA ? rocblas_operation_transpose : rocblas_operation_none, N, M, K, &one, B, ldb, sB, A,
        lda, sA, &zero, C, ldc, sC, batch);
    if (st != rocblas_status_success)
        return fail(CE_EHIP, std::string("rocblas_sgemm_strided_batched failed: ") +
                                 rocblas_status_to_string(st));
    return CE_OK;
}

void lt_free(LtGemm &g) {
    if (g.op) hipblasLtMatmulDescDestroy(g.op);
    for (hipblasLtMatrixLayout_t l : {g.la, g.lb, g.ld})
        if (l) hipblasLtMatrixLayoutDestroy(l);
    g = LtGemm{};
}

hipblasLtMatrixLayout_t lt_layout(uint64_t rows, uint64_t cols, int64_t ld, int batch, int64_t stride) {
    hipblasLtMatrixLayout_t l = nullptr;
    if (hipblasLtMatrixLayoutCreate(&l, HIP_R_32F, rows, cols, ld) != HIPBLAS_STATUS_SUCCESS) return nullptr;
    const int32_t b = batch;
    if (hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_BATCH_COUNT, &b, sizeof(b)) !=
            HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatrixLayoutSetAttribute(l, HIPBLASLT_MATRIX_LAYOUT_STRIDED_BATCH_OFFSET, &stride,
                                          sizeof(stride)) != HIPBLAS_STATUS_SUCCESS) {
        hipblasLtMatrixLayoutDestroy(l);
        return nullptr;
    }
    return l;
}

// Row-major relu(A[M][K] B[K][N]) batched: the column-major D^T (N x M) =
// B^T (N x K) A^T (K x M), so hipBLASLt's "A" is the weight slab and its "B"
// the activations.  g.ok stays false when the library offers no solution.
void lt_setup(hipblasLtHandle_t h, LtGemm &g, int M, int N, int K, int lda, int64_t sA, int ldb,
              int64_t sB, int ldc, int64_t sC, int batch) {
    lt_free(g);
    if (hipblasLtMatmulDescCreate(&g.op, HIPBLAS_COMPUTE_32F, HIP_R_32F) != HIPBLAS_STATUS_SUCCESS) return;
    const hipblasOperation_t nt = HIPBLAS_OP_N;
    const hipblasLtEpilogue_t ep = HIPBLASLT_EPILOGUE_RELU;
    if (hipblasLtMatmulDescSetAttribute(g.op, HIPBLASLT_MATMUL_DESC_TRANSA, &nt, sizeof(nt)) !=
            HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatmulDescSetAttribute(g.op, HIPBLASLT_MATMUL_DESC_TRANSB, &nt, sizeof(nt)) !=
            HIPBLAS_STATUS_SUCCESS ||
        hipblasLtMatmulDescSetAttribute(g.op, HIPBLASLT_MATMUL_DESC_EPILOGUE, &ep, sizeof(ep)) !=
            HIPBLAS_STATUS_SUCCESS)
        return;
    g.la = lt_layout(N, K, ldb, batch, sB);
    g.lb = lt_layout(K, M, lda, batch, sA);
    g.ld = lt_layout(N, M, ldc, batch, sC);
    if (!g.la || !g.lb || !g.ld) return;
    hipblasLtMatmulPreference_t pref = nullptr;
    if (hipblasLtMatmulPreferenceCreate(&pref) != HIPBLAS_STATUS_SUCCESS) return;
    const uint64_t wmax = kLtWorkspace;
    hipblasLtMatmulPreferenceSetAttribute(pref, HIPBLASLT_MATMUL_PREF_MAX_WORKSPACE_BYTES, &wmax,
                                          sizeof(wmax));
    hipblasLtMatmulHeuristicResult_t res[1];
    int n = 0;
    const hipblasStatus_t st = hipblasLtMatmulAlgoGetHeuristic(h, g.op, g.la, g.lb, g.ld, g.ld, pref,
                                                               1, res, &n);
    hipblasLtMatmulPreferenceDestroy(pref);
    if (st != HIPBLAS_STATUS_SUCCESS || n < 1 || res[0].state != HIPBLAS_STATUS_SUCCESS) return;
    g.algo = res[0].algo;
    g.ws = res[0].workspaceSize;
    g.ok = g.ws <= kLtWorkspace;
}

int lt_run(hipblasLtHandle_t h, const LtGemm &g, const float *A, const float *B, float *C,
           void *ws, hipStream_t s) {
    const float one = 1.0f, zero = 0.0f;
    const hipblasStatus_t st = hipblasLtMatmul(h, g.op, &one, B, g.la, A, g.lb, &zero, C, g.ld, C,
                                               g.ld, &g.algo, ws, kLtWorkspace, s);
    if (st != HIPBLAS_STATUS_SUCCESS) return fail(CE_EHIP, "network: hipblasLtMatmul failed");
    return CE_OK;
}

void fill_aug(float *buf, size_t rows, int d, const float *src = nullptr) {
    const size_t n = rows * ld_aug(d);
    hipLaunchKernelGGL(net_aug_kernel, dim3(blocks_for(n, 8192)), dim3(kNetBlock), 0, nullptr, buf, rows,
                       ld_aug(d), d, src);
}

}  // namespace

int net_create(NetPlan **out, const NetArgs &a, int device) {
    *out = nullptr;
    if (a.n_hidden < 1 || a.n_hidden > kNetMaxHidden)
        return fail(CE_EUNSUPPORTED, "network: 1 to 4 hidden layers");
    if (a.K > kNetMaxK) return fail(CE_EUNSUPPORTED, "network: at most 32 classes");
    if (a.E > 65535) return fail(CE_EUNSUPPORTED, "network: at most 65535 envs per engine");
    NetPlan *p = new (std::nothrow) NetPlan();
    if (!p) return fail(CE_ENOMEM, "network: host allocation failed");
    auto bail = [&](int rc) {
        net_destroy(p);
        return rc;
    };
    p->nl = a.n_hidden + 1;
    p->dims[0] = a.F;
    for (int l = 0; l < a.n_hidden; ++l) {
        if (a.hidden[l] <= 0) return bail(fail(CE_EINVAL, "network: hidden widths must be positive"));
        p->dims[l + 1] = a.hidden[l];
    }
    p->dims[p->nl] = a.K;
    int64_t off = 0;
    for (int l = 0; l < p->nl; ++l) {
        p->offW[l] = off;
        off += static_cast<int64_t>(p->dims[l]) * p->dims[l + 1];
        p->offb[l] = off;
        off += p->dims[l + 1];
        if (l < a.n_hidden) p->dmax = std::max(p->dmax, p->dims[l + 1]);
    }
    if (off != a.P) return bail(fail(CE_EINVAL, "network: parameter count mismatch"));
    const size_t E = a.E, B = a.B, N = a.N;
    int rc;
    if (hipSetDevice(device) != hipSuccess) return bail(fail(CE_EHIP, "network: hipSetDevice"));
    if ((rc = dev_alloc(&p->xaug, N * ld_aug(a.F))) != CE_OK) return bail(rc);
    fill_aug(p->xaug, N, a.F, a.X);
    if (B < N) {
        if ((rc = dev_alloc(&p->xb, E * B * ld_aug(a.F))) != CE_OK) return bail(rc);
        fill_aug(p->xb, E * B, a.F);
        if ((rc = dev_alloc(&p->yb, E * B)) != CE_OK) return bail(rc);
        for (int l = 0; l < a.n_hidden; ++l) {
            if ((rc = dev_alloc(&p->inf[l], E * N * ld_aug(p->dims[l + 1]))) != CE_OK) return bail(rc);
            fill_aug(p->inf[l], E * N, p->dims[l + 1]);
        }
        if ((rc = dev_alloc(&p->inf_out, E * N * a.K)) != CE_OK) return bail(rc);
        if ((rc = dev_alloc(&p->inf_loss, E)) != CE_OK) return bail(rc);
        if ((rc = dev_alloc(&p->inf_hits, E)) != CE_OK) return bail(rc);
    }
    for (int l = 0; l < a.n_hidden; ++l) {
        if ((rc = dev_alloc(&p->mb_act[l], E * B * ld_aug(p->dims[l + 1]))) != CE_OK) return bail(rc);
        fill_aug(p->mb_act[l], E * B, p->dims[l + 1]);
    }
    if ((rc = dev_alloc(&p->mb_out, E * B * a.K)) != CE_OK) return bail(rc);
    if ((rc = dev_alloc(&p->dbuf[0], E * B * ld_aug(p->dmax))) != CE_OK) return bail(rc);
    if ((rc = dev_alloc(&p->dbuf[1], E * B * ld_aug(p->dmax))) != CE_OK) return bail(rc);
    if ((rc = dev_alloc(&p->grad, E * static_cast<size_t>(a.P))) != CE_OK) return bail(rc);
    if ((rc = dev_alloc(&p->mb_loss, E)) != CE_OK) return bail(rc);
    if ((rc = dev_alloc(&p->mb_hits, E)) != CE_OK) return bail(rc);
    CE_HIP(hipGetLastError());
    CE_HIP(hipDeviceSynchronize());
    if (rocblas_create_handle(&p->blas) != rocblas_status_success)
        return bail(fail(CE_EHIP, "network: rocblas_create_handle failed"));
    // a fixed workspace, so no call allocates (hipGraph capture, ce_step_many)
    constexpr size_t kWorkspace = 64u << 20;
    if (hipMalloc(&p->workspace, kWorkspace) != hipSuccess)
        return bail(fail(CE_ENOMEM, "network: workspace allocation failed"));
    if (rocblas_set_workspace(p->blas, p->workspace, kWorkspace) != rocblas_status_success)
        return bail(fail(CE_EHIP, "network: rocblas_set_workspace failed"));
    // hidden-layer forwards with the relu epilogue (CE_NET_LT=0: rocBLAS and
    // a relu pass instead, the A/B arm; also what a shape without a hipBLASLt
    // solution runs)
    const char *lt_env = std::getenv("CE_NET_LT");
    if (!(lt_env && lt_env[0] == '0')) {
        if (hipblasLtCreate(&p->lt) != HIPBLAS_STATUS_SUCCESS)
            return bail(fail(CE_EHIP, "network: hipblasLtCreate failed"));
        if (hipMalloc(&p->lt_workspace, kLtWorkspace) != hipSuccess)
            return bail(fail(CE_ENOMEM, "network: hipBLASLt workspace allocation failed"));
        for (int l = 0; l < a.n_hidden; ++l) {
            const int din = p->dims[l], dout = p->dims[l + 1];
            const int ldi = ld_aug(din), ldo = ld_aug(dout);
            const int64_t sin = l == 0 ? (B < N ? static_cast<int64_t>(B) * ldi : 0)
                                       : static_cast<int64_t>(B) * ldi;
            lt_setup(p->lt, p->fw_mb[l], static_cast<int>(B), dout, din + 1, ldi, sin, dout, a.P, ldo,
                     static_cast<int64_t>(B) * ldo, static_cast<int>(E));
            if (B < N)
                lt_setup(p->lt, p->fw_inf[l], static_cast<int>(N), dout, din + 1, ldi,
                         l == 0 ? 0 : static_cast<int64_t>(N) * ldi, dout, a.P, ldo,
                         static_cast<int64_t>(N) * ldo, static_cast<int>(E));
        }
    }
    *out = p;
    return CE_OK;
}

bool net_forward_lt(const NetPlan *p) {
    for (int l = 0; l + 1 < p->nl; ++l)
        if (!p->fw_mb[l].ok || (p->xb && !p->fw_inf[l].ok)) return false;
    return true;
}

void net_destroy(NetPlan *p) {
    if (!p) return;
    if (p->blas) rocblas_destroy_handle(p->blas);
    for (int l = 0; l < kNetMaxHidden; ++l) {
        lt_free(p->fw_mb[l]);
        lt_free(p->fw_inf[l]);
    }
    if (p->lt) hipblasLtDestroy(p->lt);
    void *bufs[] = {p->workspace, p->lt_workspace, p->xaug, p->xb, p->yb, p->mb_out, p->dbuf[0],
                    p->dbuf[1], p->grad, p->inf_out, p->mb_loss, p->inf_loss, p->mb_hits,
                    p->inf_hits};
    for (void *b : bufs)
        if (b) (void)hipFree(b);
    for (float *b : p->mb_act)
        if (b) (void)hipFree(b);
    for (float *b : p->inf)
        if (b) (void)hipFree(b);
    delete p;
}

namespace {

// one hidden layer's forward: relu(H_aug W_aug) into the augmented output
int hidden_forward(NetPlan *p, const LtGemm &g, int rows, int din, int dout, const float *h, int64_t sh,
                   const float *W, int64_t P, float *o, int E, hipStream_t s) {
    const int ldi = ld_aug(din), ldo = ld_aug(dout);
    if (g.ok) return lt_run(p->lt, g, h, W, o, p->lt_workspace, s);
    int rc;
    if ((rc = gemm_rm(p->blas, false, false, rows, dout, din + 1, h, ldi, sh, W, dout, P, o, ldo,
                      static_cast<int64_t>(rows) * ldo, E)) != CE_OK)
        return rc;
    const size_t n = static_cast<size_t>(E) * rows * ldo;
    hipLaunchKernelGGL(net_relu_kernel, dim3(blocks_for(n, 8192)), dim3(kNetBlock), 0, s, o, n);
    return CE_OK;
}

}  // namespace

int net_step(NetPlan *p, const NetArgs &a, hipStream_t s) {
    const int E = a.E, B = a.B, N = a.N, K = a.K, nl = p->nl;
    const int64_t P = a.P;
    const bool full = B == N;
    if (rocblas_set_stream(p->blas, s) != rocblas_status_success)
        return fail(CE_EHIP, "network: rocblas_set_stream failed");
    const size_t EP = static_cast<size_t>(E) * P;
    hipLaunchKernelGGL(net_update_kernel, dim3(blocks_for(EP, 8192)), dim3(kNetBlock), 0, s, a.W,
                       a.act, EP, a.step, E);
    // the minibatch: gathered rows (B < N) or the shared dataset (B == N),
    // both with the ones column
    const int ldx = ld_aug(a.F);
    const float *x = full ? p->xaug : p->xb;
    const int64_t sx = full ? 0 : static_cast<int64_t>(B) * ldx;
    const int32_t *y = full ? a.label : p->yb;
    const int64_t sy = full ? 0 : B;
    if (!full)
        hipLaunchKernelGGL(net_gather_kernel, dim3(blocks_for(static_cast<size_t>(B) * a.F, 64), E),
                           dim3(kNetBlock), 0, s, a, p->xb, p->yb);
    int rc;
    // forward on the minibatch
    const float *h = x;
    int64_t sh = sx;
    for (int l = 0; l < nl; ++l) {
        const int din = p->dims[l], dout = p->dims[l + 1];
        if (l + 1 < nl) {
            if ((rc = hidden_forward(p, p->fw_mb[l], B, din, dout, h, sh, a.W + p->offW[l], P,
                                     p->mb_act[l], E, s)) != CE_OK)
                return rc;
            h = p->mb_act[l];
            sh = static_cast<int64_t>(B) * ld_aug(dout);
        } else if ((rc = gemm_rm(p->blas, false, false, B, dout, din + 1, h, ld_aug(din), sh,
                                 a.W + p->offW[l], dout, P, p->mb_out, dout,
                                 static_cast<int64_t>(B) * dout, E)) != CE_OK) {
            return rc;
        }
    }
    hipLaunchKernelGGL(net_softmax_kernel, dim3(E), dim3(kNetBlock), 0, s, p->mb_out, B, K, y, sy, true,
                       p->mb_loss, p->mb_hits);
    // backward: [dW_l; db_l] = H_{l-1,aug}^T dZ_l, dH_{l-1} = dZ_l W_l^T, relu'
    const float *dz = p->mb_out;
    int lddz = K;
    for (int l = nl - 1; l >= 0; --l) {
        const int din = p->dims[l], dout = p->dims[l + 1];
        const float *hin = l == 0 ? x : p->mb_act[l - 1];
        const int ldi = ld_aug(din);
        const int64_t shin = l == 0 ? sx : static_cast<int64_t>(B) * ldi;
        const int64_t sdz = static_cast<int64_t>(B) * lddz;
        if ((rc = gemm_rm(p->blas, true, false, din + 1, dout, B, hin, ldi, shin, dz, lddz, sdz,
                          p->grad + p->offW[l], dout, P, E)) != CE_OK)
            return rc;
        if (l == 0) break;
        float *dh = p->dbuf[l & 1];
        if ((rc = gemm_rm(p->blas, false, true, B, din, dout, dz, lddz, sdz, a.W + p->offW[l], dout,
                          P, dh, ldi, static_cast<int64_t>(B) * ldi, E)) != CE_OK)
            return rc;
        const size_t n = static_cast<size_t>(E) * B * ldi;
        hipLaunchKernelGGL(net_relu_back_kernel, dim3(blocks_for(n, 8192)), dim3(kNetBlock), 0, s,
                           dh, p->mb_act[l - 1], n);
        dz = dh;
        lddz = ldi;
    }
    // info['objective'] / ['accuracy'] on every row (B < N)
    if (!full) {
        const float *hi = p->xaug;
        int64_t shi = 0;
        for (int l = 0; l < nl; ++l) {
            const int din = p->dims[l], dout = p->dims[l + 1];
            if (l + 1 < nl) {
                if ((rc = hidden_forward(p, p->fw_inf[l], N, din, dout, hi, shi, a.W + p->offW[l], P,
                                         p->inf[l], E, s)) != CE_OK)
                    return rc;
                hi = p->inf[l];
                shi = static_cast<int64_t>(N) * ld_aug(dout);
            } else if ((rc = gemm_rm(p->blas, false, false, N, dout, din + 1, hi, ld_aug(din), shi,
                                     a.W + p->offW[l], dout, P, p->inf_out, dout,
                                     static_cast<int64_t>(N) * dout, E)) != CE_OK) {
                return rc;
            }
        }
        hipLaunchKernelGGL(net_softmax_kernel, dim3(E), dim3(kNetBlock), 0, s, p->inf_out, N, K, a.label,
                           int64_t(0), false, p->inf_loss, p->inf_hits);
    }
    hipLaunchKernelGGL(net_epilogue_kernel, dim3(blocks_for(static_cast<size_t>(P + 1) / 2, 1024), E),
                       dim3(kNetBlock), 0, s, a, p->grad);
    hipLaunchKernelGGL(net_finish_kernel, dim3(E), dim3(kNetBlock), 0, s, a, p->mb_loss, p->mb_hits,
                       p->inf_loss, p->inf_hits);
    CE_HIP(hipGetLastError());
    return CE_OK;
}

int net_reset(NetPlan *p, const NetArgs &a, hipStream_t s) {
    (void)p;
    hipLaunchKernelGGL(net_reset_params_kernel,
                       dim3(blocks_for(2 * static_cast<size_t>(a.P) + 1, 1024), a.E), dim3(kNetBlock),
                       0, s, a);
    hipLaunchKernelGGL(net_reset_env_kernel, dim3(a.E), dim3(kNetBlock), 0, s, a);
    CE_HIP(hipGetLastError());
    return CE_OK;
}

}  // namespace ce
