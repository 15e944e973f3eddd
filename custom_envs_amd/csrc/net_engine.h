// Optimize-v0 over a general OptimizeNN network (SURVEY 8f rank 3 as the
// Optimize-v0 problem): F -> hidden[0] -> ... -> hidden[L-1] (relu) -> K
// softmax, float32, any batch size 1..N (custom_envs/problems/optimize_nn.py:
// 22-64, create_neural_net utils_tf.py:74-86; default layers (256, 256)).
// The fused config-3 kernel (mlp_kernels.h) keeps the one shape it is
// written for (hidden 64, B = 32); every other network runs here.
//
// One VecEnv.step of E envs is a fixed sequence of launches on one stream:
//   net_update_kernel   W' = W - a (optimize.py:74-75), step += 1, and the
//                       minibatch rows of each env gathered through its
//                       row order (sequence[0], B < N)
//   forward             per layer one strided-batched f32 GEMM over the E envs,
//                       H_l = relu([H_{l-1} | 1] [W_l; b_l]): the bias by the
//                       ones column of the augmented input, the relu as the
//                       hipBLASLt epilogue (rocBLAS + a relu pass where no
//                       hipBLASLt solution fits, or CE_NET_LT=0) -- the dense
//                       products are plain library GEMMs; the per-env
//                       parameter slabs are the GEMM batch
//   net_softmax_kernel  softmax, -log(p_y + 1e-16), argmax hit per row, the
//                       per-env loss / hit sums, dZ = P - Y (utils_math.py:
//                       25-34,51-63)
//   backward            [dW_l; db_l] = [H_{l-1} | 1]^T dZ_l straight into the
//                       env's gradient slab (one GEMM), dH_{l-1} = dZ_l W_l^T,
//                       relu' (net_relu_back_kernel)
//   info (B < N)        the full-data forward for info['objective'] /
//                       ['accuracy'] (optimize.py:94-97); B == N reuses the
//                       minibatch numbers, as the reference computes the same
//                       values twice
//   net_epilogue_kernel G' = (g / B) / (|G| + 1) in float64, the observation
//                       [0 | L' | G'], the auto-reset's W <- W0, G <- 0
//   net_finish_kernel   per env: L', reward, done, info, episode length, and
//                       the auto-reset's order <- order[perm], L, step
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace ce {

constexpr int kNetMaxHidden = 4;

struct NetArgs {
    int E, N, F, K, B, P, max_steps, auto_reset;
    int n_hidden;                  // hidden layers L
    int hidden[kNetMaxHidden];
    const float *X;                // [N][F] dataset rows
    const int32_t *label;          // [N]
    float *W;                      // [E][P] flat [W1 | b1 | W2 | b2 | ...]
    const float *W0;               // [E][P]
    double *G;                     // [E][P] grad_hist[idx] (float64)
    double *L;                     // [E]
    int32_t *step;                 // [E]
    const int32_t *perm;           // [E][N] reset permutation (B < N)
    int32_t *order;                // [2][E][N] row order ping-pong (B < N)
    int32_t *order_sel;            // [E]
    const float *act;              // [E][P]
    float *obs;                    // [E][2P + 1]
    float *reward;
    uint8_t *done;
    float *objective;
    float *accuracy;
    int32_t *episode_len;
};

struct NetPlan;

// Work buffers, the rocBLAS / hipBLASLt handles and the forward GEMMs'
// hipBLASLt algorithms for E envs of this shape.
int net_create(NetPlan **out, const NetArgs &shape, int device);
void net_destroy(NetPlan *plan);
// Stream-ordered launches of one step / one reset (no host synchronisation:
// capturable into a hipGraph).
int net_step(NetPlan *plan, const NetArgs &a, hipStream_t stream);
int net_reset(NetPlan *plan, const NetArgs &a, hipStream_t stream);
// True when every hidden-layer forward has a hipBLASLt relu-epilogue algorithm.
bool net_forward_lt(const NetPlan *plan);
// Flat parameter count of the network.
int64_t net_params(int F, int K, int n_hidden, const int *hidden);

}  // namespace ce
