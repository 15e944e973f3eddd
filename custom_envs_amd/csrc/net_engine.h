// Optimize-v0 over a general OptimizeNN network (SURVEY 8f rank 3 as the
// Optimize-v0 problem): F -> hidden[0] -> ... -> hidden[L-1] (relu) -> K
// softmax, float32, any batch size 1..N (custom_envs/problems/optimize_nn.py:
// 22-64, create_neural_net utils_tf.py:74-86; default layers (256, 256)).
// The fused config-3 kernel (mlp_kernels.h) keeps the one shape it is
// written for (hidden 64, B = 32); every other network runs here, on the
// hand-written MFMA kernels of net_kernels.h (the launch sequence is listed
// there) when every hidden layer is at most 256 wide; a network with a wider
// hidden layer runs on the wide-layer kernels of net_wide.h (a natural weight
// image, plain tiled float32 kernels).  Limits: 1-4 hidden layers, K <= 32
// classes.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

namespace ce {

constexpr int kNetMaxHidden = 4;
constexpr int kNetL = kNetMaxHidden + 1;  // dense layers: hidden + the output layer
constexpr int kNetMaxOp = 256;            // widest padded layer (hidden widths <= 256)
constexpr int kNetMaxClasses = 32;
// weight rows per LDS slot of the forward (CE_NET_CHUNK: 32, or 16 for
// three workgroups per CU; the image's row order is defined on 32-row groups
// either way, net_img_row)
#ifndef CE_NET_CHUNK
#define CE_NET_CHUNK 32
#endif
constexpr int kNetChunk = CE_NET_CHUNK;
static_assert(kNetChunk == 16 || kNetChunk == 32, "CE_NET_CHUNK: 16 or 32");

// Shape of the network and of its per-env weight IMAGE (net_kernels.h).
struct NetGeom {
    int wide;                        // a hidden layer > kNetMaxOp: the natural image, net_wide.h
    int nl;                          // dense layers (hidden + output)
    int din[kNetL], dout[kNetL];     // true widths
    int op[kNetL];                   // d_out padded to a multiple of 64
    int nchunk[kNetL];               // 32-row image chunks of layer l
    int chunk0[kNetL + 1];           // first global chunk of layer l; chunk0[nl] = all
    int row0[kNetL + 1];             // first image row of layer l (update kernel)
    int bias_rel[kNetL];             // layer l's bias in the bias area (floats)
    int bias_total;                  // floats of the bias area (multiple of 64)
    int64_t img_off[kNetL];          // layer l's rows, floats from the env image start
    int64_t bias_base;               // the bias area, floats from the env image start
    int64_t flat_w[kNetL];           // layer l's kernel in the flat vector (bias at + din*dout)
    int64_t Pimg;                    // floats per env image (multiple of 64)
    int64_t P;                       // flat parameters
};

// The natural image of the wide path: layer l's rows are its input units in
// order (op_l columns), its biases in unit order.
constexpr int kNetMaxWide = 8192;         // widest hidden layer of the wide path
// Image row of input unit u of layer l.  Layer 0: the feature index.  A
// hidden layer's input unit u = 64c + 16g + 4i + j is register i of block
// (c, j) in lane group g of the previous layer's 16x16 accumulators; chunk
// 2c + (j >> 1) holds the 32 units of blocks (c, j & 2), (c, (j & 2) + 1) at
// rho = 16 (j & 1) + 4i + g.
__host__ __device__ inline int net_img_row(int l, int u) {
    if (l == 0) return u;
    const int c = u >> 6, w = u & 63, j = w & 3, i = (w >> 2) & 3, g = w >> 4;
    return (2 * c + (j >> 1)) * 32 + 16 * (j & 1) + 4 * i + g;
}
// inverse of net_img_row
__host__ __device__ inline int net_row_unit(int l, int q) {
    if (l == 0) return q;
    const int chunk = q >> 5, rho = q & 31, c = chunk >> 1, jj = chunk & 1;
    const int j = 2 * jj + (rho >> 4), i = (rho >> 2) & 3, g = rho & 3;
    return 64 * c + 16 * g + 4 * i + j;
}
// position of output unit u's bias in its layer's permuted bias block:
// block (c, j), lane group g, register i -- one float4 per lane and block
__host__ __device__ inline int net_bias_slot(int u) {
    const int c = u >> 6, w = u & 63, j = w & 3, i = (w >> 2) & 3, g = w >> 4;
    return ((c * 4 + j) * 4 + g) * 4 + i;
}
__host__ __device__ inline int net_bias_unit(int s) {
    const int i = s & 3, g = (s >> 2) & 3, j = (s >> 4) & 3, c = s >> 6;
    return 64 * c + 16 * g + 4 * i + j;
}

// dims = F, hidden..., K (n_hidden + 2 entries).  CE_OK or CE_EUNSUPPORTED
// with the reason in ce_last_error().
int net_geometry(int n_hidden, const int *dims, NetGeom *g);
// one env's flat [W1 | b1 | ...] vector <-> its image (padding zero)
void net_flat_to_image(const NetGeom &g, const float *flat, float *img);
void net_image_to_flat(const NetGeom &g, const float *img, float *flat);

struct NetArgs {
    int E, N, F, K, B, P, max_steps, auto_reset;
    int n_hidden;                  // hidden layers L
    int hidden[kNetMaxHidden];
    const float *X;                // [N][F] dataset rows
    const int32_t *label;          // [N]
    float *W;                      // [E][Pimg] weight images
    const float *W0;               // [E][Pimg]
    double *G;                     // [E][P] grad_hist[idx] (float64), flat order
    double *L;                     // [E]
    int32_t *step;                 // [E]
    const int32_t *perm;           // [E][N] reset permutation (B < N)
    int32_t *order;                // [2][E][N] row order ping-pong (B < N)
    int32_t *order_sel;            // [E]
    const float *act;              // [E][P] flat
    float *obs;                    // [E][2P + 1]
    float *reward;
    uint8_t *done;
    float *objective;
    float *accuracy;
    int32_t *episode_len;
};

struct NetPlan;

// Work buffers for E envs of this shape (the dataset in MFMA operand order,
// the gathered minibatch rows, their activations and dZ) and the side stream
// the gradient chain runs on.
int net_create(NetPlan **out, const NetArgs &shape, int device);
void net_destroy(NetPlan *plan);
const NetGeom &net_geom(const NetPlan *plan);
// Stream-ordered launches of one step / one reset (no host synchronisation:
// capturable into a hipGraph -- the step forks onto the plan's side stream
// and joins back with events, the capture pattern).
int net_step(NetPlan *plan, const NetArgs &a, hipStream_t stream);
int net_reset(NetPlan *plan, const NetArgs &a, hipStream_t stream);
// Flat parameter count of the network.
int64_t net_params(int F, int K, int n_hidden, const int *hidden);

}  // namespace ce
