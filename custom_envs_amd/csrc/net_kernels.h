// Hand-written CDNA4 kernels of the layered network path (Optimize-v0 over
// an OptimizeNN network: custom_envs/problems/optimize_nn.py:22-64,
// create_neural_net utils_tf.py:74-86; the env step optimize.py:69-100).
// No library GEMM: every dense product runs on v_mfma_f32_16x16x4_f32 /
// v_mfma_f32_32x32x2_f32 issued from these kernels.
//
// One VecEnv.step (net_engine.hip), two streams:
//   net_update_kernel  W' = W - a into the env's weight IMAGE (below), step += 1
//   net_gather_kernel  the env's minibatch rows (sequence[0] of its row order)
//                      into the forward's B-operand layout, with their labels
//   net_fwd_kernel     (minibatch mode) the minibatch forward: activations,
//                      dZ = P - Y, loss / hits (optimize.py:74-76)
//   then, concurrently:
//     main stream  net_fwd_kernel (info mode): the forward of every dataset
//                  row (info['objective'] / ['accuracy'], optimize.py:94-97)
//                  -- 64 rows x one env per workgroup, the whole layer chain
//                  in registers; MFMA-bound
//     side stream  net_bwd_kernel: dZ_l = (dZ_{l+1} W_{l+1}^T) * relu'(H_l),
//                  one hidden layer per launch, top down; net_grad_kernel:
//                  [dW_l; db_l] = [H_{l-1} | 1]^T dZ_l on MFMA, and in the same
//                  registers the float64 epilogue G' = (g / B) / (|G| + 1),
//                  obs = [0 | L' | G'] (optimize.py:78-91); HBM-bound, so it
//                  runs in the VGPRs / issue slots the forward leaves free
//   net_finish_kernel  per env: L', reward, done, info, the auto-reset
//                      (utils_venv.py:31: W <- W0, order <- order[perm])
// With B == N (full batch) the two forwards are one: the info forward also
// leaves the minibatch outputs, and the chain after it is serial.
//
// The weight IMAGE of an env (floats, NetGeom::Pimg per env) is the layout the
// forward streams through LDS by LDS-DMA (global_load_lds_dwordx4), one
// 32-row chunk per slot:
//   layer l rows  [nchunk_l * 32][op_l]: op_l = d_out rounded up to 64 (zero
//                 columns beyond d_out); layer 0 rows are the input features
//                 in order (zero rows past F); a hidden layer's rows are its
//                 input units in the order the previous layer's MFMA
//                 accumulators hold them (net_img_row), so a chunk is 32
//                 contiguous rows and a lane's 16-byte read gives four output
//                 blocks
//   bias area     every layer's bias, permuted so a lane reads its four
//                 accumulator rows of a block as one float4 (net_bias_slot)
// The flat [W1 | b1 | W2 | b2 | ...] vector (the reference's
// trainable_variables order, utils_common.flatten_arrays) is what the C ABI
// hands out; the engine converts at seed / get_state / set_state.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "net_engine.h"

namespace ce {

constexpr int kNetWaveRows = 16;      // dataset rows per wave (16x16x4 MFMA N)
constexpr int kNetFwdWaves = 4;
constexpr int kNetTile = kNetWaveRows * kNetFwdWaves;   // rows per forward workgroup
constexpr int kNetSlotFloats = kNetChunk * kNetMaxOp;  // 32 / 16 KB
constexpr int kNetHalves = kNetChunk / 16;              // 16-row MFMA K blocks per chunk
constexpr int kNetFwdOcc = kNetChunk == 16 ? 3 : 2;      // forward workgroups per CU
constexpr int kNetMaxBias = 4 * kNetMaxOp + 64;
constexpr int kNetThreads = 256;

typedef float net_f4 __attribute__((ext_vector_type(4)));
typedef float net_f16 __attribute__((ext_vector_type(16)));

// ---------------------------------------------------------------------------
// W' = W - a (optimize.py:74-75: one float32 subtraction, as numpy), from the
// caller's flat action into the image; current_step += 1
// (baseenvironment.py:30-41).  One wave per image row, four columns per lane.
struct NetUpdArgs {
    NetGeom g;
    int E, P;
    float *img;                      // [E][Pimg]
    const float *act;                // [E][P] flat
    int32_t *step;
};

// One layer's rows [0, rows) of the image: row q holds input unit
// net_row_unit(l, q); lane c4 updates columns 4 lane .. + 3 (U rows in
// flight per wave).  The layer index is a compile-time constant at every
// call, so its geometry comes from scalar registers, not memory.
template <int U>
__device__ __forceinline__ void net_update_rows(float *img_l, const float *act_l, int l, int rows,
                                               int din, int dout, int op, int r0, int stride,
                                               int lane) {
    const int v = 4 * lane;
    const bool vin = v < dout;
    for (int r = r0; r < rows; r += U * stride) {
        net_f4 w[U];
        float av[U][4];
        bool ok[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const int q = r + u * stride;                   // wave-uniform
            const int k = net_row_unit(l, q < rows ? q : 0);
            ok[u] = q < rows && k < din && vin;
            const int qc = ok[u] ? q : 0, kc = ok[u] ? k : 0, vc = vin ? v : 0;
            w[u] = *reinterpret_cast<const net_f4 *>(img_l + static_cast<int64_t>(qc) * op + vc);
            const float *ar = act_l + static_cast<int64_t>(kc) * dout + vc;
#pragma unroll
            for (int c = 0; c < 4; ++c) av[u][c] = v + c < dout ? ar[c] : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (ok[u])
                *reinterpret_cast<net_f4 *>(img_l + static_cast<int64_t>(r + u * stride) * op + v) =
                    net_f4{w[u][0] - av[u][0], w[u][1] - av[u][1], w[u][2] - av[u][2], w[u][3] - av[u][3]};
    }
}

__global__ __launch_bounds__(kNetThreads) void net_update_kernel(NetUpdArgs a) {
    const int e = blockIdx.y;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) a.step[e] += 1;
    float *img = a.img + static_cast<size_t>(e) * a.g.Pimg;
    const float *act = a.act + static_cast<size_t>(e) * a.P;
    const int stride = gridDim.x * 4;                       // waves over this env
    const int r0 = blockIdx.x * 4 + wave;
#pragma unroll
    for (int l = 0; l < kNetL; ++l) {
        if (l >= a.g.nl) break;
        net_update_rows<4>(img + a.g.img_off[l], act + a.g.flat_w[l], l, a.g.nchunk[l] * kNetChunk,
                           a.g.din[l], a.g.dout[l], a.g.op[l], r0, stride, lane);
    }
    // the bias area: slot s of layer l's block is unit net_bias_unit(s)
    const int s = (r0 * 64 + lane) * 4;                     // one float4 per lane
    for (int s4 = s; s4 < a.g.bias_total; s4 += stride * 256) {
#pragma unroll
        for (int l = 0; l < kNetL; ++l) {
            if (l >= a.g.nl) break;
            const int rel = s4 - a.g.bias_rel[l];
            if (rel < 0 || rel >= a.g.op[l]) continue;
            float *dst = img + a.g.bias_base + s4;
            net_f4 w = *reinterpret_cast<const net_f4 *>(dst);
            const float *b = act + a.g.flat_w[l] + static_cast<int64_t>(a.g.din[l]) * a.g.dout[l];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int un = net_bias_unit(rel + c);
                if (un < a.g.dout[l]) w[c] -= b[un];
            }
            *reinterpret_cast<net_f4 *>(dst) = w;
        }
    }
}

// ---------------------------------------------------------------------------
// The forward.  Workgroup = one env x 64 dataset rows, 4 waves x 16 rows.
// Hidden activations stay in MFMA accumulators: layer l's output block
// (c, j) holds units 64c + 16g + 4i + j (lane group g, register i) for row
// n = lane & 15, which is exactly the B operand layout of layer l + 1's
// K steps (net_img_row), so the chain never leaves registers.  A operand:
// the lane's 16-byte LDS read of weight row k, columns 64c + 4m .. +3 =
// four output blocks (c, 0..3).  Weights stream through two LDS slots in
// 32-row chunks, the chunk sequence running across layer boundaries: chunk
// ci + 1 is loaded into registers while chunk ci is multiplied, and written
// to the free slot after it (register staging: an LDS-DMA in flight makes
// the compiler wait for it before every LDS read).
// Two modes: info (rows = N, the shared dataset image, no stores but the
// partials) and minibatch (mb = 1: rows = B, the env's gathered rows; row r is
// minibatch slot r and leaves its activations and dZ).
struct NetFwdArgs {
    NetGeom g;
    int E, rows, T, F16, mb;
    float *img;                      // [E][Pimg] (FUSED writes W')
    const float *Xt;                 // [T * 4][F16][64 lanes][4]: rows in B-operand order
    int64_t xt_env;                  // floats between envs' Xt (0: shared)
    const int32_t *label;            // [T * 64] per env
    int64_t label_env;               // ints between envs' labels (0: shared)
    double *part_loss;               // [E][T]
    int32_t *part_hits;              // [E][T]
    float *act_mb[kNetL];            // hidden layer l: [E][B][op_l] post-relu minibatch rows
    float *dz_out;                   // [E][B][op_{nl-1}] P - Y of the minibatch rows
    // FUSED only: the update's action and the minibatch rows
    int N, F, P;
    const float *X;                  // [N][F]
    const float *act;                // [E][P] flat
    int32_t *step;
    const int32_t *order;            // [2][E][N] (nullptr: rows in order)
    const int32_t *order_sel;
};

__device__ __forceinline__ net_f4 net_mfma16(float a, float b, net_f4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// Four K steps (half s of a 32-row chunk) into the NCG output groups (op =
// 64 NCG): step b takes B operand bv[b]; its A operand is LDS row 16s + 4g + b
// (layer 0: lane group g holds features 16t + 4g .. + 3 of the Xt image) or
// 16s + 4b + g (hidden layers: chunk row rho = 16 (j & 1) + 4i + g).  The
// reads of step b + 1 issue under step b's MFMAs; the empty asm keeps the
// compiler from hoisting more (it would run out of registers).
template <int NCG, bool L0>
__device__ __forceinline__ void net_half_mm(const float *sl, int s, int g, int n, const net_f4 &bv,
                                            net_f4 (&hout)[16]) {
    constexpr int op = 64 * NCG;
    net_f4 w[2][NCG];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        if (k < 4) {
            const float *wr = sl + (16 * s + (L0 ? 4 * g + k : 4 * k + g)) * op + 4 * n;
#pragma unroll
            for (int c = 0; c < NCG; ++c) w[k & 1][c] = *reinterpret_cast<const net_f4 *>(wr + 64 * c);
        }
        if (k > 0) {
            const int kk = k - 1;
#pragma unroll
            for (int c = 0; c < NCG; ++c)
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    hout[c * 4 + j] = net_mfma16(w[kk & 1][c][j], bv[kk], hout[c * 4 + j]);
        }
        asm volatile("" ::: "memory");
    }
}

// Per-workgroup state of the forward's weight stream.  The image's chunks
// are contiguous in stream order (layer after layer; a layer-0 padding
// chunk is not in the image), so the next chunk's source is a running
// pointer and its width is known statically: no geometry lookup (a runtime
// index into the kernel-argument arrays costs a memory round trip).  The two
// slots are DISTINCT __shared__ arrays and every access names one
// statically: the compiler then knows an LDS-DMA in flight into one slot
// does not alias the reads of the other, and inserts no vmcnt wait before
// them (with a runtime slot index it waited for the DMA before every read).
struct NetStream {
    const float *next;               // source of the next chunk to load
    int wave, lane;
    bool dma;                        // false: producer waves fill the slots (FUSED)
};

// LDS-DMA (global_load_lds_dwordx4, 1 KB per wave instruction) of the next
// chunk (32 rows x op floats) into dst; op == 0: nothing to load
__device__ __forceinline__ void net_issue(NetStream &ws, int op, float *dst) {
    if (op == 0 || !ws.dma) return;
    const int ninst = op * kNetChunk / 256;
    for (int k = ws.wave; k < ninst; k += kNetFwdWaves)
        __builtin_amdgcn_global_load_lds(
            (__attribute__((address_space(1))) void *)(ws.next + k * 256 + ws.lane * 4),
            (__attribute__((address_space(3))) void *)(dst + k * 256), 16, 0, 0);
    ws.next += kNetChunk * op;
}

// top of a chunk: this wave's DMA (and X loads) of the chunk landed, then
// the workgroup's; the other slot is free for the next chunk (net_issue).
// (The builtin, not inline asm: the compiler's wait tracking sees it and
// knows the X operands loaded with the chunk are in, instead of waiting for
// them again behind the next DMA -- vmcnt counts in order.)
__device__ __forceinline__ void net_chunk_wait() {
    __builtin_amdgcn_s_waitcnt(0x0f70);                     // vmcnt(0), expcnt / lgkmcnt untouched
    __syncthreads();
}

// Layer 0 over its nch chunks, padded to even (slot A for even positions, B
// for odd): B operands from the Xt image, prefetched a chunk ahead.
// op_next: width of the next layer's chunks (loaded once this layer's are).
// xf(t): the lane's float4 of feature group t (t < F16).
template <int NCG, typename XF>
__device__ __forceinline__ void net_layer0(NetStream &ws, int nch, int op_next, int F16, const XF &xf,
                                           int g, int n, float *sa, float *sb, bool active,
                                           net_f4 (&hout)[16]) {
    constexpr int op = 64 * NCG;
    // what position q of the padded sequence loads: a real chunk, the padding
    // (nothing), or the next layer's first chunk
    auto op_at = [&](int q) { return q < nch ? op : (q == nch && (nch & 1) ? 0 : op_next); };
    constexpr int H = kNetHalves;
    net_f4 xn[H], xc[H];
    auto xload = [&](int lc) {
#pragma unroll
        for (int t = 0; t < H; ++t) xn[t] = H * lc + t < F16 ? xf(H * lc + t) : net_f4{0.0f, 0.0f, 0.0f, 0.0f};
    };
    xload(0);
    // the X operands are copied out before the next DMA issues (vmcnt counts
    // in order: a later use would wait for that DMA as well).  A 16-row block
    // past the features (F = 784 fills 24.5 32-row chunks) is zero rows times
    // zero features: skipped.
    for (int lc = 0; lc < nch; lc += 2) {
        net_chunk_wait();
#pragma unroll
        for (int t = 0; t < H; ++t) xc[t] = xn[t];
        net_issue(ws, op_at(lc + 1), sb);
        if (lc + 1 < nch) xload(lc + 1);
        if (active)
#pragma unroll
            for (int t = 0; t < H; ++t)
                if (t == 0 || H * lc + t < F16) net_half_mm<NCG, true>(sa, t, g, n, xc[t], hout);
        net_chunk_wait();
#pragma unroll
        for (int t = 0; t < H; ++t) xc[t] = xn[t];
        net_issue(ws, op_at(lc + 2), sa);
        if (lc + 1 < nch && active) {                       // not the padding chunk
            if (lc + 2 < nch) xload(lc + 2);
#pragma unroll
            for (int t = 0; t < H; ++t)
                if (t == 0 || H * (lc + 1) + t < F16) net_half_mm<NCG, true>(sb, t, g, n, xc[t], hout);
        }
    }
}

// A hidden-to-next layer over its nch (2 or 8) chunks: chunk lc holds the
// units of input blocks (lc >> 1, 2 (lc & 1) + {0, 1}), B operands straight
// from the previous layer's accumulators.  hin rotates down by four blocks
// per chunk pair, so the loop keeps static register indices (fully unrolled
// it spilled 4-28k VGPRs).  op_next: 0 after the output layer.
template <int NCG>
__device__ __forceinline__ void net_layer(NetStream &ws, int nch, int op_next, int g, int n,
                                          float *sa, float *sb, bool active, net_f4 (&hin)[16],
                                          net_f4 (&hout)[16]) {
    constexpr int op = 64 * NCG, H = kNetHalves;
    for (int lc = 0; lc < nch; lc += 2) {
        net_chunk_wait();
        net_issue(ws, op, sb);                              // lc + 1 < nch: nch is even
        if (active)
#pragma unroll
            for (int t = 0; t < H; ++t) net_half_mm<NCG, false>(sa, t, g, n, hin[t], hout);
        net_chunk_wait();
        net_issue(ws, lc + 2 < nch ? op : op_next, sa);
        if (active)
#pragma unroll
            for (int t = 0; t < H; ++t) net_half_mm<NCG, false>(sb, t, g, n, hin[H + t], hout);
#pragma unroll
        for (int i = 0; i < 16 - 2 * H; ++i) hin[i] = hin[i + 2 * H];
    }
}

// The output layer for K <= 16 classes ("narrow"): one MFMA block per K step
// instead of four.  The lane's A operand is the scalar at column n of image
// row 16 s + 4 k + g (unit n: the image keeps its 64-column layout), so block
// lane (g, n) register i ends as unit 4 g + i of row n; the four-block form
// computed 64 units for <= 16 real ones (5 % of the forward's MFMAs).
__device__ __forceinline__ void net_half_mm_narrow(const float *sl, int s, int g, int n, const net_f4 &bv,
                                                   net_f4 &h0) {
    float w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = sl[(16 * s + 4 * k + g) * 64 + n];
#pragma unroll
    for (int k = 0; k < 4; ++k) h0 = net_mfma16(w[k], bv[k], h0);
}

__device__ __forceinline__ void net_layer_narrow(NetStream &ws, int nch, int g, int n, float *sa, float *sb,
                                                 bool active, net_f4 (&hin)[16], net_f4 &h0) {
    constexpr int H = kNetHalves;
    for (int lc = 0; lc < nch; lc += 2) {
        net_chunk_wait();
        net_issue(ws, 64, sb);                              // lc + 1 < nch: nch is even
        if (active)
#pragma unroll
            for (int t = 0; t < H; ++t) net_half_mm_narrow(sa, t, g, n, hin[t], h0);
        net_chunk_wait();
        if (lc + 2 < nch) net_issue(ws, 64, sa);
        if (active)
#pragma unroll
            for (int t = 0; t < H; ++t) net_half_mm_narrow(sb, t, g, n, hin[H + t], h0);
#pragma unroll
        for (int i = 0; i < 16 - 2 * H; ++i) hin[i] = hin[i + 2 * H];
    }
}

// FUSED mode's producer waves (2 and 3; the minibatch's <= 32 rows are waves
// 0 and 1): the update W' = W - a (optimize.py:74-75, as net_update_kernel)
// streamed chunk by chunk through registers -- W' to the env's image in HBM
// and into the LDS slot the consumer waves multiply next.  The barrier
// schedule is the consumers': the sbias barrier, one per chunk position of
// the stream (layer 0's count padded to even), and the partials' barrier.
// After barrier p the slot of chunk p - 1 is free: chunk p + 1 goes there and
// chunk p + 2's loads are issued, a whole chunk of consumer work ahead.
template <int NCGH>
__device__ __forceinline__ void net_producer(const NetFwdArgs &a, int e, int pw, int lane, float *slot_a,
                                             float *slot_b, float *sbias, double *red_loss, int *red_hits) {
    constexpr int OPH = 64 * NCGH;
    constexpr int R = kNetChunk / 2;                        // rows per producer wave and chunk
    const int nl = a.g.nl;
    float *img = a.img + static_cast<size_t>(e) * a.g.Pimg;
    const float *act = a.act + static_cast<size_t>(e) * a.P;
    // the bias area (slot s of layer l's block is unit net_bias_unit(s))
    for (int s4 = (pw * 64 + lane) * 4; s4 < a.g.bias_total; s4 += 128 * 4) {
        net_f4 w = *reinterpret_cast<const net_f4 *>(img + a.g.bias_base + s4);
#pragma unroll
        for (int l = 0; l < kNetL; ++l) {
            if (l >= nl) break;
            const int rel = s4 - a.g.bias_rel[l];
            if (rel < 0 || rel >= a.g.op[l]) continue;
            const float *b = act + a.g.flat_w[l] + static_cast<int64_t>(a.g.din[l]) * a.g.dout[l];
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                const int un = net_bias_unit(rel + c);
                if (un < a.g.dout[l]) w[c] -= b[un];
            }
        }
        *reinterpret_cast<net_f4 *>(img + a.g.bias_base + s4) = w;
        *reinterpret_cast<net_f4 *>(sbias + s4) = w;
    }
    const int nch0 = a.g.nchunk[0], p0 = nch0 + (nch0 & 1);
    constexpr int PL = OPH / kNetChunk;                     // chunk positions of layers >= 1
    const int np = p0 + (nl - 1) * PL;
    net_f4 wv[R];
    float av[R][4];
    // chunk position p -> layer, chunk (false: layer 0's padding or the end)
    auto locate = [&](int p, int &l, int &c) {
        if (p < p0) {
            l = 0;
            c = p;
            return p < nch0;
        }
        l = 1 + (p - p0) / PL;
        c = (p - p0) % PL;
        return p < np;
    };
    auto load = [&](int p) {
        int l, c;
        if (!locate(p, l, c)) return;
        const int op = l == nl - 1 ? 64 : OPH, din = a.g.din[l], dout = a.g.dout[l];
        const float *src = img + a.g.img_off[l] + static_cast<int64_t>(c) * kNetChunk * op;
        const float *al = act + a.g.flat_w[l];
        const int v = 4 * lane;
        const bool wok = v < op;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int rho = pw + 2 * i, k = net_row_unit(l, c * kNetChunk + rho);
            wv[i] = wok ? *reinterpret_cast<const net_f4 *>(src + rho * op + v) : net_f4{0.0f, 0.0f, 0.0f, 0.0f};
            const float *ar = al + static_cast<int64_t>(k < din ? k : 0) * dout;
#pragma unroll
            for (int q = 0; q < 4; ++q) av[i][q] = k < din && v + q < dout ? ar[v + q] : 0.0f;
        }
    };
    auto store = [&](int p, float *slot) {
        int l, c;
        if (!locate(p, l, c)) return;
        const int op = l == nl - 1 ? 64 : OPH;
        float *dst = img + a.g.img_off[l] + static_cast<int64_t>(c) * kNetChunk * op;
        const int v = 4 * lane;
        if (v >= op) return;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const int rho = pw + 2 * i;
            const net_f4 w = {wv[i][0] - av[i][0], wv[i][1] - av[i][1], wv[i][2] - av[i][2], wv[i][3] - av[i][3]};
            *reinterpret_cast<net_f4 *>(dst + rho * op + v) = w;
            *reinterpret_cast<net_f4 *>(slot + rho * op + v) = w;
        }
    };
    load(0);
    __builtin_amdgcn_s_waitcnt(0x0f70);
    store(0, slot_a);
    load(1);
    __syncthreads();                                        // sbias + chunk 0
    for (int p = 0; p < np; ++p) {
        __syncthreads();                                    // the consumers' chunk p
        __builtin_amdgcn_s_waitcnt(0x0f70);                 // chunk p + 1 is in registers
        if ((p + 1) & 1) store(p + 1, slot_b);
        else store(p + 1, slot_a);
        load(p + 2);
    }
    if (lane == 0) {
        red_loss[2 + pw] = 0.0;
        red_hits[2 + pw] = 0;
    }
    __syncthreads();                                        // the partials
}

// NCGH: 64-unit output groups of every hidden layer (net_geometry pads all
// hidden widths to one op = 64 NCGH, 64 or 256); the output layer has one
// (K <= 32).  So layer l's op, chunk count and bias offset are static
// functions of l: op = 64 NCGH (hidden) / 64 (output), nchunk = 2 NCGH
// (l >= 1), bias at l * 64 NCGH.
// NARROW: the output layer has <= 16 classes (net_layer_narrow).
// FUSED: the minibatch forward (rows = B <= 32, one workgroup per env) with
// the update in its producer waves (net_producer) and the minibatch's
// dataset rows read straight from X through the env's row order -- replaces
// net_update_kernel, net_gather_kernel and the separate minibatch forward.
template <int NCGH, bool NARROW, bool FUSED>
__global__ __launch_bounds__(kNetThreads, kNetFwdOcc) void net_fwd_kernel(NetFwdArgs a) {
    constexpr int OPH = 64 * NCGH;
    __shared__ __attribute__((aligned(16))) float slot_a[kNetSlotFloats];
    __shared__ __attribute__((aligned(16))) float slot_b[kNetSlotFloats];
    __shared__ __attribute__((aligned(16))) float sbias[kNetMaxBias];
    __shared__ double red_loss[kNetFwdWaves];
    __shared__ int red_hits[kNetFwdWaves];

    // XCD-aware: blocks b and b + 8 share an XCD (MI355X_MICROARCH), so the T
    // row tiles of one env are consecutive on ONE XCD and its L2 serves the
    // env's weight chunks to all of them
    const int b = blockIdx.x, xcd = b & 7, qd = b >> 3;
    const int e = (qd / a.T) * 8 + xcd, tile = qd - (qd / a.T) * a.T;
    if (e >= a.E) return;                                   // whole workgroup, before any barrier
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63, g = lane >> 4, n = lane & 15;
    const int row = tile * kNetTile + wave * kNetWaveRows + n;
    const bool rvalid = row < a.rows;
    // a wave without a valid row (the minibatch's last tile) keeps the DMA
    // and barriers but issues no MFMA: its SIMD serves the other workgroup
    const bool active = tile * kNetTile + wave * kNetWaveRows < a.rows;
    const float *img = a.img + static_cast<size_t>(e) * a.g.Pimg;
    const int nl = a.g.nl;
    NetStream ws{img, wave, lane, !FUSED};

    if (FUSED && wave >= 2) {
        net_producer<NCGH>(a, e, wave - 2, lane, slot_a, slot_b, sbias, red_loss, red_hits);
        return;
    }
    int xrow = 0;                                           // FUSED: the dataset row
    if (FUSED) {
        if (tid == 0) a.step[e] += 1;                       // current_step += 1 (baseenvironment.py:30-41)
        if (rvalid)
            xrow = a.order ? a.order[(static_cast<size_t>(a.order_sel[e]) * a.E + e) * a.N + row] : row;
    } else {
        for (int i = tid; i < a.g.bias_total; i += kNetThreads) sbias[i] = img[a.g.bias_base + i];
    }
    const int slot_n = a.mb && rvalid ? row : -1;
    const int yl = rvalid ? (FUSED ? a.label[xrow] : a.label[e * a.label_env + row]) : 0;

    net_f4 hin[16], hout[16];
    auto bias_init = [&](int l, int ncg) {
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j)
                hout[c * 4 + j] = c < ncg ? *reinterpret_cast<const net_f4 *>(
                                                &sbias[l * OPH + ((c * 4 + j) * 4 + g) * 4])
                                          : net_f4{0.0f, 0.0f, 0.0f, 0.0f};
    };
    auto op_of = [&](int l) { return l >= nl ? 0 : (l == nl - 1 ? 64 : OPH); };

    net_issue(ws, OPH, slot_a);
    __syncthreads();                                        // sbias
    bias_init(0, NCGH);

    // ---- layer 0: K = the input features, B operand = X rows
    if (FUSED) {
        // features 16 t + 4 g .. + 3 of the row, from X itself
        const float *xr = a.X + static_cast<size_t>(xrow) * a.F;
        const bool x4 = (a.F & 3) == 0;
        auto xf = [&](int t) {
            const int f0 = 16 * t + 4 * g;
            net_f4 v = {0.0f, 0.0f, 0.0f, 0.0f};
            if (!rvalid) return v;
            if (x4 && f0 < a.F) return *reinterpret_cast<const net_f4 *>(xr + f0);
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = f0 + q < a.F ? xr[f0 + q] : 0.0f;
            return v;
        };
        net_layer0<NCGH>(ws, a.g.nchunk[0], op_of(1), a.F16, xf, g, n, slot_a, slot_b, active, hout);
    } else {
        // (this wave's 16-row block of Xt, the lane's float4 of feature group t)
        const float *xt = a.Xt + e * a.xt_env +
                          (static_cast<size_t>(tile * (kNetTile / 16) + wave) * a.F16 * 64 + lane) * 4;
        auto xf = [&](int t) { return *reinterpret_cast<const net_f4 *>(xt + t * 256); };
        net_layer0<NCGH>(ws, a.g.nchunk[0], op_of(1), a.F16, xf, g, n, slot_a, slot_b, active, hout);
    }

    // ---- layers 1 .. nl-1: K = the previous layer's units, from registers
    for (int l = 0; l + 1 < nl; ++l) {
        // hidden layer l done: relu (optimize_nn.py: Dense(relu)), the
        // minibatch rows' activations out, next layer's bias in the accumulators
#pragma unroll
        for (int c = 0; c < NCGH; ++c)
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int i = 0; i < 4; ++i) hin[c * 4 + j][i] = fmaxf(hout[c * 4 + j][i], 0.0f);
        if (slot_n >= 0) {
            float *dst = a.act_mb[l] + (static_cast<size_t>(e) * a.rows + slot_n) * OPH;   // mb mode: rows = B
#pragma unroll
            for (int c = 0; c < NCGH; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    *reinterpret_cast<net_f4 *>(dst + 64 * c + 16 * g + 4 * i) =
                        net_f4{hin[c * 4 + 0][i], hin[c * 4 + 1][i], hin[c * 4 + 2][i], hin[c * 4 + 3][i]};
        }
        if (l + 2 < nl) {
            bias_init(l + 1, NCGH);
            net_layer<NCGH>(ws, OPH / kNetChunk, op_of(l + 2), g, n, slot_a, slot_b, active, hin, hout);
        }
    }
    const int K = a.g.dout[nl - 1];
    float z[kNetMaxClasses];
    if (NARROW) {
        // bias of unit 4 g + i: permuted slot 16 i + g of the layer (net_bias_slot)
#pragma unroll
        for (int i = 0; i < 4; ++i) hout[0][i] = sbias[(nl - 1) * OPH + 16 * i + g];
        net_layer_narrow(ws, OPH / kNetChunk, g, n, slot_a, slot_b, active, hin, hout[0]);
        // class 4 g' + i of row n sits in lane 16 g' + n, register i
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int gp = 0; gp < 4; ++gp) z[4 * gp + i] = __shfl(hout[0][i], 16 * gp + n);
#pragma unroll
        for (int k = 16; k < kNetMaxClasses; ++k) z[k] = 0.0f;
    } else {
        bias_init(nl - 1, 1);
        net_layer<1>(ws, OPH / kNetChunk, 0, g, n, slot_a, slot_b, active, hin, hout);   // the output layer
        // class 16g + 4i + j of row n sits in lane group g: lane group 0
        // gathers the row
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                z[4 * i + j] = hout[j][i];
                z[16 + 4 * i + j] = __shfl_down(hout[j][i], 16);
            }
    }

    // ---- logits -> softmax (utils_math.py:51-63), -log(p_y + 1e-16)
    // (utils_math.py:25-34), np.argmax's first maximum of P, in lane group 0
    double loss_r = 0.0;
    int hit_r = 0;
    const bool owner = g == 0 && rvalid;
    if (owner) {
        float m = z[0];
#pragma unroll
        for (int k = 1; k < kNetMaxClasses; ++k)
            if (k < K) m = fmaxf(m, z[k]);
        float s = 0.0f;
#pragma unroll
        for (int k = 0; k < kNetMaxClasses; ++k)
            if (k < K) {
                z[k] = expf(z[k] - m);
                s += z[k];
            }
        int arg = 0;
        float best = -1.0f, py = 0.0f;
#pragma unroll
        for (int k = 0; k < kNetMaxClasses; ++k)
            if (k < K) {
                z[k] = z[k] / s;                             // P
                if (z[k] > best) {
                    best = z[k];
                    arg = k;
                }
                if (k == yl) py = z[k];
            }
        loss_r = static_cast<double>(-logf(py + 1e-16f));
        hit_r = arg == yl ? 1 : 0;
        if (slot_n >= 0) {
            float *dz = a.dz_out + (static_cast<size_t>(e) * a.rows + slot_n) * 64;   // output op = 64
#pragma unroll
            for (int k = 0; k < kNetMaxClasses; ++k)
                if (k < K) dz[k] = z[k] - (k == yl ? 1.0f : 0.0f);
        }
    }
    double lsum = loss_r;
    int hsum = hit_r;
#pragma unroll
    for (int w = 8; w > 0; w >>= 1) {
        lsum += __shfl_xor(lsum, w);
        hsum += __shfl_xor(hsum, w);
    }
    if (lane == 0) {
        red_loss[wave] = lsum;
        red_hits[wave] = hsum;
    }
    __syncthreads();
    if (tid == 0) {
        double l = 0.0;
        int h = 0;
#pragma unroll
        for (int w = 0; w < kNetFwdWaves; ++w) {
            l += red_loss[w];
            h += red_hits[w];
        }
        const size_t o = static_cast<size_t>(e) * a.T + tile;
        a.part_loss[o] = l;
        a.part_hits[o] = h;
    }
}

// ---------------------------------------------------------------------------
// The minibatch rows of env e -- dataset row order[sel][e][i] for slot
// i < B (optimize.py:72-76: sequence[0] of the env's row order) -- in the
// forward's B-operand layout (lane g * 16 + n of 16-row block rb, feature
// group t holds row 16 rb + n's features 16 t + 4 g .. + 3; zeros past F and
// past B), with their labels.  One workgroup per 16-row block.
struct NetGatherArgs {
    int E, N, B, F, F16, Tmb;
    const float *X;                  // [N][F]
    const int32_t *label;            // [N]
    const int32_t *order;            // [2][E][N] (nullptr: rows in order)
    const int32_t *order_sel;
    float *Xmb;                      // [E][Tmb * 4][F16][64][4]
    int32_t *label_mb;               // [E][Tmb * 64]
};

__global__ __launch_bounds__(kNetThreads) void net_gather_kernel(NetGatherArgs a) {
    const int e = blockIdx.y, rb = blockIdx.x;
    __shared__ int32_t src[16];
    if (threadIdx.x < 16) {
        const int i = rb * 16 + threadIdx.x;
        int32_t r = -1;
        if (i < a.B)
            r = a.order ? a.order[(static_cast<size_t>(a.order_sel[e]) * a.E + e) * a.N + i] : i;
        src[threadIdx.x] = r;
        a.label_mb[static_cast<size_t>(e) * a.Tmb * 64 + i] = r >= 0 ? a.label[r] : 0;
    }
    __syncthreads();
    float *dst = a.Xmb + ((static_cast<size_t>(e) * a.Tmb * 4 + rb) * a.F16) * 256;
    for (int q = threadIdx.x; q < a.F16 * 64; q += kNetThreads) {
        const int t = q >> 6, ln = q & 63;
        const int32_t r = src[ln & 15];
        const int f0 = 16 * t + 4 * (ln >> 4);
        net_f4 v = {0.0f, 0.0f, 0.0f, 0.0f};
        if (r >= 0) {
            const float *x = a.X + static_cast<size_t>(r) * a.F;
#pragma unroll
            for (int c = 0; c < 4; ++c) v[c] = f0 + c < a.F ? x[f0 + c] : 0.0f;
        }
        *reinterpret_cast<net_f4 *>(dst + static_cast<size_t>(q) * 4) = v;
    }
}

// ---------------------------------------------------------------------------
// dH_l = dZ_{l+1} W_{l+1}^T, dZ_l = dH_l * (H_l > 0) over the minibatch rows
// (tf.gradients of the summed cross-entropy, optimize_nn.py:48-52), for one
// hidden layer lh; one workgroup per env.  dH^T (units x rows) on 16x16x4:
// A = W_{l+1} rows (its image rows are the units of H_l), B = dZ_{l+1}.
struct NetBwdArgs {
    NetGeom g;
    int E, B, lh;
    const float *img;
    const float *dz_next;            // [E][B][op_{lh+1}]
    const float *act;                // [E][B][op_lh] post-relu H_lh
    float *dz;                       // [E][B][op_lh]
};

__global__ __launch_bounds__(kNetThreads) void net_bwd_kernel(NetBwdArgs a) {
    const int e = blockIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, g = lane >> 4, n = lane & 15;
    const int lh = a.lh, lo = lh + 1;
    const int op = a.g.op[lh], opn = a.g.op[lo];
    const int vend = (a.g.dout[lo] + 15) & ~15;
    const float *W = a.img + static_cast<size_t>(e) * a.g.Pimg + a.g.img_off[lo];
    const float *dzn = a.dz_next + static_cast<size_t>(e) * a.B * opn;
    const float *H = a.act + static_cast<size_t>(e) * a.B * op;
    float *dz = a.dz + static_cast<size_t>(e) * a.B * op;
    const int nrb = (a.B + 15) >> 4, nub = op >> 4;
    for (int t = wave; t < nrb * nub; t += kNetFwdWaves) {
        const int rbk = t / nub, ub = t - rbk * nub;
        const int u = 16 * ub + n, r = 16 * rbk + n;
        const float *wr = W + static_cast<int64_t>(net_img_row(lo, u)) * opn + 4 * g;
        const float *zr = dzn + static_cast<int64_t>(r) * opn + 4 * g;
        const bool rok = r < a.B;
        net_f4 acc = {0.0f, 0.0f, 0.0f, 0.0f};
        for (int v0 = 0; v0 < vend; v0 += 16) {
            const net_f4 wv = *reinterpret_cast<const net_f4 *>(wr + v0);
            const net_f4 zv = rok ? *reinterpret_cast<const net_f4 *>(zr + v0) : net_f4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int q = 0; q < 4; ++q) acc = net_mfma16(wv[q], zv[q], acc);
        }
        // acc[i] = dH[row 16 rbk + n][unit 16 ub + 4g + i]
        if (rok) {
            const size_t o = static_cast<size_t>(r) * op + 16 * ub + 4 * g;
            const net_f4 h = *reinterpret_cast<const net_f4 *>(H + o);
            *reinterpret_cast<net_f4 *>(dz + o) =
                net_f4{h[0] > 0.0f ? acc[0] : 0.0f, h[1] > 0.0f ? acc[1] : 0.0f,
                       h[2] > 0.0f ? acc[2] : 0.0f, h[3] > 0.0f ? acc[3] : 0.0f};
        }
    }
}

// ---------------------------------------------------------------------------
// [dW_l; db_l] = [H_{l-1} | 1]^T dZ_l over the minibatch rows on
// v_mfma_f32_32x32x2_f32 (the ones column gives db = sum of dZ rows), and the
// float64 epilogue straight from the accumulators: g = grad / B (float32, as
// numpy divides the float32 gradient), G' = g / (|G| + 1) in float64
// (grad_hist float64, optimize.py:78-83), obs = [0 (P) | L' | G' (P)]; an env
// whose step ends its episode (utils_venv.py:31) writes the reset
// observation and G <- 0.  Workgroup = 32 rows of [dW; db] x kNetGradTile units of one
// layer of one env; wave = 32 kNetGradWaveBlocks units (32x32 blocks).
struct NetGradArgs {
    NetGeom g;
    int E, N, B, P, F, max_steps, auto_reset, tpe;
    int task0[kNetL + 1];            // first task of layer l within an env
    int ut[kNetL];                   // kNetGradTile-unit tiles of layer l
    const float *X;                  // [N][F]
    const int32_t *order;            // [2][E][N] (nullptr: B == N, rows in order)
    const int32_t *order_sel;
    const float *act_mb[kNetL];
    const float *dz_mb[kNetL];       // hidden layers; the output layer reads dz_out
    const float *dz_out;
    const int32_t *step;
    double *G;                       // [E][P]
    float *obs;                      // [E][2P + 1]
};

typedef uint32_t net_u2 __attribute__((ext_vector_type(2)));
// cache-policy bits of the epilogue's buffer loads / stores (build-time A/B;
// gfx950: bit 1 = nt)
#ifndef CE_NET_GRAD_AUX_LD
#define CE_NET_GRAD_AUX_LD 0
#endif
#ifndef CE_NET_GRAD_AUX_ST
#define CE_NET_GRAD_AUX_ST 0
#endif

// A raw buffer resource over [p, p + bytes): 32-bit offsets, and an access
// at or past `bytes` is dropped (store) or reads 0 (load) in hardware
__device__ __forceinline__ __amdgpu_buffer_rsrc_t net_rsrc(const void *p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(p), 0, static_cast<int>(bytes), 0x00020000);
}

__device__ __forceinline__ net_f16 net_mfma32(float a, float b, net_f16 c) {
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// K steps of the [dW; db] product loaded in one batch (their loads in flight
// together, then the MFMAs)
constexpr int kNetGradBatch = 16;
// 32-unit accumulator blocks per wave (CE_NET_GRAD_BLOCKS, build-time A/B):
// 2 = a 256-unit workgroup tile, 1 = 128 units and half the accumulator and
// float64 epilogue registers (more waves in flight on the gathers)
#ifndef CE_NET_GRAD_BLOCKS
#define CE_NET_GRAD_BLOCKS 2
#endif
constexpr int kNetGradWaveBlocks = CE_NET_GRAD_BLOCKS;
constexpr int kNetGradTile = 4 * 32 * kNetGradWaveBlocks;   // units per workgroup task

// Persistent grid (a multiple of 8 workgroups): workgroup b works on XCD
// b & 7 (MI355X_MICROARCH: round-robin dispatch) and walks that XCD's envs
// (e = xcd + 8 j) task by task with the XCD's other workgroups, so an env's
// minibatch activations are pulled into ONE L2.  Beside the forward the grid
// is one workgroup per CU: it fits in the VGPRs the forward's two workgroups
// leave and never holds a slot the forward's next workgroup needs.
__global__ __launch_bounds__(kNetThreads) void net_grad_kernel(NetGradArgs a) {
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, h = lane >> 5, m = lane & 31;
    const int nl = a.g.nl;
    const int xcd = blockIdx.x & 7, per_xcd = gridDim.x >> 3;
    const int n_env = a.E > xcd ? (a.E - xcd + 7) >> 3 : 0;       // this XCD's envs
    const float fB = static_cast<float>(a.B);
    // g / B: a power-of-two B divides exactly by its reciprocal (one multiply
    // instead of the ten-instruction IEEE division sequence; this kernel runs
    // beside the MFMA-bound forward, whose SIMDs its VALU work shares)
    const bool pow2 = (a.B & (a.B - 1)) == 0;
    const float rB = 1.0f / fB;
    const size_t P = a.P;
    for (int q = blockIdx.x >> 3; q < n_env * a.tpe; q += per_xcd) {
        const int j = q / a.tpe, task = q - j * a.tpe;
        const int e = xcd + 8 * j;
        const bool wipe = a.step[e] >= a.max_steps && a.auto_reset;
        double *G = a.G + static_cast<size_t>(e) * P;
        float *obs = a.obs + static_cast<size_t>(e) * (2 * P + 1);
        const int32_t *rows =
            a.order ? a.order + (static_cast<size_t>(a.order_sel[e]) * a.E + e) * a.N : nullptr;
        int l = 0;
        while (l + 1 < nl && task >= a.task0[l + 1]) ++l;
        const int tl = task - a.task0[l];
        const int kt = tl / a.ut[l], ut = tl - kt * a.ut[l];
        const int din = a.g.din[l], dout = a.g.dout[l];
        const int u0 = ut * kNetGradTile + 32 * kNetGradWaveBlocks * wave;
        if (u0 >= dout) continue;                           // wave-uniform; no barriers here
        const int k0 = kt * 32, k = k0 + m;
        // A: [H_{l-1} | 1] rows (layer 0: the dataset rows of sequence[0]).
        // Branch-free: clamped indices, every load of a batch issued before
        // any is used, invalid entries zeroed by selects afterwards (a
        // guarded load per step made two dependent round trips per step)
        const bool kin = k < din, kone = k == din;
        const int kc = kin ? k : din - 1;
        const float *Hin = nullptr;
        int hstride = 0;
        if (l > 0) {
            hstride = a.g.op[l - 1];
            Hin = a.act_mb[l - 1] + static_cast<size_t>(e) * a.B * hstride;
        }
        const int opl = a.g.op[l];
        const float *dz = (l + 1 == nl ? a.dz_out : a.dz_mb[l]) + static_cast<size_t>(e) * a.B * opl + u0 + m;
        net_f16 acc[kNetGradWaveBlocks] = {};
        const int steps = (a.B + 1) >> 1;
        for (int s0 = 0; s0 < steps; s0 += kNetGradBatch) {
            int rr[kNetGradBatch];
            float xa[kNetGradBatch], bz[kNetGradWaveBlocks][kNetGradBatch];
#pragma unroll
            for (int q = 0; q < kNetGradBatch; ++q) {
                const int r = 2 * (s0 + q) + h;
                rr[q] = r < a.B ? r : a.B - 1;
            }
            if (l == 0) {                                   // wave-uniform
                int xr[kNetGradBatch];
#pragma unroll
                for (int q = 0; q < kNetGradBatch; ++q) xr[q] = rows ? rows[rr[q]] : rr[q];
#pragma unroll
                for (int q = 0; q < kNetGradBatch; ++q) xa[q] = a.X[static_cast<size_t>(xr[q]) * a.F + kc];
            } else {
#pragma unroll
                for (int q = 0; q < kNetGradBatch; ++q) xa[q] = Hin[static_cast<size_t>(rr[q]) * hstride + kc];
            }
#pragma unroll
            for (int q = 0; q < kNetGradBatch; ++q)
#pragma unroll
                for (int bb = 0; bb < kNetGradWaveBlocks; ++bb)
                    bz[bb][q] = dz[static_cast<size_t>(rr[q]) * opl + 32 * bb];
#pragma unroll
            for (int q = 0; q < kNetGradBatch; ++q) {
                const bool ok = 2 * (s0 + q) + h < a.B;
                const float av = ok ? (kin ? xa[q] : (kone ? 1.0f : 0.0f)) : 0.0f;   // the bias row: 1
#pragma unroll
                for (int bb = 0; bb < kNetGradWaveBlocks; ++bb)
                    acc[bb] = net_mfma32(av, ok ? bz[bb][q] : 0.0f, acc[bb]);
            }
        }
        // epilogue: accumulator r of lane (h, m) = row k0 + 8(r>>2) + 4h + (r&3)
        // of [dW; db], unit u0 + 32 bb + m; every G load of a block in flight
        // before its stores
        // Raw buffer accesses over the layer's [dW; db] range: 32-bit
        // offsets (no 64-bit address arithmetic per element), and rows past
        // the bias row are out of range -- their loads return 0 and their
        // stores are dropped by the hardware, so no clamps or row masks
        const int64_t fw = a.g.flat_w[l];
        const uint32_t nb = static_cast<uint32_t>(din + 1) * dout;
        const __amdgpu_buffer_rsrc_t rG = net_rsrc(G + fw, nb * 8);
        const __amdgpu_buffer_rsrc_t rW = net_rsrc(obs + fw, nb * 4);
        const __amdgpu_buffer_rsrc_t rO = net_rsrc(obs + P + 1 + fw, nb * 4);
#pragma unroll
        for (int bb = 0; bb < kNetGradWaveBlocks; ++bb) {
            const int u = u0 + 32 * bb + m;
            if (u >= dout) continue;                        // per lane, once per block
            const int base = (k0 + 4 * h) * dout + u;
            double gold[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = base + (8 * (r >> 2) + (r & 3)) * dout;
                gold[r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rG, o * 8, 0, CE_NET_GRAD_AUX_LD));
            }
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int o = base + (8 * (r >> 2) + (r & 3)) * dout;
                const float gv = pow2 ? acc[bb][r] * rB : acc[bb][r] / fB;
                const double gn = static_cast<double>(gv) / (fabs(gold[r]) + 1.0);
                // wght_hist is identically 0
                __builtin_amdgcn_raw_buffer_store_b32(0u, rW, o * 4, 0, CE_NET_GRAD_AUX_ST);
                __builtin_amdgcn_raw_buffer_store_b32(
                    __builtin_bit_cast(uint32_t, wipe ? 0.0f : static_cast<float>(gn)), rO, o * 4, 0, CE_NET_GRAD_AUX_ST);
                __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(net_u2, wipe ? 0.0 : gn), rG, o * 8, 0,
                                                      CE_NET_GRAD_AUX_ST);
            }
        }
    }
}

// ---------------------------------------------------------------------------
// Per env: the minibatch / full-data loss and hits from the forward's tile
// partials; L' = (loss - L)/(L + 0.1) (optimize.py:80-81), reward = -loss,
// done = current_step >= max_steps (:102-103), info, episode length; the
// auto-reset: W <- W0 (the image), L, step, order <- order[perm] and the
// minibatch slots of the new order.
struct NetFinArgs {
    int E, N, B, P, T, Tmb, max_steps, auto_reset;
    int64_t Pimg;
    const double *part_loss;         // [E][T]: the info forward's tiles
    const int32_t *part_hits;
    const double *mb_loss;           // [E][Tmb]: the minibatch forward's
    const int32_t *mb_hits;
    float *img;
    const float *img0;
    double *L;
    int32_t *step;
    const int32_t *perm;
    int32_t *order;
    int32_t *order_sel;
    float *obs;
    float *reward;
    uint8_t *done;
    float *objective;
    float *accuracy;
    int32_t *episode_len;
};

// order <- order[perm] (the reset's shuffle composed onto the current row
// order)
__device__ inline void net_compose_order(const NetFinArgs &a, int e) {
    const int sel = a.order_sel[e];
    const int32_t *cur = a.order + (static_cast<size_t>(sel) * a.E + e) * a.N;
    int32_t *nxt = a.order + (static_cast<size_t>(1 - sel) * a.E + e) * a.N;
    const int32_t *pm = a.perm + static_cast<size_t>(e) * a.N;
    for (int i = threadIdx.x; i < a.N; i += kNetThreads) nxt[i] = cur[pm[i]];
    __syncthreads();
    if (threadIdx.x == 0) a.order_sel[e] = 1 - sel;
}

__global__ __launch_bounds__(kNetThreads) void net_finish_kernel(NetFinArgs a) {
    const int e = blockIdx.x;
    const int cur = a.step[e];
    const bool done = cur >= a.max_steps;
    const bool wipe = done && a.auto_reset;
    __syncthreads();                                        // every thread has read step[e]
    if (threadIdx.x == 0) {
        double lm = 0.0, li = 0.0;
        int hm = 0, hi = 0;
        for (int t = 0; t < a.T; ++t) {
            li += a.part_loss[static_cast<size_t>(e) * a.T + t];
            hi += a.part_hits[static_cast<size_t>(e) * a.T + t];
        }
        for (int t = 0; t < a.Tmb; ++t) {
            lm += a.mb_loss[static_cast<size_t>(e) * a.Tmb + t];
            hm += a.mb_hits[static_cast<size_t>(e) * a.Tmb + t];
        }
        // the loss is a float32 mean in the reference (TF / numpy float32)
        const float loss = static_cast<float>(lm / a.B);
        const float acc = static_cast<float>(static_cast<double>(hm) / a.B);
        const bool full = a.B == a.N;
        const float obj = full ? loss : static_cast<float>(li / a.N);
        const float oacc = full ? acc : static_cast<float>(static_cast<double>(hi) / a.N);
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
    if (!wipe) return;
    const size_t n4 = static_cast<size_t>(a.Pimg) >> 2;
    net_f4 *w = reinterpret_cast<net_f4 *>(a.img + static_cast<size_t>(e) * a.Pimg);
    const net_f4 *w0 = reinterpret_cast<const net_f4 *>(a.img0 + static_cast<size_t>(e) * a.Pimg);
    for (size_t i = threadIdx.x; i < n4; i += kNetThreads) w[i] = w0[i];
    if (a.order != nullptr) net_compose_order(a, e);
}

// Reset (optimize.py:58-67): W <- W0, G <- 0, obs <- 0
struct NetResetArgs {
    int E, P;
    int64_t Pimg;
    float *img;
    const float *img0;
    double *G;
    float *obs;
};

__global__ __launch_bounds__(kNetThreads) void net_reset_params_kernel(NetResetArgs a) {
    const int e = blockIdx.y;
    const size_t P = a.P;
    const size_t t0 = static_cast<size_t>(blockIdx.x) * kNetThreads + threadIdx.x;
    const size_t st = static_cast<size_t>(gridDim.x) * kNetThreads;
    float *obs = a.obs + static_cast<size_t>(e) * (2 * P + 1);
    for (size_t p = t0; p < 2 * P + 1; p += st) {
        obs[p] = 0.0f;
        if (p < P) a.G[static_cast<size_t>(e) * P + p] = 0.0;
    }
    const size_t n4 = static_cast<size_t>(a.Pimg) >> 2;
    net_f4 *w = reinterpret_cast<net_f4 *>(a.img + static_cast<size_t>(e) * a.Pimg);
    const net_f4 *w0 = reinterpret_cast<const net_f4 *>(a.img0 + static_cast<size_t>(e) * a.Pimg);
    for (size_t i = t0; i < n4; i += st) w[i] = w0[i];
}

// per env: L, step, and order <- order[perm]
__global__ __launch_bounds__(kNetThreads) void net_reset_env_kernel(NetFinArgs a) {
    const int e = blockIdx.x;
    if (threadIdx.x == 0) {
        a.L[e] = 0.0;
        a.step[e] = 0;
    }
    if (a.order != nullptr) net_compose_order(a, e);
}

}  // namespace ce
