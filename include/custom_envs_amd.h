/*
 * custom_envs_amd -- C ABI of the MI355X vectorised Optimize-v0 engine.
 *
 * The reference (adolfogonzalez3/custom_envs) is pure Python and has no FFI;
 * every entry point below replaces one Python-level interface on the hot
 * path, cited as file:line relative to the reference root:
 *
 *   ce_create      Optimize.__init__            custom_envs/envs/optimize.py:40-56
 *                  + ConcurrentVecEnv.__init__   custom_envs/vectorize/concurrentvecenv.py:77-95
 *   ce_seed        BaseEnvironment.seed          custom_envs/envs/baseenvironment.py:20-28
 *   ce_seed_draws / ce_seed_draws_mlp
 *                  Optimize.base_reset draws     custom_envs/envs/optimize.py:63-64
 *                  (model.reset then sequence.shuffle under use_random_state,
 *                   custom_envs/utils/utils_math.py:9-22)
 *   ce_reset       ConcurrentVecEnv.reset        custom_envs/vectorize/concurrentvecenv.py:109-113
 *                  -> BaseEnvironment.reset       custom_envs/envs/baseenvironment.py:43-49
 *   ce_step        VecEnv.step = step_async+step_wait
 *                                                custom_envs/vectorize/concurrentvecenv.py:97-107
 *                  -> _worker 'step' + auto-reset custom_envs/utils/utils_venv.py:24-56 (:31)
 *                  -> BaseEnvironment.step        custom_envs/envs/baseenvironment.py:30-41
 *                  -> Optimize.base_step          custom_envs/envs/optimize.py:69-100
 *   ce_step_async  ConcurrentVecEnv.step_async   custom_envs/vectorize/concurrentvecenv.py:97-100
 *   ce_wait        ConcurrentVecEnv.step_wait    custom_envs/vectorize/concurrentvecenv.py:102-107
 *   ce_step_many   K consecutive VecEnv.step calls with device-resident actions
 *                  (benchmark / GPU-resident agent mode; one hipGraph)
 *   ce_step_many_prepare
 *                  instantiate + upload that hipGraph without running it (graphs
 *                  are cached per (k, actions, stride, outputs, stream), so a
 *                  timed region never captures)
 *   ce_step_many_strided
 *                  K consecutive VecEnv.step calls in ONE persistent launch
 *                  (concurrentvecenv.py:94-107 x K over optimize.py:69-100 and
 *                  the utils_venv.py:31 auto-reset), step t's outputs into
 *                  record t of a [K] output slab (a device-resident rollout)
 *   ce_set_persistent / ce_step_many_kernel
 *                  choose / name the K-step launch form (no reference analogue)
 *   ce_get_state / ce_set_state
 *                  the per-env attributes model.weights, loss_hist, grad_hist,
 *                  current_step (optimize.py:45-50, baseenvironment.py:18)
 *   ce_destroy     ConcurrentVecEnv.close        custom_envs/vectorize/concurrentvecenv.py:115-125
 *
 * Multi-agent learning-rate path (MultiOptLRs-v0 under OptVecEnv):
 *   ce_multi_create  MultiOptLRs.__init__        custom_envs/envs/multioptlrs.py:39-61
 *                    + OptVecEnv.__init__         custom_envs/vectorize/optvecenv.py:57-68
 *                    + OptimizeFunction.__init__  custom_envs/problems/optimize_function.py:20-61
 *   ce_multi_reset   OptVecEnv.reset              custom_envs/vectorize/optvecenv.py:90-91
 *                    -> MultiOptLRs.base_reset    custom_envs/envs/multioptlrs.py:66-78
 *   ce_multi_step    OptVecEnv.step_async/wait    custom_envs/vectorize/optvecenv.py:70-88
 *                    -> OptEnvRunner.step         custom_envs/vectorize/optvecenv.py:38-46
 *                    -> MultiOptLRs.base_step     custom_envs/envs/multioptlrs.py:80-129
 *   ce_multi_step_async / ce_multi_wait / ce_multi_step_many(_prepare) / ce_multi_host_outputs /
 *   ce_multi_get_state / ce_multi_set_stream / ce_multi_destroy /
 *   ce_multi_step_many_strided / ce_multi_set_persistent / ce_multi_step_many_kernel:
 *                    as for Optimize-v0.
 *
 * MultiOptLRs-v0 over the neural-network problem (get_problem('nn')):
 *   ce_nn_create     MultiOptLRs.__init__(problem='nn')  multioptlrs.py:39-61
 *                    + OptimizeNN.__init__        custom_envs/problems/optimize_nn.py:22-64
 *                      (create_neural_net layers, custom_envs/utils/utils_tf.py:74-86)
 *                    + OptVecEnv.__init__         optvecenv.py:57-68
 *   ce_nn_seed       BaseEnvironment.seed         baseenvironment.py:20-28
 *   ce_nn_seed_draws the reset's kernel init + shuffle and the epoch-end shuffle
 *                    (optimize_nn.py:102-120 under use_random_state)
 *   ce_nn_reset      OptVecEnv.reset -> MultiOptLRs.base_reset  multioptlrs.py:66-78
 *   ce_nn_step       OptVecEnv.step -> MultiOptLRs.base_step    multioptlrs.py:80-129
 *                    (+ OptimizeNN.get_gradient/get/next, optimize_nn.py:102-159)
 *   ce_nn_step_async / ce_nn_wait / ce_nn_step_many(_prepare) / ce_nn_host_outputs /
 *   ce_nn_get_state / ce_nn_set_stream / ce_nn_destroy / ce_nn_n_params:
 *                    as for ce_multi_*.
 *
 * Conventions
 *   - Every function returns CE_OK (0) or a negative ce_status; nothing
 *     throws across the ABI.  ce_last_error() returns a thread-local message.
 *   - The engine owns all device memory (dataset, per-env state).  The caller
 *     owns the buffers it passes in.  With CE_PTR_DEVICE the caller's
 *     pointers are device pointers and the call is stream-ordered
 *     (asynchronous) on the engine stream (ce_set_stream); otherwise they are
 *     host pointers and the call synchronises before returning.
 *   - One engine per host thread; calls on one engine are not re-entrant.
 */
#ifndef CUSTOM_ENVS_AMD_H
#define CUSTOM_ENVS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define CE_ABI_VERSION 5

typedef struct ce_engine ce_engine;

typedef enum ce_status {
    CE_OK = 0,
    CE_EINVAL = -1,      /* bad argument or configuration                 */
    CE_EHIP = -2,        /* HIP runtime error                             */
    CE_ENOMEM = -3,      /* allocation failed                             */
    CE_ESTATE = -4,      /* e.g. step before the first reset              */
    CE_EUNSUPPORTED = -5 /* shape has no compiled kernel instance         */
} ce_status;

typedef enum ce_problem {
    /* softmax classifier without bias (the missing ModelNumpy) */
    CE_PROBLEM_SOFTMAX = 0,
    /* F -> hidden... (relu) -> K softmax network, float32 (OptimizeNN,
       custom_envs/problems/optimize_nn.py:22-64, create_neural_net
       utils_tf.py:74-86); flat parameters
       [W1 | b1 | W2 | b2 | ...] in trainable_variables order; CE_F32 only.
       One hidden layer of 64 with B = 32 runs the fused config-3 kernel;
       every other network (1-4 hidden layers, any widths, any B in 1..N,
       K <= 32) the layered path (net_engine.hip) */
    CE_PROBLEM_MLP = 1
} ce_problem;

typedef enum ce_precision {
    CE_F64 = 0, /* float64 state and arithmetic (the reference's numpy dtype) */
    CE_F32 = 1  /* float32 arithmetic, float64 loss recurrence                 */
} ce_precision;

enum {
    CE_PTR_DEVICE = 1u << 0 /* pointers passed to the call are device pointers */
};

typedef struct ce_config {
    int32_t abi_version; /* CE_ABI_VERSION                                  */
    int32_t problem;     /* ce_problem                                      */
    int32_t precision;   /* ce_precision                                    */
    int32_t device;      /* HIP device ordinal                              */
    int32_t num_envs;    /* E: envs owned by this engine (one rank's shard) */
    int32_t n_rows;      /* N: dataset rows                                 */
    int32_t n_features;  /* F                                               */
    int32_t n_classes;   /* K (targets are one-hot, to_onehot semantics)    */
    int32_t batch_size;  /* B rows per minibatch; B == N for batch_size=None */
    int32_t max_steps;   /* episode length, optimize.py:102-103 (40)        */
    int32_t auto_reset;  /* 1: VecEnv auto-reset on done (utils_venv.py:31);
                            0: single gym.Env (baseenvironment.py:30-41)   */
    int32_t n_hidden;    /* CE_PROBLEM_MLP hidden units of a one-layer
                            network (create_neural_net layers,
                            utils_tf.py:74-86); ignored otherwise          */
    int32_t n_layers;    /* CE_PROBLEM_MLP: 0 = one layer of n_hidden;
                            1..4 = that many hidden layers, widths below   */
    int32_t hidden[4];   /* the hidden widths when n_layers > 0            */
} ce_config;

/* Per-step outputs, one row per env.  obs is [E][2P+1] with P the problem's
   parameter count (F*K for the softmax classifier). */
typedef struct ce_outputs {
    float *obs;        /* concat(wght_hist[idx], loss_hist[idx], grad_hist[idx]) */
    float *reward;     /* -loss (minibatch, after the update)                */
    uint8_t *done;     /* current_step >= max_steps                          */
    float *objective;  /* info['objective']: full-dataset loss               */
    float *accuracy;   /* info['accuracy']                                   */
    int32_t *episode_len; /* info['episode']['l'] (current_step of the step) */
} ce_outputs;

/* Host-side copies of the per-env state (any pointer may be NULL). */
typedef struct ce_state {
    double *weights;      /* [E][P]  model.weights                         */
    double *grad_hist;    /* [E][P]  grad_hist[idx] of the last step       */
    double *loss_hist;    /* [E]     loss_hist[idx] of the last step       */
    int32_t *step;        /* [E]     current_step                          */
    double *init_weights; /* [E][P]  W0 every reset restores               */
    int32_t *order;       /* [E][N]  current row order (B < N only)        */
} ce_state;

int ce_abi_version(void);
const char *ce_last_error(void);
/* Sticky HIP errors an entry point found pending when it started (left by
 * another component, e.g. a caller's aborted stream capture) and cleared so
 * that they are not reported as its own failure: how many so far in this
 * process, and a note naming the last one ("" if none). */
int64_t ce_stale_error_count(void);
const char *ce_stale_error_note(void);

int ce_create(const ce_config *cfg, const double *features /* [N][F] */,
              const int32_t *labels /* [N] class index */, ce_engine **out);
void ce_destroy(ce_engine *eng);

int ce_set_stream(ce_engine *eng, void *hip_stream /* NULL: engine's own */);
/* Compact output form for the per-step all-gather (SURVEY 8e, config 4;
 * replaces nothing in the reference, whose VecEnv np.stacks full obs rows,
 * concurrentvecenv.py:99-104).  When on, every CE_PTR_DEVICE call and
 * ce_step_many writes obs as [E][P + 1] = (loss_hist[idx], grad_hist[idx])
 * only -- the wght_hist block of the observation is identically 0
 * (optimize.py:84-86) and is not stored -- and `done` may be NULL
 * (done == episode_len >= max_steps).  Host-mode calls keep the full form.
 * CE_EUNSUPPORTED unless the engine runs the two-class full-batch float64
 * kernel (ce_step_kernel "optimize_lr_mfma_kernel<...>"). */
int ce_set_compact_outputs(ce_engine *eng, int32_t on);
int ce_num_envs(const ce_engine *eng);
int ce_obs_dim(const ce_engine *eng);
int ce_act_dim(const ce_engine *eng);

/* seeds[i] seeds env i exactly as gym.utils.seeding.np_random(seeds[i]). */
int ce_seed(ce_engine *eng, const uint64_t *seeds, int32_t n);
/* Host-only: the (W0, perm) that every reset of a seed draws.  No GPU. */
int ce_seed_draws(uint64_t seed, int32_t n_features, int32_t n_classes,
                  int32_t n_rows, double *init_weights, int32_t *perm);
/* Host-only, CE_PROBLEM_MLP: glorot-uniform W1 then W2 (float32, zero
   biases, flat order) then the row permutation.  No GPU. */
int ce_seed_draws_mlp(uint64_t seed, int32_t n_features, int32_t n_hidden,
                      int32_t n_classes, int32_t n_rows, float *init_weights,
                      int32_t *perm);

int ce_reset(ce_engine *eng, const ce_outputs *out, uint32_t flags);
int ce_step(ce_engine *eng, const float *actions /* [E][P] */,
            const ce_outputs *out, uint32_t flags);
int ce_step_async(ce_engine *eng, const float *actions, const ce_outputs *out,
                  uint32_t flags);
int ce_wait(ce_engine *eng);
int ce_step_many(ce_engine *eng, int32_t k, const float *actions,
                 int64_t action_step_stride /* elements between steps */,
                 const ce_outputs *out /* device pointers */);
int ce_step_many_prepare(ce_engine *eng, int32_t k, const float *actions,
                         int64_t action_step_stride, const ce_outputs *out);
/* K steps whose outputs are kept: step t reads actions + t * action_step_stride
 * and writes every output of `out` (device pointers) advanced by
 * t * out_step_bytes -- a [K] array of output records, e.g. one buffer per
 * field of [K][E] rows (out_step_bytes = that field's E rows) or one packed
 * record per step.  out_step_bytes == 0 overwrites the same outputs every step
 * (ce_step_many).  Where the engine has a persistent kernel (two-class,
 * B == N, float64, n_rows <= 512: ce_step_many_kernel names it) the K steps
 * are ONE launch: the per-env state stays in registers across them and is
 * stored once; otherwise K step launches.  Stream-ordered, asynchronous.
 * obs must be 16-byte aligned and out_step_bytes a multiple of 16, else
 * CE_EINVAL. */
int ce_step_many_strided(ce_engine *eng, int32_t k, const float *actions,
                         int64_t action_step_stride, const ce_outputs *out,
                         int64_t out_step_bytes);
/* on = 1 (default; CE_PERSIST=0 in the environment at ce_create makes it 0):
 * ce_step_many and ce_step_many_strided use the persistent K-step kernel where
 * the engine has one; on = 0: one launch per step (the A/B form).  With the
 * persistent kernel selected, every K-step entry (ce_step_many, _prepare,
 * _strided) refuses an obs that is not 16-byte aligned with CE_EINVAL: the
 * kernel ce_step_many_kernel names is the one that runs, or none. */
int ce_set_persistent(ce_engine *eng, int32_t on);
/* The kernel ce_step_many runs: "optimize_lr_persist_kernel<NKF,TPW,PAD>" when
 * persistent, else ce_step_kernel's name. */
const char *ce_step_many_kernel(const ce_engine *eng);

/* Pinned host buffers holding the last host-mode outputs (zero-copy views). */
int ce_host_outputs(ce_engine *eng, ce_outputs *view);

/* Name of the step kernel the engine launches (introspection for profiles:
 * "optimize_pair_kernel<double,10,2>", "optimize_step_kernel<...>", ...).
 * Static storage, valid for the engine's lifetime; "" for a null engine. */
const char *ce_step_kernel(const ce_engine *eng);

int ce_get_state(ce_engine *eng, const ce_state *st);
int ce_set_state(ce_engine *eng, const ce_state *st);

/* ------------------------------------------------------------------------
 * MultiOptLRs-v0: one agent per problem parameter picks its learning rate.
 * Rows are (env, agent) in sorted agent-name order ('parameter-0',
 * 'parameter-1', 'parameter-10', ...), as OptVecEnv flattens them.
 */
typedef struct ce_multi_engine ce_multi_engine;

#define CE_MULTI_MAX_PARAMS 64

typedef enum ce_function {
    /* sum of Rosenbrock 100(y - x^2)^2 + (1 - x)^2 over coordinate pairs
       (utils_functions.py:4-6); 2 params = the reference's default problem */
    CE_FUNC_ROSENBROCK_PAIRS = 0
} ce_function;

/* info columns, multioptlrs.py:112-127 ('loss' is NaN when not terminal) */
typedef enum ce_multi_info {
    CE_INFO_LOSS = 0, CE_INFO_BATCH_LOSS, CE_INFO_WEIGHTS_MEAN, CE_INFO_WEIGHTS_SUM,
    CE_INFO_ACTIONS_MEAN, CE_INFO_ACTIONS_STD, CE_INFO_STATES_MEAN, CE_INFO_STATES_SUM,
    CE_INFO_GRADS_MEAN, CE_INFO_GRADS_SUM, CE_INFO_LOSS_MEAN, CE_INFO_ADJUSTED_LOSS,
    CE_INFO_ADJUSTED_GRAD, CE_INFO_GRAD_DIFF, CE_MULTI_INFO
} ce_multi_info;

typedef struct ce_multi_config {
    int32_t abi_version;
    int32_t device;
    int32_t num_envs;     /* E                                               */
    int32_t n_params;     /* P: agents per env = problem dimensions (even)   */
    int32_t function;     /* ce_function                                     */
    int32_t max_history;  /* H, adjusted-history length (multioptlrs.py:39)  */
    int32_t max_batches;  /* episode length (multioptlrs.py:39, default 400) */
    int32_t auto_reset;   /* 1: OptVecEnv auto-reset; 0: single env          */
    float initial_points[CE_MULTI_MAX_PARAMS];
} ce_multi_config;

typedef struct ce_multi_outputs {
    float *obs;           /* [E*P][3H] rows                                  */
    float *reward;        /* [E*P] (replicated per agent, optvecenv.py:43)   */
    uint8_t *done;        /* [E*P]                                           */
    float *info;          /* [E][CE_MULTI_INFO]                              */
    int32_t *episode_len; /* [E] info['episode']['l']                        */
} ce_multi_outputs;

int ce_multi_create(const ce_multi_config *cfg, ce_multi_engine **out);
void ce_multi_destroy(ce_multi_engine *eng);
int ce_multi_set_stream(ce_multi_engine *eng, void *hip_stream);
int ce_multi_reset(ce_multi_engine *eng, const ce_multi_outputs *out, uint32_t flags);
int ce_multi_step(ce_multi_engine *eng, const float *actions /* [E*P] rows */,
                  const ce_multi_outputs *out, uint32_t flags);
int ce_multi_step_async(ce_multi_engine *eng, const float *actions,
                        const ce_multi_outputs *out, uint32_t flags);
int ce_multi_wait(ce_multi_engine *eng);
int ce_multi_step_many(ce_multi_engine *eng, int32_t k, const float *actions,
                       int64_t action_step_stride, const ce_multi_outputs *out);
int ce_multi_step_many_prepare(ce_multi_engine *eng, int32_t k, const float *actions,
                               int64_t action_step_stride, const ce_multi_outputs *out);
/* As ce_step_many_strided: step t writes every output advanced by
 * t * out_step_bytes.  With max_history == 5 (the reference default,
 * multioptlrs.py:39) the K steps are ONE launch of multi_persist_kernel (the
 * state in registers across them); otherwise K step launches. */
int ce_multi_step_many_strided(ce_multi_engine *eng, int32_t k, const float *actions,
                               int64_t action_step_stride, const ce_multi_outputs *out,
                               int64_t out_step_bytes);
/* As ce_set_persistent / ce_step_many_kernel. */
int ce_multi_set_persistent(ce_multi_engine *eng, int32_t on);
const char *ce_multi_step_many_kernel(const ce_multi_engine *eng);
int ce_multi_host_outputs(ce_multi_engine *eng, ce_multi_outputs *view);
/* theta [E][P] (problem parameters in agent order) and current_step [E] */
int ce_multi_get_state(ce_multi_engine *eng, float *theta, int32_t *step);

/* ------------------------------------------------------------------------
 * MultiOptLRs-v0 over OptimizeNN: one agent per network parameter.  The
 * network is F -> hidden[0] -> ... (relu) -> K (softmax), float32, flat
 * parameters in Keras trainable_variables order [W1 | b1 | W2 | b2 | ...].
 * Rows and outputs as for ce_multi_* (ce_multi_outputs).
 */
typedef struct ce_nn_engine ce_nn_engine;

#define CE_NN_MAX_HIDDEN 4

typedef struct ce_nn_config {
    int32_t abi_version;
    int32_t device;
    int32_t num_envs;      /* E                                                 */
    int32_t n_rows;        /* N dataset rows                                    */
    int32_t n_features;    /* F                                                 */
    int32_t n_classes;     /* K (<= 32)                                         */
    int32_t batch_size;    /* B rows per batch (load_data default 32; <= 32)    */
    int32_t n_hidden;      /* hidden layers, 1..CE_NN_MAX_HIDDEN                */
    int32_t hidden[CE_NN_MAX_HIDDEN]; /* units per hidden layer (multiples of 32,
                              <= 512); create_neural_net default (256, 256)    */
    int32_t max_history;   /* H (<= 16)                                         */
    int32_t max_batches;   /* episode length (default 400)                      */
    int32_t auto_reset;    /* 1: OptVecEnv auto-reset; 0: single env            */
} ce_nn_config;

int ce_nn_create(const ce_nn_config *cfg, const float *features /* [N][F] */,
                 const int32_t *labels /* [N] class index */, ce_nn_engine **out);
void ce_nn_destroy(ce_nn_engine *eng);
int ce_nn_set_stream(ce_nn_engine *eng, void *hip_stream);
/* P: parameters (= agents) per env */
int ce_nn_n_params(const ce_nn_engine *eng);
/* seeds[i] seeds env i as gym.utils.seeding.np_random(seeds[i]); must precede
   the first reset */
int ce_nn_seed(ce_nn_engine *eng, const uint64_t *seeds, int32_t n);
/* Host-only: the float32 initial parameters [P], the reset shuffle [N] and
   the epoch-end shuffle [N] of a seed (any output may be NULL).  No GPU. */
int ce_nn_seed_draws(uint64_t seed, int32_t n_dims, const int32_t *dims /* F, hidden..., K */,
                     int32_t n_rows, float *init_weights, int32_t *reset_perm,
                     int32_t *epoch_perm);
int ce_nn_reset(ce_nn_engine *eng, const ce_multi_outputs *out, uint32_t flags);
int ce_nn_step(ce_nn_engine *eng, const float *actions /* [E*P] rows */,
               const ce_multi_outputs *out, uint32_t flags);
int ce_nn_step_async(ce_nn_engine *eng, const float *actions, const ce_multi_outputs *out,
                     uint32_t flags);
int ce_nn_wait(ce_nn_engine *eng);
int ce_nn_step_many(ce_nn_engine *eng, int32_t k, const float *actions,
                    int64_t action_step_stride, const ce_multi_outputs *out);
int ce_nn_step_many_prepare(ce_nn_engine *eng, int32_t k, const float *actions,
                            int64_t action_step_stride, const ce_multi_outputs *out);
int ce_nn_host_outputs(ce_nn_engine *eng, ce_multi_outputs *view);
/* theta [E][P] (agent order), gprev [E][P] (newest raw-history gradient),
   step [E], cursor [E] (batch index in the epoch), order [E][N] (dataset row
   of each current row); any pointer may be NULL */
int ce_nn_get_state(ce_nn_engine *eng, float *theta, float *gprev, int32_t *step,
                    int32_t *cursor, int32_t *order);

#ifdef __cplusplus
}
#endif

#endif /* CUSTOM_ENVS_AMD_H */
