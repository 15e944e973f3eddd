"""MultiOptLRs-v0 over the OptimizeNN problem (TEST INFRASTRUCTURE ONLY).

Float32 numpy restatement of the neural-network problem that
``get_problem('nn')`` builds (custom_envs/problems/__init__.py:7-16), as the
MultiOptLRs env drives it (custom_envs/envs/multioptlrs.py:39-129):

  OptimizeNN.__init__          problems/optimize_nn.py:22-64
    network                    create_neural_net(layers=(256, 256), 'relu')
                               (utils/utils_tf.py:74-86) + Dense(K, softmax)
    loss                       keras categorical_crossentropy per sample,
                               reduce_mean for the reported loss (:46-52)
    gradient                   tf.gradients of the per-sample loss vector =
                               d(sum_i CE_i)/dtheta, flattened in
                               trainable_variables order [W1, b1, W2, b2, ...]
                               (utils_common.flatten_arrays)
  OptimizeNN.next              :102-112 (batch cycling; on_epoch_end reshuffles)
  OptimizeNN.reset             :114-120 (variables re-initialised, iterator
                               emptied, next() -> on_epoch_end)
  InMemoryDataSet + keras Sequence iteration
                               dataset/inmemorydataset.py:8-38 (ragged last
                               batch), Sequence.__iter__ = self[i] for i in
                               range(len(self))
  BaseEnvironment.step/reset under use_random_state
                               envs/baseenvironment.py:30-49,
                               utils/utils_math.py:9-22

TensorFlow is absent from this image, so two pieces are build-defined and
the float32 values are "parity unpinned" against TF itself:
  * initialisation: Keras draws glorot-uniform kernels from TF's RNG (not
    reproducible, and separate from numpy's); here each kernel is
    ``uniform(-l, l)`` with l = sqrt(6 / (fan_in + fan_out)), kernels in
    layer order, zero biases, rounded to float32 -- the same rule as the
    config-3 MLP (oracle/optimize.py ModelMLP) -- drawn from a stand-in for
    TF's RNG: a RandomState started at the env RNG's seeded state.  Like
    TF's, it does not advance the global npr, so the reset's shuffle
    (next() -> on_epoch_end, optimize_nn.py:102-120) is the first draw of
    the fresh env stream, the same permutation as every epoch end;
  * the loss: tf.keras (>= 1.13) routes categorical_crossentropy of a
    Softmax output through softmax_cross_entropy_with_logits on the logits:
    CE_i = log(sum_k exp(z_ik - m_i)) - (z_iy - m_i), dCE/dz = softmax - y.
Because use_random_state hands the step a fresh copy of the env RNG, every
epoch-end reshuffle inside a step draws the same permutation (the first
legacy shuffle of arange(N) from the seed), and so does every reset: the
permutation is fixed per seed, and the row order composes it at every reset
and every epoch end.
"""
import numpy as np
import numpy.random as npr

from oracle.multioptlrs import MultiOptLRs
from oracle.optimize import InMemoryDataSet, use_random_state
from oracle.seeding import np_random


class SequenceDataSet(InMemoryDataSet):
    """InMemoryDataSet with keras Sequence iteration (dataset.py:11 base)."""

    def __iter__(self):
        return (self[i] for i in range(len(self)))


class OptimizeNN:
    """problems/optimize_nn.py:19-159 in float32 numpy."""

    def __init__(self, features, targets, hidden=(256, 256), batch_size=32):
        self.data_set = SequenceDataSet(np.asarray(features, np.float32),
                                        np.asarray(targets, np.float32), batch_size)
        F, K = self.data_set.feature_shape[0], self.data_set.target_shape[0]
        self.dims = (F,) + tuple(int(h) for h in hidden) + (K,)
        self.shapes = []
        for a, b in zip(self.dims[:-1], self.dims[1:]):
            self.shapes += [(a, b), (b,)]
        self.size = int(sum(np.prod(s) for s in self.shapes))
        self.params = np.zeros(self.size, np.float32)
        self.data_set_iter = iter(())
        self.current_batch = None

    # --- BaseProblem surface used by MultiOptLRs ------------------------------
    def reset(self):
        """:114-120 under the env's use_random_state (build-defined init from
        the TF-RNG stand-in; the global npr is not advanced)."""
        tf_rng = np.random.RandomState()
        tf_rng.set_state(npr.get_state())
        parts = []
        for a, b in zip(self.dims[:-1], self.dims[1:]):
            limit = np.sqrt(6.0 / (a + b))
            parts.append(tf_rng.uniform(-limit, limit, (a, b)).ravel())
            parts.append(np.zeros(b))
        self.params = np.concatenate(parts).astype(np.float32)
        self.data_set_iter = iter(())
        self.next()

    def next(self):
        """:102-112."""
        try:
            batch = next(self.data_set_iter)
        except StopIteration:
            self.data_set.on_epoch_end()
            self.data_set_iter = iter(self.data_set)
            batch = next(self.data_set_iter)
        self.current_batch = batch

    @property
    def parameters(self):
        return self.params.copy()

    def set_parameters(self, params):
        self.params = np.asarray(params, np.float32).reshape(-1)

    def unflatten(self, params=None):
        params = self.params if params is None else params
        out, start = [], 0
        for shape in self.shapes:
            n = int(np.prod(shape))
            out.append(params[start:start + n].reshape(shape))
            start += n
        return out

    def evaluate(self, params=None, batch=None):
        """(flat float32 gradient of sum_i CE_i, float32 mean CE) on a batch."""
        features, targets = self.current_batch if batch is None else batch
        tensors = self.unflatten(params)
        weights, biases = tensors[0::2], tensors[1::2]
        acts, zs = [features], []
        h = features
        for w, b in zip(weights[:-1], biases[:-1]):
            z = h @ w + b
            zs.append(z)
            h = np.maximum(z, np.float32(0))
            acts.append(h)
        logits = h @ weights[-1] + biases[-1]
        shifted = logits - np.max(logits, axis=1, keepdims=True)
        e = np.exp(shifted)
        se = np.sum(e, axis=1, keepdims=True)
        ce = np.log(se)[:, 0] - np.sum(shifted * targets, axis=1)
        loss = np.float32(np.mean(ce, dtype=np.float32))
        d = e / se - targets
        grads = [None] * len(tensors)
        for layer in range(len(weights) - 1, -1, -1):
            grads[2 * layer] = acts[layer].T @ d
            grads[2 * layer + 1] = np.sum(d, axis=0)
            if layer:
                d = (d @ weights[layer].T) * (zs[layer - 1] > 0)
        grad = np.concatenate([g.ravel() for g in grads]).astype(np.float32)
        return grad, loss

    def get_gradient(self):
        return self.evaluate()[0]

    def get_loss(self):
        return self.evaluate()[1]

    def get(self):
        grad, loss = self.evaluate()
        return grad, loss, self.params.copy()


class MultiOptLRsNN(MultiOptLRs):
    """MultiOptLRs(problem='nn') with BaseEnvironment's use_random_state
    around reset and step (baseenvironment.py:30-49)."""

    def __init__(self, features, targets, hidden=(256, 256), batch_size=32,
                 max_batches=400, max_history=5):
        super().__init__(ndims=2, max_batches=max_batches, max_history=max_history)
        from oracle.multioptlrs import AGENT_FMT, History
        self.model = OptimizeNN(features, targets, hidden, batch_size)
        size = self.model.size
        self.history = History(5, losses=(), gradients=(size,), weights=(size,))
        self.adjusted_history = History(max_history, weights=(size,), losses=(),
                                        gradients=(size,))
        self.names = [AGENT_FMT.format(i) for i in range(size)]

    def reset(self):
        with use_random_state(self.random_generator):
            return super().reset()

    def step(self, action):
        self.current_step += 1
        with use_random_state(self.random_generator):
            state, reward, terminal, info = self.base_step(action)
        info['episode'] = {'r': reward, 'l': self.current_step}
        return state, reward, terminal, info

    def order(self):
        """Dataset-row index of every current row (composed shuffles)."""
        return self.model.data_set.order.copy()


def nn_draws(seed, dims, n_rows):
    """(theta0, reset_perm, epoch_perm) of an env seeded with ``seed``: the
    kernels (TF-RNG stand-in), the shuffle of every reset and the shuffle of
    every epoch end inside a step.  The two shuffles are both the first draw
    of the never-advanced env RandomState, so they are equal."""
    rng, _ = np_random(seed)
    parts = []
    for a, b in zip(dims[:-1], dims[1:]):
        limit = np.sqrt(6.0 / (a + b))
        parts.append(rng.uniform(-limit, limit, (a, b)).ravel())
        parts.append(np.zeros(b))
    rng, _ = np_random(seed)
    reset_perm = np.arange(n_rows)
    rng.shuffle(reset_perm)
    rng, _ = np_random(seed)
    epoch_perm = np.arange(n_rows)
    rng.shuffle(epoch_perm)
    return np.concatenate(parts).astype(np.float32), reset_perm, epoch_perm
