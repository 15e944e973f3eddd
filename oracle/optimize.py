"""Float64 numpy restatement of Optimize-v0 (TEST INFRASTRUCTURE ONLY).

Follows, line by line:
  custom_envs/envs/baseenvironment.py:16-49   (current_step, seed, step, reset)
  custom_envs/envs/optimize.py:40-103         (__init__, base_reset, base_step,
                                               _terminal)
  custom_envs/utils/utils_math.py:9-22,25-34,51-63
                                              (use_random_state, cross_entropy,
                                               softmax)
  custom_envs/utils/utils_common.py:12-23     (shuffle on the global npr)
  custom_envs/dataset/inmemorydataset.py:8-38 (InMemoryDataSet)

Build-defined pieces (the reference does not ship them):
  A7  ``custom_envs.models.ModelNumpy`` -- softmax classifier without bias,
      W of shape (F, K); ``reset`` draws ``npr.normal(size=(F, K))`` from the
      global RandomState (precedent: envs/optimizesign.py:131);
      ``compute_backprop`` returns the mean cross-entropy, the *summed*
      gradient X^T (P - Y) (the env divides by B at optimize.py:78) and the
      accuracy ``mean(argmax P == argmax Y)``.
  A9  ``sequence.shuffle`` == ``on_epoch_end``; ``label_shape`` ==
      ``target_shape``; ``labels`` == ``targets``.
  A12 ``model='mlp'`` (config 3): the Optimize env over a float32 MLP
      F -> hidden (relu) -> K (softmax), the OptimizeNN network
      (problems/optimize_nn.py:35-52, utils_tf.py:74-86) in numpy.  Flat
      parameters in Keras ``trainable_variables`` order [W1 (F,H) row-major,
      b1, W2 (H,K), b2] (utils_common.flatten_arrays); ``reset`` draws
      glorot-uniform W1 then W2 from the global RandomState
      (``uniform(-l, l)``, l = sqrt(6 / (fan_in + fan_out)), cast to
      float32), zero biases; ``compute_backprop`` returns the float32 mean
      cross-entropy (the ModelNumpy form ``-log(P + 1e-16)``), the summed
      gradient (tf.gradients of the per-sample loss vector, optimize_nn.py:
      48-52) and the accuracy.  The env's histories stay float64 (np.zeros).

The oracle also records ``order``: the dataset-row index of every current
row, composed exactly as ``on_epoch_end`` composes permutations, so tests can
compare the engine's minibatch indices bit for bit.
"""
from contextlib import contextmanager

import numpy as np
import numpy.random as npr

from oracle.seeding import np_random


@contextmanager
def use_random_state(random_state):
    """utils_math.py:9-22 -- run under a *copy* of the env RNG state."""
    saved = npr.get_state()
    try:
        npr.set_state(random_state.get_state())
        yield random_state
    finally:
        npr.set_state(saved)


def softmax(logits):
    """utils_math.py:51-63 (numexpr exp replaced by np.exp)."""
    shifted = np.exp(logits - np.max(logits, axis=1)[:, None])
    return shifted / np.sum(shifted, axis=1)[:, None]


def cross_entropy(prob, ground_truth):
    """utils_math.py:25-34."""
    return np.mean(np.sum(-np.log(prob + 1e-16) * ground_truth, axis=1))


def shuffle(*arrays):
    """utils_common.py:12-23 with the default (global) ``np_random=npr``."""
    index = np.arange(len(arrays[0]))
    npr.shuffle(index)
    return [arr[index] for arr in arrays]


class InMemoryDataSet:
    """inmemorydataset.py:8-38 plus the A9 shims used by optimize.py."""

    def __init__(self, features, targets, batch_size=None):
        assert len(features) == len(targets)
        self.features = features
        self.targets = targets
        self.order = np.arange(len(features))
        self.batch_size = len(features) if batch_size is None else batch_size

    def on_epoch_end(self):
        self.features, self.targets, self.order = shuffle(
            self.features, self.targets, self.order)

    shuffle = on_epoch_end

    def __len__(self):
        return -(-len(self.features) // self.batch_size)

    def __getitem__(self, idx):
        begin = idx * self.batch_size
        end = begin + self.batch_size
        rows = slice(begin, end if idx < len(self) else None)
        return self.features[rows], self.targets[rows]

    @property
    def feature_shape(self):
        return self.features.shape[1:]

    @property
    def target_shape(self):
        return self.targets.shape[1:]

    label_shape = target_shape

    @property
    def labels(self):
        return self.targets


class ModelNumpy:
    """Build-defined stand-in for the missing custom_envs.models.ModelNumpy."""

    def __init__(self, feature_size, num_of_labels):
        self.shape = (feature_size, num_of_labels)
        self.weights = np.zeros(self.shape)

    @property
    def size(self):
        return self.shape[0] * self.shape[1]

    def reset(self):
        self.weights = npr.normal(size=self.shape)

    def set_weights(self, weights):
        self.weights = weights

    def compute_backprop(self, features, labels):
        prob = softmax(features @ self.weights)
        loss = cross_entropy(prob, labels)
        grad = features.T @ (prob - labels)
        accuracy = np.mean(np.argmax(prob, axis=1) == np.argmax(labels, axis=1))
        return loss, grad, accuracy


class ModelMLP:
    """A12: float32 F -> hidden... (relu) -> K (softmax) classifier, flat
    params [W1 | b1 | W2 | b2 | ...] in trainable_variables order
    (optimize_nn.py:22-64, create_neural_net utils_tf.py:74-86).  ``hidden``:
    one width (config 3: 64) or a tuple of widths (the reference default
    (256, 256))."""

    def __init__(self, feature_size, num_of_labels, hidden=64):
        hidden = (int(hidden),) if np.isscalar(hidden) else tuple(int(h) for h in hidden)
        self.dims = (feature_size,) + hidden + (num_of_labels,)
        shapes = []
        for fan_in, fan_out in zip(self.dims[:-1], self.dims[1:]):
            shapes += [(fan_in, fan_out), (fan_out,)]
        self.shapes = tuple(shapes)
        self.size = int(sum(np.prod(s) for s in self.shapes))
        self.weights = np.zeros(self.size, np.float32)

    def reset(self):
        """glorot-uniform kernels layer by layer from the global npr, zero biases."""
        parts = []
        for fan_in, fan_out in zip(self.dims[:-1], self.dims[1:]):
            lim = np.sqrt(6.0 / (fan_in + fan_out))
            parts += [npr.uniform(-lim, lim, (fan_in, fan_out)).ravel(), np.zeros(fan_out)]
        self.weights = np.concatenate(parts).astype(np.float32)

    def set_weights(self, weights):
        self.weights = np.asarray(weights, np.float32).reshape(-1)

    def unflatten(self):
        out, start = [], 0
        for shape in self.shapes:
            n = int(np.prod(shape))
            out.append(self.weights[start:start + n].reshape(shape))
            start += n
        return out

    def compute_backprop(self, features, labels):
        params = self.unflatten()
        kernels, biases = params[0::2], params[1::2]
        acts, pre = [features], []
        for w, b in zip(kernels[:-1], biases[:-1]):
            z = acts[-1] @ w + b
            pre.append(z)
            acts.append(np.maximum(z, np.float32(0)))
        prob = softmax(acts[-1] @ kernels[-1] + biases[-1])
        loss = cross_entropy(prob, labels)
        dz = prob - labels
        grads = []
        for layer in range(len(kernels) - 1, -1, -1):
            grads = [(acts[layer].T @ dz).ravel(), dz.sum(axis=0)] + grads
            if layer > 0:
                dz = (dz @ kernels[layer].T) * (pre[layer - 1] > 0)
        accuracy = np.mean(np.argmax(prob, axis=1) == np.argmax(labels, axis=1))
        return loss, np.concatenate(grads), accuracy


class Optimize:
    """optimize.py:14-109 over baseenvironment.py:11-57."""

    def __init__(self, features, targets, batch_size=None, max_steps=40, model='linear',
                 hidden=64):
        # BaseEnvironment.__init__ (:16-18)
        self.random_generator, _ = np_random()
        self.current_step = 0
        # Optimize.__init__ (:40-56); load_data replaced by explicit arrays
        if model == 'mlp':              # the TF feed is float32 (optimize_nn.py:35-36)
            features = np.asarray(features, np.float32)
            targets = np.asarray(targets, np.float32)
        self.sequence = InMemoryDataSet(features, targets, batch_size)
        num_of_labels = self.sequence.label_shape[0]
        feature_size = self.sequence.feature_shape[0]
        if model == 'mlp':
            self.model = ModelMLP(feature_size, num_of_labels, hidden)
            hist_shape = (3, self.model.size)
        else:
            self.model = ModelNumpy(feature_size, num_of_labels)
            hist_shape = (3, feature_size, num_of_labels)
        self.loss_hist = np.zeros((3, 1))
        self.grad_hist = np.zeros(hist_shape)
        self.wght_hist = np.zeros(self.grad_hist.shape)
        self.obs_size = 2 * self.model.size + 1
        self.max_steps = max_steps
        self.seed()

    # --- BaseEnvironment --------------------------------------------------
    def seed(self, seed=None):
        self.random_generator, _ = np_random(seed)

    def step(self, action):
        self.current_step += 1
        with use_random_state(self.random_generator):
            state, reward, terminal, info = self.base_step(action)
        info['episode'] = {'r': reward, 'l': self.current_step}
        return state, reward, terminal, info

    def reset(self):
        self.current_step = 0
        with use_random_state(self.random_generator):
            return self.base_reset()

    # --- Optimize -----------------------------------------------------------
    def base_reset(self):
        self.loss_hist.fill(0)
        self.grad_hist.fill(0)
        self.wght_hist.fill(0)
        self.model.reset()
        self.sequence.shuffle()
        return np.concatenate([self.wght_hist[0].ravel(),
                               self.loss_hist[0].ravel(),
                               self.grad_hist[0].ravel()])

    def base_step(self, action):
        idx = self.current_step % len(self.loss_hist)
        features, labels = self.sequence[0]
        self.model.set_weights(self.model.weights -
                               action.reshape((-1, self.wght_hist.shape[-1])))
        loss, grad, _ = self.model.compute_backprop(features, labels)
        grad = grad / len(features)
        np.divide(loss - self.loss_hist[idx - 1],
                  self.loss_hist[idx - 1] + 0.1, out=self.loss_hist[idx])
        np.divide(grad, np.abs(self.grad_hist[idx - 1]) + 1,
                  out=self.grad_hist[idx])
        np.divide(np.abs(self.wght_hist[idx - 1] - self.wght_hist[idx - 2]),
                  np.abs(self.wght_hist[idx] - self.wght_hist[idx - 1]) + 0.1,
                  out=self.wght_hist[idx])
        state = np.concatenate([self.wght_hist[idx].ravel(),
                                self.loss_hist[idx].ravel(),
                                self.grad_hist[idx].ravel()])
        reward = -loss
        terminal = self._terminal()
        objective, _, accuracy = self.model.compute_backprop(
            self.sequence.features, self.sequence.labels)
        info = {'objective': objective, 'accuracy': accuracy}
        return state, reward, terminal, info

    def _terminal(self):
        return self.current_step >= self.max_steps

    def render(self, mode='human'):
        pass

    def close(self):
        pass


def initial_draws_mlp(seed, n_features, hidden, n_classes, n_rows):
    """(W0 flat float32, perm) of the A12 MLP: glorot-uniform kernels layer by
    layer, zero biases, then shuffle(arange(N)), all from the env's (never
    advanced) RandomState.  ``hidden``: a width or a tuple of widths."""
    rng, _ = np_random(seed)
    hidden = (int(hidden),) if np.isscalar(hidden) else tuple(int(h) for h in hidden)
    dims = (n_features,) + hidden + (n_classes,)
    parts = []
    for fan_in, fan_out in zip(dims[:-1], dims[1:]):
        lim = np.sqrt(6.0 / (fan_in + fan_out))
        parts += [rng.uniform(-lim, lim, (fan_in, fan_out)).ravel(), np.zeros(fan_out)]
    perm = np.arange(n_rows)
    rng.shuffle(perm)
    return np.concatenate(parts).astype(np.float32), perm


def initial_draws(seed, n_features, n_classes, n_rows):
    """(W0, perm) that every reset of an env seeded with ``seed`` draws.

    ``use_random_state`` never advances the env RNG, so each reset replays
    the same stream: ``normal(size=(F, K))`` then ``shuffle(arange(N))``.
    """
    rng, _ = np_random(seed)
    weights = rng.normal(size=(n_features, n_classes))
    perm = np.arange(n_rows)
    rng.shuffle(perm)
    return weights, perm
