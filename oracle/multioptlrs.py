"""Restatement of MultiOptLRs-v0 and OptVecEnv (TEST INFRASTRUCTURE ONLY).

Follows, line by line:
  custom_envs/envs/multioptlrs.py:39-132      (__init__, base_reset, base_step)
  custom_envs/utils/utils_env.py:9-47,50-68,71-99,102-123,126-164
                                              (obs v3, action space v2, reward
                                               v6, action v0, observation v3)
  custom_envs/utils/utils_common.py:102-196   (History, build_multistate)
  custom_envs/problems/optimize_function.py:20-61,130-137 and
  custom_envs/utils/utils_functions.py:4-6    (Rosenbrock problem)
  custom_envs/vectorize/optvecenv.py:10-91    (flatten_dictionary,
                                               OptEnvRunner, OptVecEnv)

The TF1 problem is restated in float32 numpy in the order TF1's graph and
tf.gradients evaluate it (RosenbrockPairs._eval).  TF itself is absent, so
that order is read off the graph, not run: parity of the float32 problem
values against TF is "unpinned" beyond float32 rounding.  Build-defined
(SURVEY 8d config 5): ``rosenbrock_pairs`` = sum of Rosenbrock over
consecutive coordinate pairs, start [-1.9, 2.0] repeated.
"""
from collections import deque
from itertools import chain, cycle

import numpy as np

from oracle.seeding import np_random

BOUNDS = 1e2
AGENT_FMT = 'parameter-{:d}'


class History:
    """utils_common.py:102-196."""

    def __init__(self, max_history, **named_shapes):
        self.max_history = max_history
        self.shapes = {k: tuple(s) if s else (1,) for k, s in named_shapes.items()}
        self.reset()

    def __getitem__(self, key):
        return np.asarray(list(reversed(self.history[key])))

    def __iter__(self):
        return iter(self.history)

    def keys(self):
        return self.history.keys()

    def reset(self):
        self.history = {k: deque([np.zeros(s)] * self.max_history, maxlen=self.max_history)
                        for k, s in self.shapes.items()}

    def append(self, **named_items):
        assert self.keys() == named_items.keys()
        for name, item in named_items.items():
            self.history[name].append(np.reshape(item, self.shapes[name]))

    def build_multistate(self):
        rows = [self[key].reshape((self.max_history, -1)).tolist() for key in self]
        rows = list(chain.from_iterable(rows))
        rows = [cycle(r) if len(r) == 1 else r for r in rows]
        return list(zip(*rows))


def rosenbrock(x, y):
    """utils_functions.py:4-6."""
    return 100 * (y - x ** 2) ** 2 + (1 - x) ** 2


class RosenbrockPairs:
    """OptimizeFunction (optimize_function.py:20-137) for f = sum of Rosenbrock
    over coordinate pairs, float32 like the TF1 variables."""

    def __init__(self, ndims=2, initial_points=None):
        assert ndims % 2 == 0
        if initial_points is None:
            initial_points = [-1.9, 2.0] * (ndims // 2)
        self.initial = np.asarray(initial_points, dtype=np.float32)
        self.size = ndims
        self.reset()

    def reset(self):
        self.params = self.initial.copy()

    def _eval(self, p):
        """Float32 in TF1's graph order: 100 * pow(d, 2) with pow(d, 2) = d*d,
        pairs summed left to right; gradients as tf.gradients forms them
        (pow grad g*2*x, 100 folded into 200*d, the (1-x) branch -2(1-x))."""
        x, y = p[0::2], p[1::2]
        one, c100, c2, c200 = np.float32(1), np.float32(100), np.float32(2), np.float32(200)
        d = y - x * x
        r = one - x
        terms = c100 * (d * d) + r * r
        loss = np.float32(0)
        for term in terms:
            loss = np.float32(loss + term)
        t = c200 * d
        grad = np.empty_like(p)
        grad[0::2] = -((c2 * t) * x) - c2 * r
        grad[1::2] = t
        return grad, loss

    def get_gradient(self):
        return self._eval(self.params)[0]

    def get_loss(self):
        return self._eval(self.params)[1]

    @property
    def parameters(self):
        return self.params.copy()

    def set_parameters(self, params):
        self.params = np.asarray(params, dtype=np.float32)

    def get(self):
        grad, loss = self._eval(self.params)
        return grad, loss, self.params.copy()

    def next(self):
        pass


def get_observation_v3(history):
    """utils_env.py:126-164, version 3."""
    losses, grads, weights = history['losses'], history['gradients'], history['weights']
    with np.errstate(divide='ignore', invalid='ignore'):
        adj_grad = np.nan_to_num(grads[0] / np.abs(grads[1]))
        adj_wght = np.nan_to_num(weights[0] / np.abs(weights[1]))
        adj_loss = np.nan_to_num(losses[0] / np.abs(losses[1]))
    return float(np.ravel(adj_loss)[0]), adj_wght, adj_grad


class MultiOptLRs:
    """multioptlrs.py:19-138 (version (3, 3, 0, 6))."""

    def __init__(self, ndims=2, initial_points=None, max_batches=400, max_history=5):
        self.random_generator, _ = np_random()
        self.current_step = 0
        self.model = RosenbrockPairs(ndims, initial_points)
        size = self.model.size
        self.history = History(5, losses=(), gradients=(size,), weights=(size,))
        self.adjusted_history = History(max_history, weights=(size,), losses=(),
                                        gradients=(size,))
        self.max_history = max_history
        self.max_batches = max_batches
        self.names = [AGENT_FMT.format(i) for i in range(size)]

    def seed(self, seed=None):
        self.random_generator, _ = np_random(seed)

    def reset(self):
        self.current_step = 0
        self.adjusted_history.reset()
        self.model.reset()
        self.history.reset()
        grad, loss, weight = self.model.get()
        self.history.append(losses=loss, gradients=grad, weights=weight)
        states = self.adjusted_history.build_multistate()
        return {AGENT_FMT.format(i): np.clip(np.nan_to_num(list(v)), -BOUNDS, BOUNDS) - 1
                for i, v in enumerate(states)}

    def step(self, action):
        self.current_step += 1
        state, reward, terminal, info = self.base_step(action)
        info['episode'] = {'r': reward, 'l': self.current_step}
        return state, reward, terminal, info

    def base_step(self, action):
        size = self.model.size
        action = np.reshape([np.asarray(action[AGENT_FMT.format(i)]).ravel()
                             for i in range(size)], (-1,))
        grad = self.model.get_gradient()
        # utils_env.py:113-114: 10 ** (a - 4) in float32.  numpy leaves the
        # float32 pow unpinned (2.x's SIMD loop is 1 ulp off on ~21% of inputs,
        # libm powf is correctly rounded); take the correctly rounded value
        action = (10.0 ** (action - np.float32(4)).astype(np.float64)).astype(np.float32)
        self.model.set_parameters(self.model.parameters - grad * action)
        grad, loss, weights = self.model.get()
        self.history.append(losses=loss, gradients=grad, weights=weights)
        adj_loss, adj_wght, adj_grad = get_observation_v3(self.history)
        self.adjusted_history.append(weights=adj_wght, losses=adj_loss, gradients=adj_grad)
        state = self.adjusted_history.build_multistate()
        states = {AGENT_FMT.format(i): np.clip(np.nan_to_num(list(v)), -BOUNDS, BOUNDS) - 1
                  for i, v in enumerate(state)}
        reward = -(float(adj_loss) - 1)                   # utils_env.py:95-96
        reward = np.clip(reward, -BOUNDS, BOUNDS)
        terminal = self.current_step >= self.max_batches
        if not terminal and loss > 1e4:
            terminal = True
            reward -= (self.max_batches - self.current_step)
        final_loss = self.model.get_loss() if terminal else None
        past_grads = self.history['gradients']
        with np.errstate(invalid='ignore', over='ignore'):
            info = {
                'loss': final_loss,
                'batch_loss': loss,
                'weights_mean': np.mean(np.abs(weights)),
                'weights_sum': np.sum(np.abs(weights)),
                'actions_mean': np.mean(action),
                'actions_std': np.std(action),
                'states_mean': np.mean(np.abs(state)),
                'states_sum': np.sum(np.abs(state)),
                'grads_mean': np.mean(self.history['gradients']),
                'grads_sum': np.sum(self.history['gradients']),
                'loss_mean': np.mean(self.history['losses']),
                'adjusted_loss': float(adj_loss),
                'adjusted_grad': np.mean(np.abs(adj_grad)),
                'grad_diff': np.mean(np.abs(past_grads[0] - past_grads[1])),
            }
        self.model.next()
        return states, reward, terminal, info

    def close(self):
        pass


def flatten_dictionary(dictionary):
    """optvecenv.py:10-14 (values in sorted-name order)."""
    _, values = zip(*sorted(dictionary.items(), key=lambda x: x[0]))
    return values


class OptEnvRunner:
    """optvecenv.py:17-54 (one env's agents as rows)."""

    def __init__(self, environment):
        self._environment = environment
        self._names = sorted(environment.names, key=lambda x: x[0])
        self._num_agents = len(self._names)

    def reset(self):
        return flatten_dictionary(self._environment.reset())

    def step(self, actions):
        actions = {name: a for name, a in zip(sorted(self._names), actions)}
        states, reward, terminal, info = self._environment.step(actions)
        n = self._num_agents
        return flatten_dictionary(states), [reward] * n, [terminal] * n, [info] * n

    def __getattr__(self, attr):                          # optvecenv.py:51-54
        if attr.startswith('_'):
            raise AttributeError(attr)
        return getattr(self._environment, attr)


class OptVecEnv:
    """optvecenv.py:57-91 over the restated ThreadVecEnv (the reference's
    multi-agent vector path; bench.py's config-5 CPU baseline)."""

    def __init__(self, environment_fns):
        from oracle.vectorize import ThreadVecEnv
        self.venv = ThreadVecEnv([_runner_factory(fn) for fn in environment_fns])
        self.agent_no_list = self.venv.get_attr('_num_agents')
        self.num_envs = sum(self.agent_no_list)

    def reset(self):
        return np.concatenate(list(self.venv.reset()))

    def step(self, actions):
        grouped, start = [], 0
        for n in self.agent_no_list:                       # optvecenv.py:70-76
            grouped.append(list(actions[start:start + n]))
            start += n
        states, rewards, dones, infos = self.venv.step(grouped)
        return (np.concatenate(list(states)), np.concatenate(list(rewards)),
                np.concatenate(list(dones)), [i for group in infos for i in group])

    def close(self):
        self.venv.close()


def _runner_factory(fn):
    def make():
        return OptEnvRunner(fn())
    return make
