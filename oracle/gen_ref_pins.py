"""Golden fixtures produced by the REFERENCE's own code (run in this container).

    python -m oracle.gen_ref_pins        # -> tests/golden/ref_*.npz

TEST INFRASTRUCTURE ONLY.  oracle/refexec.py compiles the named definitions
from the reference's source files; this script fills their module globals
and rolls them out.  What runs from the reference (file: definitions):

  custom_envs/envs/optimize.py           Optimize (__init__, base_reset,
                                         base_step, _terminal)
  custom_envs/envs/baseenvironment.py    BaseEnvironment, BaseMultiEnvironment
  custom_envs/envs/multioptlrs.py        VersionType, BOUNDS, MultiOptLRs
  custom_envs/utils/utils_math.py        use_random_state
  custom_envs/utils/utils_common.py      shuffle, History
  custom_envs/utils/utils_env.py         get_obs_version, get_action_space_optlrs,
                                         get_reward, get_action_optlrs,
                                         get_observation
  custom_envs/utils/utils_functions.py   compute_rosenbrock (its formula)
  custom_envs/dataset/inmemorydataset.py InMemoryDataSet
  custom_envs/utils/utils_venv.py        _worker  (``if done:`` auto-reset, Optimize-v0)
  custom_envs/vectorize/concurrentvecenv.py
                                         _worker  (``if any(done):``, OptVecEnv)
  custom_envs/vectorize/optvecenv.py     flatten_dictionary, OptEnvRunner
  custom_envs/data/load_data.py          load_mnist, load_data (the 'mnist' and
                                         'mnist-test' branches, over synthetic
                                         IDX .xz files this script writes)
  custom_envs/utils/utils_image.py       resize_array, resize_array_many (PIL)
  custom_envs/utils/utils_common.py      to_onehot

What the namespaces supply instead of the modules the reference imports
(absent here, or missing from the reference itself):
  gym.Env -> object; gym.spaces.Box/Dict -> custom_envs_amd.spaces;
  gym.utils.seeding.np_random -> oracle.seeding.np_random (gym's published
  algorithm; seed -> stream parity stays unpinned, gym is absent);
  custom_envs.models.ModelNumpy (MISSING from the reference) ->
  oracle.optimize.ModelNumpy, the build-defined A7 model;
  load_data(name, batch_size) -> the fixture data set in the reference's
  InMemoryDataSet, plus the A9 shims the reference's Optimize calls
  (shuffle = on_epoch_end, label_shape = target_shape, labels = targets);
  DataSet (a keras Sequence) -> object;
  utils_math.normalize (numexpr is absent) -> the same expression in numpy;
  load_data's ``__file__`` -> a directory holding the synthetic IDX files;
  get_problem('func'|'func4') -> oracle.multioptlrs.RosenbrockPairs, whose
  float32 evaluation order restates the TF1 graph (TF is absent) and whose
  loss is checked against the reference's compute_rosenbrock here.
So these fixtures pin the env / dataset / vectorize logic to the reference's
own code; the model arithmetic inside stays the build-defined A7 / TF
restatement.
"""
import math
import os
import threading
from abc import abstractmethod
from collections import deque, namedtuple
from collections.abc import Mapping
from contextlib import contextmanager
from itertools import chain, cycle
from multiprocessing import Pipe
from types import SimpleNamespace

import numpy as np
import numpy.random as npr

from oracle.refexec import load

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, os.pardir, 'tests', 'golden')


def _spaces():
    from custom_envs_amd.spaces import Box, Dict
    return Box, Dict


def reference_modules():
    """Namespaces holding the reference's definitions (see module doc)."""
    from oracle.seeding import np_random
    Box, Dict = _spaces()
    math_ns = load('custom_envs/utils/utils_math.py', ['use_random_state'],
                   {'np': np, 'npr': npr, 'contextmanager': contextmanager})
    common = load('custom_envs/utils/utils_common.py', ['shuffle', 'History'],
                  {'np': np, 'npr': npr, 'deque': deque, 'Mapping': Mapping, 'chain': chain,
                   'cycle': cycle})
    funcs = load('custom_envs/utils/utils_functions.py', ['compute_rosenbrock'], {})
    env_ns = load('custom_envs/utils/utils_env.py',
                  ['get_obs_version', 'get_action_space_optlrs', 'get_reward',
                   'get_action_optlrs', 'get_observation'],
                  {'np': np, 'Box': Box, 'History': common['History']})
    ds = load('custom_envs/dataset/inmemorydataset.py', ['InMemoryDataSet'],
              {'DataSet': object, 'math': math, 'shuffle': common['shuffle'],
               'BatchType': namedtuple('BatchType', ['features', 'labels'])})
    base = load('custom_envs/envs/baseenvironment.py',
                ['BaseEnvironment', 'BaseMultiEnvironment'],
                {'Env': object, 'np_random': np_random, 'abstractmethod': abstractmethod,
                 'use_random_state': math_ns['use_random_state']})
    venv = load('custom_envs/utils/utils_venv.py', ['_worker'], {'np': np})
    cvenv = load('custom_envs/vectorize/concurrentvecenv.py', ['_worker'], {'np': np})
    optv = load('custom_envs/vectorize/optvecenv.py', ['flatten_dictionary', 'OptEnvRunner'],
                {'np': np})
    return SimpleNamespace(math=math_ns, common=common, funcs=funcs, env=env_ns, ds=ds,
                           base=base, venv=venv, cvenv=cvenv, optv=optv)


def reference_optimize(mods, features, targets, batch_size):
    """The reference's Optimize class over the A7 model and the fixture set."""
    from oracle.optimize import ModelNumpy
    Box, _ = _spaces()
    Base = mods.ds['InMemoryDataSet']

    class FixtureDataSet(Base):
        """The reference's InMemoryDataSet + the A9 shims Optimize calls."""
        shuffle = Base.on_epoch_end
        label_shape = Base.target_shape

        @property
        def labels(self):
            return self.targets

    ns = load('custom_envs/envs/optimize.py', ['Optimize'],
              {'np': np, 'npr': npr, 'Box': Box, 'Model': ModelNumpy,
               'BaseEnvironment': mods.base['BaseEnvironment'],
               'load_data': lambda name, bs: FixtureDataSet(features.copy(), targets.copy(), bs)})
    return ns['Optimize'](data_set='fixture', batch_size=batch_size)


class WorkerEnv:
    """One env served by a reference ``_worker`` loop on a thread over a Pipe
    (the reference's VecEnv worker, including its auto-reset)."""

    def __init__(self, worker, env):
        self.env = env
        self.remote, child = Pipe(True)
        self.thread = threading.Thread(target=worker,
                                       args=(child, SimpleNamespace(var=lambda: env)),
                                       daemon=True)
        self.thread.start()

    def call(self, cmd, data=None):
        self.remote.send((cmd, data))
        return self.remote.recv()

    def close(self):
        self.remote.send(('close', None))
        self.thread.join()


def rollout_optimize(mods, features, targets, seed, batch_size, steps, action_seed):
    env = reference_optimize(mods, features, targets, batch_size)
    env.seed(seed)
    worker = WorkerEnv(mods.venv['_worker'], env)
    P = env.model.size
    actions = np.random.RandomState(action_seed).normal(0, 0.01, (steps, P)).astype(np.float32)
    first = worker.call('reset')
    rec = {k: [] for k in ('obs', 'reward', 'done', 'objective', 'accuracy', 'ep_len',
                           'weights')}
    for t in range(steps):
        obs, reward, done, info = worker.call('step', actions[t])
        rec['obs'].append(obs)
        rec['reward'].append(reward)
        rec['done'].append(done)
        rec['objective'].append(info['objective'])
        rec['accuracy'].append(info['accuracy'])
        rec['ep_len'].append(info['episode']['l'])
        rec['weights'].append(env.model.weights.ravel().copy())
    worker.close()
    out = {k: np.array(v) for k, v in rec.items()}
    out.update(actions=actions, reset_obs=first, seed=np.array(seed),
               batch_size=np.array(-1 if batch_size is None else batch_size))
    return out


def reference_multioptlrs(mods, ndims, max_batches, max_history):
    from oracle.multioptlrs import RosenbrockPairs
    _, Dict = _spaces()

    def get_problem(name='func', **kwargs):
        problem = RosenbrockPairs({'func': 2, 'func4': 4}[name])
        # the restated float32 problem evaluates the reference's formula
        x = problem.params.astype(np.float64)
        ref = sum(mods.funcs['compute_rosenbrock'](x[i], x[i + 1]) for i in range(0, ndims, 2))
        assert abs(float(problem.get_loss()) - ref) <= 1e-6 * abs(ref)
        return problem

    ns = load('custom_envs/envs/multioptlrs.py', ['VersionType', 'BOUNDS', 'MultiOptLRs'],
              {'np': np, 'Dict': Dict, 'namedtuple': namedtuple, 'History': mods.common['History'],
               'utils_env': SimpleNamespace(**{k: v for k, v in mods.env.items()
                                               if k.startswith('get_')}),
               'BaseMultiEnvironment': mods.base['BaseMultiEnvironment'],
               'get_problem': get_problem})
    return ns['MultiOptLRs'](problem={2: 'func', 4: 'func4'}[ndims], max_batches=max_batches,
                             max_history=max_history)


INFO_KEYS = ('loss', 'batch_loss', 'weights_mean', 'weights_sum', 'actions_mean',
             'actions_std', 'states_mean', 'states_sum', 'grads_mean', 'grads_sum',
             'loss_mean', 'adjusted_loss', 'adjusted_grad', 'grad_diff')


def rollout_multi(mods, ndims, max_batches, max_history, steps, action_seed, low, high):
    env = reference_multioptlrs(mods, ndims, max_batches, max_history)
    runner = mods.optv['OptEnvRunner'](lambda: env)
    worker = WorkerEnv(mods.cvenv['_worker'], runner)
    actions = np.random.RandomState(action_seed).uniform(low, high, (steps, ndims, 1)).astype(
        np.float32)
    first = np.stack(worker.call('reset'))
    rec = {k: [] for k in ('obs', 'reward', 'done', 'info', 'ep_len', 'theta')}
    with np.errstate(divide='ignore', invalid='ignore', over='ignore'):
        for t in range(steps):
            states, rewards, dones, infos = worker.call('step', list(actions[t]))
            info = infos[0]
            rec['obs'].append(np.stack(states))
            rec['reward'].append(rewards[0])
            rec['done'].append(dones[0])
            rec['ep_len'].append(info['episode']['l'])
            rec['info'].append([np.nan if info[k] is None else float(info[k])
                                for k in INFO_KEYS])
            rec['theta'].append(env.model.params.copy())
    worker.close()
    out = {k: np.array(v) for k, v in rec.items()}
    out.update(actions=actions, reset_obs=first)
    return out


def utils_env_vectors(mods, rng):
    """Known-answer vectors of utils_env's numeric functions, every version."""
    History = mods.common['History']
    vec = {}
    for version in range(4):
        hist = History(3, weights=(6,), losses=(), gradients=(6,))
        for _ in range(3):
            w = rng.normal(size=6)
            g = rng.normal(size=6)
            g[0] = 0.0                   # a zero denominator (nan_to_num paths)
            hist.append(weights=w, losses=abs(rng.normal()), gradients=g)
        with np.errstate(divide='ignore', invalid='ignore'):
            loss, wght, grad = mods.env['get_observation'](hist, version)
        vec['obs_in_w_v%d' % version] = hist['weights']
        vec['obs_in_l_v%d' % version] = hist['losses']
        vec['obs_in_g_v%d' % version] = hist['gradients']
        vec['obs_loss_v%d' % version] = np.array(loss)
        vec['obs_wght_v%d' % version] = np.asarray(wght)
        vec['obs_grad_v%d' % version] = np.asarray(grad)
    losses = np.abs(rng.normal(size=7)) + 0.1
    adjusted = rng.normal(size=7)
    vec['reward_loss'], vec['reward_adjusted'] = losses, adjusted
    vec['reward'] = np.array([[mods.env['get_reward'](lv, av, version) for lv, av in
                               zip(losses, adjusted)] for version in range(7)])
    acts = rng.uniform(-4, 6, 9).astype(np.float32)
    vec['action_in'] = acts
    vec['action'] = np.stack([np.asarray(mods.env['get_action_optlrs'](acts, version),
                                         dtype=np.float64) for version in range(4)])
    return vec


IDX_DIR = os.path.join(GOLDEN, 'idx')


def synthetic_digits(n, seed):
    """uint8 28x28 'digit' images: one smooth blob per class at a class-
    dependent position (compresses well; the pixels are not MNIST's)."""
    rs = np.random.RandomState(seed)
    labels = rs.randint(0, 10, n).astype(np.uint8)
    yy, xx = np.mgrid[0:28, 0:28]
    images = np.zeros((n, 28, 28), np.uint8)
    for i, y in enumerate(labels.astype(int)):
        cy, cx = 6 + 2 * (y % 5) + rs.randint(-2, 3), 7 + 3 * (y // 5) + rs.randint(-2, 3)
        r2 = ((yy - cy) ** 2 + (xx - cx) ** 2) / (2.0 * (2.0 + (y % 3)) ** 2)
        images[i] = np.round(255 * np.exp(-r2)).astype(np.uint8)
    return images, labels


def write_idx(path, array, magic):
    import lzma
    import struct
    header = struct.pack('>II', magic, len(array))
    if magic == 2051:
        header += struct.pack('>II', 28, 28)
    with lzma.open(path, 'wb') as fh:
        fh.write(header + np.ascontiguousarray(array, np.uint8).tobytes())


def write_idx_fixture():
    """tests/golden/idx/mnist/{train,t10k}-*-ubyte.xz, laid out like the
    reference's custom_envs/data/mnist/ (load_data.py:15-28)."""
    base = os.path.join(IDX_DIR, 'mnist')
    os.makedirs(base, exist_ok=True)
    for kind, n, seed in (('train', 240, 31), ('t10k', 96, 32)):
        images, labels = synthetic_digits(n, seed)
        write_idx(os.path.join(base, '%s-labels-idx1-ubyte.xz' % kind), labels, 2049)
        write_idx(os.path.join(base, '%s-images-idx3-ubyte.xz' % kind), images, 2051)


def reference_load_data(mods):
    """The reference's load_data reading IDX_DIR (its ``__file__`` points there)."""
    from PIL import Image
    img = load('custom_envs/utils/utils_image.py', ['resize_array', 'resize_array_many'],
               {'np': np, 'Image': Image})
    common = load('custom_envs/utils/utils_common.py', ['to_onehot'], {'np': np})

    def normalize(data):        # utils_math.py:77-87 without numexpr
        mins, maxes = np.min(data, axis=0), np.max(data, axis=0)
        return (data - mins) / (maxes - mins + 1e-8)

    import lzma
    from pathlib import Path
    ns = load('custom_envs/data/load_data.py', ['load_mnist', 'load_emnist', 'load_data'],
              {'np': np, 'lzma': lzma, 'Path': Path, 'tf': None, 'datasets': None,
               '__file__': os.path.join(IDX_DIR, 'load_data.py'),
               'InMemoryDataSet': mods.ds['InMemoryDataSet'],
               'resize_array_many': img['resize_array_many'], 'convert_many': None,
               'to_onehot': common['to_onehot'], 'normalize': normalize})
    return ns['load_data'], img['resize_array_many']


def main():
    from oracle.data import gaussians
    os.makedirs(GOLDEN, exist_ok=True)
    mods = reference_modules()
    features, targets = gaussians(256, 10, 0)
    for seed in (0, 1):
        rec = rollout_optimize(mods, features, targets, seed, None, 45, 1234 + seed)
        np.savez_compressed(os.path.join(GOLDEN, 'ref_optimize_s%d.npz' % seed), **rec)
    rec = rollout_optimize(mods, features, targets, 3, 32, 85, 99 + 3)
    np.savez_compressed(os.path.join(GOLDEN, 'ref_optimize_b32_s3.npz'), **rec)
    cases = [('ref_multi_func4_h5', 4, 400, 5, 60, 8, 1.0, 3.0),
             ('ref_multi_func4_h3_b25', 4, 25, 3, 90, 9, -1.0, 0.7)]
    for name, ndims, max_batches, hist, steps, seed, low, high in cases:
        rec = rollout_multi(mods, ndims, max_batches, hist, steps, seed, low, high)
        np.savez_compressed(os.path.join(GOLDEN, name + '.npz'), **rec)
    vec = utils_env_vectors(mods, np.random.RandomState(21))
    np.savez_compressed(os.path.join(GOLDEN, 'ref_utils_env.npz'), **vec)
    write_idx_fixture()
    ref_load_data, resize_many = reference_load_data(mods)
    out = {}
    for name in ('mnist', 'mnist-test'):
        seq = ref_load_data(name, batch_size=None)
        key = name.replace('-', '_')
        out[key + '_features'] = np.asarray(seq.features)
        out[key + '_targets'] = np.asarray(seq.targets)
    # PIL NEAREST on other shapes too (utils_image.py:6-25)
    rs = np.random.RandomState(5)
    imgs = rs.randint(0, 256, (6, 28, 28)).astype(np.uint8)
    out['resize_in'] = imgs
    for shape in ((7, 7), (5, 9), (14, 3)):
        out['resize_%dx%d' % shape] = np.stack(resize_many(imgs, shape))
    np.savez_compressed(os.path.join(GOLDEN, 'ref_load_data.npz'), **out)


if __name__ == '__main__':
    main()
