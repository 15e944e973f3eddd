"""The reference's own test suite, restated against this package.

Each test below is one of /root/reference/tests/**, with `custom_envs` /
`gym` replaced by `custom_envs_amd` and its old-gym spaces; the assertions
are the reference's.  A caller that moves from custom_envs to this package
keeps every contract these tests check.

  tests/envs/test_env.py                  -> test_env_step / test_env_reset (GPU engine)
  tests/vectorize/test_concurrentvecenv.py -> test_vec_env_reset / _step
  tests/vectorize/test_optvecenv.py        -> test_optvecenv_reset / _step
  tests/dataset/test_inmemorydataset.py    -> test_dataset_*
  tests/wrappers/test_optimizewrappers.py  -> test_historywrapper_* / test_subsetwrapper_*
"""
from functools import partial
from itertools import chain

import numpy as np
import numpy.random as npr
import pytest

from custom_envs_amd.core import Env
from custom_envs_amd.dataset import InMemoryDataSet
from custom_envs_amd.spaces import Box, Dict
from custom_envs_amd.vectorize import SubprocVecEnv, ThreadVecEnv
from custom_envs_amd.vectorize.optvecenv import OptVecEnv, flatten_dictionary
import custom_envs_amd.wrappers.optimizewrappers as wrappers

NUMBER_OF_PROCESSORS = 2


class StubEnv(Env):
    """tests/vectorize/test_concurrentvecenv.py:16-46 (and the wrappers' copy)."""

    def __init__(self):
        self.counter = 0
        self.observation_space = Dict({
            'test1d': Box(low=-1e3, high=1e3, dtype=np.float32, shape=[5]),
            'test2d': Box(low=-1e3, high=1e3, dtype=np.float32, shape=[5] * 2),
            'test3d': Box(low=-1e3, high=1e3, dtype=np.float32, shape=[5] * 3)
        })
        self.action_space = Box(low=-1e3, high=1e3, dtype=np.float32, shape=(25,))
        self.observation_space_old = self.observation_space
        self.action_space_old = self.action_space

    def step(self, action):
        self.counter += 1
        return self.observation_space_old.sample(), 0, self.terminal(), {}

    def terminal(self):
        return self.counter >= 10

    def render(self, mode='human'):
        pass

    def reset(self):
        self.counter = 0
        return self.observation_space_old.sample()


class StubOptEnv(StubEnv):
    """tests/vectorize/test_optvecenv.py:11-38: three 5-vectors, the action
    space is the observation space."""

    def __init__(self):
        super().__init__()
        self.observation_space = Dict({
            'test1d': Box(low=-1e3, high=1e3, dtype=np.float32, shape=[5]),
            'test2d': Box(low=-1e3, high=1e3, dtype=np.float32, shape=[5]),
            'test3d': Box(low=-1e3, high=1e3, dtype=np.float32, shape=[5])
        })
        self.action_space = self.observation_space
        self.observation_space_old = self.observation_space


# ---------------------------------------------------------------- envs (GPU)
@pytest.mark.gpu
def test_env_step(lr_dataset):
    """tests/envs/test_env.py:7-24 for Optimize-v0.  The sampled action is
    scaled by 1e-3: a raw Box(-1e3, 1e3) sample sends the loss ratio L' (obs
    entry P, optimize.py:80-81) past the observation bound within a step."""
    import custom_envs_amd
    environ = custom_envs_amd.make('Optimize-v0', data_set=lr_dataset)
    environ.reset()
    assert environ.current_step == 0
    action = environ.action_space.sample() * 1e-3
    for i in range(1, 10):
        state, reward, terminal, info = environ.step(action)
        assert environ.current_step == i
        assert environ.observation_space.contains(state)
        assert isinstance(reward, float)
        assert isinstance(terminal, bool)
        assert isinstance(info, dict)
        if terminal:
            break
    environ.close()


@pytest.mark.gpu
def test_env_reset(lr_dataset):
    """tests/envs/test_env.py:27-31."""
    import custom_envs_amd
    environ = custom_envs_amd.make('Optimize-v0', data_set=lr_dataset)
    state = environ.reset()
    assert environ.observation_space.contains(state)
    environ.close()


# ------------------------------------------------------------------ vectorize
VECENV_CLASSES = [SubprocVecEnv, ThreadVecEnv]


@pytest.mark.parametrize('vecenv_class', VECENV_CLASSES)
def test_vec_env_reset(vecenv_class):
    """tests/vectorize/test_concurrentvecenv.py:49-54."""
    envs = [partial(StubEnv) for _ in range(NUMBER_OF_PROCESSORS)]
    vec_env = vecenv_class(envs)
    states = vec_env.reset()
    assert len(states['test1d']) == NUMBER_OF_PROCESSORS
    vec_env.close()


@pytest.mark.parametrize('vecenv_class', VECENV_CLASSES)
def test_vec_env_step(vecenv_class):
    """tests/vectorize/test_concurrentvecenv.py:57-73."""
    test = StubEnv()
    envs = [partial(StubEnv) for _ in range(NUMBER_OF_PROCESSORS)]
    vec_env = vecenv_class(envs)
    vec_env.reset()
    terminal = False
    while not terminal:
        actions = [test.action_space.sample() for _ in range(NUMBER_OF_PROCESSORS)]
        states, rewards, terminal, info = vec_env.step(actions)
        assert len(states['test1d']) == NUMBER_OF_PROCESSORS
        assert len(rewards) == NUMBER_OF_PROCESSORS
        assert len(terminal) == NUMBER_OF_PROCESSORS
        assert len(info) == NUMBER_OF_PROCESSORS
        terminal = np.all(terminal)
    vec_env.close()


def test_optvecenv_reset():
    """tests/vectorize/test_optvecenv.py:41-45."""
    vec_env = OptVecEnv([StubOptEnv])
    vec_env.reset()
    vec_env.close()


def test_optvecenv_step():
    """tests/vectorize/test_optvecenv.py:48-59."""
    vec_env = OptVecEnv([StubOptEnv] * 2)
    vec_env.reset()
    terminal = False
    while not terminal:
        actions = [flatten_dictionary(StubOptEnv().action_space.sample())] * 2
        actions = list(chain.from_iterable(actions))
        states, rewards, terminals, infos = vec_env.step(actions)
        assert len(states) == vec_env.num_envs
        terminal = np.any(terminals)
    vec_env.close()


# -------------------------------------------------------------------- dataset
def random_data_set(sample_shape=(10,), num_of_targets=1, batch_size=None):
    features = npr.rand(*sample_shape)
    targets = npr.rand(sample_shape[0], num_of_targets)
    return InMemoryDataSet(features, targets, batch_size=batch_size)


def test_dataset_on_epoch_end():
    """tests/dataset/test_inmemorydataset.py:15-24."""
    features = npr.rand(10)
    targets = npr.rand(10)
    data_set = InMemoryDataSet(features, targets)
    assert np.all(features == data_set.features)
    assert np.all(targets == data_set.targets)
    data_set.on_epoch_end()
    assert not np.all(features == data_set.features)
    assert not np.all(targets == data_set.targets)


def test_dataset_len():
    """tests/dataset/test_inmemorydataset.py:27-32."""
    assert len(random_data_set(sample_shape=(10,))) == 1
    assert len(random_data_set(sample_shape=(10,), batch_size=2)) == 5


def test_dataset_getitem():
    """tests/dataset/test_inmemorydataset.py:35-40."""
    assert len(random_data_set(sample_shape=(10,))[0].features) == 10
    assert len(random_data_set(sample_shape=(10,), batch_size=2)[0].features) == 2


def test_dataset_shapes():
    """tests/dataset/test_inmemorydataset.py:43-52."""
    assert random_data_set().feature_shape == ()
    assert random_data_set().target_shape == (1,)


# ------------------------------------------------------------------- wrappers
def test_historywrapper_spaces():
    """tests/wrappers/test_optimizewrappers.py:45-57."""
    max_history = 5
    env = StubEnv()
    obs_space_old = env.observation_space.spaces
    action_space_old = env.action_space
    env = wrappers.HistoryWrapper(env, max_history)
    assert obs_space_old.keys() == env.observation_space.spaces.keys()
    for name, space in obs_space_old.items():
        assert np.all(env.observation_space[name].low == space.low)
        assert np.all(env.observation_space[name].high == space.high)
        assert env.observation_space[name].shape == (max_history, *space.shape)
    assert action_space_old == env.action_space


def test_historywrapper_step_and_reset():
    """tests/wrappers/test_optimizewrappers.py:60-76."""
    env = wrappers.HistoryWrapper(StubEnv(), 5)
    obs, reward, terminal, info = env.step(env.action_space.sample())
    assert env.observation_space.contains(obs)
    assert isinstance(reward, (float, int))
    assert isinstance(terminal, bool)
    assert isinstance(info, dict)
    env = wrappers.HistoryWrapper(StubEnv(), 5)
    assert env.observation_space.contains(env.reset())


def test_subsetwrapper_spaces():
    """tests/wrappers/test_optimizewrappers.py:79-90."""
    env = StubEnv()
    obs_space_old = env.observation_space
    action_space_old = env.action_space
    env = wrappers.SubSetWrapper(env, ['test1d', 'test2d'])
    assert obs_space_old.spaces.keys() >= env.observation_space.spaces.keys()
    for name, space in env.observation_space.spaces.items():
        assert np.all(obs_space_old[name].low == space.low)
        assert np.all(obs_space_old[name].high == space.high)
        assert obs_space_old[name].shape == space.shape
    assert action_space_old == env.action_space


def test_subsetwrapper_step_and_reset():
    """tests/wrappers/test_optimizewrappers.py:93-109."""
    env = wrappers.SubSetWrapper(StubEnv(), ['test1d', 'test2d'])
    obs, reward, terminal, info = env.step(env.action_space.sample())
    assert env.observation_space.contains(obs)
    assert isinstance(reward, (float, int))
    assert isinstance(terminal, bool)
    assert isinstance(info, dict)
    env = wrappers.SubSetWrapper(StubEnv(), ['test1d', 'test2d'])
    assert env.observation_space.contains(env.reset())
