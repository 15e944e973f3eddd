"""The reference's factory patterns on the real engine: ``partial(gym.make,
...)`` factories, the scripts' ``partial(Monitor, ...)`` wrapping, and the
gym.vector-style surface, checked against the CPU oracle."""
import functools
import sys
import types

import numpy as np
import pytest

from oracle.optimize import Optimize as OracleEnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a ROCm device (run under gpurun)')


@pytest.fixture
def stub_gym(monkeypatch):
    gym = types.ModuleType('gym')

    def make(env_id, **kwargs):
        import custom_envs
        return custom_envs.make(env_id, **kwargs)
    make.__module__ = 'gym.envs.registration'
    gym.make = make
    monkeypatch.setitem(sys.modules, 'gym', gym)
    return gym


def test_monitored_optimize_threadvecenv(stub_gym, tmp_path, lr_dataset):
    """utils_logging.create_env's monitoring (Monitor(info_keywords=
    ('objective', 'accuracy'), chunk_size=10), utils_logging.py:159-175) on
    the factory list a ThreadVecEnv takes: one engine, one VecMonitor, the
    same .mon.csv episode rows as per-env Monitors."""
    import pandas as pd
    from custom_envs.utils.utils_logging import Monitor
    from custom_envs.utils.utils_venv import ThreadVecEnv
    E, T = 5, 85
    fns = [functools.partial(Monitor, functools.partial(stub_gym.make, 'Optimize-v0',
                                                        data_set=lr_dataset),
                             str(tmp_path / str(i)), chunk_size=1,
                             info_keywords=('objective', 'accuracy')) for i in range(E)]
    venv = ThreadVecEnv(fns)
    assert venv.engine_backed and venv.num_envs == E
    venv.seed(40)
    venv.reset()
    refs = []
    for i in range(E):
        env = OracleEnv(*lr_dataset)
        env.seed(40 + i)
        env.reset()
        refs.append(env)
    acts = np.random.RandomState(4).normal(0, 0.01, (T, E, 20)).astype(np.float32)
    episodes = [[] for _ in range(E)]
    ep_r = np.zeros(E)
    for t in range(T):
        obs, rews, dones, infos = venv.step(acts[t])
        for i, env in enumerate(refs):
            o, r, d, info = env.step(acts[t, i])
            ep_r[i] += np.float32(r)
            assert bool(dones[i]) == d
            if d:
                env.reset()
                episodes[i].append((ep_r[i], info['objective'], info['accuracy']))
                ep_r[i] = 0
                assert infos[i]['episode']['l'] == 40
                assert infos[i]['episode']['r'] == pytest.approx(episodes[i][-1][0], rel=1e-6)
    assert venv.env_method('get_episode_lengths') == [[40, 40]] * E
    venv.close()
    for i in range(E):
        frame = pd.read_csv(tmp_path / ('%d.mon.csv' % i))
        assert list(frame['l']) == [40, 40]
        assert list(frame['episode']) == [1, 2]
        np.testing.assert_allclose(frame['r'], [e[0] for e in episodes[i]], rtol=1e-6)
        np.testing.assert_allclose(frame['objective'], [e[1] for e in episodes[i]], rtol=1e-6)
        np.testing.assert_allclose(frame['accuracy'], [e[2] for e in episodes[i]], rtol=1e-6)


def test_gym_make_multioptlrs_factories_are_engine_backed(stub_gym):
    """search_optimize_hyperparam.py:99-112: partial(Monitor, partial(gym.make,
    'MultiOptLRs-v0', **kw), path, ...) per env -> one engine."""
    from custom_envs.vectorize.optvecenv import OptVecEnv
    E = 8
    venv = OptVecEnv([functools.partial(stub_gym.make, 'MultiOptLRs-v0', problem='func4',
                                        max_batches=30)] * E)
    assert venv.engine_backed and venv.num_envs == 4 * E
    obs = venv.reset()
    assert obs.shape == (4 * E, 15) and np.all(obs == -1)
    states, rewards, dones, infos = venv.step(np.full((4 * E, 1), 1.5, np.float32))
    assert states.shape == (4 * E, 15) and len(infos) == 4 * E
    venv.close()


def test_vector_env_surface(lr_dataset):
    """gym.vector.VectorEnv names: batched spaces + single_* spaces."""
    from custom_envs.vectorize import make_vec
    E = 6
    venv = make_vec('Optimize-v0', E, data_set=lr_dataset, seed=3)
    assert venv.is_vector_env and venv.num_envs == E
    assert venv.observation_space.shape == (E, 41)
    assert venv.action_space.shape == (E, 20)
    assert venv.single_observation_space.shape == (41,)
    assert venv.single_action_space.shape == (20,)
    obs = venv.reset()
    assert venv.observation_space.contains(obs)
    acts = np.stack([venv.single_action_space.sample() * 1e-4 for _ in range(E)])
    obs, rews, dones, infos = venv.step(acts)
    assert obs.shape == (E, 41) and rews.shape == (E,) and len(infos) == E
    venv.close()


def test_sb_monitor_factories_batch_into_one_engine(tmp_path, lr_dataset):
    """The stable-baselines style custom_envs.wrappers.Monitor
    (wrappers/monitor.py:11-163) around Optimize-v0 factories batches into one
    engine with a VecMonitor, and writes the same .mon.csv rows (r, l +
    info_keywords; t is wall time) as per-env wrappers run on host workers."""
    import pandas as pd
    import custom_envs
    from custom_envs.vectorize import ThreadVecEnv
    from custom_envs.wrappers import Monitor
    E, T = 4, 83
    acts = np.random.RandomState(6).normal(0, 0.01, (T, E, 20)).astype(np.float32)
    outs = {}
    for kind in ('batched', 'per_env'):
        paths = [str(tmp_path / ('%s_%d' % (kind, i))) for i in range(E)]
        if kind == 'batched':
            fns = [functools.partial(Monitor, custom_envs.make('Optimize-v0', data_set=lr_dataset),
                                     paths[i], info_keywords=('objective', 'accuracy'))
                   for i in range(E)]
        else:                      # a lambda is not a recognised spec: one host worker per env
            fns = [(lambda p=p: Monitor(custom_envs.make('Optimize-v0', data_set=lr_dataset), p,
                                        info_keywords=('objective', 'accuracy'))) for p in paths]
        venv = ThreadVecEnv(fns)
        assert venv.engine_backed == (kind == 'batched')
        venv.env_method('seed', 7)
        venv.reset()
        infos_done = []
        for t in range(T):
            _, rews, dones, infos = venv.step(acts[t])
            for i in np.flatnonzero(dones):
                infos_done.append((t, int(i), infos[i]['episode']['l'],
                                   round(float(infos[i]['episode']['r']), 4)))
        assert venv.env_method('get_episode_lengths') == [[40, 40]] * E
        outs[kind] = ([pd.read_csv(p + '.mon.csv') for p in paths], infos_done)
        venv.close()
    for a, b in zip(outs['batched'][0], outs['per_env'][0]):
        assert sorted(a.columns) == sorted(b.columns) == ['accuracy', 'l', 'objective', 'r', 't']
        assert list(a['l']) == list(b['l']) == [40, 40]
        np.testing.assert_allclose(a['r'], b['r'], rtol=1e-6)
        np.testing.assert_allclose(a['objective'], b['objective'], rtol=1e-6)
        np.testing.assert_array_equal(a['accuracy'], b['accuracy'])
    assert outs['batched'][1] == outs['per_env'][1]


def test_sb_monitor_refuses_early_reset(lr_dataset):
    """allow_early_resets=False (the SB default): a VecEnv reset in the middle
    of an episode raises, as the per-env wrapper does (monitor.py:69-75)."""
    import custom_envs
    from custom_envs.vectorize import ThreadVecEnv
    from custom_envs.wrappers import Monitor
    fns = [functools.partial(Monitor, custom_envs.make('Optimize-v0', data_set=lr_dataset), None)
           for _ in range(3)]
    venv = ThreadVecEnv(fns)
    assert venv.engine_backed
    venv.reset()
    venv.step(np.zeros((3, 20), np.float32))
    with pytest.raises(RuntimeError, match='allow early resets'):
        venv.reset()
    venv.close()


def test_sb_monitor_reset_keywords_batch_and_raise(lr_dataset):
    """An SB Monitor factory with ``reset_keywords`` batches into one engine;
    its VecEnv reset (which passes no kwargs) raises the per-env wrapper's
    ValueError (monitor.py:76-80), and a step before any reset raises its
    RuntimeError (monitor.py:87-88), before the engine launches."""
    import custom_envs
    from custom_envs.vectorize import ThreadVecEnv
    from custom_envs.wrappers import Monitor
    fns = [functools.partial(Monitor, custom_envs.make('Optimize-v0', data_set=lr_dataset), None,
                             reset_keywords=('tag',)) for _ in range(3)]
    venv = ThreadVecEnv(fns)
    assert venv.engine_backed
    with pytest.raises(RuntimeError, match='needs reset'):
        venv.step(np.zeros((3, 20), np.float32))
    with pytest.raises(ValueError, match='kwarg tag'):
        venv.reset()
    venv.close()
