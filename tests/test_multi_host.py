"""Multi-agent path on the CPU: oracle pins, host facades, wrappers, Monitor.

Pins: the restated ``History`` / ``build_multistate`` agree
with the reference's importable ``custom_envs/utils/utils_common.py``
(when /root/reference exists); committed MultiOptLRs rollouts regenerate
bit for bit.  The host surface (OptVecEnv's reference path, Monitor CSV
chunks, History/SubSet wrappers) runs on stub envs, as the reference tests do
(tests/vectorize/test_optvecenv.py:11-59, tests/wrappers/*).
"""
import functools
import importlib.util
import os

import numpy as np
import pytest

from conftest import REFERENCE, golden
from custom_envs_amd.spaces import Box, Dict


def _ref_utils_common():
    path = os.path.join(REFERENCE, 'custom_envs', 'utils', 'utils_common.py')
    if not os.path.exists(path):
        pytest.skip('reference checkout not present')
    spec = importlib.util.spec_from_file_location('ref_utils_common_m', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize('impl', ['oracle', 'package'])
def test_history_matches_reference(impl):
    ref = _ref_utils_common()
    if impl == 'oracle':
        from oracle.multioptlrs import History
    else:
        from custom_envs_amd.utils.utils_common import History
    rs = np.random.RandomState(0)
    a = ref.History(4, weights=(3,), losses=(), gradients=(3,))
    b = History(4, weights=(3,), losses=(), gradients=(3,))
    for _ in range(6):
        item = dict(weights=rs.rand(3), losses=rs.rand(), gradients=rs.rand(3))
        a.append(**item)
        b.append(**item)
        for key in ('weights', 'losses', 'gradients'):
            assert np.array_equal(a[key], b[key])
        assert a.build_multistate() == b.build_multistate()


def test_rosenbrock_terms_match_reference_function():
    """The oracle's float32 Rosenbrock pair terms are bit-identical to the
    reference's own ``compute_rosenbrock`` (utils_functions.py:4-6, imported
    by path) on float32 inputs: numpy evaluates 100*(y - x**2)**2 + (1 - x)**2
    in the same float32 operation order (x**2 is x*x)."""
    path = os.path.join(REFERENCE, 'custom_envs', 'utils', 'utils_functions.py')
    if not os.path.exists(path):
        pytest.skip('reference checkout not present')
    spec = importlib.util.spec_from_file_location('ref_utils_functions', path)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    from oracle.multioptlrs import RosenbrockPairs
    rs = np.random.RandomState(11)
    prob = RosenbrockPairs(ndims=8)
    for scale in (0.5, 2.0, 30.0):
        p = (rs.normal(size=8) * scale).astype(np.float32)
        x, y = p[0::2], p[1::2]
        ref_terms = ref.compute_rosenbrock(x, y)
        assert ref_terms.dtype == np.float32
        one, c100 = np.float32(1), np.float32(100)
        d = y - x * x
        ours = c100 * (d * d) + (one - x) * (one - x)
        assert np.array_equal(ours, ref_terms)
        loss = np.float32(0)
        for term in ref_terms:
            loss = np.float32(loss + term)
        prob.params = p.copy()
        assert prob._eval(p)[1] == loss


@pytest.mark.parametrize('name,ndims,max_batches,hist,steps,seed,low,high', [
    ('multi_func2_h5', 2, 400, 5, 150, 7, -1.0, 0.5),
    ('multi_func4_h5', 4, 400, 5, 60, 8, 1.0, 3.0),
    ('multi_func4_h3_b25', 4, 25, 3, 90, 9, -1.0, 0.7)])
def test_multi_fixtures_regenerate(name, ndims, max_batches, hist, steps, seed, low, high):
    from oracle.gen_golden import rollout_multi
    fx = golden(name + '.npz')
    rec = rollout_multi(ndims, max_batches, hist, steps, seed, low, high)
    for key in ('obs', 'reward', 'done', 'ep_len', 'theta', 'reset_obs'):
        assert np.array_equal(rec[key], fx[key]), key
    np.testing.assert_array_equal(rec['info'], fx['info'])


class StubMultiEnv:
    """tests/vectorize/test_optvecenv.py:11-38 style: Dict spaces, 10 steps."""

    def __init__(self, agents=3):
        names = ['parameter-%d' % i for i in range(agents)]
        self.observation_space = Dict({n: Box(-1e3, 1e3, (4,)) for n in names})
        self.action_space = Dict({n: Box(-1e3, 1e3, (1,)) for n in names})
        self.counter = 0

    def reset(self):
        self.counter = 0
        return {n: np.full(4, i, np.float32) for i, n in enumerate(sorted(self.observation_space.spaces))}

    def step(self, action):
        self.counter += 1
        obs = {n: np.full(4, float(np.asarray(action[n]).ravel()[0]), np.float32)
               for n in self.observation_space.spaces}
        return obs, 1.0, self.counter >= 10, {'counter': self.counter}

    def close(self):
        pass


def test_optvecenv_host_path_rows_and_callbacks():
    from custom_envs_amd.vectorize import OptVecEnv
    seen = []
    venv = OptVecEnv([functools.partial(StubMultiEnv, 3), functools.partial(StubMultiEnv, 2)],
                     callbacks=[lambda *a: seen.append(len(a[0]))])
    assert not venv.engine_backed
    assert venv.agent_no_list == [3, 2] and venv.num_envs == 5
    obs = venv.reset()
    assert obs.shape == (5, 4)
    actions = np.arange(5, dtype=np.float32).reshape(5, 1)
    states, rewards, dones, infos = venv.step(actions)
    # row r of env k carries that env's agent in sorted-name order
    assert np.array_equal(states[:, 0], np.arange(5))
    assert rewards.shape == (5,) and dones.shape == (5,) and len(infos) == 5
    assert infos[0] is infos[1] and infos[3] is infos[4]
    assert seen == [5]
    venv.close()


def test_batch_request_recognises_engine_factories():
    from custom_envs_amd.core import make
    from custom_envs_amd.utils.utils_logging import Monitor
    from custom_envs_amd.vectorize.optvecenv import _batch_request
    fns = [functools.partial(make, 'MultiOptLRs-v0', problem='func4', max_batches=50)] * 3
    kwargs, mon, built = _batch_request(fns)
    assert kwargs == {'problem': 'func4', 'max_batches': 50} and mon is None and not built
    mon_fns = [functools.partial(Monitor, functools.partial(make, 'MultiOptLRs-v0'), 'log_%d' % i,
                                 allow_early_resets=True, info_keywords=('loss',), chunk_size=5)
               for i in range(2)]
    kwargs, mon, built = _batch_request(mon_fns)
    assert mon[0] == ['log_0', 'log_1'] and mon[1] == {'info_keywords': ('loss',), 'chunk_size': 5}
    assert _batch_request([functools.partial(StubMultiEnv, 3)]) is None
    mixed = [fns[0], functools.partial(make, 'MultiOptLRs-v0', problem='func')]
    assert _batch_request(mixed) is None


class StubEnv:
    observation_space = Box(-1, 1, (2,))
    action_space = Box(-1, 1, (1,))

    def __init__(self):
        self.t = 0

    def reset(self, **kwargs):
        self.t = 0
        return np.zeros(2)

    def step(self, action):
        self.t += 1
        return np.ones(2), 0.5, self.t >= 3, {'objective': float(self.t)}

    def close(self):
        pass


def test_monitor_writes_chunked_csv(tmp_path):
    import pandas as pd
    from custom_envs_amd.utils.utils_logging import Monitor
    calls = []
    env = Monitor(StubEnv(), str(tmp_path / 'run'), info_keywords=('objective',), chunk_size=2,
                  callbacks=[calls.append])
    for _ in range(3):
        env.reset()
        done = False
        while not done:
            _, _, done, info = env.step(0)
    env.close()
    frame = pd.read_csv(tmp_path / 'run.mon.csv')
    assert list(frame.columns) == sorted(['r', 'l', 't', 'current_reward', 'episode', 'objective'])
    assert list(frame['l']) == [3, 3, 3] and list(frame['episode']) == [1, 2, 3]
    assert np.allclose(frame['r'], 1.5) and len(calls) == 9
    assert env.get_episode_rewards() == [1.5] * 3 and env.get_total_steps() == 9


def test_vec_monitor_matches_per_env_monitor(tmp_path):
    import pandas as pd
    from custom_envs_amd.utils.utils_logging import VecMonitor
    mon = VecMonitor(2, [str(tmp_path / 'a'), str(tmp_path / 'b')], info_keywords=('objective',),
                     chunk_size=1)
    mon.reset()
    infos = [{'objective': 1.0}, {'objective': 2.0}]
    for t in range(1, 5):
        finished = mon.step(np.array([0.5, 0.25]), np.array([t % 2 == 0, t == 4]), infos)
        if t == 2:
            assert set(finished) == {0} and finished[0]['l'] == 2
    mon.close()
    a = pd.read_csv(tmp_path / 'a.mon.csv')
    b = pd.read_csv(tmp_path / 'b.mon.csv')
    assert list(a['l']) == [2, 2] and list(a['episode']) == [1, 2]
    assert list(b['l']) == [4] and np.isclose(b['r'][0], 1.0)
    assert mon.get_episode_rewards() == [[1.0, 1.0], [1.0]]


def test_sb_monitor_contract(tmp_path):
    from custom_envs_amd.wrappers import Monitor
    env = Monitor(StubEnv(), str(tmp_path / 'sb'), reset_keywords=('tag',))
    with pytest.raises(RuntimeError):
        env.step(0)
    with pytest.raises(ValueError):
        env.reset()
    # like monitor.py:84-85, the episode counts as started before the check
    env = Monitor(StubEnv(), str(tmp_path / 'sb'), reset_keywords=('tag',))
    env.reset(tag='x')
    with pytest.raises(RuntimeError):
        env.reset(tag='x')
    for _ in range(3):
        _, _, done, info = env.step(0)
    assert done and info['episode']['tag'] == 'x' and info['episode']['l'] == 3
    env.close()


def test_vec_monitor_sb_reset_keywords_and_step_check(tmp_path):
    """The batched SB Monitor: step before reset and a reset without the
    reset_keywords raise as the per-env wrapper does (monitor.py:76-88); the
    keyword values ride on every episode row."""
    from custom_envs_amd.utils.utils_logging import VecMonitor
    mon = VecMonitor(2, str(tmp_path / 'v'), style='sb', reset_keywords=('tag',))
    with pytest.raises(RuntimeError, match='needs reset'):
        mon.check_step()
    with pytest.raises(ValueError, match='kwarg tag'):
        mon.reset()
    mon.check_step()             # the episode counted as started (monitor.py:84-85)
    mon = VecMonitor(2, str(tmp_path / 'w'), style='sb', allow_early_resets=True,
                     reset_keywords=('tag',))
    mon.reset(tag='x')
    assert mon.step(np.array([1.0, 2.0]), np.array([False, False]), [{}, {}]) == {}
    # the auto-reset after an episode passes no kwargs: it raises as the
    # worker's ``env.reset()`` would (utils_venv.py:31), after the row is kept
    with pytest.raises(ValueError, match='kwarg tag'):
        mon.step(np.array([1.0, 2.0]), np.array([True, False]), [{}, {}])
    import pandas as pd
    row = pd.read_csv(tmp_path / 'w_0.mon.csv').iloc[0]
    assert (row['r'], row['l'], row['tag']) == (2.0, 2, 'x')
    with pytest.raises(ValueError):
        VecMonitor(1, None, reset_keywords=('tag',))


def test_history_and_subset_wrappers():
    from custom_envs_amd.wrappers import HistoryWrapper, SubSetWrapper
    env = HistoryWrapper(StubMultiEnv(2), max_history=3)
    first = env.reset()
    assert first['parameter-1'].shape == (3, 4) and np.all(first['parameter-1'] == 1)
    obs, _, _, _ = env.step({'parameter-0': 7.0, 'parameter-1': 9.0})
    assert np.all(obs['parameter-0'][0] == 7) and np.all(obs['parameter-0'][1] == 0)
    assert env.observation_space['parameter-0'].shape == (3, 4)
    sub = SubSetWrapper(StubMultiEnv(2), ['parameter-1'])
    assert list(sub.reset()) == ['parameter-1']
    assert list(sub.observation_space.spaces) == ['parameter-1']
