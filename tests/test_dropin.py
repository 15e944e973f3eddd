"""The reference's import lines and factory patterns resolve to the engine
(CPU: import surface and batching decisions; the engine itself is exercised
by tests/test_gpu_dropin.py)."""
import functools
import os
import sys
import types

import pytest

from conftest import REFERENCE

# The import lines of the two agent scripts north_star names, minus the
# nonexistent custom_envs.multiagent (run_multiagent_exp_single.py:20) and
# the out-of-scope bookkeeping module utils_file.
SCRIPT_IMPORTS = {
    'play_optimize.py': (22, [
        'import custom_envs.utils.utils_common as utils_common',
        'from custom_envs.utils.utils_logging import Monitor',
        'from custom_envs.vectorize.optvecenv import OptVecEnv',
        'from custom_envs.utils.utils_functions import compute_rosenbrock',
    ]),
    'run_multiagent_exp_single.py': (21, [
        'from custom_envs.utils.utils_logging import Monitor',
        'from custom_envs.utils.utils_venv import ThreadVecEnv',
        'from custom_envs.envs.multioptlrs import MultiOptLRs',
        'from custom_envs.envs.multioptimize import MultiOptimize',
        'from custom_envs.vectorize.optvecenv import OptVecEnv',
    ]),
    'search_optimize_hyperparam.py': (15, [
        'from custom_envs.utils.utils_logging import Monitor',
        'from custom_envs.vectorize.optvecenv import OptVecEnv',
    ]),
}


@pytest.mark.parametrize('script', sorted(SCRIPT_IMPORTS))
def test_script_import_lines_resolve(script):
    first, lines = SCRIPT_IMPORTS[script]
    path = os.path.join(REFERENCE, script)
    if os.path.exists(path):            # the lines are the reference's own
        with open(path) as fh:
            src = fh.read().splitlines()
        got = src[first - 1:first - 1 + len(lines)]
        assert got == lines, got
    namespace = {}
    exec('\n'.join(lines), namespace)   # noqa: S102 (import statements only)
    import custom_envs_amd.vectorize.optvecenv as amd_opt
    if 'OptVecEnv' in namespace:
        assert namespace['OptVecEnv'] is amd_opt.OptVecEnv
    if 'compute_rosenbrock' in namespace:
        assert namespace['compute_rosenbrock'](1.0, 1.0) == 0
        assert namespace['compute_rosenbrock'](-1.9, 2.0) == pytest.approx(
            100 * (2.0 - 3.61) ** 2 + 2.9 ** 2)


def test_package_surface():
    import custom_envs
    import custom_envs_amd
    from custom_envs.data import load_data
    from custom_envs.vectorize import SubprocVecEnv, ThreadVecEnv  # noqa: F401
    from custom_envs.wrappers import HistoryWrapper, SubSetWrapper  # noqa: F401
    from custom_envs.dataset import InMemoryDataSet
    from custom_envs.envs import SINGLE_AGENT_ENVIRONMENTS, MultiOptimize
    assert custom_envs.make is custom_envs_amd.make
    assert {'Optimize-v0', 'MultiOptLRs-v0', 'MultiOptimize-v0'} <= set(custom_envs.registry)
    seq = load_data('gaussians_256x10', batch_size=32)
    assert isinstance(seq, InMemoryDataSet) and len(seq) == 8
    assert MultiOptimize in SINGLE_AGENT_ENVIRONMENTS
    with pytest.raises(TypeError):        # multioptimize.py:44, as in the reference
        custom_envs.make('MultiOptimize-v0')


@pytest.fixture
def stub_gym(monkeypatch):
    """A stand-in ``gym`` module whose ``make`` is recognised by name and
    module, as the real ``gym.envs.registration.make`` would be."""
    gym = types.ModuleType('gym')

    def make(env_id, **kwargs):
        import custom_envs_amd
        return custom_envs_amd.make(env_id, **kwargs)
    make.__module__ = 'gym.envs.registration'
    gym.make = make
    monkeypatch.setitem(sys.modules, 'gym', gym)
    return gym


def test_gym_make_factories_batch(stub_gym):
    """search_optimize_hyperparam.py:99-112 and play_optimize.py:106-107 build
    ``partial(gym.make, id, **kw)`` factories (inside Monitor partials)."""
    from custom_envs.utils.utils_logging import Monitor
    from custom_envs_amd.vectorize.concurrent import _engine_request
    from custom_envs_amd.vectorize.optvecenv import _batch_request
    E = 6
    fns = [functools.partial(Monitor, functools.partial(stub_gym.make, 'MultiOptLRs-v0',
                                                        problem='func4', max_batches=50),
                             'mon_%d' % i, info_keywords=('loss',), chunk_size=5)
           for i in range(E)]
    kwargs, mon, built = _batch_request(fns)
    assert kwargs['problem'] == 'func4' and kwargs['max_batches'] == 50 and built == []
    assert mon[0] == ['mon_%d' % i for i in range(E)] and mon[1]['chunk_size'] == 5
    plain = [functools.partial(stub_gym.make, 'MultiOptLRs-v0')] * E
    assert _batch_request(plain)[0] == {}
    # Optimize-v0 through ThreadVecEnv's factory list, with and without Monitor
    opt = [functools.partial(stub_gym.make, 'Optimize-v0', data_set='gaussians_256x10')] * E
    kwargs, mon, built = _engine_request(opt)
    assert kwargs['data_set'] == 'gaussians_256x10' and mon is None
    mon_fns = [functools.partial(Monitor, functools.partial(stub_gym.make, 'Optimize-v0'),
                                 'run_%d' % i, chunk_size=10,
                                 info_keywords=('objective', 'accuracy')) for i in range(E)]
    kwargs, mon, built = _engine_request(mon_fns)
    assert mon[1]['info_keywords'] == ('objective', 'accuracy')
    # mixed specs or mixed monitoring stay on the host workers
    assert _engine_request(opt[:2] + [functools.partial(stub_gym.make, 'Optimize-v0',
                                                        batch_size=32)]) is None
    assert _engine_request(opt[:2] + mon_fns[:2]) is None
    assert _engine_request([functools.partial(stub_gym.make, 'Optimize-v0', bogus=1)]) is None
    # a partial naming the defaults explicitly is the same spec
    same = [functools.partial(stub_gym.make, 'Optimize-v0', data_set='gaussians_256x10',
                              batch_size=None, max_steps=40)]
    assert _engine_request(opt[:1] + same) is not None


def test_vector_env_spaces_without_gpu():
    from custom_envs_amd.envs.optimize import optimize_spaces
    from custom_envs_amd.vectorize.gpuvecenv import batch_space
    obs, act = optimize_spaces(20)
    b = batch_space(obs, 7)
    assert b.shape == (7, 41) and b.dtype == obs.dtype
    assert (b.low == -1e3).all() and (b.high == 1e3).all()
    assert batch_space(act, 3).shape == (3, 20)
