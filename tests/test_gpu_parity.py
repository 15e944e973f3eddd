"""HIP engine vs the CPU oracle (golden fixtures + live oracle runs).

Tolerances (written here, per SURVEY.md 7 "Parity tolerance"):
  - integer/index work is bit-exact: done flags, episode lengths, the
    composed minibatch row order, seeded W0;
  - f64 engine: obs/reward/info are float64 results rounded to float32, so
    they must equal the oracle's float64 values within F64_RTOL (a few f32
    ulps); the float64 state (weights, loss_hist) within 1e-12 relative;
  - f32 engine (hardware v_exp_f32/v_log_f32): per obs row
    ||d||_inf / ||ref||_inf <= 1e-5 (the north-star bound), plus elementwise
    1e-3 relative where |ref| >= 1e-2 ||ref||_inf (gradient entries far
    below the row maximum come out of a cancelling sum over rows and carry
    float32 rounding of the row terms, SURVEY.md 7 "Parity tolerance").
"""
import numpy as np
import pytest

from conftest import golden
from oracle.optimize import Optimize as OracleEnv

pytestmark = pytest.mark.gpu

F64_RTOL = 1e-6
F64_ATOL = 1e-9


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a ROCm device (run under gpurun)')


def _engine(dataset, num_envs, batch_size=None, precision='f64', auto_reset=True):
    from custom_envs_amd.engine import OptimizeEngine
    return OptimizeEngine(*dataset, num_envs=num_envs, batch_size=batch_size,
                          precision=precision, auto_reset=auto_reset)


def _run(eng, seeds, actions):
    """actions [T][E][P] -> dict of stacked per-step outputs."""
    eng.seed(list(seeds))
    reset_obs = eng.reset()
    rec = {k: [] for k in ('obs', 'reward', 'done', 'objective', 'accuracy', 'episode_len')}
    for t in range(actions.shape[0]):
        out = eng.step(actions[t])
        for k in rec:
            rec[k].append(out[k].copy())
    res = {k: np.array(v) for k, v in rec.items()}
    res['reset_obs'] = reset_obs
    return res


def _close_f32_rows(got, ref, tol=1e-5, elem_tol=1e-3, elem_floor=1e-2):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = np.maximum(np.abs(ref).max(axis=-1, keepdims=True), 1e-30)
    row_err = np.abs(got - ref).max(axis=-1) / scale[..., 0]
    assert np.all(row_err <= tol), row_err.max()
    big = np.abs(ref) >= elem_floor * scale
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)
    assert np.all(rel[big] <= elem_tol), rel[big].max()


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_golden_rollout_f64(lr_dataset, seed):
    fx = golden('optimize_lr_s%d.npz' % seed)
    eng = _engine(lr_dataset, 1)
    res = _run(eng, [seed], fx['actions'][:, None, :])
    assert np.all(res['reset_obs'] == 0)
    assert np.array_equal(res['done'][:, 0].astype(bool), fx['done'])
    assert np.array_equal(res['episode_len'][:, 0], fx['ep_len'])
    np.testing.assert_allclose(res['obs'][:, 0], fx['obs'], rtol=F64_RTOL, atol=F64_ATOL)
    np.testing.assert_allclose(res['reward'][:, 0], fx['reward'], rtol=F64_RTOL)
    np.testing.assert_allclose(res['objective'][:, 0], fx['objective'], rtol=F64_RTOL)
    np.testing.assert_array_equal(res['accuracy'][:, 0], fx['accuracy'].astype(np.float32))
    st = eng.get_state()
    np.testing.assert_allclose(st['weights'][0], fx['weights'][-1], rtol=1e-12, atol=1e-14)
    eng.close()


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_golden_rollout_f32(lr_dataset, seed):
    fx = golden('optimize_lr_s%d.npz' % seed)
    eng = _engine(lr_dataset, 1, precision='f32')
    res = _run(eng, [seed], fx['actions'][:, None, :])
    assert np.array_equal(res['done'][:, 0].astype(bool), fx['done'])
    live = ~fx['done']          # terminal rows carry the (all-zero) reset obs
    _close_f32_rows(res['obs'][live, 0], fx['obs'][live])
    np.testing.assert_allclose(res['reward'][:, 0], fx['reward'], rtol=1e-5)
    np.testing.assert_allclose(res['objective'][:, 0], fx['objective'], rtol=1e-5)
    eng.close()


@pytest.mark.parametrize('seed', [3, 4])
@pytest.mark.parametrize('precision', ['f64', 'f32'])
def test_golden_minibatch_rollout(lr_dataset, seed, precision):
    """batch_size=32 < N: minibatch rows and their order must be bit-exact."""
    fx = golden('optimize_lr_b32_s%d.npz' % seed)
    eng = _engine(lr_dataset, 1, batch_size=32, precision=precision)
    eng.seed([seed])
    eng.reset()
    for t in range(fx['actions'].shape[0]):
        out = eng.step(fx['actions'][t][None])
        order = eng.get_state()['order'][0]
        assert np.array_equal(order, fx['order'][t]), t
        if precision == 'f64':
            np.testing.assert_allclose(out['obs'][0], fx['obs'][t], rtol=F64_RTOL, atol=F64_ATOL)
            np.testing.assert_allclose(out['reward'][0], fx['reward'][t], rtol=F64_RTOL)
            np.testing.assert_allclose(out['objective'][0], fx['objective'][t], rtol=F64_RTOL)
            assert out['accuracy'][0] == np.float32(fx['accuracy'][t])
        elif not fx['done'][t]:
            _close_f32_rows(out['obs'][0][None], fx['obs'][t][None])
    eng.close()


def test_many_envs_against_live_oracle(lr_dataset):
    """E=256 independent envs, each its own seed and action stream."""
    E, T = 256, 45
    seeds = [1000 + i for i in range(E)]
    P = 20
    actions = np.random.RandomState(7).normal(0, 0.01, (T, E, P)).astype(np.float32)
    eng = _engine(lr_dataset, E)
    res = _run(eng, seeds, actions)
    for i in range(0, E, 17):
        env = OracleEnv(*lr_dataset)
        env.seed(seeds[i])
        env.reset()
        for t in range(T):
            obs, rew, done, info = env.step(actions[t, i])
            if done:
                obs = env.reset()
            np.testing.assert_allclose(res['obs'][t, i], obs, rtol=F64_RTOL, atol=F64_ATOL)
            assert res['reward'][t, i] == pytest.approx(rew, rel=F64_RTOL)
            assert bool(res['done'][t, i]) == done
            assert res['episode_len'][t, i] == info['episode']['l']
    eng.close()


def test_init_weights_match_seeding(lr_dataset):
    from oracle.optimize import initial_draws
    eng = _engine(lr_dataset, 8)
    eng.seed([5 * i for i in range(8)])
    eng.reset()
    st = eng.get_state()
    for i in range(8):
        w0, _ = initial_draws(5 * i, 10, 2, 256)
        assert np.array_equal(st['init_weights'][i], w0.ravel())
        assert np.array_equal(st['weights'][i], w0.ravel())
    eng.close()


def test_full_size_properties(lr_dataset):
    """E=4096 (the benchmark size): properties that hold at any size."""
    E, P = 4096, 20
    eng = _engine(lr_dataset, E)
    eng.seed(0)
    eng.reset()
    rs = np.random.RandomState(3)
    for t in range(1, 83):
        out = eng.step(rs.normal(0, 0.01, (E, P)).astype(np.float32))
        expect_len = (t - 1) % 40 + 1
        assert np.all(out['episode_len'] == expect_len)
        assert np.all(out['done'] == (expect_len == 40))
        if expect_len == 40:
            assert np.all(out['obs'] == 0)        # auto-reset obs
        else:
            assert np.all(out['obs'][:, :P] == 0)  # wght_hist stays 0
        # B == N: objective is the minibatch loss (optimize.py:94-96)
        assert np.array_equal(out['reward'], -out['objective'])
        assert np.all((out['accuracy'] >= 0) & (out['accuracy'] <= 1))
    eng.close()
    # determinism: identical seeds and actions reproduce the same bits
    a = _engine(lr_dataset, E)
    b = _engine(lr_dataset, E)
    act = np.random.RandomState(9).normal(0, 0.01, (E, P)).astype(np.float32)
    for eng in (a, b):
        eng.seed(0)
        eng.reset()
    oa = a.step(act)['obs'].copy()
    ob = b.step(act)['obs'].copy()
    assert np.array_equal(oa, ob)
    a.close()
    b.close()


def test_single_env_api_matches_oracle(lr_dataset):
    """make('Optimize-v0') single env, including stepping past the terminal."""
    import custom_envs_amd
    env = custom_envs_amd.make('Optimize-v0', data_set=lr_dataset)
    env.seed(21)
    obs = env.reset()
    assert env.current_step == 0 and env.observation_space.contains(obs)
    ref = OracleEnv(*lr_dataset)
    ref.seed(21)
    ref.reset()
    rs = np.random.RandomState(2)
    for t in range(1, 45):
        a = rs.normal(0, 0.01, 20).astype(np.float32)
        obs, rew, done, info = env.step(a)
        robs, rrew, rdone, rinfo = ref.step(a)
        assert env.current_step == t
        assert isinstance(rew, float) and isinstance(done, bool) and isinstance(info, dict)
        assert done == rdone
        np.testing.assert_allclose(obs, robs, rtol=F64_RTOL, atol=F64_ATOL)
        assert info['episode']['l'] == rinfo['episode']['l']
        assert info['objective'] == pytest.approx(rinfo['objective'], rel=F64_RTOL)
    env.close()


@pytest.mark.parametrize('many_direct,bound,persist', [('32', False, '0'), ('0', False, '0'),
                                                       ('32', True, '0'), ('32', False, '1'),
                                                       ('32', True, '1')])
def test_device_path_matches_host_path(lr_dataset, many_direct, bound, persist, monkeypatch):
    """ce_step_many as plain launches (k <= CE_MANY_DIRECT, default 32), as a
    replayed hipGraph (CE_MANY_DIRECT=0), through the pre-bound many_runner,
    and as ONE persistent launch (CE_PERSIST=1, the default) give the host
    path's bits."""
    import torch
    monkeypatch.setenv('CE_MANY_DIRECT', many_direct)
    monkeypatch.setenv('CE_PERSIST', persist)
    E, P, K = 512, 20, 12
    acts = np.random.RandomState(4).normal(0, 0.01, (K, E, P)).astype(np.float32)
    host = _engine(lr_dataset, E)
    host.seed(0)
    host.reset()
    for t in range(K):
        ref = host.step(acts[t])
    dev = _engine(lr_dataset, E)
    assert dev.persistent == (persist == '1')
    dev.seed(0)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        dev.set_stream(stream.cuda_stream)
        out = dev.alloc_device_outputs()
        dact = torch.from_numpy(acts).cuda()
        dev.reset_device(out)
        if bound:
            run = dev.many_runner(K // 2, dact[:K // 2], out)
            run()
            dev.many_runner(K - K // 2, dact[K // 2:], out)()
        else:
            dev.step_many_device(K, dact, out)
    torch.cuda.synchronize()
    assert np.array_equal(out['obs'].cpu().numpy(), ref['obs'])
    assert np.array_equal(out['reward'].cpu().numpy(), ref['reward'])
    assert np.array_equal(out['episode_len'].cpu().numpy(), ref['episode_len'])
    host.close()
    dev.close()


def test_vecenv_surface(lr_dataset):
    import functools
    import custom_envs_amd
    from custom_envs_amd.vectorize import ThreadVecEnv
    fns = [functools.partial(custom_envs_amd.make, 'Optimize-v0', data_set=lr_dataset)] * 8
    venv = ThreadVecEnv(fns)
    assert venv.engine_backed and venv.num_envs == 8
    venv.seed(0)
    obs = venv.reset()
    assert obs.shape == (8, 41)
    obs, rews, dones, infos = venv.step(np.zeros((8, 20), np.float32))
    assert rews.shape == (8,) and dones.dtype == bool and len(infos) == 8
    assert set(infos[3]) == {'objective', 'accuracy', 'episode'}
    assert venv.get_attr('current_step') == [1] * 8
    venv.close()


def test_step_before_reset_is_an_error(lr_dataset):
    from custom_envs_amd import NativeEngineError
    eng = _engine(lr_dataset, 4)
    with pytest.raises(NativeEngineError, match='before the first reset'):
        eng.step(np.zeros((4, 20), np.float32))
    eng.close()


def test_benchmark_config_against_live_oracle(lr_dataset):
    """The bench's own configuration (config 2 as bench.py runs it): 4096
    envs, 256 x 10, B = N, the default kernel instance (4 waves, row-loop
    mode 3), seeds 0..4095, actions N(0, 0.01) -- ten envs spread over the
    grid, the first and last workgroups included (env 4095 is the last lane
    of the last group), against live oracle envs over 83 steps (two
    in-kernel auto-resets), plus their float64 weights at the end."""
    E, P, T = 4096, 20, 83
    eng = _engine(lr_dataset, E)
    assert eng.step_kernel == 'optimize_lr_mfma_kernel<3,3,4>'
    check = [0, 5, 15, 16, 1029, 2047, 2048, 3071, 4080, 4095]
    seeds = list(range(E))
    eng.seed(seeds)
    eng.reset()
    refs = {}
    for i in check:
        env = OracleEnv(*lr_dataset)
        env.seed(seeds[i])
        env.reset()
        refs[i] = env
    rs = np.random.RandomState(1234)
    for t in range(T):
        act = rs.normal(0, 0.01, (E, P)).astype(np.float32)
        out = eng.step(act)
        for i, env in refs.items():
            obs, rew, done, info = env.step(act[i])
            if done:
                obs = env.reset()
            assert bool(out['done'][i]) == done, (i, t)
            assert out['episode_len'][i] == info['episode']['l'], (i, t)
            np.testing.assert_allclose(out['obs'][i], obs, rtol=F64_RTOL, atol=F64_ATOL,
                                       err_msg='env %d step %d' % (i, t))
            assert out['reward'][i] == pytest.approx(rew, rel=F64_RTOL), (i, t)
            assert out['objective'][i] == pytest.approx(info['objective'], rel=F64_RTOL), (i, t)
            assert out['accuracy'][i] == np.float32(info['accuracy']), (i, t)
    st = eng.get_state()
    for i, env in refs.items():
        np.testing.assert_allclose(st['weights'][i], env.model.weights.ravel(), rtol=1e-12,
                                   atol=1e-14)
    eng.close()


def test_long_run_device_path_against_oracle(lr_dataset):
    """1000 steps (25 episodes, 24 in-kernel auto-resets) of the benchmark
    kernel through the bench's own device path -- chunks of 20 plain launches
    and of 50 as a replayed hipGraph -- against live oracle envs: at every
    chunk end the last step's outputs, and at the end the float64 weights and
    loss history, so no drift across episodes goes unseen
    (optimize.py:69-100, utils_venv.py:31)."""
    import torch
    E, P, T = 512, 20, 1000
    check = [0, 1, 15, 16, 255, 256, 510, 511]
    eng = _engine(lr_dataset, E)
    assert eng.step_kernel == 'optimize_lr_mfma_kernel<3,3,4>'
    eng.seed(list(range(E)))
    refs = {}
    for i in check:
        env = OracleEnv(*lr_dataset)
        env.seed(i)
        env.reset()
        refs[i] = env
    rs = np.random.RandomState(77)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        eng.set_stream(stream.cuda_stream)
        out = eng.alloc_device_outputs()
        eng.reset_device(out)
        t = 0
        while t < T:
            k = min(20 if (t // 70) % 2 == 0 else 50, T - t)
            acts = rs.normal(0, 0.01, (k, E, P)).astype(np.float32)
            eng.step_many_device(k, torch.from_numpy(acts).cuda(), out)
            stream.synchronize()
            got = {name: out[name].cpu().numpy() for name in ('obs', 'reward', 'done', 'episode_len',
                                                               'objective', 'accuracy')}
            for i, env in refs.items():
                for s in range(k):
                    obs, rew, done, info = env.step(acts[s, i])
                    if done:
                        obs = env.reset()
                assert bool(got['done'][i]) == done, (i, t + k)
                assert got['episode_len'][i] == info['episode']['l'], (i, t + k)
                np.testing.assert_allclose(got['obs'][i], obs, rtol=F64_RTOL, atol=F64_ATOL,
                                           err_msg='env %d step %d' % (i, t + k))
                assert got['reward'][i] == pytest.approx(rew, rel=F64_RTOL), (i, t + k)
                assert got['objective'][i] == pytest.approx(info['objective'], rel=F64_RTOL)
                assert got['accuracy'][i] == np.float32(info['accuracy']), (i, t + k)
            t += k
    st = eng.get_state()
    for i, env in refs.items():
        np.testing.assert_allclose(st['weights'][i], env.model.weights.ravel(), rtol=1e-12,
                                   atol=1e-14)
        assert st['step'][i] == T % 40
    eng.close()


def test_config4_global_size_on_one_gpu(lr_dataset):
    """Config 4's global batch (32,768 envs, BASELINE configs[3]) as ONE
    engine: 2048 workgroups of the benchmark kernel, eight per CU.  Sampled
    envs across the whole grid (the last lane of the last workgroup
    included) against live oracle envs over 42 steps (one auto-reset), with
    device-resident actions and outputs, plus a 4096-env engine seeded with
    the same global indices giving the same bits for its envs (seeds =
    global index: a shard of the batch reproduces the whole)."""
    import torch
    E, P, T = 32768, 20, 42
    sample = [0, 17, 4095, 4096, 16383, 20000, 32766, 32767]
    eng = _engine(lr_dataset, E)
    assert eng.step_kernel == 'optimize_lr_mfma_kernel<3,3,4>'
    eng.seed(list(range(E)))
    part = _engine(lr_dataset, 4096)
    part.seed(list(range(16384, 16384 + 4096)))
    refs = {}
    for i in sample:
        env = OracleEnv(*lr_dataset)
        env.seed(i)
        env.reset()
        refs[i] = env
    out = eng.alloc_device_outputs()
    pout = part.alloc_device_outputs()
    eng.reset_device(out)
    part.reset_device(pout)
    gen = torch.Generator(device='cuda')
    gen.manual_seed(4)
    acts = torch.empty((E, P), dtype=torch.float32, device='cuda')
    idx = torch.tensor(sample, device='cuda')
    for t in range(T):
        acts.normal_(0.0, 0.01, generator=gen)
        torch.cuda.synchronize()
        eng.step_device(acts, out)
        part.step_device(acts[16384:16384 + 4096].contiguous(), pout)
        eng.wait()
        part.wait()
        a = acts.index_select(0, idx).cpu().numpy()
        got = {k: out[k].index_select(0, idx).cpu().numpy()
               for k in ('obs', 'reward', 'done', 'episode_len', 'objective', 'accuracy')}
        for j, i in enumerate(sample):
            obs, rew, done, info = refs[i].step(a[j])
            if done:
                obs = refs[i].reset()
            assert bool(got['done'][j]) == done, (i, t)
            assert got['episode_len'][j] == info['episode']['l'], (i, t)
            np.testing.assert_allclose(got['obs'][j], obs, rtol=F64_RTOL, atol=F64_ATOL,
                                       err_msg='env %d step %d' % (i, t))
            assert got['reward'][j] == pytest.approx(rew, rel=F64_RTOL), (i, t)
            assert got['accuracy'][j] == np.float32(info['accuracy']), (i, t)
        for k in ('obs', 'reward', 'episode_len'):
            assert torch.equal(out[k][16384:16384 + 4096], pout[k]), (k, t)
    eng.close()
    part.close()
