"""Every bench workload's kernel against the oracle AT ITS BENCH SIZE.

The bench lines run config 2 in float32 at 1024 envs, the image shape at
4096 envs and the default (256, 256) network at 1024 envs; the kernels
that run there (the float32 two-class register kernel, the
class-concatenated f64 MFMA kernel, the layered network path's persistent
XCD-walking gradient grid) are compared here with live oracle envs sampled
across the whole grid (first / last lanes of workgroups, the last env),
through the reference step (optimize.py:69-100 with the utils_venv.py:31
auto-reset; the network problem optimize_nn.py:22-64 as A12 restates it).

Tolerances (as the per-kernel test files):
  - float32 two-class kernel: per obs row ||d||_inf / ||ref||_inf <= 1e-5
    (the north-star bound), elementwise 1e-3 where |ref| >= 1e-2 ||ref||_inf;
    reward / objective 1e-5 relative; done, lengths, accuracy exact;
  - float64 kernels: obs within 1e-6 relative (atol 1e-9) -- float64
    results rounded to float32; accuracy exact;
  - the float32 network: test_gpu_mlp.py's _row_close rule (per row 1e-5
    relative to the row max), with its relu-tie rule (_relu_ties,
    _tie_variant_rows) -- a minibatch pre-activation within float32 rounding
    of 0 may take either side of the relu.
"""
import numpy as np
import pytest

from oracle.optimize import Optimize as OracleEnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a ROCm device (run under gpurun)')


def _close_f32_rows(got, ref, tol=1e-5, elem_tol=1e-3, elem_floor=1e-2, what=''):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    scale = max(np.abs(ref).max(), 1e-30)
    assert np.abs(got - ref).max() / scale <= tol, (what, np.abs(got - ref).max() / scale)
    big = np.abs(ref) >= elem_floor * scale
    rel = np.abs(got - ref) / np.maximum(np.abs(ref), 1e-30)
    assert np.all(rel[big] <= elem_tol), (what, rel[big].max())


def test_config2_f32_at_1024_envs(lr_dataset):
    """BASELINE configs[1]: 1024 parallel Optimize-v0 envs, logistic
    regression 256 x 10, fp32 -- the float32 two-class kernel at 1024 envs,
    envs 0, 15, 16, 511 and 1023 over 45 steps (one auto-reset)."""
    from custom_envs_amd.engine import OptimizeEngine
    E, P, T = 1024, 20, 45
    sample = [0, 15, 16, 511, 1023]
    eng = OptimizeEngine(*lr_dataset, num_envs=E, precision='f32')
    assert eng.step_kernel.startswith('optimize_pair_kernel<float,10,')
    eng.seed(list(range(E)))
    assert np.all(eng.reset() == 0)
    refs = {}
    for i in sample:
        env = OracleEnv(*lr_dataset)
        env.seed(i)
        env.reset()
        refs[i] = env
    rs = np.random.RandomState(2024)
    resets = 0
    for t in range(T):
        act = rs.normal(0, 0.01, (E, P)).astype(np.float32)
        out = eng.step(act)
        for i, env in refs.items():
            obs, rew, done, info = env.step(act[i])
            where = 'env %d step %d' % (i, t)
            assert bool(out['done'][i]) == done, where
            assert out['episode_len'][i] == info['episode']['l'], where
            if done:
                resets += 1
                assert np.all(out['obs'][i] == 0), where       # the reset observation
                env.reset()
            else:
                _close_f32_rows(out['obs'][i], obs, what=where)
            assert out['reward'][i] == pytest.approx(rew, rel=1e-5), where
            assert out['objective'][i] == pytest.approx(info['objective'], rel=1e-5), where
            assert out['accuracy'][i] == np.float32(info['accuracy']), where
    assert resets == len(sample)
    st = eng.get_state()
    for i, env in refs.items():
        np.testing.assert_allclose(st['weights'][i], env.model.weights.ravel(), rtol=1e-6,
                                   atol=1e-6)
    eng.close()


def test_image_shape_at_4096_envs():
    """The image-shape bench line: load_data('mnist') shape (60,000 x 49, 10
    classes, B = N) on the class-concatenated kernel at 4096 envs (512
    workgroups of 8 envs): envs 0, 7, 8, 2047 and 4095 over 41 steps (one
    auto-reset), device-resident actions and outputs as in bench.py."""
    import torch
    from custom_envs_amd.data import load_data
    from custom_envs_amd.engine import OptimizeEngine
    seq = load_data('mnist7x7_synthetic', batch_size=None)
    ds = (seq.features, seq.targets)
    E, T = 4096, 41
    sample = [0, 7, 8, 2047, 4095]
    eng = OptimizeEngine(*ds, num_envs=E)
    assert eng.step_kernel == 'optimize_cat_kernel<13,true,10>'
    P = eng.act_dim
    eng.seed(list(range(E)))
    out = eng.alloc_device_outputs()
    eng.reset_device(out)
    refs = {}
    for i in sample:
        env = OracleEnv(*ds)
        env.seed(i)
        env.reset()
        refs[i] = env
    gen = torch.Generator(device='cuda')
    gen.manual_seed(17)
    acts = torch.empty((E, P), dtype=torch.float32, device='cuda')
    idx = torch.tensor(sample, device='cuda')
    for t in range(T):
        acts.normal_(0.0, 0.01, generator=gen)
        torch.cuda.synchronize()
        eng.step_device(acts, out)
        eng.wait()
        a = acts.index_select(0, idx).cpu().numpy()
        got = {k: out[k].view(E, -1).index_select(0, idx).cpu().numpy()
               for k in ('obs', 'reward', 'done', 'objective', 'accuracy', 'episode_len')}
        for j, i in enumerate(sample):
            obs, rew, done, info = refs[i].step(a[j])
            if done:
                obs = refs[i].reset()
            where = 'env %d step %d' % (i, t)
            assert bool(got['done'][j, 0]) == done, where
            assert got['episode_len'][j, 0] == info['episode']['l'], where
            np.testing.assert_allclose(got['obs'][j], obs, rtol=1e-6, atol=1e-9, err_msg=where)
            assert got['reward'][j, 0] == pytest.approx(rew, rel=1e-6), where
            assert got['objective'][j, 0] == pytest.approx(info['objective'], rel=1e-6), where
            assert got['accuracy'][j, 0] == np.float32(info['accuracy']), where
    st = eng.get_state()
    for i, env in refs.items():
        np.testing.assert_allclose(st['weights'][i], env.model.weights.ravel(), rtol=1e-12,
                                   atol=1e-14)
    eng.close()


def test_network_256x256_at_1024_envs():
    """The network bench line: Optimize-v0 over create_neural_net's default
    (256, 256) network (784-256-256-10, P = 269,322), B = 32 of N = 1024, at
    1024 envs -- the regime where net_grad_kernel's XCD-walking grid has
    work on every workgroup.  Envs 0, 1, 511, 512, 1022 and 1023 over 41
    steps (one auto-reset), device-resident actions and outputs."""
    import torch
    from test_gpu_mlp import RTOL, _rel, _relu_ties, _row_close, _tie_variant_rows
    from custom_envs_amd.data import load_data
    from custom_envs_amd.engine import OptimizeEngine
    seq = load_data('mnist_synthetic', batch_size=32)
    E, T = 1024, 41
    sample = [0, 1, 511, 512, 1022, 1023]
    hidden = (256, 256)
    eng = OptimizeEngine(seq.features, seq.targets, num_envs=E, batch_size=32, model='mlp',
                         hidden=hidden)
    try:
        assert eng.step_kernel == 'net<784,256,256,10>:mfma'
        P = eng.act_dim
        eng.seed(list(range(E)))
        out = eng.alloc_device_outputs()
        eng.reset_device(out)
        eng.wait()
        refs = []
        for s in sample:
            env = OracleEnv(seq.features, seq.targets, batch_size=32, model='mlp', hidden=hidden)
            env.seed(s)
            env.reset()
            refs.append(env)
        gen = torch.Generator(device='cuda')
        gen.manual_seed(4242)
        acts = torch.empty((E, P), dtype=torch.float32, device='cuda')
        idx = torch.tensor(sample, device='cuda')
        ties = 0
        n_rows = len(seq.features)
        for t in range(T):
            acts.normal_(0.0, 1e-3, generator=gen)
            torch.cuda.synchronize()
            eng.step_device(acts, out)
            eng.wait()
            a = acts.index_select(0, idx).cpu().numpy()
            obs_e = out['obs'].view(E, -1).index_select(0, idx).cpu().numpy()
            got = {k: out[k].index_select(0, idx).cpu().numpy()
                   for k in ('reward', 'done', 'objective', 'accuracy', 'episode_len')}
            for j, env in enumerate(refs):
                where = 'env %d step %d' % (sample[j], t)
                w_new = env.model.weights - a[j]
                X, Y = env.sequence[0]
                tie = _relu_ties(env.model, w_new, X)
                g_prev = env.grad_hist[env.current_step % 3].ravel().copy()
                obs, reward, done, info = env.step(a[j])
                if done:
                    obs = env.reset()
                assert bool(got['done'][j]) == done, where
                assert int(got['episode_len'][j]) == info['episode']['l'], where
                assert not obs_e[j][:P].any(), where
                if tie and not done:
                    ties += 1
                    if len(tie) <= 4:
                        rows = _tie_variant_rows(env.model, w_new, X, Y, g_prev, obs[P], tie)
                        errs = []
                        for k, row in enumerate(rows):
                            try:
                                _row_close(obs_e[j], row, what=where)
                                break
                            except AssertionError as exc:
                                errs.append(str(exc))
                        else:
                            raise AssertionError('no side choice of %d relu ties matches: %s'
                                                 % (len(tie), errs[0]))
                        if k:   # the engine took the other side: follow its gradient history
                            env.grad_hist[env.current_step % 3] = \
                                obs_e[j][P + 1:].astype(np.float64).reshape(
                                    env.grad_hist[env.current_step % 3].shape)
                    else:
                        scale_r = max(np.abs(obs).max(), 1e-30)
                        bad = np.abs(obs_e[j].astype(np.float64) - obs) > RTOL * scale_r
                        assert bad.mean() <= 5e-3, (where, int(bad.sum()))
                else:
                    _row_close(obs_e[j], obs, what=where)
                assert _rel(got['reward'][j], reward) <= RTOL, where
                assert _rel(got['objective'][j], info['objective']) <= RTOL, where
                assert abs(float(got['accuracy'][j]) - info['accuracy']) <= 1.5 / n_rows, where
        # step 41 opened a new episode: W = W0 - a, one float32 subtraction
        st = eng.get_state()
        for j, env in enumerate(refs):
            assert np.array_equal(st['weights'][sample[j]].astype(np.float32), env.model.weights)
    finally:
        eng.close()
