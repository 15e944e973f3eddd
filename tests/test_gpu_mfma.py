"""The runtime-shape f64 MFMA step kernel (optimize_mfma_kernel.h) against
the CPU oracle: the reference's own image-set shape (7x7 = 49 features, 10
classes; load_data('mnist'), optimize.py:40) through the real IDX loader,
ragged N (padded LDS blocks), minibatches, every feature-tile count, the
largest K, odd env counts (a partial workgroup), across auto-resets; and the
shapes the register kernels serve, forced onto this kernel (CE_GENERIC=1).
Tolerance as test_gpu_parity.py: float64 results rounded to float32 within
1e-6 relative (atol 1e-9), accuracy exact."""
import os

import numpy as np
import pytest

from conftest import GOLDEN, golden
from oracle.optimize import Optimize as OracleEnv

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _need_gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail('GPU tests need a ROCm device (run under gpurun)')


def _engine(dataset, num_envs, batch_size=None, generic=False, lr=False, lr_waves=0, gen_tail=1,
            lr_mode=3, cat=False, **kw):
    """cat=False keeps full-batch shapes on the one-env-per-wave kernel
    (CE_GEN_CAT=0); cat=True lets the class-concatenated kernel take them."""
    from custom_envs_amd.engine import OptimizeEngine
    flags = {'CE_GENERIC': '1' if generic else '0', 'CE_LR_MFMA': '1' if lr else '0',
             'CE_LR_WAVES': str(lr_waves), 'CE_GEN_TAIL': str(gen_tail),
             'CE_LR_MODE': str(lr_mode), 'CE_GEN_CAT': '1' if cat else '0'}
    old = {k: os.environ.get(k) for k in flags}
    os.environ.update(flags)
    try:
        return OptimizeEngine(*dataset, num_envs=num_envs, batch_size=batch_size, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k)
            else:
                os.environ[k] = v


def _classes(n_rows, n_features, n_classes, seed):
    rs = np.random.RandomState(seed)
    centers = rs.normal(0, 1.0, (n_classes, n_features))
    y = rs.randint(0, n_classes, n_rows)
    x = centers[y] + rs.normal(0, 1.0, (n_rows, n_features))
    return x, np.eye(n_classes)[y]


def _check(dataset, batch_size, eng, envs, steps, seed0=11, scale=0.02):
    E, P = eng.num_envs, eng.act_dim
    seeds = [seed0 + 3 * i for i in range(E)]
    acts = np.random.RandomState(E + P).normal(0, scale, (steps, E, P)).astype(np.float32)
    eng.seed(seeds)
    assert np.all(eng.reset() == 0)
    refs = {}
    for i in envs:
        env = OracleEnv(*dataset, batch_size=batch_size)
        env.seed(seeds[i])
        env.reset()
        refs[i] = env
    for t in range(steps):
        out = eng.step(acts[t])
        for i, env in refs.items():
            obs, rew, done, info = env.step(acts[t, i])
            if done:
                obs = env.reset()
            assert bool(out['done'][i]) == done, (i, t)
            assert out['episode_len'][i] == info['episode']['l']
            np.testing.assert_allclose(out['obs'][i], obs, rtol=1e-6, atol=1e-9,
                                       err_msg='env %d step %d' % (i, t))
            assert out['reward'][i] == pytest.approx(rew, rel=1e-6)
            assert out['objective'][i] == pytest.approx(info['objective'], rel=1e-6)
            assert out['accuracy'][i] == np.float32(info['accuracy']), (i, t)
    return refs


def test_mnist_idx_fixture_through_make():
    """make('Optimize-v0', data_set='mnist', data_dir=...) on the committed
    synthetic IDX files: the reference's default data set shape (F = 49,
    K = 10) runs, on the MFMA kernel, and matches the oracle."""
    from custom_envs_amd import make
    from custom_envs_amd.data import load_data
    data_dir = os.path.join(GOLDEN, 'idx')
    env = make('Optimize-v0', data_set='mnist', data_dir=data_dir)
    # NK = ceil(49 / 4); the full batch of the 8-env class-concatenated kernel
    assert env.engine.step_kernel == 'optimize_cat_kernel<13,true,10>'
    assert env.observation_space.shape == (2 * 490 + 1,) and env.action_space.shape == (490,)
    seq = load_data('mnist', batch_size=None, data_dir=data_dir)
    ref = OracleEnv(seq.features, seq.targets)
    env.seed(3)
    ref.seed(3)
    np.testing.assert_array_equal(env.reset(), ref.reset())
    acts = np.random.RandomState(0).normal(0, 0.05, (42, 490)).astype(np.float32)
    for t in range(42):
        obs, rew, done, info = env.step(acts[t])
        robs, rrew, rdone, rinfo = ref.step(acts[t])
        assert done == rdone and info['episode']['l'] == rinfo['episode']['l']
        np.testing.assert_allclose(obs, robs, rtol=1e-6, atol=1e-9)
        assert rew == pytest.approx(rrew, rel=1e-6)
        assert info['accuracy'] == np.float32(rinfo['accuracy'])
        if done:
            break
    env.close()


@pytest.mark.parametrize('batch_size', [None, 32, 100])
def test_image_shape_many_envs(batch_size):
    """49 x 10 at N = 1000 (not a multiple of the 64-row block), 13 envs
    (one full and one partial workgroup), 43 steps across an auto-reset."""
    ds = _classes(1000, 49, 10, 1)
    eng = _engine(ds, 13, batch_size)
    assert eng.step_kernel == 'optimize_mfma_kernel<13>'
    _check(ds, batch_size, eng, [0, 7, 8, 12], 43)
    eng.close()


@pytest.mark.parametrize('gen_tail', [1, 0])
@pytest.mark.parametrize('shape', [(4, 3), (17, 2), (33, 7), (64, 16), (49, 10), (1, 5)])
def test_every_feature_tile_count(shape, gen_tail):
    """Every feature-tile count; F = 17, 33, 49 (one feature in the last
    k-step and tile) with the last feature on the VALU (gen_tail=1, the
    default for the full data set) and on the matrix pipe (gen_tail=0)."""
    F, K = shape
    ds = _classes(300, F, K, F + K)
    eng = _engine(ds, 9, None, generic=True, gen_tail=gen_tail)
    assert eng.step_kernel == 'optimize_mfma_kernel<%d>' % ((F + 3) // 4)
    _check(ds, None, eng, [0, 8], 41)
    eng.close()


@pytest.mark.parametrize('batch_size', [None, 32])
def test_register_shapes_forced_generic(lr_dataset, batch_size):
    """The benchmark shape (256 x 10, K = 2) on the MFMA kernel agrees with
    the oracle as the register kernels do."""
    eng = _engine(lr_dataset, 10, batch_size, generic=True)
    assert eng.step_kernel == 'optimize_mfma_kernel<3>'
    _check(lr_dataset, batch_size, eng, [0, 9], 42)
    eng.close()


@pytest.mark.parametrize('name', ['ref_optimize_s0', 'ref_optimize_b32_s3'])
def test_generic_vs_reference_code(lr_dataset, name):
    fx = golden(name + '.npz')
    bs = int(fx['batch_size'])
    eng = _engine(lr_dataset, 1, None if bs < 0 else bs, generic=True)
    eng.seed([int(fx['seed'])])
    eng.reset()
    for t in range(fx['actions'].shape[0]):
        out = eng.step(fx['actions'][t][None])
        assert bool(out['done'][0]) == bool(fx['done'][t])
        np.testing.assert_allclose(out['obs'][0], fx['obs'][t], rtol=1e-6, atol=1e-9)
        assert out['accuracy'][0] == np.float32(fx['accuracy'][t])
    eng.close()


def test_state_roundtrip_and_device_path():
    """get/set_state and the device-pointer path on the MFMA kernel."""
    import torch
    ds = _classes(200, 49, 10, 7)
    eng = _engine(ds, 5, 32)
    eng.seed(list(range(5)))
    eng.reset()
    acts = np.random.RandomState(1).normal(0, 0.02, (3, 5, 490)).astype(np.float32)
    for t in range(3):
        eng.step(acts[t])
    st = eng.get_state()
    host = {k: v.copy() for k, v in eng.step(acts[0]).items()}
    eng.set_state(**st)
    out = eng.alloc_device_outputs()
    eng.step_device(torch.from_numpy(acts[0]).cuda(), out)
    eng.wait()
    np.testing.assert_array_equal(out['obs'].cpu().numpy(), host['obs'])
    np.testing.assert_array_equal(out['accuracy'].cpu().numpy(), host['accuracy'])
    eng.close()


def test_unsupported_shapes_fail_loudly():
    from custom_envs_amd._native import NativeEngineError
    ds = _classes(64, 65, 3, 0)
    with pytest.raises(NativeEngineError, match='F <= 64'):
        _engine(ds, 2)
    ds = _classes(64, 49, 10, 0)
    with pytest.raises(NativeEngineError, match='float64'):
        _engine(ds, 2, precision='f32')


# ---------------------------------------------------------------------------
# The two-class full-batch kernel with envs on the MFMA N dimension
# (optimize_lr_mfma.h; the default, CE_LR_MFMA=0 selects the register
# kernel) for K = 2, F <= 16, B = N in float64.

def _two_class(n_rows, n_features, seed):
    rs = np.random.RandomState(seed)
    x = rs.normal(0, 1.0, (n_rows, n_features))
    y = (x @ rs.normal(size=n_features) + rs.normal(0, 0.7, n_rows) > 0).astype(int)
    return x, np.eye(2)[y]


@pytest.mark.parametrize('lr_waves', [8, 4, 16])
@pytest.mark.parametrize('n_rows,n_features,num_envs', [
    (256, 10, 37), (200, 1, 16), (203, 13, 17), (1000, 16, 5), (4000, 4, 3), (256, 5, 1),
    (384, 7, 21), (512, 3, 33), (1024, 10, 18)])
def test_lr_mfma_kernel_matches_oracle(n_rows, n_features, num_envs, lr_waves):
    """Ragged row tiles (N % 16 != 0), partial 16-env groups, every k-step
    count, many tiles per wave (the cross-entropy product folds), and the
    four row-loop modes (lr_mode: 8 waves -- 256, 512, 1024 tile pairs, 384
    one unmasked tile at a time, the others masked; 4 waves -- 256, 1024
    groups of 4 tiles, 384 pairs; 16 waves -- one tile at a time), at every
    wave count (4 waves: two (env, parameter) roles per thread)."""
    ds = _two_class(n_rows, n_features, n_rows + n_features)
    eng = _engine(ds, num_envs, None, lr=True, lr_waves=lr_waves)
    assert eng.step_kernel.startswith('optimize_lr_mfma_kernel<%d,' % ((n_features + 3) // 4))
    envs = sorted({0, num_envs // 2, num_envs - 1})
    _check(ds, None, eng, envs, 43)
    eng.close()


@pytest.mark.parametrize('lr_mode', [0, 1, 2])
@pytest.mark.parametrize('lr_waves', [4, 8])
def test_lr_mfma_mode_caps(lr_mode, lr_waves):
    """CE_LR_MODE caps the row-loop mode below what the shape allows: the
    benchmark shape (256 x 10) with every tile masked one at a time (0),
    unmasked one at a time (1) and in pairs (2), at 4 and 8 waves."""
    ds = _two_class(256, 10, 3)
    eng = _engine(ds, 35, None, lr=True, lr_waves=lr_waves, lr_mode=lr_mode)
    assert eng.step_kernel == 'optimize_lr_mfma_kernel<3,%d,%d>' % (lr_mode, lr_waves)
    _check(ds, None, eng, [0, 16, 34], 42)
    eng.close()


def test_lr_mfma_agrees_with_register_kernel(lr_dataset):
    """Same envs through the MFMA kernel and the two-envs-per-wave register
    kernel (CE_LR_MFMA=0): float64 results agree to float32
    rounding."""
    E, T = 64, 45
    acts = np.random.RandomState(3).normal(0, 0.02, (T, E, 20)).astype(np.float32)
    outs = []
    for flag in ('1', '0'):
        eng = _engine(lr_dataset, E, None, lr=flag == '1')
        assert ('lr_mfma' in eng.step_kernel) == (flag == '1')
        eng.seed(list(range(E)))
        eng.reset()
        outs.append([{k: v.copy() for k, v in eng.step(acts[t]).items()} for t in range(T)])
        eng.close()
    for a, b in zip(*outs):
        np.testing.assert_allclose(a['obs'], b['obs'], rtol=2e-6, atol=1e-9)
        assert np.array_equal(a['done'], b['done'])
        assert np.array_equal(a['episode_len'], b['episode_len'])
        assert np.array_equal(a['accuracy'], b['accuracy'])


@pytest.mark.parametrize('n_rows', [256, 203])
@pytest.mark.parametrize('lr', [True, False])
def test_two_class_ties_take_class_zero(n_rows, lr):
    """Zero rows give z = 0 exactly, a probability tie whatever the weights:
    np.argmax then picks class 0, so such a row is a hit iff y == 0.  The
    two-class kernels count hits as z > 0 and re-walk a wave's rows only when
    max(t) == 1 flags a tie (the LR MFMA kernel with and without padding
    rows, and the register pair kernel)."""
    x, y = _two_class(n_rows, 10, 5)
    x[::7] = 0.0                       # ties, of both labels
    eng = _engine((x, y), 19, None, lr=lr)
    assert ('lr_mfma' in eng.step_kernel) == lr
    _check((x, y), None, eng, [0, 9, 18], 12)
    eng.close()


def test_image_shape_full_size():
    """The reference's default data shape at its real size: load_data('mnist')
    gives 60,000 rows of 7 x 7 = 49 features and 10 classes, batch_size=None
    (optimize.py:40, load_data.py:65-71).  The bench's data set
    (mnist7x7_synthetic), 9 envs (one full 8-env workgroup and a partial
    one), 42 steps across an auto-reset, against the oracle: the f64
    gradient sums and the per-lane cross-entropy product folded every 16
    factors accumulate over all 60,000 rows."""
    from custom_envs_amd.data import load_data
    seq = load_data('mnist7x7_synthetic', batch_size=None)
    ds = (seq.features, seq.targets)
    assert ds[0].shape == (60000, 49) and ds[1].shape == (60000, 10)
    for cat, kernel in ((True, 'optimize_cat_kernel<13,true,10>'), (False, 'optimize_mfma_kernel<13>')):
        eng = _engine(ds, 9, None, cat=cat)
        assert eng.step_kernel == kernel
        _check(ds, None, eng, [0, 7, 8], 42, scale=0.01)
        eng.close()


@pytest.mark.parametrize('shape', [(49, 10, 1000), (17, 10, 300), (16, 10, 203), (12, 3, 300),
                                   (32, 16, 130)])
def test_class_concatenated_kernel(shape):
    """The full-batch class-concatenated kernel (optimize_cat_kernel.h) at
    every compiled shape: the image sets' 49 x 10 with a ragged last row
    block (N = 1000), the VALU tail at F = 17, no tail (F = 16), class
    padding in the last tile (K = 3: 24 class-pairs in 2 tiles of 16) and
    K = 16; 13 envs (a full 8-env workgroup and a partial one), across an
    auto-reset."""
    F, K, N = shape
    ds = _classes(N, F, K, F + K + N)
    eng = _engine(ds, 13, None, cat=True)
    nk = (F + 3) // 4
    tail = 'true' if F == 4 * (nk - 1) + 1 and nk % 4 == 1 and nk > 1 else 'false'
    assert eng.step_kernel == 'optimize_cat_kernel<%d,%s,%d>' % (nk, tail, K)
    _check(ds, None, eng, [0, 7, 8, 12], 43)
    eng.close()


def test_class_concatenated_agrees_with_per_env_kernel():
    """The same 12 envs through both full-batch kernels: float64 results
    agree to float32 rounding, done / episode length / accuracy exactly."""
    ds = _classes(640, 49, 10, 3)
    E, T = 12, 42
    acts = np.random.RandomState(3).normal(0, 0.02, (T, E, 490)).astype(np.float32)
    outs = []
    for cat in (True, False):
        eng = _engine(ds, E, None, cat=cat)
        eng.seed(list(range(E)))
        eng.reset()
        outs.append([{k: v.copy() for k, v in eng.step(acts[t]).items()} for t in range(T)])
        eng.close()
    for a, b in zip(*outs):
        np.testing.assert_allclose(a['obs'], b['obs'], rtol=2e-6, atol=1e-9)
        assert np.array_equal(a['done'], b['done'])
        assert np.array_equal(a['episode_len'], b['episode_len'])
        assert np.array_equal(a['accuracy'], b['accuracy'])


@pytest.mark.parametrize('lr_waves', [4, 8])
def test_lr_mfma_extreme_logits(lr_waves):
    """Envs whose weights reach |u| far past the exp's range (actions of scale
    40 on some envs) next to ordinary ones: workgroups whose |u| bound stays
    below 650 run the row loop without the argument clamp, the others with it
    (CE_LR_NOCLAMP); p_y + 1e-16 and q must match the oracle's max-subtracted
    softmax either way, including p_y underflowing to 0."""
    ds = _two_class(256, 10, 21)
    E, T = 40, 42
    eng = _engine(ds, E, None, lr=True, lr_waves=lr_waves)
    P = eng.act_dim
    scale = np.where(np.arange(E) >= 32, 40.0, 0.01)          # the last group: huge weights
    scale[5] = 40.0                                            # and one env in the first group
    acts = (np.random.RandomState(4).normal(0, 1, (T, E, P)) * scale[None, :, None]).astype(np.float32)
    seeds = [300 + i for i in range(E)]
    eng.seed(seeds)
    eng.reset()
    check = [0, 5, 16, 31, 32, 39]
    refs = {}
    for i in check:
        env = OracleEnv(*ds)
        env.seed(seeds[i])
        env.reset()
        refs[i] = env
    for t in range(T):
        out = eng.step(acts[t])
        for i, env in refs.items():
            obs, rew, done, info = env.step(acts[t, i])
            if done:
                obs = env.reset()
            assert bool(out['done'][i]) == done
            np.testing.assert_allclose(out['obs'][i], obs, rtol=1e-6, atol=1e-9,
                                       err_msg='env %d step %d' % (i, t))
            assert out['reward'][i] == pytest.approx(rew, rel=1e-6)
            assert out['accuracy'][i] == np.float32(info['accuracy'])
    eng.close()
