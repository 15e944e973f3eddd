"""Pins against outputs of the REFERENCE's own code (CPU).

tests/golden/ref_*.npz were produced by oracle/gen_ref_pins.py, which runs
the reference's own definitions (Optimize, BaseEnvironment, InMemoryDataSet,
the VecEnv workers' auto-reset, MultiOptLRs, OptEnvRunner, History,
utils_env, load_data's IDX branches, utils_image's PIL resize) from their
source text in the build container.  Here the CPU oracle -- the checker the
GPU parity tests use -- and the package's host functions must reproduce them.
The missing ModelNumpy and the TF problems are build-defined in both, so
these pins cover the env/dataset/vectorize logic around the model.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN, REFERENCE, golden


@pytest.mark.parametrize('name,seed,batch_size,steps,action_seed', [
    ('ref_optimize_s0', 0, None, 45, 1234), ('ref_optimize_s1', 1, None, 45, 1235),
    ('ref_optimize_b32_s3', 3, 32, 85, 102)])
def test_oracle_optimize_is_the_reference(lr_dataset, name, seed, batch_size, steps,
                                          action_seed):
    """Bit for bit: the reference's Optimize / BaseEnvironment / InMemoryDataSet
    / utils_venv._worker vs the oracle, over the same A7 model."""
    from oracle.gen_golden import rollout
    ref = golden(name + '.npz')
    got = rollout(*lr_dataset, seed, batch_size, steps, action_seed)
    np.testing.assert_array_equal(got['actions'], ref['actions'])
    np.testing.assert_array_equal(got['reset_obs'], ref['reset_obs'])
    for key in ('obs', 'reward', 'done', 'objective', 'accuracy', 'ep_len', 'weights'):
        np.testing.assert_array_equal(got[key], ref[key], err_msg=key)


@pytest.mark.parametrize('name,ndims,max_batches,hist,steps,seed,low,high', [
    ('ref_multi_func4_h5', 4, 400, 5, 60, 8, 1.0, 3.0),
    ('ref_multi_func4_h3_b25', 4, 25, 3, 90, 9, -1.0, 0.7)])
def test_oracle_multioptlrs_matches_the_reference(name, ndims, max_batches, hist, steps, seed,
                                                  low, high):
    """The reference's MultiOptLRs / History / utils_env / OptEnvRunner /
    concurrentvecenv._worker.  Exact: done, episode length, and every state
    of the stable case.  The reference's float32 ``10**(a - 4)`` is numpy's
    SIMD pow (1 ulp off the correctly rounded value on ~25 % of inputs, the
    oracle and the engine round correctly), so the divergent case agrees to
    float32 rounding."""
    from oracle.gen_golden import rollout_multi
    ref = golden(name + '.npz')
    got = rollout_multi(ndims, max_batches, hist, steps, seed, low, high)
    np.testing.assert_array_equal(got['done'], ref['done'])
    np.testing.assert_array_equal(got['ep_len'], ref['ep_len'])
    np.testing.assert_array_equal(got['reset_obs'], ref['reset_obs'])
    live = ~ref['done']          # the reference worker resets before theta is read
    np.testing.assert_allclose(got['theta'][live], ref['theta'][live], rtol=1e-6)
    np.testing.assert_allclose(got['obs'], ref['obs'], rtol=1e-5, atol=1e-12)
    np.testing.assert_allclose(got['reward'], ref['reward'], rtol=1e-5)
    np.testing.assert_allclose(got['info'], ref['info'], rtol=1e-5, equal_nan=True)
    if name.endswith('b25'):
        np.testing.assert_array_equal(got['obs'], ref['obs'])
        np.testing.assert_array_equal(got['theta'][live], ref['theta'][live])


def test_utils_env_is_the_reference():
    """custom_envs_amd.utils.utils_env == the reference's utils_env, every version."""
    from custom_envs_amd.utils import utils_env
    from custom_envs_amd.utils.utils_common import History
    vec = golden('ref_utils_env.npz')
    for version in range(4):
        hist = History(3, weights=(6,), losses=(), gradients=(6,))
        w, l, g = (vec['obs_in_%s_v%d' % (k, version)] for k in 'wlg')
        for i in (2, 1, 0):                 # oldest first
            hist.append(weights=w[i], losses=l[i], gradients=g[i])
        loss, wght, grad = utils_env.get_observation(hist, version)
        assert loss == float(vec['obs_loss_v%d' % version])
        np.testing.assert_array_equal(wght, vec['obs_wght_v%d' % version])
        np.testing.assert_array_equal(grad, vec['obs_grad_v%d' % version])
    for version in range(7):
        got = [utils_env.get_reward(lv, av, version)
               for lv, av in zip(vec['reward_loss'], vec['reward_adjusted'])]
        np.testing.assert_array_equal(got, vec['reward'][version])
    for version in range(4):
        got = utils_env.get_action_optlrs(vec['action_in'], version)
        np.testing.assert_array_equal(np.asarray(got, np.float64), vec['action'][version])


def test_load_data_idx_is_the_reference():
    """The reference's load_data('mnist' | 'mnist-test') (IDX .xz, PIL
    NEAREST 28x28 -> 7x7, normalize, to_onehot) on the committed synthetic
    IDX fixture: this package's reader gives the same arrays bit for bit."""
    from custom_envs_amd.data import load_data
    ref = golden('ref_load_data.npz')
    data_dir = os.path.join(GOLDEN, 'idx')
    for name in ('mnist', 'mnist-test'):
        seq = load_data(name, batch_size=None, data_dir=data_dir)
        key = name.replace('-', '_')
        assert seq.features.shape[1] == 49 and seq.targets.shape[1] == 10
        np.testing.assert_array_equal(seq.features, ref[key + '_features'])
        np.testing.assert_array_equal(seq.targets, ref[key + '_targets'])


@pytest.mark.parametrize('shape', [(7, 7), (5, 9), (14, 3)])
def test_resize_nearest_is_pil(shape):
    """files.resize_nearest == utils_image.resize_array_many (PIL NEAREST)."""
    from custom_envs_amd.data.files import resize_nearest
    ref = golden('ref_load_data.npz')
    got = resize_nearest(ref['resize_in'], shape)
    np.testing.assert_array_equal(got, ref['resize_%dx%d' % shape])


@pytest.mark.skipif(not os.path.isdir(os.path.join(REFERENCE, 'custom_envs')),
                    reason='reference sources only in the build container')
def test_resize_nearest_live_against_reference_pil():
    """Live: the reference's resize_array_many (numpy + PIL, both importable
    here) on random images and shapes."""
    from PIL import Image
    from custom_envs_amd.data.files import resize_nearest
    from oracle.refexec import load
    img = load('custom_envs/utils/utils_image.py', ['resize_array', 'resize_array_many'],
               {'np': np, 'Image': Image})
    rs = np.random.RandomState(0)
    for h, w, shape in ((28, 28, (7, 7)), (28, 28, (13, 6)), (17, 23, (7, 11)),
                        (9, 9, (20, 4))):
        images = rs.randint(0, 256, (4, h, w)).astype(np.uint8)
        np.testing.assert_array_equal(resize_nearest(images, shape),
                                      np.stack(img['resize_array_many'](images, shape)))
