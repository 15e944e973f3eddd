"""The CPU oracle against its golden fixtures and the reference's own pieces.

Pins:
  - committed rollouts regenerate bit for bit (the oracle is deterministic);
  - the restated shuffle / to_onehot / History agree with the reference's
    importable ``custom_envs/utils/utils_common.py`` (imported by file path,
    only when /root/reference exists: it never travels to the GPU box);
  - property tests the reference's tests hold for softmax / cross-entropy /
    use_random_state (tests/utils/test_utils_math.py:17-66).
"""
import importlib.util
import os

import numpy as np
import numpy.random as npr
import pytest

from conftest import REFERENCE, golden
from oracle import optimize as ref
from oracle.gen_golden import SEEDS, rollout
from oracle.seeding import np_random, seed_key


def _reference_utils_common():
    path = os.path.join(REFERENCE, 'custom_envs', 'utils', 'utils_common.py')
    if not os.path.exists(path):
        pytest.skip('reference checkout not present')
    spec = importlib.util.spec_from_file_location('ref_utils_common', path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_dataset_fixture_regenerates():
    from oracle.data import gaussians
    d = golden('lr_256x10.npz')
    feats, targs = gaussians(256, 10, 0)
    assert np.array_equal(feats, d['features'])
    assert np.array_equal(targs, d['targets'])


@pytest.mark.parametrize('seed', [0, 1, 2])
def test_rollout_fixture_regenerates(lr_dataset, seed):
    fx = golden('optimize_lr_s%d.npz' % seed)
    rec = rollout(*lr_dataset, seed, None, 45, 1234 + seed)
    for key in ('obs', 'reward', 'done', 'objective', 'accuracy', 'ep_len', 'weights'):
        assert np.array_equal(rec[key], fx[key]), key


@pytest.mark.parametrize('seed', [3, 4])
def test_minibatch_rollout_fixture_regenerates(lr_dataset, seed):
    fx = golden('optimize_lr_b32_s%d.npz' % seed)
    rec = rollout(*lr_dataset, seed, 32, 85, 99 + seed)
    for key in ('obs', 'reward', 'order', 'objective', 'accuracy'):
        assert np.array_equal(rec[key], fx[key]), key


def test_seeding_fixture():
    fx = golden('seeding.npz')
    for i, seed in enumerate(SEEDS):
        key = seed_key(seed)
        assert list(fx['keys'][i, :fx['key_len'][i]]) == key
        w0, perm = ref.initial_draws(seed, 10, 2, 256)
        assert np.array_equal(w0, fx['weights'][i])
        assert np.array_equal(perm, fx['perms'][i])


def test_reset_is_idempotent(lr_dataset):
    """use_random_state never advances the env RNG (utils_math.py:9-22)."""
    env = ref.Optimize(*lr_dataset, batch_size=32)
    env.seed(11)
    env.reset()
    w_a = env.model.weights.copy()
    order_a = env.sequence.order.copy()
    env.reset()
    assert np.array_equal(env.model.weights, w_a)
    # the dataset permutation composes: order_2 = order_1[perm]
    assert np.array_equal(env.sequence.order, order_a[order_a])


def test_oracle_matches_reference_shuffle_and_onehot():
    mod = _reference_utils_common()
    from oracle.data import to_onehot
    for seed in range(3):
        npr.seed(seed)
        a = mod.shuffle(np.arange(25, 0, -1), np.arange(25))
        npr.seed(seed)
        b = ref.shuffle(np.arange(25, 0, -1), np.arange(25))
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
    labels = np.array([3, 1, 3, 2, 1, 0, 2])
    ra, na = mod.to_onehot(labels)
    oa, no = to_onehot(labels)
    assert na == no and np.array_equal(ra, oa)


def test_softmax_and_cross_entropy_properties():
    """tests/utils/test_utils_math.py:29-66 as properties of the oracle."""
    for seed in range(3):
        for mag in range(3):
            rs = np.random.RandomState(seed)
            logits = rs.uniform(-10 ** mag, 10 ** mag, size=(8, 4))
            prob = ref.softmax(logits)
            assert np.all(prob >= 0) and np.all(prob <= 1)
            assert np.allclose(prob.sum(axis=1), 1)
            labels = rs.uniform(size=(8, 4))
            assert ref.cross_entropy(prob, labels) >= 0


def test_use_random_state_reproduces_stream():
    """tests/utils/test_utils_math.py:17-24."""
    for seed in range(3):
        with ref.use_random_state(npr.RandomState(seed)):
            got = [npr.rand() for _ in range(20)]
        rs = npr.RandomState(seed)
        assert got == [rs.rand() for _ in range(20)]


def test_np_random_contract():
    rng, seed = np_random(5)
    assert seed == 5 and isinstance(rng, npr.RandomState)
    with pytest.raises(ValueError):
        np_random(-1)


def test_mlp_backprop_matches_torch_autograd():
    """The oracle's float32 MLP gradient (A12) against float64 torch autograd of
    sum_i -log(P_i + 1e-16) . Y_i (the tf.gradients of the per-sample loss
    vector, optimize_nn.py:48-52)."""
    import torch
    from oracle.gen_golden import mlp_dataset
    from oracle.optimize import ModelMLP, initial_draws_mlp
    features, targets = mlp_dataset()
    model = ModelMLP(16, 10, 64)
    model.set_weights(initial_draws_mlp(4, 16, 64, 10, 128)[0])
    x32, y32 = features[:32].astype(np.float32), targets[:32].astype(np.float32)
    loss, grad, acc = model.compute_backprop(x32, y32)
    params = [torch.tensor(p.astype(np.float64), requires_grad=True) for p in model.unflatten()]
    w1, b1, w2, b2 = params
    x, y = torch.tensor(x32, dtype=torch.float64), torch.tensor(y32, dtype=torch.float64)
    prob = torch.softmax(torch.relu(x @ w1 + b1) @ w2 + b2, dim=1)
    per_sample = -(torch.log(prob + 1e-16) * y).sum(dim=1)
    per_sample.sum().backward()
    ref = torch.cat([p.grad.reshape(-1) for p in params]).numpy()
    assert abs(loss - per_sample.mean().item()) <= 1e-6 * abs(loss)
    scale = np.abs(ref).max()
    assert np.abs(grad - ref).max() <= 1e-5 * scale
    assert acc == (prob.argmax(1) == y.argmax(1)).double().mean().item()


@pytest.mark.parametrize('seed', [5, 6])
def test_mlp_rollout_fixture_regenerates(seed):
    from oracle.gen_golden import mlp_dataset, rollout_mlp
    data = golden('mlp_data_128x16.npz')
    features, targets = mlp_dataset()
    assert np.array_equal(features, data['features']) and np.array_equal(targets, data['targets'])
    fx = golden('optimize_mlp_s%d.npz' % seed)
    rec = rollout_mlp(features, targets, seed, action_seed=int(fx['action_seed']))
    for key in ('reward', 'done', 'objective', 'accuracy', 'ep_len', 'loss_obs', 'obs',
                'weights', 'reset_obs', 'init_weights'):
        assert np.array_equal(rec[key], fx[key]), key
