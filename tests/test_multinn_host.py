"""MultiOptLRs over OptimizeNN on the CPU: oracle pins and the host ABI.

Pins: the row order the oracle composes (reset shuffle, then
one shuffle per finished epoch) uses the reference's own
``utils_common.shuffle`` (imported by path when /root/reference exists);
the oracle's backward pass matches central differences of its forward pass
in float64; the native seeding (``ce_nn_seed_draws``) reproduces the
oracle's draws bit for bit.  TensorFlow is absent, so the float32 network
values themselves are "parity unpinned" against TF (oracle/multinn.py).
"""
import ctypes
import importlib.util
import os

import numpy as np
import pytest

from conftest import REFERENCE
from custom_envs_amd import _native
from oracle.multinn import MultiOptLRsNN, OptimizeNN, nn_draws


def _iris():
    from custom_envs_amd.data import load_data
    ds = load_data('iris_synthetic', batch_size=32)
    return ds.features, ds.targets


@pytest.mark.parametrize('dims', [(4, 256, 256, 3), (7, 64, 5), (4, 32, 64, 96, 3)])
@pytest.mark.parametrize('seed', [0, 3, 2**40 + 1])
def test_native_nn_draws_match_oracle(dims, seed):
    lib = _native.load()
    th_ref, rp_ref, ep_ref = nn_draws(seed, dims, 150)
    th = np.zeros(th_ref.size, np.float32)
    rp = np.zeros(150, np.int32)
    ep = np.zeros(150, np.int32)
    d = np.asarray(dims, np.int32)
    _native.check(lib.ce_nn_seed_draws(seed, len(dims), d.ctypes.data, 150, th.ctypes.data,
                                       rp.ctypes.data, ep.ctypes.data), 'ce_nn_seed_draws')
    assert np.array_equal(th, th_ref)
    assert np.array_equal(rp, rp_ref) and np.array_equal(ep, ep_ref)


def _eval64(prob, theta, batch):
    """The oracle's forward/backward (OptimizeNN.evaluate) in float64."""
    features, targets = batch
    tensors = prob.unflatten(theta)
    weights, biases = tensors[0::2], tensors[1::2]
    acts, zs, h = [features], [], features
    for w, b in zip(weights[:-1], biases[:-1]):
        z = h @ w + b
        zs.append(z)
        h = np.maximum(z, 0.0)
        acts.append(h)
    logits = h @ weights[-1] + biases[-1]
    shifted = logits - logits.max(axis=1, keepdims=True)
    e = np.exp(shifted)
    se = e.sum(axis=1, keepdims=True)
    loss = np.mean(np.log(se)[:, 0] - np.sum(shifted * targets, axis=1))
    d = e / se - targets
    grads = [None] * len(tensors)
    for layer in range(len(weights) - 1, -1, -1):
        grads[2 * layer] = acts[layer].T @ d
        grads[2 * layer + 1] = d.sum(axis=0)
        if layer:
            d = (d @ weights[layer].T) * (zs[layer - 1] > 0)
    return np.concatenate([g.ravel() for g in grads]), loss


def test_oracle_backprop_matches_central_differences():
    """Gradient of sum_i CE_i (what tf.gradients differentiates,
    optimize_nn.py:48-52) against central differences of the mean loss."""
    x, y = _iris()
    prob = OptimizeNN(x[:32], y[:32], hidden=(8, 8), batch_size=32)
    rs = np.random.RandomState(0)
    theta = rs.normal(0, 0.5, prob.size)
    batch = (x[:32].astype(np.float64), y[:32].astype(np.float64))
    grad, _ = _eval64(prob, theta, batch)
    for p in rs.choice(prob.size, 25, replace=False):
        h = 1e-6
        tp, tm = theta.copy(), theta.copy()
        tp[p] += h
        tm[p] -= h
        num = (_eval64(prob, tp, batch)[1] - _eval64(prob, tm, batch)[1]) * 32 / (2 * h)
        assert abs(num - grad[p]) <= 1e-6 * max(1.0, abs(grad[p])), (p, num, grad[p])


def test_oracle_float32_matches_float64_restatement():
    """The float32 oracle and its float64 twin agree to float32 rounding."""
    x, y = _iris()
    prob = OptimizeNN(x, y, hidden=(32, 32), batch_size=32)
    rs = np.random.RandomState(1)
    theta = rs.normal(0, 0.3, prob.size).astype(np.float32)
    batch = (x[:32].astype(np.float32), y[:32].astype(np.float32))
    g32, l32 = prob.evaluate(theta, batch)
    g64, l64 = _eval64(prob, theta.astype(np.float64),
                       (batch[0].astype(np.float64), batch[1].astype(np.float64)))
    assert abs(l32 - l64) <= 1e-5 * abs(l64)
    assert np.abs(g32 - g64).max() <= 1e-4 * np.abs(g64).max()


def test_batch_cycling_and_order_composition():
    """optimize_nn.py:102-120 with InMemoryDataSet's ragged last batch
    (inmemorydataset.py:21-28): 150 rows in batches of 32 are 32,32,32,32,22;
    the row order is the reset shuffle, then the epoch shuffle per finished
    epoch, composed as utils_common.shuffle composes them."""
    x, y = _iris()
    env = MultiOptLRsNN(x, y, hidden=(32,), batch_size=32, max_batches=400)
    env.seed(11)
    env.reset()
    th0, rho, pi = nn_draws(11, env.model.dims, 150)
    assert np.array_equal(env.model.params, th0)
    assert np.array_equal(env.order(), rho)
    sizes = []
    act = {n: np.float32(1.0) for n in env.names}
    order = rho.copy()
    for t in range(12):
        sizes.append(len(env.model.current_batch[0]))
        env.step(act)
        if (t + 1) % 5 == 0:
            order = order[pi]
        assert np.array_equal(env.order(), order), t
    assert sizes[:6] == [32, 32, 32, 32, 22, 32]


def test_order_composition_uses_the_reference_shuffle():
    """The reference's own utils_common.shuffle (imported by path) under a
    copy of the env RandomState reproduces the oracle's epoch permutation."""
    path = os.path.join(REFERENCE, 'custom_envs', 'utils', 'utils_common.py')
    if not os.path.exists(path):
        pytest.skip('reference checkout not present')
    spec = importlib.util.spec_from_file_location('ref_utils_common_nn', path)
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    from oracle.seeding import np_random
    for seed in (0, 5, 123456):
        rng, _ = np_random(seed)
        (shuffled,) = ref.shuffle(np.arange(150), np_random=rng)
        assert np.array_equal(shuffled, nn_draws(seed, (4, 32, 3), 150)[2])


@pytest.mark.parametrize('change', [dict(hidden=(48,)), dict(hidden=(1024,)),
                                    dict(n_classes=40), dict(batch_size=64),
                                    dict(hidden=()), dict(max_history=17)])
def test_unsupported_nn_shape_is_loud(change):
    lib = _native.load()
    base = dict(n_rows=150, n_features=4, n_classes=3, batch_size=32, hidden=(256, 256),
                max_history=5)
    base.update(change)
    hidden = base.pop('hidden')
    cfg = _native.CeNnConfig(abi_version=_native.ABI_VERSION, num_envs=2, max_batches=400,
                             n_hidden=len(hidden), **base)
    for i, w in enumerate(hidden):
        cfg.hidden[i] = w
    x = np.zeros((150, 4), np.float32)
    y = np.zeros(150, np.int32)
    handle = ctypes.c_void_p()
    assert lib.ce_nn_create(ctypes.byref(cfg), x.ctypes.data, y.ctypes.data,
                            ctypes.byref(handle)) == _native.CE_EUNSUPPORTED


def test_nn_engine_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip('a GPU is present')
    from custom_envs_amd.multi_engine import NNMultiEngine
    with pytest.raises(_native.NativeEngineError):
        NNMultiEngine(2)
