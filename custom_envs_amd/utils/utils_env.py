"""Versioned observation / action / reward helpers of the Multi* envs
(custom_envs/utils/utils_env.py:9-164), host side.

MultiOptLRs-v0 runs versions (3, 3, 0, 6) in-kernel (csrc/multiopt_kernels.h);
these functions keep the reference's module for host code and are pinned
against the reference's own functions (tests/test_ref_pins.py).
"""
import numpy as np

from custom_envs_amd.spaces import Box
from custom_envs_amd.utils.utils_common import History


def get_obs_version(shape, max_history, version=0):
    """(space, History) per observation version (utils_env.py:9-47)."""
    table = {
        0: (dict(gradients=shape), 1, (1,)),
        1: (dict(losses=(), gradients=shape), max_history, (2 * max_history,)),
        2: (dict(weights=shape, losses=(), gradients=shape), 1, (3,)),
        3: (dict(weights=shape, losses=(), gradients=shape), max_history, (3 * max_history,)),
        4: (dict(gradients=shape), max_history, (max_history,)),
        5: (dict(weights=shape, losses=(), gradients=shape, actions=shape), max_history,
            (4 * max_history,)),
    }
    if version not in table:
        raise RuntimeError()
    keys, length, space_shape = table[version]
    return (Box(low=-1e6, high=1e6, dtype=np.float32, shape=space_shape),
            History(length, **keys))


def get_action_space_optlrs(version=0):
    """utils_env.py:50-68."""
    bounds = {0: (-4., 6.), 1: (0., 1e4), 2: (-1e3, 1e4)}
    if version not in bounds:
        raise RuntimeError()
    low, high = bounds[version]
    return Box(low=low, high=high, dtype=np.float32, shape=(1,))


def _scalar(v):
    """float(v) for a scalar or a one-element array (the reference's float())."""
    return float(np.ravel(v)[0])


def get_reward(loss, adjusted_loss, version=0):
    """utils_env.py:71-99."""
    if version == 0:
        return -_scalar(adjusted_loss)
    if version == 1:
        return _scalar(1 / loss)
    if version == 2:
        return -_scalar(adjusted_loss) * 100
    if version == 3:
        return _scalar(1 / loss) * 100
    if version == 4:
        return np.log(1 / loss)
    if version == 5:
        return -(_scalar(adjusted_loss) - 1) ** 2
    if version == 6:
        return -(_scalar(adjusted_loss) - 1)
    raise RuntimeError()


def get_action_optlrs(action, version):
    """utils_env.py:102-123."""
    if version == 0:
        return 10 ** (action - 4)
    if version == 1:
        return action * 1e-3
    if version == 2:
        return 2 ** action
    if version == 3:
        return np.clip((action + 1e3) * 1e-6, 0, np.inf)
    raise RuntimeError()


def get_observation(history, version=0):
    """(adjusted loss, weights, gradients) from a History (utils_env.py:126-164)."""
    losses, grads, weights = history['losses'], history['gradients'], history['weights']
    adj_loss = losses[0] / (np.abs(losses[1]) + 1e-3)
    adj_wght = weights[0] / (np.abs(weights[1]) + 1e-3)
    adj_grad = grads[0] / (np.abs(grads[1]) + 1e-3)
    if version == 0:
        pass
    elif version == 1:
        adj_grad = grads[0] * 1e2
    elif version == 2:
        adj_loss = (losses[0] - losses[1]) / (np.abs(losses[1] - losses[2]) + 1e-3)
        adj_wght = np.abs(weights[1] - weights[2]) / (np.abs(weights[0] - weights[1]) + 1e-8)
        adj_grad = (grads[0] - grads[1]) / (np.abs(grads[1] - grads[2]) + 1e-3)
    elif version == 3:
        with np.errstate(divide='ignore', invalid='ignore'):
            adj_grad = np.nan_to_num(grads[0] / np.abs(grads[1]))
            adj_wght = np.nan_to_num(weights[0] / np.abs(weights[1]))
            adj_loss = np.nan_to_num(losses[0] / np.abs(losses[1]))
    else:
        raise RuntimeError()
    return float(np.ravel(adj_loss)[0]), adj_wght, adj_grad
