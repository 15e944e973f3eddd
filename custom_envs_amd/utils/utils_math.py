"""Host-side math helpers of the custom_envs surface (utils_math.py:9-87).

The engine fuses softmax / cross-entropy into its kernels; these serve host
code that imports them (``BaseEnvironment`` uses ``use_random_state``).  The
reference evaluates the exps with numexpr, absent here; numpy computes the
same expressions.
"""
from contextlib import contextmanager

import numpy as np
import numpy.random as npr


@contextmanager
def use_random_state(random_state):
    """Run under a copy of ``random_state`` as the global npr state
    (utils_math.py:9-22); the global state is restored afterwards."""
    saved_state = npr.get_state()
    try:
        npr.set_state(random_state.get_state())
        yield random_state
    finally:
        npr.set_state(saved_state)


def cross_entropy(prob, ground_truth):
    """utils_math.py:25-34."""
    return np.mean(np.sum(-np.log(prob + 1e-16) * ground_truth, axis=1))


def mse(prediction, ground_truth):
    """utils_math.py:37-48."""
    return np.mean(np.sum((prediction - ground_truth) ** 2, axis=1) / 2)


def softmax(logits):
    """Row-max-stabilised softmax (utils_math.py:51-63)."""
    p_exp = np.exp(logits - np.max(logits, axis=1)[:, None])
    return p_exp / np.sum(p_exp, axis=1)[:, None]


def sigmoid(logits):
    """utils_math.py:66-74."""
    return 1 / (1 + np.exp(-logits - 1e-8))


def normalize(data):
    """Per column (x - min) / (max - min + 1e-8) (utils_math.py:77-87)."""
    mins, maxes = np.min(data, axis=0), np.max(data, axis=0)
    return (data - mins) / (maxes - mins + 1e-8)
