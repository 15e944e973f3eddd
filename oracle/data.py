"""Synthetic datasets named by the configs (TEST INFRASTRUCTURE ONLY).

``custom_envs/data/load_data.py:105-107`` builds ``random_gaussians`` with
``sklearn.datasets.make_classification()`` and one-hot labels, without
``normalize``.  The configs fix a 256x10 variant (SURVEY.md section 8d,
config 1): ``make_classification(n_samples=256, n_features=10,
random_state=0)``.  The committed fixture ``tests/golden/lr_256x10.npz`` is
the source of truth; this module only regenerates it.
"""
import numpy as np


def to_onehot(labels, num_of_labels=None):
    """``custom_envs/utils/utils_common.py:88-99`` (np.unique ordering)."""
    classes, inverse = np.unique(labels, return_inverse=True)
    if num_of_labels is None:
        num_of_labels = classes.size
    onehot = np.zeros((len(inverse), num_of_labels))
    onehot[np.arange(len(inverse)), inverse] = 1
    return onehot, num_of_labels


def gaussians(n_samples=256, n_features=10, random_state=0):
    from sklearn.datasets import make_classification
    features, labels = make_classification(
        n_samples=n_samples, n_features=n_features, random_state=random_state)
    targets, _ = to_onehot(labels, 2)
    return features.astype(np.float64), targets
