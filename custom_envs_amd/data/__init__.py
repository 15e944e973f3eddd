"""Dataset loaders (custom_envs/data/load_data.py:47-112), synthetic only.

Every real data file in the reference (iris.npz, the MNIST/EMNIST/fashion
IDX archives) is a git-LFS pointer, so only the synthetic sets are served:

  random_gaussians   sklearn make_classification() + one-hot(2), exactly the
                     reference's branch (load_data.py:105-107)
  gaussians_256x10   the configs' logistic-regression set:
                     make_classification(n_samples=256, n_features=10,
                     random_state=0), one-hot(2), not normalised
  mnist_synthetic    "MNIST-sized" features for the MLP config:
                     RandomState(0).rand(1024, 784), labels argmax(X T) with
                     T = RandomState(1).normal(size=(784, 10))
"""
import numpy as np

from custom_envs_amd.dataset import InMemoryDataSet


def to_onehot(array, num_of_labels=None):
    """utils_common.py:88-99: one-hot in np.unique order."""
    classes, inverse = np.unique(array, return_inverse=True)
    if num_of_labels is None:
        num_of_labels = classes.size
    onehot = np.zeros((len(inverse), num_of_labels))
    onehot[np.arange(len(inverse)), inverse] = 1
    return onehot, num_of_labels


def _gaussians(**kwargs):
    from sklearn.datasets import make_classification
    features, labels = make_classification(**kwargs)
    return features.astype(np.float64), to_onehot(labels, 2)[0]


def _mnist_synthetic(num_of_labels=None):
    features = np.random.RandomState(0).rand(1024, 784)
    proj = np.random.RandomState(1).normal(size=(784, 10))
    labels = np.argmax(features @ proj, axis=1)
    return features, to_onehot(labels, num_of_labels or 10)[0]


LOADERS = {
    'random_gaussians': lambda n: _gaussians(),
    'gaussians_256x10': lambda n: _gaussians(n_samples=256, n_features=10, random_state=0),
    'mnist_synthetic': _mnist_synthetic,
}


def load_data(name='gaussians_256x10', batch_size=32, num_of_labels=None):
    """Return an ``InMemoryDataSet`` (load_data.py:47-112 signature)."""
    if name not in LOADERS:
        raise RuntimeError('No such data set named: {} (real-data loaders are out of '
                           'scope: the reference ships them as git-LFS pointers)'.format(name))
    features, targets = LOADERS[name](num_of_labels)
    return InMemoryDataSet(features, targets, batch_size)
