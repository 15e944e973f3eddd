"""Dataset loaders (custom_envs/data/load_data.py:47-112).

The file-backed sets ('mnist', 'mnist-test', 'fashion', 'emnist-digits',
'iris', 'skin') read files a user supplies (``data_dir`` or
$CUSTOM_ENVS_DATA_DIR; data/files.py): every data file in the reference is a
git-LFS pointer.  Built in, no files needed:

  random_gaussians   sklearn make_classification() + one-hot(2), exactly the
                     reference's branch (load_data.py:105-107)
  gaussians_256x10   the configs' logistic-regression set:
                     make_classification(n_samples=256, n_features=10,
                     random_state=0), one-hot(2), not normalised
  mnist_synthetic    "MNIST-sized" features for the MLP config:
                     RandomState(0).rand(1024, 784), labels argmax(X T) with
                     T = RandomState(1).normal(size=(784, 10))
  mnist7x7_synthetic the shape load_data('mnist') gives (60,000 rows of
                     7x7 = 49 features in [0, 1], 10 classes): synthetic
                     28x28 uint8 "digits" (class-dependent blobs + noise)
                     sampled at the PIL NEAREST 28 -> 7 pixels, normalised
                     as the mnist branch does (load_data.py:65-71)
  iris_synthetic     iris-shaped stand-in for 'iris' (load_data's default,
                     the data set of get_problem('nn')): 150 rows, 4
                     features, 3 classes of 50, Gaussian blobs at the iris
                     class means/spreads from RandomState(0), then the iris
                     branch's normalize + to_onehot (load_data.py:61-64)
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


def _mnist7x7_synthetic(num_of_labels=None, n_rows=60000, seed=0):
    rs = np.random.RandomState(seed)
    labels = rs.randint(0, 10, n_rows)
    pos = np.arange(2, 28, 4).astype(np.float64)         # NEAREST 28 -> 7 samples
    cy = (6 + 2 * (labels % 5) + rs.randint(-3, 4, n_rows))[:, None, None]
    cx = (7 + 3 * (labels // 5) + rs.randint(-3, 4, n_rows))[:, None, None]
    sig = (3.0 + labels % 3)[:, None, None]
    r2 = (pos[None, :, None] - cy) ** 2 + (pos[None, None, :] - cx) ** 2
    img = 255 * np.exp(-r2 / (2 * sig ** 2)) + rs.normal(0, 24, (n_rows, 7, 7))
    img = np.clip(np.round(img), 0, 255).astype(np.uint8).reshape(n_rows, 49)
    return normalize(img), to_onehot(labels, num_of_labels)[0]


def normalize(data):
    """utils_math.py:77-87: per column (x - min) / (max - min + 1e-8)."""
    mins, maxes = np.min(data, axis=0), np.max(data, axis=0)
    return (data - mins) / (maxes - mins + 1e-8)


_IRIS_MEANS = ((5.006, 3.428, 1.462, 0.246), (5.936, 2.770, 4.260, 1.326),
               (6.588, 2.974, 5.552, 2.026))
_IRIS_STDS = ((0.352, 0.379, 0.174, 0.105), (0.516, 0.314, 0.470, 0.198),
              (0.636, 0.322, 0.552, 0.275))


def _iris_synthetic(num_of_labels=None):
    rs = np.random.RandomState(0)
    features = np.concatenate([rs.normal(m, s, (50, 4)) for m, s in zip(_IRIS_MEANS, _IRIS_STDS)])
    labels = np.repeat(np.arange(3), 50)
    return normalize(features), to_onehot(labels, num_of_labels)[0]


LOADERS = {
    'random_gaussians': lambda n: _gaussians(),
    'gaussians_256x10': lambda n: _gaussians(n_samples=256, n_features=10, random_state=0),
    'mnist_synthetic': _mnist_synthetic,
    'iris_synthetic': _iris_synthetic,
    'mnist7x7_synthetic': _mnist7x7_synthetic,
}


def load_data(name='gaussians_256x10', batch_size=32, num_of_labels=None, data_dir=None):
    """Return an ``InMemoryDataSet`` (load_data.py:47-112 signature).

    The file-backed sets ('mnist', 'mnist-test', 'fashion', 'emnist-digits',
    'iris', 'skin'; custom_envs_amd/data/files.py) read ``data_dir`` (default:
    the CUSTOM_ENVS_DATA_DIR environment variable), laid out
    as the reference's custom_envs/data/ directory; the reference's own copies
    are git-LFS pointers and are refused.  'cifar-10' needs a keras download
    and is not served."""
    import os
    from custom_envs_amd.data import files
    if name in files.IDX_SETS + files.TABLE_SETS:
        data_dir = data_dir or os.environ.get('CUSTOM_ENVS_DATA_DIR')
        if data_dir is None:
            raise RuntimeError('data set %r reads files: pass data_dir (the reference ships '
                               'them as git-LFS pointers)' % name)
        load = files.load_idx_set if name in files.IDX_SETS else files.load_table_set
        features, targets = load(data_dir, name, num_of_labels, normalize, to_onehot)
        return InMemoryDataSet(features, targets, batch_size)
    if name not in LOADERS:
        raise RuntimeError('No such data set named: {}'.format(name))
    features, targets = LOADERS[name](num_of_labels)
    return InMemoryDataSet(features, targets, batch_size)
