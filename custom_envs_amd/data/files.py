"""On-disk data set readers (custom_envs/data/load_data.py:15-104), host side.

The reference ships every data file as a git-LFS pointer, so these readers
only run on files a user supplies (``load_data(name, data_dir=...)``); a
pointer or a missing file raises ``RuntimeError``.

  load_mnist / load_emnist   IDX-ubyte label + image files, .xz (the
                             reference's), .gz or raw (load_data.py:15-44)
  resize_nearest             PIL ``Image.resize(shape, NEAREST)`` for uint8
                             images (utils_image.py:6-25)
  iris / skin                the .npz 'data' array / tab-separated text with
                             the label in the last column (load_data.py:61-64,
                             79-83)
The resize restates Pillow's scale-only affine path (ImagingScaleAffine):
source index = int(o) with o starting at s/2 and advanced by s = in/out in
float64 per output pixel -- an accumulated sum, which is not always
floor((x + 0.5) s).  tests/test_ref_pins.py pins it bit for bit against the
reference's own utils_image.resize_array_many (numpy + PIL, both importable
in the build container; fixture tests/golden/ref_load_data.npz).
"""
import gzip
import lzma
import os
import struct

import numpy as np

IDX_LABELS, IDX_IMAGES = 2049, 2051
LFS_MAGIC = b'version https://git-lfs'


def _check_not_pointer(path):
    with open(path, 'rb') as fh:
        if fh.read(len(LFS_MAGIC)) == LFS_MAGIC:
            raise RuntimeError('%s is a git-LFS pointer, not data' % path)


def _open(path):
    """Bytes of ``path``, or of ``path`` with .xz / .gz appended."""
    for cand in (path, path + '.xz', path + '.gz'):
        if os.path.exists(cand):
            _check_not_pointer(cand)
            opener = lzma.open if cand.endswith('.xz') else (
                gzip.open if cand.endswith('.gz') else open)
            with opener(cand, 'rb') as fh:
                return fh.read()
    raise RuntimeError('data file not found: %s[.xz|.gz]' % path)


def read_idx(path, magic):
    """IDX-ubyte array (labels: magic 2049, n; images: 2051, n, rows, cols)."""
    raw = _open(path)
    if magic == IDX_LABELS:
        got, n = struct.unpack('>II', raw[:8])
        shape, offset = (n,), 8
    else:
        got, n, rows, cols = struct.unpack('>IIII', raw[:16])
        shape, offset = (n, rows * cols), 16
    if got != magic:
        raise RuntimeError('%s: IDX magic %d, expected %d' % (path, got, magic))
    return np.frombuffer(raw, dtype=np.uint8, offset=offset).reshape(shape)


def load_mnist(data_dir, name='fashion', kind='train'):
    """load_data.py:15-28 (``name``/``kind``-labels|images-idx*-ubyte)."""
    base = os.path.join(data_dir, name)
    labels = read_idx(os.path.join(base, '%s-labels-idx1-ubyte' % kind), IDX_LABELS)
    images = read_idx(os.path.join(base, '%s-images-idx3-ubyte' % kind), IDX_IMAGES)
    return images.reshape(len(labels), -1), labels


def load_emnist(data_dir, name='emnist', kind='train'):
    """load_data.py:31-44 (the digits split)."""
    base = os.path.join(data_dir, name, 'digits')
    labels = read_idx(os.path.join(base, 'emnist-digits-%s-labels-idx1-ubyte' % kind), IDX_LABELS)
    images = read_idx(os.path.join(base, 'emnist-digits-%s-images-idx3-ubyte' % kind), IDX_IMAGES)
    return images.reshape(len(labels), -1), labels


def _nearest_positions(n_in, n_out):
    """Source index of each output pixel, in Pillow's float64 accumulation order."""
    scale = n_in / n_out
    pos = np.empty(n_out, np.int64)
    o = scale * 0.5
    for i in range(n_out):
        pos[i] = int(o)
        o += scale
    return pos


def resize_nearest(images, shape):
    """PIL NEAREST resize of uint8 images [n][h][w] to shape = (width, height)
    (PIL's order, utils_image.py:14)."""
    images = np.asarray(images)
    h, w = images.shape[-2:]
    out_w, out_h = shape
    ys = _nearest_positions(h, out_h)
    xs = _nearest_positions(w, out_w)
    return images[..., ys[:, None], xs[None, :]]


IDX_SETS = ('mnist', 'mnist-test', 'fashion', 'emnist-digits')
TABLE_SETS = ('iris', 'skin')


def load_idx_set(data_dir, name, num_of_labels, normalize, to_onehot):
    """The mnist / mnist-test / fashion / emnist-digits branches of
    load_data.py:65-97: 28x28 images resized to 7x7, flattened, normalised,
    labels one-hot."""
    if name == 'mnist':
        images, labels = load_mnist(data_dir, 'mnist')
    elif name == 'mnist-test':
        images, labels = load_mnist(data_dir, 'mnist', 't10k')
    elif name == 'fashion':
        images, labels = load_mnist(data_dir)
    else:
        images, labels = load_emnist(data_dir)
    small = resize_nearest(images.reshape(-1, 28, 28), (7, 7)).reshape(len(labels), -1)
    return normalize(small), to_onehot(labels, num_of_labels)[0]


def load_table_set(data_dir, name, num_of_labels, normalize, to_onehot):
    """iris (load_data.py:61-64) and skin (:79-83)."""
    path = os.path.join(data_dir, 'iris.npz' if name == 'iris' else 'skin.txt')
    if not os.path.exists(path):
        raise RuntimeError('data file not found: %s' % path)
    _check_not_pointer(path)
    if name == 'iris':
        data = np.load(path)['data']                     # allow_pickle stays False
        return normalize(data[..., :-1]), to_onehot(data[..., -1], num_of_labels)[0]
    data = np.loadtxt(path, delimiter='\t')
    features = np.zeros((data.shape[0], 4))
    features[:, :3] = normalize(data[..., :-1])
    return features, to_onehot(data[..., -1], 3)[0]
