"""File-backed data sets (custom_envs/data/load_data.py:15-104) on files the
test writes itself: IDX-ubyte (.xz, as the reference ships them, and .gz),
the iris .npz and the skin text table.  The reference's own files are
git-LFS pointers; the loader refuses them.  The NEAREST resize is pinned
against PIL itself here (Pillow is importable in this image) and against the
reference's utils_image in tests/test_ref_pins.py."""
import gzip
import lzma
import os
import struct

import numpy as np
import pytest

from conftest import REFERENCE
from custom_envs_amd.data import load_data, normalize, to_onehot
from custom_envs_amd.data.files import resize_nearest


def _write_idx(path, array, magic, compress):
    if magic == 2049:
        head = struct.pack('>II', magic, array.shape[0])
    else:
        head = struct.pack('>IIII', magic, array.shape[0], 28, 28)
    blob = head + array.astype(np.uint8).tobytes()
    opener = lzma.open if compress == 'xz' else gzip.open
    with opener(path + '.' + compress, 'wb') as fh:
        fh.write(blob)


@pytest.mark.parametrize('compress', ['xz', 'gz'])
@pytest.mark.parametrize('name,sub,prefix', [('mnist', 'mnist', 'train'),
                                             ('mnist-test', 'mnist', 't10k'),
                                             ('fashion', 'fashion', 'train'),
                                             ('emnist-digits', 'emnist/digits',
                                              'emnist-digits-train')])
def test_idx_sets(tmp_path, compress, name, sub, prefix):
    rs = np.random.RandomState(0)
    images = rs.randint(0, 256, (20, 28, 28))
    labels = rs.randint(0, 10, 20)
    d = tmp_path / sub
    d.mkdir(parents=True)
    _write_idx(str(d / ('%s-labels-idx1-ubyte' % prefix)), labels, 2049, compress)
    _write_idx(str(d / ('%s-images-idx3-ubyte' % prefix)), images.reshape(20, -1), 2051, compress)
    ds = load_data(name, batch_size=4, data_dir=str(tmp_path))
    small = images[:, 2::4, 2::4].reshape(20, -1)          # PIL NEAREST 28 -> 7
    np.testing.assert_array_equal(ds.features, normalize(small))
    np.testing.assert_array_equal(ds.targets, to_onehot(labels)[0])
    assert len(ds) == 5 and ds.feature_shape == (49,)


def test_resize_matches_pil_nearest():
    from PIL import Image
    rs = np.random.RandomState(1)
    for (h, w), (ow, oh) in (((28, 28), (7, 7)), ((32, 32), (7, 7)), ((10, 14), (4, 6)),
                             ((28, 28), (9, 5)), ((13, 17), (40, 3))):
        img = rs.randint(0, 256, (3, h, w)).astype(np.uint8)
        ref = np.stack([np.asarray(Image.fromarray(im).resize((ow, oh), Image.NEAREST))
                        for im in img])
        np.testing.assert_array_equal(resize_nearest(img, (ow, oh)), ref)


def test_iris_and_skin_tables(tmp_path):
    rs = np.random.RandomState(2)
    iris = np.concatenate([rs.rand(30, 4), rs.randint(0, 3, (30, 1))], axis=1)
    np.savez(tmp_path / 'iris.npz', data=iris)
    ds = load_data('iris', batch_size=8, data_dir=str(tmp_path))
    np.testing.assert_array_equal(ds.features, normalize(iris[:, :-1]))
    np.testing.assert_array_equal(ds.targets, to_onehot(iris[:, -1])[0])
    skin = np.concatenate([rs.randint(0, 256, (25, 3)), rs.randint(1, 3, (25, 1))], axis=1)
    np.savetxt(tmp_path / 'skin.txt', skin, delimiter='\t', fmt='%d')
    ds = load_data('skin', data_dir=str(tmp_path))
    assert ds.features.shape == (25, 4) and np.all(ds.features[:, 3] == 0)
    np.testing.assert_allclose(ds.features[:, :3], normalize(skin[:, :-1].astype(float)))
    assert ds.targets.shape == (25, 3)


def test_reference_lfs_pointers_are_refused():
    data_dir = os.path.join(REFERENCE, 'custom_envs', 'data')
    if not os.path.isdir(data_dir):
        pytest.skip('reference checkout not present')
    for name in ('mnist', 'iris', 'skin', 'fashion'):
        with pytest.raises(RuntimeError, match='LFS|not found'):
            load_data(name, data_dir=data_dir)


def test_file_sets_need_a_directory():
    with pytest.raises(RuntimeError, match='data_dir'):
        load_data('mnist')
