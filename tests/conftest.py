import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, 'tests', 'golden')
REFERENCE = '/root/reference'


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs the HIP engine)')


def golden(name):
    return np.load(os.path.join(GOLDEN, name))


@pytest.fixture(scope='session')
def lr_dataset():
    d = golden('lr_256x10.npz')
    return d['features'], d['targets']
