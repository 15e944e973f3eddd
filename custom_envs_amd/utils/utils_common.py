"""Host-side helpers the wrappers need (custom_envs/utils/utils_common.py).

``History`` is the fixed-length, newest-first history the reference keeps
per observation key (utils_common.py:102-196); the engine keeps the same
structure as device rings, this class serves ``HistoryWrapper``.
"""
from collections import deque
from collections.abc import Mapping
from itertools import chain, cycle

import numpy as np


def shuffle(*arrays, np_random=np.random):
    """Permute rows of every array with one permutation (utils_common.py:12-23)."""
    index = np.arange(len(arrays[0]))
    np_random.shuffle(index)
    return [a[index] for a in arrays]


def to_onehot(array, num_of_labels=None):
    from custom_envs_amd.data import to_onehot as _onehot
    return _onehot(array, num_of_labels)


class History(Mapping):
    def __init__(self, max_history, **named_shapes):
        self.max_history = max_history
        self.shapes = {k: tuple(s) if s else (1,) for k, s in named_shapes.items()}
        self.reset()
        self.iteration = 0

    def __repr__(self):
        return '<History<max_history={}, shapes={!r}>>'.format(self.max_history, self.shapes)

    def __getitem__(self, key):
        return np.asarray(list(reversed(self.history[key])))

    def __iter__(self):
        return iter(self.history)

    def __len__(self):
        return len(self.history)

    def _fill(self, make):
        self.history = {k: deque([make(k)] * self.max_history, maxlen=self.max_history)
                        for k in self.shapes}
        self.iteration = 0

    def reset_with_value(self, value):
        self._fill(lambda k: np.full(self.shapes[k], value))

    def reset(self, **named_items):
        if named_items:
            assert self.keys() == named_items.keys()
            self._fill(lambda k: np.reshape(named_items[k], self.shapes[k]))
        else:
            self._fill(lambda k: np.zeros(self.shapes[k]))

    def append(self, **named_items):
        assert self.keys() == named_items.keys()
        for name, item in named_items.items():
            self.history[name].append(np.reshape(item, self.shapes[name]))
        self.iteration = (self.iteration + 1) % self.max_history

    def build_multistate(self):
        rows = list(chain.from_iterable(
            self[key].reshape((self.max_history, -1)).tolist() for key in self))
        rows = [cycle(r) if len(r) == 1 else r for r in rows]
        return list(zip(*rows))


def flatten_arrays(arrays, dtype=np.float64):
    return np.fromiter(chain.from_iterable(a.ravel() for a in arrays), dtype,
                       sum(a.size for a in arrays))


def from_flat(array, shapes):
    out, start = [], 0
    for shape in shapes:
        end = start + int(np.prod(shape))
        out.append(np.reshape(array[start:end], shape))
        start = end
    return out
