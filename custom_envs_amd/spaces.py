"""Minimal old-gym ``Box`` / ``Dict`` spaces (gym is absent from this image).

Semantics follow gym<=0.21, the version the reference's 4-tuple step API and
RandomState seeding imply: ``Box(low, high, shape, dtype)`` with scalar or
array bounds, ``Dict`` ordering keys lexicographically when given a plain
dict (the agent-row order ``OptVecEnv`` relies on,
custom_envs/vectorize/optvecenv.py:10-14).
"""
from collections import OrderedDict

import numpy as np


class Space:
    def __init__(self, shape=None, dtype=None):
        self.shape = None if shape is None else tuple(shape)
        self.dtype = None if dtype is None else np.dtype(dtype)
        self.np_random = np.random.RandomState()

    def seed(self, seed=None):
        self.np_random = np.random.RandomState(seed)
        return [seed]

    def __contains__(self, x):
        return self.contains(x)


class Box(Space):
    def __init__(self, low, high, shape=None, dtype=np.float32):
        dtype = np.dtype(dtype)
        if shape is None:
            shape = np.shape(low) if np.ndim(low) else np.shape(high)
        shape = tuple(shape)
        self.low = np.broadcast_to(np.asarray(low, dtype=dtype), shape).copy()
        self.high = np.broadcast_to(np.asarray(high, dtype=dtype), shape).copy()
        super().__init__(shape, dtype)

    def sample(self):
        return self.np_random.uniform(self.low, self.high, self.shape).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return (x.shape == self.shape and np.all(x >= self.low)
                and np.all(x <= self.high))

    def __eq__(self, other):
        return (isinstance(other, Box) and self.shape == other.shape
                and np.allclose(self.low, other.low) and np.allclose(self.high, other.high))

    def __repr__(self):
        return 'Box(%s, %s)' % (self.shape, self.dtype)


class Dict(Space):
    def __init__(self, spaces=None, **kwargs):
        spaces = kwargs if spaces is None else spaces
        if isinstance(spaces, dict) and not isinstance(spaces, OrderedDict):
            spaces = OrderedDict(sorted(spaces.items()))
        elif not isinstance(spaces, OrderedDict):
            spaces = OrderedDict(spaces)
        self.spaces = spaces
        super().__init__(None, None)

    def seed(self, seed=None):
        for space in self.spaces.values():
            space.seed(seed)
        return [seed]

    def sample(self):
        return OrderedDict((k, s.sample()) for k, s in self.spaces.items())

    def contains(self, x):
        return (isinstance(x, dict) and len(x) == len(self.spaces)
                and all(k in x and s.contains(x[k]) for k, s in self.spaces.items()))

    def __getitem__(self, key):
        return self.spaces[key]

    def __iter__(self):
        return iter(self.spaces)

    def __eq__(self, other):
        return isinstance(other, Dict) and self.spaces == other.spaces

    def __repr__(self):
        return 'Dict(%s)' % ', '.join('%s:%r' % kv for kv in self.spaces.items())
