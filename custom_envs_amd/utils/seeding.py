"""Host-side old-gym seeding for user-defined envs (``BaseEnvironment``).

The engine-backed envs seed natively (csrc/seeding.cpp); this is the same
algorithm for envs that stay on the host: ``gym.utils.seeding.np_random``
of gym <= 0.21 (called at custom_envs/envs/baseenvironment.py:17,28):
seed -> int mod 2**64 (os.urandom when None) -> first 8 bytes of
sha512(str(seed)) as little-endian uint32 words -> ``RandomState.seed``.
"""
import hashlib
import os

import numpy as np


def _words(data):
    data = data + b'\0' * (-len(data) % 4)
    return [int.from_bytes(data[i:i + 4], 'little') for i in range(0, len(data), 4)]


def key_words(seed):
    """uint32 key ``RandomState.seed`` receives for a normalised seed."""
    digest = hashlib.sha512(str(seed).encode('utf8')).digest()[:8]
    words = _words(digest)
    while len(words) > 1 and words[-1] == 0:
        words.pop()
    return words


def np_random(seed=None):
    """(RandomState, seed) as gym's ``np_random``."""
    if seed is None:
        seed = int.from_bytes(os.urandom(8), 'little')
    elif isinstance(seed, (int, np.integer)) and seed >= 0:
        seed = int(seed) % (1 << 64)
    else:
        raise ValueError('seed must be a non-negative integer or None, got %r' % (seed,))
    rng = np.random.RandomState()
    rng.seed(key_words(seed))
    return rng, seed
