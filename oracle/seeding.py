"""Restatement of old-gym seeding (TEST INFRASTRUCTURE ONLY).

The reference seeds every environment with ``gym.utils.seeding.np_random``
(``custom_envs/envs/baseenvironment.py:17,28``).  ``gym`` is not installed
in this image and ``setup.py:13-22`` leaves it unpinned; the RandomState
return type used by ``use_random_state`` (``custom_envs/utils/utils_math.py:
9-22``) implies gym <= 0.21, whose published algorithm is restated here:

    np_random(seed):  seed = create_seed(seed)            (int mod 2**64)
                      key  = _int_list_from_bigint(hash_seed(seed))
                      rng  = numpy.random.RandomState(); rng.seed(key)
    hash_seed(seed):  first 8 bytes of sha512(str(seed)) read as
                      little-endian uint32 words -> big integer
    _int_list_from_bigint: base-2**32 digits, least significant first

No reference test pins seed -> stream, so this part of the oracle is
"parity unpinned" (DESIGN.md, section Oracle).
"""
import hashlib
import os
import struct

import numpy as np


def _bigint_from_bytes(data):
    """gym.utils.seeding._bigint_from_bytes (4-byte little-endian words)."""
    pad = 4 - len(data) % 4
    data = data + b"\0" * pad
    words = struct.unpack("<%dI" % (len(data) // 4), data)
    total = 0
    for i, word in enumerate(words):
        total += word << (32 * i)
    return total


def _int_list_from_bigint(value):
    if value < 0:
        raise ValueError("seed must be non-negative")
    if value == 0:
        return [0]
    out = []
    while value > 0:
        value, low = divmod(value, 1 << 32)
        out.append(low)
    return out


def create_seed(seed=None, max_bytes=8):
    if seed is None:
        return _bigint_from_bytes(os.urandom(max_bytes))
    if isinstance(seed, str):
        raw = seed.encode("utf8")
        raw += hashlib.sha512(raw).digest()
        return _bigint_from_bytes(raw[:max_bytes])
    if isinstance(seed, (int, np.integer)):
        return int(seed) % (1 << (8 * max_bytes))
    raise TypeError("invalid seed type %r" % type(seed))


def hash_seed(seed=None, max_bytes=8):
    if seed is None:
        seed = create_seed(max_bytes=max_bytes)
    digest = hashlib.sha512(str(seed).encode("utf8")).digest()
    return _bigint_from_bytes(digest[:max_bytes])


def seed_key(seed):
    """The uint32 key array handed to ``RandomState.seed`` for ``seed``."""
    return _int_list_from_bigint(hash_seed(create_seed(seed)))


def np_random(seed=None):
    """Old-gym ``np_random``: returns ``(RandomState, seed)``."""
    if seed is not None and not (isinstance(seed, (int, np.integer))
                                 and seed >= 0):
        raise ValueError("seed must be a non-negative integer or None")
    seed = create_seed(seed)
    rng = np.random.RandomState()
    rng.seed(_int_list_from_bigint(hash_seed(seed)))
    return rng, seed
