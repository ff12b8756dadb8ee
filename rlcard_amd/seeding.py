"""Seed -> MT19937 init_by_array key, the host half of the per-env RNG contract.

Mirrors rlcard/utils/seeding.py:33-113: an int seed is reduced mod 2**64 (create_seed, :75-96), hashed with
sha512(str(seed)) and the first 8 bytes read as a little-endian integer (hash_seed, :51-73 and _bigint_from_bytes,
:99-108), which is split into little-endian u32 words with trailing zero words dropped (_int_list_from_bigint,
:110-121; 0 -> [0]). numpy's RandomState.seed(list) then runs init_by_array over those words; the device does the
same (mt_init_by_array, rlcard_amd/csrc/cs_kernels.hip). ``seed=None`` draws the seed from os.urandom like the reference.
"""
import hashlib
import os

import numpy as np

__all__ = ['create_seed', 'seed_key', 'seed_keys', 'seed_keys_range']


def create_seed(seed=None, max_bytes=8):
    if seed is None:
        return int.from_bytes(os.urandom(max_bytes), 'little')
    if isinstance(seed, str):
        b = seed.encode('utf8')
        b += hashlib.sha512(b).digest()
        return int.from_bytes(b[:max_bytes], 'little')
    if isinstance(seed, (int, np.integer)) and not isinstance(seed, bool):
        seed = int(seed)
        if seed < 0:
            raise ValueError('Seed must be a non-negative integer or omitted, not {}'.format(seed))
        return seed % (1 << (8 * max_bytes))
    raise ValueError('Invalid type for seed: {} ({})'.format(type(seed), seed))


def seed_key(seed=None):
    """-> (words, length): the init_by_array key for an env seed (1 or 2 u32 words)."""
    s = create_seed(seed)
    v = int.from_bytes(hashlib.sha512(str(s).encode('utf8')).digest()[:8], 'little')
    if v == 0:
        return (0, 0), 1
    lo, hi = v & 0xFFFFFFFF, v >> 32
    return ((lo, hi), 2) if hi else ((lo, 0), 1)


def seed_keys(seeds):
    """Per-env keys for an iterable of seeds -> (uint32 [n, 2], int32 [n])."""
    seeds = list(seeds)
    keys = np.zeros((len(seeds), 2), dtype=np.uint32)
    lens = np.zeros(len(seeds), dtype=np.int32)
    for i, s in enumerate(seeds):
        (k0, k1), n = seed_key(s)
        keys[i, 0], keys[i, 1], lens[i] = k0, k1, n
    return keys, lens


def seed_keys_range(base_seed, first, count):
    """Keys for the seeds base_seed + first .. base_seed + first + count - 1 (env i gets seed base + i)."""
    return seed_keys(range(int(base_seed) + int(first), int(base_seed) + int(first) + int(count)))
