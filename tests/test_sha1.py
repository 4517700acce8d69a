"""Batched InfoHash::get: SHA-1 of keys (infohash.cpp:46-61). The reference
hashes with GnuTLS (absent here, version unpinned: gnutls >= 3.3), so the oracle's FIPS 180-4 SHA-1
is pinned by the standard's test vectors, then the GPU is checked against the oracle."""
import hashlib

import numpy as np
import pytest
import torch

import oracle as O
from opendht_amd import ops

FIPS = [  # FIPS 180-4 / 180-2 appendix A examples
    (b"abc", "a9993e364706816aba3e25717850c26c9cd0d89d"),
    (b"abcdbcdecdefdefgefghfghighijhijkijkljklmklmnlmnomnopnopq", "84983e441c3bd26ebaae4aa1f95129e5e54670f1"),
    (b"a" * 1_000_000, "34aa973cd4c4daa4f61eeb2bdbad27316534016f"),
    (b"", "da39a3ee5e6b4b0d3255bfef95601890afd80709"),
]


def _keys(n, seed):
    rng = np.random.default_rng(seed)
    lens = np.concatenate([np.arange(0, 140), rng.integers(0, 300, n - 140)])
    return [rng.integers(0, 256, int(m), dtype=np.uint8).tobytes() for m in lens]


def test_oracle_sha1_fips_vectors():
    got = O.infohash_get([m for m, _ in FIPS])
    for (m, h), g in zip(FIPS, got):
        assert bytes(g).hex() == h


def test_oracle_sha1_matches_hashlib():
    keys = _keys(600, 1)
    got = O.infohash_get(keys)
    for k, g in zip(keys, got):
        assert bytes(g) == hashlib.sha1(k).digest()


@pytest.mark.gpu
def test_infohash_get_gpu(gpu):
    keys = [m for m, _ in FIPS] + _keys(5000, 2) + [b"key:%d" % i for i in range(3000)]
    data = np.frombuffer(b"".join(keys), np.uint8)
    off = np.concatenate([[0], np.cumsum([len(k) for k in keys])]).astype(np.int64)
    # odd start: every key boundary at every byte alignment
    buf = torch.from_numpy(np.concatenate([np.zeros(3, np.uint8), data])).to(gpu)
    out = ops.infohash_get(buf[3:], torch.from_numpy(off).to(gpu))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), O.infohash_get(keys))
    for (m, h), g in zip(FIPS, out.cpu().numpy()):
        assert bytes(g).hex() == h
