"""The Python InfoHash value type (control-path helper) against the oracle's restatement."""
import numpy as np

import oracle as O
from opendht_amd import InfoHash, zeroes


def test_infohash_scalars_match_oracle():
    rng = np.random.default_rng(4)
    for _ in range(500):
        a, b, t = (rng.integers(0, 256, 20, dtype=np.uint8).tobytes() for _ in range(3))
        if rng.random() < 0.5:
            k = int(rng.integers(0, 21))
            b = a[:k] + b[k:]
        A, B, T = InfoHash(a), InfoHash(b), InfoHash(t)
        assert InfoHash.commonBits(A, B) == O.common_bits(a, b)
        assert T.xorCmp(A, B) == O.xor_cmp(t, a, b)
        assert A.lowbit() == O.lowbit(a)
        assert InfoHash.cmp(A, B) == O.cmp(a, b)
        assert (A < B) == (O.cmp(a, b) < 0)


def test_infohash_bits_and_construction():
    h = InfoHash()
    assert h == zeroes and not h and h.lowbit() == 0xFFFFFFFF
    h.setBit(0, True)
    assert h.getBit(0) and h[0] == 0x80 and h.lowbit() == 0
    h.setBit(159, True)
    assert h[19] == 1 and h.lowbit() == 159
    h.setBit(0, False)
    assert not h.getBit(0)
    assert InfoHash("ab" * 20).toString() == "ab" * 20
    assert InfoHash(b"\x01\x02") == zeroes  # too short -> zeroes (infohash.h:62-67)
