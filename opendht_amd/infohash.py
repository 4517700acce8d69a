"""InfoHash: the 160-bit node/key identifier (reference include/opendht/infohash.h:58-215).

A host-side value type with the reference's scalar API (cmp, xorCmp, commonBits, lowbit,
getBit/setBit, ordering). Scalars are control-path helpers, as the reference's inline header
functions are; the batched, data-parallel forms run on the GPU (``kad_xor_cmp_batch``,
``kad_common_bits_batch``, ``kad_lowbit_batch``) and are exposed in ``opendht_amd.ops``.
"""
from __future__ import annotations

import os

HASH_LEN = 20  # infohash.h:49


class InfoHash:
    __slots__ = ("_b",)

    def __init__(self, data: bytes | bytearray | str | None = None):
        if data is None:
            self._b = bytes(HASH_LEN)
        elif isinstance(data, str):  # infohash.h:74 (hex, at least 40 chars; extra ignored)
            if len(data) < 2 * HASH_LEN:
                self._b = bytes(HASH_LEN)
            else:
                self._b = bytes.fromhex(data[: 2 * HASH_LEN])
        else:
            b = bytes(data)
            # infohash.h:62-67: shorter input -> zeroes, longer -> first HASH_LEN bytes
            self._b = b[:HASH_LEN] if len(b) >= HASH_LEN else bytes(HASH_LEN)

    # -- construction --------------------------------------------------------------------
    @staticmethod
    def getRandom() -> "InfoHash":  # infohash.cpp:63-75
        return InfoHash(os.urandom(HASH_LEN))

    def toString(self) -> str:
        return self._b.hex()

    def __bytes__(self) -> bytes:
        return self._b

    def __repr__(self) -> str:
        return f"InfoHash({self._b.hex()})"

    def __hash__(self) -> int:
        return hash(self._b)

    def __bool__(self) -> bool:
        return any(self._b)

    def __getitem__(self, i: int) -> int:
        return self._b[i]

    # -- ordering: memcmp, byte 0 most significant (infohash.h:101-103, 173-180) -----------
    def __eq__(self, o) -> bool:
        return isinstance(o, InfoHash) and self._b == o._b

    def __lt__(self, o: "InfoHash") -> bool:
        return self._b < o._b

    def __le__(self, o: "InfoHash") -> bool:
        return self._b <= o._b

    def __gt__(self, o: "InfoHash") -> bool:
        return self._b > o._b

    def __ge__(self, o: "InfoHash") -> bool:
        return self._b >= o._b

    @staticmethod
    def cmp(a: "InfoHash", b: "InfoHash") -> int:
        return (a._b > b._b) - (a._b < b._b)

    # -- XOR metric ------------------------------------------------------------------------
    def xorCmp(self, id1: "InfoHash", id2: "InfoHash") -> int:  # infohash.h:131-146
        t = int.from_bytes(self._b, "big")
        d1 = int.from_bytes(id1._b, "big") ^ t
        d2 = int.from_bytes(id2._b, "big") ^ t
        return (d1 > d2) - (d1 < d2)

    @staticmethod
    def commonBits(a: "InfoHash", b: "InfoHash") -> int:  # infohash.h:106-128
        x = int.from_bytes(a._b, "big") ^ int.from_bytes(b._b, "big")
        return 8 * HASH_LEN - x.bit_length()

    def lowbit(self) -> int:  # infohash.h:84-95; (unsigned)-1 for zero
        x = int.from_bytes(self._b, "big")
        if x == 0:
            return 0xFFFFFFFF
        return 8 * HASH_LEN - 1 - ((x & -x).bit_length() - 1)

    def getBit(self, n: int) -> bool:  # infohash.h:148-154
        return bool((self._b[n // 8] >> (7 - n % 8)) & 1)

    def setBit(self, n: int, b: bool) -> None:  # infohash.h:156-162
        a = bytearray(self._b)
        bit = 7 - n % 8
        a[n // 8] = (a[n // 8] & ~(1 << bit)) | (int(bool(b)) << bit)
        self._b = bytes(a)


zeroes = InfoHash()  # infohash.h:217
