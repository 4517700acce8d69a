"""The window-line kernel's comparator networks (opendht_amd/csrc/kad_engine.hip: SORT8, merge8),
checked exhaustively by the 0-1 principle: a comparator network sorts every input iff it sorts
every 0-1 input. The tables are parsed from the kernel source, so the test checks what ships."""
import itertools
import os
import random
import re

import numpy as np

SRC = os.path.join(os.path.dirname(__file__), "..", "opendht_amd", "csrc", "kad_engine.hip")


def _net(name):
    s = open(SRC).read()
    m = re.search(name + r"\[" + name + r"_LEN\]\[2\]\s*=\s*\{(.*?)\};", s, re.S)
    pairs = [tuple(map(int, p)) for p in re.findall(r"\{(\d+),\s*(\d+)\}", m.group(1))]
    n = int(re.search(name + r"_LEN = (\d+);", s).group(1))
    assert len(pairs) == n
    return pairs


def _sort8():
    return _net("SORT8")


def _apply(net, v):
    v = list(v)
    for a, b in net:
        if v[a] > v[b]:
            v[a], v[b] = v[b], v[a]
    return v


def _merge8(a, s):
    """merge8 of kad_engine.hip: bitonic min of (a, reversed s), then a half-cleaner cascade."""
    a = [min(a[i], s[7 - i]) for i in range(8)]
    net = [(i, i + 4) for i in range(4)] + [(i, i + 2) for i in range(8) if (i & 2) == 0] + \
          [(i, i + 1) for i in range(0, 8, 2)]
    return _apply(net, a)


def test_sort8_sorts_all_01_inputs():
    net = _sort8()
    assert all(a < b for a, b in net)
    for bits in itertools.product((0, 1), repeat=8):
        assert _apply(net, bits) == sorted(bits), bits


def test_merge8_keeps_8_smallest_sorted():
    # 0-1 principle over all sorted 0-1 pairs, plus random integer lists with duplicates
    for za in range(9):
        for zs in range(9):
            a = [0] * za + [1] * (8 - za)
            s = [0] * zs + [1] * (8 - zs)
            assert _merge8(a, s) == sorted(a + s)[:8]
    rng = np.random.default_rng(7)
    for _ in range(2000):
        a = sorted(rng.integers(0, 40, 8).tolist())
        s = sorted(rng.integers(0, 40, 8).tolist())
        assert _merge8(a, s) == sorted(a + s)[:8]


def test_top8_of_24():
    """sort8 x 3 + merge8 x 2 (the kernel's ranking) = the 8 smallest of 24, sorted."""
    net = _sort8()
    rnd = random.Random(11)
    for _ in range(3000):
        v = rnd.sample(range(1 << 20), 24)
        g = [_apply(net, v[i:i + 8]) for i in (0, 8, 16)]
        acc = _merge8(_merge8(g[0], g[1]), g[2])
        assert acc == sorted(v)[:8]


def test_sort16_sorts_all_01_inputs():
    net = _net("SORT16")
    assert all(a < b for a, b in net)
    for x in range(1 << 16):
        bits = [(x >> i) & 1 for i in range(16)]
        assert _apply(net, bits) == sorted(bits), bits


def _merge16(a, s):
    """merge16 of kad_engine.hip."""
    a = [min(a[i], s[15 - i]) for i in range(16)]
    net = [(i, i + w) for w in (8, 4, 2, 1) for i in range(16) if (i & w) == 0]
    return _apply(net, a)


def test_top16_of_32():
    net = _net("SORT16")
    rnd = random.Random(12)
    for _ in range(2000):
        v = rnd.sample(range(1 << 20), 32)
        acc = _merge16(_apply(net, v[:16]), _apply(net, v[16:]))
        assert acc == sorted(v)[:16]


def _join_sorted(a):
    """join_sorted<H> of kad_engine.hip: a sorted 2H from two sorted halves."""
    h = len(a) // 2
    net = [(i, 2 * h - 1 - i) for i in range(h)]
    w = h // 2
    while w >= 1:
        net += [(i, i + w) for i in range(2 * h) if (i & w) == 0]
        w //= 2
    return _apply(net, a)


def _merge32(a, s):
    """merge32 of kad_engine.hip."""
    a = [min(a[i], s[31 - i]) for i in range(32)]
    net = [(i, i + w) for w in (16, 8, 4, 2, 1) for i in range(32) if (i & w) == 0]
    return _apply(net, a)


def test_join_sorted_01():
    # 0-1 principle: every pair of sorted 0-1 halves of 16
    for za in range(17):
        for zb in range(17):
            a = [0] * za + [1] * (16 - za) + [0] * zb + [1] * (16 - zb)
            assert _join_sorted(a) == sorted(a)


def test_top32_of_64():
    """sort16 x 4 + join_sorted<16> x 2 + merge32 (the 64-slot lines' ranking) = the 32 smallest of
    64, sorted; random distinct values and values with duplicates (the NONE padding)."""
    net = _net("SORT16")
    rnd = random.Random(13)
    for trial in range(1500):
        if trial % 3 == 0:
            v = [rnd.randrange(40) for _ in range(64)]
        else:
            v = rnd.sample(range(1 << 20), 64)
        g = [_apply(net, v[i:i + 16]) for i in (0, 16, 32, 48)]
        acc = _merge32(_join_sorted(g[0] + g[1]), _join_sorted(g[2] + g[3]))
        assert acc == sorted(v)[:32]

