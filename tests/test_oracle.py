"""CPU tests of the oracle (test infrastructure): known-answer tests of the InfoHash primitives,
agreement of the two independent restatements (structure-faithful list/map vs closed-form flat)
on every test table, and the committed golden fixtures.

Parity status: "parity unpinned" -- the OpenDHT reference cannot be built here (DESIGN.md
"Oracle"), so the known answers below are derived by hand from infohash.h's definitions."""
import numpy as np
import pytest

import oracle as O
import tables as TB


def h(s: str) -> bytes:
    return bytes.fromhex(s.ljust(40, "0"))


Z = bytes(20)
F = b"\xff" * 20


class TestPrimitiveKAT:
    # infohash.h:106-128 commonBits
    @pytest.mark.parametrize("a,b,want", [
        (Z, Z, 160), (F, F, 160), (Z, F, 0), (h("80"), Z, 0), (h("40"), Z, 1), (h("01"), Z, 7),
        (h("0001"), Z, 15), (Z[:19] + b"\x01", Z, 159), (h("00000000000000000001"), Z, 79),
    ])
    def test_common_bits(self, a, b, want):
        assert O.common_bits(a, b) == want

    # infohash.h:84-95 lowbit: index from MSB of the lowest set bit; (unsigned)-1 for zero
    @pytest.mark.parametrize("a,want", [
        (Z, 0xFFFFFFFF), (h("80"), 0), (h("01"), 7), (h("0080"), 8), (F, 159), (Z[:19] + b"\x02", 158),
        (h("c0"), 1),
    ])
    def test_lowbit(self, a, want):
        assert O.lowbit(a) == want

    # infohash.h:131-146 xorCmp: which of id1/id2 is closer to the target
    @pytest.mark.parametrize("t,a,b,want", [
        (Z, h("01"), h("02"), -1), (Z, h("02"), h("01"), 1), (Z, h("05"), h("05"), 0),
        (F, h("ff"), h("7f"), -1), (h("80"), h("7f"), h("ff"), 1), (h("12"), h("13"), h("10"), -1),
        (Z, Z[:19] + b"\x02", Z[:19] + b"\x01", 1),
    ])
    def test_xor_cmp(self, t, a, b, want):
        assert O.xor_cmp(t, a, b) == want

    def test_cmp_is_memcmp(self):
        assert O.cmp(h("01"), h("02")) == -1 and O.cmp(h("ff"), h("01")) == 1 and O.cmp(Z, Z) == 0

    def test_xor_cmp_is_unsigned_160_compare(self):
        rng = np.random.default_rng(0)
        for _ in range(2000):
            t, a, b = (rng.integers(0, 256, 20, dtype=np.uint8).tobytes() for _ in range(3))
            if rng.random() < 0.3:  # shared prefixes
                k = int(rng.integers(0, 20))
                b = a[:k] + b[k:]
            ti, ai, bi = (int.from_bytes(x, "big") for x in (t, a, b))
            want = ((ai ^ ti) > (bi ^ ti)) - ((ai ^ ti) < (bi ^ ti))
            assert O.xor_cmp(t, a, b) == want


def _check_restatements(t, targets, counts=(0, 1, 8, 14, 16, 32)):
    T = O.FaithfulTable(t["ids"], t["status"], t["first"], t["off"], with_nc=t["sorted"])
    for k in counts:
        a, ac = T.rt_closest(targets, k)
        b, bc = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], targets, k)
        np.testing.assert_array_equal(ac, bc, err_msg=f"{t['name']} k={k} counts")
        np.testing.assert_array_equal(a, b, err_msg=f"{t['name']} k={k} idx")
        if t["sorted"]:
            a, ac = T.nc_closest(targets, k)
            b, bc = O.flat_nc_closest(t["ids"], t["status"], targets, k)
            np.testing.assert_array_equal(ac, bc, err_msg=f"{t['name']} nc k={k}")
            np.testing.assert_array_equal(a, b, err_msg=f"{t['name']} nc k={k}")


@pytest.mark.parametrize("t", TB.all_small_tables(), ids=lambda t: t["name"])
def test_restatements_agree(t):
    if t["first"] is None:
        pytest.skip("no buckets")
    _check_restatements(t, TB.adversarial_targets(t))


def test_results_sorted_by_xor_distance():
    t = TB.split_config(10_000)
    tg = TB.adversarial_targets(t)
    idx, cnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], tg, 16)
    for i in range(tg.shape[0]):
        rows = idx[i, : cnt[i]]
        assert (t["status"][rows] & 1).all()
        d = [int.from_bytes((t["ids"][r] ^ tg[i]).tobytes(), "big") for r in rows]
        assert d == sorted(d)


def test_reference_is_not_global_knn():
    """the window semantics differ from a brute-force global top-k."""
    t = TB.split_config(10_000)
    tg = TB.adversarial_targets(t, extra=400)[-400:]
    idx, cnt = O.flat_rt_closest(t["ids"], t["status"], t["first"], t["off"], tg, 8)
    good = np.nonzero(t["status"] & 1)[0]
    gi = [int.from_bytes(t["ids"][g].tobytes(), "big") for g in good]
    diff = 0
    for i in range(tg.shape[0]):
        ti = int.from_bytes(tg[i].tobytes(), "big")
        best = [good[j] for j in sorted(range(len(good)), key=lambda j: gi[j] ^ ti)[:8]]
        diff += list(idx[i, : cnt[i]]) != best
    assert diff > 0


def test_golden_fixtures():
    import os
    path = os.path.join(os.path.dirname(__file__), "golden", "config1.npz")
    g = np.load(path, allow_pickle=False)
    for shape in ("S", "U"):
        ids, st, first, off, tg = (g[f"{shape}_{k}"] for k in ("ids", "status", "first", "off", "targets"))
        for k in (8, 16, 32):
            idx, cnt = O.flat_rt_closest(ids, st, first, off, tg, k)
            np.testing.assert_array_equal(idx, g[f"{shape}_rt_idx_k{k}"])
            np.testing.assert_array_equal(cnt, g[f"{shape}_rt_cnt_k{k}"])
        if shape == "U":
            for k in (8, 14, 32):
                idx, cnt = O.flat_nc_closest(ids, st, tg, k)
                np.testing.assert_array_equal(idx, g[f"U_nc_idx_k{k}"])
                np.testing.assert_array_equal(cnt, g[f"U_nc_cnt_k{k}"])


def test_split_builder_matches_faithful():
    from opendht_amd import synth as S
    for n, seed in ((10_000, S.SEED_IDS), (3000, 11), (50, 12)):
        ids = S.random_ids(n, seed)
        a = S.split_table(ids)
        b = O.split_table(ids)
        for x, y in zip(a, b):
            np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize("t", [x for x in TB.all_small_tables() if x["sorted"] and x["first"] is not None],
                         ids=lambda t: t["name"])
def test_restatements_agree_large_counts(t):
    """Both restatements for counts above the line kernels' (RoutingTable and NodeCache take any size_t count,
    routing_table.h:48, node_cache.h:32), up to counts larger than the table."""
    _check_restatements(t, TB.adversarial_targets(t, extra=64), counts=(65, 300, 1000, t["ids"].shape[0] + 7))
