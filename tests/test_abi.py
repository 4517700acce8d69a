"""CPU tests of the C ABI library: it loads, exports every symbol include/kadgpu.h declares,
its host-side builders agree with the oracle, and table creation fails loudly without a GPU."""
import os
import re

import numpy as np
import pytest

import oracle as O
from opendht_amd import _lib
from opendht_amd import synth as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "kadgpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kad_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.SIGNATURES), set(syms) ^ set(_lib.SIGNATURES)


def test_version():
    assert _lib.lib().kad_version() >= 100


def test_synth_ids_match_oracle_recipe():
    for n, seed in ((1000, S.SEED_IDS), (5000, 123)):
        np.testing.assert_array_equal(S.random_ids(n, seed), O.synth_ids(n, seed))
        np.testing.assert_array_equal(S.random_status(n, seed), O.synth_status(n, seed))


def test_uniform_buckets():
    ids, _ = S.sort_ids(S.random_ids(5000))
    first, off = S.uniform_buckets(ids, 8)
    assert first.shape == (256, 20) and off[0] == 0 and off[-1] == 5000
    assert (np.diff(off.astype(np.int64)) >= 0).all()
    top = ids[:, 0]
    for b in (0, 17, 255):
        assert (top[off[b]:off[b + 1]] == b).all()


def test_uniform_shard_reproducible_by_range():
    a_ids, a_st, a_off = S.uniform_shard(5, 10, 0, 1024, 6.0)
    b_ids, b_st, b_off = S.uniform_shard(5, 10, 300, 700, 6.0)
    n0 = a_off[300]
    np.testing.assert_array_equal(a_ids[n0:a_off[700]], b_ids)
    np.testing.assert_array_equal(a_st[n0:a_off[700]], b_st)
    np.testing.assert_array_equal(a_off[300:701] - n0, b_off)
    assert (np.diff(a_ids.view(">u4").reshape(-1, 5)[:, 0].astype(np.int64)) >= 0).all()


def test_table_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from opendht_amd import DeviceTable, KadError
    t_ids, _ = S.sort_ids(S.random_ids(100))
    first, off = S.uniform_buckets(t_ids, 4)
    with pytest.raises(KadError) as e:
        DeviceTable(t_ids, np.ones(100, np.uint8), first, off)
    assert "NO_DEVICE" in str(e.value)


def test_bad_directory_rejected_before_device():
    from opendht_amd import DeviceTable, KadError
    t_ids, _ = S.sort_ids(S.random_ids(100))
    first, off = S.uniform_buckets(t_ids, 4)
    off_bad = off.copy()
    off_bad[-1] = 99
    with pytest.raises(KadError) as e:
        DeviceTable(t_ids, np.ones(100, np.uint8), first, off_bad)
    assert "INVALID" in str(e.value)
    with pytest.raises(KadError) as e:
        DeviceTable(t_ids[::-1], np.ones(100, np.uint8), None, None, sorted=True)
    assert "NOT_SORTED" in str(e.value)
