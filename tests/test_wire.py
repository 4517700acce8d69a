"""Wire step after the query: NetworkEngine::bufferNodes packing
(network_engine.cpp:942-974) and the deserializeNodes filter (:788-828, isMartian :308-339).
CPU: the oracle against hand-derived known answers. GPU: kad_buffer_nodes_batch /
kad_parse_nodes_batch bit-exact against the oracle."""
import socket

import numpy as np
import pytest
import torch

import oracle as O
import tables as TB
from opendht_amd import DeviceTable, ops


def v4(ip, port):
    return np.frombuffer(socket.inet_pton(socket.AF_INET, ip) + port.to_bytes(2, "big"), np.uint8)


def v6(ip, port):
    return np.frombuffer(socket.inet_pton(socket.AF_INET6, ip) + port.to_bytes(2, "big"), np.uint8)


MARTIAN4 = [("0.1.2.3", 80), ("127.0.0.1", 4222), ("224.0.0.1", 4222), ("255.255.255.255", 1), ("8.8.8.8", 0)]
SANE4 = [("8.8.8.8", 4222), ("192.168.1.2", 1), ("223.255.255.255", 65535), ("1.0.0.0", 4222)]
MARTIAN6 = [("ff02::1", 4222), ("fe80::1", 4222), ("febf::1", 4222), ("::", 4222), ("::1", 4222),
            ("::ffff:8.8.8.8", 4222), ("2001:db8::1", 0)]
SANE6 = [("2001:db8::1", 4222), ("fec0::1", 4222), ("::2", 4222), ("::fffe:8.8.8.8", 4222), ("fe00::1", 1)]


def test_is_martian_known_answers():
    for ip, port in MARTIAN4:
        assert O.lib().orc_is_martian(v4(ip, port).tobytes(), 6), (ip, port)
    for ip, port in SANE4:
        assert not O.lib().orc_is_martian(v4(ip, port).tobytes(), 6), (ip, port)
    for ip, port in MARTIAN6:
        assert O.lib().orc_is_martian(v6(ip, port).tobytes(), 18), (ip, port)
    for ip, port in SANE6:
        assert not O.lib().orc_is_martian(v6(ip, port).tobytes(), 18), (ip, port)


def test_buffer_nodes_known_answer():
    """Three nodes, target 00..0: sorted ascending by ID (= XOR distance), records = ID + addr."""
    ids = np.zeros((3, 20), np.uint8)
    ids[0, 0], ids[1, 0], ids[2, 19] = 0x80, 0x01, 0x05
    addrs = np.stack([v4("10.0.0.1", 1), v4("10.0.0.2", 2), v4("10.0.0.3", 3)])
    out, n = O.buffer_nodes(np.zeros((1, 20), np.uint8), ids, addrs, np.array([[0, 1, 2]], np.uint32),
                            np.array([3], np.uint8))
    assert n[0] == 3
    rec = out[0].reshape(8, 26)
    for slot, node in enumerate((2, 1, 0)):
        assert bytes(rec[slot, :20]) == bytes(ids[node]) and bytes(rec[slot, 20:]) == bytes(addrs[node])
    # truncation to SEND_NODES = 8
    ids = np.arange(12 * 20, dtype=np.uint8).reshape(12, 20)
    addrs = np.zeros((12, 6), np.uint8)
    out, n = O.buffer_nodes(np.zeros((1, 20), np.uint8), ids, addrs, np.arange(12, dtype=np.uint32)[None],
                            np.array([12], np.uint8))
    assert n[0] == 8 and bytes(out[0].reshape(8, 26)[7, :20]) == bytes(ids[7])


def _addrs(n, six, seed):
    rng = np.random.default_rng(seed)
    a = rng.integers(0, 256, (n, 18 if six else 6), dtype=np.uint8)
    return a


@pytest.mark.gpu
@pytest.mark.parametrize("six", [False, True], ids=["v4", "v6"])
def test_buffer_nodes_parity(gpu, six):
    t = TB.uniform_config(20_000, 11, seed=0xB0F + six)
    targets = TB.adversarial_targets(t, extra=3000)
    tg = torch.from_numpy(targets).to(gpu)
    addrs = _addrs(t["ids"].shape[0], six, 5)
    with DeviceTable(t["ids"], t["status"], t["first"], t["off"], device=gpu.index or 0, sorted=True) as T:
        T.set_addrs(addrs)
        for kind, k in (("rt", 8), ("rt", 32), ("nc", 14), ("nc", 32)):
            idx, cnt = T.rt_closest(tg, k) if kind == "rt" else T.nc_closest(tg, k)
            for use_cnt in (True, False):
                out, n = T.buffer_nodes(tg, idx, cnt if use_cnt else None)
                torch.cuda.synchronize()
                want, wn = O.buffer_nodes(targets, t["ids"], addrs, idx.cpu().numpy().view(np.uint32),
                                          cnt.cpu().numpy())
                np.testing.assert_array_equal(n.cpu().numpy(), wn, err_msg=f"{kind} k={k}")
                np.testing.assert_array_equal(out.cpu().numpy(), want, err_msg=f"{kind} k={k} cnt={use_cnt}")


@pytest.mark.gpu
@pytest.mark.parametrize("rec_len", [26, 38])
def test_parse_nodes_parity(gpu, rec_len):
    rng = np.random.default_rng(rec_len)
    n = 5000
    rec = rng.integers(0, 256, (n, rec_len), dtype=np.uint8)
    myid = rng.integers(0, 256, 20, dtype=np.uint8)
    rec[::17, :20] = myid
    fam = [(MARTIAN4 + SANE4, v4)] if rec_len == 26 else [(MARTIAN6 + SANE6, v6)]
    for j, (ip, port) in enumerate(fam[0][0]):
        rec[3 + 11 * j, 20:] = fam[0][1](ip, port)
    rec[5::7, 20] = 127 if rec_len == 26 else 0xFF
    keep = ops.parse_nodes(torch.from_numpy(rec.reshape(-1)).to(gpu), rec_len, myid.tobytes())
    torch.cuda.synchronize()
    want = O.parse_nodes(rec, rec_len, myid)
    np.testing.assert_array_equal(keep.cpu().numpy(), want)
    assert 0 < want.sum() < n
