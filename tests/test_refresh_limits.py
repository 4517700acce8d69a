"""The one-launch small refresh at its inline limits (kad_engine.hip rf_nodes_kernel, host side
small_refresh / rf_check_inline): kernel arguments carry up to 128 passed-deadline nodes (RF_INLINE), their buckets
and, for window-line tables, up to 16 runs of lines to rebuild with up to 256 bucket offsets (RF_HOFF). One refresh
here passes exactly 128 chosen deadlines (node.cpp:34-40) in buckets laid out to fill those limits exactly —
16 runs, 256 offsets, runs at bucket 0 and bucket B - 1 — and just past them (17 runs; 257 offsets), where the host
falls back to letting the builder blocks derive the lines. After each refresh every derived array (window, short,
general, slot and NodeCache lines, good counts, directory masks) equals a fresh build bit for bit, the queries equal
the oracle, and no kernel bounds guard fired (kad_table_refresh_diag)."""
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

import oracle as O
import rf_cases as R
import tables as TB
from opendht_amd import DeviceTable, _lib

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _layouts(B):
    """(name, runs, expected hoff entries): the exact limits and one past each."""
    gap = 20
    # 16 runs: 6 buckets at bucket 0, 11 interior runs of 6 and 3 of 4, 6 buckets ending at B - 1: 6 + 6 + 6
    # (ends) ... = 12 + 14 * 11 + 90 = 256 offsets
    sizes = [6] + [6] * 11 + [4] * 3 + [6]
    runs, f = [], 0
    for i, m in enumerate(sizes[:-1]):
        runs.append((f, m))
        f += m + gap
    runs.append((B - sizes[-1], sizes[-1]))
    exact = runs
    r17 = runs[:-1] + [(f, 1)] + [runs[-1]]                          # a 17th run (of one bucket)
    r257 = [runs[0], (runs[1][0], runs[1][1] + 1)] + runs[2:]         # one more bucket in run 1: 257 offsets
    return [("16runs_256off", exact, 256), ("17runs", r17, None), ("257off", r257, 257)]


def _case(gpu, t, runs, slot_lines=True, seed=1):
    B = t["off"].shape[0] - 1
    buckets = R.runs_layout(B, runs)
    now0 = 1000 * 3600 * 10**9
    time_ns, reply_ns, expired, chosen = R.times_for(t, buckets, 128, now0, seed)
    st0 = R.status_at(time_ns, reply_ns, expired, now0)
    with DeviceTable(t["ids"], st0, t["first"], t["off"], device=0, sorted=t["sorted"], eager=True,
                     slot_lines=slot_lines) as T:
        T.set_times(time_ns, reply_ns, expired)
        T.refresh_status(now0)
        now1 = now0 + 10**4
        T.refresh_status(now1)
        torch.cuda.synchronize()
        st1 = R.status_at(time_ns, reply_ns, expired, now1)
        assert int((st0 != st1).sum()) == 128  # exactly the chosen nodes flipped
        np.testing.assert_array_equal(T.export_status(), st1)
        R.compare_fresh(DeviceTable, _lib, T, t, st1, "after 128 deadlines", slot_lines=slot_lines)
        # targets in and next to every run's buckets (first bucket, last bucket included) and random ones
        near = np.concatenate([t["ids"][t["off"][max(0, f - 3)]:t["off"][min(B, f + m + 3)]] for f, m in runs])
        targets = np.ascontiguousarray(np.concatenate([TB.adversarial_targets(t, extra=500), near]))
        tg = torch.from_numpy(targets).to(gpu)
        for k in (1, 8, 14, 32):
            idx, cnt = T.rt_closest(tg, k)
            torch.cuda.synchronize()
            want, wcnt = O.flat_rt_closest(t["ids"], st1, t["first"], t["off"], targets, k, nthreads=8)
            np.testing.assert_array_equal(cnt.cpu().numpy(), wcnt, err_msg=f"k={k} counts")
            np.testing.assert_array_equal(idx.cpu().numpy().view(np.uint32), want, err_msg=f"k={k}")
        return T.refresh_diag()


@pytest.mark.parametrize("n", [40_000, 60_000])
@pytest.mark.parametrize("layout", [0, 1, 2], ids=["16runs_256off", "17runs", "257off"])
def test_inline_limits_window_lines(gpu, n, layout):
    """Uniform U(12) tables (window lines, the FUSE 1 launch). At ~10 nodes per bucket about a third of the
    W(2) windows exceed 64 nodes, at ~15 most do: their builder waves stage them (up to 1,024 nodes) with this
    refresh's statuses and build them without waiting for block 0."""
    t = TB.uniform_config(n, 12, seed=0x1A0 + n)
    B = t["off"].shape[0] - 1
    name, runs, want_off = _layouts(B)[layout]
    if want_off is not None:
        assert R.hoff_entries(B, runs) == want_off, name
    assert runs[0][0] == 0 and runs[-1][0] + runs[-1][1] == B
    d = _case(gpu, t, runs, seed=layout)
    assert d["guard_errors"] == 0, d
    assert d["spin_timeouts"] == 0, d
    # windows of 65 .. 1,024 nodes (most of them at n = 60,000) are staged and built by their builder waves
    assert d["last_block_lines"] == 0, d


def test_huge_windows_last_block(gpu):
    """U(6) at 60,000 nodes: ~940 nodes per bucket, so every W(2) exceeds the builders' 1,024-node staging and the
    host turns the completion protocol on; the launch's last block builds those lines."""
    t = TB.uniform_config(60_000, 6, seed=0x1A9)
    runs = [(0, 2), (30, 2), (62, 2)]
    d = _case(gpu, t, runs, seed=3)
    assert d["guard_errors"] == 0 and d["spin_timeouts"] == 0, d
    assert d["last_block_lines"] > 0, d


@pytest.mark.parametrize("layout", [0, 1], ids=["16runs_256off", "17runs"])
def test_inline_limits_general_lines(gpu, layout):
    """A split-policy table without slot lines (the FUSE 2 launch: block 0 publishes the general-line list)."""
    t = TB.split_config(40_000, seed=0x1A7)
    B = t["off"].shape[0] - 1
    name, runs, _ = _layouts(B)[layout]
    d = _case(gpu, t, runs, slot_lines=False, seed=10 + layout)
    assert d["guard_errors"] == 0 and d["spin_timeouts"] == 0, d


def test_block0_delayed_builders_time_out():
    """The builders' wait for block 0's list is bounded (1 s); when it times out (block 0 not running, here held
    back on purpose by the tools build's KAD_RF_ABL=3 hook) the launch's last block builds the lines, so the
    results stay exact and the timeout is counted (kad_table_refresh_diag). Runs in a child process because it
    loads the tools library (libkadgpu_abl.so)."""
    abl = os.path.join(os.path.dirname(HERE), "opendht_amd", "libkadgpu_abl.so")
    if not os.path.exists(abl):
        pytest.fail("libkadgpu_abl.so is missing (make -C opendht_amd/csrc ablations)")
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rf_delay_worker.py")], capture_output=True, text=True,
                       timeout=240)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "RF_DELAY_OK" in r.stdout
