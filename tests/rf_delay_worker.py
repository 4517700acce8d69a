"""Child process of tests/test_refresh_limits.py::test_block0_delayed_builders_time_out: loads the tools library
(libkadgpu_abl.so) and refreshes with KAD_RF_ABL=3, which holds block 0 of the fused small refresh back for
RF_SPIN_TICKS + 0.2 s. The general-line builders' wait for block 0's list times out; the launch's last block must
then build the lines (results equal a fresh build), and the timeout must be counted. The window-line launch (its
builders never wait) is run the same way. Prints RF_DELAY_OK on success."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

from opendht_amd import _lib  # noqa: E402

_lib.use_ablation_build()

import numpy as np  # noqa: E402
import torch  # noqa: E402

import rf_cases as R  # noqa: E402
import tables as TB  # noqa: E402
from opendht_amd import DeviceTable  # noqa: E402


def run(t, runs, slot_lines, expect_timeouts):
    B = t["off"].shape[0] - 1
    buckets = R.runs_layout(B, runs)
    now0 = 2000 * 3600 * 10**9
    time_ns, reply_ns, expired, _ = R.times_for(t, buckets, 40, now0, 5)
    st0 = R.status_at(time_ns, reply_ns, expired, now0)
    with DeviceTable(t["ids"], st0, t["first"], t["off"], device=0, sorted=t["sorted"], eager=True,
                     slot_lines=slot_lines) as T:
        T.set_times(time_ns, reply_ns, expired)
        T.refresh_status(now0)
        torch.cuda.synchronize()
        os.environ["KAD_RF_ABL"] = "3"
        now1 = now0 + 10**4
        T.refresh_status(now1)
        torch.cuda.synchronize()
        os.environ.pop("KAD_RF_ABL")
        st1 = R.status_at(time_ns, reply_ns, expired, now1)
        np.testing.assert_array_equal(T.export_status(), st1)
        R.compare_fresh(DeviceTable, _lib, T, t, st1, f"{t['name']} delayed block 0", slot_lines=slot_lines)
        d = T.refresh_diag()
        print(t["name"], "slot_lines" if slot_lines else "no slot lines", d, flush=True)
        assert d["guard_errors"] == 0, d
        if expect_timeouts:
            assert d["spin_timeouts"] > 0 and d["last_block_lines"] > 0, d
            # after a timeout the table no longer fuses its general-line builds: the same delay
            # again spins nowhere (the count stays), and the rows are still exact
            os.environ["KAD_RF_ABL"] = "3"
            now2 = now1 + 10**4
            T.refresh_status(now2)
            torch.cuda.synchronize()
            os.environ.pop("KAD_RF_ABL")
            st2 = R.status_at(time_ns, reply_ns, expired, now2)
            np.testing.assert_array_equal(T.export_status(), st2)
            R.compare_fresh(DeviceTable, _lib, T, t, st2, f"{t['name']} delayed block 0, demoted", slot_lines=slot_lines)
            d2 = T.refresh_diag()
            print(t["name"], "after demotion", d2, flush=True)
            assert d2["spin_timeouts"] == d["spin_timeouts"] and d2["guard_errors"] == 0, (d, d2)
        else:
            assert d["spin_timeouts"] == 0, d


def main():
    torch.cuda.init()
    t = TB.split_config(30_000, seed=0x1B1)
    run(t, [(100, 10), (600, 10), (2000, 10)], slot_lines=False, expect_timeouts=True)   # FUSE 2
    u = TB.uniform_config(60_000, 12, seed=0x1B2)
    run(u, [(0, 4), (1000, 10), (4090, 6)], slot_lines=True, expect_timeouts=False)       # FUSE 1
    print("RF_DELAY_OK", flush=True)


if __name__ == "__main__":
    main()
