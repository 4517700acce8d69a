"""RCCL on the device: the multi-GPU modules branch on dist.get_backend() == "nccl"
(global_shard.exchange_into / gather_into / Exchange.overflowed / grown, sharded.route_queries / return_results),
and the CPU tests only run the gloo branches. This test opens a one-rank RCCL group on the box's GPU in a child
process (tests/rccl_world1_worker.py: a collective that hangs or a process group that fails cannot take the test
runner with it) and runs every one of those branches on device tensors, each result bit-exact against the
oracle."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def test_rccl_branches_world1():
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_world1_worker.py")], capture_output=True,
                       text=True, timeout=300, env=env)
    print(r.stdout[-4000:], r.stderr[-4000:])
    assert r.returncode == 0, r.stderr[-4000:]
    assert "RCCL_WORLD1_OK" in r.stdout
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    t = json.loads(line)["rccl_world1"]
    assert t["step_us_rccl"] > 0 and t["step_us_no_collective"] > 0
