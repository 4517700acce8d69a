"""bench.py's N-rank flow on one GPU (a rehearsal of the driver's `bench.py --gpus N` on an 8-GPU node):
`python bench.py --gpus 2` starts two ranks itself; with KADGPU_BENCH_ONE_GPU=1 both use cuda:0 and gloo
(RCCL needs a GPU per rank). Both variants must complete: owner routing (weak scaling, 2 shards of the
100M-node table), the owner-routed serving step (targets to their owners and packed rows back through
all_to_all_single) and the north-star all-gather (the 100M-node table split in two, gathered rows and
parts, device merge), and rank 0 prints one line with n_gpus = 2."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_two_ranks_on_one_gpu():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env["KADGPU_BENCH_ONE_GPU"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
                        "--no-cpu", "--queries", str(1 << 18)], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    print(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0
    assert d["verified"]["rows"] == 2 * (1 << 16) and d["verified"]["mismatches"] == 0
    ag = d["allgather"]
    assert "error" not in ag, ag
    assert ag["n_gpus"] == 2 and ag["value"] > 0 and ag["gathered_bytes_per_step"] > 0
    assert ag["verified"]["rows"] > 0 and ag["verified"]["mismatches"] == 0
    ow = d["owner_routed"]  # the owner-routed serving step at N = 2 (all_to_alls through gloo here)
    assert "error" not in ow, ow
    assert ow["n_gpus"] == 2 and ow["queries_per_s"] > 0 and not ow["overflow"]
    assert ow["verified"]["rows"] > 0 and ow["verified"]["mismatches"] == 0
    # every rank's returned rows are checked by their owners, the ones answered by the other rank included
    assert ow["verified"]["rows"] == 2 * (1 << 16) and ow["verified"]["rows_answered_by_another_rank"] > 0
    assert ow["collective"] == "all_to_all_single (gloo)"  # the rehearsal: RCCL needs a GPU per rank
    pw = ow["pipelined"]  # the overlapped OwnerPipeline, same batches
    assert "error" not in pw and not pw["overflow"], pw
    assert pw["verified"]["rows"] == 2 * (1 << 16) and pw["verified"]["mismatches"] == 0
    ap = ag["pipelined"]  # the north-star step pipelined
    assert "error" not in ap and not ap["overflow"], ap
    assert ap["verified"]["rows"] > 0 and ap["verified"]["mismatches"] == 0
