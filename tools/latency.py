"""bench.py's latency object alone: one Dht request's findClosestNodes through the boundary on a ~170-node
live-shaped table (launch path, resident query service, the CPU port). Usage: python tools/latency.py"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    print(json.dumps(bench.latency_pass(torch.device("cuda", 0))))
