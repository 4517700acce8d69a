"""bench.py's configs object alone (BASELINE configs 1, 2, 4, 5 beside the headline). Usage: python tools/configs_only.py"""
import json, sys, torch
sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import bench
print(json.dumps(bench.configs_pass(torch.device("cuda", 0))))
