#!/usr/bin/env python3
"""bench.py's wal_payload_batches alone (not product code): python3 tools/wal_payload_probe.py"""
import sys, json
sys.path.insert(0, '.')
import torch
import bench
import tinykvpp_amd as tk
torch.cuda.set_device(0); tk.set_device(0)
ora = bench.load_oracle()
r = bench.wal_payload_batches(torch.device('cuda:0'), ora)
print(json.dumps({k: (v['GB_per_s'] if isinstance(v, dict) else v) for k, v in r.items()}))
