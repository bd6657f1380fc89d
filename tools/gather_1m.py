"""The embedding gather on DRAM-resident rows (bench.py bench_gather_1m) alone, for rocprofv3
(--kernel-trace --stats, or --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes).
  python tools/gather_1m.py [--iters N]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import recsys_amd  # noqa: E402,F401

ap = argparse.ArgumentParser()
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--rows", type=int, default=1_000_000)
args = ap.parse_args()
torch.cuda.set_device(0)
print(json.dumps(bench.bench_gather_1m(torch.device("cuda", 0), rows=args.rows, iters=args.iters)))
