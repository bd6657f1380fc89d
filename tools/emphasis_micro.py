"""full_batch_hard_emphasis_loss forward + backward at N rows (bench.bench_hard_emphasis's inputs), for
rocprofv3 --kernel-trace --stats. Prints the bench line's JSON.

  python tools/emphasis_micro.py --n 16384
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    print(json.dumps(bench.bench_hard_emphasis(args, torch.device("cuda", 0), args.n)), flush=True)


if __name__ == "__main__":
    main()
