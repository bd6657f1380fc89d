"""The SimCSE item-tower train step alone (bench.bench_simcse_train: two views, bert-base-shaped local BERT,
AdamW), for rocprofv3 --kernel-trace --stats. Prints the bench line's JSON.

  python tools/simcse_micro.py --batch 192 --iters 3
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
    ap.add_argument("--batch", type=int, default=192)
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()
    print(json.dumps(bench.bench_simcse_train(args, torch.device("cuda", 0), args.batch, args.iters)), flush=True)


if __name__ == "__main__":
    main()
