"""Micro-benchmark of rsx_retrieve_topk at configs[4]'s shape (Q = 4096 normalised queries,
1M-item normalised corpus, k = 100). Prints avg ms per call, the fallback flag and a checksum
of the indices. RSX_TOPK_BF16=0 selects the previous two-pass fp32 path (A/B).

  python tools/retrieval_micro.py --iters 10
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--q", type=int, default=4096)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--k", type=int, default=100)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--save", default=None, help="write indices to this .pt file")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    corpus = torch.nn.functional.normalize(torch.randn(args.items, 128, generator=g), dim=1).to(dev)
    users = torch.nn.functional.normalize(torch.randn(args.q, 128, generator=g), dim=1).to(dev)
    diag = {}
    s, i = ops.retrieve_topk(users, corpus, args.k, diag=diag)
    for _ in range(2):
        ops.retrieve_topk(users, corpus, args.k)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(args.iters):
        ops.retrieve_topk(users, corpus, args.k)
    b.record()
    torch.cuda.synchronize()
    ms = a.elapsed_time(b) / args.iters
    flops = 2.0 * args.q * args.items * 128
    if args.save:
        torch.save({"s": s.cpu(), "i": i.cpu()}, args.save)
    print(json.dumps({"path": "legacy-two-pass" if os.environ.get("RSX_TOPK_BF16") == "0" else "bf16-single-scan",
                      "avg_ms": round(ms, 4), "algorithmic_TFLOPs": round(flops / ms / 1e9, 2),
                      "fallback_queries": diag.get("fallback_queries"), "idx_checksum": int(i.sum().item()),
                      "score_sum": float(s.double().sum().item())}))


if __name__ == "__main__":
    main()
