"""Micro-benchmark of the LayerNorm kernels at the training step's token count (both views at
batch 8192: 316k packed rows of 128): plain LN, residual-add + dropout + LN (the encoder's fused
form), LN + GELU. Prints avg ms and the effective HBM rate of each.

  python tools/ln_micro.py [--tokens 316416]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402


def bench(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=316416)
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    T, D = a.tokens, 128
    x = torch.randn(T, D, device=dev)
    r = torch.randn(T, D, device=dev)
    w = torch.randn(D, device=dev)
    b = torch.randn(D, device=dev)
    res = {}
    with torch.no_grad():
        ms = bench(lambda: ops.layer_norm(x, w, b), a.iters)
        res["ln"] = {"ms": round(ms, 4), "GB/s": round(2 * T * D * 4 / ms / 1e6, 1)}
        ms = bench(lambda: ops.layer_norm(x, w, b, act=2), a.iters)
        res["ln_gelu"] = {"ms": round(ms, 4), "GB/s": round(2 * T * D * 4 / ms / 1e6, 1)}
        ms = bench(lambda: ops.add_layer_norm(x, r, w, b, p_drop=0.2), a.iters)
        res["add_drop_ln"] = {"ms": round(ms, 4), "GB/s": round(4 * T * D * 4 / ms / 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
