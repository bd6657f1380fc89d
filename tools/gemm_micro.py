"""Micro-benchmark of rsx_gemm_x3 / rsx_linear_wgrad_x3 at the training step's token-linear
shapes (T = 160k tokens: both dropout views at batch 4096). Prints avg ms and the effective
HBM rate (compulsory bytes: A read once, C (+aux) written once) per shape.

  python tools/gemm_micro.py --iters 20
"""
from __future__ import annotations

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
    ap.add_argument("--tokens", type=int, default=158720)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    T = args.tokens
    g = torch.Generator(device="cpu").manual_seed(0)
    res = {}
    shapes = [("fwd_128x128", 128, 128, 0), ("fwd_384x128", 384, 128, 0), ("dx_128x384", 128, 384, 0),
              ("dx_128x256", 128, 256, 0), ("gelu_256x128", 256, 128, 1), ("dgelu_256x128", 256, 128, 2)]
    for name, n, k, epi in shapes:
        a = torch.randn(T, k, generator=g).to(dev)
        b = (torch.randn(n, k, generator=g) / k ** 0.5).to(dev)
        bias = torch.randn(n, generator=g).to(dev)
        aux = torch.rand(T, n, device=dev) if epi else None
        for _ in range(3):
            ops.gemm_x3(a, b, bias if epi != 2 else None, epi, aux, 0.1, 7)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            ops.gemm_x3(a, b, bias if epi != 2 else None, epi, aux, 0.1, 7)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        byts = T * k * 4 + T * n * 4 * (2 if epi else 1)
        res[name] = {"ms": round(ms, 4), "GB/s": round(byts / ms / 1e6, 1)}
    for name, n, k in [("wgrad_384x128", 384, 128), ("wgrad_128x128", 128, 128), ("wgrad_128x256", 128, 256)]:
        dy = torch.randn(T, n, generator=g).to(dev)
        x = torch.randn(T, k, generator=g).to(dev)
        for _ in range(3):
            ops.linear_wgrad(dy, x, (n, k), True)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            ops.linear_wgrad(dy, x, (n, k), True)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        res[name] = {"ms": round(ms, 4), "GB/s": round(T * (n + k) * 4 / ms / 1e6, 1)}
    # copy ceilings of the same byte mixes (torch's copy kernel): [T,128] -> [T,128] (1:1) and
    # [T,128] -> [T,384] (1:3, three strided copies into one output)
    x = torch.randn(T, 128, device=dev)
    y1 = torch.empty_like(x)
    y3 = torch.empty(T, 384, device=dev)
    for name, fn, byts in [("copy_1to1", lambda: y1.copy_(x), T * 128 * 8),
                           ("copy_1to3", lambda: [y3[:, 128 * i:128 * (i + 1)].copy_(x) for i in range(3)],
                            T * 128 * 4 * 6)]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        res[name] = {"ms": round(ms, 4), "GB/s": round(byts / ms / 1e6, 1)}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
