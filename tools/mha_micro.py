"""Micro-benchmark of the causal attention kernels at the bench shape (4096 users, H&M-shaped
lengths, H=4, Dh=32): packed with dropout 0.2 (the training step), packed without dropout,
and dense [T/50, 50] (no segment search). Prints avg ms of forward and forward+backward.

  python tools/mha_micro.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops, synth  # noqa: E402
from recsys_amd.tower_code.v1_refine_usertower import PackedTokens  # noqa: E402


def bench(fn, n=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / n, 4)


def main():
    dev = torch.device("cuda", 0)
    items = synth.make_items(seed=0)
    b = synth.make_batch(items, int(os.environ.get("BATCH", "8192")), seed=100)
    pk = PackedTokens(b["padding_mask"].to(dev))
    T = pk.flat.numel()
    g = torch.Generator(device="cpu").manual_seed(0)
    qkv = torch.randn(T, 384, generator=g).to(dev).requires_grad_()
    gy = torch.randn(T, 128, generator=g).to(dev)
    res = {"tokens": T}
    for p in (0.2, 0.0):
        f = lambda: ops.mha(qkv, pk.tok_pad, 4, causal=True, p_drop=p, seg_off=pk.seg_off)
        res[f"packed_p{p}_fwd_ms"] = bench(f)
        res[f"packed_p{p}_fwdbwd_ms"] = bench(lambda: torch.autograd.grad(f(), qkv, gy))
    Bd = T // 50
    qd = qkv.detach()[:Bd * 50].reshape(Bd, 50, 384).clone().requires_grad_()
    gd = gy[:Bd * 50].reshape(Bd, 50, 128)
    fd = lambda: ops.mha(qd, None, 4, causal=True, p_drop=0.2)
    res["dense_fwd_ms"] = bench(fd)
    res["dense_fwdbwd_ms"] = bench(lambda: torch.autograd.grad(fd(), qd, gd))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
