"""Micro-benchmark of the packed causal attention kernels at the bench shape (4096 users,
H&M-shaped lengths, H=4, Dh=32, dropout 0.2). Prints avg ms of fwd and bwd."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops, synth  # noqa: E402
from recsys_amd.tower_code.v1_refine_usertower import PackedTokens  # noqa: E402

dev = torch.device("cuda", 0)
items = synth.make_items(seed=0)
b = synth.make_batch(items, 4096, seed=100)
pk = PackedTokens(b["padding_mask"].to(dev))
T = pk.flat.numel()
g = torch.Generator(device="cpu").manual_seed(0)
qkv = torch.randn(T, 384, generator=g).to(dev).requires_grad_()
gy = torch.randn(T, 128, generator=g).to(dev)
res = {"tokens": T}
for name in ("fwd", "bwd"):
    for it in range(3):
        out = ops.mha(qkv, pk.tok_pad, 4, causal=True, p_drop=0.2, seg_off=pk.seg_off)
        if name == "bwd":
            torch.autograd.grad(out, qkv, gy)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for it in range(n):
        out = ops.mha(qkv, pk.tok_pad, 4, causal=True, p_drop=0.2, seg_off=pk.seg_off)
        if name == "bwd":
            torch.autograd.grad(out, qkv, gy)
    e1.record()
    torch.cuda.synchronize()
    res[name + "_total_ms"] = round(e0.elapsed_time(e1) / n, 4)
print(json.dumps(res))
