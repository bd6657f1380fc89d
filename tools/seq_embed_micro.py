"""Micro-benchmark of rsx_seq_embed_bwd at the bench shape (packed T ~ 80k tokens, L = 50,
D = 128, tables: item 47063, time 10, four hashed 1001) with subsets of the gradients
requested, to attribute its time. Prints avg ms per variant."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device="cpu").manual_seed(0)
T, L, D = 80946, 50, 128
rows = [47063, 10, 1001, 1001, 1001, 1001]
ids = [torch.randint(0, r, (T,), generator=g).to(dev) for r in rows]
tok_pos = torch.randint(0, L, (T,), generator=g).to(dev)
base0 = torch.randn(T, D, generator=g).to(dev)
tabs0 = [torch.randn(r, D, generator=g).to(dev) * 0.1 for r in rows]
gate0 = torch.rand(6, generator=g).to(dev)
pos0 = torch.randn(L, D, generator=g).to(dev)
lnw0, lnb0 = torch.ones(D, device=dev), torch.zeros(D, device=dev)
gy = torch.randn(T, D, generator=g).to(dev)


def run(variant, iters=10):
    base = base0.clone().requires_grad_("base" in variant)
    tabs = [t.clone().requires_grad_("tabs" in variant) for t in tabs0]
    gate = gate0.clone().requires_grad_("gate" in variant)
    pos = pos0.clone().requires_grad_("pos" in variant)
    lnw = lnw0.clone().requires_grad_("ln" in variant)
    lnb = lnb0.clone().requires_grad_("ln" in variant)
    ins = [t for t in [base, gate, pos, lnw, lnb] + tabs if t.requires_grad]
    out = ops.seq_embed(base, ids, tabs, gate, pos, lnw, lnb, p_drop=0.2, padding_idx=[0] * 6, tok_pos=tok_pos)
    for _ in range(2):
        torch.autograd.grad(out, ins, gy, retain_graph=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.autograd.grad(out, ins, gy, retain_graph=True)
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / iters, 4)


res = {}
for v in [("base",), ("base", "ln"), ("base", "ln", "pos"), ("base", "ln", "gate"), ("base", "ln", "tabs"),
          ("base", "ln", "pos", "gate", "tabs")]:
    res["+".join(v)] = run(v)
print(json.dumps(res))
