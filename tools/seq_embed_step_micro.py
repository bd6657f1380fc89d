"""Seq-embed forward / backward at the bench step's shape: both dropout views packed into one
call (T ~ 316k tokens of 8192 users, positions consecutive per user segment), item table
47,064 rows (its gradient through the sorted segment sums, as the step does), time table 12
rows, the other four tables gated off (the reference's s_mask), LayerNorm, dropout 0.2.
Prints avg ms of the forward and of the backward (the rsx_seq_embed_bwd op window plus the
segment sums). RSX_SEQ_EMBED_BWD_ABL selects a timing ablation of the backward kernel.

  python tools/seq_embed_step_micro.py --iters 20
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
    ap.add_argument("--users", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    L, D = 50, 128
    # per-user token counts ~ the synthetic H&M length distribution (mean ~19.3 incl. the extra row)
    cnt = torch.clamp((torch.distributions.Exponential(1 / 18.0).sample((args.users,)) + 1).long(), 1, L)
    cnt = torch.cat([cnt, cnt])  # two views
    T = int(cnt.sum())
    tok_pos = torch.cat([torch.arange(L - int(c), L) for c in cnt]).to(dev)
    rows = [47064, 12, 1001, 1001, 1001, 1001]
    zipf = torch.distributions.Categorical(probs=1.0 / torch.arange(1, rows[0], dtype=torch.float64))
    ids = [(zipf.sample((T,)) + 1)] + [torch.randint(0, r, (T,), generator=g) for r in rows[1:]]
    ids = [t.to(dev) for t in ids]
    base = torch.randn(T, D, generator=g).to(dev).requires_grad_(True)
    tabs = [(torch.randn(r, D, generator=g) * 0.02).to(dev).requires_grad_(True) for r in rows]
    gate_p = torch.zeros(6, device=dev, requires_grad=True)
    mask = torch.tensor([1.0, 1.0, 0, 0, 0, 0], device=dev)
    pos = torch.randn(L, D, generator=g).to(dev).requires_grad_(True)
    lnw = torch.ones(D, device=dev, requires_grad=True)
    lnb = torch.zeros(D, device=dev, requires_grad=True)
    seg = ops.sort_segments(ids[0])
    gy = torch.randn(T, D, generator=g).to(dev)
    ins = [base, gate_p, pos, lnw, lnb] + tabs

    def fwd():
        gate = torch.sigmoid(gate_p) * mask
        return ops.seq_embed(base, ids, tabs, gate, pos, lnw, lnb, p_drop=0.2, padding_idx=[0] * 6,
                             tok_pos=tok_pos, tab0_seg=seg)

    out = fwd()
    for _ in range(3):
        torch.autograd.grad(out, ins, gy, retain_graph=True, allow_unused=True)
        fwd()
    torch.cuda.synchronize()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
    e[0].record()
    for _ in range(args.iters):
        fwd()
    e[1].record()
    for _ in range(args.iters):
        torch.autograd.grad(out, ins, gy, retain_graph=True, allow_unused=True)
    e[2].record()
    torch.cuda.synchronize()
    print(json.dumps({"T": T, "abl": os.environ.get("RSX_SEQ_EMBED_BWD_ABL", "0"),
                      "fwd_ms": round(e[0].elapsed_time(e[1]) / args.iters, 4),
                      "bwd_ms": round(e[1].elapsed_time(e[2]) / args.iters, 4)}))


if __name__ == "__main__":
    main()
