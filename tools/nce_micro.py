"""Micro-benchmark of the grouped LogQ-loss kernels at the bench workload's shape.

Builds one global batch exactly as bench.py does (4096 users, H&M-shaped lengths, Zipf(1.0)
targets), with random L2-normalised step embeddings in place of the tower output, and runs
the grouped fwd + both backward passes. Prints per-kernel average ms. Meant to be run under
rocprofv3 (kernel trace / PMC passes) so a profile isolates these kernels.

  python tools/nce_micro.py --iters 20 --precision bf16x3
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--precision", default="bf16x3", choices=["bf16x3", "fp32", "f16"])
    ap.add_argument("--compare", action="store_true",
                    help="also report the loss / gradient deviation from the fp32 mode on the same inputs")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--global-batch", type=int, default=0,
                    help="emulate one rank of a DP run: rows of the first --batch users, columns = the "
                         "distinct targets of a global batch of this many users")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    items = synth.make_items(seed=args.seed)
    gb = max(args.global_batch, args.batch)
    b = synth.make_batch(items, gb, seed=args.seed + 100)
    valid = ~b["padding_mask"]
    t_all = b["target_ids"][valid].to(dev)
    valid = valid[:args.batch]
    t = b["target_ids"][:args.batch][valid].to(dev)
    users = torch.arange(args.batch).unsqueeze(1).expand_as(valid)[valid].to(dev)
    n = t.numel()
    g = torch.Generator(device="cpu").manual_seed(args.seed)
    U = F.normalize(torch.randn(n, 128, generator=g), dim=1).to(dev).requires_grad_()
    W = items.pretrained.to(dev)
    grp = ops.TargetGroups(t, users, t_cols=t_all) if gb > args.batch else ops.TargetGroups(t, users)
    B = W[grp.uniq].contiguous().requires_grad_()
    bias = items.log_q.to(dev)[grp.uniq].contiguous()
    for i in range(3):
        s, c = ops.nce_grouped_sum(U, B, bias, grp, tau=0.1, tag="micro", precision=args.precision)
        s.backward()
    torch.cuda.synchronize()
    import ctypes
    from recsys_amd import _native as N
    U.grad = None
    B.grad = None
    ops.timing_start()
    N.lib().rsx_kernel_events(1)
    for i in range(args.iters):
        s, c = ops.nce_grouped_sum(U, B, bias, grp, tau=0.1, tag="micro", precision=args.precision)
        s.backward()
    torch.cuda.synchronize()
    kt = ops.timing_stop()
    kev = (ctypes.c_float * 256)()
    nk = N.lib().rsx_kernel_events_read(kev, 256)
    N.lib().rsx_kernel_events(0)
    kms = [float(kev[i]) for i in range(max(nk, 0))]
    flops = 4.0 * n * int(grp.uniq.numel()) * 128
    out = {"rows": n, "distinct_targets": int(grp.uniq.numel()), "precision": args.precision,
           "env_fwdg": os.environ.get("RSX_NCE_FWDG", ""), "loss_sum": float(s.item()),
           "grad_u_abs_sum": float(U.grad.abs().sum().item()) / args.iters,
           "grad_b_abs_sum": float(B.grad.abs().sum().item()) / args.iters,
           "fwd_kernel_ms": round(sum(kms) / len(kms), 4) if kms else None,
           "fwd_kernel_frac_bf16x3": (round(flops / (sum(kms) / len(kms) / 1e3) / 838.9e12, 4) if kms else None),
           "avg_ms": {k: round(ms / max(cnt, 1), 4) for k, (cnt, ms) in sorted(kt.items())}}
    if args.compare:
        def run(prec):
            U.grad = None
            B.grad = None
            s1, _ = ops.nce_grouped_sum(U, B, bias, grp, tau=0.1, tag="cmp", precision=prec)
            s1.backward()
            return float(s1.item()), U.grad.detach().clone(), B.grad.detach().clone()
        l0, gu0, gb0 = run("fp32")
        l1, gu1, gb1 = run(args.precision)
        out["vs_fp32"] = {"loss_rel": abs(l1 - l0) / abs(l0),
                          "grad_u_max_err_over_scale": float((gu1 - gu0).abs().max() / gu0.abs().max()),
                          "grad_b_max_err_over_scale": float((gb1 - gb0).abs().max() / gb0.abs().max()),
                          "grad_u_rel_fro": float((gu1 - gu0).norm() / gu0.norm()),
                          "grad_b_rel_fro": float((gb1 - gb0).norm() / gb0.norm())}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
