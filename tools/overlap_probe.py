"""Probe: does the main loss's column backward (MFMA-bound, ~5 ms) overlap with HBM-bound token
GEMMs / the attention backward on a second stream? Times each alone and both concurrently.

  python tools/overlap_probe.py
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops, synth  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    items = synth.make_items(seed=0)
    b = synth.make_batch(items, 8192, seed=100)
    valid = ~b["padding_mask"]
    t = b["target_ids"][valid].to(dev)
    users = torch.arange(8192).unsqueeze(1).expand_as(valid)[valid].to(dev)
    n = t.numel()
    g = torch.Generator(device="cpu").manual_seed(0)
    U = F.normalize(torch.randn(n, 128, generator=g), dim=1).to(dev).requires_grad_()
    W = items.pretrained.to(dev)
    grp = ops.TargetGroups(t, users)
    B = W[grp.uniq].contiguous().requires_grad_()
    bias = items.log_q.to(dev)[grp.uniq].contiguous()
    T = 306000
    a = torch.randn(T, 128, device=dev)
    w = torch.randn(384, 128, device=dev) / 11.3
    bb = torch.randn(384, device=dev)

    def loss_bwd():
        s, c = ops.nce_grouped_sum(U, B, bias, grp, tau=0.1, tag="probe")
        s.backward()

    def gemms():
        for _ in range(25):
            ops.gemm_x3(a, w, bb)

    side = torch.cuda.Stream()
    res = {}
    for name, fn in [("loss_fwd_bwd", loss_bwd), ("gemms_x25", gemms)]:
        for _ in range(2):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) / 3, 3)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            gemms()
        loss_bwd()
        torch.cuda.current_stream().wait_stream(side)
    e1.record()
    torch.cuda.synchronize()
    res["concurrent"] = round(e0.elapsed_time(e1) / 3, 3)
    res["serial_sum"] = round(res["loss_fwd_bwd"] + res["gemms_x25"], 3)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
