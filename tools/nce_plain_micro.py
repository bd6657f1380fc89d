"""Micro-benchmark of the plain bf16x3 InfoNCE passes at the DuoRec / SupCon shape of the bench
step (B = 8192 "last" vectors per view): ops.nce_sum forward + backward for flags NCE_PLAIN and
NCE_SUPCON. Prints avg ms per op (HIP events around each).

  python tools/nce_plain_micro.py [--b 8192]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--b", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(0)
    z1 = F.normalize(torch.randn(a.b, 128, generator=g), dim=1).to(dev).requires_grad_()
    z2 = F.normalize(torch.randn(a.b, 128, generator=g), dim=1).to(dev).requires_grad_()
    t = torch.randint(0, 2000, (a.b,), generator=g).to(dev)
    keys = t.to(torch.int32)

    def step():
        un, _ = ops.nce_sum(z1, z2, tau=0.1, flags=ops.NCE_PLAIN, tag="duorec")
        sup, _ = ops.nce_sum(z1, z1, None, keys, keys, tau=0.1, flags=ops.NCE_SUPCON, tag="supcon")
        (un + sup).backward()

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    ops.timing_start()
    for _ in range(a.iters):
        step()
    kt = ops.timing_stop()
    print(json.dumps({k: round(ms / max(n, 1), 4) for k, (n, ms) in sorted(kt.items())}), flush=True)


if __name__ == "__main__":
    main()
