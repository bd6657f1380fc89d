"""Fused in_proj + attention forward (rsx_mha_qkv_fwd_x3) against linear_tok + mha at the bench
step's shape: both dropout views' packed tokens (T ~ 316k, 16,384 segments of 1..51 tokens),
D = 128, 4 heads, causal + key padding, dropout 0.2. Prints avg ms of each forward (HIP events)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    cnt = torch.clamp((torch.distributions.Exponential(1 / 18.0).sample((16384,)) + 1).long(), 1, 51)
    seg = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(cnt, 0)]).to(torch.int32).to(dev)
    T = int(cnt.sum())
    x = torch.randn(T, 128, generator=g).to(dev)
    w = (torch.randn(384, 128, generator=g) * 128 ** -0.5).to(dev)
    b = (torch.randn(384, generator=g) * 0.1).to(dev)
    pad = torch.zeros(T, dtype=torch.uint8, device=dev)

    def fused():
        return ops._QKVMHA.apply(x, w, b, pad, seg, 4, True, 0.2, 7)

    def twoop():
        return ops._MHA.apply(ops.linear_tok(x, w, b), pad, seg, 4, True, 0.2, 7)

    res = {"T": T}
    for name, fn in (("fused", fused), ("two_op", twoop)):
        with torch.no_grad():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(20):
                fn()
            e1.record()
            torch.cuda.synchronize()
        res[name + "_ms"] = round(e0.elapsed_time(e1) / 20, 4)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
