"""Out-projection + residual add + LayerNorm: rsx_gemm_x3_addln (one kernel) against
linear_tok + add_layer_norm (two), forward and forward + backward, at the headline's token
count (317.5k packed tokens, D = 128, dropout 0.2). Usage: python tools/addln_micro.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n


def main():
    dev = torch.device("cuda", 0)
    T = int(os.environ.get("T", "317506"))
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(T, 128, device=dev, generator=g)
    a = torch.randn(T, 128, device=dev, generator=g)
    W = torch.randn(128, 128, device=dev, generator=g) * 0.09
    bW = torch.zeros(128, device=dev)
    w = torch.ones(128, device=dev)
    b = torch.zeros(128, device=dev)
    gs = torch.randn(T, 128, device=dev, generator=g)
    gy = torch.randn(T, 128, device=dev, generator=g)
    out = {"T": T}
    for name, fused in (("fused", True), ("unfused", False)):
        def fwd():
            if fused:
                return ops._LinearAddLayerNorm.apply(x, a, W, bW, w, b, 1e-5, 0.2, 7)
            return ops._AddLayerNorm.apply(x, ops.linear_tok(a, W, bW), w, b, 1e-5, 0.2, 7)

        xx, aa, WW = (t.clone().requires_grad_() for t in (x, a, W))

        def fwdbwd():
            if fused:
                s, y = ops._LinearAddLayerNorm.apply(xx, aa, WW, bW, w, b, 1e-5, 0.2, 7)
            else:
                s, y = ops._AddLayerNorm.apply(xx, ops.linear_tok(aa, WW, bW), w, b, 1e-5, 0.2, 7)
            torch.autograd.backward([s, y], [gs, gy])

        with torch.no_grad():
            out[name + "_fwd_ms"] = round(timeit(fwd), 4)
        out[name + "_fwd_bwd_ms"] = round(timeit(fwdbwd), 4)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
