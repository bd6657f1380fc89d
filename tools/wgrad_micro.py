"""Micro-benchmark: rsx_linear_wgrad vs the library GEMM (dY^T X) at the user tower's shapes.
  python tools/wgrad_micro.py  (run under rocprofv3 --kernel-trace --stats for per-kernel times)"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
T = int(os.environ.get("T", "317506"))  # packed tokens of the headline step (both views)
res = {}
for (n, k) in [(384, 128), (128, 128), (256, 128), (128, 256)]:
    dy = torch.randn(T, n, device=dev)
    x = torch.randn(T, k, device=dev)
    for name, fn in [("rsx", lambda: ops.linear_wgrad(dy, x, (n, k), True)),
                     ("blas", lambda: (dy.t() @ x, dy.sum(0)))]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 20
        res[f"{name}_{n}x{k}"] = {"ms": round(ms, 4), "TFLOPs": round(2 * T * n * k / ms / 1e9, 1)}
print(json.dumps(res))
