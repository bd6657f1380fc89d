"""PMC target: the weight-stationary token GEMM (rsx_gemm_x3, K = N = 128) over the headline's
317.5k packed tokens, 5 launches. Usage: rocprofv3 --pmc <counters> -- python tools/gemm_ws_pmc.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
T = int(os.environ.get("T", "317506"))
x = torch.randn(T, 128, device=dev)
w = torch.randn(128, 128, device=dev) * 0.09
b = torch.zeros(128, device=dev)
for _ in range(5):
    y = ops.gemm_x3(x, w, b)
torch.cuda.synchronize()
print("ok", float(y[0, 0]))
