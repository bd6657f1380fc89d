"""Times rsx_hnm_mine against the reference's torch formulation of the same mining step
(v1_refine_usertower.py:641-669: two N x N GEMMs, three masks, masked_fill, topk) on the GPU."""
import json
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import recsys_amd  # noqa: F401,E402
from recsys_amd import ops  # noqa: E402


def torch_mine(u, it, t, k, thr, tau):
    cos = u @ it.T
    same = t.unsqueeze(1) == t.unsqueeze(0)
    diag = torch.eye(u.shape[0], dtype=torch.bool, device=u.device)
    ignore = same | ((it @ it.T > thr) & ~diag)
    m = (cos / tau).masked_fill(ignore, float("-inf"))
    return torch.topk(m, k, dim=1)[1], (~ignore).sum(1)


def bench(fn, it=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(it):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / it


out = []
for N in (1024, 4096, 16384):
    k = max(1, int((N - 1) * 0.01))
    g = torch.Generator().manual_seed(N)
    W = F.normalize(torch.randn(N // 2 + 1, 128, generator=g), dim=1).cuda()
    t = torch.randint(1, N // 2 + 1, (N,), generator=g).cuda()
    u = F.normalize(torch.randn(N, 128, generator=g), dim=1).cuda()
    it = W[t].contiguous()
    ms_k = bench(lambda: ops.hnm_mine(u, it, t, k, 0.9, 0.1))
    ms_t = bench(lambda: torch_mine(u, it, t, k, 0.9, 0.1))
    i1, _, a1 = ops.hnm_mine(u, it, t, k, 0.9, 0.1)
    i2, a2 = torch_mine(u, it, t, k, 0.9, 0.1)
    same = (i1.sort(1).values == i2.sort(1).values).all(1).float().mean().item()
    flops = 4.0 * N * N * 128
    out.append({"N": N, "k": k, "hnm_mine_ms": round(ms_k, 4), "torch_ms": round(ms_t, 4),
                "speedup": round(ms_t / ms_k, 2), "valu_tflops": round(flops / ms_k / 1e9, 1),
                "rows_same_set_as_torch": same, "avail_equal": bool(torch.equal(a1.long(), a2))})
    print(json.dumps(out[-1]), flush=True)
