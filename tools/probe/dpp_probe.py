"""Run tools/probe/dpp_probe.hip (build: hipcc -O3 --offload-arch=gfx950 -shared -fPIC
tools/probe/dpp_probe.hip -o tools/probe/libdpp_probe.so) and print what each lane move delivers
and whether the DPP butterfly sum equals the shuffle butterfly bit for bit."""
import ctypes
import json
import os

import torch

lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libdpp_probe.so"))
dev = torch.device("cuda", 0)
n = 64
g = torch.Generator().manual_seed(0)
x = (torch.randn(n, 64, generator=g) * torch.logspace(-3, 3, n).unsqueeze(1)).float().to(dev)
moves = torch.zeros(8, 64, device=dev)
sums = torch.zeros(n, 6, 64, device=dev)
rc = lib.dpp_probe(ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(moves.data_ptr()), ctypes.c_void_p(sums.data_ptr()),
                   n, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
m = moves.cpu().int().tolist()
names = ["permlane16_swap[0]", "permlane16_swap[1]", "permlane32_swap[0]", "permlane32_swap[1]",
         "row_ror:8", "row_ror:4", "row_ror:2", "row_ror:1"]
s = sums.cpu()
res = {"rc": rc, "moves (source lane seen by lanes 0..63)": {k: v for k, v in zip(names, m)}}
for wi, w in enumerate((16, 32, 64)):
    a, b = s[:, 2 * wi], s[:, 2 * wi + 1]
    res[f"width {w}: sets with any lane differing"] = int((a != b).any(dim=1).sum())
    res[f"width {w}: max |diff| / |sum|"] = float(((a - b).abs() / a.abs().clamp(min=1e-30)).max())
print(json.dumps(res))
