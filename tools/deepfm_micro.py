"""Micro-benchmark of the DeepFM forward (BASELINE configs[2]: 65,536 rows x 39 fields, d=16,
vocab 1e6/field, Zipf(1.1) ids). Prints per-call ms for the selected path
(RSX_DEEPFM_FUSED=0: gather + fp32-MFMA linears). Run under rocprofv3 for per-kernel times."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd.temp_model.ranker_skelet import DeepFM  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--uniform", action="store_true")
    ap.add_argument("--zero", action="store_true", help="every id 0 (L2-resident lines: the non-gather cost)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    model = DeepFM([a.vocab] * 39, device=dev)
    rng = np.random.default_rng(3)
    if a.zero:
        x = torch.zeros(a.rows, 39, dtype=torch.int64, device=dev)
    elif a.uniform:
        x = torch.from_numpy(rng.integers(0, a.vocab, (a.rows, 39))).to(dev)
    else:
        x = torch.from_numpy(((rng.zipf(1.1, size=(a.rows, 39)) - 1) % a.vocab).astype(np.int64)).to(dev)
    for _ in range(3):
        model.forward_logits(x)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.iters):
        model.forward_logits(x)
    torch.cuda.synchronize()
    print(f"deepfm rows {a.rows}: {(time.perf_counter() - t0) / a.iters * 1e3:.4f} ms/call", flush=True)


if __name__ == "__main__":
    main()
