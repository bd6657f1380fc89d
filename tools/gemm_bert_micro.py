"""rsx_gemm_x3 at the text BERT's token-GEMM shapes (M = 3,000 packed tokens, bert-base widths: QKV
2304 x 768, out-projection 768 x 768, FFN 3072 x 768 with the GELU epilogue and 768 x 3072), where the
output tiles number fewer than the CUs. Prints ms per call, TF/s (bf16x3 products counted once) and a
checksum per shape; RSX_GEMM_DEEP=0 / 1 selects the one-stage / four-stage prefetch (checksums equal).

  python tools/gemm_bert_micro.py --tokens 3000 --iters 20
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=3000)
    ap.add_argument("--iters", type=int, default=20)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    T = args.tokens
    g = torch.Generator(device="cpu").manual_seed(0)
    res = {"tokens": T, "deep": os.environ.get("RSX_GEMM_DEEP", "1")}
    shapes = [("qkv_2304x768", 2304, 768, 0), ("out_768x768", 768, 768, 0), ("ffn1_3072x768_gelu", 3072, 768, 1),
              ("ffn2_768x3072", 768, 3072, 0), ("dx_768x2304", 768, 2304, 0)]
    for name, n, k, epi in shapes:
        a = torch.randn(T, k, generator=g).to(dev)
        b = (torch.randn(n, k, generator=g) / k ** 0.5).to(dev)
        bias = torch.randn(n, generator=g).to(dev)
        aux = torch.rand(T, n, device=dev) if epi else None
        for _ in range(3):
            out = ops.gemm_x3(a, b, bias, epi, aux, 0.0, 7)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(args.iters):
            out = ops.gemm_x3(a, b, bias, epi, aux, 0.0, 7)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / args.iters
        res[name] = {"ms": round(ms, 4), "tflops": round(2.0 * T * n * k / ms / 1e9, 1),
                     "checksum": float(out.double().sum())}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
