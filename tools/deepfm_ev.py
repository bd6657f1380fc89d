"""Kernel-only timing of the fused DeepFM forward at configs[2] (65,536 rows x 39 fields, vocab
1e6): the C-ABI entry point called directly (weight images and packed tables prepared once),
50 launches between HIP events on the launching stream. --zero: every id 0 (L2-resident lines,
the non-gather cost); --uniform: uniform ids; default Zipf(1.1)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import _native as N  # noqa: E402
from recsys_amd import ops  # noqa: E402
from recsys_amd.temp_model.ranker_skelet import DeepFM  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--vocab", type=int, default=1_000_000)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--uniform", action="store_true")
    ap.add_argument("--zero", action="store_true")
    ap.add_argument("--abl", default="0", help="comma list of RSX_DEEPFM_ABL values to time in turn")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    F = 39
    model = DeepFM([a.vocab] * F, device=dev)
    rng = np.random.default_rng(3)
    if a.zero:
        x = torch.zeros(a.rows, F, dtype=torch.int64, device=dev)
    elif a.uniform:
        x = torch.from_numpy(rng.integers(0, a.vocab, (a.rows, F))).to(dev)
    else:
        x = torch.from_numpy(((rng.zipf(1.1, size=(a.rows, F)) - 1) % a.vocab).astype(np.int64)).to(dev)
    model.forward_logits(x)  # builds the weight images / packed tables in the module's cache
    st = model._fused_cache["fused_state"]  # device state kept by ops.deepfm_forward
    logit = torch.empty(a.rows, device=dev)
    prob = torch.empty(a.rows, device=dev)
    args = (N.ptr(x), a.rows, F, st["V"], st["W"], st["P"], float(model.out.bias.item()), st["b1"], st["b2"],
            st["wo"], st["ws"], N.ptr(logit), N.ptr(prob), N.stream())
    ids = "zero" if a.zero else ("uniform" if a.uniform else "zipf1.1")
    for abl in a.abl.split(","):
        os.environ["RSX_DEEPFM_ABL"] = abl
        for _ in range(5):
            N.check(N.lib().rsx_deepfm_fused_run(*args), "run")
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            N.lib().rsx_deepfm_fused_run(*args)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.iters
        print(json.dumps({"ids": ids, "abl": abl, "ms": round(ms, 4), "rows_per_s": round(a.rows / ms * 1e3)}),
              flush=True)
    os.environ.pop("RSX_DEEPFM_ABL", None)


if __name__ == "__main__":
    main()
