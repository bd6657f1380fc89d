"""The user tower's native program alone (rsx_tower_fwd / rsx_tower_bwd, csrc/tower.hip) at the headline
batch: both dropout views of 8192 synthetic users, tail rows, dropout 0.2 -- the bench step's tower call
without the losses, the static profile or the optimizer. Each iteration is bracketed by marker kernels
(torch.cuda._sleep) so a rocprofv3 --pmc pass can attribute FETCH_SIZE / WRITE_SIZE to the forward and
the backward call (tools/tower_traffic.py). Prints the HIP-event time of each call.

  python tools/tower_micro.py --iters 6
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import dist as D  # noqa: E402
from recsys_amd import ops, synth  # noqa: E402
from recsys_amd.tower_code import v1_usertower_train as TT  # noqa: E402
from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--iters", type=int, default=6)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    hs = synth.HASH_SIZE
    cfg = TT.PipelineConfig(num_items=47_062, num_prod_types=hs, num_colors=hs, num_graphics=hs, num_sections=hs,
                            dropout=0.2)
    items = synth.make_items(num_items=47_062, d=128, seed=0)
    torch.manual_seed(0)
    model = SASRecUserTower(cfg).to(dev).train()
    batch = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in synth.make_batch(items, args.batch, seed=100).items()}
    ix = D.prepare_step_index(batch, pretrained_lookup=items.pretrained.to(dev))
    pk, pk2, tok_ids, pv, static = ix.packed
    p = model.dropout_rate
    with torch.no_grad():
        s_g = torch.sigmoid(model.seq_gate) * model._seq_gate_mask
        profile = model._static_profile(*static, p, pk2.B)
    profile = profile.detach().requires_grad_()
    params = ops.tower_native_ok(model, pk2, pv)
    assert params is not None, "native tower program not applicable"
    T = int(pv.shape[0])
    g = torch.Generator(device="cpu").manual_seed(3)
    w = None
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    fwd_ms, bwd_ms = [], []
    for it in range(args.iters + 2):
        torch.cuda._sleep(1000)  # marker: forward begins
        ev[0].record()
        out = ops.tower_packed(model, pk2, pv, tok_ids, s_g, profile, p, params, pk.last_tok)
        ev[1].record()
        torch.cuda._sleep(1000)  # marker: backward begins
        if w is None:
            w = torch.randn(out.shape, generator=g).to(dev)
        out.backward(w)
        ev[2].record()
        torch.cuda._sleep(1000)  # marker: iteration ends
        torch.cuda.synchronize()
        if it == args.iters + 1:  # last iteration: checksums of the output and every gradient (A/B builds
            # must agree bit for bit: same seeds, same per-element arithmetic)
            cks = {"out": float(out.detach().double().sum()), "out_abs": float(out.detach().double().abs().sum()),
                   "grads": float(sum(q.grad.double().abs().sum() for q in model.parameters() if q.grad is not None)),
                   "profile_grad": float(profile.grad.double().abs().sum())}
        model.zero_grad(set_to_none=True)
        profile.grad = None
        if it >= 2:
            fwd_ms.append(ev[0].elapsed_time(ev[1]))
            bwd_ms.append(ev[1].elapsed_time(ev[2]))
    print(json.dumps({"batch": args.batch, "packed_tokens_T": T, "tail_rows_R": int(out.shape[0]),
                      "tower_fwd_ms": round(sum(fwd_ms) / len(fwd_ms), 4),
                      "tower_bwd_ms_incl_autograd": round(sum(bwd_ms) / len(bwd_ms), 4), "checksums": cks}), flush=True)


if __name__ == "__main__":
    main()
