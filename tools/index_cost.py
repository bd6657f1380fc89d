"""Experiment (not a bench line): what the per-step index build costs the headline step.

Runs bench.train_bench at the headline batch twice in one process: (a) as bench.py does (the
next batch's StepIndex built every step), (b) with dist.prepare_step_index memoised per batch
(the two alternating batches' indexes built once, outside the timed steps) -- the step with
zero index cost, i.e. the ceiling of any faster index build. Prints one JSON line."""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--inline", action="store_true", help="no prefetch thread (index built inline)")
    a = ap.parse_args()
    sys.argv = ["bench.py", "--steps", str(a.steps)] + (["--no-prefetch-index"] if a.inline else [])
    import bench
    args = bench.parse()
    args.batch = a.batch
    import recsys_amd  # noqa: F401
    from recsys_amd import dist as D
    from recsys_amd import ops, synth
    from recsys_amd.tower_code import v1_usertower_train as TT
    from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
    device = torch.device("cuda", 0)
    torch.cuda.set_device(device)
    hs = synth.HASH_SIZE
    cfg = TT.PipelineConfig(num_items=args.items, num_prod_types=hs, num_colors=hs, num_graphics=hs,
                            num_sections=hs, dropout=args.dropout)
    items = synth.make_items(num_items=args.items, d=cfg.d_model, seed=args.seed)
    torch.manual_seed(args.seed)
    model = SASRecUserTower(cfg).to(device).train()
    it = TT.SASRecItemTower(args.items, cfg.d_model, items.log_q.clone()).to(device)
    it.init_from_pretrained(items.pretrained.to(device))
    it.set_freeze_state(False)
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay, fused=True)
    opt.add_param_group({"params": list(it.parameters()), "lr": cfg.lr * 0.05})
    bucket = D.GradBucket(list(model.parameters()) + list(it.parameters()))
    out = {}
    tb = bench.train_bench(args, args.batch, args.steps, 3, items, cfg, model, it, opt, bucket, 0, 1, device)
    out["built_every_step_ms"] = round(1e3 * tb["elapsed"] / args.steps, 3)
    out["built_every_step_host_enqueue_ms"] = tb["host_enqueue_ms"]
    real = D.prepare_step_index
    memo = {}

    def cached(batch, pretrained_vecs=None, pretrained_lookup=None):
        k = id(batch["item_ids"])
        if k not in memo:
            memo[k] = real(batch, pretrained_vecs, pretrained_lookup)
        ix = memo[k]
        ix.ready = None
        return ix

    D.prepare_step_index = cached
    tb = bench.train_bench(args, args.batch, args.steps, 3, items, cfg, model, it, opt, bucket, 0, 1, device)
    out["memoised_ms"] = round(1e3 * tb["elapsed"] / args.steps, 3)
    out["memoised_host_enqueue_ms"] = tb["host_enqueue_ms"]
    out["batch"], out["inline"] = args.batch, a.inline
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
