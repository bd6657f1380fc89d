"""Lists the host-synchronising calls of one training step (torch sync debug mode) and times
the host side of a step: python tools/sync_probe.py"""
import os
import sys
import time
import traceback
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import dist as D  # noqa: E402
from recsys_amd import synth  # noqa: E402
from recsys_amd.tower_code import v1_usertower_train as TT  # noqa: E402
from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    hs = synth.HASH_SIZE
    cfg = TT.PipelineConfig(num_items=47062, num_prod_types=hs, num_colors=hs, num_graphics=hs, num_sections=hs,
                            dropout=0.2)
    items = synth.make_items(num_items=47062, d=128, seed=0)
    torch.manual_seed(0)
    model = SASRecUserTower(cfg).to(dev)
    model.train()
    it = TT.SASRecItemTower(47062, 128, items.log_q.clone()).to(dev)
    it.init_from_pretrained(items.pretrained.to(dev))
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay, fused=True)
    opt.add_param_group({"params": list(it.parameters()), "lr": cfg.lr * 0.05})
    bucket = D.GradBucket(list(model.parameters()) + list(it.parameters()))
    g = synth.make_batch(items, 4096, seed=100)
    batch = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in g.items()}
    lookup = items.pretrained.to(dev)
    state = {"ix": None}

    def step():
        ix = state["ix"] or D.prepare_step_index(batch, pretrained_lookup=lookup)
        out = D.contrastive_step_dp(model, it, it.log_q, batch, opt, cfg, lookup, bucket, index=ix)
        state["ix"] = D.prepare_step_index_async(batch, pretrained_lookup=lookup)
        return out
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    sites = {}
    def hook(message, category, filename, lineno, file=None, line=None):
        st = traceback.extract_stack()[:-1]
        frames = [f for f in st if "recsys_amd" in f.filename or "content-based" in f.filename]
        key = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in frames[-3:])
        sites[key] = sites.get(key, 0) + 1
    warnings.showwarning = hook
    ix = state["ix"]
    torch.cuda.set_sync_debug_mode("warn")
    D.contrastive_step_dp(model, it, it.log_q, batch, opt, cfg, lookup, bucket, index=ix)  # main-stream syncs only
    torch.cuda.set_sync_debug_mode(0)
    state["ix"] = None
    torch.cuda.synchronize()
    for k, v in sorted(sites.items(), key=lambda x: -x[1]):
        print(v, k)
    # host time per step when the GPU never waits for it (10 steps queued, then one sync)
    t0 = time.perf_counter()
    for _ in range(10):
        step()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print("host issue ms/step %.3f   wall ms/step %.3f" % ((t1 - t0) * 100, (t2 - t0) * 100))


if __name__ == "__main__":
    main()
