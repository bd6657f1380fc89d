"""torch.profiler view of the training step (op names + input shapes + CUDA time), to find
the small framework kernels around the HIP ops. Usage: python tools/torch_prof_step.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import dist as D  # noqa: E402
from recsys_amd import synth  # noqa: E402
from recsys_amd.tower_code import v1_usertower_train as TT  # noqa: E402
from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    hs = synth.HASH_SIZE
    cfg = TT.PipelineConfig(num_items=47062, num_prod_types=hs, num_colors=hs, num_graphics=hs, num_sections=hs,
                            dropout=0.2)
    items = synth.make_items(num_items=47062, d=128, seed=0)
    torch.manual_seed(0)
    model = SASRecUserTower(cfg).to(dev).train()
    it = TT.SASRecItemTower(47062, 128, items.log_q.clone()).to(dev)
    it.init_from_pretrained(items.pretrained.to(dev))
    it.set_freeze_state(False)
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay, fused=True)
    opt.add_param_group({"params": list(it.parameters()), "lr": cfg.lr * 0.05})
    bucket = D.GradBucket(list(model.parameters()) + list(it.parameters()))
    lookup = items.pretrained.to(dev)
    batch = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in synth.make_batch(items, int(os.environ.get("BATCH", "8192")), seed=100).items()}
    ix = D.prepare_step_index(batch, pretrained_lookup=lookup)
    for _ in range(3):
        D.contrastive_step_dp(model, it, it.log_q, batch, opt, cfg, lookup, bucket, index=ix)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        for _ in range(3):
            D.contrastive_step_dp(model, it, it.log_q, batch, opt, cfg, lookup, bucket, index=ix)
        torch.cuda.synchronize()
    print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=60,
                                                               max_name_column_width=60, max_shapes_column_width=70))
    # the framework ops with the largest device time, with their python call sites (one step)
    evs = [e for e in prof.events() if e.name in ("aten::zeros", "aten::zero_", "aten::add_", "aten::add", "aten::copy_",
                                                 "aten::clone", "aten::contiguous", "aten::mm", "aten::cat",
                                                 "aten::addmm", "aten::mul", "aten::fill_")]
    evs.sort(key=lambda e: -e.device_time_total)
    seen = set()
    for e in evs:
        st = tuple(f for f in e.stack if "recsys_amd" in f or "llm-driven" in f or "tools/" in f)[:4]
        key = (e.name, st)
        if key in seen or e.device_time_total < 8:
            continue
        seen.add(key)
        print(f"EV {e.device_time_total:8.1f} us  {e.name}  shapes={e.input_shapes}")
        for fr in st:
            print("        ", fr)
    # the small framework ops (fills, copies, cats, index) with their python call sites
    ka = prof.key_averages(group_by_stack_n=6)
    small = [e for e in ka if any(k in e.key for k in ("fill_", "zero_", "copy_", "cat", "index", "zeros", "empty", "add", "mm",
                                                       "layer_norm", "gelu", "linear", "clone", "contiguous"))]
    small.sort(key=lambda e: -e.device_time_total)
    for e in small[:40]:
        print(f"{e.device_time_total / 3:9.1f} us/step  n={e.count // 3:4d}  {e.key}")
        for fr in e.stack[:6]:
            print("        ", fr)


if __name__ == "__main__":
    main()
