"""Which framework (aten) ops run inside one training step, with their Python call sites: the
fills, copies and small elementwise kernels around the HIP ops. Usage: python tools/glue_trace.py"""
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import recsys_amd  # noqa: E402,F401
from recsys_amd import dist as D  # noqa: E402
from recsys_amd import synth  # noqa: E402
from recsys_amd.tower_code import v1_usertower_train as TT  # noqa: E402
from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower  # noqa: E402

QUIET = ("aten.empty", "aten.empty_like", "aten.empty_strided", "aten.view", "aten._unsafe_view", "aten.t.",
         "aten.detach", "aten.alias", "aten.as_strided", "aten.slice", "aten.select", "aten.expand",
         "aten.unsqueeze", "aten.squeeze", "aten.permute", "aten.transpose", "aten.split", "aten.unbind",
         "aten.reshape", "aten._reshape_alias", "aten.lift_fresh", "aten.is_same_size", "aten.new_empty",
         "aten.set_", "aten._local_scalar_dense")


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        if not name.startswith(QUIET):
            shapes = tuple(tuple(a.shape) for a in args if torch.is_tensor(a))[:3]
            fr = [f for f in traceback.extract_stack()[:-1] if "recsys_amd" in f.filename or "llm-driven" in f.filename]
            site = " < ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in fr[-3:][::-1])
            self.rows[(name, shapes, site)] += 1
        return func(*args, **(kwargs or {}))


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
    batch = {k: (v.to(dev) if torch.is_tensor(v) else v)
             for k, v in synth.make_batch(items, int(os.environ.get("BATCH", "8192")), seed=100).items()}
    ix = D.prepare_step_index(batch, pretrained_lookup=lookup)
    for _ in range(2):
        D.contrastive_step_dp(model, it, it.log_q, batch, opt, cfg, lookup, bucket, index=ix)
    torch.cuda.synchronize()
    log = Log()
    with log:
        D.contrastive_step_dp(model, it, it.log_q, batch, opt, cfg, lookup, bucket, index=ix)
    torch.cuda.synchronize()
    for (name, shapes, site), n in sorted(log.rows.items(), key=lambda kv: kv[0][0]):
        print(f"{n:3d}  {name:40s} {str(shapes)[:60]:60s} {site}")


if __name__ == "__main__":
    main()
