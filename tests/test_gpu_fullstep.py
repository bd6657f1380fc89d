"""configs[1]'s WHOLE train step at its real size: global batch 4096 users of the
synthetic H&M-shaped data (N ~ 77k valid steps, D ~ 16k distinct targets, the 47,062-item table),
two views, the grouped LogQ loss + DuoRec, backward, clip_grad_norm_(5.0), AdamW with the item matrix
unfrozen (lr x 0.05), run as the headline runs it (dist.contrastive_step_dp: packed tower program,
grouped loss kernels, native clip + AdamW) against oracle/user_tower.py contrastive_step (the
restatement of tower_code/v1_usertower_train.py:717-893, fp32 PyTorch CPU, main loss row-chunked:
same per-element arithmetic) from the same state: the oracle's weights after a 64-user warm-up step,
its item matrix and its AdamW moments, dropout 0.

Criteria (oracle/agreement.py): total / main / cl within 1e-4; every parameter gradient (clipped)
within 1e-3 of its scale; post-AdamW parameters within 1e-5 wherever the gradient is resolved at that
tolerance. The CPU side takes ~35-60 s on 16 threads."""
import dataclasses

import pytest
import torch

import bench
import recsys_amd  # noqa: F401
from oracle import agreement as OA
from oracle import user_tower as O
from recsys_amd import synth
from recsys_amd.tower_code import v1_usertower_train as TT

pytestmark = pytest.mark.gpu


@pytest.mark.timeout(900)
def test_full_step_b4096_matches_oracle(gpu):
    items_n = 47_062
    hs = synth.HASH_SIZE
    cfg = TT.PipelineConfig(num_items=items_n, num_prod_types=hs, num_colors=hs, num_graphics=hs, num_sections=hs,
                            dropout=0.0)
    items = synth.make_items(num_items=items_n, d=cfg.d_model, seed=0)
    torch.manual_seed(0)
    model = O.OracleUserTower(cfg)
    model.train()
    W = torch.nn.Parameter(items.pretrained.clone())
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay)
    opt.add_param_group({"params": [W], "lr": cfg.lr * 0.05})
    O.contrastive_step(model, W, items.log_q, synth.make_batch(items, 64, seed=7), opt, items.pretrained,
                       loss_chunk=64)
    batch = synth.make_batch(items, 4096, seed=100)
    n_valid = int((~batch["padding_mask"]).sum())
    assert n_valid > 60_000
    state = bench.oracle_state(model, W, opt)
    losses = O.contrastive_step(model, W, items.log_q, batch, opt, items.pretrained, loss_chunk=256)
    ref = OA.capture(model, W, losses)
    dut = bench.gpu_step_from_state(state, dataclasses.replace(cfg), items, batch, gpu)
    agr = OA.compare_step(ref, dut)
    print("full-step agreement at B=4096:", agr)
    assert max(agr["loss_abs_err"]) <= OA.LOSS_TOL, agr
    assert agr["grad_max_err_over_scale"] <= OA.GRAD_TOL, agr
    assert agr["param_max_abs_err_resolved"] <= OA.PARAM_TOL, agr
    assert agr["params_over_1e-5"] == agr["params_over_1e-5_unresolved"], agr
    assert agr["ok"]
