"""Generates the committed golden fixtures under tests/golden/ (run from the repo root:
``python tests/golden/make_goldens.py``). Deterministic: fixed seeds, fp32 CPU.

Provenance. The reference ships no tests, fixtures or golden vectors for this path, and
importing its modules was denied by the environment during the survey, so
the expected values here come from the CPU restatement in oracle/ (itself written from the
reference source, file:line cited there). They pin two things: (1) the oracle against future
edits (CPU tests recompute every expected tensor from the stored inputs), and (2) the HIP path
against stored data rather than a live oracle run (GPU tests). Parity with the reference
itself stays UNPINNED.

Each fixture is one safetensors file (tensors only: inputs, weights, expected outputs) plus a
JSON sidecar with the scalar configuration.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F
from safetensors.torch import save_file

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

import recsys_amd  # noqa: E402,F401
from recsys_amd import synth  # noqa: E402
from recsys_amd.tower_code.v1_usertower_train import PipelineConfig  # noqa: E402
from oracle import deepfm as OD  # noqa: E402
from oracle import retrieval as OR  # noqa: E402
from oracle import user_tower as O  # noqa: E402

# the gradients pinned by the tower fixture (a cross-section of every stage of the tower)
TOWER_GRADS = ("item_proj.weight", "item_id_emb.weight", "time_emb.weight", "pos_emb.weight", "seq_gate",
               "static_gate", "emb_ln.weight", "transformer_encoder.layers.0.self_attn.in_proj_weight",
               "transformer_encoder.layers.0.self_attn.out_proj.bias", "transformer_encoder.layers.1.linear1.weight",
               "transformer_encoder.layers.1.norm2.bias", "age_emb.weight", "cont_proj.weight",
               "static_mlp.0.weight", "output_proj.0.weight", "output_proj.3.weight")


def _save(name, tensors, meta):
    tensors = {k: v.detach().contiguous().cpu() for k, v in tensors.items()}
    save_file(tensors, os.path.join(HERE, name + ".safetensors"))
    with open(os.path.join(HERE, name + ".json"), "w") as f:
        json.dump(meta, f, indent=1, sort_keys=True)
    print(f"{name}: {sum(v.numel() * v.element_size() for v in tensors.values()) / 1e6:.2f} MB")


def tower_cfg():
    return PipelineConfig(num_items=300, num_prod_types=50, num_colors=50, num_graphics=50, num_sections=50,
                          dropout=0.0)


def user_tower_fixture():
    """SASRecUserTower forward (train + eval mode) and the two-view contrastive losses with
    their gradients, B = 8 users, L = 50, d = 128, dropout 0 (v1_refine_usertower.py:417-510,
    v1_usertower_train.py:787-845). Includes users whose valid length is 1 (fully masked
    attention rows) and target collisions across users (same-item masking)."""
    cfg = tower_cfg()
    items = synth.make_items(num_items=300, d=128, seed=11)
    items.side = items.side % 51
    batch = synth.make_batch(items, 8, seed=12)
    # force the edge cases: a user with one valid step, two users sharing targets
    pm = batch["padding_mask"]
    pm[0] = True
    pm[0, -1] = False
    batch["target_ids"][2, -3:] = batch["target_ids"][1, -3:]
    batch["item_ids"][pm] = 0
    torch.manual_seed(13)
    model = O.OracleUserTower(cfg)
    model.train()
    W = torch.nn.Parameter(items.pretrained.clone())
    kw = synth.forward_kwargs(batch, items.pretrained[batch["item_ids"]], training_mode=True)
    with torch.no_grad():
        out_train = model(**kw)
        model.eval()
        kw["training_mode"] = False
        out_eval = model(**kw)
        model.train()
    total, main, cl = O.contrastive_losses(model, W, items.log_q, batch, items.pretrained)
    total.backward()
    t = {f"w.{k}": v for k, v in model.state_dict().items()}
    t.update({f"in.{k}": batch[k] for k in synth.FORWARD_KEYS})
    t["in.target_ids"] = batch["target_ids"]
    t["in.pretrained"] = items.pretrained
    t["in.log_q"] = items.log_q
    t["out.train"] = out_train
    t["out.eval"] = out_eval
    t["out.losses"] = torch.stack([total.detach(), main.detach(), cl.detach()])
    params = dict(model.named_parameters())
    for k in TOWER_GRADS:
        t[f"g.{k}"] = params[k].grad
    t["g.item_matrix"] = W.grad
    _save("user_tower_b8", t, {"num_items": 300, "hash_size": 50, "batch": 8, "max_len": 50, "d_model": 128,
                               "dropout": 0.0, "generator": "oracle/user_tower.py OracleUserTower, torch seed 13",
                               "grads": list(TOWER_GRADS)})


def logq_loss_fixture():
    """Live inbatch_corrected_logq_loss (v1_refine_usertower.py:826-861) on N = 257 rows with
    Zipf targets (many collisions), 17 users (same-user masking), a row with target 0
    (logQ[0] = -20) and its gradients w.r.t. the user rows and the normalised item table."""
    g = torch.Generator().manual_seed(21)
    I, N, d = 200, 257, 128
    raw = synth.zipf_probs(I, 1.0)
    log_q = synth.logq_from_probs(raw)
    rng = np.random.default_rng(22)
    tgt = torch.from_numpy(rng.choice(np.arange(1, I + 1), size=N, p=raw / raw.sum()).astype(np.int64))
    tgt[5] = 0
    users = torch.from_numpy(np.sort(rng.integers(0, 17, N)).astype(np.int64))
    U = torch.randn(N, d, generator=g)
    Wt = torch.randn(I + 1, d, generator=g)
    U.requires_grad_(True)
    Wt.requires_grad_(True)
    un = F.normalize(U, dim=1)
    wn = F.normalize(Wt, dim=1)
    loss = O.inbatch_corrected_logq_loss(un, wn, tgt, users, log_q, temperature=0.1, lambda_logq=1.0)
    loss.backward()
    _save("logq_loss_n257", {"in.user": U.detach(), "in.items": Wt.detach(), "in.target_ids": tgt,
                             "in.user_ids": users, "in.log_q": log_q, "out.loss": loss.detach().reshape(1),
                             "g.user": U.grad, "g.items": Wt.grad},
          {"temperature": 0.1, "lambda_logq": 1.0, "note": "loss(normalize(user), normalize(items)); grads "
                                                          "w.r.t. the un-normalised inputs"})


def duorec_fixture():
    """duorec_loss_refined (v1_refine_usertower.py:576-627): InfoNCE between views + 0.1 x
    SupCon on same-target rows; targets with duplicates and 0 (excluded from positives)."""
    g = torch.Generator().manual_seed(31)
    B, d = 96, 128
    z1 = torch.randn(B, d, generator=g).requires_grad_(True)
    z2 = torch.randn(B, d, generator=g).requires_grad_(True)
    tgt = torch.randint(0, 40, (B,), generator=g)
    tgt[:4] = 0
    loss = O.duorec_loss_refined(z1, z2, tgt, temperature=0.1, lambda_sup=0.1)
    loss.backward()
    _save("duorec_b96", {"in.z1": z1.detach(), "in.z2": z2.detach(), "in.target_ids": tgt,
                         "out.loss": loss.detach().reshape(1), "g.z1": z1.grad, "g.z2": z2.grad},
          {"temperature": 0.1, "lambda_sup": 0.1})


def simcse_fixture():
    """Item-tower SimCSE loss (item_tower.py:1072-1079), tau 0.08, both CE directions."""
    g = torch.Generator().manual_seed(41)
    e1 = F.normalize(torch.randn(64, 128, generator=g), dim=1).requires_grad_(True)
    e2 = F.normalize(torch.randn(64, 128, generator=g), dim=1).requires_grad_(True)
    loss = O.simcse_item_loss(e1, e2, 0.08)
    loss.backward()
    _save("simcse_b64", {"in.e1": e1.detach(), "in.e2": e2.detach(), "out.loss": loss.detach().reshape(1),
                         "g.e1": e1.grad, "g.e2": e2.grad}, {"temperature": 0.08})


def deepfm_fixture():
    """DeepFM forward (deepctr-torch 0.2.9 formulation; PARITY UNPINNED): 128 rows,
    39 fields, vocab 200 per field, d = 16, DNN (256, 128). Expected values in float64."""
    g = torch.Generator().manual_seed(51)
    R, Fn, V, E = 128, 39, 200, 16
    x = torch.randint(0, V, (R, Fn), generator=g)
    x[0] = 0
    x[1] = V - 1
    emb = [torch.randn(V, E, generator=g) * 0.1 for _ in range(Fn)]
    lin = [torch.randn(V, 1, generator=g) * 0.1 for _ in range(Fn)]
    dims = [Fn * E, 256, 128]
    ws = [torch.randn(dims[i + 1], dims[i], generator=g) / dims[i] ** 0.5 for i in range(2)]
    bs = [torch.randn(dims[i + 1], generator=g) * 0.01 for i in range(2)]
    wo = torch.randn(1, 128, generator=g) / 128 ** 0.5
    bias = 0.25
    logit, prob = OD.deepfm_forward(x, emb, lin, bias, ws, bs, wo)
    t = {"in.x": x, "w.dnn0": ws[0], "w.dnn1": ws[1], "b.dnn0": bs[0], "b.dnn1": bs[1], "w.out": wo,
         "out.logit": logit, "out.prob": prob}
    t["w.emb"] = torch.stack(emb)
    t["w.lin"] = torch.stack(lin)
    _save("deepfm_r128", t, {"rows": R, "fields": Fn, "vocab": V, "embed_dim": E, "dnn": [256, 128], "bias": bias})


def retrieval_fixture():
    """Exact top-k retrieval (v1_usertower_train.py:672-675; ranker_skelet.py:193-196) on
    dyadic inputs (every dot product exact in fp32), with planted exact ties resolved by
    (score desc, index asc)."""
    g = torch.Generator().manual_seed(61)
    Q, I, k = 24, 3000, 50
    qn = torch.randint(-8, 9, (Q, 128), generator=g).to(torch.int8)
    itn = torch.randint(-8, 9, (I, 128), generator=g).to(torch.int8)
    itn[1000] = itn[7]
    itn[2999] = itn[7]
    itn[1500:1510] = itn[3]
    sc, idx = OR.retrieve_topk(qn.float() / 8, itn.float() / 16, k)
    _save("retrieval_q24", {"in.queries_x8": qn, "in.items_x16": itn, "out.scores": sc, "out.index": idx},
          {"k": k, "tie_break": "score desc, index asc", "queries": "in.queries_x8 / 8",
           "items": "in.items_x16 / 16"})


def hnm_fixture():
    """Hard-negative mining (v1_refine_usertower.py:641-669, 705-728, 776-790) on integer inputs
    (every product exact in fp32): duplicated item rows give exact ties and item-similarity hits,
    repeated targets give same-item masks; expected (value desc, column asc) top-k and the
    available counts, plus the inbatch_hnm_corrected loss on the normalised rows."""
    g = torch.Generator().manual_seed(71)
    N, D, k, thr = 600, 128, 12, 30.0
    u = torch.randint(-2, 3, (N, D), generator=g).to(torch.int8)
    it = torch.randint(-2, 3, (N, D), generator=g).to(torch.int8)
    it[1::5] = it[0::5]
    tgt = torch.randint(1, 150, (N,), generator=g)
    idx, avail = O.hnm_mine(u.float(), it.float(), tgt, k, thr, 1.0)
    W = torch.randn(150, D, generator=g)
    lq = torch.log_softmax(torch.randn(150, generator=g), 0)
    U = torch.randn(N, D, generator=g)
    loss, st = O.inbatch_hnm_corrected_loss_with_stats(U, W, tgt, lq, top_k_percent=0.02)
    _save("hnm_n600", {"in.u": u, "in.items": it, "in.target_ids": tgt, "out.top_idx": idx, "out.avail": avail,
                       "in.user": U, "in.table": W, "in.log_q": lq, "out.loss": loss.detach().reshape(1)},
          {"k": k, "hnm_threshold": thr, "temperature_mining": 1.0, "order": "value desc, column asc",
           "loss_top_k_percent": 0.02, "num_active_hard_negs": st["num_active_hard_negs"]})


def main():
    torch.set_num_threads(1)
    user_tower_fixture()
    logq_loss_fixture()
    duorec_fixture()
    simcse_fixture()
    deepfm_fixture()
    retrieval_fixture()
    hnm_fixture()


if __name__ == "__main__":
    main()
