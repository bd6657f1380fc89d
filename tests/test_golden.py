"""Golden fixtures (tests/golden/, made by tests/golden/make_goldens.py from the CPU oracle).

CPU tests: the oracle recomputes every stored expected tensor from the stored inputs (pins the
oracle against edits). GPU tests: the HIP path on the same stored inputs against the stored
expected tensors (the reference itself ships no fixtures: parity with it is unpinned, see
make_goldens.py). Tolerances are written per test."""
from __future__ import annotations

import json
import os

import pytest
import torch
import torch.nn.functional as F
from safetensors.torch import load_file

import recsys_amd  # noqa: F401
from recsys_amd.tower_code.v1_usertower_train import PipelineConfig
from oracle import deepfm as OD
from oracle import retrieval as OR
from oracle import user_tower as O

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FORWARD_KEYS = ("item_ids", "time_bucket_ids", "type_ids", "color_ids", "graphic_ids", "section_ids",
                "age_bucket", "price_bucket", "cnt_bucket", "recency_bucket", "channel_ids", "club_status_ids",
                "news_freq_ids", "fn_ids", "active_ids", "cont_feats", "padding_mask")


def load(name):
    t = load_file(os.path.join(GOLD, name + ".safetensors"))
    with open(os.path.join(GOLD, name + ".json")) as f:
        meta = json.load(f)
    return t, meta


def sub(t, prefix):
    return {k[len(prefix):]: v for k, v in t.items() if k.startswith(prefix)}


def tower_cfg(meta):
    h = meta["hash_size"]
    return PipelineConfig(num_items=meta["num_items"], num_prod_types=h, num_colors=h, num_graphics=h,
                          num_sections=h, dropout=meta["dropout"])


def tower_batch(t):
    b = sub(t, "in.")
    return {k: b[k] for k in FORWARD_KEYS + ("target_ids",)}


def deepfm_inputs(t):
    emb = list(t["w.emb"].unbind(0))
    lin = list(t["w.lin"].unbind(0))
    return emb, lin, [t["w.dnn0"], t["w.dnn1"]], [t["b.dnn0"], t["b.dnn1"]], t["w.out"]


def assert_grad_close(got, exp, rel, name):
    scale = exp.abs().max().item() + 1e-12
    err = (got.double() - exp.double()).abs().max().item()
    assert err <= rel * scale + 1e-7, f"{name}: max err {err:.3e} vs grad scale {scale:.3e}"


# ------------------------------------------------------------------ CPU: oracle vs fixtures
def test_golden_oracle_user_tower():
    t, meta = load("user_tower_b8")
    model = O.OracleUserTower(tower_cfg(meta))
    model.load_state_dict(sub(t, "w."))
    model.train()
    batch = tower_batch(t)
    pre = t["in.pretrained"]
    kw = {k: batch[k] for k in FORWARD_KEYS}
    kw["pretrained_vecs"] = pre[batch["item_ids"]]
    with torch.no_grad():
        torch.testing.assert_close(model(**kw, training_mode=True), t["out.train"], atol=1e-5, rtol=1e-5)
        model.eval()
        torch.testing.assert_close(model(**kw, training_mode=False), t["out.eval"], atol=1e-5, rtol=1e-5)
        model.train()
    W = torch.nn.Parameter(pre.clone())
    total, main, cl = O.contrastive_losses(model, W, t["in.log_q"], batch, pre)
    torch.testing.assert_close(torch.stack([total, main, cl]).detach(), t["out.losses"], atol=1e-5, rtol=1e-6)
    total.backward()
    params = dict(model.named_parameters())
    for k in meta["grads"]:
        assert_grad_close(params[k].grad, t["g." + k], 1e-5, k)
    assert_grad_close(W.grad, t["g.item_matrix"], 1e-5, "item_matrix")


def test_golden_fixture_edge_cases_present():
    """The tower fixture carries the Appendix-B traps it is meant to pin."""
    t, _ = load("user_tower_b8")
    pm = t["in.padding_mask"]
    assert int((~pm[0]).sum()) == 1                      # one valid step: fully masked attention rows
    assert torch.equal(t["in.target_ids"][2, -3:], t["in.target_ids"][1, -3:])  # cross-user collisions
    assert t["w.item_id_emb.weight"][0].abs().sum() > 0  # padding row non-zero after _init_weights
    lq, _ = load("logq_loss_n257")
    assert lq["in.target_ids"][5] == 0 and lq["in.log_q"][0] == -20.0
    r, _ = load("retrieval_q24")
    assert torch.equal(r["in.items_x16"][1000], r["in.items_x16"][7])  # planted exact ties


def test_golden_oracle_losses():
    t, meta = load("logq_loss_n257")
    U = t["in.user"].clone().requires_grad_(True)
    Wt = t["in.items"].clone().requires_grad_(True)
    loss = O.inbatch_corrected_logq_loss(F.normalize(U, dim=1), F.normalize(Wt, dim=1), t["in.target_ids"],
                                         t["in.user_ids"], t["in.log_q"], meta["temperature"], meta["lambda_logq"])
    loss.backward()
    torch.testing.assert_close(loss.detach().reshape(1), t["out.loss"], atol=1e-6, rtol=1e-6)
    assert_grad_close(U.grad, t["g.user"], 1e-5, "user")
    assert_grad_close(Wt.grad, t["g.items"], 1e-5, "items")

    t, meta = load("duorec_b96")
    z1 = t["in.z1"].clone().requires_grad_(True)
    z2 = t["in.z2"].clone().requires_grad_(True)
    loss = O.duorec_loss_refined(z1, z2, t["in.target_ids"], meta["temperature"], meta["lambda_sup"])
    loss.backward()
    torch.testing.assert_close(loss.detach().reshape(1), t["out.loss"], atol=1e-6, rtol=1e-6)
    assert_grad_close(z1.grad, t["g.z1"], 1e-5, "z1")
    assert_grad_close(z2.grad, t["g.z2"], 1e-5, "z2")

    t, meta = load("simcse_b64")
    loss = O.simcse_item_loss(t["in.e1"], t["in.e2"], meta["temperature"])
    torch.testing.assert_close(loss.reshape(1), t["out.loss"], atol=1e-6, rtol=1e-6)


def test_golden_oracle_deepfm_and_retrieval():
    t, meta = load("deepfm_r128")
    emb, lin, ws, bs, wo = deepfm_inputs(t)
    logit, prob = OD.deepfm_forward(t["in.x"], emb, lin, meta["bias"], ws, bs, wo)
    torch.testing.assert_close(logit, t["out.logit"], atol=1e-12, rtol=1e-12)
    t, meta = load("retrieval_q24")
    sc, idx = OR.retrieve_topk(t["in.queries_x8"].float() / 8, t["in.items_x16"].float() / 16, meta["k"])
    assert torch.equal(idx, t["out.index"]) and torch.equal(sc, t["out.scores"])
    # the chunked form (the 1M-item tests' oracle) on the same fixture, with chunks that cut
    # through the planted tie groups, in both score dtypes (dyadic inputs: fp32 scores are exact)
    for dtype in (torch.float64, torch.float32):
        sc2, idx2 = OR.retrieve_topk_chunked(t["in.queries_x8"].float() / 8, t["in.items_x16"].float() / 16,
                                             meta["k"], dtype=dtype, chunk=333)
        assert torch.equal(idx2, t["out.index"]) and torch.equal(sc2.double(), t["out.scores"])


# ------------------------------------------------------------------ GPU: HIP path vs fixtures
@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16x3", "fp32", "f16"])
def test_golden_gpu_user_tower(gpu, precision):
    from recsys_amd import ops
    from recsys_amd.tower_code import v1_usertower_train as TT
    from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
    t, meta = load("user_tower_b8")
    cfg = tower_cfg(meta)
    dut = SASRecUserTower(cfg)
    dut.load_state_dict(sub(t, "w."))
    dut = dut.to(gpu).train()
    batch = {k: v.to(gpu) for k, v in tower_batch(t).items()}
    pre = t["in.pretrained"].to(gpu)
    kw = {k: batch[k] for k in FORWARD_KEYS}
    kw["pretrained_vecs"] = TT.lookup_pretrained(pre, batch["item_ids"])
    prev_n = ops.set_nce_precision(precision)
    prev_g = ops.set_gemm_precision("fp32" if precision == "fp32" else "bf16x3")
    try:
        with torch.no_grad():
            torch.testing.assert_close(dut(**kw, training_mode=True).cpu(), t["out.train"], atol=2e-5, rtol=1e-4)
            torch.testing.assert_close(dut(**kw, training_mode=False).cpu(), t["out.eval"], atol=2e-5, rtol=1e-4)
        item_tower = TT.SASRecItemTower(meta["num_items"], 128, t["in.log_q"].clone()).to(gpu)
        item_tower.init_from_pretrained(pre)
        item_tower.set_freeze_state(False)
        tot, main, cl = TT.contrastive_losses(dut, item_tower, item_tower.log_q, batch, cfg, kw["pretrained_vecs"])
        got = torch.stack([tot, main, cl]).detach().cpu()
        torch.testing.assert_close(got, t["out.losses"], atol=1e-4, rtol=0)   # north_star: fp32 within 1e-4
        tot.backward()
        params = dict(dut.named_parameters())
        for k in meta["grads"]:
            assert_grad_close(params[k].grad.cpu(), t["g." + k], 2e-3, k)
        assert_grad_close(item_tower.item_matrix.weight.grad.cpu(), t["g.item_matrix"], 2e-3, "item_matrix")
    finally:
        ops.set_nce_precision(prev_n)
        ops.set_gemm_precision(prev_g)


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16x3", "f16"])
def test_golden_gpu_losses(gpu, precision):
    """Loss fixtures; the live LogQ loss in the given grouped-loss precision: bf16x3 gradients within
    1e-4 of their scale, f16 (single fp16 MFMA gradient products, the reference's autocast arithmetic)
    within 1e-3 (its logits are fp16x3: the loss stays within 1e-4)."""
    from recsys_amd import item_tower as IT
    from recsys_amd import ops
    from recsys_amd.tower_code import v1_refine_usertower as T
    gtol = 1e-4 if precision == "bf16x3" else 1e-3
    t, meta = load("logq_loss_n257")
    U = t["in.user"].to(gpu).requires_grad_(True)
    Wt = t["in.items"].to(gpu).requires_grad_(True)
    prev = ops.set_nce_precision(precision)
    try:
        loss = T.inbatch_corrected_logq_loss(ops.l2_normalize(U), ops.l2_normalize(Wt), t["in.target_ids"].to(gpu),
                                             t["in.user_ids"].to(gpu), t["in.log_q"].to(gpu), meta["temperature"],
                                             meta["lambda_logq"])
        loss.backward()
    finally:
        ops.set_nce_precision(prev)
    assert abs(loss.item() - t["out.loss"].item()) < 1e-4
    assert_grad_close(U.grad.cpu(), t["g.user"], gtol, "user")
    assert_grad_close(Wt.grad.cpu(), t["g.items"], gtol, "items")

    t, meta = load("duorec_b96")
    z1 = t["in.z1"].to(gpu).requires_grad_(True)
    z2 = t["in.z2"].to(gpu).requires_grad_(True)
    loss = T.duorec_loss_refined(z1, z2, t["in.target_ids"].to(gpu), meta["temperature"], meta["lambda_sup"])
    loss.backward()
    assert abs(loss.item() - t["out.loss"].item()) < 1e-4
    assert_grad_close(z1.grad.cpu(), t["g.z1"], 1e-4, "z1")
    assert_grad_close(z2.grad.cpu(), t["g.z2"], 1e-4, "z2")

    t, meta = load("simcse_b64")
    e1 = t["in.e1"].to(gpu).requires_grad_(True)
    e2 = t["in.e2"].to(gpu).requires_grad_(True)
    loss = IT.simcse_loss(e1, e2, meta["temperature"])
    loss.backward()
    assert abs(loss.item() - t["out.loss"].item()) < 1e-4
    assert_grad_close(e1.grad.cpu(), t["g.e1"], 1e-4, "e1")
    assert_grad_close(e2.grad.cpu(), t["g.e2"], 1e-4, "e2")


@pytest.mark.gpu
@pytest.mark.parametrize("cached", [False, True])  # raw V/W tables, or the packed images of a table cache
def test_golden_gpu_deepfm(gpu, cached):
    from recsys_amd import ops
    t, meta = load("deepfm_r128")
    emb, lin, ws, bs, wo = deepfm_inputs(t)
    cache = {} if cached else None
    args = (t["in.x"].to(gpu), [e.to(gpu) for e in emb], [w.to(gpu) for w in lin], meta["bias"],
            [w.to(gpu) for w in ws], [b.to(gpu) for b in bs], wo.to(gpu))
    for _ in range(2 if cached else 1):  # the second call reuses the cached images
        logit, prob = ops.deepfm_forward(*args, cache=cache)
        torch.testing.assert_close(logit.cpu().double(), t["out.logit"], atol=1e-4, rtol=0)  # fp32 logits within 1e-4
        torch.testing.assert_close(prob.cpu().double(), t["out.prob"], atol=1e-5, rtol=0)


@pytest.mark.gpu
@pytest.mark.parametrize("k", [50, 7])
def test_golden_gpu_retrieval_bit_exact(gpu, k):
    from recsys_amd import ops
    t, meta = load("retrieval_q24")
    q = (t["in.queries_x8"].float() / 8).to(gpu)
    it = (t["in.items_x16"].float() / 16).to(gpu)
    sc, idx = ops.retrieve_topk(q, it, k)
    assert torch.equal(idx.cpu(), t["out.index"][:, :k])       # bit-exact indices, ties by index
    assert torch.equal(sc.cpu().double(), t["out.scores"][:, :k])


def test_golden_oracle_hnm():
    """The HNM golden re-derived by the oracle (mining order and counts exact; loss 1e-6)."""
    from oracle import user_tower as OU
    t, meta = load("hnm_n600")
    idx, avail = OU.hnm_mine(t["in.u"].float(), t["in.items"].float(), t["in.target_ids"], meta["k"],
                             meta["hnm_threshold"], meta["temperature_mining"])
    assert torch.equal(idx, t["out.top_idx"]) and torch.equal(avail, t["out.avail"])
    loss, st = OU.inbatch_hnm_corrected_loss_with_stats(t["in.user"], t["in.table"], t["in.target_ids"],
                                                        t["in.log_q"], top_k_percent=meta["loss_top_k_percent"])
    assert st["num_active_hard_negs"] == meta["num_active_hard_negs"]
    torch.testing.assert_close(loss.reshape(1), t["out.loss"], atol=1e-6, rtol=1e-6)


@pytest.mark.gpu
def test_golden_gpu_hnm(gpu):
    """rsx_hnm_mine bit-exact on the golden's integer inputs; the HNM loss within 1e-5."""
    from recsys_amd import ops
    from recsys_amd.tower_code import v1_refine_usertower as T
    t, meta = load("hnm_n600")
    idx, cos, avail = ops.hnm_mine(t["in.u"].float().to(gpu), t["in.items"].float().to(gpu),
                                   t["in.target_ids"].to(gpu), meta["k"], meta["hnm_threshold"],
                                   meta["temperature_mining"])
    assert torch.equal(idx.cpu(), t["out.top_idx"])
    assert torch.equal(avail.cpu().long(), t["out.avail"])
    loss, st = T.inbatch_hnm_corrected_loss_with_stats(t["in.user"].to(gpu), t["in.table"].to(gpu),
                                                       t["in.target_ids"].to(gpu), t["in.log_q"].to(gpu),
                                                       top_k_percent=meta["loss_top_k_percent"])
    assert st["num_active_hard_negs"] == meta["num_active_hard_negs"]
    assert abs(loss.item() - t["out.loss"].item()) <= 1e-5 * abs(t["out.loss"].item())
