"""Item tower (item_tower.py:41-322), SimCSE loss (:1069-1082) and the hard-emphasis loss
(v1_refine_usertower.py:762-822): recsys_amd on cuda:0 vs the CPU oracle with identical
weights. The BERT on both sides is one locally built, randomly initialised BertModel
(no pretrained weights offline: parity unpinned against the reference's bert-base-uncased)."""
import copy

import pytest
import torch
import torch.nn.functional as F

import recsys_amd  # noqa: F401
from recsys_amd import item_tower as IT
from recsys_amd import ops
from recsys_amd.tower_code import v1_refine_usertower as T
from recsys_amd.tower_code import v1_usertower_train as TT
from recsys_amd import synth
from oracle import item_tower as OIT
from oracle import user_tower as O
from tests.helpers import paired_towers, small_cfg, small_universe, to_dev

pytestmark = pytest.mark.gpu


def _tiny_bert(hidden=64):
    return IT.build_local_bert(hidden_size=hidden, num_layers=2, num_heads=2, intermediate=2 * hidden,
                               vocab_size=2000, max_position=64, seed=3)


def _inputs(B, n_std=6, vocab=384, R=32, S=32, seed=0):
    g = torch.Generator().manual_seed(seed)
    std = torch.randint(0, vocab, (B, n_std), generator=g)
    std[torch.rand(B, n_std, generator=g) < 0.1] = 0
    lens = torch.randint(2, R + 1, (B, 9), generator=g)
    re_ids = torch.randint(1000, 2000, (B, 9, R), generator=g)
    re_mask = (torch.arange(R).view(1, 1, R) < lens.unsqueeze(-1)).long()
    re_ids = re_ids * re_mask
    re_ids[:, :, 0] = 101
    tl = torch.randint(2, S + 1, (B,), generator=g)
    txt_mask = (torch.arange(S).view(1, S) < tl.unsqueeze(-1)).long()
    txt = torch.randint(1000, 2000, (B, S), generator=g) * txt_mask
    txt[:, 0] = 101
    return [std, re_ids, re_mask, txt, txt_mask]


def _pair(embed_dim, out_dim=128):
    bert = _tiny_bert()
    torch.manual_seed(7)
    ref = OIT.OracleHybridItemTower(384, 6, embed_dim, out_dim, bert_model=bert)
    dut = IT.HybridItemTower(384, 6, embed_dim, out_dim, bert_model=copy.deepcopy(bert))
    dut.load_state_dict(ref.state_dict())
    return ref, dut


@pytest.mark.parametrize("embed_dim", [64, 128])
def test_hybrid_item_tower_forward_and_grads(gpu, embed_dim):
    """Eval-mode forward (dropout off) and the gradients of a scalar of the output, every
    parameter: rtol 1e-4 / atol 2e-5 (value), 1e-3 relative to the gradient's max (grads)."""
    ref, dut = _pair(embed_dim)
    ref.eval()
    dut = dut.to(gpu).eval()
    x = _inputs(24, seed=embed_dim)
    g = torch.Generator().manual_seed(1)
    w = torch.randn(24, 128, generator=g)
    y_ref = ref(*x)
    (y_ref * w).sum().backward()
    y = dut(*[t.to(gpu) for t in x])
    (y * w.to(gpu)).sum().backward()
    torch.testing.assert_close(y.detach().cpu(), y_ref.detach(), atol=2e-5, rtol=1e-4)
    ref_p = dict(ref.named_parameters())
    n = 0
    for name, p in dut.named_parameters():
        if p.grad is None:
            assert ref_p[name].grad is None or ref_p[name].grad.abs().max() == 0, name
            continue
        gr = ref_p[name].grad
        scale = gr.abs().max().item() + 1e-12
        err = (p.grad.cpu() - gr).abs().max().item()
        assert err <= 1e-3 * scale + 1e-7, (name, err, scale)
        n += 1
    assert n > 30


def _config0_inputs(B=256, n_std=6, vocab=384, R=32, S=32, seed=0):
    """SURVEY.md 8d config 1 (BASELINE configs[0]): std [B, 6] ~ U{0..383} with ~10 % PAD;
    RE ids [B, 9, 32] and text [B, 32]: [CLS]=101, length ~ U{2..32} ([CLS][SEP] for an empty
    field), word pieces ~ U{1000..30521}, [SEP]=102 last, 0-padded, masks 1 / 0."""
    g = torch.Generator().manual_seed(seed)
    std = torch.randint(0, vocab, (B, n_std), generator=g)
    std[torch.rand(B, n_std, generator=g) < 0.1] = 0

    def seqs(shape, width):
        lens = torch.randint(2, width + 1, shape, generator=g)
        ar = torch.arange(width).view(*([1] * len(shape)), width)
        ids = torch.randint(1000, 30522, shape + (width,), generator=g)
        ids = torch.where(ar == 0, torch.full_like(ids, 101), ids)
        ids = torch.where(ar == (lens - 1).unsqueeze(-1), torch.full_like(ids, 102), ids)
        mask = (ar < lens.unsqueeze(-1)).long()
        return ids * mask, mask

    re_ids, re_mask = seqs((B, 9), R)
    txt, txt_mask = seqs((B,), S)
    return [std, re_ids, re_mask, txt, txt_mask]


@pytest.mark.parametrize("grad", [False, True])
def test_hybrid_item_tower_config0_full_size(gpu, grad):
    """BASELINE configs[0] at its size: HybridItemTower(384, 6, embed_dim=64, output_dim=128) on 256
    items with a bert-base-shaped BERT (hidden 768, 12 heads, intermediate 3072, vocab 30522;
    2 of its 12 layers, to bound the CPU oracle's time), eval mode, against
    oracle/item_tower.py (item_tower.py:228-286): rtol 1e-4. no_grad is the serving /
    refresh path (the text BERT over packed valid tokens, bf16x3 GEMMs); with grad the text BERT
    is HF's module and the rest runs on this package's kernels."""
    bert = IT.build_local_bert(hidden_size=768, num_layers=2, num_heads=12, intermediate=3072, vocab_size=30522,
                               max_position=512, seed=5)
    torch.manual_seed(8)
    ref = OIT.OracleHybridItemTower(384, 6, 64, 128, bert_model=bert).eval()
    dut = IT.HybridItemTower(384, 6, 64, 128, bert_model=copy.deepcopy(bert))
    dut.load_state_dict(ref.state_dict())
    dut = dut.to(gpu).eval()
    x = _config0_inputs()
    with torch.no_grad():
        y_ref = ref(*x)
    xd = [t.to(gpu) for t in x]
    if grad:
        y = dut(*xd)
        y.sum().backward()
    else:
        with torch.no_grad():
            y = dut(*xd)
    assert y.shape == (256, 128)
    torch.testing.assert_close(y.detach().cpu(), y_ref, atol=1e-5, rtol=1e-4)


def test_projector_wrapper_and_simcse_loss(gpu):
    """OptimizedItemTower + SimCSEModelWrapper forward and the symmetric SimCSE loss (fused
    InfoNCE, both directions) vs the oracle: loss within 1e-5 relative, grads 1e-4."""
    torch.manual_seed(2)
    ref_proj = OIT.OracleOptimizedItemTower(128, 128)
    dut_proj = IT.OptimizedItemTower(128, 128)
    dut_proj.load_state_dict(ref_proj.state_dict())
    dut_proj = dut_proj.to(gpu)
    g = torch.Generator().manual_seed(4)
    e = torch.randn(300, 128, generator=g)
    e2 = e + 0.3 * torch.randn(300, 128, generator=g)
    a1 = e.clone().requires_grad_()
    a2 = e2.clone().requires_grad_()
    l_ref = OIT.simcse_loss(ref_proj(a1), ref_proj(a2))
    l_ref.backward()
    b1 = e.to(gpu).requires_grad_()
    b2 = e2.to(gpu).requires_grad_()
    l_dut = IT.simcse_loss(dut_proj(b1), dut_proj(b2))
    l_dut.backward()
    assert abs(l_dut.item() - l_ref.item()) <= 1e-5 * abs(l_ref.item()) + 1e-6
    torch.testing.assert_close(b1.grad.cpu(), a1.grad, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(b2.grad.cpu(), a2.grad, atol=1e-6, rtol=1e-4)


def test_simcse_train_step_runs(gpu):
    """Train-mode SimCSE step (dropout on, two views) through the wrapper: finite loss, every
    trainable non-BERT parameter receives a gradient, calculate_metrics is finite."""
    _, dut = _pair(64)
    model = IT.SimCSEModelWrapper(dut, IT.OptimizedItemTower(128, 128)).to(gpu).train()
    opt = torch.optim.AdamW([p for n, p in model.named_parameters() if "bert_model" not in n], lr=1e-4)
    x = [t.to(gpu) for t in _inputs(32, seed=9)]
    loss, e1, e2 = IT.simcse_train_step(model, x, x, opt)
    assert torch.isfinite(loss)
    align, uni = IT.calculate_metrics(e1, e2)
    assert align >= 0 and uni == uni


@pytest.mark.parametrize("N,lambda_logq", [(700, 1.0), (257, 0.0)])
def test_hard_emphasis_loss_parity(gpu, N, lambda_logq):
    """full_batch_hard_emphasis_loss vs the oracle: loss 1e-5 relative, user / item-matrix
    gradients 1e-4; near-duplicate items exercise the item-similarity mask."""
    g = torch.Generator().manual_seed(N)
    I = 200
    W = torch.randn(I + 1, 128, generator=g)
    W[5] = W[4] + 0.01 * torch.randn(128, generator=g)   # cos > 0.9 pair
    lq = torch.log_softmax(torch.randn(I + 1, generator=g), 0)
    t = torch.randint(1, I + 1, (N,), generator=g)
    t[:3] = 4
    t[3:6] = 5
    U = torch.randn(N, 128, generator=g)
    u1 = U.clone().requires_grad_()
    w1 = W.clone().requires_grad_()
    l_ref, s_ref = O.full_batch_hard_emphasis_loss(u1, w1, t, lq, hard_margin=0.2, temperature=0.15,
                                                   lambda_logq=lambda_logq)
    l_ref.backward()
    u2 = U.to(gpu).requires_grad_()
    w2 = W.to(gpu).requires_grad_()
    l_dut, s_dut = T.full_batch_hard_emphasis_loss(u2, w2, t.to(gpu), lq.to(gpu), hard_margin=0.2,
                                                   temperature=0.15, lambda_logq=lambda_logq)
    l_dut.backward()
    assert s_dut["num_hard"] == s_ref["num_hard"]
    assert abs(l_dut.item() - l_ref.item()) <= 1e-5 * abs(l_ref.item())
    assert abs(s_dut["avg_hn_similarity"] - s_ref["avg_hn_similarity"]) < 1e-5
    torch.testing.assert_close(u2.grad.cpu(), u1.grad, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(w2.grad.cpu(), w1.grad, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("N", [4096])
def test_hard_emphasis_loss_large_matches_dense_form(gpu, N):
    """ops.nce_emphasis_loss (dense masked InfoNCE + O(N k) margin correction, no N x N tensor) against the
    reference's own dense arithmetic (:546-554: N x N cosines, scatter_ of margin / tau on the mined columns,
    same-item masked_fill, F.cross_entropy) in float64 on the same mined columns, with duplicated targets
    (same-item masking) and mined columns on rows that share a target: loss 1e-5 relative, gradients
    1e-4 of their scale."""
    g = torch.Generator().manual_seed(N + 1)
    I = 1500                                                   # ~N / I repeats per target: many same-item pairs
    W = F.normalize(torch.randn(I, 128, generator=g), dim=1)
    lq = torch.log_softmax(torch.randn(I, generator=g), 0)
    t = torch.randint(0, I, (N,), generator=g)
    U = torch.randn(N, 128, generator=g)
    tau, margin = 0.1, 0.2
    u2 = U.to(gpu).requires_grad_()
    w2 = W.to(gpu).requires_grad_()
    loss, st = T.full_batch_hard_emphasis_loss(u2, w2, t.to(gpu), lq.to(gpu), temperature=tau, hard_margin=margin)
    loss.backward()
    k = st["num_hard"]
    un = F.normalize(U.to(gpu), dim=1)
    itn = F.normalize(W.to(gpu)[t.to(gpu)], dim=1)
    top, _, _ = ops.hnm_mine(un, itn, t.to(gpu), k, 0.9, 1.0)
    top = top.cpu()
    u1 = U.double().requires_grad_()
    w1 = W.double().requires_grad_()
    u, it = F.normalize(u1, dim=1), F.normalize(w1[t], dim=1)
    logits = (u @ it.T) / tau - lq.double()[t].view(1, -1)
    emph = torch.zeros_like(logits).scatter_(1, top, margin / tau)
    same = t.view(-1, 1) == t.view(1, -1)
    same.fill_diagonal_(False)
    ref = F.cross_entropy((logits + emph).masked_fill(same, float("-inf")), torch.arange(N))
    ref.backward()
    assert abs(loss.item() - ref.item()) <= 1e-5 * abs(ref.item())
    for got, want in ((u2.grad, u1.grad), (w2.grad, w1.grad)):
        err = float((got.cpu().double() - want).abs().max()) / float(want.abs().max())
        assert err <= 1e-4, err


def test_hard_emphasis_step_parity(gpu):
    """train_user_tower's step losses (eval mode: dropout off, both views equal) vs the oracle
    tower + oracle losses with the same weights."""
    cfg = small_cfg(num_items=500)
    items = small_universe(500)
    batch = synth.make_batch(items, 96, seed=21)
    ref, dut = paired_towers(cfg, gpu)
    ref.eval(); dut.eval()
    log_q = items.log_q
    kw = {k: batch[k] for k in O._FWD_KEYS}
    kw["pretrained_vecs"] = items.pretrained[batch["item_ids"]]
    out = ref(**kw, training_mode=True)
    last = out[:, -1, :]
    valid = ~batch["padding_mask"][:, -1]
    m_ref, _ = O.full_batch_hard_emphasis_loss(F.normalize(last[valid], dim=1), items.pretrained,
                                               batch["target_ids"][:, -1][valid], log_q,
                                               top_k_percent=cfg.top_k_percent, hard_margin=cfg.hard_margin,
                                               hnm_threshold=cfg.hnm_threshold, temperature=0.15,
                                               lambda_logq=cfg.lambda_logq)
    c_ref = O.duorec_loss_refined(last, last, batch["target_ids"][:, -1], lambda_sup=cfg.lambda_sup)
    it = TT.SASRecItemTower(500, 128, log_q.clone()).to(gpu)
    it.init_from_pretrained(items.pretrained.to(gpu))
    b = to_dev(batch, gpu)
    b["pretrained_vecs"] = items.pretrained.to(gpu)[b["item_ids"]]
    total, main, cl, _ = TT.hard_emphasis_losses(dut, it, log_q.to(gpu), b, cfg)
    assert abs(main.item() - m_ref.item()) <= 1e-4 * abs(m_ref.item())
    assert abs(cl.item() - c_ref.item()) <= 1e-4 * abs(c_ref.item())


def test_evaluate_model_recall_matches_oracle(gpu, tmp_path):
    """evaluate_model (v1_usertower_train.py:548-711): Recall@K from the GPU tower + fused
    top-k equals the oracle tower + explicit top-k on the same weights / targets."""
    import pandas as pd
    from oracle.retrieval import retrieve_topk as ref_topk
    cfg = small_cfg(num_items=500)
    items = small_universe(500)
    ref, dut = paired_towers(cfg, gpu)
    ref.eval(); dut.eval()
    batches = []
    targets = {}
    g = torch.Generator().manual_seed(8)
    for bi in range(3):
        b = synth.make_batch(items, 40, seed=30 + bi)
        b["user_ids"] = [f"u{bi}_{j}" for j in range(40)]
        b["pretrained_vecs"] = items.pretrained[b["item_ids"]]
        for j, u in enumerate(b["user_ids"]):
            if j % 7 == 3:
                continue                      # users without targets are skipped
            n = int(torch.randint(1, 4, (1,), generator=g))
            targets[u] = [f"a{int(t)}" for t in torch.randint(1, 501, (n,), generator=g)]
        batches.append(b)
    path = tmp_path / "targets.parquet"
    pd.DataFrame({"customer_id": list(targets), "target_ids": list(targets.values())}).to_parquet(path)

    class Proc:
        item2id = {f"a{i}": i for i in range(1, 501)}

    it = TT.SASRecItemTower(500, 128, items.log_q.clone()).to(gpu)
    it.init_from_pretrained(items.pretrained.to(gpu))
    res = TT.evaluate_model(dut, it, batches, str(path), gpu, Proc(), k_list=[5, 20, 100])
    # oracle
    hits = {k: 0 for k in (5, 20, 100)}
    n = 0
    W = F.normalize(items.pretrained, dim=1)
    for b in batches:
        kw = {k: b[k] for k in O._FWD_KEYS}
        kw["pretrained_vecs"] = b["pretrained_vecs"]
        with torch.no_grad():
            u = F.normalize(ref(**kw, training_mode=False), dim=1)
        valid = [i for i, uid in enumerate(b["user_ids"]) if uid in targets]
        _, top = ref_topk(u[valid], W, 100)
        for r, i in enumerate(valid):
            actual = {Proc.item2id[t] for t in targets[b["user_ids"][i]]}
            n += 1
            for k in hits:
                hits[k] += int(not actual.isdisjoint(top[r, :k].tolist()))
    for k in hits:
        assert abs(res[f"Recall@{k}"] - hits[k] / n * 100) < 1e-9, (k, res, hits, n)


@pytest.mark.parametrize("hidden,heads,layers", [(256, 4, 2), (768, 12, 1)])
def test_bert_cls_packed_matches_bertmodel(gpu, hidden, heads, layers):
    """Packed-token BERT inference (item_tower.bert_cls_packed: bf16x3 GEMMs, varlen attention,
    fused residual+LayerNorm, [CLS]-only last feed-forward) against HF BertModel's dense masked
    forward, [CLS] row, eval: atol 2e-4 / rtol 1e-4 (the GEMMs are bf16x3, ~2^-17 per product)."""
    bert = IT.build_local_bert(hidden_size=hidden, num_layers=layers, num_heads=heads, intermediate=4 * hidden,
                               vocab_size=2000, max_position=64, seed=5).to(gpu).eval()
    g = torch.Generator().manual_seed(hidden)
    B, S = 40, 32
    tl = torch.randint(1, S + 1, (B,), generator=g)
    tl[0], tl[1] = 1, S                                            # single-token row, full row
    mask = (torch.arange(S).view(1, S) < tl.unsqueeze(-1)).long()
    ids = torch.randint(1000, 2000, (B, S), generator=g) * mask
    ids[:, 0] = 101
    ids, mask = ids.to(gpu), mask.to(gpu)
    with torch.no_grad():
        assert IT.bert_packed_ok(bert, ids, mask)
        got = IT.bert_cls_packed(bert, ids, mask)
        want = bert(input_ids=ids, attention_mask=mask).last_hidden_state[:, 0, :]
    torch.testing.assert_close(got, want, atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize("hidden,heads,layers,S", [(768, 12, 2, 32), (256, 4, 2, 48), (512, 8, 1, 24)])
def test_bert_cls_packed_train_matches_bertmodel(gpu, hidden, heads, layers, S):
    """The packed BERT under autograd (item_tower.bert_cls_packed_train: bf16x3 token GEMMs, varlen
    attention with the fp32 head-dim-64 backward, fused residual + LayerNorm both ways, [CLS]-only last
    layer) against HF BertModel's dense masked forward and backward, eval mode (dropout off): the [CLS]
    rows atol 2e-4 / rtol 1e-4, every parameter gradient of a random projection of them within 1e-3 of
    that gradient's scale (max |g|) -- the SimCSE step's BERT fine-tuning (item_tower.py:264-272)."""
    ref = IT.build_local_bert(hidden_size=hidden, num_layers=layers, num_heads=heads, intermediate=4 * hidden,
                              vocab_size=2000, max_position=64, seed=11).to(gpu).eval()
    dut = copy.deepcopy(ref)
    g = torch.Generator().manual_seed(hidden + S)
    B = 40
    tl = torch.randint(1, S + 1, (B,), generator=g)
    tl[0], tl[1] = 1, S
    mask = (torch.arange(S).view(1, S) < tl.unsqueeze(-1)).long()
    ids = torch.randint(1000, 2000, (B, S), generator=g) * mask
    ids[:, 0] = 101
    ids, mask = ids.to(gpu), mask.to(gpu)
    w = torch.randn(B, hidden, generator=g).to(gpu)
    assert IT.bert_packed_ok(dut, ids, mask)
    got = IT.bert_cls_packed_train(dut, ids, mask)
    want = ref(input_ids=ids, attention_mask=mask).last_hidden_state[:, 0, :]
    torch.testing.assert_close(got.detach(), want.detach(), atol=2e-4, rtol=1e-4)
    (got * w).sum().backward()
    (want * w).sum().backward()
    used = 0
    # the key bias's gradient is zero in exact arithmetic (a shift of every key adds a per-row constant to the
    # scores): both sides hold rounding noise there, judged against the largest gradient of the model
    floor = 1e-4 * max(float(p.grad.abs().max()) for p in ref.parameters() if p.grad is not None)
    for (n, pr), (_, pd) in zip(ref.named_parameters(), dut.named_parameters()):
        if pr.grad is None:                     # the pooler: not on the [CLS]-hidden path
            assert pd.grad is None or not pd.grad.any(), n
            continue
        used += 1
        scale = max(float(pr.grad.abs().max()), floor if n.endswith("key.bias") else 0.0) + 1e-30
        err = float((pd.grad - pr.grad).abs().max()) / scale
        assert err <= 1e-3, (n, err)
    assert used == 5 + 16 * layers


def test_bert_train_dropout_active(gpu):
    """Training mode: the packed path applies BERT's dropouts (two calls differ, both finite, the
    gradients flow to every encoder weight)."""
    bert = IT.build_local_bert(hidden_size=256, num_layers=2, num_heads=4, intermediate=1024, vocab_size=2000,
                               max_position=64, seed=12).to(gpu).train()
    x = [t.to(gpu) for t in _inputs(16, seed=6)]
    a = IT.bert_cls_packed_train(bert, x[3], x[4])
    b = IT.bert_cls_packed_train(bert, x[3], x[4])
    assert torch.isfinite(a).all() and not torch.equal(a, b)
    a.sum().backward()
    for n, p in bert.named_parameters():
        if "pooler" not in n:
            assert p.grad is not None and torch.isfinite(p.grad).all(), n


def test_item_tower_inference_uses_packed_bert_and_falls_back(gpu):
    """HybridItemTower under no_grad + eval takes the packed BERT (same vectors as the module
    path with gradients enabled); a batch whose position 0 is masked in some row is not
    packable (BertModel still emits that row) and takes BertModel, with the same result."""
    bert = IT.build_local_bert(hidden_size=256, num_layers=2, num_heads=4, intermediate=1024, vocab_size=2000,
                               max_position=64, seed=9)
    torch.manual_seed(1)
    tower = IT.HybridItemTower(384, 6, 128, 128, bert_model=bert).to(gpu).eval()
    x = [t.to(gpu) for t in _inputs(32, seed=4)]
    with IT.bert_train_native(False):
        want = tower(*x).detach()                                  # grad enabled, native train path off: BertModel
    with torch.no_grad():
        got = tower(*x)
    torch.testing.assert_close(got, want, atol=2e-4, rtol=1e-4)
    x[4] = x[4].clone()
    x[4][3, 0] = 0
    with torch.no_grad():
        assert not IT.bert_packed_ok(tower.bert_model, x[3], x[4])
        got2 = tower(*x)
    want2 = tower(*x).detach()
    torch.testing.assert_close(got2, want2, atol=1e-5, rtol=1e-5)


def test_std_id_range_checked_on_device(gpu):
    """An STD id outside the embedding (here 384 for std_vocab_size 384) is caught by the device
    check (rsx_ids_check, no host sync in forward): check_inputs() -- and, once the flag has
    reached the host, the next forward -- raises IndexError; the gather itself never reads out
    of bounds, and in-range batches after the error run normally."""
    _, dut = _pair(64)
    dut = dut.to(gpu).eval()
    x = [t.to(gpu) for t in _inputs(8, seed=5)]
    with torch.no_grad():
        good = dut(*x)
        dut.check_inputs()
        bad = [t.clone() for t in x]
        bad[0][3, 2] = 384
        dut(*bad)
        with pytest.raises(IndexError, match=r"out of range \[0, 384\)"):
            dut.check_inputs()
        again = dut(*x)                       # the error was reported once; in-range runs on
        dut.check_inputs()
        torch.testing.assert_close(again, good, atol=0, rtol=0)
        bad[0][0, 0] = -1
        dut(*bad)
        torch.cuda.synchronize()
        with pytest.raises(IndexError):
            dut(*x)                           # the flag is visible: raised by the next forward
