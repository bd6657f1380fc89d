"""Module- and step-level parity: recsys_amd SASRecUserTower + contrastive step on cuda:0 vs
the CPU oracle (same weights, same inputs, dropout p=0 so both views are deterministic)."""
import pytest
import torch
import torch.nn.functional as F

import recsys_amd  # noqa: F401
from recsys_amd import ops, synth
from recsys_amd.tower_code import v1_refine_usertower as T
from recsys_amd.tower_code import v1_usertower_train as TT
from oracle import user_tower as O
from tests.helpers import paired_towers, small_cfg, small_universe, to_dev

pytestmark = pytest.mark.gpu


def _kw(batch, pretrained):
    kw = {k: batch[k] for k in O._FWD_KEYS}
    kw["pretrained_vecs"] = pretrained[batch["item_ids"]]
    return kw


@pytest.mark.parametrize("training_mode", [True, False])
def test_tower_forward_parity(gpu, training_mode):
    cfg = small_cfg(num_items=500)
    items = small_universe(500)
    batch = synth.make_batch(items, 48, seed=11)
    ref, dut = paired_towers(cfg, gpu)
    ref.train(); dut.train()
    kw = _kw(batch, items.pretrained)
    y_ref = ref(**kw, training_mode=training_mode)
    y = dut(**{k: (v.to(gpu) if torch.is_tensor(v) else v) for k, v in kw.items()}, training_mode=training_mode)
    assert torch.isfinite(y).all()
    torch.testing.assert_close(y.cpu(), y_ref.detach(), atol=2e-5, rtol=1e-4)


def test_step_losses_and_grads_parity(gpu):
    cfg = small_cfg(num_items=500)
    items = small_universe(500)
    batch = synth.make_batch(items, 64, seed=12)
    ref, dut = paired_towers(cfg, gpu)
    ref.train(); dut.train()
    W_ref = items.pretrained.clone().requires_grad_()
    tot_r, main_r, cl_r = O.contrastive_losses(ref, W_ref, items.log_q, batch, items.pretrained)
    tot_r.backward()

    item_tower = TT.SASRecItemTower(500, 128, items.log_q.clone()).to(gpu)
    item_tower.init_from_pretrained(items.pretrained.to(gpu))
    item_tower.set_freeze_state(False)
    bd = to_dev(batch, gpu)
    pv = TT.lookup_pretrained(items.pretrained.to(gpu), bd["item_ids"])
    tot, main, cl = TT.contrastive_losses(dut, item_tower, item_tower.log_q, bd, cfg, pv)
    for a, b in [(tot, tot_r), (main, main_r), (cl, cl_r)]:
        assert abs(a.item() - b.item()) < 1e-4, (a.item(), b.item())
    tot.backward()
    for (name, pr), (_, pd) in zip(ref.named_parameters(), dut.named_parameters()):
        gr = pr.grad if pr.grad is not None else torch.zeros_like(pr)
        gd = pd.grad.cpu() if pd.grad is not None else torch.zeros_like(pr)
        scale = gr.abs().max().item() + 1e-12
        err = (gd - gr).abs().max().item()
        assert err <= 2e-3 * scale + 1e-6, f"{name}: max err {err} vs grad scale {scale}"
    gw = item_tower.item_matrix.weight.grad.cpu()
    err = (gw - W_ref.grad).abs().max().item()
    assert err <= 2e-3 * W_ref.grad.abs().max().item() + 1e-6


def test_step_runs_with_dropout_and_updates(gpu):
    cfg = small_cfg(num_items=500, dropout=0.2)
    items = small_universe(500)
    batch = to_dev(synth.make_batch(items, 64, seed=13), gpu)
    torch.manual_seed(0)
    model = T.SASRecUserTower(cfg).to(gpu)
    item_tower = TT.SASRecItemTower(500, 128, items.log_q.clone()).to(gpu)
    item_tower.init_from_pretrained(items.pretrained.to(gpu))
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay)
    before = model.item_proj.weight.detach().clone()
    lookup = items.pretrained.to(gpu)
    losses = []
    for _ in range(3):
        tot, main, cl = TT.contrastive_step(model, item_tower, item_tower.log_q, batch, opt, None, cfg,
                                            pretrained_lookup=lookup)
        losses.append(tot.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert not torch.equal(before, model.item_proj.weight.detach())
    # the two dropout views differ, so the DuoRec InfoNCE term is not at its p=0 minimum
    assert cl.item() > 0


def test_dp_objective_single_rank_equals_single_gpu_step(gpu):
    """dist.contrastive_objective_dp at world size 1 == v1_usertower_train.contrastive_losses."""
    from recsys_amd import dist as Dd
    cfg = small_cfg(num_items=500)
    items = small_universe(500)
    bd = to_dev(synth.make_batch(items, 64, seed=21), gpu)
    _, dut = paired_towers(cfg, gpu)
    dut.train()
    it = TT.SASRecItemTower(500, 128, items.log_q.clone()).to(gpu)
    it.init_from_pretrained(items.pretrained.to(gpu))
    it.set_freeze_state(False)
    pv = TT.lookup_pretrained(items.pretrained.to(gpu), bd["item_ids"])
    tot, main, cl = TT.contrastive_losses(dut, it, it.log_q, bd, cfg, pv)
    tot.backward()
    g1 = [p.grad.clone() for p in dut.parameters()]
    gw1 = it.item_matrix.weight.grad.clone()
    dut.zero_grad(); it.zero_grad()
    obj, tot2, main2, cl2 = Dd.contrastive_objective_dp(dut, it, it.log_q, bd, cfg, pretrained_vecs=pv)
    for a, b in [(obj, tot), (tot2, tot), (main2, main), (cl2, cl)]:
        assert abs(a.item() - b.item()) < 1e-5
    obj.backward()
    for a, p in zip(g1, dut.parameters()):
        torch.testing.assert_close(p.grad, a, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(it.item_matrix.weight.grad, gw1, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("gemm", ["fp32", "bf16x3"])
def test_packed_forward_equals_dense_rows(gpu, gemm):
    """forward_packed outputs == forward(training_mode=True) at the packed positions, including
    the padded DuoRec "last" positions (dropout 0). fp32 token GEMMs: atol 2e-6 (same
    arithmetic as the dense path); bf16x3 token GEMMs (the default): atol 2e-5 / rtol 1e-4 on the
    unit-norm outputs (~2^-17 relative error per product through two encoder layers)."""
    prev = ops._gemm_precision
    ops.set_gemm_precision(gemm)
    try:
        _packed_vs_dense(gpu, 2e-6 if gemm == "fp32" else 2e-5, 1e-5 if gemm == "fp32" else 1e-4)
    finally:
        ops.set_gemm_precision(prev)


def _packed_vs_dense(gpu, atol, rtol):
    cfg = small_cfg(num_items=500)
    items = small_universe(500)
    bd = to_dev(synth.make_batch(items, 40, seed=31), gpu)
    _, dut = paired_towers(cfg, gpu)
    dut.train()
    pv = items.pretrained.to(gpu)[bd["item_ids"]]
    dense = dut(**{k: bd[k] for k in O._FWD_KEYS}, pretrained_vecs=pv, training_mode=True)
    pk, o1, _ = TT.packed_views(dut, bd, pretrained_vecs=pv)
    assert (pk.tok_pad == 1).sum() > 0  # some users' last index falls on padding
    torch.testing.assert_close(o1, dense.reshape(-1, dense.shape[-1])[pk.flat], atol=atol, rtol=rtol)


def test_gated_off_tables_still_decay(gpu):
    """Appendix B trap 4: s_mask zeroes the gates of the type/color/graphic/section tables
    (v1_refine_usertower.py:437-438), but the reference still gathers them, so their gradients
    are zero TENSORS (not None) and AdamW's decoupled weight decay shrinks them every step:
    p <- p * (1 - lr * wd) exactly (the Adam update of a zero gradient is 0)."""
    cfg = small_cfg(num_items=500, dropout=0.0)
    items = small_universe(500)
    batch = to_dev(synth.make_batch(items, 32, seed=3), gpu)
    torch.manual_seed(0)
    model = T.SASRecUserTower(cfg).to(gpu)
    item_tower = TT.SASRecItemTower(500, 128, items.log_q.clone()).to(gpu)
    item_tower.init_from_pretrained(items.pretrained.to(gpu))
    opt = torch.optim.AdamW(model.parameters(), lr=cfg.lr, weight_decay=cfg.weight_decay)
    names = ["type_emb.weight", "color_emb.weight", "graphic_emb.weight", "section_emb.weight"]
    params = dict(model.named_parameters())
    before = {n: params[n].detach().clone() for n in names}
    TT.contrastive_step(model, item_tower, item_tower.log_q, batch, opt, None, cfg,
                        pretrained_lookup=items.pretrained.to(gpu))
    for n in names:
        g = params[n].grad
        assert g is not None and torch.count_nonzero(g) == 0, n
        torch.testing.assert_close(params[n].detach(), before[n] * (1 - cfg.lr * cfg.weight_decay),
                                   atol=0, rtol=1e-6)


def test_index_prefetcher_steps_equal_inline(gpu):
    """dist.IndexPrefetcher (indexes built two steps ahead on a background thread, the bench's
    single-rank loop) gives exactly the inline-index training trajectory: same losses, same
    parameters after four AdamW steps over two alternating batches with dropout."""
    from recsys_amd import dist as Dd
    cfg = small_cfg(num_items=500, dropout=0.2)
    items = small_universe(500)
    batches = [to_dev(synth.make_batch(items, 64, seed=s), gpu) for s in (31, 32)]
    lookup = items.pretrained.to(gpu)

    def run(prefetch):
        torch.manual_seed(0)
        model = T.SASRecUserTower(cfg).to(gpu).train()
        it = TT.SASRecItemTower(500, 128, items.log_q.clone()).to(gpu)
        it.init_from_pretrained(lookup)
        it.set_freeze_state(False)
        opt = torch.optim.AdamW(list(model.parameters()) + list(it.parameters()), lr=cfg.lr)
        bucket = Dd.GradBucket(list(model.parameters()) + list(it.parameters()))
        pf = Dd.IndexPrefetcher() if prefetch else None
        losses = []
        for i in range(4):
            ix = pf.pop(i) if pf else None
            if ix is None:
                ix = Dd.prepare_step_index(batches[i % 2], pretrained_lookup=lookup)
            out = Dd.contrastive_step_dp(model, it, it.log_q, batches[i % 2], opt, cfg, lookup, bucket, index=ix)
            losses.append([float(v) for v in out])
            if pf:
                pf.submit(i + 2, batches[i % 2], pretrained_lookup=lookup)
        if pf:
            pf.close()
        torch.cuda.synchronize()
        return losses, [p.detach().clone() for p in model.parameters()]

    l0, p0 = run(False)
    l1, p1 = run(True)
    assert l0 == l1
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)


def test_step_parity_on_reference_sample_batch(gpu):
    """A real SASRecDataset batch (the 13 customers of the reference's own sample file, through
    FeatureProcessor + the DataLoader's default collation, tests/test_user_dataset_cpu.py) through
    the GPU step's losses and gradients vs the oracle: the drop-in producer feeds the drop-in step."""
    from torch.utils.data import default_collate
    from tests.test_user_dataset_cpu import _frames
    users, items_df, sq, _ = _frames(cap=10_000)
    fp = T.FeatureProcessor(users, items_df, sq)
    ds = T.SASRecDataset(fp, max_len=50, is_train=True)
    batch = default_collate([ds[i] for i in range(len(ds))])
    I = fp.num_items
    cfg = small_cfg(num_items=I, hash_size=100)
    g = torch.Generator().manual_seed(31)
    pre = F.normalize(torch.randn(I + 1, 128, generator=g), dim=1)
    pre[0] = 0.0
    log_q = fp.get_logq_probs("cpu")
    ref, dut = paired_towers(cfg, gpu)
    ref.train(); dut.train()
    W_ref = pre.clone().requires_grad_()
    tot_r, main_r, cl_r = O.contrastive_losses(ref, W_ref, log_q, batch, pre)
    tot_r.backward()
    item_tower = TT.SASRecItemTower(I, 128, log_q.clone()).to(gpu)
    item_tower.init_from_pretrained(pre.to(gpu))
    item_tower.set_freeze_state(False)
    bd = to_dev(batch, gpu)
    tot, main, cl = TT.contrastive_losses(dut, item_tower, item_tower.log_q, bd, cfg,
                                          pretrained_lookup=pre.to(gpu))
    for a, b in [(tot, tot_r), (main, main_r), (cl, cl_r)]:
        assert abs(a.item() - b.item()) < 1e-4, (a.item(), b.item())
    tot.backward()
    for (name, pr), (_, pd) in zip(ref.named_parameters(), dut.named_parameters()):
        gr = pr.grad if pr.grad is not None else torch.zeros_like(pr)
        gd = pd.grad.cpu() if pd.grad is not None else torch.zeros_like(pr)
        err = (gd - gr).abs().max().item()
        assert err <= 2e-3 * (gr.abs().max().item() + 1e-12) + 1e-6, f"{name}: max err {err}"
    gw = item_tower.item_matrix.weight.grad.cpu()
    assert (gw - W_ref.grad).abs().max().item() <= 2e-3 * W_ref.grad.abs().max().item() + 1e-6


@pytest.mark.parametrize("p_drop", [0.0, 0.2])
def test_native_tower_program_equals_per_op_path(gpu, p_drop):
    """rsx_tower_fwd / rsx_tower_bwd (csrc/tower.hip: the packed forward and its backward as one
    native call each) against forward_packed's per-op path (RSX_TOWER_NATIVE=0): the same kernels
    with the same arguments and dropout seeds, so the output and every gradient are bit-identical,
    with dropout too (same torch seed -> same per-op seeds)."""
    cfg = small_cfg(num_items=500, dropout=p_drop)
    items = small_universe(500)
    batch = to_dev(synth.make_batch(items, 96, seed=21), gpu)
    lookup = items.pretrained.to(gpu)
    from recsys_amd import dist as D
    ix = D.prepare_step_index(batch, pretrained_lookup=lookup)
    res = []
    for native in (True, False):
        torch.manual_seed(5)
        model = T.SASRecUserTower(cfg).to(gpu).train()
        prev = ops._TOWER_NATIVE
        ops._TOWER_NATIVE = native
        try:
            pk, pk2, tok_ids, pv, static = ix.packed
            assert (ops.tower_native_ok(model, pk2, pv) is not None) == native
            torch.manual_seed(9)
            torch.cuda.manual_seed(9)
            out = model.forward_packed(pk2, pv, tok_ids, *static)
            g = torch.Generator(device="cpu").manual_seed(3)
            w = torch.randn(out.shape, generator=g).to(gpu)
            (out * w).sum().backward()
        finally:
            ops._TOWER_NATIVE = prev
        torch.cuda.synchronize()
        res.append((out.detach(), {n: p.grad.detach().clone() for n, p in model.named_parameters()
                                   if p.grad is not None}))
    (o1, g1), (o2, g2) = res
    assert torch.equal(o1, o2)
    assert g1.keys() == g2.keys() and len(g1) > 40
    for n in g1:
        assert torch.equal(g1[n], g2[n]), n


def test_native_tower_tail_rows(gpu):
    """The tail form (forward_packed tail_last: the last layer from its attention on and the head
    on the rows the losses read: all of view 1 and view 2's "last" row per user) against the
    per-op path computing every row and keeping those (dropout 0). View 1's rows are per-row
    identical; view 2's last rows come from the fp32 single-query attention (tw_lastq_fwd_k)
    instead of the bf16x3 sequence kernel: outputs within 2e-5, gradients within 2e-5 of each
    gradient's scale (the weight-gradient sums also skip the zero rows)."""
    cfg = small_cfg(num_items=500, dropout=0.0)
    items = small_universe(500)
    batch = to_dev(synth.make_batch(items, 96, seed=23), gpu)
    lookup = items.pretrained.to(gpu)
    from recsys_amd import dist as D
    ix = D.prepare_step_index(batch, pretrained_lookup=lookup)
    pk, pk2, tok_ids, pv, static = ix.packed
    res = []
    for native in (True, False):
        torch.manual_seed(5)
        model = T.SASRecUserTower(cfg).to(gpu).train()
        prev = ops._TOWER_NATIVE
        ops._TOWER_NATIVE = native
        try:
            out = model.forward_packed(pk2, pv, tok_ids, *static, tail_last=pk.last_tok)
            assert out.shape == (pk.flat.numel() + pk.last_tok.numel(), 128)
            g = torch.Generator(device="cpu").manual_seed(3)
            w = torch.randn(out.shape, generator=g).to(gpu)
            (out * w).sum().backward()
        finally:
            ops._TOWER_NATIVE = prev
        torch.cuda.synchronize()
        res.append((out.detach(), {n: p.grad.detach().clone() for n, p in model.named_parameters()
                                   if p.grad is not None}))
    (o1, g1), (o2, g2) = res
    T1 = pk.flat.numel()
    assert torch.equal(o1[:T1], o2[:T1])           # view 1: the same kernels row for row
    torch.testing.assert_close(o1, o2, atol=2e-5, rtol=1e-4)
    assert g1.keys() == g2.keys()
    for n in g1:
        scale = float(g2[n].abs().max()) + 1e-30
        assert (g1[n] - g2[n]).abs().max().item() <= 2e-5 * scale, n


def test_native_tower_tail_rows_dropout(gpu):
    """Tail form at p = 0.2 (the headline step's setting): view 1's rows are keyed exactly as in the
    per-op all-rows program (attention by packed row, per-row ops by row index < T/2), so they are
    bit-identical to it; view 2's last query rows key their attention mask by their packed row as
    well (it used the user index, i.e. view 1's token masks), while the last layer's
    per-row ops past the attention key view 2's kept rows by their tail index (a different draw than
    the all-rows program, not shared with any view-1 row), so those rows are only checked to be
    finite and dropout-perturbed."""
    cfg = small_cfg(num_items=500, dropout=0.2)
    items = small_universe(500)
    batch = to_dev(synth.make_batch(items, 96, seed=23), gpu)
    lookup = items.pretrained.to(gpu)
    from recsys_amd import dist as D
    ix = D.prepare_step_index(batch, pretrained_lookup=lookup)
    pk, pk2, tok_ids, pv, static = ix.packed
    outs = []
    for native in (True, False):
        torch.manual_seed(5)
        model = T.SASRecUserTower(cfg).to(gpu).train()
        prev = ops._TOWER_NATIVE
        ops._TOWER_NATIVE = native
        try:
            outs.append(model.forward_packed(pk2, pv, tok_ids, *static, tail_last=pk.last_tok).detach())
        finally:
            ops._TOWER_NATIVE = prev
    torch.cuda.synchronize()
    o1, o2 = outs
    T1 = pk.flat.numel()
    assert torch.equal(o1[:T1], o2[:T1])
    assert torch.isfinite(o1).all()
    assert (o1[T1:] - o2[T1:]).abs().max().item() > 1e-3   # different (independent) post-attention masks
