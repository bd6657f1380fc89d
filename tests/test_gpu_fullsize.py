"""Parity at BASELINE.json's full sizes (configs[1] / the metric's batch 8192, and configs[2]).

* The grouped LogQ loss (rsx_nce_grouped_*, the step's dominant kernels) on the real synthetic
  batch of 4096 / 8192 users (N = 76.8k / 153k valid rows, D = 16.4k / 24.4k distinct targets,
  so the column-split and XCD-remap branches run), in both precisions, against the reference
  formulation inbatch_corrected_logq_loss (v1_refine_usertower.py:826-861: ungrouped N x N logits,
  -inf same-item / same-user mask off the diagonal, CE): the oracle's row-chunked form evaluated in
  float64 (on the device, torch's own kernels, for the whole-batch loss and both gradients) and
  the plain CPU float64 evaluation of >= 1,024 sampled rows (loss gradient of each sampled row).
* DeepFM (configs[2]): 65,536 rows x 39 fields at vocab 1e6 per field (2.5 GB of tables, ids up
  to vocab - 1), sampled rows against oracle/deepfm.py in float64.
"""
import pytest
import torch
import torch.nn.functional as F

import recsys_amd  # noqa: F401
from recsys_amd import ops, synth
from oracle import deepfm as OD
from oracle import user_tower as O

pytestmark = pytest.mark.gpu

_ITEMS = {}


def _universe():
    if "u" not in _ITEMS:
        _ITEMS["u"] = synth.make_items(num_items=47_062, d=128, seed=0)
    return _ITEMS["u"]


def _cpu_rows_f64(U, Wn, t, uid, lq, rows, tau=0.1):
    """Reference row losses and row gradients (float64, CPU) of the sampled rows: row i's term of
    inbatch_corrected_logq_loss over ALL N columns, and d(row loss)/d u_i."""
    cols = Wn[t]                                   # [N, 128]
    bias = lq[t]
    out_l, out_g = [], []
    for r0 in range(0, rows.numel(), 256):
        r = rows[r0:r0 + 256]
        u = U[r]
        s = u @ cols.T / tau - bias.view(1, -1)
        mask = (t[r].unsqueeze(1) == t.unsqueeze(0)) | (uid[r].unsqueeze(1) == uid.unsqueeze(0))
        mask[torch.arange(r.numel()), r] = False
        s.masked_fill_(mask, float("-inf"))
        lse = torch.logsumexp(s, dim=1)
        out_l.append(lse - s[torch.arange(r.numel()), r])
        p = torch.exp(s - lse.unsqueeze(1))
        out_g.append((p @ cols - cols[r]) / tau)
    return torch.cat(out_l), torch.cat(out_g)


@pytest.mark.parametrize("B", [4096, 8192])
@pytest.mark.parametrize("precision", ["fp32", "bf16x3", "f16"])
def test_grouped_logq_loss_full_size(gpu, B, precision):
    items = _universe()
    batch = synth.make_batch(items, B, seed=100)
    valid = ~batch["padding_mask"]
    t = batch["target_ids"][valid]
    uid = torch.arange(B).unsqueeze(1).expand(-1, valid.shape[1])[valid]
    N = t.numel()
    g = torch.Generator().manual_seed(B)
    U = F.normalize(torch.randn(N, 128, generator=g), dim=1)
    Wn = F.normalize(items.pretrained, dim=1)
    lq = items.log_q

    # the HIP path (as the step calls it)
    Ud = U.to(gpu).requires_grad_()
    groups = ops.TargetGroups(t.to(gpu), uid.to(gpu))
    assert groups.n_cols > 10_000
    items_d = Wn.to(gpu)[groups.uniq].clone().requires_grad_()
    bias = lq.to(gpu)[groups.uniq]
    s, cnt = ops.nce_grouped_sum(Ud, items_d, bias, groups, tau=0.1, tag="fullsize", precision=precision)
    loss = s / cnt
    loss.backward()
    assert int(cnt.item()) == N

    # whole-batch reference: the oracle's row-chunked reference formula in float64 (device-side)
    U64 = U.double().to(gpu).requires_grad_()
    W64 = Wn.double().to(gpu).requires_grad_()
    ref = O.inbatch_corrected_logq_loss_chunked(U64, W64, t.to(gpu), uid.to(gpu), lq.double().to(gpu),
                                                chunk=2048)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-4, (loss.item(), ref.item())
    gu_ref = U64.grad
    scale_u = gu_ref.abs().max().item()
    err_u = (Ud.grad.double() - gu_ref).abs().max().item()
    assert err_u <= 1e-3 * scale_u, (err_u, scale_u)
    gw_ref = W64.grad[groups.uniq]
    scale_w = gw_ref.abs().max().item()
    err_w = (items_d.grad.double() - gw_ref).abs().max().item()
    assert err_w <= 1e-3 * scale_w, (err_w, scale_w)
    del U64, W64, gu_ref, gw_ref, ref
    torch.cuda.empty_cache()

    # plain CPU float64 evaluation of 1,024 sampled rows (first / last rows included)
    rows = torch.cat([torch.tensor([0, 1, N - 2, N - 1]),
                      torch.randperm(N, generator=g)[:1020]]).unique()
    l_cpu, g_cpu = _cpu_rows_f64(U.double(), Wn.double(), t, uid, lq.double(), rows)
    assert torch.isfinite(l_cpu).all()
    g_dut = Ud.grad.detach().cpu().double()[rows] * N        # d(row loss)/du_i = N * dLoss/du_i
    err = (g_dut - g_cpu).abs().max().item()
    assert err <= 1e-3 * g_cpu.abs().max().item(), err


@pytest.mark.parametrize("precision", ["fp32", "bf16x3", "f16"])
def test_grouped_logq_loss_near_converged(gpu, precision):
    """The cancellation case of the row gradient: every user step u_i close to its
    own target's item vector, so row i's softmax puts >= 0.9 of its mass on its label column and
    dL/du_i = (sum_d p_id B_d - B_d(i)) / tau is a small difference of two near-equal vectors (the
    reduced-precision gradient products' worst case). 2,048 users of the synthetic batch, tau 0.07
    and no logQ term (with the LogQ correction the rare negatives' -logQ boost keeps p_pos low on
    this data); float64 oracle (the chunked reference formula); loss 1e-4, both gradients 1e-3 of
    their scale."""
    items = _universe()
    B, tau = 2048, 0.07
    batch = synth.make_batch(items, B, seed=400)
    valid = ~batch["padding_mask"]
    t = batch["target_ids"][valid]
    uid = torch.arange(B).unsqueeze(1).expand(-1, valid.shape[1])[valid]
    N = t.numel()
    g = torch.Generator().manual_seed(7)
    Wn = F.normalize(items.pretrained, dim=1)
    U = F.normalize(Wn[t] + 0.01 * torch.randn(N, 128, generator=g), dim=1)
    lq = torch.zeros_like(items.log_q)
    U64 = U.double().to(gpu).requires_grad_()
    W64 = Wn.double().to(gpu).requires_grad_()
    ref = O.inbatch_corrected_logq_loss_chunked(U64, W64, t.to(gpu), uid.to(gpu), lq.double().to(gpu),
                                                temperature=tau, chunk=2048)
    ref.backward()
    # the regime under test: p_pos >= 1 - |g_i| tau / 2 (|sum_d p_d (B_d - B_pos)| <= 2 (1 - p_pos))
    with torch.no_grad():
        rows = torch.arange(0, N, 97)
        _, gr = _cpu_rows_f64(U.double(), Wn.double(), t, uid, lq.double(), rows, tau=tau)
        p_pos_lb = 1.0 - gr.norm(dim=1) * tau / 2.0
    assert float(p_pos_lb.median()) > 0.9, float(p_pos_lb.median())
    groups = ops.TargetGroups(t.to(gpu), uid.to(gpu))
    Ud = U.to(gpu).requires_grad_()
    items_d = Wn.to(gpu)[groups.uniq].clone().requires_grad_()
    s, cnt = ops.nce_grouped_sum(Ud, items_d, lq.to(gpu)[groups.uniq], groups, tau=tau, tag="nearconv",
                                 precision=precision)
    loss = s / cnt
    loss.backward()
    assert abs(loss.item() - ref.item()) < 1e-4, (loss.item(), ref.item())
    gu_ref, gw_ref = U64.grad, W64.grad[groups.uniq]
    eu = (Ud.grad.double() - gu_ref).abs().max().item() / gu_ref.abs().max().item()
    ew = (items_d.grad.double() - gw_ref).abs().max().item() / gw_ref.abs().max().item()
    print(f"[near-converged {precision}] N={N} median p_pos >= {float(p_pos_lb.median()):.3f} loss {loss.item():.5f} "
          f"grad_u {eu:.2e} grad_w {ew:.2e}")
    assert eu <= 1e-3 and ew <= 1e-3, (eu, ew)


def test_grouped_logq_loss_global_batch_32768(gpu):
    """configs[3]'s global batch (32,768 users: N ~ 600k valid rows, D ~ 41.3k distinct targets)
    on one device, both precisions, against the oracle's chunked reference formula in float64 (one
    evaluation shared by both precisions; 1,024-row chunks of the N x N logits): loss 1e-4, both
    gradients 1e-3 of their scale; plus 512 sampled rows in plain CPU float64."""
    items = _universe()
    B = 32_768
    batch = synth.make_batch(items, B, seed=300)
    valid = ~batch["padding_mask"]
    t = batch["target_ids"][valid]
    uid = torch.arange(B).unsqueeze(1).expand(-1, valid.shape[1])[valid]
    N = t.numel()
    assert N > 500_000
    g = torch.Generator().manual_seed(B)
    U = F.normalize(torch.randn(N, 128, generator=g), dim=1)
    Wn = F.normalize(items.pretrained, dim=1)
    lq = items.log_q

    U64 = U.double().to(gpu).requires_grad_()
    W64 = Wn.double().to(gpu).requires_grad_()
    ref = O.inbatch_corrected_logq_loss_chunked(U64, W64, t.to(gpu), uid.to(gpu), lq.double().to(gpu), chunk=1024)
    ref.backward()
    ref_loss = ref.item()
    gu_ref = U64.grad.detach()
    del U64, ref
    torch.cuda.empty_cache()

    rows = torch.cat([torch.tensor([0, 1, N - 2, N - 1]), torch.randperm(N, generator=g)[:508]]).unique()
    l_cpu, g_cpu = _cpu_rows_f64(U.double(), Wn.double(), t, uid, lq.double(), rows)
    assert torch.isfinite(l_cpu).all()

    groups = ops.TargetGroups(t.to(gpu), uid.to(gpu))
    assert groups.n_cols > 35_000
    gw_ref = W64.grad[groups.uniq]
    for precision in ("bf16x3", "fp32", "f16"):
        Ud = U.to(gpu).requires_grad_()
        items_d = Wn.to(gpu)[groups.uniq].clone().requires_grad_()
        s, cnt = ops.nce_grouped_sum(Ud, items_d, lq.to(gpu)[groups.uniq], groups, tau=0.1, tag="fullsize",
                                     precision=precision)
        loss = s / cnt
        loss.backward()
        assert int(cnt.item()) == N
        assert abs(loss.item() - ref_loss) < 1e-4, (precision, loss.item(), ref_loss)
        err_u = (Ud.grad.double() - gu_ref).abs().max().item()
        assert err_u <= 1e-3 * gu_ref.abs().max().item(), (precision, err_u)
        err_w = (items_d.grad.double() - gw_ref).abs().max().item()
        assert err_w <= 1e-3 * gw_ref.abs().max().item(), (precision, err_w)
        g_dut = Ud.grad.detach().cpu().double()[rows] * N
        err = (g_dut - g_cpu).abs().max().item()
        assert err <= 1e-3 * g_cpu.abs().max().item(), (precision, err)
        print(f"[32768 {precision}] N={N} D={groups.n_cols} |dloss|={abs(loss.item() - ref_loss):.2e} "
              f"grad_u {err_u / gu_ref.abs().max().item():.2e} grad_w {err_w / gw_ref.abs().max().item():.2e}")
        del Ud, items_d, s, cnt, loss


def test_deepfm_full_size_vocab_1e6(gpu):
    from recsys_amd.temp_model.ranker_skelet import DeepFM
    R, Fn, V = 65_536, 39, 1_000_000
    model = DeepFM([V] * Fn, init_std=0.05, device=gpu)
    with torch.no_grad():
        model.out.bias.fill_(0.1)
        for lin in model.dnn.linears:
            lin.bias.normal_(0, 0.05)
    g = torch.Generator().manual_seed(7)
    x = torch.randint(0, V, (R, Fn), generator=g)
    x[-1] = V - 1                                  # the last table row of every field
    x[-2] = torch.arange(Fn) + (V - Fn)
    x[0] = 0
    logit, prob = model.forward_logits(x.to(gpu))
    rows = torch.cat([torch.tensor([0, 1, R - 2, R - 1]), torch.randperm(R, generator=g)[:2044]]).unique()
    # compact per-field tables of the sampled rows (gathered by torch, independent of the kernel)
    xs = x[rows]
    xd = xs.to(gpu)
    names = model.field_names
    emb = [model.embedding_dict[n].weight[xd[:, f]].cpu() for f, n in enumerate(names)]
    lin = [model.linear_model.embedding_dict[n].weight[xd[:, f]].cpu() for f, n in enumerate(names)]
    xc = torch.arange(rows.numel()).unsqueeze(1).expand(-1, Fn).contiguous()
    ref_l, ref_p = OD.deepfm_forward(xc, emb, lin, 0.1, [l.weight.cpu() for l in model.dnn.linears],
                                     [l.bias.cpu() for l in model.dnn.linears], model.dnn_linear.weight.cpu())
    torch.testing.assert_close(logit[rows.to(gpu)].cpu().double(), ref_l, atol=1e-4, rtol=1e-5)
    torch.testing.assert_close(prob[rows.to(gpu)].cpu().double(), ref_p, atol=1e-5, rtol=1e-5)
