"""rsx_static_profile_fwd / _bwd (ops.static_profile) against a plain PyTorch fp32 restatement of
the user tower's phase 2 (tower_code/v1_refine_usertower.py:472-494) on the same module weights:
sigmoid(static_gate), nine gated embeddings (padding_idx 0), relu(cont_proj(cont)) * u_g[9],
static_mlp = Linear(100 -> 128) + LayerNorm + GELU + Dropout.

Tolerance: the MLP GEMM and its gradients run as bf16x3 (~2^-17 relative per product), the rest
in fp32: output atol 2e-5, gradients 1e-4 relative to their scale. Dropout (p > 0) is checked
against the same restatement with the kernel's keep-mask read off the output."""
import pytest
import torch
import torch.nn.functional as F

from recsys_amd import ops
from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
from recsys_amd.tower_code.v1_usertower_train import PipelineConfig

pytestmark = pytest.mark.gpu


def _model(seed=0):
    torch.manual_seed(seed)
    cfg = PipelineConfig(num_items=100, num_prod_types=50, num_colors=50, num_graphics=50, num_sections=50)
    m = SASRecUserTower(cfg).cuda()
    with torch.no_grad():   # non-trivial gates and biases
        m.static_gate.copy_(torch.randn(10) * 0.5)
        m.cont_proj.bias.copy_(torch.randn(16) * 0.1)
        m.static_mlp[0].bias.copy_(torch.randn(128) * 0.1)
        m.static_mlp[1].weight.copy_(1 + 0.1 * torch.randn(128))
        m.static_mlp[1].bias.copy_(0.1 * torch.randn(128))
    return m


def _inputs(U, seed=1):
    g = torch.Generator().manual_seed(seed)
    rows = [11, 11, 11, 11, 4, 4, 3, 3, 3]
    ids = [torch.randint(0, r, (U,), generator=g).cuda() for r in rows]
    cont = torch.randn(U, 4, generator=g).cuda()
    return ids, cont


def _reference(m, ids, cont, mask=None, scale=1.0):
    embs = [m.age_emb, m.price_emb, m.cnt_emb, m.recency_emb, m.channel_emb, m.club_status_emb, m.news_freq_emb,
            m.fn_emb, m.active_emb]
    u_g = torch.sigmoid(m.static_gate)
    parts = [F.embedding(i, e.weight, padding_idx=0) * u_g[j] for j, (i, e) in enumerate(zip(ids, embs))]
    parts.append(F.relu(m.cont_proj(cont)) * u_g[9])
    h = m.static_mlp[0](torch.cat(parts, dim=1))
    y = F.gelu(m.static_mlp[1](h))
    if mask is not None:
        y = y * mask * scale
    return y


def _grads(m):
    return {n: (p.grad.detach().clone() if p.grad is not None else None) for n, p in m.named_parameters()
            if n.split(".")[0] in ("age_emb", "price_emb", "cnt_emb", "recency_emb", "channel_emb",
                                   "club_status_emb", "news_freq_emb", "fn_emb", "active_emb", "cont_proj",
                                   "static_mlp", "static_gate")}


@pytest.mark.parametrize("U,p_drop", [(1, 0.0), (257, 0.0), (8192, 0.0), (1000, 0.3)])
def test_static_profile_matches_torch(U, p_drop):
    m = _model()
    ids, cont = _inputs(U)
    dy = torch.randn(U, 128, device="cuda")
    m.zero_grad(set_to_none=True)
    out = ops.static_profile(m, ids, cont, p_drop)
    out.backward(dy)
    g_native = _grads(m)
    mask, scale = None, 1.0
    if p_drop > 0:
        with torch.no_grad():
            y0 = _reference(m, ids, cont)
        mask = ((out != 0) | (y0 == 0)).float()
        scale = 1.0 / (1.0 - p_drop)
        kept = mask.mean().item()
        assert abs(kept - (1 - p_drop)) < 0.02, kept
    m.zero_grad(set_to_none=True)
    ref = _reference(m, ids, cont, mask, scale)
    ref.backward(dy)
    g_ref = _grads(m)
    torch.testing.assert_close(out, ref.detach(), atol=2e-5, rtol=1e-4)
    assert set(g_native) == set(g_ref)
    for n in g_ref:
        a, b = g_native[n], g_ref[n]
        assert a is not None and b is not None, n
        tol = 1e-4 * max(float(b.abs().max()), 1e-6) + 1e-7
        assert (a - b).abs().max().item() <= tol, (n, (a - b).abs().max().item(), tol)
    # padding rows get exactly no gradient
    assert torch.count_nonzero(g_native["age_emb.weight"][0]) == 0


def test_static_profile_deterministic_and_eval():
    m = _model(3)
    ids, cont = _inputs(4096, seed=5)
    outs, grads = [], []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        o = ops.static_profile(m, ids, cont, 0.0)
        o.square().sum().backward()
        outs.append(o.detach())
        grads.append(_grads(m))
    assert torch.equal(outs[0], outs[1])
    for n in grads[0]:
        assert torch.equal(grads[0][n], grads[1][n]), n
    with torch.no_grad():
        assert torch.equal(ops.static_profile(m, ids, cont, 0.0), outs[0])


def test_static_profile_shared_rows_equal_doubled_inputs():
    """rows = 2B (the contrastive step's two dropout views read the same B users): identical to
    the program run on the explicitly doubled inputs, output and every gradient (dropout 0)."""
    m = _model(4)
    ids, cont = _inputs(300, seed=7)
    dy = torch.randn(600, 128, device="cuda")
    res = []
    for shared in (True, False):
        m.zero_grad(set_to_none=True)
        if shared:
            o = ops.static_profile(m, ids, cont, 0.0, rows=600)
        else:
            o = ops.static_profile(m, [torch.cat([i, i]) for i in ids], torch.cat([cont, cont]), 0.0)
        o.backward(dy)
        res.append((o.detach(), _grads(m)))
    assert torch.equal(res[0][0], res[1][0])
    for n in res[0][1]:
        assert torch.equal(res[0][1][n], res[1][1][n]), n


def test_static_profile_out_of_range_id_raises_and_stays_in_bounds():
    """An id outside its table (nn.Embedding raises IndexError, v1_refine_usertower.py:472-481): the
    kernel reads and scatters row 0 instead (no out-of-bounds access) and the flag it sets in the
    arena is raised as IndexError at the guard's check; an in-place change of a saved parameter
    between forward and backward is caught by autograd's version check."""
    m = _model()
    ids, cont = _inputs(64)
    ops._STATIC_IDS.check()
    bad = [t.clone() for t in ids]
    bad[4][7] = 4          # channel table has 4 rows
    bad[0][3] = -1
    before = [e.weight.detach().clone() for e in (m.age_emb, m.channel_emb)]
    out = ops.static_profile(m, bad, cont, 0.0)
    out.sum().backward()
    torch.cuda.synchronize()
    with pytest.raises(IndexError, match="out of range"):
        ops._STATIC_IDS.check()
    assert torch.isfinite(out).all()
    assert torch.equal(before[0], m.age_emb.weight) and torch.equal(before[1], m.channel_emb.weight)
    ops._STATIC_IDS.check()  # cleared: in-range ids pass again
    out = ops.static_profile(m, ids, cont, 0.0)
    with torch.no_grad():
        m.static_mlp[0].weight.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified by an inplace operation"):
        out.sum().backward()
    ops._STATIC_IDS.check()
