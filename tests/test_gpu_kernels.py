"""Kernel-level parity: librecsys_amd.so (cuda:0) vs the CPU oracle / float64 restatements.

Tolerances (fp32 kernels vs CPU): gathers bit-exact; LayerNorm outputs 1e-6 abs;
logits / losses 1e-4 abs (north-star bound: fp32 logits within 1e-4); gradients 1e-5 abs
+ 1e-4 rel unless stated.
"""
import math

import pytest
import torch
import torch.nn.functional as F

import recsys_amd  # noqa: F401
from recsys_amd import ops

pytestmark = pytest.mark.gpu


# ------------------------------------------------------------------ seq embed (A2)
def _embed_inputs(B=37, L=50, D=128, rows=(301, 12, 51, 51, 51, 51), seed=0):
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(B, L, D, generator=g)
    tables = [torch.randn(r, D, generator=g) * 0.02 for r in rows]
    ids = [torch.randint(0, r, (B, L), generator=g) for r in rows]
    pad = torch.rand(B, L, generator=g) < 0.4
    for t in ids:
        t[pad] = 0
    gate = torch.sigmoid(torch.randn(6, generator=g)) * torch.tensor([1.0, 1.0, 0.0, 0.0, 0.0, 0.0])
    pos = torch.randn(L, D, generator=g) * 0.02
    lw = 1 + 0.1 * torch.randn(D, generator=g)
    lb = 0.1 * torch.randn(D, generator=g)
    return base, tables, ids, gate, pos, lw, lb


def _embed_ref(base, tables, ids, gate, pos):
    x = base.clone()
    for t, i, gj in zip(tables, ids, gate):
        x += t[i] * gj           # same op order as v1_refine_usertower.py:447-453
    x += pos.unsqueeze(0)
    return x


def test_seq_embed_gather_bit_exact(gpu):
    base, tables, ids, gate, pos, lw, lb = _embed_inputs()
    ref = _embed_ref(base, tables, ids, gate, pos)
    d = lambda t: t.to(gpu)
    out = ops.seq_embed(d(base), [d(i) for i in ids], [d(t) for t in tables], d(gate), d(pos), None, None)
    assert torch.equal(out.cpu(), ref), (out.cpu() - ref).abs().max()


@pytest.mark.parametrize("seg", [False, True])
def test_seq_embed_layernorm_and_backward(gpu, seg):
    """Forward (atol 2e-6) and every gradient (atol 2e-5 / rtol 1e-4) vs float64; seg=True
    takes table 0's gradient from the sorted segmented sums (rsx_segment_sum_rows)."""
    base, tables, ids, gate, pos, lw, lb = _embed_inputs(seed=1)
    leaves = [t.clone().double().requires_grad_() for t in [base, *tables, gate, pos, lw, lb]]
    b64, t64, g64, p64, w64, bb64 = leaves[0], leaves[1:7], leaves[7], leaves[8], leaves[9], leaves[10]
    x = b64.clone()
    for t, i, j in zip(t64, ids, range(6)):
        x = x + t[i] * g64[j]
    x = x + p64.unsqueeze(0)
    ref = F.layer_norm(x, (128,), w64, bb64, 1e-5)
    dout = torch.randn_like(ref)
    (ref * dout).sum().backward()

    dev = [t.clone().to(gpu).requires_grad_() for t in [base, *tables, gate, pos, lw, lb]]
    out = ops.seq_embed(dev[0], [i.to(gpu) for i in ids], dev[1:7], dev[7], dev[8], dev[9], dev[10],
                        eps=1e-5, padding_idx=[0] * 6,
                        tab0_seg=ops.sort_segments(ids[0].to(gpu)) if seg else None)
    torch.testing.assert_close(out.cpu().double(), ref.detach(), atol=2e-6, rtol=0)
    (out * dout.float().to(gpu)).sum().backward()
    names = ["base"] + [f"table{j}" for j in range(6)] + ["gate", "pos", "ln_w", "ln_b"]
    for name, a, r in zip(names, dev, leaves):
        gr = r.grad.clone()
        if name.startswith("table"):
            gr[0] = 0.0                            # nn.Embedding padding_idx=0: no gradient to row 0
            j = int(name[-1])
            if gate[j] == 0:
                gr.zero_()                          # zero gate (s_mask) => zero table gradient
        if name == "gate":
            gr = gr * (gate != 0)                   # masked gates: d s_g is multiplied by 0 upstream
        torch.testing.assert_close(a.grad.cpu().double(), gr, atol=2e-5, rtol=1e-4, msg=name)


@pytest.mark.parametrize("keysum", [True, False])
def test_seq_embed_backward_packed_step_shape(gpu, keysum, monkeypatch):
    """Packed layout as the step runs it (tok_pos per token, item table through the sorted
    segment sums, time table + positions through seq_embed_keysum_k's one-hot MFMA sums, or
    with keysum=False the LDS-atomic kernel): 24,576 tokens over 40 workgroups' worth of keysum
    blocks, every gradient vs float64 (atol 5e-5 / rtol 1e-4: sums over ~500-2,000 tokens per
    position / time row)."""
    if not keysum:
        monkeypatch.setenv("RSX_SEQ_EMBED_KEYSUM", "0")
    g = torch.Generator().manual_seed(11)
    T, L, D = 24576, 50, 128
    rows = (997, 12, 51, 51, 51, 51)
    base = torch.randn(T, D, generator=g)
    tables = [torch.randn(r, D, generator=g) * 0.02 for r in rows]
    ids = [torch.randint(0, r, (T,), generator=g) for r in rows]
    ids[1][torch.rand(T, generator=g) < 0.1] = 0          # time padding rows
    tok_pos = torch.randint(0, L, (T,), generator=g)
    gate = torch.sigmoid(torch.randn(6, generator=g)) * torch.tensor([1.0, 1.0, 0.0, 0.0, 0.0, 0.0])
    pos = torch.randn(L, D, generator=g) * 0.02
    lw = 1 + 0.1 * torch.randn(D, generator=g)
    lb = 0.1 * torch.randn(D, generator=g)
    leaves = [t.clone().double().requires_grad_() for t in [base, *tables, gate, pos, lw, lb]]
    b64, t64, g64, p64, w64, bb64 = leaves[0], leaves[1:7], leaves[7], leaves[8], leaves[9], leaves[10]
    x = b64.clone()
    for t, i, j in zip(t64, ids, range(6)):
        x = x + t[i] * g64[j]
    x = x + p64[tok_pos]
    ref = F.layer_norm(x, (D,), w64, bb64, 1e-5)
    dout = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    (ref * dout).sum().backward()
    dev = [t.clone().to(gpu).requires_grad_() for t in [base, *tables, gate, pos, lw, lb]]
    ids_d = [i.to(gpu) for i in ids]
    out = ops.seq_embed(dev[0], ids_d, dev[1:7], dev[7], dev[8], dev[9], dev[10], eps=1e-5,
                        padding_idx=[0] * 6, tok_pos=tok_pos.to(gpu), tab0_seg=ops.sort_segments(ids_d[0]))
    (out * dout.float().to(gpu)).sum().backward()
    names = ["base"] + [f"table{j}" for j in range(6)] + ["gate", "pos", "ln_w", "ln_b"]
    for name, a, r in zip(names, dev, leaves):
        gr = r.grad.clone()
        if name.startswith("table"):
            gr[0] = 0.0
            if gate[int(name[-1])] == 0:
                gr.zero_()
        if name == "gate":
            gr = gr * (gate != 0)
        # sums over up to 24,576 tokens: fp32 rounding of the running partial sums scales with the
        # gradient's magnitude, not with each element (an ln_b column near 0 still carries it)
        torch.testing.assert_close(a.grad.cpu().double(), gr, atol=5e-5 + 1e-5 * gr.abs().max().item(),
                                   rtol=1e-4, msg=lambda m, name=name: f"{name}: {m}")


def test_seq_embed_dropout_mask_consistent(gpu):
    base, tables, ids, gate, pos, lw, lb = _embed_inputs(seed=2)
    x = base.to(gpu).requires_grad_()
    out = ops.seq_embed(x, [i.to(gpu) for i in ids], [t.to(gpu) for t in tables], gate.to(gpu), pos.to(gpu),
                        None, None, p_drop=0.2)
    ref = _embed_ref(base, tables, ids, gate, pos).to(gpu)
    keep = out != 0
    frac = keep.float().mean().item()
    assert abs(frac - 0.8) < 0.01
    torch.testing.assert_close(out[keep], ref[keep] / 0.8, atol=1e-5, rtol=1e-5)
    out.sum().backward()
    torch.testing.assert_close(x.grad, keep.float() / 0.8)


# ------------------------------------------------------------------ MHA core (A3/A9)
def _mha_ref(qkv, pad, H, causal):
    B, L, D3 = qkv.shape
    D = D3 // 3
    dh = D // H
    q, k, v = qkv.split(D, -1)
    q = q.view(B, L, H, dh).transpose(1, 2)
    k = k.view(B, L, H, dh).transpose(1, 2)
    v = v.view(B, L, H, dh).transpose(1, 2)
    s = q @ k.transpose(-1, -2) / math.sqrt(dh)
    blocked = torch.zeros(B, L, L, dtype=torch.bool)
    if causal:
        blocked |= torch.triu(torch.ones(L, L, dtype=torch.bool), 1)
    if pad is not None:
        blocked |= pad[:, None, :]
    s = s.masked_fill(blocked[:, None], float("-inf"))
    p = torch.nan_to_num(torch.softmax(s, -1), nan=0.0)
    return (p @ v).transpose(1, 2).reshape(B, L, D)


# (output atol, gradient atol) per attention precision: fp32 kernels ~1e-6; bf16x3 adds ~3*2^-18
# relative error per product over 32-dim scores with |q||k| ~ 32 on N(0,1) inputs (score error
# ~1e-5 after the 1/sqrt(32) scale), which reaches O and the gradients as ~1e-5 relative.
_MHA_TOL = {"fp32": (2e-5, 5e-5), "bf16x3": (6e-5, 2e-4)}


@pytest.fixture(params=["bf16x3", "fp32"])
def mha_precision(request):
    prev = ops.mha_precision()
    ops.set_mha_precision(request.param)
    yield request.param
    ops.set_mha_precision(prev)


@pytest.mark.parametrize("L,H,dh,causal,use_pad", [(50, 4, 32, True, True), (16, 4, 32, False, False),
                                                   (16, 4, 16, False, False), (7, 2, 32, True, False),
                                                   (64, 4, 32, True, True), (33, 1, 32, False, True),
                                                   (50, 4, 64, True, True), (20, 2, 64, False, True),
                                                   (32, 12, 64, False, False)])
def test_mha_forward_backward(gpu, mha_precision, L, H, dh, causal, use_pad):
    g = torch.Generator().manual_seed(L * 7 + dh)
    B = 33
    qkv = torch.randn(B, L, 3 * H * dh, generator=g)
    pad = None
    if use_pad:
        lens = torch.randint(1, L + 1, (B,), generator=g)
        lens[0] = L
        pad = torch.arange(L)[None, :] < (L - lens)[:, None]  # left padding
    q64 = qkv.double().requires_grad_()
    ref = _mha_ref(q64, pad, H, causal)
    dout = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    (ref * dout).sum().backward()
    qd = qkv.to(gpu).requires_grad_()
    out = ops.mha(qd, pad.to(gpu) if pad is not None else None, H, causal)
    torch.testing.assert_close(out.cpu().double(), ref.detach(), atol=_MHA_TOL[mha_precision][0], rtol=1e-5)
    (out * dout.float().to(gpu)).sum().backward()
    torch.testing.assert_close(qd.grad.cpu().double(), q64.grad, atol=_MHA_TOL[mha_precision][1], rtol=1e-4)
    if use_pad and causal:  # left-padded query rows see no key under the causal mask: exactly zero
        assert (out[pad.to(gpu)] == 0).all()


@pytest.mark.parametrize("dh,max_len", [(32, None), (16, None), (64, None), (64, 32)])
def test_mha_packed_segments(gpu, mha_precision, dh, max_len):
    """Packed variable-length segments (seg_off, lengths 1..51 -- 1..32 with max_len 32, the head-dim-64
    backward's small-LDS instance --, a padded last key in some): outputs and dqkv equal the per-segment
    dense float64 reference (atol _MHA_TOL)."""
    g = torch.Generator().manual_seed(dh)
    H = 4
    lens = torch.randint(1, (max_len or 51) + 1, (37,), generator=g)
    seg = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(lens, 0)])
    T = int(seg[-1])
    qkv = torch.randn(T, 3 * H * dh, generator=g)
    pad = torch.zeros(T, dtype=torch.bool)
    pad[seg[1:] - 1] = torch.rand(len(lens), generator=g) < 0.3  # some segments end on a padded key
    q64 = qkv.double().requires_grad_()
    outs = []
    for b in range(len(lens)):
        s0, s1 = int(seg[b]), int(seg[b + 1])
        outs.append(_mha_ref(q64[s0:s1][None], pad[s0:s1][None], H, True)[0])
    ref = torch.cat(outs)
    dout = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    (ref * dout).sum().backward()
    qd = qkv.to(gpu).requires_grad_()
    out = ops.mha(qd, pad.to(gpu), H, True, seg_off=seg.to(gpu), max_len=max_len)
    torch.testing.assert_close(out.cpu().double(), ref.detach(), atol=_MHA_TOL[mha_precision][0], rtol=1e-5)
    (out * dout.float().to(gpu)).sum().backward()
    torch.testing.assert_close(qd.grad.cpu().double(), q64.grad, atol=_MHA_TOL[mha_precision][1], rtol=1e-4)


@pytest.mark.parametrize("L,H,causal,use_pad,packed", [(50, 4, True, True, False), (64, 2, True, True, False),
                                                       (64, 4, False, False, False), (33, 3, False, True, False),
                                                       (64, 4, True, True, True), (64, 12, False, False, True)])
def test_mha_head_dim_64_forward(gpu, mha_precision, L, H, causal, use_pad, packed):
    """Head dim 64 (BERT's 768 / 12; forward only — the x3 kernel mha_fwd_x3b64_k under bf16x3,
    mha_fwd_k<64> under fp32): dense [B, L] with left padding / causal, and packed segments of
    1..64 tokens (bert_packed_ok allows up to 64: NB = 3 / 4 query blocks), against the float64
    reference at the bf16x3 tolerance."""
    g = torch.Generator().manual_seed(L * 13 + H)
    dh = 64
    if packed:
        lens = torch.randint(1, L + 1, (29,), generator=g)
        lens[:3] = torch.tensor([L, 1, 33])
        seg = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(lens, 0)])
        qkv = torch.randn(int(seg[-1]), 3 * H * dh, generator=g)
        pad = torch.zeros(qkv.shape[0], dtype=torch.bool)
        if use_pad:
            pad[seg[1:] - 1] = torch.rand(len(lens), generator=g) < 0.3
        ref = torch.cat([_mha_ref(qkv.double()[int(seg[b]):int(seg[b + 1])][None],
                                  pad[int(seg[b]):int(seg[b + 1])][None], H, causal)[0] for b in range(len(lens))])
        out = ops.mha(qkv.to(gpu), pad.to(gpu) if use_pad else None, H, causal, seg_off=seg.to(gpu))
    else:
        B = 21
        qkv = torch.randn(B, L, 3 * H * dh, generator=g)
        pad = None
        if use_pad:
            lens = torch.randint(1, L + 1, (B,), generator=g)
            lens[0] = L
            pad = torch.arange(L)[None, :] < (L - lens)[:, None]
        ref = _mha_ref(qkv.double(), pad, H, causal)
        out = ops.mha(qkv.to(gpu), pad.to(gpu) if pad is not None else None, H, causal)
        if use_pad and causal:
            assert (out[pad.to(gpu)] == 0).all()
    # 64-dim scores have twice the terms of the 32-dim case: same per-product bound, 2x atol
    torch.testing.assert_close(out.cpu().double(), ref, atol=2 * _MHA_TOL[mha_precision][0], rtol=1e-5)


def test_mha_head_dim_64_dropout_matches_fp32(gpu):
    """Head dim 64 with dropout: the bf16x3 forward draws the fp32 kernel's keep mask (same hash
    index), so the outputs agree to the bf16x3 tolerance; about 20 % of probabilities dropped."""
    g = torch.Generator().manual_seed(64)
    B, L, H, dh = 12, 64, 4, 64
    qkv = torch.randn(B, L, 3 * H * dh, generator=g).to(gpu)
    pad = (torch.arange(L)[None, :] < torch.randint(0, L, (B,), generator=g)[:, None]).to(gpu)
    res = {}
    prev = ops.mha_precision()
    try:
        for p in ("fp32", "bf16x3"):
            ops.set_mha_precision(p)
            with torch.no_grad():
                res[p] = ops._MHA.apply(qkv, pad, None, H, True, 0.2, 4242)
                res[p + "_nodrop"] = ops._MHA.apply(qkv, pad, None, H, True, 0.0, 0)
    finally:
        ops.set_mha_precision(prev)
    torch.testing.assert_close(res["bf16x3"], res["fp32"], atol=2 * _MHA_TOL["bf16x3"][0], rtol=1e-5)
    assert not torch.equal(res["fp32"], res["fp32_nodrop"])


def test_mha_precisions_share_dropout_mask(gpu):
    """With dropout the bf16x3 and fp32 kernels draw the same keep mask (same hash index), so
    outputs and gradients agree to the bf16x3 tolerance (_MHA_TOL)."""
    g = torch.Generator().manual_seed(9)
    B, L, H, dh = 16, 50, 4, 32
    qkv = torch.randn(B, L, 3 * H * dh, generator=g).to(gpu)
    pad = (torch.arange(L)[None, :] < torch.randint(0, L, (B,), generator=g)[:, None]).to(gpu)
    w = torch.randn(B, L, H * dh, generator=g).to(gpu)
    res = {}
    prev = ops.mha_precision()
    try:
        for p in ("fp32", "bf16x3"):
            ops.set_mha_precision(p)
            x = qkv.clone().requires_grad_()
            out = ops._MHA.apply(x, pad, None, H, True, 0.2, 777)
            (out * w).sum().backward()
            res[p] = (out.detach(), x.grad)
    finally:
        ops.set_mha_precision(prev)
    torch.testing.assert_close(res["bf16x3"][0], res["fp32"][0], atol=_MHA_TOL["bf16x3"][0], rtol=1e-5)
    torch.testing.assert_close(res["bf16x3"][1], res["fp32"][1], atol=_MHA_TOL["bf16x3"][1], rtol=1e-4)


def test_mha_dropout_directional_derivative(gpu, mha_precision):
    g = torch.Generator().manual_seed(5)
    B, L, H, dh = 8, 50, 4, 32
    qkv = torch.randn(B, L, 3 * H * dh, generator=g).to(gpu)
    pad = (torch.arange(L)[None, :] < torch.randint(0, L, (B,), generator=g)[:, None]).to(gpu)
    v = torch.randn_like(qkv)
    w = torch.randn(B, L, H * dh, device=gpu)
    f = lambda x: (ops._MHA.apply(x, pad, None, H, True, 0.2, 1234) * w).sum()
    x = qkv.clone().requires_grad_()
    f(x).backward()
    eps = 1e-2
    num = (f(qkv.double().float() + eps * v) - f(qkv - eps * v)) / (2 * eps)
    ana = (x.grad * v).sum()
    assert abs(num.item() - ana.item()) < 2e-2 * max(1.0, abs(ana.item()))


# ------------------------------------------------------------------ fused InfoNCE (A6/A7/A12)
def _nce_ref(A, B, bias, k1a, k1b, k2a, k2b, tau, flags):
    S = A @ B.T / tau
    if bias is not None:
        S = S - bias[None, :]
    n, m = S.shape
    idx_i = torch.arange(n)[:, None]
    idx_j = torch.arange(m)[None, :]
    off = idx_i != idx_j
    excl = torch.zeros(n, m, dtype=torch.bool)
    if flags & 1:
        excl |= ~off
    if flags & 2:
        excl |= off & (k1a[:, None] == k1b[None, :])
    if flags & 4:
        excl |= off & (k2a[:, None] == k2b[None, :])
    Sm = S.masked_fill(excl, float("-inf"))
    lse = torch.logsumexp(Sm, 1)
    if flags & 8:
        pos = off & (k1a[:, None] == k1b[None, :]) & (k1a[:, None] != 0) & ~excl
        cnt = pos.sum(1)
        valid = cnt > 0
        if valid.sum() == 0:
            return (S * 0).sum()
        psum = (S * pos).sum(1)
        return (lse - psum / cnt.clamp(min=1))[valid].mean()
    return (lse - S.diagonal()).mean()


@pytest.fixture(params=["bf16x3", "fp32"])
def nce_precision(request):
    prev = ops.nce_precision()
    ops.set_nce_precision(request.param)
    yield request.param
    ops.set_nce_precision(prev)


@pytest.mark.parametrize("flags", [0, 2, 6, 9])
@pytest.mark.parametrize("n", [1, 77, 300, 1029, 5000])
def test_nce_forward_backward(gpu, nce_precision, flags, n):
    """Plain InfoNCE (DuoRec unsup / sup, SimCSE; both precisions) vs float64: loss within
    1e-4, gradients atol 2e-6 / rtol 1e-4 (the bf16x3 logit error ~3e-6 / tau stays inside)."""
    g = torch.Generator().manual_seed(n * 13 + flags)
    A = F.normalize(torch.randn(n, 128, generator=g), dim=1)
    B = F.normalize(torch.randn(n, 128, generator=g), dim=1)
    if flags == 9:
        B = A.clone()
    bias = torch.log_softmax(torch.randn(n, generator=g), 0) if flags in (2, 6) else None
    k1 = torch.randint(0, max(2, n // 3), (n,), generator=g)
    k2 = torch.randint(0, max(2, n // 20), (n,), generator=g)
    tau = 0.1
    A64 = A.double().requires_grad_()
    B64 = (A64 if flags == 9 else B.double().requires_grad_())
    ref = _nce_ref(A64, B64, bias.double() if bias is not None else None, k1, k1, k2, k2, tau, flags)
    ref.backward()
    Ad = A.to(gpu).requires_grad_()
    Bd = Ad if flags == 9 else B.to(gpu).requires_grad_()
    dev = lambda t: None if t is None else t.to(gpu)
    loss = ops.nce_loss(Ad, Bd, dev(bias), dev(k1), dev(k1), dev(k2), dev(k2), tau=tau, flags=flags)
    assert abs(loss.item() - ref.item()) < 1e-4, (loss.item(), ref.item())
    loss.backward()
    torch.testing.assert_close(Ad.grad.cpu().double(), A64.grad, atol=2e-6, rtol=1e-4)
    if flags != 9:
        torch.testing.assert_close(Bd.grad.cpu().double(), B64.grad, atol=2e-6, rtol=1e-4)


def test_nce_grad_scales_with_upstream(gpu):
    g = torch.Generator().manual_seed(0)
    A = F.normalize(torch.randn(200, 128, generator=g), dim=1).to(gpu).requires_grad_()
    B = F.normalize(torch.randn(200, 128, generator=g), dim=1).to(gpu)
    l = ops.nce_loss(A, B, tau=0.1)
    (3.0 * l).backward()
    ga = A.grad.clone()
    A.grad = None
    ops.nce_loss(A, B, tau=0.1).backward()
    torch.testing.assert_close(ga, 3.0 * A.grad)


# ------------------------------------------------------------------ rows
def test_gather_normalize_and_scatter(gpu):
    g = torch.Generator().manual_seed(0)
    W = torch.randn(1000, 128, generator=g)
    W[7] = 0.0  # zero row: F.normalize eps branch
    idx = torch.randint(0, 1000, (3000,), generator=g)
    idx[:5] = 7
    W64 = W.double().requires_grad_()
    ref = F.normalize(W64, p=2, dim=1)[idx]
    dy = torch.randn(ref.shape, generator=g, dtype=torch.float64)
    (ref * dy).sum().backward()
    Wd = W.to(gpu).requires_grad_()
    out = ops.gather_rows(Wd, idx.to(gpu), normalize=True)
    torch.testing.assert_close(out.cpu().double(), ref.detach(), atol=1e-7, rtol=1e-6)
    (out * dy.float().to(gpu)).sum().backward()
    torch.testing.assert_close(Wd.grad.cpu().double(), W64.grad, atol=1e-5, rtol=1e-5)
    plain = ops.gather_rows(Wd, idx.to(gpu))
    assert torch.equal(plain.detach().cpu(), W[idx])


def _nce_rows_ref(A, B, bias, k1a, k1b, k2a, k2b, tau, flags, off):
    """Per-row losses (and validity) with row i's label at column i + off (float64)."""
    S = A @ B.T / tau
    if bias is not None:
        S = S - bias[None, :]
    n, m = S.shape
    lab = torch.arange(n)[:, None] + off
    off_d = torch.arange(m)[None, :] != lab
    excl = torch.zeros(n, m, dtype=torch.bool)
    if flags & 1:
        excl |= ~off_d
    if flags & 2:
        excl |= off_d & (k1a[:, None] == k1b[None, :])
    if flags & 4:
        excl |= off_d & (k2a[:, None] == k2b[None, :])
    lse = torch.logsumexp(S.masked_fill(excl, float("-inf")), 1)
    if flags & 8:
        pos = off_d & (k1a[:, None] == k1b[None, :]) & (k1a[:, None] != 0) & ~excl
        cnt = pos.sum(1)
        valid = cnt > 0
        loss = torch.where(valid, lse - (S * pos).sum(1) / cnt.clamp(min=1), torch.zeros_like(lse))
        return loss, valid
    return lse - S.gather(1, lab).squeeze(1), torch.ones(n, dtype=torch.bool)


@pytest.mark.parametrize("flags", [0, 6, 9])
def test_nce_diag_offset_shards(gpu, flags):
    """Rows [lo, hi) against all columns with diag_offset=lo reproduce those rows of the
    single-device problem: the per-rank computation of the data-parallel step."""
    g = torch.Generator().manual_seed(flags + 100)
    n = 611
    A = F.normalize(torch.randn(n, 128, generator=g), dim=1)
    B = A.clone() if flags == 9 else F.normalize(torch.randn(n, 128, generator=g), dim=1)
    bias = torch.log_softmax(torch.randn(n, generator=g), 0) if flags == 6 else None
    k1 = torch.randint(0, 150, (n,), generator=g)
    k2 = torch.randint(0, 40, (n,), generator=g)
    dev = lambda t: None if t is None else t.to(gpu)
    for lo, hi in [(0, 130), (130, 371), (371, 611)]:
        ref, valid = _nce_rows_ref(A[lo:hi].double(), B.double(), None if bias is None else bias.double(),
                                   k1[lo:hi], k1, k2[lo:hi], k2, 0.1, flags, lo)
        s, c = ops.nce_sum(dev(A[lo:hi]), dev(B), dev(bias), dev(k1[lo:hi]), dev(k1), dev(k2[lo:hi]), dev(k2),
                           tau=0.1, flags=flags, diag_offset=lo)
        assert abs(s.item() - ref.sum().item()) < 1e-3, (lo, s.item(), ref.sum().item())
        assert c.item() == valid.sum().item()


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
@pytest.mark.parametrize("n_users,max_len,n_items,seed", [(40, 30, 25, 0), (300, 50, 400, 1), (7, 3, 5, 2)])
def test_nce_grouped_equals_plain(gpu, n_users, max_len, n_items, seed, precision):
    """Grouped (distinct-target columns, exact multiplicities) == the plain N x N kernel with
    same-item + same-user masks, loss and both gradients (through the column gather).
    Tolerance: loss 1e-3 relative to max(1, |loss sum|); grads rtol 1e-4 + atol 1e-6 (fp32) or
    atol 1e-4 * max|grad| (bf16x3: every product term carries ~1e-5 relative error, so small
    entries that are sums of cancelling terms are only accurate relative to the row scale)."""
    g = torch.Generator().manual_seed(seed)
    lens = torch.randint(1, max_len + 1, (n_users,), generator=g)
    users = torch.repeat_interleave(torch.arange(n_users), lens)
    n = users.numel()
    t = torch.randint(1, n_items + 1, (n,), generator=g)
    W = torch.randn(n_items + 1, 128, generator=g)
    lq = torch.log_softmax(torch.randn(n_items + 1, generator=g), 0)
    U = F.normalize(torch.randn(n, 128, generator=g), dim=1)
    d = lambda x: x.to(gpu)
    # plain: columns = normalize(W)[t]
    U1 = d(U).requires_grad_()
    W1 = d(W).requires_grad_()
    cols = ops.gather_rows(W1, d(t), normalize=True)
    prev = ops.nce_precision()
    ops.set_nce_precision(precision)
    try:
        s1, c1 = ops.nce_sum(U1, cols, d(lq)[d(t)], d(t), d(t), d(users), d(users), tau=0.1, flags=6)
        (s1 / c1).backward()
    finally:
        ops.set_nce_precision(prev)
    # grouped
    U2 = d(U).requires_grad_()
    W2 = d(W).requires_grad_()
    grp = ops.TargetGroups(d(t), d(users))
    items_d = ops.gather_rows(W2, grp.uniq, normalize=True, unique=True)
    s2, c2 = ops.nce_grouped_sum(U2, items_d, d(lq)[grp.uniq], grp, tau=0.1, precision=precision)
    (s2 / c2).backward()
    assert c1.item() == c2.item() == n
    assert abs(s1.item() - s2.item()) < 1e-3 * max(1.0, abs(s1.item())), (s1.item(), s2.item())
    for g2, g1 in ((U2.grad, U1.grad), (W2.grad, W1.grad)):
        atol = 1e-6 if precision == "fp32" else max(1e-6, 1e-4 * g1.abs().max().item())
        torch.testing.assert_close(g2, g1, atol=atol, rtol=1e-4)


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
def test_nce_grouped_sharded_rows(gpu, precision):
    """Rows of one shard against the distinct targets of all shards (the data-parallel form),
    against a float64 restatement: |shard loss sum error| < 1e-3."""
    g = torch.Generator().manual_seed(9)
    n_users, n_items = 120, 60
    lens = torch.randint(1, 40, (n_users,), generator=g)
    users = torch.repeat_interleave(torch.arange(n_users), lens)
    n = users.numel()
    t = torch.randint(1, n_items + 1, (n,), generator=g)
    W = F.normalize(torch.randn(n_items + 1, 128, generator=g), dim=1)
    lq = torch.log_softmax(torch.randn(n_items + 1, generator=g), 0)
    U = F.normalize(torch.randn(n, 128, generator=g), dim=1)
    d = lambda x: x.to(gpu)
    ref, _ = _nce_rows_ref(U.double(), W[t].double(), lq[t].double(), t, t, users, users, 0.1, 6, 0)
    cut = int(torch.nonzero(users == 50)[0])  # shard boundary on a user boundary
    tot = 0.0
    for lo, hi in [(0, cut), (cut, n)]:
        grp = ops.TargetGroups(d(t[lo:hi]), d(users[lo:hi]), t_cols=d(t))
        s, c = ops.nce_grouped_sum(d(U[lo:hi]), d(W)[grp.uniq], d(lq)[grp.uniq], grp, tau=0.1,
                                   precision=precision)
        assert abs(s.item() - ref[lo:hi].sum().item()) < 1e-3
        tot += s.item()
    assert abs(tot - ref.sum().item()) < 2e-3


@pytest.fixture(params=["bf16x3", "fp32"])
def gemm_precision(request):
    prev = ops._gemm_precision
    ops.set_gemm_precision(request.param)
    yield request.param
    ops.set_gemm_precision(prev)


@pytest.mark.parametrize("T,N,K", [(80001, 384, 128), (4133, 128, 256), (37, 64, 48), (5, 16, 16), (0, 32, 32),
                                   (70000, 256, 128), (1000, 400, 144), (9, 512, 32), (256, 64, 64),
                                   (33, 64, 768), (256, 64, 768)])
def test_linear_wgrad_against_float64(gpu, gemm_precision, T, N, K):
    """dW = dY^T X and db = sum_t dY (split-K; fp32 MFMA or bf16x3) vs a float64 product: max
    error <= 2e-5 * sqrt(T) — fp32 accumulation over T terms (bf16x3 adds <= 2^-17 |dy x| per
    product, random in sign)."""
    g = torch.Generator().manual_seed(T + N + K)
    dy = torch.randn(T, N, generator=g)
    x = torch.randn(T, K, generator=g)
    dw, db = ops.linear_wgrad(dy.to(gpu), x.to(gpu), (N, K), True)
    ref_w = dy.double().t() @ x.double()
    ref_b = dy.double().sum(0)
    scale = max(1.0, math.sqrt(max(T, 1)))
    if gemm_precision == "bf16x3":  # per-element bound: each product within 2^-17 (+ fp32 sums)
        bound = 2e-5 * (dy.double().abs().t() @ x.double().abs()) + 2e-5 * scale
        assert ((dw.cpu().double() - ref_w).abs() <= bound).all()
    else:
        assert (dw.cpu().double() - ref_w).abs().max().item() <= 2e-5 * scale
    assert (db.cpu().double() - ref_b).abs().max().item() <= 2e-5 * scale


def _absprod(a, b):
    return a.double().abs() @ b.double().abs().t()


@pytest.mark.parametrize("M,N,K", [(1000, 384, 128), (777, 128, 256), (5, 256, 384), (129, 128, 32), (0, 128, 32),
                                   (1000, 256, 1024), (130, 128, 2048), (3000, 768, 3072), (3000, 2304, 768)])
def test_gemm_x3_against_float64(gpu, M, N, K):
    """rsx_gemm_x3 (bf16x3 products, fp32 accumulate) vs float64: |C - ref| <= 2e-5 * sum_k
    |a_mk b_nk| + 1e-6 per element (each bf16x3 product is within 2^-17 of exact). The last four shapes
    have fewer output tiles than CUs and a long K: split-K through ops.gemm_x3's workspace (S = 4, 8, 4)
    and the four-stage prefetch (3000 x 2304)."""
    g = torch.Generator().manual_seed(M + N + K)
    a = torch.randn(M, K, generator=g)
    b = torch.randn(N, K, generator=g)
    bias = torch.randn(N, generator=g)
    c = ops.gemm_x3(a.to(gpu), b.to(gpu), bias.to(gpu)).cpu().double()
    ref = a.double() @ b.double().t() + bias.double()
    assert c.shape == (M, N)
    if M:
        assert ((c - ref).abs() <= 2e-5 * _absprod(a, b) + 1e-6).all()


@pytest.mark.parametrize("K,K2", [(128, 128), (1024, 1024)])
def test_gemm_x3_gelu_dropout_epilogues(gpu, K, K2):
    """EPI_GELU_DROP: C = dropout(gelu(pre)) (kept entries gelu(pre) / (1 - p), drop rate ~p)
    and aux = gelu'(pre), both against float64 from the inputs (bound 2e-5 * sum|a||b| on pre,
    propagated through |gelu'| <= 1.13 and |gelu''| <= 0.6); EPI_DGELU_DROP with the same seed:
    zero exactly where the forward dropped, (dY W) / (1 - p) * aux elsewhere. K = 1024: both GEMMs
    take the split-K path (the epilogues applied in the reduction pass)."""
    g = torch.Generator().manual_seed(11)
    M, N, p, seed = 1031, 256, 0.2, 12345
    x = torch.randn(M, K, generator=g)
    w1 = torch.randn(N, K, generator=g) / math.sqrt(K)
    b1 = torch.randn(N, generator=g)
    aux = torch.empty(M, N, device=gpu)
    act = ops.gemm_x3(x.to(gpu), w1.to(gpu), b1.to(gpu), ops.EPI_GELU_DROP, aux, p, seed).cpu().double()
    aux = aux.cpu().double()
    pre = x.double() @ w1.double().t() + b1.double()
    bnd = 2e-5 * _absprod(x, w1)
    cdf = 0.5 * (1 + torch.erf(pre / math.sqrt(2.0)))
    gel = pre * cdf
    ggrad = cdf + pre * torch.exp(-0.5 * pre ** 2) / math.sqrt(2 * math.pi)
    assert ((aux - ggrad).abs() <= 0.6 * bnd + 2e-6).all()
    kept = act != 0
    assert ((act - gel / (1 - p)).abs()[kept] <= (1.13 * bnd / (1 - p) + 2e-6)[kept]).all()
    frac = 1.0 - kept.double().mean().item()
    assert abs(frac - p) < 0.01
    w2 = torch.randn(K2, N, generator=g) / math.sqrt(N)
    dy = torch.randn(M, K2, generator=g)
    dpre = ops.gemm_x3(dy.to(gpu), w2.t().to(gpu), None, ops.EPI_DGELU_DROP, aux.float().to(gpu), p,
                       seed).cpu().double()
    dact = dy.double() @ w2.double()
    ref = torch.where(kept, dact / (1 - p) * aux, torch.zeros_like(aux))
    dropped = (~kept) & (gel.abs() > 1e-6)
    assert (dpre[dropped] == 0).all()
    assert ((dpre - ref).abs() <= 2e-5 * _absprod(dy, w2.t()) / (1 - p) * aux.abs() + 1e-6).all()


def test_ffn_matches_torch(gpu):
    """ops.ffn (fused GELU epilogues, bf16x3 GEMMs) == linear2(gelu(linear1(h))) in float64
    at p = 0, in value and in all gradients: |err| <= 2e-4 + 2e-5 * max|ref| (bf16x3 products
    carry ~2^-17 relative error each; the weight gradients sum ~2k token products)."""
    g = torch.Generator().manual_seed(5)
    h = torch.randn(2, 999, 128, generator=g).to(gpu)
    w1 = (torch.randn(256, 128, generator=g) / 11).to(gpu)
    b1 = torch.randn(256, generator=g).to(gpu)
    w2 = (torch.randn(128, 256, generator=g) / 16).to(gpu)
    b2 = torch.randn(128, generator=g).to(gpu)
    gy = torch.randn(2, 999, 128, generator=g).to(gpu)
    outs = []
    for impl in ("rsx", "torch64"):
        ts = (h, w1, b1, w2, b2) if impl == "rsx" else tuple(t.double() for t in (h, w1, b1, w2, b2))
        hh, a1, c1, a2, c2 = (t.clone().requires_grad_() for t in ts)
        if impl == "rsx":
            y = ops.ffn(hh, a1, c1, a2, c2, 0.0, True)
        else:
            y = F.linear(F.gelu(F.linear(hh, a1, c1)), a2, c2)
        (y * (gy if impl == "rsx" else gy.double())).sum().backward()
        outs.append((y.detach(), hh.grad, a1.grad, c1.grad, a2.grad, c2.grad))
    for a, r in zip(*outs):
        assert (a.double() - r).abs().max().item() <= 2e-4 + 2e-5 * r.abs().max().item()


def test_linear_tok_autograd_matches_linear(gpu):
    """linear_tok == F.linear (float64) in value and in all three gradients (forward / dX on
    rsx_gemm_x3, dW/db on rsx_linear_wgrad_x3), including a weight slice view
    (output_proj[0].weight[:, :D]): |err| <= 2e-4 + 2e-5 * max|ref|."""
    g = torch.Generator().manual_seed(3)
    x = torch.randn(3, 700, 128, generator=g).to(gpu)
    w_full = torch.randn(128, 256, generator=g).to(gpu)
    b = torch.randn(128, generator=g).to(gpu)
    gy = torch.randn(3, 700, 128, generator=g).to(gpu)
    outs = []
    for fn, dt in ((ops.linear_tok, torch.float32), (F.linear, torch.float64)):
        xx = x.to(dt).clone().requires_grad_()
        ww = w_full.to(dt).clone().requires_grad_()
        bb = b.to(dt).clone().requires_grad_()
        y = fn(xx, ww[:, :128], bb)
        (y * gy.to(dt)).sum().backward()
        outs.append((y.detach(), xx.grad, ww.grad, bb.grad))
    for a, r in zip(*outs):
        assert (a.double() - r).abs().max().item() <= 2e-4 + 2e-5 * r.abs().max().item()


@pytest.mark.parametrize("D,act", [(128, 0), (128, 2), (64, 0), (256, 2), (512, 2), (768, 0), (1024, 2),
                                   (2048, 2), (2048, 0)])
def test_layer_norm_against_torch(gpu, D, act):
    """rsx LayerNorm (+GELU) forward and all gradients vs torch fp32 (atol 2e-4 / rtol 1e-4); the
    wide rows (512..2048: the item head's 4d / 16d LayerNorms) run one wave per row."""
    g = torch.Generator().manual_seed(D + act)
    x = (torch.randn(1337, D, generator=g) * 3 + 1).to(gpu)
    w = (torch.rand(D, generator=g) + 0.5).to(gpu)
    b = torch.randn(D, generator=g).to(gpu)
    gy = torch.randn(1337, D, generator=g).to(gpu)
    outs = []
    for impl in ("rsx", "torch"):
        xx, ww, bb = (t.clone().requires_grad_() for t in (x, w, b))
        if impl == "rsx":
            y = ops.layer_norm(xx, ww, bb, 1e-5, act=act)
        else:
            y = F.layer_norm(xx, (D,), ww, bb, 1e-5)
            if act == 2:
                y = F.gelu(y)
        (y * gy).sum().backward()
        outs.append((y.detach(), xx.grad, ww.grad, bb.grad))
    for a, r in zip(*outs):
        torch.testing.assert_close(a, r, atol=2e-4, rtol=1e-4)


def test_add_layer_norm_residual_and_dropout(gpu):
    """s = x + dropout(res), y = LN(s): p=0 equals torch; p>0: s - x is res*scale or 0, and the
    residual gradient is the incoming gradient through the same mask."""
    g = torch.Generator().manual_seed(5)
    x = torch.randn(999, 128, generator=g).to(gpu)
    r = torch.randn(999, 128, generator=g).to(gpu)
    w = (torch.rand(128, generator=g) + 0.5).to(gpu)
    b = torch.randn(128, generator=g).to(gpu)
    gs = torch.randn(999, 128, generator=g).to(gpu)
    gy = torch.randn(999, 128, generator=g).to(gpu)
    outs = []
    for impl in ("rsx", "torch"):
        xx, rr, ww, bb = (t.clone().requires_grad_() for t in (x, r, w, b))
        if impl == "rsx":
            s, y = ops.add_layer_norm(xx, rr, ww, bb, 1e-5, 0.0)
        else:
            s = xx + rr
            y = F.layer_norm(s, (128,), ww, bb, 1e-5)
        ((s * gs).sum() + (y * gy).sum()).backward()
        outs.append((s.detach(), y.detach(), xx.grad, rr.grad, ww.grad, bb.grad))
    for a, ref in zip(*outs):
        torch.testing.assert_close(a, ref, atol=2e-4, rtol=1e-4)
    p = 0.3
    rr = r.clone().requires_grad_()
    xx = x.clone().requires_grad_()
    s, y = ops.add_layer_norm(xx, rr, w, b, 1e-5, p)
    kept = (s - x).abs() > 1e-6
    torch.testing.assert_close((s - x)[kept], (r / (1 - p))[kept], atol=1e-5, rtol=1e-5)
    frac = kept.float().mean().item()
    assert abs(frac - (1 - p)) < 0.01, frac
    (s * gs).sum().backward()
    torch.testing.assert_close(xx.grad, gs, atol=1e-6, rtol=0)
    torch.testing.assert_close(rr.grad, torch.where(kept, gs / (1 - p), torch.zeros_like(gs)), atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("K,M", [(128, 999), (256, 4101)])
def test_linear_add_layer_norm_fused(gpu, K, M):
    """rsx_gemm_x3_addln (out-projection + residual add + LayerNorm in one epilogue): p = 0 against
    torch fp32 (forward and every gradient); p > 0 against the unfused linear_tok + add_layer_norm
    with the same dropout seed (same mask, same gradients)."""
    g = torch.Generator().manual_seed(11)
    x = torch.randn(M, 128, generator=g).to(gpu)
    a = torch.randn(M, K, generator=g).to(gpu)
    W = (torch.randn(128, K, generator=g) / K ** 0.5).to(gpu)
    bW = torch.randn(128, generator=g).to(gpu) * 0.1
    w = (torch.rand(128, generator=g) + 0.5).to(gpu)
    b = torch.randn(128, generator=g).to(gpu)
    gs = torch.randn(M, 128, generator=g).to(gpu)
    gy = torch.randn(M, 128, generator=g).to(gpu)

    def run(impl, p=0.0, seed=0):
        xx, aa, WW, bb, ww, lb = (t.clone().requires_grad_() for t in (x, a, W, bW, w, b))
        if impl == "fused":
            s, y = ops._LinearAddLayerNorm.apply(xx, aa, WW, bb, ww, lb, 1e-5, p, seed)
        elif impl == "unfused":
            s, y = ops._AddLayerNorm.apply(xx, ops.linear_tok(aa, WW, bb), ww, lb, 1e-5, p, seed)
        else:
            s = xx + F.linear(aa, WW, bb)
            y = F.layer_norm(s, (128,), ww, lb, 1e-5)
        ((s * gs).sum() + (y * gy).sum()).backward()
        return [s.detach(), y.detach(), xx.grad, aa.grad, WW.grad, bb.grad, ww.grad, lb.grad]

    for u, r in zip(run("fused"), run("torch")):  # bf16x3 products: ~1e-5 of the largest entry
        torch.testing.assert_close(u, r, atol=2e-4 + 2e-5 * r.abs().max().item(), rtol=1e-4)
    fu, un = run("fused", 0.2, 1234567), run("unfused", 0.2, 1234567)
    torch.testing.assert_close(fu[0], un[0], atol=0, rtol=0)  # same products, same mask, same add
    for u, r in zip(fu[1:], un[1:]):  # row statistics summed in another order: ulp-level y, dres
        torch.testing.assert_close(u, r, atol=2e-5 + 1e-5 * r.abs().max().item(), rtol=1e-5)
    kept = (fu[0] - x).abs() > 0
    assert abs(kept.float().mean().item() - 0.8) < 0.02


def test_static_embed_against_torch(gpu):
    """Nine gated tiny-table lookups (static profile): forward bit-exact vs torch, table and
    gate gradients (padding_idx 0 rows excluded) vs torch autograd (1e-5)."""
    g = torch.Generator().manual_seed(6)
    shapes = [(11, 16)] * 4 + [(4, 4)] * 2 + [(3, 4)] * 3
    B = 3000
    tabs = [torch.randn(r, d, generator=g) for r, d in shapes]
    ids = [torch.randint(0, r, (B,), generator=g) for r, _ in shapes]
    gate = torch.rand(9, generator=g)
    gy = torch.randn(B, sum(d for _, d in shapes), generator=g)
    outs = []
    for impl in ("rsx", "torch"):
        tt = [t.clone().to(gpu).requires_grad_() for t in tabs]
        gg = gate.clone().to(gpu).requires_grad_()
        ii = [i.to(gpu) for i in ids]
        if impl == "rsx":
            y = ops.static_embed(ii, tt, gg, [0] * 9)
        else:
            y = torch.cat([F.embedding(i, t, padding_idx=0) * gg[j] for j, (i, t) in enumerate(zip(ii, tt))], 1)
        (y * gy.to(gpu)).sum().backward()
        outs.append((y.detach(), gg.grad, [t.grad for t in tt]))
    assert torch.equal(outs[0][0], outs[1][0])
    torch.testing.assert_close(outs[0][1], outs[1][1], atol=1e-3, rtol=1e-5)
    for a, r in zip(outs[0][2], outs[1][2]):
        torch.testing.assert_close(a, r, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("users,n", [(37, 128), (300, 256)])
def test_profile_linear_matches_concat_linear(gpu, users, n):
    """ops.profile_linear == F.linear(cat(x, profile[tok_user]), W, b) in float64, value and
    all gradients: the row-add GEMM epilogue, the segmented per-user gradient and both weight
    halves written into one [N, 2D] gradient. Users with 0 tokens included."""
    g = torch.Generator().manual_seed(users)
    counts = torch.randint(0, 40, (users,), generator=g)
    counts[3] = 0
    tok_user = torch.repeat_interleave(torch.arange(users), counts)
    seg = torch.zeros(users + 1, dtype=torch.int64)
    seg[1:] = torch.cumsum(counts, 0)
    T, D = tok_user.numel(), 128
    x = torch.randn(T, D, generator=g)
    prof = torch.randn(users, D, generator=g)
    w = torch.randn(n, 2 * D, generator=g) / 16
    b = torch.randn(n, generator=g)
    gy = torch.randn(T, n, generator=g)
    outs = []
    for impl in ("rsx", "torch64"):
        if impl == "rsx":
            ts = [t.to(gpu).requires_grad_() for t in (x, prof, w, b)]
            y = ops.profile_linear(ts[0], ts[1], ts[2], ts[3], tok_user.to(gpu), seg.to(gpu))
            (y * gy.to(gpu)).sum().backward()
        else:
            ts = [t.double().requires_grad_() for t in (x, prof, w, b)]
            y = F.linear(torch.cat([ts[0], ts[1][tok_user]], 1), ts[2], ts[3])
            (y * gy.double()).sum().backward()
        outs.append([y.detach()] + [t.grad for t in ts])
    for a, r in zip(*outs):
        a = a.double().cpu()
        assert (a - r).abs().max().item() <= 2e-4 + 2e-5 * r.abs().max().item()


# ------------------------------------------------------------------ fused in_proj + attention
@pytest.mark.parametrize("packed,causal,use_pad,p_drop", [(True, True, True, 0.0), (False, True, True, 0.0),
                                                          (False, False, False, 0.0), (True, True, True, 0.2)])
def test_qkv_mha_fused_matches_two_op_path(gpu, packed, causal, use_pad, p_drop):
    """rsx_mha_qkv_fwd_x3 (in_proj fused into the attention forward) against linear_tok + mha on
    the same inputs and dropout seed: attention output, the qkv it writes for the backward, and
    dx / dW / db through the shared backward (atol 2e-5: the two paths sum the projection's k
    products in different orders). Packed segments of 1..64 tokens or dense L = 50 with left
    padding, as the user tower runs them."""
    g = torch.Generator().manual_seed(31 + int(packed) + 2 * int(causal) + int(10 * p_drop))
    D, H = 128, 4
    if packed:
        lens = torch.randint(1, 65, (61,), generator=g)
        seg = torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum(lens, 0)])
        T = int(seg[-1])
        x = torch.randn(T, D, generator=g)
        pad = torch.zeros(T, dtype=torch.bool)
        pad[seg[1:] - 1] = torch.rand(len(lens), generator=g) < 0.3
        seg_d = seg.to(gpu)
    else:
        B, L = 23, 50
        x = torch.randn(B, L, D, generator=g)
        cnt = torch.randint(1, L + 1, (B,), generator=g)
        pad = torch.arange(L)[None, :] < (L - cnt)[:, None]  # left padding
        seg_d = None
    w = torch.randn(3 * D, D, generator=g) * D ** -0.5
    b = torch.randn(3 * D, generator=g) * 0.1
    dout = torch.randn(x.shape, generator=g)
    kp = pad.to(gpu) if use_pad else None
    seed = 1234
    res = []
    for fused in (True, False):
        xd = x.to(gpu).requires_grad_()
        wd = w.to(gpu).requires_grad_()
        bd = b.to(gpu).requires_grad_()
        if fused:
            out = ops._QKVMHA.apply(xd, wd, bd, kp, None if seg_d is None else seg_d.to(torch.int32).contiguous(), H,
                                    causal, p_drop, seed)
        else:
            qkv = ops.linear_tok(xd, wd, bd)
            out = ops._MHA.apply(qkv, kp, None if seg_d is None else seg_d.to(torch.int32).contiguous(), H, causal,
                                 p_drop, seed)
        (out * dout.to(gpu)).sum().backward()
        res.append((out.detach().cpu(), xd.grad.cpu(), wd.grad.cpu(), bd.grad.cpu()))
    for name, a, r in zip(["out", "dx", "dw", "db"], res[0], res[1]):
        tol = 2e-5 * max(1.0, r.abs().max().item())
        torch.testing.assert_close(a, r, atol=tol, rtol=1e-4, msg=lambda m, name=name: f"{name}: {m}")
