"""Host-side logic of the round-5 step (no GPU): the step index's single-allocation carving
(dist._carve) and the native clip+AdamW's applicability rules (ops.clip_adamw_step declines what
it does not reproduce, leaving torch's clip_grad_norm_ + optimizer.step to run)."""
import math

import torch

from recsys_amd import dist, ops


def test_carve_shapes_alignment_and_disjointness():
    specs = [((5,), torch.int64), None, ((3, 4), torch.float32), ((0,), torch.int32), ((7,), torch.uint8),
             ((2, 0), torch.int64), ((9,), torch.int32)]
    out = dist._carve(specs, "cpu")
    assert out[1] is None
    spans = []
    base = out[0].data_ptr()  # the allocation's start (the device allocator aligns it to >= 256 B)
    for sp, t in zip(specs, out):
        if sp is None:
            continue
        assert tuple(t.shape) == sp[0] and t.dtype == sp[1] and t.is_contiguous()
        if t.numel():
            assert (t.data_ptr() - base) % 256 == 0
            spans.append((t.data_ptr(), t.data_ptr() + t.numel() * t.element_size()))
    spans.sort()
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 <= b0                                  # no two arrays overlap
    out[0].fill_(-1)
    out[2].fill_(2.5)
    out[6].fill_(7)
    assert out[0].tolist() == [-1] * 5 and float(out[2].sum()) == 30.0 and out[6].tolist() == [7] * 9


def test_clip_adamw_declines_what_it_does_not_reproduce():
    p = torch.nn.Parameter(torch.randn(8))
    p.grad = torch.randn(8)
    # CPU parameters, another optimizer, amsgrad, a tensor learning rate: nothing done, None returned
    assert ops.clip_adamw_step(torch.optim.AdamW([p]), [p], 5.0) is None
    assert ops.clip_adamw_step(torch.optim.SGD([p], lr=0.1), [p], 5.0) is None
    assert not ops._adamw_native_ok(torch.optim.AdamW([p], amsgrad=True))
    assert not ops._adamw_native_ok(torch.optim.AdamW([p], lr=torch.tensor(1e-3)))
    assert not ops._adamw_native_ok(torch.optim.Adam([p]))
    assert ops._adamw_native_ok(torch.optim.AdamW([p], lr=5e-4, weight_decay=0.01))
    assert len(torch.optim.AdamW([p]).state) == 0


def test_ln_bwd_workspace_is_monotonic_in_rows():
    """rsx_ln_bwd_workspace_floats(T) must cover every smaller row count: the tower backward sizes
    one workspace by T and runs its tail rows (R < T) on it (the block split itself is not monotonic
    in T; the 2-rank rehearsal once failed with 'workspace too small'). Host-only C-ABI call."""
    from recsys_amd import _native as N
    lib = N.lib()
    for D in (64, 128, 256):
        prev = 0
        for T in list(range(1, 5000, 37)) + list(range(150_000, 420_000, 997)):
            w = lib.rsx_ln_bwd_workspace_floats(T, D)
            assert w >= prev, (D, T, w, prev)
            prev = w
    # an unsupported row width is an error code, not a division by zero (D / 4 == 0 for D < 4)
    for D in (0, 1, 3, 4, 100, 4096):
        assert lib.rsx_ln_bwd_workspace_floats(1000, D) == -1


def test_module_params_same_set_as_parameters():
    """ops.module_params (the clip set of the native clip+AdamW) holds exactly model.parameters():
    shared parameters once, None slots skipped, nested and tied modules walked."""
    lin = torch.nn.Linear(4, 4)
    model = torch.nn.Sequential(lin, torch.nn.ReLU(), torch.nn.Sequential(torch.nn.Linear(4, 2), lin))
    model.register_parameter("nothing", None)
    model.extra = torch.nn.Parameter(torch.zeros(3))
    got = ops.module_params(model)
    assert len(got) == len(list(model.parameters()))
    assert {id(p) for p in got} == {id(p) for p in model.parameters()}


def test_emphasis_correction_identity_matches_dense_form():
    """The arithmetic rsx_nce_emphasis_fwd / _bwd implement (csrc/infonce.hip, nce_emph_*_k), checked in
    float64 against full_batch_hard_emphasis_loss's dense form (v1_refine_usertower.py:546-554): with lse
    the masked row log-sum-exp and E_i = sum over allowed mined j of exp(S_ij - lse_i),
      lse'_i = lse_i + log1p((e^m - 1) E_i),  loss'_i = lse'_i - S_ii - m [i mined],
    and the gradient w.r.t. S is exp(S_ij - lse'_i) (1 + (e^m - 1) [j mined]) - [j = i] on allowed
    columns (the dense backward with lse' in the workspace plus the mined entries' extra term)."""
    g = torch.Generator().manual_seed(3)
    N, K, m = 40, 5, 0.2 / 0.1
    S = torch.randn(N, N, generator=g, dtype=torch.float64) * 3
    keys = torch.randint(0, 25, (N,), generator=g)
    same = (keys[:, None] == keys[None, :]) & ~torch.eye(N, dtype=torch.bool)
    top = torch.stack([torch.randperm(N, generator=g)[:K] for _ in range(N)])  # may include masked / diagonal
    top[0, 0] = 0                                                                # a row whose own column is mined
    # dense reference (the reference's order: emphasis added, then the same-item mask, then CE)
    Sd = S.clone().requires_grad_()
    emph = torch.zeros(N, N, dtype=torch.float64).scatter_(1, top, m)
    logits = (Sd + emph).masked_fill(same, float("-inf"))
    ref = torch.nn.functional.cross_entropy(logits, torch.arange(N), reduction="sum")
    ref.backward()
    # the decomposition
    Sm = S.masked_fill(same, float("-inf"))
    lse = torch.logsumexp(Sm, 1)
    mined = torch.zeros(N, N, dtype=torch.bool).scatter_(1, top, True) & ~same
    E = (torch.exp(Sm - lse[:, None]) * mined).sum(1)
    lse2 = lse + torch.log1p(math.expm1(m) * E)
    self_mined = mined[torch.arange(N), torch.arange(N)]
    loss = (lse2 - S.diagonal() - m * self_mined).sum()
    assert abs(float(loss) - float(ref)) < 1e-9 * abs(float(ref))
    p2 = torch.exp(Sm - lse2[:, None])
    grad = p2 * (1 + math.expm1(m) * mined.double()) - torch.eye(N, dtype=torch.float64)
    grad = grad.masked_fill(same, 0.0)
    torch.testing.assert_close(grad, Sd.grad, atol=1e-12, rtol=1e-9)
