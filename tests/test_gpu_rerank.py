"""DeepFM forward (A16) and retrieval top-k (A14) vs the CPU oracles."""
import pytest
import torch

import recsys_amd  # noqa: F401
from recsys_amd import ops
from recsys_amd.temp_model.ranker_skelet import DeepFM, ReRankingSystem
from oracle import deepfm as OD
from oracle import retrieval as OR

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("R,F,vocab", [(1000, 39, 500), (77, 5, 50), (4096, 39, 10000)])
def test_deepfm_forward_matches_oracle(gpu, R, F, vocab):
    model = DeepFM([vocab] * F, init_std=0.05, device=gpu)  # larger init than 1e-4 so every term matters
    g = torch.Generator().manual_seed(R)
    x = torch.randint(0, vocab, (R, F), generator=g)
    with torch.no_grad():
        model.out.bias.fill_(0.1)
        for l in model.dnn.linears:
            l.bias.normal_(0, 0.05)
    logit, prob = model.forward_logits(x.to(gpu))
    names = model.field_names
    ref_l, ref_p = OD.deepfm_forward(
        x, [model.embedding_dict[n].weight.cpu() for n in names],
        [model.linear_model.embedding_dict[n].weight.cpu() for n in names], 0.1,
        [l.weight.cpu() for l in model.dnn.linears], [l.bias.cpu() for l in model.dnn.linears],
        model.dnn_linear.weight.cpu())
    torch.testing.assert_close(logit.cpu().double(), ref_l, atol=1e-4, rtol=1e-5)
    torch.testing.assert_close(prob.cpu().double(), ref_p, atol=1e-5, rtol=1e-5)
    out = model(x.to(gpu))
    assert out.shape == (R, 1)


@pytest.mark.parametrize("R,F", [(4099, 39), (64, 13), (200, 40)])
def test_deepfm_fused_matches_unfused(gpu, R, F):
    """The fused kernel (bf16x3 DNN) against the three-kernel path (fp32-MFMA DNN) on the same
    model: logits within 1e-4 (north_star's fp32-logit bound), including the F % 13 != 0 tail
    and rows past the last 64-row block."""
    model = DeepFM([3000] * F, init_std=0.05, device=gpu)
    with torch.no_grad():
        model.out.bias.fill_(-0.3)
        for l in model.dnn.linears:
            l.bias.normal_(0, 0.05)
    g = torch.Generator().manual_seed(R + F)
    x = torch.randint(0, 3000, (R, F), generator=g).to(gpu)
    assert ops._DEEPFM_FUSED
    lf, pf = model.forward_logits(x)
    ops._DEEPFM_FUSED = False
    try:
        lu, pu = model.forward_logits(x)
    finally:
        ops._DEEPFM_FUSED = True
    torch.testing.assert_close(lf, lu, atol=1e-4, rtol=0)
    torch.testing.assert_close(pf, pu, atol=2.5e-5, rtol=0)


def test_linear_act_variants(gpu):
    g = torch.Generator().manual_seed(3)
    x = torch.randn(300, 96, generator=g)
    for n, act in [(256, ops.ACT_RELU), (100, ops.ACT_GELU), (32, ops.ACT_NONE)]:
        w = torch.randn(n, 96, generator=g) * 0.1
        b = torch.randn(n, generator=g)
        y = ops.linear(x.to(gpu), w.to(gpu), b.to(gpu), act)
        ref = x.double() @ w.double().T + b.double()
        ref = torch.relu(ref) if act == ops.ACT_RELU else (torch.nn.functional.gelu(ref) if act == ops.ACT_GELU else ref)
        torch.testing.assert_close(y.cpu().double(), ref, atol=2e-5, rtol=1e-5)


@pytest.mark.parametrize("Q,NI,k", [(50, 3000, 100), (130, 20000, 500), (7, 90, 100), (300, 70000, 10)])
def test_retrieve_topk_bit_exact_on_dyadic_inputs(gpu, Q, NI, k):
    """Dyadic inputs make every fp32 dot product exact (no rounding), so the indices must be
    identical to the oracle's (score desc, index asc) order, ties included."""
    g = torch.Generator().manual_seed(Q + NI)
    U = torch.randint(-4, 5, (Q, 128), generator=g).float() / 8.0
    I = torch.randint(-4, 5, (NI, 128), generator=g).float() / 8.0
    s, i = ops.retrieve_topk(U.to(gpu), I.to(gpu), k)
    rs, ri = OR.retrieve_topk(U, I, min(k, NI))
    kk = min(k, NI)
    assert torch.equal(i[:, :kk].cpu(), ri)
    assert torch.equal(s[:, :kk].cpu().double(), rs)
    if k > NI:
        assert (i[:, NI:] == -1).all()


def test_retrieve_topk_realistic(gpu):
    g = torch.Generator().manual_seed(1)
    U = torch.nn.functional.normalize(torch.randn(64, 128, generator=g), dim=1)
    I = torch.nn.functional.normalize(torch.randn(50000, 128, generator=g), dim=1)
    s, i = ops.retrieve_topk(U.to(gpu), I.to(gpu), 100)
    rs, ri = OR.retrieve_topk(U, I, 100)
    torch.testing.assert_close(s.cpu().double(), rs, atol=1e-6, rtol=0)
    # indices agree except near-ties within fp32 noise: each returned item's float64 score equals
    # the oracle's score at that rank
    ours = torch.einsum("qkd,qd->qk", I.double()[i.cpu()], U.double())
    assert (ours - rs).abs().max().item() < 1e-6


def test_reranking_system_deepfm(gpu):
    g = torch.Generator().manual_seed(2)
    items = torch.nn.functional.normalize(torch.randn(5000, 128, generator=g), dim=1).to(gpu)
    model = DeepFM([1000] * 39, device=gpu)

    def feats(uv, idx):
        return torch.stack([(idx * 131 + f * 17) % 1000 for f in range(39)], dim=1)

    sys_ = ReRankingSystem(None, None, model, {}, items, rerank_features=feats)
    uv = torch.nn.functional.normalize(torch.randn(128, generator=g), dim=0)
    recs = sys_.recommend(uv, top_k_retrieval=100, final_k=10)
    assert len(recs) == 10
    scores = [r["final_score"] for r in recs]
    assert scores == sorted(scores, reverse=True)


@pytest.mark.parametrize("Q,NI,k,path", [(130, 100003, 100, "bf16"), (70, 60000, 500, "fast"), (257, 40000, 7, "bf16"),
                                         (5000, 70000, 64, "bf16")])
def test_retrieve_topk_fast_path_bit_exact(gpu, Q, NI, k, path):
    """Large corpora take the bf16 single scan + exact rescoring path (or, where its sample
    cannot hold 2k candidates, the fp32 candidate/threshold path): on dyadic inputs (exact dot
    products and exact bf16 images, many exact ties) the result must equal the oracle's (score
    desc, index asc), whether or not the exactness check falls back. Q = 5000 runs the bf16 path
    in two query chunks (4096 + 904)."""
    g = torch.Generator().manual_seed(Q * 7 + k)
    U = torch.randint(-4, 5, (Q, 128), generator=g).float() / 8.0
    I = torch.randint(-4, 5, (NI, 128), generator=g).float() / 8.0
    diag = {}
    s, i = ops.retrieve_topk(U.to(gpu), I.to(gpu), k, diag=diag)
    assert diag["path"] == path
    rs, ri = OR.retrieve_topk_chunked(U, I, k)
    assert torch.equal(i.cpu(), ri)
    assert torch.equal(s.cpu().double(), rs)


def test_retrieve_topk_fast_path_overflow_fallback(gpu):
    """Massive exact ties at the threshold (a corpus of 40k copies of a few rows) overflow the
    per-query buffers; the gated exact fallback must still return the oracle's result."""
    g = torch.Generator().manual_seed(11)
    base = torch.randint(-4, 5, (5, 128), generator=g).float() / 8.0
    I = base[torch.randint(0, 5, (40000,), generator=g)]
    U = torch.randint(-4, 5, (33, 128), generator=g).float() / 8.0
    s, i = ops.retrieve_topk(U.to(gpu), I.to(gpu), 100)
    rs, ri = OR.retrieve_topk(U, I, 100)
    assert torch.equal(i.cpu(), ri)
    assert torch.equal(s.cpu().double(), rs)


@pytest.mark.parametrize("Q,NI,k", [(600, 200_000, 100), (40, 200_000, 300)])
def test_retrieve_topk_single_scan_no_fallback_on_spread_data(gpu, Q, NI, k):
    """Realistic normalised data: the bf16 single scan + exact rescoring (both cases take that
    path: asserted from the workspace header) is exact by its own check (no fallback), and the
    result equals the float64 oracle up to fp32-noise near-ties."""
    g = torch.Generator().manual_seed(NI + k)
    U = torch.nn.functional.normalize(torch.randn(Q, 128, generator=g), dim=1)
    I = torch.nn.functional.normalize(torch.randn(NI, 128, generator=g), dim=1)
    diag = {}
    s, i = ops.retrieve_topk(U.to(gpu), I.to(gpu), k, diag=diag)
    assert diag["path"] == "bf16"
    assert diag["fallback"] is False
    rs, ri = OR.retrieve_topk(U, I, k)
    torch.testing.assert_close(s.cpu().double(), rs, atol=2e-6, rtol=0)
    # every returned item's float64 score equals the oracle's score at that rank up to fp32
    # noise: only near-tied neighbours may swap or be exchanged at the k-th position
    ours = torch.einsum("qkd,qd->qk", I.double()[i.cpu()], U.double())
    assert (ours - rs).abs().max().item() < 2e-6
    assert (i.cpu() != ri).float().mean().item() < 0.01


def test_retrieve_topk_single_scan_clustered_falls_back_exactly(gpu):
    """Adversarial layout: 400 near-copies of query 0 stored contiguously (they land in a few
    scan streams, each keeping only its best T), dyadic values (exact dot products). The
    exactness check must detect the possibly dropped items and route the batch to the exact
    kernels for that query (not the whole batch): result bit-identical to the oracle, ties
    included."""
    g = torch.Generator().manual_seed(77)
    Q, NI = 130, 120_000
    U = torch.randint(-4, 5, (Q, 128), generator=g).float() / 8.0
    I = torch.randint(-4, 5, (NI, 128), generator=g).float() / 8.0
    noise = torch.randint(-1, 2, (400, 128), generator=g).float() / 8.0
    I[60_000:60_400] = U[0] + noise
    I[60_400:60_410] = U[0]                  # exact ties among the top items
    diag = {}
    s, i = ops.retrieve_topk(U.to(gpu), I.to(gpu), 100, diag=diag)
    assert diag["path"] == "bf16"
    assert diag["fallback"] is True and 1 <= diag["fallback_queries"] < Q   # per query, not the batch
    rs, ri = OR.retrieve_topk(U, I, 100)
    assert torch.equal(i.cpu(), ri)
    assert torch.equal(s.cpu().double(), rs)


@pytest.mark.parametrize("B,ctx", [(1000, True), (77, False)])
def test_dcn_ranking_model_matches_oracle(gpu, B, ctx):
    """RankingModel (DCN-V2, temp_model/ranker_skelet.py:274-357) on the GPU kernels vs the
    float64 restatement; biases randomised so every term matters. Probabilities within 2e-6,
    logits (pre-sigmoid) within 1e-4; predict_for_user broadcasts one user over the items."""
    from recsys_amd.temp_model.ranker_skelet import RankingModel
    from oracle import ranker as ORK
    torch.manual_seed(B)
    model = RankingModel(128, 128, 20 if ctx else 0)
    with torch.no_grad():
        for b in model.cross_net.biases:
            b.normal_(0, 0.05)
        for m in model.deep_net:
            if isinstance(m, torch.nn.Linear):
                m.bias.normal_(0, 0.05)
    model.eval()
    g = torch.Generator().manual_seed(B + 1)
    u = torch.nn.functional.normalize(torch.randn(B, 128, generator=g), dim=1)
    it = torch.nn.functional.normalize(torch.randn(B, 128, generator=g), dim=1)
    c = torch.randn(B, 20, generator=g) if ctx else None
    ref = ORK.ranking_model_forward(model, u, it, c)
    dut = model.to(gpu)
    got = dut(u.to(gpu), it.to(gpu), c.to(gpu) if ctx else None).cpu().double()
    assert got.shape == (B, 1)
    torch.testing.assert_close(got, ref, atol=2e-6, rtol=0)
    lg, lr = torch.logit(got.clamp(1e-7, 1 - 1e-7)), torch.logit(ref.clamp(1e-7, 1 - 1e-7))
    assert (lg - lr).abs().max().item() < 1e-4
    s = dut.predict_for_user(u[0].to(gpu), it.to(gpu), c[0].to(gpu) if ctx else None).cpu().double()
    ref1 = ORK.ranking_model_forward(model.cpu(), u[:1].expand(B, -1), it,
                                     c[:1].expand(B, -1) if ctx else None).squeeze()
    torch.testing.assert_close(s, ref1, atol=2e-6, rtol=0)


def test_deepfm_weight_image_cache_follows_updates(gpu):
    """The module keeps the fused kernel's bf16 weight images between calls; an in-place update
    of a DNN weight (new version) or a replaced Parameter (new storage) must rebuild them."""
    R, F, vocab = 3000, 39, 5000
    model = DeepFM([vocab] * F, init_std=0.05, device=gpu)
    g = torch.Generator().manual_seed(11)
    x = torch.randint(0, vocab, (R, F), generator=g)

    def check():
        logit, _ = model.forward_logits(x.to(gpu))
        names = model.field_names
        ref_l, _ = OD.deepfm_forward(
            x, [model.embedding_dict[n].weight.cpu() for n in names],
            [model.linear_model.embedding_dict[n].weight.cpu() for n in names], float(model.out.bias.item()),
            [l.weight.cpu() for l in model.dnn.linears], [l.bias.cpu() for l in model.dnn.linears],
            model.dnn_linear.weight.cpu())
        torch.testing.assert_close(logit.cpu().double(), ref_l, atol=1e-4, rtol=1e-5)

    check()
    with torch.no_grad():
        model.dnn.linears[0].weight.mul_(-1.5)
    check()
    model.dnn.linears[1].weight = torch.nn.Parameter(torch.randn(128, 256, device=gpu) * 0.05)
    check()
