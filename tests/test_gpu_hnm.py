"""Hard-negative mining kernel (rsx_hnm_mine) and the HNM losses built on it
(v1_refine_usertower.py:632-757 inbatch_hnm_corrected_loss_with_stats /
inbatch_mixed_hnm_loss_with_stats, :762-822 full_batch_hard_emphasis_loss) vs the CPU oracle.

Mining is index work: on integer-valued vectors every product is exact in fp32, so the kernel's
top-k indices (value desc, column asc), available counts and cosines are compared bit-exactly,
ties included. On random normalised vectors the selected values are compared against the float64
oracle's sorted values (1e-5), and the losses to 1e-5 relative with gradients to 1e-4."""
import pytest
import torch
import torch.nn.functional as F

import recsys_amd  # noqa: F401
from recsys_amd import ops
from recsys_amd.tower_code import v1_refine_usertower as T
from oracle import user_tower as O

pytestmark = pytest.mark.gpu


def _int_case(N, D, seed, n_tgt):
    g = torch.Generator().manual_seed(seed)
    u = torch.randint(-2, 3, (N, D), generator=g).float()
    it = torch.randint(-2, 3, (N, D), generator=g).float()
    it[1::7] = it[0::7][: it[1::7].shape[0]]  # duplicated columns: exact ties and item_sim hits
    t = torch.randint(1, n_tgt + 1, (N,), generator=g)
    return u, it, t


@pytest.mark.parametrize("N,D,k,thr", [(1, 128, 1, 0.5), (7, 64, 3, 40.0), (300, 128, 17, 30.0),
                                       (1000, 64, 64, 20.0), (2049, 128, 20, 60.0), (4096, 128, 40, 60.0)])
def test_hnm_mine_exact_integer(gpu, N, D, k, thr):
    u, it, t = _int_case(N, D, N + D, n_tgt=max(2, N // 3))
    k = min(k, N)
    idx, cos, avail = ops.hnm_mine(u.to(gpu), it.to(gpu), t.to(gpu), k, thr, 1.0)
    r_idx, r_avail = O.hnm_mine(u, it, t, k, thr, 1.0)
    assert torch.equal(avail.cpu().long(), r_avail)
    assert torch.equal(idx.cpu(), r_idx)
    assert torch.equal(cos.cpu(), (u.double() @ it.double().T).gather(1, r_idx).float())


@pytest.mark.parametrize("N,k,tau", [(513, 5, 0.1), (3000, 29, 0.15), (6144, 61, 0.1)])
def test_hnm_mine_random(gpu, N, k, tau):
    g = torch.Generator().manual_seed(N)
    I = N // 2
    W = F.normalize(torch.randn(I + 1, 128, generator=g), dim=1)
    W[5] = F.normalize(W[4] + 0.1 * torch.randn(128, generator=g), dim=0)  # item cosine > 0.9
    t = torch.randint(1, I + 1, (N,), generator=g)
    t[:4] = 4
    t[4:9] = 5
    u = F.normalize(torch.randn(N, 128, generator=g), dim=1)
    it = W[t]
    idx, cos, avail = ops.hnm_mine(u.to(gpu), it.to(gpu), t.to(gpu), k, 0.9, tau)
    r_idx, r_avail = O.hnm_mine(u, it, t, k, 0.9, tau)
    assert torch.equal(avail.cpu().long(), r_avail)
    full = u.double() @ it.double().T
    torch.testing.assert_close(full.gather(1, idx.cpu()), full.gather(1, r_idx), atol=1e-5, rtol=0)
    torch.testing.assert_close(cos.cpu().double(), full.gather(1, idx.cpu()), atol=1e-5, rtol=0)
    assert (idx.cpu().sort(1).values.diff(dim=1) > 0).all()  # distinct columns per row


def test_hnm_mine_fewer_available_than_k(gpu):
    """All-but-two columns share the row's target: -inf picks fill the tail in column order and
    report their raw cosines (the reference gathers cos_sim at the picked indices)."""
    N, k = 40, 6
    g = torch.Generator().manual_seed(1)
    u = F.normalize(torch.randn(N, 64, generator=g), dim=1)
    it = F.normalize(torch.randn(N, 64, generator=g), dim=1)
    t = torch.full((N,), 3)
    t[10], t[20] = 7, 8
    idx, cos, avail = ops.hnm_mine(u.to(gpu), it.to(gpu), t.to(gpu), k, 0.9, 0.1)
    r_idx, r_avail = O.hnm_mine(u, it, t, k, 0.9, 0.1)
    assert torch.equal(avail.cpu().long(), r_avail)
    assert torch.equal(idx.cpu(), r_idx)
    torch.testing.assert_close(cos.cpu().double(), (u.double() @ it.double().T).gather(1, r_idx), atol=1e-6, rtol=0)


def test_hnm_mine_rejects_bad_k(gpu):
    x = torch.randn(8, 128, device=gpu)
    t = torch.arange(8, device=gpu)
    with pytest.raises(ValueError):
        ops.hnm_mine(x, x, t, 9)
    with pytest.raises(RuntimeError):
        ops.hnm_mine(x.cpu(), x.cpu(), t.cpu(), 2)


def _loss_case(N, seed):
    g = torch.Generator().manual_seed(seed)
    I = 300
    W = torch.randn(I + 1, 128, generator=g)
    W[5] = W[4] + 0.01 * torch.randn(128, generator=g)
    lq = torch.log_softmax(torch.randn(I + 1, generator=g), 0)
    t = torch.randint(1, I + 1, (N,), generator=g)
    t[:3] = 4
    t[3:6] = 5
    U = torch.randn(N, 128, generator=g)
    return U, W, t, lq


@pytest.mark.parametrize("N,p,lambda_logq", [(700, 0.01, 0.7), (1500, 0.02, 0.0), (64, 0.5, 0.7)])
def test_hnm_corrected_loss_parity(gpu, N, p, lambda_logq):
    U, W, t, lq = _loss_case(N, N)
    u1, w1 = U.clone().requires_grad_(), W.clone().requires_grad_()
    l_ref, s_ref = O.inbatch_hnm_corrected_loss_with_stats(u1, w1, t, lq, top_k_percent=p, temperature=0.1,
                                                           lambda_logq=lambda_logq)
    l_ref.backward()
    u2, w2 = U.to(gpu).requires_grad_(), W.to(gpu).requires_grad_()
    l_dut, s_dut = T.inbatch_hnm_corrected_loss_with_stats(u2, w2, t.to(gpu), lq.to(gpu), top_k_percent=p,
                                                           temperature=0.1, lambda_logq=lambda_logq)
    l_dut.backward()
    assert s_dut["num_active_hard_negs"] == s_ref["num_active_hard_negs"]
    assert abs(l_dut.item() - l_ref.item()) <= 1e-5 * abs(l_ref.item()) + 1e-6
    assert abs(s_dut["avg_hn_similarity"] - s_ref["avg_hn_similarity"]) < 1e-5
    torch.testing.assert_close(u2.grad.cpu(), u1.grad, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(w2.grad.cpu(), w1.grad, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("N,M", [(700, 100), (300, 17)])
def test_mixed_hnm_loss_parity(gpu, N, M):
    U, W, t, lq = _loss_case(N, N + 1)
    torch.cuda.manual_seed(1234)
    ri = torch.randint(0, N, (N, M), device=gpu).cpu()  # replay of the draw inside the loss
    u1, w1 = U.clone().requires_grad_(), W.clone().requires_grad_()
    l_ref, s_ref = O.inbatch_mixed_hnm_loss_with_stats(u1, w1, t, lq, random_sample_size=M, random_indices=ri)
    l_ref.backward()
    u2, w2 = U.to(gpu).requires_grad_(), W.to(gpu).requires_grad_()
    torch.cuda.manual_seed(1234)
    l_dut, s_dut = T.inbatch_mixed_hnm_loss_with_stats(u2, w2, t.to(gpu), lq.to(gpu), random_sample_size=M)
    l_dut.backward()
    assert (s_dut["num_hard"], s_dut["num_random"]) == (s_ref["num_hard"], s_ref["num_random"])
    assert abs(l_dut.item() - l_ref.item()) <= 1e-5 * abs(l_ref.item()) + 1e-6
    assert abs(s_dut["avg_hn_similarity"] - s_ref["avg_hn_similarity"]) < 1e-5
    torch.testing.assert_close(u2.grad.cpu(), u1.grad, atol=1e-6, rtol=1e-4)
    torch.testing.assert_close(w2.grad.cpu(), w1.grad, atol=1e-6, rtol=1e-4)


@pytest.mark.parametrize("N,k,levels", [(3000, 100, 2), (2000, 37, 1), (5000, 1000, 3)])
def test_hnm_mine_massive_ties(gpu, N, k, levels):
    """Few distinct products: the boundary bin overflows the sort buffer (or min == max), so the
    exact radix-select path runs; ties must resolve to the lowest columns exactly."""
    g = torch.Generator().manual_seed(N)
    u = torch.zeros(N, 128)
    u[:, 0] = 1.0
    it = torch.zeros(N, 128)
    it[:, 0] = torch.randint(0, levels, (N,), generator=g).float() + 1.0
    it[:, 1 + torch.arange(N) % 100] = 0.5  # off-axis part: item-item products vary, none > thr
    t = torch.arange(N)  # distinct targets: only the diagonal is ignored (same target)
    idx, cos, avail = ops.hnm_mine(u.to(gpu), it.to(gpu), t.to(gpu), k, 1e9, 1.0)
    r_idx, r_avail = O.hnm_mine(u, it, t, k, 1e9, 1.0)
    assert torch.equal(avail.cpu().long(), r_avail)
    assert torch.equal(idx.cpu(), r_idx)
    assert torch.equal(cos.cpu(), (u.double() @ it.double().T).gather(1, r_idx).float())


@pytest.mark.parametrize("planted", [False, True])
def test_hnm_ignore_mask_export_matches_mining(gpu, planted):
    """The mixed loss masks its random draws with the miner's own ignore decisions
    (ops.hnm_mine(..., ignored_at=)), as the reference derives both from one ignore_mask
    (v1_refine_usertower.py:719, 746). With the threshold planted exactly at pair similarities
    (borderline pairs whose comparison can flip with the summation order), the exported mask is
    still consistent with the mining: avail = number of columns not ignored, mined columns are
    never ignored, and the exported mask equals the reference formula on the integer case."""
    N, k = 700, 9
    g = torch.Generator().manual_seed(7)
    it = F.normalize(torch.randn(N, 128, generator=g), dim=1)
    it[1::9] = F.normalize(it[0::9][: it[1::9].shape[0]] + 0.3 * torch.randn(it[1::9].shape[0], 128, generator=g),
                           dim=1)
    u = F.normalize(torch.randn(N, 128, generator=g), dim=1)
    t = torch.randint(1, N // 3, (N,), generator=g)
    thr = 0.9
    if planted:
        sims = (it[0::9][:10] * it[1::9][:10]).sum(1)
        thr = float(sims.median())  # several pairs sit exactly at the threshold in fp32
    d = lambda x: x.to(gpu)  # noqa: E731
    cols = torch.arange(N).repeat(N, 1)
    idx, cos, avail, ign = ops.hnm_mine(d(u), d(it), d(t), k, thr, 0.1, ignored_at=d(cols))
    ign = ign.cpu()
    assert torch.equal((~ign).sum(1).int(), avail.cpu())
    full = avail.cpu() >= k
    assert not ign.gather(1, idx.cpu())[full].any()
    assert ign.diagonal().all()  # same target as itself
    # integer vectors: exact products, so the exported mask equals the reference formula
    ui, ii, ti = _int_case(300, 128, 3, n_tgt=60)
    cols = torch.randint(0, 300, (300, 50), generator=g)
    *_, ign2 = ops.hnm_mine(d(ui), d(ii), d(ti), 5, 30.0, 1.0, ignored_at=d(cols))
    sim = ii @ ii.T
    ref = (ti[cols] == ti.unsqueeze(1)) | ((sim.gather(1, cols) > 30.0) & (cols != torch.arange(300).unsqueeze(1)))
    assert torch.equal(ign2.cpu(), ref)
