"""CPU restatement of the reference's DCN-V2 re-ranker -- TEST INFRASTRUCTURE ONLY.

temp_model/ranker_skelet.py:239-357 (CrossNet, RankingModel, predict_for_user), dead code in
the reference (never instantiated there); restated in float64 from the source text.
Parity with the reference itself is UNPINNED (no fixtures; import denied).
"""
import torch
import torch.nn.functional as F


def crossnet(x, kernels, biases):
    """:258-272: x_l = x_0 * (x_l @ k + b) + x_l for each layer."""
    x0 = x
    xl = x
    for k, b in zip(kernels, biases):
        xl = x0 * (xl @ k.double() + b.double()) + xl
    return xl


def ranking_model_forward(model, user, item, context=None):
    """:313-338 in float64 with the model's parameters (eval: dropout off)."""
    x = torch.cat([user, item] + ([context] if context is not None else []), dim=1).double()
    cross = crossnet(x, [k for k in model.cross_net.kernels], [b for b in model.cross_net.biases])
    d = model.deep_net
    h = F.gelu(F.layer_norm(F.linear(x, d[0].weight.double(), d[0].bias.double()), (256,), d[1].weight.double(),
                            d[1].bias.double(), d[1].eps))
    h = F.gelu(F.layer_norm(F.linear(h, d[4].weight.double(), d[4].bias.double()), (128,), d[5].weight.double(),
                            d[5].bias.double(), d[5].eps))
    logits = F.linear(torch.cat([cross, h], 1), model.final_head.weight.double(), model.final_head.bias.double())
    return torch.sigmoid(logits)


# ---------------------------------------------------------------------------------------------
# configs[4] composition (ReRankingSystem.recommend, temp_model/ranker_skelet.py:170-237, with the
# north star's DeepFM as the ranker): fp32 scores + top-k (:193-196), hashed (user bucket, item)
# rerank ids, DeepFM, top final_k by probability.
_A, _B, _C = 0x9E3779B1, 0x85EBCA77, 0xC2B2AE35


def hashed_cross_features(user_bucket, cand_ids, vocab_sizes):
    """[Q, K, F] ids: field f of (q, j) = ((h ^ (h >> 29)) & 0x7FFFFFFF) % vocab_f with
    h = item * A + bucket[q] * B + f * C (int64), looped over fields."""
    outs = []
    for f, v in enumerate(vocab_sizes):
        h = cand_ids * _A + user_bucket.view(-1, 1) * _B + f * _C
        outs.append(((h ^ (h >> 29)) & 0x7FFFFFFF) % v)
    return torch.stack(outs, dim=-1)


def retrieve_rerank(users, corpus, deepfm_state, vocab_sizes, k=100, final_k=10, user_bucket=None,
                    chunk=250_000, score_dtype=torch.float32, rerank_dtype=torch.float32):
    """The composition on the CPU: scores = users @ corpus^T in score_dtype over corpus chunks, top-k
    per chunk merged (torch.topk), rerank ids, oracle/deepfm.py in rerank_dtype, top final_k.
    deepfm_state: {"emb", "lin", "bias", "ws", "bs", "wo"} host tensors.
    -> (cand_scores [Q, k], cand_ids [Q, k], probs [Q, k], top_ids [Q, final_k], top_p [Q, final_k])."""
    from oracle import deepfm as OD
    Q = users.shape[0]
    if user_bucket is None:
        user_bucket = torch.arange(Q, dtype=torch.int64) % 1000
    u = users.to(score_dtype)
    bs = bi = None
    for c0 in range(0, corpus.shape[0], chunk):
        sc = u @ corpus[c0:c0 + chunk].to(score_dtype).T
        s, i = torch.topk(sc, min(k, sc.shape[1]), dim=1)
        i = i + c0
        if bs is not None:
            s, j = torch.topk(torch.cat([bs, s], 1), k, dim=1)
            i = torch.gather(torch.cat([bi, i], 1), 1, j)
        bs, bi = s, i
    feats = hashed_cross_features(user_bucket, bi, vocab_sizes)
    st = deepfm_state
    _, prob = OD.deepfm_forward(feats.reshape(Q * k, -1), st["emb"], st["lin"], st["bias"], st["ws"], st["bs"],
                                st["wo"], dtype=rerank_dtype)
    prob = prob.view(Q, k)
    top_p, top_j = torch.topk(prob, final_k, dim=1)
    return bs, bi, prob, torch.gather(bi, 1, top_j), top_p


def compare_rerank(gpu_ids, gpu_p, cand_gpu, cand_ref, top_ref, p_ref_all, p_tol):
    """Checker of a device retrieve -> rerank result against the composition above, per query:
    the candidate SETS agree (retrieval differences are the retrieval tests' concern), and where
    they agree the final ids are the reference's, position by position, except swaps of items whose
    reference probabilities are within 2 p_tol (near-ties of the ranker's own rounding), with every
    final score within p_tol of the reference probability of the item it names.
    gpu_ids / gpu_p: [Q, final_k]; cand_*: [Q, K] ids; top_ref: [Q, final_k]; p_ref_all: [Q, K]
    reference probabilities of cand_ref. -> dict of counts (raises AssertionError on a violation)."""
    Q = gpu_ids.shape[0]
    same_set = exact = 0
    worst = 0.0
    for q in range(Q):
        if set(cand_gpu[q].tolist()) != set(cand_ref[q].tolist()):
            continue
        same_set += 1
        pmap = dict(zip(cand_ref[q].tolist(), p_ref_all[q].tolist()))
        g, o = gpu_ids[q].tolist(), top_ref[q].tolist()
        for r, (a, b) in enumerate(zip(g, o)):
            d = abs(float(gpu_p[q, r]) - pmap[a])
            worst = max(worst, d)
            assert d <= p_tol, (q, r, a, float(gpu_p[q, r]), pmap[a])
            assert a == b or abs(pmap[a] - pmap[b]) <= 2 * p_tol, (q, r, a, b, pmap[a], pmap[b])
        exact += int(g == o)
    return {"queries": Q, "same_candidate_set": same_set, "identical_top": exact, "max_abs_final_score_diff": worst}
