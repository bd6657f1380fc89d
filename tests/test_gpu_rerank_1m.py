"""configs[4] as a composed pipeline at its size: ReRankingSystem.recommend_batch (retrieve ->
rerank, temp_model/ranker_skelet.py:170-237 with the north star's DeepFM as the ranker; the
bench's secondary_retrieve_rerank runs this same method) over the 1,000,000-item corpus for 256
queries, against the CPU composition oracle/ranker.py retrieve_rerank: fp32 scores + top-100
(the reference arithmetic, v1_usertower_train.py:672-675 / ranker_skelet.py:193-196), hashed
(user bucket, item) rerank ids, oracle/deepfm.py in float64, top-10.

* Candidates: every query's 100 candidates are checked with the 1M retrieval tests' near-tie
  criterion (an index differing from the fp32 oracle's is a near-tie within 4 eps of the fp32
  dot-product bound), and the GPU's candidate SET equals the oracle's for >= 95 % of queries.
* Rerank: where the candidate sets agree, the final top-10 ids equal the oracle's position by
  position except swaps of items whose float64 probabilities are within 2e-5, and every
  final_score is within 1e-5 of the float64 probability of the item it names.
DeepFM: 39 fields x vocab 1e6, d = 16, DNN (256, 128) -- config 3's model (deepctr-style init);
parity of DeepFM itself is unpinned (no deepctr here), the composition is what is checked."""
import pytest
import torch
import torch.nn.functional as F

import recsys_amd  # noqa: F401
from recsys_amd import ops
from recsys_amd.temp_model.ranker_skelet import DeepFM, ReRankingSystem
from oracle import ranker as ORK
from tests.test_gpu_retrieval_1m import _check_near_ties

pytestmark = pytest.mark.gpu

NI, Q, K, V, NF = 1_000_000, 256, 100, 1_000_000, 39


def _host_state(model):
    names = model.field_names
    with torch.no_grad():
        return {"emb": [model.embedding_dict[n].weight.detach().cpu() for n in names],
                "lin": [model.linear_model.embedding_dict[n].weight.detach().cpu() for n in names],
                "ws": [m.weight.detach().cpu() for m in model.dnn.linears],
                "bs": [m.bias.detach().cpu() for m in model.dnn.linears],
                "wo": model.dnn_linear.weight.detach().cpu(), "bias": float(model.out.bias.item())}


def test_recommend_batch_1m_matches_oracle_composition(gpu):
    g = torch.Generator().manual_seed(5)
    corpus = F.normalize(torch.randn(NI, 128, generator=g), dim=1)
    users = F.normalize(torch.randn(Q, 128, generator=g), dim=1)
    torch.manual_seed(3)
    model = DeepFM([V] * NF, device=gpu)
    with torch.no_grad():   # spread the probabilities beyond deepctr's 1e-4 init (fewer exact near-ties)
        for n in model.field_names:
            model.embedding_dict[n].weight.mul_(100.0)
            model.linear_model.embedding_dict[n].weight.mul_(100.0)
    sys_ = ReRankingSystem(None, None, model, {}, corpus.to(gpu))
    ug = users.to(gpu)
    buckets = torch.arange(Q, dtype=torch.int64) % 1000
    ids, tt, p = sys_.recommend_batch(ug, buckets.to(gpu), top_k_retrieval=K, final_k=10)
    sc, cand = ops.retrieve_topk(ug, sys_.item_vectors, K)         # the candidates recommend_batch reranked
    ids, tt, p, sc, cand = ids.cpu(), tt.cpu(), p.cpu(), sc.cpu(), cand.cpu()
    for q in range(Q):
        assert set(ids[q].tolist()) <= set(cand[q].tolist())
    frac, eps = _check_near_ties(users, corpus, K, sc, cand)
    cs, ci, p_all, top_ref, top_p = ORK.retrieve_rerank(users, corpus, _host_state(model), [V] * NF, k=K,
                                                        final_k=10, user_bucket=buckets,
                                                        rerank_dtype=torch.float64)
    res = ORK.compare_rerank(ids, p, cand, ci, top_ref, p_all, p_tol=1e-5)
    print(f"[retrieve->rerank 1M] {res}; candidate index mismatches vs fp32 {frac:.5f}")
    assert res["same_candidate_set"] >= int(0.95 * Q)
    assert res["identical_top"] >= int(0.9 * res["same_candidate_set"])
    # two-tower scores of the final items are their exact fp32 scores (within the fp32 dot bound)
    ex = torch.einsum("qkd,qd->qk", corpus.double()[ids], users.double())
    assert (tt.double() - ex).abs().max().item() <= eps
