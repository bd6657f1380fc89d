"""CPU restatement of the retrieval step -- TEST INFRASTRUCTURE ONLY.

evaluate_model: scores = matmul(user, normalize(items).T); topk(max_k)
(tower_code/v1_usertower_train.py:672-675); ReRankingSystem.recommend :193-196.
Tie-break made explicit: higher score first, then lower item index.
"""
import torch


def retrieve_topk(queries, items, k):
    scores = queries.double() @ items.double().T
    n = items.shape[0]
    # stable sort on (-score, index)
    idx = torch.arange(n).expand_as(scores)
    order = torch.argsort(idx, dim=1, stable=True)
    s2 = torch.gather(scores, 1, order)
    o2 = torch.argsort(-s2, dim=1, stable=True)
    top = torch.gather(order, 1, o2)[:, :k]
    return torch.gather(scores, 1, top), top
