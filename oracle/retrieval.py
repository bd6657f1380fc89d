"""CPU restatement of the retrieval step -- TEST INFRASTRUCTURE ONLY.

evaluate_model: scores = matmul(user, normalize(items).T); topk(max_k)
(tower_code/v1_usertower_train.py:672-675); ReRankingSystem.recommend :193-196.
Tie-break made explicit: higher score first, then lower item index.

retrieve_topk scores in float64 (exact for the dyadic test inputs); retrieve_topk_chunked is the
same ranking over item chunks (bounded memory at the 1M-item corpus of BASELINE configs[4]) with
a choice of score dtype: float32 is the reference's own arithmetic (an fp32 matmul, :672),
float64 the exact ranking that fp32 results are compared against.
"""
import torch

# fp32 rounding bound of a d-term dot product: |fl(u.w) - u.w| <= gamma_d ||u|| ||w||,
# gamma_d = d u / (1 - d u), u = 2^-24 (Higham, Accuracy and Stability, Lemma 3.1 / 3.4)
_U32 = 2.0 ** -24


def fp32_dot_bound(d, u_norm, w_norm):
    g = d * _U32 / (1.0 - d * _U32)
    return g * u_norm * w_norm


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


def retrieve_topk_chunked(queries, items, k, dtype=torch.float64, chunk=131072):
    """Same (score desc, index asc) ranking as retrieve_topk with scores = queries @ items.T in
    `dtype`, over item chunks. Pass 1: v_k = the k-th largest score per query (torch.topk's
    values are exact whatever order it gives ties). Pass 2: every item with score >= v_k (ties
    at v_k included) is collected and sorted by (-score, index); the first k are returned.
    Returns (scores [Q, k] in dtype, indices [Q, k] int64); k <= number of items."""
    Q, n = queries.shape[0], items.shape[0]
    assert 1 <= k <= n
    qd = queries.to(dtype)
    vals = []
    for c0 in range(0, n, chunk):
        s = qd @ items[c0:c0 + chunk].to(dtype).T
        vals.append(torch.topk(s, min(k, s.shape[1]), dim=1).values)
    vk = torch.topk(torch.cat(vals, dim=1), k, dim=1).values[:, -1:]
    cs = [[] for _ in range(Q)]
    ci = [[] for _ in range(Q)]
    for c0 in range(0, n, chunk):
        s = qd @ items[c0:c0 + chunk].to(dtype).T
        qi, ji = torch.nonzero(s >= vk, as_tuple=True)
        sv = s[qi, ji]
        for q in torch.unique(qi).tolist():
            m = qi == q
            cs[q].append(sv[m])
            ci[q].append(ji[m] + c0)
    out_s = torch.empty(Q, k, dtype=dtype)
    out_i = torch.empty(Q, k, dtype=torch.int64)
    for q in range(Q):
        s = torch.cat(cs[q])
        j = torch.cat(ci[q])
        o = torch.argsort(j, stable=True)
        s, j = s[o], j[o]
        o = torch.argsort(-s, stable=True)[:k]
        out_s[q], out_i[q] = s[o], j[o]
    return out_s, out_i
