"""Drop-in for temp_model/ranker_skelet.py: retrieval -> rerank.

Reference (temp_model/ranker_skelet.py):
  * FeatureEngineer :13-89, RecommendationRanker (CatBoost) :95-149, ReRankingSystem :155-237
  * the neural ranker the north star asks for (DeepFM) does not exist in the reference; it
    is specified by deepctr-torch 0.2.9 (pinned in requirements.txt:41, never imported) and
    lives here as `DeepFM`, with a CatBoost-compatible `predict_proba` wrapper.
  * CrossNet :239-272 and RankingModel (DCN-V2) :274-357 — dead code in the reference, kept
    as a second neural reranker with the same parameter names and init.
Compute: DeepFM forward = rsx_deepfm_embed + rsx_linear_fwd + rsx_linear_dot_fwd; retrieval
(user_vec @ item_vectors.T -> topk, :193-196) = rsx_retrieve_topk (see ops.retrieve_topk).
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np
import torch
import torch.nn as nn

from .. import ops


class DeepFM(nn.Module):
    """deepctr-torch-style DeepFM over F sparse fields (binary task).

    Parameter names follow deepctr-torch's module tree (embedding_dict.C{i}, linear_model.
    embedding_dict.C{i}, dnn.linears.{j}, dnn_linear, out.bias) so its checkpoints map 1:1.
    forward(X [R, F] int64) -> prob [R, 1] (as deepctr's BaseModel.forward)."""

    def __init__(self, field_vocab_sizes, embed_dim=16, dnn_hidden_units=(256, 128), init_std=1e-4, seed=1024,
                 device="cpu"):
        super().__init__()
        if embed_dim != 16:
            raise ValueError("the fused kernel is specialised for embed_dim=16 (config 3)")
        torch.manual_seed(seed)
        self.field_names = [f"C{i + 1}" for i in range(len(field_vocab_sizes))]
        self.embed_dim = embed_dim
        self.embedding_dict = nn.ModuleDict(
            {n: nn.Embedding(v, embed_dim) for n, v in zip(self.field_names, field_vocab_sizes)})
        self.linear_model = nn.Module()
        self.linear_model.embedding_dict = nn.ModuleDict(
            {n: nn.Embedding(v, 1) for n, v in zip(self.field_names, field_vocab_sizes)})
        dims = [len(field_vocab_sizes) * embed_dim] + list(dnn_hidden_units)
        self.dnn = nn.Module()
        self.dnn.linears = nn.ModuleList([nn.Linear(dims[i], dims[i + 1]) for i in range(len(dims) - 1)])
        self.dnn_linear = nn.Linear(dims[-1], 1, bias=False)
        self.out = nn.Module()
        self.out.bias = nn.Parameter(torch.zeros((1,)))
        for emb in list(self.embedding_dict.values()) + list(self.linear_model.embedding_dict.values()):
            nn.init.normal_(emb.weight, mean=0, std=init_std)
        for name, t in self.dnn.linears.named_parameters():
            if "weight" in name:
                nn.init.normal_(t, mean=0, std=init_std)
        self.to(device)

    @torch.no_grad()
    def forward(self, X):
        _, prob = self.forward_logits(X)
        return prob.unsqueeze(1)

    def _bias_value(self) -> float:
        """out.bias as a host float, read once per parameter version (no sync per forward)."""
        b = self.out.bias
        c = self.__dict__.get("_bias_cache")
        if c is None or c[0] is not b or c[1] != b._version:
            c = self.__dict__["_bias_cache"] = (b, b._version, float(b.item()))
        return c[2]

    def _param_lists(self):
        """(embedding weights, linear weights, DNN weights, DNN biases, output weight), read through
        the submodules' parameter dicts from a submodule list built once: nn.Module attribute
        lookups for the 80 tensors cost more host time per call than the fused kernel itself.
        A parameter replaced on a submodule is still seen; replacing a submodule is not supported."""
        mods = self.__dict__.get("_mod_lists")
        if mods is None:
            mods = self.__dict__["_mod_lists"] = (
                [self.embedding_dict[n] for n in self.field_names],
                [self.linear_model.embedding_dict[n] for n in self.field_names],
                list(self.dnn.linears), self.dnn_linear)
        emb, lin, dnn, out = mods
        return ([m._parameters["weight"] for m in emb], [m._parameters["weight"] for m in lin],
                [m._parameters["weight"] for m in dnn], [m._parameters["bias"] for m in dnn],
                out._parameters["weight"])

    @torch.no_grad()
    def forward_logits(self, X):
        emb, lin, ws, bs, wo = self._param_lists()
        return ops.deepfm_forward(X, emb, lin, self._bias_value(), ws, bs, wo,
                                  cache=self.__dict__.setdefault("_fused_cache", {}))

    def predict_proba(self, X) -> np.ndarray:
        """CatBoost-compatible: probability of class 1 (RecommendationRanker.predict_proba :148-149)."""
        if not torch.is_tensor(X):
            X = torch.as_tensor(np.asarray(X), dtype=torch.int64)
        dev = next(self.parameters()).device
        return self.forward_logits(X.to(dev))[1].cpu().numpy()


class FeatureEngineer:
    """Reference :13-89 (per-candidate tabular features for the CatBoost ranker)."""

    def __init__(self):
        self.cat_features = ["season", "gender", "item_category", "item_material", "item_fit", "time_of_day"]

    def create_features(self, user_meta: Dict, item_meta: Dict, two_tower_score: float, user_vector: np.ndarray,
                        item_vector: np.ndarray) -> Dict:
        inter = user_vector * item_vector
        f = {"two_tower_score": two_tower_score, "vec_prod_mean": float(np.mean(inter)),
             "vec_prod_max": float(np.max(inter)), "vec_prod_std": float(np.std(inter)),
             "season": user_meta.get("season", "unknown"), "gender": user_meta.get("gender", "unknown"),
             "user_avg_price": user_meta.get("avg_price", 0.0),
             "item_category": item_meta.get("category", "unknown"),
             "item_material": item_meta.get("material", "unknown"), "item_fit": item_meta.get("fit", "unknown"),
             "item_price": item_meta.get("price", 0)}
        f["price_diff_ratio"] = ((f["item_price"] - f["user_avg_price"]) / f["user_avg_price"]
                                 if f["user_avg_price"] > 0 else 0.0)
        return f

    def prepare_batch(self, batch_data: List[Dict]):
        import pandas as pd
        rows = []
        for d in batch_data:
            row = self.create_features(d["user_meta"], d["item_meta"], d["two_tower_score"], d["user_vector"],
                                       d["item_vector"])
            if "label" in d:
                row["target"] = d["label"]
            rows.append(row)
        return pd.DataFrame(rows)


class RecommendationRanker:
    """Reference :95-149 (CatBoost). Importable without catboost; constructing it needs it."""

    def __init__(self, model_path: str = None):
        from catboost import CatBoostClassifier  # noqa: F401  (absent in this image: raises ImportError)
        self.engineer = FeatureEngineer()
        self.model = CatBoostClassifier(iterations=1000, learning_rate=0.05, depth=6, loss_function="Logloss",
                                        eval_metric="AUC", verbose=100, early_stopping_rounds=50,
                                        cat_features=self.engineer.cat_features, random_seed=42)
        self.is_fitted = False
        if model_path:
            self.model.load_model(model_path)
            self.is_fitted = True

    def predict_proba(self, X) -> np.ndarray:
        return self.model.predict_proba(X)[:, 1]


_HASH_ITEM, _HASH_USER, _HASH_FIELD = 0x9E3779B1, 0x85EBCA77, 0xC2B2AE35


def hashed_cross_features(user_bucket: torch.Tensor, cand_ids: torch.Tensor, vocab_sizes) -> torch.Tensor:
    """Sparse DeepFM rerank ids for (user, candidate) pairs ("39 sparse ids
    per (user, item) derived by hashing (user_bucket, item_id) pairs"): field f of pair (q, j) is
    mix(item * A + bucket[q] * B + f * C) % vocab_f with mix(h) = (h ^ (h >> 29)) & 0x7FFFFFFF.
    user_bucket [Q] int64, cand_ids [Q, K] int64 -> [Q, K, F] int64."""
    F = len(vocab_sizes)
    dev = cand_ids.device
    fld = torch.arange(F, device=dev, dtype=torch.int64).view(1, 1, F)
    h = cand_ids.unsqueeze(-1) * _HASH_ITEM + user_bucket.view(-1, 1, 1) * _HASH_USER + fld * _HASH_FIELD
    voc = torch.as_tensor(list(vocab_sizes), dtype=torch.int64, device=dev).view(1, 1, F)
    return ((h ^ (h >> 29)) & 0x7FFFFFFF) % voc


class ReRankingSystem:
    """Reference :155-237: retrieval (user_vec @ item_vectors.T, top-k) then rerank.

    ranker: a DeepFM (rerank features = `rerank_features(user_vec, candidate_ids)` -> [k, F]
    int64 ids, e.g. hashed (user bucket, item) crosses) or a RecommendationRanker (CatBoost
    on FeatureEngineer rows, as the reference)."""

    def __init__(self, user_tower, item_tower, ranker, item_db_metadata: Dict[int, Dict],
                 item_db_vectors: torch.Tensor, rerank_features=None):
        self.user_tower = user_tower
        self.item_tower = item_tower
        self.ranker = ranker
        self.item_metadata = item_db_metadata
        self.item_vectors = item_db_vectors
        self.rerank_features = rerank_features
        self.device = item_db_vectors.device

    def recommend(self, user_vector: torch.Tensor, user_meta_raw: Dict = None, top_k_retrieval: int = 100,
                  final_k: int = 10):
        uv = user_vector.reshape(1, -1).to(self.device, torch.float32)
        top_scores, top_idx = ops.retrieve_topk(uv, self.item_vectors, top_k_retrieval)
        idx = top_idx[0]
        if isinstance(self.ranker, DeepFM):
            feats = self.rerank_features(uv, idx)
            probs = self.ranker.predict_proba(feats)
        else:
            rows = [{"user_meta": user_meta_raw or {}, "item_meta": self.item_metadata.get(int(i), {}),
                     "two_tower_score": float(s), "user_vector": uv[0].cpu().numpy(),
                     "item_vector": self.item_vectors[int(i)].cpu().numpy()}
                    for s, i in zip(top_scores[0].tolist(), idx.tolist())]
            probs = self.ranker.predict_proba(self.ranker.engineer.prepare_batch(rows))
        order = np.argsort(probs)[::-1][:final_k]
        idx_cpu = idx.cpu().numpy()
        sc_cpu = top_scores[0].cpu().numpy()
        return [{"product_id": int(idx_cpu[o]), "two_tower_score": float(sc_cpu[o]), "final_score": float(probs[o])}
                for o in order]

    def rerank_batch(self, cand_ids: torch.Tensor, cand_scores: torch.Tensor, user_buckets: torch.Tensor,
                     final_k: int = 10, features=None):
        """The DeepFM half of recommend for a batch of queries, on the device: candidates [Q, K]
        (global item ids) -> rerank ids (features(cand_ids, user_buckets) -> [Q, K, F]; default the
        hashed (user bucket, item) crosses of hashed_cross_features) -> DeepFM probabilities -> the
        final_k most probable per query (torch.topk: probability desc). Returns (product ids,
        two-tower scores, final scores), each [Q, final_k]."""
        if not isinstance(self.ranker, DeepFM):
            raise TypeError("rerank_batch needs a DeepFM ranker (the CatBoost path is per-user, recommend)")
        Q, K = cand_ids.shape
        if features is not None:
            feats = features(cand_ids, user_buckets)
        else:
            voc = self.__dict__.get("_vocab")
            if voc is None:
                voc = self.__dict__["_vocab"] = [self.ranker.embedding_dict[n].num_embeddings
                                                 for n in self.ranker.field_names]
            feats = hashed_cross_features(user_buckets, cand_ids, voc)
        _, prob = self.ranker.forward_logits(feats.reshape(Q * K, -1))
        top_p, top_j = torch.topk(prob.view(Q, K), final_k, dim=1)
        return torch.gather(cand_ids, 1, top_j), torch.gather(cand_scores, 1, top_j), top_p

    def recommend_batch(self, user_vectors: torch.Tensor, user_buckets: torch.Tensor = None,
                        top_k_retrieval: int = 100, final_k: int = 10):
        """recommend (reference :170-237) for a batch of users with a DeepFM ranker, entirely on the
        device: exact top-k retrieval of user_vectors [Q, D] against the item vectors
        (rsx_retrieve_topk), then rerank_batch. user_buckets [Q] int64 (default: q % 1000).
        Returns (product ids, two-tower scores, final scores), each [Q, final_k]."""
        uv = user_vectors.to(self.device, torch.float32)
        Q = uv.shape[0]
        if user_buckets is None:
            user_buckets = torch.arange(Q, device=self.device, dtype=torch.int64) % 1000
        sc, idx = ops.retrieve_topk(uv, self.item_vectors, top_k_retrieval)
        return self.rerank_batch(idx, sc, user_buckets, final_k)


class CrossNet(nn.Module):
    """Reference :239-272: x_{l+1} = x_0 * (x_l @ k_l + b_l) + x_l, k_l [D, 1] (xavier normal),
    b_l [D] (zeros). GPU forward on rsx_crossnet (one wave per row, the row in registers)."""

    def __init__(self, input_dim, num_layers=3):
        super().__init__()
        self.num_layers = num_layers
        self.kernels = nn.ParameterList([nn.Parameter(torch.nn.init.xavier_normal_(torch.empty(input_dim, 1)))
                                         for _ in range(num_layers)])
        self.biases = nn.ParameterList([nn.Parameter(torch.zeros(input_dim)) for _ in range(num_layers)])

    @torch.no_grad()
    def forward(self, x):
        x_out, _ = ops.crossnet(x, list(self.kernels), list(self.biases), want_x=True)
        return x_out


class RankingModel(nn.Module):
    """Reference :274-357 (DCN-V2 re-ranker): x = cat(user, item[, context]); cross =
    CrossNet(x, 3); deep = GELU(LN(Linear(GELU(LN(Linear(x, 256))), 128))); sigmoid(final_head(
    cat(cross, deep))). Inference on the GPU: the cross network fused with the cross half of
    final_head (rsx_crossnet: neither cross_out nor the concatenation is materialised), the deep
    linears on the fp32-MFMA kernel (rsx_linear_fwd) with the LayerNorm+GELU kernel between;
    dropout is inactive (inference)."""

    def __init__(self, user_dim=128, item_dim=128, context_dim=20):
        super().__init__()
        total_input_dim = user_dim + item_dim + context_dim
        self.cross_net = CrossNet(total_input_dim, num_layers=3)
        self.deep_net = nn.Sequential(nn.Linear(total_input_dim, 256), nn.LayerNorm(256), nn.GELU(), nn.Dropout(0.2),
                                      nn.Linear(256, 128), nn.LayerNorm(128), nn.GELU())
        self.final_head = nn.Linear(total_input_dim + 128, 1)

    @torch.no_grad()
    def forward(self, user_emb, item_emb, context_emb=None):
        parts = [user_emb, item_emb] + ([context_emb] if context_emb is not None else [])
        x = torch.cat(parts, dim=1).float().contiguous()
        D = x.shape[1]
        lin1, ln1, lin2, ln2 = self.deep_net[0], self.deep_net[1], self.deep_net[4], self.deep_net[5]
        if lin1.in_features != D:
            raise ValueError(f"input width {D} != the model's {lin1.in_features} (context given / omitted?)")
        wh = self.final_head.weight.reshape(-1)
        _, head_part = ops.crossnet(x, list(self.cross_net.kernels), list(self.cross_net.biases), w_head=wh[:D])
        h = ops.layer_norm(ops.linear(x, lin1.weight, lin1.bias), ln1.weight, ln1.bias, ln1.eps,
                           act=ops.ACT_GELU_ERF)
        h = ops.layer_norm(ops.linear(h, lin2.weight, lin2.bias), ln2.weight, ln2.bias, ln2.eps,
                           act=ops.ACT_GELU_ERF)
        logits = head_part + h @ wh[D:] + self.final_head.bias
        return torch.sigmoid(logits).unsqueeze(1)

    @torch.no_grad()
    def predict_for_user(self, user_vec, item_vecs, context_vec=None):
        """Reference :327-357: one user (and context) broadcast over N candidate items -> [N]."""
        if user_vec.dim() == 1:
            user_vec = user_vec.unsqueeze(0)
        n = item_vecs.size(0)
        ctx = None
        if context_vec is not None:
            ctx = (context_vec.unsqueeze(0) if context_vec.dim() == 1 else context_vec).expand(n, -1)
        return self.forward(user_vec.expand(n, -1), item_vecs, ctx).squeeze()
