"""Drop-in for APIController/controller.py: product ingest and item-to-item similarity.

Reference: ``controller_router`` (:12) with
  * POST /products/ingest (:26-58): upsert ProductCreateRequest rows (marks them un-vectorised);
  * GET /similarity/pgvector/{item_id} (:62-124): the item's stored vector, then the 50 nearest
    other items by cosine distance through pgvector's HNSW index (ef_search = 100, approximate),
    answered as {"query_item": {id, category}, "top_5_similar": [{rank_score = 1 - distance,
    raw_distance, id, category}]} (404 unknown item, 400 no vector).
Here the vector table is an ``ItemVectorIndex`` resident in HBM (the refresh endpoint's
pretrained_item_matrix.pt / item_ids.pt, or any id -> vector map), searched EXACTLY by brute
force on the GPU (rsx_retrieve_topk over the L2-normalised matrix: 47k x 128 is 24 MB, one
pass per query), same route and response shape. Ties: higher similarity first,
then lower row. The product source is the one the serving router uses (utils/dependencies).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence

import torch
from fastapi import APIRouter, Depends, HTTPException
from pydantic import BaseModel

from .. import ops
from ..utils.dependencies import get_db, gpu_lock

controller_router = APIRouter()


class ProductCreateRequest(BaseModel):
    product_id: int
    product_name: Optional[str] = None
    feature_data: Dict[str, Any]


class ItemVectorIndex:
    """id -> L2-normalised vector rows on the GPU, with an optional category per id."""

    def __init__(self, ids: Sequence, vectors: torch.Tensor, categories: Optional[Dict[Any, str]] = None,
                 device="cuda"):
        self.ids = [int(i) for i in ids]
        self.row = {pid: r for r, pid in enumerate(self.ids)}
        v = vectors.to(device=device, dtype=torch.float32)
        self.vectors = ops.l2_normalize(v.contiguous())
        self.categories = categories or {}

    @classmethod
    def from_files(cls, matrix_path: str, ids_path: str, categories=None, device="cuda"):
        """The refresh endpoint's output (utils/inference_utils.py:205-206)."""
        return cls(torch.load(ids_path, weights_only=True), torch.load(matrix_path, weights_only=True), categories,
                   device)

    def search(self, item_id: int, k: int = 50):
        """-> (query row, [(similarity, id)] of the k nearest other items), exact cosine."""
        r = self.row[int(item_id)]
        kk = min(k + 1, len(self.ids))
        sc, ix = ops.retrieve_topk(self.vectors[r:r + 1], self.vectors, kk)
        out = [(float(s), self.ids[int(i)]) for s, i in zip(sc[0].tolist(), ix[0].tolist()) if int(i) != r and i >= 0]
        return r, out[:k]


_index: Optional[ItemVectorIndex] = None


def set_vector_index(index: Optional[ItemVectorIndex]) -> None:
    global _index
    _index = index


def get_vector_index() -> Optional[ItemVectorIndex]:
    return _index


@controller_router.post("/products/ingest")
def ingest_products(payload: List[ProductCreateRequest], db=Depends(get_db)):
    try:
        rows = {int(r["product_id"]): r for r in getattr(db, "rows", [])}
        for item in payload:
            rows[item.product_id] = {"product_id": item.product_id, "feature_data": item.feature_data,
                                     "product_name": item.product_name, "is_vectorized": False}
        db.rows = list(rows.values())
        return {"status": "success", "message": f"Saved {len(payload)} items."}
    except Exception as e:
        raise HTTPException(status_code=500, detail=str(e))


@controller_router.get("/similarity/pgvector/{item_id}")
def check_similarity_pgvector(item_id: int, index: Optional[ItemVectorIndex] = Depends(get_vector_index)):
    if index is None or int(item_id) not in index.row:
        raise HTTPException(status_code=404, detail=f"Item {item_id} not found in vector table")
    with gpu_lock():
        _, hits = index.search(item_id, 50)
    if not hits:
        return {"message": "No similar items found."}
    return {"query_item": {"id": int(item_id), "category": index.categories.get(int(item_id))},
            "top_5_similar": [{"rank_score": round(s, 4), "raw_distance": round(1.0 - s, 4), "id": pid,
                               "category": index.categories.get(pid)} for s, pid in hits]}
