"""Drop-in for APIController/serving_controller.py: the serving router of the item tower.

Reference: ``serving_controller_router = APIRouter()`` (:24), mounted by main.py under
``/ai-api`` + ``/serving`` (main.py:71-72):
  * POST /train/item-tower  (:50-59) — query ``epochs=5, lr=5e-5, checkpoint_path=None``;
    encoder / projector / db / batch size injected; runs train_simcse_from_db.
  * POST /bg/inference/refresh-item-vectors  (:131-180) — query ``save_dir="models",
    checkpoint_path=None``; runs generate_and_save_item_vectors and answers a
    VectorUpdateResponse; failures -> HTTP 500 with the error text.
Same paths, parameters, response model and error mapping. GPU work on the shared global
modules is serialised with dependencies.gpu_lock() (sync endpoints run in FastAPI's thread
pool). The DB session dependency yields the registered product source (item_data.py).
"""
from __future__ import annotations

import os
from typing import Optional

import torch.nn as nn
from fastapi import APIRouter, Depends, HTTPException, status
from pydantic import BaseModel

from ..item_tower import train_simcse_from_db
from ..utils.dependencies import get_db, get_global_batch_size, get_global_encoder, get_global_projector, gpu_lock
from ..utils.inference_utils import generate_and_save_item_vectors

serving_controller_router = APIRouter()
MODEL_DIR = "models"


class VectorUpdateResponse(BaseModel):
    status: str
    message: str
    saved_path_matrix: str
    saved_path_ids: str
    item_count: int
    vector_shape: list


@serving_controller_router.post("/train/item-tower")
def train_item_tower(encoder: nn.Module = Depends(get_global_encoder),
                     projector: nn.Module = Depends(get_global_projector),
                     db=Depends(get_db),
                     batch_size: int = Depends(get_global_batch_size),
                     epochs: int = 5,
                     lr: float = 5e-5,
                     checkpoint_path: Optional[str] = None):
    with gpu_lock():
        history = train_simcse_from_db(encoder, projector, db_session=db, batch_size=batch_size, epochs=epochs,
                                       lr=lr, checkpoint_path=checkpoint_path, model_dir=MODEL_DIR)
    return {"status": "success", "epochs": epochs, "epoch_avg_loss": history}


@serving_controller_router.post("/bg/inference/refresh-item-vectors", response_model=VectorUpdateResponse)
def update_item_vectors_api(save_dir: str = "models", db=Depends(get_db), checkpoint_path: Optional[str] = None):
    try:
        final_tensor, ordered_ids = generate_and_save_item_vectors(db, save_dir, checkpoint_path=checkpoint_path)
        if final_tensor is None:
            raise HTTPException(status_code=status.HTTP_500_INTERNAL_SERVER_ERROR,
                                detail="Vector generation returned None. Check server logs.")
        return VectorUpdateResponse(status="success", message="Item vectors successfully updated and aligned.",
                                    saved_path_matrix=os.path.join(save_dir, "pretrained_item_matrix.pt"),
                                    saved_path_ids=os.path.join(save_dir, "item_ids.pt"),
                                    item_count=len(ordered_ids), vector_shape=list(final_tensor.shape))
    except Exception as e:  # the reference maps every failure (its own 500 included) to a 500
        raise HTTPException(status_code=status.HTTP_500_INTERNAL_SERVER_ERROR,
                            detail=f"Failed to update vectors: {str(e)}")
