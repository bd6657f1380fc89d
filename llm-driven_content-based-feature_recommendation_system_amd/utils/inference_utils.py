"""Drop-in for utils/inference_utils.py: item-vector refresh (the pretrained_item_matrix.pt /
item_ids.pt pair the user-tower pipeline aligns against, v1_usertower_train.py:131-160).

Reference: generate_and_save_item_vectors :74-207 — encoder from get_global_encoder()
(optionally overwritten by a checkpoint, strict), every product fetched, parsed with the
tagged name (parse_db_row :13-50), sorted by product_id (the string id, as the reference
sorts it), collated one view per batch at 4 x the global batch size (1 x in safe mode), eval
forward under no_grad, concatenated, saved with torch.save. Returns (tensor [I, d] on the
CPU, ordered ids) or (None, None) on a missing checkpoint / empty source / GPU OOM.

The forward is HybridItemTower's GPU path (this package's kernels + BERT on hipBLASLt);
there is no CPU mode: safe mode only moves each batch's vectors to the host early.
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from ..item_data import SimCSECollator, parse_db_row
from .dependencies import get_global_batch_size, get_global_encoder, gpu_lock


def generate_and_save_item_vectors(db_session, save_dir: str = "models", safe_mode: bool = False,
                                   checkpoint_path: Optional[str] = None, collator: Optional[SimCSECollator] = None):
    save_tensor_path = os.path.join(save_dir, "pretrained_item_matrix.pt")
    save_ids_path = os.path.join(save_dir, "item_ids.pt")
    model = get_global_encoder()
    device = next(model.parameters()).device
    if checkpoint_path:
        if not os.path.exists(checkpoint_path):
            print(f"[Error] Checkpoint path not found: {checkpoint_path}")
            return None, None
        state = torch.load(checkpoint_path, map_location=device, weights_only=True)
        model.load_state_dict(state, strict=True)
    rows = db_session.fetch_products()
    if not rows:
        print("No products found.")
        return None, None
    items = [parse_db_row(r) for r in rows]
    items.sort(key=lambda x: x.product_id)       # string order, as the reference (:136-138)
    ordered_ids = [it.product_id for it in items]
    if collator is None:
        collator = SimCSECollator(std_vocab_size=model.std_embedding.num_embeddings)
    bs = get_global_batch_size() * (1 if safe_mode else 4)
    vecs = []
    with gpu_lock():
        was_training = model.training
        model.eval()
        try:
            with torch.no_grad():
                for i in range(0, len(items), bs):
                    inputs = [t.to(device, non_blocking=True) for t in collator.process_batch_items(items[i:i + bs], True)]
                    v = model(*inputs)
                    vecs.append(v.cpu() if safe_mode else v)
            final = torch.cat(vecs, dim=0).cpu()
            if hasattr(model, "check_inputs"):
                model.check_inputs()            # STD ids range-checked on the device
        except RuntimeError as e:
            if "out of memory" in str(e).lower():
                torch.cuda.empty_cache()
                return None, None
            raise
        finally:
            model.train(was_training)
    os.makedirs(save_dir, exist_ok=True)
    torch.save(final, save_tensor_path)
    torch.save(ordered_ids, save_ids_path)
    return final, ordered_ids
