"""Drop-in for utils/dependencies.py: the process-wide models the serving endpoints inject.

Reference: initialize_global_models :42-72 (HybridItemTower(std_vocab_size, num_std, 128),
OptimizedItemTower(128, 128), batch size 192), get_global_encoder / get_global_projector /
get_global_batch_size :76-94 (raise if startup has not run), database.get_db (a session per
request). Here ``get_db`` yields the registered product source (item_data.InMemoryProductStore
unless a database adapter is registered with ``set_product_store``), and ``gpu_lock()``
serialises GPU work on the shared modules: FastAPI runs sync endpoints in a thread pool.
"""
from __future__ import annotations

import threading
from typing import Optional

import torch

from ..item_data import InMemoryProductStore

global_encoder = None
global_projector = None
global_batch_size: Optional[int] = None
global_product_store = InMemoryProductStore()
_gpu_lock = threading.Lock()
DEVICE = torch.device("cuda")


def initialize_global_models(std_vocab_size: Optional[int] = None, num_std_fields: Optional[int] = None,
                             embed_dim: int = 128,
                             bert_model=None, batch_size: int = 192, device=None):
    """Builds the encoder / projector on the GPU (the reference's startup hook; its sizes are
    get_std_vocab_size() = 384 and len(get_std_field_keys()) = 6)."""
    from ..item_tower import HybridItemTower, OptimizedItemTower
    from .vocab import get_std_field_keys, get_std_vocab_size
    global global_encoder, global_projector, global_batch_size
    std_vocab_size = get_std_vocab_size() if std_vocab_size is None else std_vocab_size
    num_std_fields = len(get_std_field_keys()) if num_std_fields is None else num_std_fields
    dev = torch.device(device) if device is not None else DEVICE
    global_encoder = HybridItemTower(std_vocab_size, num_std_fields, embed_dim=embed_dim,
                                     output_dim=embed_dim, bert_model=bert_model).to(dev)
    global_projector = OptimizedItemTower(input_dim=embed_dim, output_dim=embed_dim).to(dev)
    global_batch_size = batch_size


def get_global_encoder():
    if global_encoder is None:
        raise Exception("Encoder model has not been loaded yet. Check application startup events.")
    return global_encoder


def get_global_projector():
    if global_projector is None:
        raise Exception("Projector model has not been loaded yet. Check application startup events.")
    return global_projector


def get_global_batch_size() -> int:
    if global_batch_size is None:
        raise Exception("global batch size has not been defined")
    return global_batch_size


def set_product_store(store) -> None:
    """Registers the product source (anything with fetch_products() -> list of row dicts)."""
    global global_product_store
    global_product_store = store


def get_db():
    """FastAPI dependency (database.get_db's slot): yields the product source."""
    yield global_product_store


def gpu_lock() -> threading.Lock:
    return _gpu_lock
