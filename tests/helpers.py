"""Shared builders for the parity tests (oracle on CPU vs HIP path on cuda:0)."""
from __future__ import annotations

import torch

import recsys_amd  # noqa: F401
from recsys_amd import synth
from recsys_amd.tower_code.v1_usertower_train import PipelineConfig


def small_cfg(num_items=500, dropout=0.0, hash_size=50):
    return PipelineConfig(num_items=num_items, num_prod_types=hash_size, num_colors=hash_size,
                          num_graphics=hash_size, num_sections=hash_size, dropout=dropout)


def small_universe(num_items=500, seed=0, hash_size=50):
    items = synth.make_items(num_items=num_items, d=128, seed=seed)
    items.side = items.side % (hash_size + 1)
    return items


def to_dev(batch, device):
    return {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in batch.items()}


def paired_towers(cfg, device, seed=0):
    """(oracle CPU tower, HIP tower on device) with identical weights."""
    from oracle.user_tower import OracleUserTower
    from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
    torch.manual_seed(seed)
    ref = OracleUserTower(cfg)
    torch.manual_seed(seed)
    dut = SASRecUserTower(cfg)
    dut.load_state_dict(ref.state_dict())
    return ref, dut.to(device)
