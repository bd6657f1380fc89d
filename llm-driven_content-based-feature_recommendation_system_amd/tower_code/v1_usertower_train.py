"""Drop-in for tower_code/v1_usertower_train.py: config, item matrix, contrastive train step.

The step (`contrastive_step`) is the hot path named by BASELINE.json: two dropout views of
SASRecUserTower, the all-time-steps LogQ in-batch loss with same-item/same-user masking,
the DuoRec term on the (bug-compatible) "last" index, backward, clip_grad_norm_(5.0) and
AdamW. `train_user_tower_all_time` keeps the reference signature and loops it.
"""
from __future__ import annotations

import os
from dataclasses import dataclass

import torch
import torch.nn as nn

from .. import ops
from .v1_refine_usertower import (FeatureProcessor, PackedTokens, SASRecDataset, SASRecUserTower,  # noqa: F401
                                  duorec_loss_refined, full_batch_hard_emphasis_loss, inbatch_corrected_logq_loss,
                                  inbatch_hnm_corrected_loss_with_stats, inbatch_mixed_hnm_loss_with_stats)

try:  # the reference hard-imports wandb (v1_usertower_train.py:14); here it is optional
    import wandb  # type: ignore
except Exception:  # pragma: no cover - not installed in this image
    wandb = None


@dataclass
class PipelineConfig:
    """Reference :21-60 (paths default to local dirs instead of the author's Windows paths)."""
    base_dir: str = "localprops"
    model_dir: str = "models"
    batch_size: int = 768
    lr: float = 5e-4
    weight_decay: float = 1e-4
    epochs: int = 15
    d_model: int = 128
    max_len: int = 50
    dropout: float = 0.2
    pretrained_dim: int = 128
    nhead: int = 4
    num_layers: int = 2
    lambda_logq: float = 1.0
    lambda_sup: float = 0.1
    lambda_cl: float = 0.2
    top_k_percent: float = 0.01
    hnm_threshold: float = 0.90
    hard_margin: float = 0.01
    freeze_item_tower: bool = True
    item_tower_pth_name: str = "encoder_ep03_loss0.8129.pth"
    num_items: int = 0
    num_prod_types: int = 0
    num_colors: int = 0
    num_graphics: int = 0
    num_sections: int = 0
    num_age_groups: int = 10


class SASRecItemTower(nn.Module):
    """Reference :266-293 (learnable item matrix + log_q buffer)."""

    def __init__(self, num_items, d_model, log_q_tensor=None):
        super().__init__()
        self.item_matrix = nn.Embedding(num_items + 1, d_model, padding_idx=0)
        if log_q_tensor is not None:
            self.register_buffer("log_q", log_q_tensor)
        else:
            self.register_buffer("log_q", torch.zeros(num_items + 1))

    def get_all_embeddings(self):
        return self.item_matrix.weight

    def get_log_q(self):
        return self.log_q

    def set_freeze_state(self, freeze: bool):
        for param in self.parameters():
            param.requires_grad = not freeze

    def init_from_pretrained(self, pretrained_vecs):
        with torch.no_grad():
            self.item_matrix.weight.copy_(pretrained_vecs)


def setup_models(cfg: PipelineConfig, device, item_state_dict=None, log_q_tensor=None):
    """Reference :295-328."""
    user_tower = SASRecUserTower(cfg).to(device)
    item_tower = SASRecItemTower(num_items=cfg.num_items, d_model=cfg.d_model, log_q_tensor=log_q_tensor).to(device)
    if item_state_dict is not None:
        item_tower.load_state_dict(item_state_dict, strict=False)
    item_tower.set_freeze_state(cfg.freeze_item_tower)
    return user_tower, item_tower


_FWD_KEYS = ("item_ids", "time_bucket_ids", "type_ids", "color_ids", "graphic_ids", "section_ids", "age_bucket",
             "price_bucket", "cnt_bucket", "recency_bucket", "channel_ids", "club_status_ids", "news_freq_ids",
             "fn_ids", "active_ids", "cont_feats", "padding_mask")


def lookup_pretrained(pretrained_lookup: torch.Tensor, item_ids: torch.Tensor) -> torch.Tensor:
    """pretrained_lookup[item_ids] (reference :760 does it on the CPU + H2D; here the aligned
    matrix stays resident in HBM and rows are gathered by rsx_gather_rows)."""
    B, L = item_ids.shape
    return ops.gather_rows(pretrained_lookup, item_ids.reshape(-1)).view(B, L, -1)


_STATIC_KEYS = ("age_bucket", "price_bucket", "cnt_bucket", "recency_bucket", "channel_ids", "club_status_ids",
                "news_freq_ids", "fn_ids", "active_ids", "cont_feats")
_SEQ_ID_KEYS = ("item_ids", "time_bucket_ids", "type_ids", "color_ids", "graphic_ids", "section_ids")


def pack_inputs(batch, pretrained_vecs=None, pretrained_lookup=None):
    """The data-dependent half of packed_views (no model state): packed token sets of one view
    and of the doubled batch, and the per-token inputs of the doubled batch. Its size queries
    synchronise the host with the stream it runs on (see dist.prepare_step_index_async)."""
    pm = batch["padding_mask"]
    pk = PackedTokens(pm)
    pk2 = PackedTokens(torch.cat([pm, pm]))
    T = pk.flat.numel()
    tok_ids = [torch.cat([t, t]) for t in (pk.take(batch[k]) for k in _SEQ_ID_KEYS)]
    if tok_ids[0].is_cuda:
        pk2.item_seg = ops.sort_segments(tok_ids[0])  # item-id embedding gradient without atomics
    if pretrained_vecs is not None:
        pv_tok = pk.take(pretrained_vecs)
    else:
        pv_tok = ops.gather_rows(pretrained_lookup, tok_ids[0][:T])
    pv_tok = torch.cat([pv_tok, pv_tok])
    from ..dist import static_inputs
    return pk, pk2, tok_ids, pv_tok, static_inputs(batch)


def packed_views(model, batch, pretrained_vecs=None, pretrained_lookup=None, packed=None, tail=False):
    """Both dropout views (reference :788-789) on the packed token set of the step, run as ONE
    packed pass over the doubled batch: users b and B + b carry the same inputs, so view 1 is
    tokens [0, T) and view 2 tokens [T, 2T) of the output. The views still draw independent
    dropout masks (the kernels key their masks by token row; torch dropout is per element), and
    every kernel launch covers both views (half the launches, no per-parameter gradient adds).
    packed: pack_inputs(batch, ...) computed ahead (else computed here).
    Returns (packed tokens of one view, out_1 [T, D], out_2 [T, D]); tail: out_2 holds only each
    user's "last" row [B, D] (the only view-2 rows the losses read; forward_packed tail_last)."""
    pk, out = packed_out(model, batch, pretrained_vecs, pretrained_lookup, packed, tail=tail)
    T = pk.flat.numel()
    return pk, out[:T], out[T:]


def packed_out(model, batch, pretrained_vecs=None, pretrained_lookup=None, packed=None, tail=False):
    """packed_views without the split: (packed tokens of one view, out [2T, D]); view 2's token t
    is row T + t (for row gathers of both views in one autograd node, ops.gather_rows_multi).
    tail: out [T + B, D], view 2's "last" row of user b at row T + b."""
    if packed is None:
        packed = pack_inputs(batch, pretrained_vecs, pretrained_lookup)
    pk, pk2, tok_ids, pv_tok, static = packed
    return pk, model.forward_packed(pk2, pv_tok, tok_ids, *static, tail_last=pk.last_tok if tail else None)


def contrastive_losses(model, item_tower, log_q_tensor, batch, cfg, pretrained_vecs=None, pretrained_lookup=None):
    """Forward of one step (reference :787-845) on the packed token set. Returns (total, main, cl)."""
    device = batch["item_ids"].device
    target_ids = batch["target_ids"]
    pk, out1, out2 = packed_views(model, batch, pretrained_vecs, pretrained_lookup, tail=True)
    n_valid = pk.valid_tok.numel()
    if n_valid > 0:
        # flat_output = output_1[valid_mask] (row-major b, t); F.normalize(flat_output)
        flat_user_emb = ops.gather_rows(out1, pk.valid_tok, normalize=True, unique=True)
        flat_pos = pk.flat[pk.valid_tok]
        flat_targets = target_ids.reshape(-1)[flat_pos]
        flat_user_ids = pk.tok_user[pk.valid_tok]
        # Grouped evaluation of inbatch_corrected_logq_loss (v1_refine_usertower.py:826-861):
        # the columns normalize(item_matrix)[flat_targets] collapse onto the distinct targets
        # with exact multiplicities (see csrc/infonce.hip); same result, N/D fewer FLOPs.
        groups = ops.TargetGroups(flat_targets, flat_user_ids)
        items_d = ops.gather_rows(item_tower.get_all_embeddings(), groups.uniq, normalize=True, unique=True)
        bias = log_q_tensor[groups.uniq] * cfg.lambda_logq if cfg.lambda_logq > 0.0 else None
        main_sum, main_cnt = ops.nce_grouped_sum(flat_user_emb, items_d, bias, groups, tau=0.1, tag="main")
        main_loss = main_sum / main_cnt.clamp(min=1.0)
    else:
        main_loss = torch.zeros((), device=device)

    # DuoRec on the "last" step: count_valid - 1 (bug-compatible on left-padded rows, :830-835)
    last_output_1 = ops.gather_rows(out1, pk.last_tok, unique=True)
    last_output_2 = out2  # the tail rows: view 2's "last" row of every user, in user order
    last_targets = target_ids.reshape(-1)[pk.flat[pk.last_tok]]
    cl_loss = duorec_loss_refined(last_output_1, last_output_2, last_targets, lambda_sup=cfg.lambda_sup)
    total_loss = main_loss + cfg.lambda_cl * cl_loss
    return total_loss, main_loss, cl_loss


def contrastive_step(model, item_tower, log_q_tensor, batch, optimizer, scaler, cfg, pretrained_lookup=None,
                     max_norm=5.0, grad_sync=None):
    """One full training step (forward x2, losses, backward, clip, AdamW). No host sync
    except the valid-position count. Returns detached (total, main, cl) loss tensors.
    grad_sync: optional callable run between backward and clipping (data-parallel all-reduce)."""
    optimizer.zero_grad(set_to_none=True)
    total, main, cl = contrastive_losses(model, item_tower, log_q_tensor, batch, cfg,
                                         pretrained_vecs=batch.get("pretrained_vecs"),
                                         pretrained_lookup=pretrained_lookup)
    if scaler is not None and scaler.is_enabled():
        scaler.scale(total).backward()
        if grad_sync is not None:
            grad_sync()
        scaler.unscale_(optimizer)
        torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)
        scaler.step(optimizer)
        scaler.update()
    else:
        total.backward()
        if grad_sync is not None:
            grad_sync()
        if ops.clip_adamw_step(optimizer, ops.module_params(model), max_norm) is None:   # rsx_clip_adamw
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)
            optimizer.step()
    return total.detach(), main.detach(), cl.detach()


def _to_device(batch, device):
    return {k: (v.to(device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in batch.items()}


def train_user_tower_all_time(epoch, model, item_tower, log_q_tensor, dataloader, optimizer, scaler, cfg, device,
                              seq_labels=None, static_labels=None):
    """Reference :717-893 (same signature; wandb logging only if wandb is importable)."""
    model.train()
    total_acc = main_acc = cl_acc = 0.0
    lookup = getattr(getattr(dataloader, "dataset", None), "pretrained_lookup", None)
    if lookup is not None and lookup.device != torch.device(device):
        lookup = lookup.to(device)
    n = 0
    for batch_idx, batch in enumerate(dataloader):
        batch = _to_device(batch, device)
        total, main, cl = contrastive_step(model, item_tower, log_q_tensor, batch, optimizer, scaler, cfg,
                                           pretrained_lookup=lookup)
        total_acc += total.item()
        main_acc += main.item()
        cl_acc += cl.item()
        n += 1
        if wandb is not None and batch_idx % 100 == 0 and getattr(wandb, "run", None) is not None:
            wandb.log({"Train/Main_Loss_Step": main.item(), "Train/CL_Loss_Step": cl.item(),
                       "Step": epoch * len(dataloader) + batch_idx})
    avg = total_acc / max(n, 1)
    print(f"Epoch {epoch} Completed | Avg Total: {avg:.4f} (Main: {main_acc / max(n, 1):.4f}, "
          f"CL: {cl_acc / max(n, 1):.4f})")
    return avg


def hard_emphasis_losses(model, item_tower, log_q_tensor, batch, cfg, pretrained_lookup=None):
    """Forward of train_user_tower's step (reference :431-483): two dropout views, main loss =
    full_batch_hard_emphasis_loss on the last position of users whose last position is valid
    (tau 0.15), DuoRec on the last position. Only the last position's output is needed, so the
    tower runs with training_mode=False (same values as output[:, -1] of the full-length
    training-mode output; dropout follows model.training). Returns (total, main, cl, stats)."""
    pv = batch.get("pretrained_vecs")
    if pv is None:
        pv = lookup_pretrained(pretrained_lookup, batch["item_ids"])
    kw = {k: batch[k] for k in _SEQ_ID_KEYS + _STATIC_KEYS}
    kw["padding_mask"] = batch["padding_mask"]
    last_1 = model(pretrained_vecs=pv, training_mode=False, **kw)
    last_2 = model(pretrained_vecs=pv, training_mode=False, **kw)
    last_targets = batch["target_ids"][:, -1]
    valid = ~batch["padding_mask"][:, -1]
    vidx = valid.nonzero().squeeze(1)
    if vidx.numel() > 0:
        user = ops.l2_normalize(ops.gather_rows(last_1, vidx))
        main, stats = full_batch_hard_emphasis_loss(user, item_tower.get_all_embeddings(), last_targets[vidx],
                                                    log_q_tensor, top_k_percent=cfg.top_k_percent,
                                                    hard_margin=cfg.hard_margin, hnm_threshold=cfg.hnm_threshold,
                                                    temperature=0.15, lambda_logq=cfg.lambda_logq)
    else:
        main = torch.zeros((), device=last_1.device)
        stats = {"avg_hn_similarity": 0.0, "num_active_hard_negs": 0}
    cl = duorec_loss_refined(last_1, last_2, last_targets, lambda_sup=cfg.lambda_sup)
    return main + cfg.lambda_cl * cl, main, cl, stats


def train_user_tower(epoch, model, item_tower, log_q_tensor, dataloader, optimizer, scaler, cfg, device,
                     seq_labels=None, static_labels=None):
    """Reference train_user_tower (v1_usertower_train.py:367-540): hard-emphasis main loss on
    the last position + DuoRec; clip 5.0; AdamW. Same signature; wandb only if importable."""
    model.train()
    lookup = getattr(getattr(dataloader, "dataset", None), "pretrained_lookup", None)
    if lookup is not None and lookup.device != torch.device(device):
        lookup = lookup.to(device)
    tot = main_acc = cl_acc = 0.0
    n = 0
    for batch_idx, batch in enumerate(dataloader):
        batch = _to_device(batch, device)
        optimizer.zero_grad(set_to_none=True)
        total, main, cl, stats = hard_emphasis_losses(model, item_tower, log_q_tensor, batch, cfg, lookup)
        total.backward()
        if ops.clip_adamw_step(optimizer, ops.module_params(model), 5.0) is None:
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0)
            optimizer.step()
        tot += total.item()
        main_acc += main.item()
        cl_acc += cl.item()
        n += 1
        if wandb is not None and batch_idx % 100 == 0 and getattr(wandb, "run", None) is not None:
            wandb.log({"Train/Main_Loss_Step": main.item(), "HNM/Avg_Hard_Negative_Sim": stats.get(
                "avg_hn_similarity", 0), "Step": epoch * len(dataloader) + batch_idx})
    avg = tot / max(n, 1)
    print(f"Epoch {epoch} Completed | Avg Total: {avg:.4f} (Main: {main_acc / max(n, 1):.4f}, "
          f"CL: {cl_acc / max(n, 1):.4f})")
    return avg


def evaluate_model(model, item_tower, dataloader, target_df_path, device, processor, k_list=[20, 100, 500]):
    """Reference :548-711 (same signature and result dict {"Recall@K": percent}).
    Per batch: eval-mode tower (last position, training_mode=False), F.normalize, then the
    top-max_k items of U normalize(W)^T by rsx_retrieve_topk (no [Q, I] score matrix; ties
    -> lower item index, torch.topk leaves them unspecified). Hits are counted on the host
    against target_df's sets exactly as the reference (users with no known target skipped)."""
    import pandas as pd
    model.eval()
    item_tower.eval()
    target_df = pd.read_parquet(target_df_path)
    target_dict = target_df.set_index("customer_id")["target_ids"].to_dict()
    max_k = max(k_list)
    hits = {k: 0.0 for k in k_list}
    n_users = 0
    lookup = getattr(getattr(dataloader, "dataset", None), "pretrained_lookup", None)
    with torch.no_grad():
        items_n = ops.l2_normalize(item_tower.get_all_embeddings())
        for batch in dataloader:
            user_ids = batch["user_ids"]
            dev_batch = {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in batch.items()}
            if "pretrained_vecs" in dev_batch:
                pv = dev_batch["pretrained_vecs"]
            else:
                lk = lookup if lookup.device == torch.device(device) else lookup.to(device)
                pv = lookup_pretrained(lk, dev_batch["item_ids"])
            kw = {k: dev_batch[k] for k in _SEQ_ID_KEYS + _STATIC_KEYS}
            out = model(pretrained_vecs=pv, padding_mask=dev_batch["padding_mask"], training_mode=False, **kw)
            user = ops.l2_normalize(out)
            valid = [i for i, u in enumerate(user_ids) if u in target_dict and len(target_dict[u]) > 0]
            if not valid:
                continue
            v_idx = torch.tensor(valid, device=device)
            _, top = ops.retrieve_topk(user[v_idx], items_n, max_k)
            pred = top.cpu().numpy()
            for i, orig in enumerate(valid):
                raw = target_dict[user_ids[orig]]
                if isinstance(raw, str) or not hasattr(raw, "__iter__"):
                    raw = [raw]
                actual = set(processor.item2id[t] for t in raw if t in processor.item2id)
                if not actual:
                    continue
                n_users += 1
                for k in k_list:
                    if not actual.isdisjoint(pred[i, :k].tolist()):
                        hits[k] += 1
    res = {}
    if n_users > 0:
        for k in k_list:
            res[f"Recall@{k}"] = hits[k] / n_users * 100
    print(f"[Validation Results] Valid Users: {n_users}")
    return res


def create_dataloaders(processor, cfg: PipelineConfig, aligned_pretrained_vecs=None, is_train=True):
    """Reference :162-184: SASRecDataset(processor, cfg.max_len, is_train) with the aligned
    pretrained lookup attached (the step gathers its rows on the device), shuffled with
    drop_last for training, in order with every user for validation."""
    dataset = SASRecDataset(processor, max_len=cfg.max_len, is_train=is_train)
    dataset.pretrained_lookup = aligned_pretrained_vecs
    return torch.utils.data.DataLoader(dataset, batch_size=cfg.batch_size, shuffle=is_train, num_workers=0,
                                       pin_memory=torch.cuda.is_available(), drop_last=is_train)


def load_aligned_pretrained_embeddings(processor, model_dir, pretrained_dim):
    """Reference :131-160 (torch.load with weights_only=True)."""
    emb_path = os.path.join(model_dir, "pretrained_item_matrix.pt")
    ids_path = os.path.join(model_dir, "item_ids.pt")
    num_embeddings = processor.num_items + 1
    aligned_weight = torch.randn(num_embeddings, pretrained_dim) * 0.01
    aligned_weight[0] = 0.0
    try:
        pretrained_emb = torch.load(emb_path, map_location="cpu", weights_only=True)
        if isinstance(pretrained_emb, dict):
            pretrained_emb = pretrained_emb.get("weight", pretrained_emb.get("item_content_emb.weight"))
        pretrained_ids = torch.load(ids_path, map_location="cpu", weights_only=True)
        pretrained_map = {str(iid.item()) if isinstance(iid, torch.Tensor) else str(iid): pretrained_emb[idx]
                          for idx, iid in enumerate(pretrained_ids)}
        for i, current_id_str in enumerate(processor.item_ids):
            if current_id_str in pretrained_map:
                aligned_weight[i + 1] = pretrained_map[current_id_str]
    except Exception as e:  # same fallback as the reference
        print(f"[Warning] Failed to load Pretrained files: {e}. Using random init.")
    return aligned_weight
