"""CPU restatement of SASRecUserTower (tower_code/v1_refine_usertower.py:312-510),
the user-tower losses (:520-861) and the contrastive step (tower_code/v1_usertower_train.py:717-893).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned).
"""
from __future__ import annotations

import math

import torch
import torch.nn as nn
import torch.nn.functional as F


class OracleUserTower(nn.Module):
    """Same parameters, names and init order as the reference constructor (:313-412)."""

    def __init__(self, args, explicit_attention: bool = True):
        super().__init__()
        self.d_model = args.d_model
        self.max_len = args.max_len
        self.dropout_rate = args.dropout
        self.explicit_attention = explicit_attention
        d = self.d_model
        self.item_proj = nn.Linear(args.pretrained_dim, d)                       # :322
        self.item_id_emb = nn.Embedding(args.num_items + 1, d, padding_idx=0)    # :323
        self.type_emb = nn.Embedding(args.num_prod_types + 1, d, padding_idx=0)  # :325
        self.color_emb = nn.Embedding(args.num_colors + 1, d, padding_idx=0)
        self.graphic_emb = nn.Embedding(args.num_graphics + 1, d, padding_idx=0)
        self.section_emb = nn.Embedding(args.num_sections + 1, d, padding_idx=0)
        self.pos_emb = nn.Embedding(self.max_len, d)                              # :330
        self.seq_gate = nn.Parameter(torch.ones(6))                               # :332
        self.static_gate = nn.Parameter(torch.ones(10))                           # :335
        self.time_emb = nn.Embedding(12, d, padding_idx=0)                        # :337-338
        self.emb_ln = nn.LayerNorm(d)
        self.emb_dropout = nn.Dropout(self.dropout_rate)
        layer = nn.TransformerEncoderLayer(d_model=d, nhead=args.nhead, dim_feedforward=d * 2,
                                           dropout=self.dropout_rate, activation="gelu", norm_first=True,
                                           batch_first=True)                      # :343-351
        self.transformer_encoder = nn.TransformerEncoder(layer, num_layers=args.num_layers,
                                                         enable_nested_tensor=False)
        self.age_emb = nn.Embedding(11, 16, padding_idx=0)                        # :361-364
        self.price_emb = nn.Embedding(11, 16, padding_idx=0)
        self.cnt_emb = nn.Embedding(11, 16, padding_idx=0)
        self.recency_emb = nn.Embedding(11, 16, padding_idx=0)
        self.channel_emb = nn.Embedding(4, 4, padding_idx=0)                      # :368-372
        self.club_status_emb = nn.Embedding(4, 4, padding_idx=0)
        self.news_freq_emb = nn.Embedding(3, 4, padding_idx=0)
        self.fn_emb = nn.Embedding(3, 4, padding_idx=0)
        self.active_emb = nn.Embedding(3, 4, padding_idx=0)
        self.num_cont_feats = 4
        self.cont_proj = nn.Linear(4, 16)                                         # :378
        self.static_mlp = nn.Sequential(nn.Linear(100, d), nn.LayerNorm(d), nn.GELU(),
                                        nn.Dropout(self.dropout_rate))            # :384-389
        self.output_proj = nn.Sequential(nn.Linear(2 * d, d), nn.LayerNorm(d), nn.GELU(),
                                         nn.Linear(d, d))                          # :394-399
        self.apply(self._init_weights)                                             # :401

    @staticmethod
    def _init_weights(module):  # :403-412
        if isinstance(module, nn.Linear):
            nn.init.kaiming_normal_(module.weight, mode="fan_in", nonlinearity="relu")
            if module.bias is not None:
                nn.init.constant_(module.bias, 0)
        elif isinstance(module, nn.Embedding):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
        elif isinstance(module, nn.LayerNorm):
            nn.init.constant_(module.bias, 0)
            nn.init.constant_(module.weight, 1.0)

    def _attention(self, layer, h, padding_mask):
        """Explicit training-path MHA: bool masks -> -inf, fully-masked rows -> zero probs."""
        sa = layer.self_attn
        B, L, d = h.shape
        H = sa.num_heads
        dh = d // H
        qkv = F.linear(h, sa.in_proj_weight, sa.in_proj_bias)
        q, k, v = qkv.split(d, dim=-1)
        q = q.view(B, L, H, dh).transpose(1, 2)
        k = k.view(B, L, H, dh).transpose(1, 2)
        v = v.view(B, L, H, dh).transpose(1, 2)
        s = (q @ k.transpose(-1, -2)) / math.sqrt(dh)
        blocked = torch.triu(torch.ones(L, L, dtype=torch.bool), 1).unsqueeze(0)  # :413-415
        if padding_mask is not None:
            blocked = blocked | padding_mask[:, None, :]
        s = s.masked_fill(blocked[:, None], float("-inf"))
        p = torch.softmax(s, dim=-1)
        p = torch.nan_to_num(p, nan=0.0)  # training-path (safe softmax) semantics
        p = F.dropout(p, self.dropout_rate, self.training)
        o = (p @ v).transpose(1, 2).reshape(B, L, d)
        return F.linear(o, sa.out_proj.weight, sa.out_proj.bias)

    def _encode(self, x, padding_mask):
        if not self.explicit_attention:
            causal = torch.triu(torch.ones(x.shape[1], x.shape[1], dtype=torch.bool), 1)
            return self.transformer_encoder(x, mask=causal, src_key_padding_mask=padding_mask)
        for layer in self.transformer_encoder.layers:
            a = self._attention(layer, layer.norm1(x), padding_mask)
            x = x + layer.dropout1(a)
            f = layer.linear2(layer.dropout(F.gelu(layer.linear1(layer.norm2(x)))))
            x = x + layer.dropout2(f)
        return x

    def forward(self, pretrained_vecs, item_ids, time_bucket_ids, type_ids, color_ids, graphic_ids, section_ids,
                age_bucket, price_bucket, cnt_bucket, recency_bucket, channel_ids, club_status_ids, news_freq_ids,
                fn_ids, active_ids, cont_feats, padding_mask=None, training_mode=True):
        seq_len = item_ids.size(1)
        s_g = torch.sigmoid(self.seq_gate) * torch.tensor([1.0, 1.0, 0.0, 0.0, 0.0, 0.0])  # :434-438
        u_g = torch.sigmoid(self.static_gate) * torch.ones(10)                             # :435-442
        x = self.item_proj(pretrained_vecs)                                                # :447
        x += self.item_id_emb(item_ids) * s_g[0]
        x += self.time_emb(time_bucket_ids) * s_g[1]
        x += self.type_emb(type_ids) * s_g[2]
        x += self.color_emb(color_ids) * s_g[3]
        x += self.graphic_emb(graphic_ids) * s_g[4]
        x += self.section_emb(section_ids) * s_g[5]
        x += self.pos_emb(torch.arange(seq_len).unsqueeze(0))                               # :455-456
        x = self.emb_dropout(self.emb_ln(x))                                               # :458-459
        output = self._encode(x, padding_mask)                                             # :461-466
        static_input = torch.cat([                                                          # :472-491
            self.age_emb(age_bucket) * u_g[0], self.price_emb(price_bucket) * u_g[1],
            self.cnt_emb(cnt_bucket) * u_g[2], self.recency_emb(recency_bucket) * u_g[3],
            self.channel_emb(channel_ids) * u_g[4], self.club_status_emb(club_status_ids) * u_g[5],
            self.news_freq_emb(news_freq_ids) * u_g[6], self.fn_emb(fn_ids) * u_g[7],
            self.active_emb(active_ids) * u_g[8], F.relu(self.cont_proj(cont_feats)) * u_g[9]], dim=1)
        profile = self.static_mlp(static_input)                                             # :494
        if training_mode:                                                                    # :499-504
            fused = torch.cat([output, profile.unsqueeze(1).expand(-1, seq_len, -1)], dim=-1)
        else:                                                                                # :505-510
            fused = torch.cat([output[:, -1, :], profile], dim=-1)
        return F.normalize(self.output_proj(fused), p=2, dim=-1)

    def embedding_stage(self, pretrained_vecs, item_ids, time_bucket_ids, type_ids, color_ids, graphic_ids,
                        section_ids, with_ln=True):
        """Pre-encoder activations (:447-459) for kernel-level parity tests."""
        seq_len = item_ids.size(1)
        s_g = torch.sigmoid(self.seq_gate) * torch.tensor([1.0, 1.0, 0.0, 0.0, 0.0, 0.0])
        x = self.item_proj(pretrained_vecs)
        x += self.item_id_emb(item_ids) * s_g[0]
        x += self.time_emb(time_bucket_ids) * s_g[1]
        x += self.type_emb(type_ids) * s_g[2]
        x += self.color_emb(color_ids) * s_g[3]
        x += self.graphic_emb(graphic_ids) * s_g[4]
        x += self.section_emb(section_ids) * s_g[5]
        x += self.pos_emb(torch.arange(seq_len).unsqueeze(0))
        return self.emb_ln(x) if with_ln else x


# ---------------------------------------------------------------- losses (materialised N x N)
def inbatch_corrected_logq_loss(user_emb, item_tower_emb, target_ids, user_ids, log_q_tensor, temperature=0.1,
                                lambda_logq=1.0):
    """Live definition, v1_refine_usertower.py:826-861."""
    n = user_emb.size(0)
    logits = torch.matmul(user_emb, item_tower_emb[target_ids].T)
    logits.div_(temperature)
    if lambda_logq > 0.0:
        logits = logits - log_q_tensor[target_ids].view(1, -1) * lambda_logq
    same_item = target_ids.unsqueeze(1) == target_ids.unsqueeze(0)
    same_user = user_ids.unsqueeze(1) == user_ids.unsqueeze(0)
    diag = torch.eye(n, dtype=torch.bool)
    logits.masked_fill_((same_item | same_user) & ~diag, float("-inf"))
    return F.cross_entropy(logits, torch.arange(n))


def inbatch_corrected_logq_loss_chunked(user_emb, item_tower_emb, target_ids, user_ids, log_q_tensor,
                                        temperature=0.1, lambda_logq=1.0, chunk=2048):
    """inbatch_corrected_logq_loss (v1_refine_usertower.py:826-861) over row chunks of the N x N
    logits, each chunk under activation checkpointing: the same per-element arithmetic (matmul,
    /tau, - logQ per column, -inf off-diagonal same-item / same-user mask, CE), with the mean taken
    as the sum of chunk sums / N. Bounded RAM (chunk x N floats) at the sizes where the reference's
    one-shot N x N tensors do not fit (N ~ 153k valid steps at batch 8192)."""
    from torch.utils.checkpoint import checkpoint
    n = user_emb.size(0)
    cols = item_tower_emb[target_ids]
    bias = log_q_tensor[target_ids].view(1, -1) * lambda_logq if lambda_logq > 0.0 else None

    def part(u, c, r0):
        r1 = r0 + u.size(0)
        logits = torch.matmul(u, c.T)
        logits.div_(temperature)
        if bias is not None:
            logits = logits - bias
        mask = (target_ids[r0:r1].unsqueeze(1) == target_ids.unsqueeze(0)) | \
               (user_ids[r0:r1].unsqueeze(1) == user_ids.unsqueeze(0))
        rows = torch.arange(r1 - r0, device=u.device)
        mask[rows, rows + r0] = False
        logits.masked_fill_(mask, float("-inf"))
        return F.cross_entropy(logits, rows + r0, reduction="sum")

    total = user_emb.new_zeros(())
    for r0 in range(0, n, chunk):
        total = total + checkpoint(part, user_emb[r0:r0 + chunk], cols, r0, use_reentrant=False)
    return total / n


def inbatch_corrected_logq_loss_no_user(user_emb, item_tower_emb, target_ids, log_q_tensor, temperature=0.1,
                                        lambda_logq=1.0):
    """Shadowed first definition, v1_refine_usertower.py:520-573."""
    n = user_emb.size(0)
    logits = torch.matmul(user_emb, item_tower_emb[target_ids].T)
    logits.div_(temperature)
    if lambda_logq > 0.0:
        logits = logits - log_q_tensor[target_ids].view(1, -1) * lambda_logq
    same_item = target_ids.unsqueeze(1) == target_ids.unsqueeze(0)
    logits.masked_fill_(same_item & ~torch.eye(n, dtype=torch.bool), float("-inf"))
    return F.cross_entropy(logits, torch.arange(n))


def duorec_loss_refined(user_emb_1, user_emb_2, target_ids, temperature=0.1, lambda_sup=0.1):
    """v1_refine_usertower.py:576-627."""
    b = user_emb_1.size(0)
    z_i = F.normalize(user_emb_1, dim=1)
    z_j = F.normalize(user_emb_2, dim=1)
    loss_unsup = F.cross_entropy(torch.matmul(z_i, z_j.T) / temperature, torch.arange(b))
    loss_sup = torch.tensor(0.0)
    if lambda_sup > 0:
        t = target_ids.view(-1, 1)
        mask = torch.eq(t, t.T).float() * (1 - (t == 0).float())
        mask.fill_diagonal_(0)
        if mask.sum() > 0:
            logits_sup = torch.matmul(z_i, z_i.T) / temperature
            diag = torch.eye(b).bool()
            logits_sup.masked_fill_(diag, float("-inf"))
            log_prob = F.log_softmax(logits_sup, dim=1).masked_fill(diag, 0.0)
            valid = mask.sum(1) > 0
            if valid.sum() > 0:
                loss_sup = (-(mask[valid] * log_prob[valid]).sum(1) / mask[valid].sum(1)).mean()
    return loss_unsup + lambda_sup * loss_sup


def simcse_item_loss(emb1, emb2, temperature=0.08):
    """Item-tower SimCSE loss, item_tower.py:1075-1082."""
    sim = torch.matmul(emb1, emb2.T) / temperature
    labels = torch.arange(emb1.size(0))
    return (F.cross_entropy(sim, labels) + F.cross_entropy(sim.T, labels)) / 2


# ---------------------------------------------------------------- step
_FWD_KEYS = ("item_ids", "time_bucket_ids", "type_ids", "color_ids", "graphic_ids", "section_ids", "age_bucket",
             "price_bucket", "cnt_bucket", "recency_bucket", "channel_ids", "club_status_ids", "news_freq_ids",
             "fn_ids", "active_ids", "cont_feats", "padding_mask")


def contrastive_losses(model, item_matrix, log_q_tensor, batch, pretrained_lookup, lambda_logq=1.0,
                       lambda_sup=0.1, lambda_cl=0.2, loss_chunk=None):
    """Forward part of train_user_tower_all_time, v1_usertower_train.py:757-845 (fp32, no AMP).
    loss_chunk: evaluate the main loss row-chunked (inbatch_corrected_logq_loss_chunked)."""
    kw = {k: batch[k] for k in _FWD_KEYS}
    kw["pretrained_vecs"] = pretrained_lookup[batch["item_ids"]]                  # :760
    kw["training_mode"] = True
    out1 = model(**kw)                                                             # :788
    out2 = model(**kw)                                                             # :789
    padding_mask, target_ids = batch["padding_mask"], batch["target_ids"]
    valid = ~padding_mask                                                          # :794
    bsz, seq_len = batch["item_ids"].shape
    flat_output = out1[valid]
    flat_targets = target_ids[valid]
    flat_user_ids = torch.arange(bsz).unsqueeze(1).expand(-1, seq_len)[valid]      # :803-804
    if flat_output.size(0) > 0:
        kw = {"chunk": loss_chunk} if loss_chunk else {}
        fn = inbatch_corrected_logq_loss_chunked if loss_chunk else inbatch_corrected_logq_loss
        main = fn(F.normalize(flat_output, p=2, dim=1), F.normalize(item_matrix, p=2, dim=1), flat_targets,
                  flat_user_ids, log_q_tensor, temperature=0.1, lambda_logq=lambda_logq, **kw)
    else:
        main = torch.tensor(0.0)
    last = (valid.sum(dim=1) - 1).clamp(min=0)                                     # :830
    br = torch.arange(bsz)
    cl = duorec_loss_refined(out1[br, last], out2[br, last], target_ids[br, last], lambda_sup=lambda_sup)
    return main + lambda_cl * cl, main, cl


def contrastive_step(model, item_matrix_param, log_q_tensor, batch, optimizer, pretrained_lookup, max_norm=5.0,
                     loss_chunk=None):
    """One optimiser step (:850-854, without GradScaler: fp32 on CPU)."""
    optimizer.zero_grad()
    total, main, cl = contrastive_losses(model, item_matrix_param, log_q_tensor, batch, pretrained_lookup,
                                         loss_chunk=loss_chunk)
    total.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=max_norm)
    optimizer.step()
    return total.detach(), main.detach(), cl.detach()


def full_batch_hard_emphasis_loss(user_emb, item_tower_emb, target_ids, log_q_tensor, top_k_percent=0.01,
                                  hard_margin=0.2, hnm_threshold=0.90, temperature=0.1, lambda_logq=1.0):
    """v1_refine_usertower.py:762-822, restated (CPU fp32)."""
    N = user_emb.size(0)
    u_norm = F.normalize(user_emb, p=2, dim=1)
    i_norm = F.normalize(item_tower_emb[target_ids], p=2, dim=1)
    cos_sim = u_norm @ i_norm.T
    same = target_ids.unsqueeze(1) == target_ids.unsqueeze(0)
    diag = torch.eye(N, dtype=torch.bool)
    ignore = same | ((i_norm @ i_norm.T > hnm_threshold) & ~diag)
    with torch.no_grad():
        mining = cos_sim.detach().clone().masked_fill_(ignore, float("-inf"))
        num_k = max(1, int((N - 1) * top_k_percent))
        _, top_k_indices = torch.topk(mining, k=num_k, dim=1)
    logits = cos_sim / temperature
    if lambda_logq > 0.0:
        logits = logits - log_q_tensor[target_ids].view(1, -1) * lambda_logq
    emphasis = torch.zeros_like(logits, dtype=torch.bool)
    emphasis.scatter_(1, top_k_indices, True)
    logits = logits + emphasis.float() * (hard_margin / temperature)
    logits = logits.masked_fill(same & ~diag, float("-inf"))
    loss = F.cross_entropy(logits, torch.arange(N))
    avg = torch.gather(cos_sim, 1, top_k_indices).mean().item()
    return loss, {"avg_hn_similarity": avg, "num_hard": num_k}


def inbatch_hnm_corrected_loss_with_stats(user_emb, item_tower_emb, target_ids, log_q_tensor, top_k_percent=0.01,
                                          hnm_threshold=0.90, temperature=0.1, lambda_logq=0.7, lambda_cl=0.2):
    """v1_refine_usertower.py:632-692, restated (CPU fp32)."""
    N = user_emb.size(0)
    u_norm = F.normalize(user_emb, p=2, dim=1)
    i_norm = F.normalize(item_tower_emb[target_ids], p=2, dim=1)
    cos_sim = u_norm @ i_norm.T
    same = target_ids.unsqueeze(1) == target_ids.unsqueeze(0)
    diag = torch.eye(N, dtype=torch.bool)
    with torch.no_grad():
        too_similar = (i_norm @ i_norm.T > hnm_threshold) & ~diag
    ignore = same | too_similar
    mining = (cos_sim / temperature).detach().clone().masked_fill_(ignore, float("-inf"))
    available = (~ignore).sum(dim=1)
    num_k = max(1, min(int((N - 1) * top_k_percent), available.min().item()))
    _, top_k_indices = torch.topk(mining, k=num_k, dim=1)
    logits = cos_sim / temperature
    if lambda_logq > 0.0:
        logits = logits - log_q_tensor[target_ids].view(1, -1) * lambda_logq
    final = torch.cat([torch.diagonal(logits).unsqueeze(1), torch.gather(logits, 1, top_k_indices)], dim=1)
    loss = F.cross_entropy(final, torch.zeros(N, dtype=torch.long))
    with torch.no_grad():
        avg = torch.gather(cos_sim, 1, top_k_indices).mean().item()
    return loss, {"avg_hn_similarity": avg, "num_active_hard_negs": num_k}


def inbatch_mixed_hnm_loss_with_stats(user_emb, item_tower_emb, target_ids, log_q_tensor, top_k_percent=0.01,
                                      random_sample_size=100, hnm_threshold=0.90, temperature=0.1, lambda_logq=0.7,
                                      random_indices=None):
    """v1_refine_usertower.py:695-757, restated (CPU fp32). random_indices: the [N, M] draws of
    :730 (the reference draws them with torch.randint on its device; tests replay the GPU
    draw and pass it here)."""
    N = user_emb.size(0)
    u_norm = F.normalize(user_emb, p=2, dim=1)
    i_norm = F.normalize(item_tower_emb[target_ids], p=2, dim=1)
    cos_sim = u_norm @ i_norm.T
    same = target_ids.unsqueeze(1) == target_ids.unsqueeze(0)
    diag = torch.eye(N, dtype=torch.bool)
    with torch.no_grad():
        too_similar = (i_norm @ i_norm.T > hnm_threshold) & ~diag
    ignore = same | too_similar
    mining = (cos_sim / temperature).detach().clone().masked_fill_(ignore, float("-inf"))
    num_k = max(1, int((N - 1) * top_k_percent))
    _, top_k_indices = torch.topk(mining, k=num_k, dim=1)
    if random_indices is None:
        random_indices = torch.randint(0, N, (N, random_sample_size))
    logits = cos_sim / temperature
    if lambda_logq > 0.0:
        logits = logits - log_q_tensor[target_ids].view(1, -1) * lambda_logq
    pos = torch.diagonal(logits).unsqueeze(1)
    hard = torch.gather(logits, 1, top_k_indices)
    rnd = torch.gather(logits, 1, random_indices).masked_fill(torch.gather(ignore, 1, random_indices), -1e9)
    loss = F.cross_entropy(torch.cat([pos, hard, rnd], dim=1), torch.zeros(N, dtype=torch.long))
    with torch.no_grad():
        avg = torch.gather(cos_sim, 1, top_k_indices).mean().item()
    return loss, {"avg_hn_similarity": avg, "num_hard": num_k, "num_random": random_sample_size}


def hnm_mine(u_norm, i_norm, target_ids, k, hnm_threshold=0.90, temperature=1.0):
    """The mining step shared by :641-669, :705-728, :776-790 in float64, with the total order
    the kernel promises (mining value desc, then column index asc): (top_idx, avail)."""
    u = u_norm.double()
    it = i_norm.double()
    N = u.shape[0]
    same = target_ids.unsqueeze(1) == target_ids.unsqueeze(0)
    diag = torch.eye(N, dtype=torch.bool)
    ignore = same | ((it @ it.T > hnm_threshold) & ~diag)
    mining = (u @ it.T / temperature).masked_fill(ignore, float("-inf"))
    # a stable descending sort keeps equal values in ascending column order
    order = torch.argsort(mining, dim=1, descending=True, stable=True)
    return order[:, :k], (~ignore).sum(dim=1)
