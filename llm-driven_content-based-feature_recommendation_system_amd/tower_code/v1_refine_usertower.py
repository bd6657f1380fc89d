"""Drop-in for tower_code/v1_refine_usertower.py: SASRecUserTower, its input producer
(FeatureProcessor, SASRecDataset) and its losses.

Same constructor arguments, parameter names/shapes/init (so state_dicts load both ways)
and forward signature as the reference; the forward runs on the MI355X kernels of
librecsys_amd.so:
  * embedding stage (gathers + gated sum + pos + LayerNorm + dropout): rsx_seq_embed_*
  * token linears (item_proj, in/out_proj, FFN with GELU + dropout epilogues, static MLP,
    output_proj): rsx_gemm_x3 (bf16x3 products, fp32 accumulation; out_proj fused with the
    residual add + LayerNorm, output_proj[0]'s per-user profile half added in the epilogue),
    weight gradients on the split-K rsx_linear_wgrad_x3
  * masked self-attention core of each encoder layer:                  rsx_mha_*
  * LayerNorm (+ GELU):                                                 rsx_ln_*
  * final F.normalize:                                                  rsx_gather_rows
  * losses (no N x N materialisation; bf16x3 or fp32 MFMA products):   rsx_nce_*
RSX_GEMM_PRECISION=fp32 / ops.set_gemm_precision("fp32") puts the token linears on exact fp32
products (the library GEMM) instead.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import ops


def get_logq_probs(raw_probs, device="cpu"):
    """FeatureProcessor.get_logq_probs (reference :124-137) on the item-ordered raw
    probabilities: nan -> 0, + 1e-6, normalise, log; index 0 (padding) = -20. [I+1] fp32."""
    import numpy as np
    p = np.nan_to_num(np.asarray(raw_probs, dtype=np.float64), nan=0.0) + 1e-6
    p = p / p.sum()
    full = np.zeros(len(p) + 1, dtype=np.float32)
    full[1:] = np.log(p).astype(np.float32)
    full[0] = -20.0
    return torch.tensor(full, dtype=torch.float32).to(device)


def _frame(src):
    """A parquet path (the reference's pd.read_parquet) or an in-memory DataFrame (copied)."""
    import pandas as pd
    return src.copy() if isinstance(src, pd.DataFrame) else pd.read_parquet(src)


_U_BUCKET_COLS = ("age_bucket", "user_avg_price_bucket", "total_cnt_bucket", "recency_bucket")
_U_CAT_COLS = ("preferred_channel", "club_member_status_idx", "fashion_news_frequency_idx", "FN", "Active")
_U_CONT_COLS = ("price_std_scaled", "last_price_diff_scaled", "repurchase_ratio_scaled", "weekend_ratio_scaled")
_I_SIDE_COLS = ("type_id", "color_id", "graphic_id", "section_id")


class FeatureProcessor:
    """Reference FeatureProcessor (:40-137): the user / item / sequence frames (parquet paths as
    in the reference, or DataFrames), 1-based id maps (0 = padding; a validation processor
    inherits the train item map through base_processor) and the dense lookup arrays
    SASRecDataset indexes. The arrays are filled column-wise instead of by iterrows (same values:
    every user of the frame is in user2id; item rows outside item2id are skipped, missing item
    side columns give 0 as row.get(col, 0) does)."""

    def __init__(self, user_path, item_path, seq_path, base_processor=None):
        import numpy as np
        users = _frame(user_path).drop_duplicates(subset=["customer_id"]).set_index("customer_id")
        items = _frame(item_path).drop_duplicates(subset=["article_id"]).set_index("article_id")
        seqs = _frame(seq_path).set_index("customer_id")
        users.index = users.index.astype(str)
        items.index = items.index.astype(str)
        seqs.index = seqs.index.astype(str)
        self.users, self.items, self.seqs = users, items, seqs
        self.user_ids = seqs.index.tolist()
        self.user2id = {uid: i + 1 for i, uid in enumerate(users.index)}
        if base_processor is None:
            self.item_ids = items.index.tolist()
            self.item2id = {iid: i + 1 for i, iid in enumerate(self.item_ids)}
        else:
            self.item_ids = base_processor.item_ids
            self.item2id = base_processor.item2id
        self.num_items = len(self.item_ids)

        n_users = len(users) + 1
        self.u_bucket_arr = np.zeros((n_users, 4), dtype=np.int64)
        self.u_cat_arr = np.zeros((n_users, 5), dtype=np.int64)
        self.u_cont_arr = np.zeros((n_users, 4), dtype=np.float32)
        if len(users):
            rows = np.fromiter((self.user2id[u] for u in users.index), dtype=np.int64, count=len(users))
            self.u_bucket_arr[rows] = users[list(_U_BUCKET_COLS)].to_numpy(dtype=np.float64)
            self.u_cat_arr[rows] = users[list(_U_CAT_COLS)].to_numpy(dtype=np.float64)
            self.u_cont_arr[rows] = users[list(_U_CONT_COLS)].to_numpy(dtype=np.float64)
        self.i_side_arr = np.zeros((self.num_items + 1, 4), dtype=np.int64)
        known = [iid for iid in items.index if iid in self.item2id]
        if known:
            rows = np.array([self.item2id[iid] for iid in known], dtype=np.int64)
            sub = items.loc[known]
            for j, col in enumerate(_I_SIDE_COLS):
                if col in sub.columns:
                    self.i_side_arr[rows, j] = sub[col].to_numpy(dtype=np.float64)

    def get_logq_probs(self, device):
        return get_logq_probs(self.items["raw_probability"].reindex(self.item_ids).values, device)


TIME_BUCKET_BINS = (0, 3, 7, 14, 30, 60, 180, 330, 395)


class SASRecDataset(torch.utils.data.Dataset):
    """Reference SASRecDataset (:194-306), the user-side input producer of the training step
    (create_dataloaders, v1_usertower_train.py:162-184). processor: anything with user_ids,
    user2id, item2id, seqs (customer_id-indexed, columns sequence_ids / sequence_deltas),
    i_side_arr, u_bucket_arr, u_cat_arr, u_cont_arr (FeatureProcessor above).

    One sample: the customer's item ids mapped through item2id (unknown -> 0), days-ago deltas
    bucketed by np.digitize(delta, TIME_BUCKET_BINS) (1..9); train: the last max_len + 1
    purchases, input = seq[:-1], target = seq[1:], input_time = buckets[:-1] (a single purchase
    is its own target); eval: the last max_len inputs, target all 0. Left padding with 0,
    padding_mask True on pads, side ids i_side_arr[input] (pad -> row 0), the user's static
    rows through user2id (unknown user -> row 0)."""

    def __init__(self, processor, max_len=30, is_train=True):
        self.processor = processor
        self.max_len = max_len
        self.is_train = is_train
        self.user_ids = processor.user_ids

    def __len__(self):
        return len(self.user_ids)

    def __getitem__(self, idx):
        import numpy as np
        pr = self.processor
        L = self.max_len
        user_id = self.user_ids[idx]
        u = pr.user2id.get(user_id, 0)
        seq = [pr.item2id.get(item, 0) for item in pr.seqs.loc[user_id, "sequence_ids"]]
        tb = np.digitize(pr.seqs.loc[user_id, "sequence_deltas"], np.array(TIME_BUCKET_BINS), right=False).tolist()
        if self.is_train:
            seq, tb = seq[-(L + 1):], tb[-(L + 1):]
            if len(seq) > 1:
                inp, tgt, tin = seq[:-1], seq[1:], tb[:-1]
            else:
                inp, tgt, tin = seq, seq, tb
        else:
            inp, tgt, tin = seq[-L:], [], tb[-L:]
        pad = L - len(inp)
        item = np.zeros(L, dtype=np.int64)
        time_ = np.zeros(L, dtype=np.int64)
        target = np.zeros(L, dtype=np.int64)
        item[pad:] = inp
        time_[pad:] = tin
        if self.is_train:
            target[pad:] = tgt
        side = pr.i_side_arr[item]
        mask = np.zeros(L, dtype=bool)
        mask[:pad] = True
        ub, uc, ucont = pr.u_bucket_arr[u], pr.u_cat_arr[u], pr.u_cont_arr[u]
        long = torch.long
        return {
            "user_ids": user_id,
            "item_ids": torch.from_numpy(item), "target_ids": torch.from_numpy(target),
            "padding_mask": torch.from_numpy(mask), "time_bucket_ids": torch.from_numpy(time_),
            "type_ids": torch.from_numpy(side[:, 0].copy()), "color_ids": torch.from_numpy(side[:, 1].copy()),
            "graphic_ids": torch.from_numpy(side[:, 2].copy()), "section_ids": torch.from_numpy(side[:, 3].copy()),
            "age_bucket": torch.tensor(ub[0], dtype=long), "price_bucket": torch.tensor(ub[1], dtype=long),
            "cnt_bucket": torch.tensor(ub[2], dtype=long), "recency_bucket": torch.tensor(ub[3], dtype=long),
            "channel_ids": torch.tensor(uc[0], dtype=long), "club_status_ids": torch.tensor(uc[1], dtype=long),
            "news_freq_ids": torch.tensor(uc[2], dtype=long), "fn_ids": torch.tensor(uc[3], dtype=long),
            "active_ids": torch.tensor(uc[4], dtype=long),
            "cont_feats": torch.tensor(ucont, dtype=torch.float32),
        }


_ADDLN = os.environ.get("RSX_LINEAR_ADDLN", "1") != "0"


def encoder_stack(layers, x, key_pad, p, training, causal=True, seg_off=None):
    """norm_first nn.TransformerEncoderLayer stack (gelu), reference semantics
    (v1_refine_usertower.py:343-352, item_tower.py:169-182):
      x = x + drop(out_proj(mha(norm1(x)))) ; x = x + drop(linear2(drop(gelu(linear1(norm2(x))))))
    Each residual add is fused with the LayerNorm that follows it (ops.add_layer_norm; after the
    attention that add and LayerNorm run in the out-projection GEMM's epilogue,
    ops.linear_add_layer_norm, unless RSX_LINEAR_ADDLN=0), the
    first norm1 folds the residual path's gradient into its backward (ops.layer_norm_pass), the
    last residual add + dropout is one pass (ops.add_dropout); the token linears run on the
    bf16x3 GEMMs (ops.linear_tok), the feed-forward's GELU and dropout in their epilogues
    (ops.ffn)."""
    layers = list(layers)
    D = x.shape[-1]
    fused = D in (64, 128, 256)
    if fused:
        x, h = ops.layer_norm_pass(x, layers[0].norm1.weight, layers[0].norm1.bias, layers[0].norm1.eps)
    else:
        h = ops.layer_norm(x, layers[0].norm1.weight, layers[0].norm1.bias, layers[0].norm1.eps)
    for i, layer in enumerate(layers):
        sa = layer.self_attn
        a = ops.qkv_mha(h, sa.in_proj_weight, sa.in_proj_bias, key_pad, sa.num_heads, causal=causal, p_drop=p,
                        seg_off=seg_off)
        if fused and _ADDLN:
            x, h = ops.linear_add_layer_norm(x, a, sa.out_proj.weight, sa.out_proj.bias, layer.norm2.weight,
                                             layer.norm2.bias, layer.norm2.eps, p)
        else:
            a = ops.linear_tok(a, sa.out_proj.weight, sa.out_proj.bias)
            x, h = ops.add_layer_norm(x, a, layer.norm2.weight, layer.norm2.bias, layer.norm2.eps, p)
        f = ops.ffn(h, layer.linear1.weight, layer.linear1.bias, layer.linear2.weight, layer.linear2.bias, p,
                    training)
        if i + 1 < len(layers):
            nxt = layers[i + 1].norm1
            x, h = ops.add_layer_norm(x, f, nxt.weight, nxt.bias, nxt.eps, p)
        elif fused:
            x = ops.add_dropout(x, f, p, training)
        else:
            x = x + F.dropout(f, p, training)
    return x


class SASRecUserTower(nn.Module):
    """Reference: tower_code/v1_refine_usertower.py:312-510."""

    def __init__(self, args):
        super().__init__()
        self.d_model = args.d_model
        self.max_len = args.max_len
        self.dropout_rate = args.dropout

        # Module construction order == reference (:322-399), so torch.manual_seed gives
        # bit-identical initial weights.
        self.item_proj = nn.Linear(args.pretrained_dim, self.d_model)
        self.item_id_emb = nn.Embedding(args.num_items + 1, self.d_model, padding_idx=0)
        self.type_emb = nn.Embedding(args.num_prod_types + 1, self.d_model, padding_idx=0)
        self.color_emb = nn.Embedding(args.num_colors + 1, self.d_model, padding_idx=0)
        self.graphic_emb = nn.Embedding(args.num_graphics + 1, self.d_model, padding_idx=0)
        self.section_emb = nn.Embedding(args.num_sections + 1, self.d_model, padding_idx=0)
        self.pos_emb = nn.Embedding(self.max_len, self.d_model)
        self.seq_gate = nn.Parameter(torch.ones(6))
        self.static_gate = nn.Parameter(torch.ones(10))
        num_time_buckets = 12
        self.time_emb = nn.Embedding(num_time_buckets, self.d_model, padding_idx=0)
        self.emb_ln = nn.LayerNorm(self.d_model)
        self.emb_dropout = nn.Dropout(self.dropout_rate)

        encoder_layer = nn.TransformerEncoderLayer(
            d_model=self.d_model, nhead=args.nhead, dim_feedforward=self.d_model * 2, dropout=self.dropout_rate,
            activation="gelu", norm_first=True, batch_first=True)
        self.transformer_encoder = nn.TransformerEncoder(encoder_layer, num_layers=args.num_layers,
                                                         enable_nested_tensor=False)

        mid_dim, low_dim = 16, 4
        self.age_emb = nn.Embedding(11, mid_dim, padding_idx=0)
        self.price_emb = nn.Embedding(11, mid_dim, padding_idx=0)
        self.cnt_emb = nn.Embedding(11, mid_dim, padding_idx=0)
        self.recency_emb = nn.Embedding(11, mid_dim, padding_idx=0)
        self.channel_emb = nn.Embedding(4, low_dim, padding_idx=0)
        self.club_status_emb = nn.Embedding(4, low_dim, padding_idx=0)
        self.news_freq_emb = nn.Embedding(3, low_dim, padding_idx=0)
        self.fn_emb = nn.Embedding(3, low_dim, padding_idx=0)
        self.active_emb = nn.Embedding(3, low_dim, padding_idx=0)
        self.num_cont_feats = 4
        cont_proj_dim = 16
        self.cont_proj = nn.Linear(self.num_cont_feats, cont_proj_dim)
        total_static_input_dim = (mid_dim * 4) + (low_dim * 5) + cont_proj_dim
        self.static_mlp = nn.Sequential(
            nn.Linear(total_static_input_dim, self.d_model), nn.LayerNorm(self.d_model), nn.GELU(),
            nn.Dropout(self.dropout_rate))
        self.output_proj = nn.Sequential(
            nn.Linear(self.d_model * 2, self.d_model), nn.LayerNorm(self.d_model), nn.GELU(),
            nn.Linear(self.d_model, self.d_model))
        self.apply(self._init_weights)
        self.register_buffer("_seq_gate_mask", torch.tensor([1.0, 1.0, 0.0, 0.0, 0.0, 0.0]), persistent=False)

    def _init_weights(self, module):
        # reference :403-412 (note: embedding padding rows are re-initialised, i.e. non-zero)
        if isinstance(module, nn.Linear):
            nn.init.kaiming_normal_(module.weight, mode="fan_in", nonlinearity="relu")
            if module.bias is not None:
                nn.init.constant_(module.bias, 0)
        elif isinstance(module, nn.Embedding):
            nn.init.normal_(module.weight, mean=0.0, std=0.02)
        elif isinstance(module, nn.LayerNorm):
            nn.init.constant_(module.bias, 0)
            nn.init.constant_(module.weight, 1.0)

    def get_causal_mask(self, seq_len, device):
        return torch.triu(torch.ones(seq_len, seq_len, device=device, dtype=torch.bool), diagonal=1)

    def _encoder_stack(self, x, key_pad, p, seg_off=None):
        return encoder_stack(self.transformer_encoder.layers, x, key_pad, p, self.training, causal=True,
                             seg_off=seg_off)

    def forward(self, pretrained_vecs, item_ids, time_bucket_ids, type_ids, color_ids, graphic_ids, section_ids,
                age_bucket, price_bucket, cnt_bucket, recency_bucket, channel_ids, club_status_ids, news_freq_ids,
                fn_ids, active_ids, cont_feats, padding_mask=None, training_mode=True):
        B, seq_len = item_ids.shape
        p = self.dropout_rate if self.training else 0.0

        s_g = torch.sigmoid(self.seq_gate) * self._seq_gate_mask

        # Phase 1: sequence encoding (reference :447-466)
        base = ops.linear_tok(pretrained_vecs, self.item_proj.weight, self.item_proj.bias)
        x = ops.seq_embed(
            base,
            [item_ids, time_bucket_ids, type_ids, color_ids, graphic_ids, section_ids],
            [self.item_id_emb.weight, self.time_emb.weight, self.type_emb.weight, self.color_emb.weight,
             self.graphic_emb.weight, self.section_emb.weight],
            s_g, self.pos_emb.weight[:seq_len], self.emb_ln.weight, self.emb_ln.bias, eps=self.emb_ln.eps,
            p_drop=p, padding_idx=[0, 0, 0, 0, 0, 0])
        output = self._encoder_stack(x, padding_mask, p)

        user_profile_vec = self._static_profile(age_bucket, price_bucket, cnt_bucket, recency_bucket, channel_ids,
                                                club_status_ids, news_freq_ids, fn_ids, active_ids, cont_feats, p)

        # Phase 3: late fusion (reference :499-510). Training mode: Linear(cat[token, profile[user]])
        # over all B*L tokens as ops.profile_linear (the per-user profile half computed once per
        # user and added in the token GEMM's epilogue, no broadcast tensor); eval mode: the last
        # position only, one GEMM over cat(last, profile) [B, 2D].
        lin0, ln, lin3 = self.output_proj[0], self.output_proj[1], self.output_proj[3]
        D = self.d_model
        if training_mode:
            dev = output.device
            tok_user = torch.arange(B, device=dev).repeat_interleave(seq_len)
            seg = torch.arange(0, B * seq_len + 1, seq_len, device=dev)
            h = ops.profile_linear(output.reshape(B * seq_len, D), user_profile_vec, lin0.weight, lin0.bias,
                                   tok_user, seg).view(B, seq_len, -1)
        else:
            h = ops.linear_tok(torch.cat([output[:, -1, :], user_profile_vec], dim=1), lin0.weight, lin0.bias)
        h = ops.layer_norm(h, ln.weight, ln.bias, ln.eps, act=ops.ACT_GELU_ERF)
        final_vec = ops.linear_tok(h, lin3.weight, lin3.bias)
        return ops.l2_normalize(final_vec)

    def _static_profile(self, age_bucket, price_bucket, cnt_bucket, recency_bucket, channel_ids, club_status_ids,
                        news_freq_ids, fn_ids, active_ids, cont_feats, p, rows=None):
        # Phase 2: static encoding (reference :472-494) as one native call per direction
        # (ops.static_profile -> rsx_static_profile_fwd / _bwd): sigmoid(static_gate), the nine
        # gated lookups, relu(cont_proj(cont)) * u_g[9] and static_mlp (Linear 100 -> d on the
        # bf16x3 GEMM with the input zero-padded to 128 columns, LayerNorm + GELU, Dropout).
        ids = [age_bucket, price_bucket, cnt_bucket, recency_bucket, channel_ids, club_status_ids, news_freq_ids,
               fn_ids, active_ids]
        return ops.static_profile(self, ids, cont_feats, p, rows)

    def forward_packed(self, packed, pretrained_tok, tok_ids, age_bucket, price_bucket, cnt_bucket, recency_bucket,
                       channel_ids, club_status_ids, news_freq_ids, fn_ids, active_ids, cont_feats, tail_last=None):
        """Training-mode forward restricted to the tokens whose outputs the contrastive step
        reads (every valid step + the bug-compatible DuoRec "last" position of each user).

        Returns the L2-normalised outputs of those tokens [T, D] in packed (b, t) order; each
        equals the corresponding row of forward(..., training_mode=True): with left padding a
        valid query never attends to padded keys, a padded query attends to nothing, and
        every other op is per token, so dropping the other padded tokens changes no value
        the losses see. tok_ids: [item, time, type, color, graphic, section] ids per token.

        tail_last (view 1's DuoRec "last" token of each user, [B]; packed = both views, view 2's
        tokens at rows T/2 + t): return only the rows the contrastive step reads, all of view 1
        and view 2's last row per user ([T/2 + B, D], view 2's in user order). The native program
        then runs the last layer past its attention and the output head on those rows only."""
        p = self.dropout_rate if self.training else 0.0
        s_g = torch.sigmoid(self.seq_gate) * self._seq_gate_mask
        # the static profile first (its dropout seed is drawn before the tower's, on both paths)
        profile = self._static_profile(age_bucket, price_bucket, cnt_bucket, recency_bucket, channel_ids,
                                       club_status_ids, news_freq_ids, fn_ids, active_ids, cont_feats, p, packed.B)
        params = ops.tower_native_ok(self, packed, pretrained_tok) if torch.is_grad_enabled() else None
        if params is not None:
            # the same kernels in the same order as below, issued by the library in one call per
            # direction (rsx_tower_fwd / rsx_tower_bwd)
            return ops.tower_packed(self, packed, pretrained_tok, tok_ids, s_g, profile, p, params, tail_last)
        base = ops.linear_tok(pretrained_tok, self.item_proj.weight, self.item_proj.bias)
        x = ops.seq_embed(
            base, tok_ids,
            [self.item_id_emb.weight, self.time_emb.weight, self.type_emb.weight, self.color_emb.weight,
             self.graphic_emb.weight, self.section_emb.weight],
            s_g, self.pos_emb.weight, self.emb_ln.weight, self.emb_ln.bias, eps=self.emb_ln.eps, p_drop=p,
            padding_idx=[0, 0, 0, 0, 0, 0], tok_pos=packed.tok_pos, tab0_seg=getattr(packed, "item_seg", None))
        x = self._encoder_stack(x, packed.tok_pad, p, seg_off=packed.seg_off)
        lin0, ln, lin3 = self.output_proj[0], self.output_proj[1], self.output_proj[3]
        D = self.d_model
        h = ops.profile_linear(x, profile, lin0.weight, lin0.bias, packed.tok_user, packed.seg_off64)
        h = ops.layer_norm(h, ln.weight, ln.bias, ln.eps, act=ops.ACT_GELU_ERF)
        out = ops.l2_normalize(ops.linear_tok(h, lin3.weight, lin3.bias))
        if tail_last is not None:  # the per-op path computes every row and keeps the tail ones
            T1 = out.shape[0] // 2
            keep = torch.cat([torch.arange(T1, device=out.device), tail_last + T1])
            out = ops.gather_rows(out, keep, unique=True)
        return out


class PackedTokens:
    """Token selection of the contrastive step for a left-padded [B, L] batch: all valid
    positions plus, per user, the DuoRec "last" index count-1 when it falls on padding
    (v1_usertower_train.py:830-835), in row-major (b, t) order, segmented by user."""

    def __init__(self, padding_mask: torch.Tensor):
        B, L = padding_mask.shape
        dev = padding_mask.device
        valid = ~padding_mask
        cnt = valid.sum(1)
        last = (cnt - 1).clamp(min=0)
        ar = torch.arange(B, device=dev)
        need_extra = padding_mask[ar, last]
        sel = valid.clone()
        sel[ar, last] = sel[ar, last] | need_extra
        self.flat = sel.reshape(-1).nonzero().squeeze(1)             # [T] flat (b*L + t)
        self.tok_user = torch.div(self.flat, L, rounding_mode="floor")
        self.tok_pos = self.flat % L
        self.tok_pad = padding_mask.reshape(-1)[self.flat].to(torch.uint8)
        seg = torch.zeros(B + 1, device=dev, dtype=torch.int64)
        seg[1:] = torch.cumsum(torch.bincount(self.tok_user, minlength=B), 0)
        self.seg_off = seg.to(torch.int32)
        self.seg_off64 = seg
        self.valid_tok = (self.tok_pad == 0).nonzero().squeeze(1)   # loss rows (valid steps, flat order)
        pad_len = L - cnt
        self.last_tok = seg[:-1] + torch.where(need_extra, torch.zeros_like(last), last - pad_len)
        self.B, self.L = B, L

    def take(self, t: torch.Tensor) -> torch.Tensor:
        """[B, L] (or [B, L, ...]) per-position tensor -> per packed token."""
        return t.reshape((-1,) + tuple(t.shape[2:]))[self.flat]


# ==========================================
# Losses (reference :520-861). The live inbatch_corrected_logq_loss is the second
# definition (:826); the first (:520) is shadowed at import time in the reference too.
# ==========================================
def _as_keys(t):
    return t.reshape(-1).to(torch.int32)


def inbatch_corrected_logq_loss(user_emb, item_tower_emb, target_ids, user_ids, log_q_tensor, temperature=0.1,
                                lambda_logq=1.0):
    """Reference :826-861. item_tower_emb is the (already normalised) full item matrix."""
    tgt = target_ids.reshape(-1)
    batch_item_emb = ops.gather_rows(item_tower_emb, tgt)
    bias = None
    if lambda_logq > 0.0:
        bias = log_q_tensor[tgt] * lambda_logq
    k1 = _as_keys(tgt)
    k2 = _as_keys(user_ids)
    return ops.nce_loss(user_emb, batch_item_emb, bias, k1, k1, k2, k2, tau=temperature,
                        flags=ops.NCE_MASK_ITEM_USER)


def inbatch_corrected_logq_loss_no_user(user_emb, item_tower_emb, target_ids, log_q_tensor, temperature=0.1,
                                        lambda_logq=1.0):
    """The shadowed first definition (reference :520-573): same-item masking only."""
    tgt = target_ids.reshape(-1)
    batch_item_emb = ops.gather_rows(item_tower_emb, tgt)
    bias = log_q_tensor[tgt] * lambda_logq if lambda_logq > 0.0 else None
    k1 = _as_keys(tgt)
    return ops.nce_loss(user_emb, batch_item_emb, bias, k1, k1, tau=temperature, flags=ops.NCE_MASK_ITEM)


def duorec_loss_refined(user_emb_1, user_emb_2, target_ids, temperature=0.1, lambda_sup=0.1):
    """Reference :576-627 (InfoNCE between views + lambda_sup * SupCon on same targets)."""
    z_i = ops.l2_normalize(user_emb_1)
    z_j = ops.l2_normalize(user_emb_2)
    loss_unsup = ops.nce_loss(z_i, z_j, tau=temperature, flags=ops.NCE_PLAIN)
    if lambda_sup > 0:
        k = _as_keys(target_ids)
        loss_sup = ops.nce_loss(z_i, z_i, None, k, k, tau=temperature, flags=ops.NCE_SUPCON)
        return loss_unsup + lambda_sup * loss_sup
    return loss_unsup + lambda_sup * torch.zeros((), device=z_i.device)


def _hnm_rows(user_emb, item_tower_emb, target_ids):
    """u_norm, normalize(item_tower_emb[target_ids]) (reference :642-643, 706-707, 777-778)."""
    return ops.l2_normalize(user_emb), ops.gather_rows(item_tower_emb, target_ids, normalize=True)


def _hnm_logits(u, it, cols, target_ids, log_q_tensor, temperature, lambda_logq):
    """logits[i, c] = cos(u_i, it_cols[i, c]) / tau - lambda_logq * logQ[target[cols[i, c]]]
    for a [N, C] column-index table (the reference's torch.gather over the N x N logits,
    :675-680, 735-741): only the N x C gathered entries are formed, with autograd to u and it."""
    cos = torch.einsum("nd,ncd->nc", u, it[cols])
    logits = cos / temperature
    if lambda_logq > 0.0:
        logits = logits - log_q_tensor[target_ids][cols] * lambda_logq
    return logits


def inbatch_hnm_corrected_loss_with_stats(user_emb, item_tower_emb, target_ids, log_q_tensor, top_k_percent=0.01,
                                          hnm_threshold=0.90, temperature=0.1, lambda_logq=0.7, lambda_cl=0.2):
    """Reference :632-692. Hard negatives mined on the masked cosines / tau by rsx_hnm_mine
    (no N x N tensors); k = max(1, min(floor((N-1) * top_k_percent), min_i available_i)) —
    the kernel returns the sorted top floor((N-1) p) and the per-row available counts, so the
    reference's host sync on available_negs.min() becomes a slice. Loss = CE over
    [positive, k hard negatives] with the LogQ correction applied after selection.
    lambda_cl is accepted and unused, as in the reference."""
    N = user_emb.size(0)
    device = user_emb.device
    tgt = target_ids.reshape(-1)
    u, it = _hnm_rows(user_emb, item_tower_emb, tgt)
    k_cap = int((N - 1) * top_k_percent)
    top_idx, top_cos, avail = ops.hnm_mine(u, it, tgt, max(1, min(k_cap, N)), hnm_threshold, temperature)
    num_k = max(1, min(k_cap, int(avail.min().item())))
    top_idx, top_cos = top_idx[:, :num_k], top_cos[:, :num_k]
    diag = torch.arange(N, device=device).unsqueeze(1)
    final_logits = _hnm_logits(u, it, torch.cat([diag, top_idx], dim=1), tgt, log_q_tensor, temperature,
                               lambda_logq)
    loss = F.cross_entropy(final_logits, torch.zeros(N, dtype=torch.long, device=device))
    return loss, {"avg_hn_similarity": top_cos.mean().item(), "num_active_hard_negs": num_k}


def inbatch_mixed_hnm_loss_with_stats(user_emb, item_tower_emb, target_ids, log_q_tensor, top_k_percent=0.01,
                                      random_sample_size=100, hnm_threshold=0.90, temperature=0.1, lambda_logq=0.7):
    """Reference :695-757: k = max(1, floor((N-1) p)) mined hard negatives (rsx_hnm_mine) plus
    random_sample_size uniform column draws per row (torch.randint(0, N, (N, M)) on the same
    device, so the same generator state draws the same columns), random draws that hit an
    ignored column (same target, or item cosine > hnm_threshold off the diagonal) get -1e9.
    Rows with fewer than k available negatives pick -inf-valued columns in ascending index
    order (torch.topk leaves that order unspecified)."""
    N = user_emb.size(0)
    device = user_emb.device
    tgt = target_ids.reshape(-1)
    u, it = _hnm_rows(user_emb, item_tower_emb, tgt)
    num_k = max(1, int((N - 1) * top_k_percent))
    # the random draws first (same generator use as the reference: randint after mining does
    # not consume from the GPU generator in between), so the mining kernel can also report its
    # ignore decision at exactly those columns: the reference derives both masks from one
    # ignore_mask (:719, :746), so a draw is masked iff the miner ignores that column
    random_indices = torch.randint(0, N, (N, random_sample_size), device=device)
    top_idx, top_cos, _, random_mask = ops.hnm_mine(u, it, tgt, num_k, hnm_threshold, temperature,
                                                    ignored_at=random_indices)
    diag = torch.arange(N, device=device).unsqueeze(1)
    cols = torch.cat([diag, top_idx, random_indices], dim=1)
    final_logits = _hnm_logits(u, it, cols, tgt, log_q_tensor, temperature, lambda_logq)
    with torch.no_grad():
        fill = torch.zeros_like(final_logits, dtype=torch.bool)
        fill[:, 1 + num_k:] = random_mask
    final_logits = final_logits.masked_fill(fill, -1e9)
    loss = F.cross_entropy(final_logits, torch.zeros(N, dtype=torch.long, device=device))
    return loss, {"avg_hn_similarity": top_cos.mean().item(), "num_hard": num_k, "num_random": random_sample_size}


def full_batch_hard_emphasis_loss(user_emb, item_tower_emb, target_ids, log_q_tensor, top_k_percent=0.01,
                                  hard_margin=0.2, hnm_threshold=0.90, temperature=0.1, lambda_logq=1.0):
    """Reference :762-822 (the loss of train_user_tower, v1_usertower_train.py:459-469).
    Cosine logits over the batch, ignore mask (same item, or item-item cosine > hnm_threshold off the
    diagonal), top-k hard negatives (k = max(1, floor((N-1) * top_k_percent))) mined on the masked cosines
    get +margin/tau, same-item off-diagonal columns -> -inf, CE against the diagonal. Column rows are
    gathered + L2-normalised by rsx_gather_rows, the mining (both products, mask, top-k) is the fused
    rsx_hnm_mine kernel, and the cross-entropy is ops.nce_emphasis_loss: the dense masked InfoNCE pass
    plus an O(N k) correction for the mined columns' margin -- no N x N tensor in either direction.
    Returns (loss, {"avg_hn_similarity", "num_hard"})."""
    N = user_emb.size(0)
    tgt = target_ids.reshape(-1)
    u, it = _hnm_rows(user_emb, item_tower_emb, tgt)
    num_k = max(1, int((N - 1) * top_k_percent))
    top_idx, top_cos, _ = ops.hnm_mine(u, it, tgt, num_k, hnm_threshold, 1.0)
    bias = log_q_tensor[tgt] * lambda_logq if lambda_logq > 0.0 else None
    loss = ops.nce_emphasis_loss(u, it, tgt, top_idx, hard_margin / temperature, bias=bias, tau=temperature)
    return loss, {"avg_hn_similarity": top_cos.mean().item(), "num_hard": num_k}
