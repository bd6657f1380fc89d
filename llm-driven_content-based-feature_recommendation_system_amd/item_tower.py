"""Drop-in for item_tower.py's model half: HybridItemTower, its head blocks, the SimCSE
projector / wrapper and the symmetric SimCSE loss, on the MI355X kernels.

Reference (item_tower.py):
  * SEResidualBlock :41-75, DeepResidualHead :77-128, HybridItemTower :131-286,
    OptimizedItemTower :289-305, SimCSEModelWrapper :308-322
  * SimCSE loss in train_simcse_from_db :1069-1082 (S = e1 e2^T / 0.08, CE both directions)
  * calculate_metrics :607-645 (alignment / uniformity health check)
Module trees and parameter names are the reference's, so state_dicts load unchanged.

Differences by design:
  * the BERT is injected (``bert_model=``) or built locally from a config — the reference
    downloads ``bert-base-uncased`` by name (:149-150), which has no offline equivalent;
  * forward runs the token work on this package's kernels: fused LayerNorm(+GELU), the
    token linears with split-K weight gradients, the MHA kernel (no mask, 16 field tokens)
    and the InfoNCE kernel for the loss. Under no_grad (the refresh-item-vectors inference,
    utils/inference_utils.py) the text BERT runs over the packed valid tokens
    (``bert_cls_packed``: bf16x3 GEMMs, the varlen attention kernel, fused residual+LayerNorm,
    the last layer's feed-forward on the [CLS] rows only); with gradients it stays HF's module.
``train_simcse_from_db`` keeps the reference driver's signature and loop; its ``db_session`` is
any product source with ``fetch_products()`` (item_data.py; PostgreSQL itself is out of scope)
and ``simcse_train_step`` is its per-batch GPU step.
"""
from __future__ import annotations

import contextlib
import os
from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _native as N
from . import ops
from .tower_code.v1_refine_usertower import encoder_stack

from .utils.vocab import PAD_ID, UNK_ID  # noqa: E402,F401
EMBED_DIM = 128
OUTPUT_DIM_ENCODER = 128
OUTPUT_DIM_PROJECTOR = 128


_LN_WIDTHS = (64, 128, 256, 512, 768, 1024, 2048)


def _ln(x, ln: nn.LayerNorm, gelu: bool = False):
    """LayerNorm (+ exact GELU) on the fused kernel (rsx_ln_fwd / rsx_ln_bwd: every width the
    item tower uses at d = 64 / 128, including the head's 2d, 4d and the SE blocks' 16d rows);
    another width would fall to torch's ROCm LayerNorm. GPU only: no CPU path."""
    N.ensure_device(x)
    if x.shape[-1] in _LN_WIDTHS:
        return ops.layer_norm(x, ln.weight, ln.bias, ln.eps, act=ops.ACT_GELU_ERF if gelu else 0)
    y = F.layer_norm(x, (x.shape[-1],), ln.weight, ln.bias, ln.eps)
    return F.gelu(y) if gelu else y


def _lin(x, layer: nn.Linear):
    return ops.linear_tok(x, layer.weight, layer.bias)


class SEResidualBlock(nn.Module):
    """item_tower.py:41-75: x + block(x) * sigmoid(SE(block(x)))."""

    def __init__(self, dim, dropout=0.2, expansion_factor=4):
        super().__init__()
        self.block = nn.Sequential(
            nn.Linear(dim, dim * expansion_factor), nn.LayerNorm(dim * expansion_factor), nn.GELU(),
            nn.Dropout(dropout), nn.Linear(dim * expansion_factor, dim), nn.LayerNorm(dim))
        self.se_block = nn.Sequential(nn.Linear(dim, dim // 4), nn.ReLU(), nn.Linear(dim // 4, dim), nn.Sigmoid())

    def forward(self, x):
        b = self.block
        h = _ln(_lin(x, b[0]), b[1], gelu=True)
        h = b[3](h)
        out = _ln(_lin(h, b[4]), b[5])
        s = self.se_block
        w = torch.sigmoid(_lin(F.relu(_lin(out, s[0])), s[2]))
        return x + out * w


class DeepResidualHead(nn.Module):
    """item_tower.py:77-128: d -> 2d -> 4d, two SE residual blocks, 4d -> out, plus a d -> out
    input shortcut."""

    def __init__(self, input_dim, output_dim=128):
        super().__init__()
        mid_dim, hidden_dim = input_dim * 2, input_dim * 4
        self.expand_layer1 = nn.Sequential(nn.Linear(input_dim, mid_dim), nn.LayerNorm(mid_dim), nn.GELU(),
                                           nn.Dropout(0.1))
        self.expand_layer2 = nn.Sequential(nn.Linear(mid_dim, hidden_dim), nn.LayerNorm(hidden_dim), nn.GELU(),
                                           nn.Dropout(0.1))
        self.res_blocks = nn.Sequential(SEResidualBlock(hidden_dim, dropout=0.2),
                                        SEResidualBlock(hidden_dim, dropout=0.2))
        self.final_proj = nn.Linear(hidden_dim, output_dim)
        self.input_skip = nn.Linear(input_dim, output_dim)

    def forward(self, x):
        e1, e2 = self.expand_layer1, self.expand_layer2
        m = e1[3](_ln(_lin(x, e1[0]), e1[1], gelu=True))
        h = e2[3](_ln(_lin(m, e2[0]), e2[1], gelu=True))
        h = self.res_blocks(h)
        return _lin(h, self.final_proj) + _lin(x, self.input_skip)


def build_local_bert(hidden_size: int = 768, num_layers: int = 12, num_heads: int = 12, intermediate: int = 3072,
                     vocab_size: int = 30522, max_position: int = 512, seed: int = 0):
    """A randomly initialised BertModel of the given shape (bert-base by default): the offline
    stand-in for AutoModel.from_pretrained("bert-base-uncased") (item_tower.py:149-150)."""
    from transformers import BertConfig, BertModel
    cfg = BertConfig(vocab_size=vocab_size, hidden_size=hidden_size, num_hidden_layers=num_layers,
                     num_attention_heads=num_heads, intermediate_size=intermediate,
                     max_position_embeddings=max_position)
    torch.manual_seed(seed)
    return BertModel(cfg)


# RSX_BERT_TRAIN_NATIVE=0: the text BERT under grad runs through transformers' BertModel (A/B)
_BERT_TRAIN_NATIVE = os.environ.get("RSX_BERT_TRAIN_NATIVE", "1") != "0"


@contextlib.contextmanager
def bert_train_native(on: bool):
    """Temporarily route HybridItemTower's BERT under grad through bert_cls_packed_train (on) or BertModel."""
    global _BERT_TRAIN_NATIVE
    prev, _BERT_TRAIN_NATIVE = _BERT_TRAIN_NATIVE, bool(on)
    try:
        yield
    finally:
        _BERT_TRAIN_NATIVE = prev


def _bert_qkv(att_self):
    """[3D, D] weight / [3D] bias of BertSelfAttention's query, key, value concatenated (the
    qkv row layout of rsx_mha_fwd: Q | K | V, head h at columns h*dh), rebuilt when one changes."""
    ps = (att_self.query.weight, att_self.key.weight, att_self.value.weight,
          att_self.query.bias, att_self.key.bias, att_self.value.bias)
    key = ops._tensor_key(ps)
    c = att_self.__dict__.get("_rsx_qkv")
    if c is None or not ops._key_eq(c[0], key):
        c = (key, torch.cat(ps[:3], 0).contiguous(), torch.cat(ps[3:], 0).contiguous())
        att_self.__dict__["_rsx_qkv"] = c
    return c[1], c[2]


def _bert_linear(x, lin, gelu=False):
    W = lin.weight
    if ops._x3_ok(W.shape[0], W.shape[1]):
        return ops.gemm_x3(x, W, lin.bias, epi=ops.EPI_GELU_DROP if gelu else ops.EPI_BIAS, tag="bert_linear")
    y = F.linear(x, W, lin.bias)
    return F.gelu(y) if gelu else y


def bert_packed_ok(bert, input_ids, attn_mask) -> bool:
    """Whether bert_cls_packed computes exactly what BertModel does for this call: absolute
    positions, erf GELU, head dim 16/32/64, hidden a multiple of 256 (<= 1024), sequences of at
    most 64 tokens, and position 0 ([CLS]) valid in every row (a masked position still produces
    an output row in BertModel, which packing drops). One host sync (the mask check)."""
    cfg = bert.config
    D, H = cfg.hidden_size, cfg.num_attention_heads
    if (getattr(cfg, "position_embedding_type", "absolute") or "absolute") != "absolute":
        return False
    if cfg.hidden_act != "gelu" or D % 256 or D > 1024 or D // H not in (16, 32, 64) or input_ids.shape[1] > 64:
        return False
    return bool(attn_mask[:, 0].all().item())


@torch.no_grad()
def bert_cls_packed(bert, input_ids, attn_mask):
    """BertModel(input_ids, attention_mask).last_hidden_state[:, 0] (item_tower.py:264-268) for
    inference, over the packed valid tokens only: BertEmbeddings on the packed ids
    (rsx_embed3_ln, position = column index as BertModel's default position ids), then per layer
    the fused QKV GEMM, the varlen attention kernel (the mask's padded keys are simply absent
    from each row's segment), out-proj, residual + LayerNorm, GELU intermediate (in the GEMM
    epilogue), output GEMM, residual + LayerNorm. The last layer needs every token's K / V but
    only the [CLS] queries, so its attention output, out-proj and feed-forward run on B rows.
    Call only when bert_packed_ok(); eval mode (no dropout)."""
    B, S = input_ids.shape
    m = attn_mask != 0
    flat = m.reshape(-1).nonzero().squeeze(1)
    seg = torch.zeros(B + 1, device=input_ids.device, dtype=torch.int64)
    seg[1:] = torch.cumsum(m.sum(dim=1), 0)
    cls_rows = seg[:-1]
    h = ops.bert_embed_packed(bert.embeddings, input_ids.reshape(-1)[flat], flat % S)
    H = bert.config.num_attention_heads
    layers = bert.encoder.layer
    seg32 = seg.to(torch.int32)
    for li, layer in enumerate(layers):
        att = layer.attention
        wqkv, bqkv = _bert_qkv(att.self)
        qkv = _bert_linear(h, _Lin(wqkv, bqkv))
        ctx = ops.mha(qkv, None, H, causal=False, p_drop=0.0, seg_off=seg32)
        if li == len(layers) - 1:
            ctx, h = ctx[cls_rows], h[cls_rows]
        ln = att.output.LayerNorm
        h = ops.add_layer_norm_infer(_bert_linear(ctx, att.output.dense), h, ln.weight, ln.bias, ln.eps)
        inter = _bert_linear(h, layer.intermediate.dense, gelu=True)
        ln = layer.output.LayerNorm
        h = ops.add_layer_norm_infer(_bert_linear(inter, layer.output.dense), h, ln.weight, ln.bias, ln.eps)
    if len(layers) == 0:
        h = h[cls_rows]
    return h


def bert_cls_packed_train(bert, input_ids, attn_mask):
    """BertModel(input_ids, attention_mask).last_hidden_state[:, 0] under autograd, for the SimCSE
    training step (item_tower.py:264-272 with BERT fine-tuned at lr 1e-5, :1012-1022), over the packed
    valid tokens: the embedding sum (word + position = column index + token type 0) and its LayerNorm,
    then per layer the fused QKV token linear (bf16x3 GEMM forward / dX, split-K weight gradient), the
    varlen attention (bf16x3 forward, the head-dim-64 fp32 backward mha_bwd64_k), the out-projection,
    residual + dropout + LayerNorm (one kernel each way), the GELU feed-forward (GELU in the GEMM
    epilogue) and the second residual + LayerNorm. The last layer's attention output, out-projection
    and feed-forward run on the [CLS] rows only (the only rows read); its keys and values still see
    every token. Dropout: attention probabilities and the two residual branches by the library's counter
    hash, the embedding output by torch (BertModel's placements; its RNG stream is not reproduced).
    Call only when bert_packed_ok()."""
    B, S = input_ids.shape
    m = attn_mask != 0
    flat = m.reshape(-1).nonzero().squeeze(1)
    seg = torch.zeros(B + 1, device=input_ids.device, dtype=torch.int64)
    seg[1:] = torch.cumsum(m.sum(dim=1), 0)
    cls_rows = seg[:-1]
    seg32 = seg.to(torch.int32)
    emb = bert.embeddings
    ids = input_ids.reshape(-1)[flat]
    pos = flat % S
    x = emb.word_embeddings(ids) + emb.position_embeddings(pos) + emb.token_type_embeddings(torch.zeros_like(ids))
    h = ops.layer_norm(x, emb.LayerNorm.weight, emb.LayerNorm.bias, emb.LayerNorm.eps)
    cfg = bert.config
    p_h = cfg.hidden_dropout_prob if bert.training else 0.0
    p_a = cfg.attention_probs_dropout_prob if bert.training else 0.0
    h = F.dropout(h, p_h, bert.training)
    H = cfg.num_attention_heads
    layers = bert.encoder.layer
    for li, layer in enumerate(layers):
        att = layer.attention
        sa = att.self
        wqkv = torch.cat([sa.query.weight, sa.key.weight, sa.value.weight], 0)
        bqkv = torch.cat([sa.query.bias, sa.key.bias, sa.value.bias], 0)
        ctx = ops.mha(ops.linear_tok(h, wqkv, bqkv), None, H, causal=False, p_drop=p_a, seg_off=seg32, max_len=S)
        if li == len(layers) - 1:
            ctx, h = ctx[cls_rows], h[cls_rows]
        ln = att.output.LayerNorm
        _, h = ops.add_layer_norm(h, ops.linear_tok(ctx, att.output.dense.weight, att.output.dense.bias), ln.weight,
                                  ln.bias, ln.eps, p_drop=p_h)
        f = ops.ffn(h, layer.intermediate.dense.weight, layer.intermediate.dense.bias, layer.output.dense.weight,
                    layer.output.dense.bias, p_drop=0.0)
        ln = layer.output.LayerNorm
        _, h = ops.add_layer_norm(h, f, ln.weight, ln.bias, ln.eps, p_drop=p_h)
    if len(layers) == 0:
        h = h[cls_rows]
    return h


class _Lin:  # weight / bias pair in nn.Linear's attribute names
    def __init__(self, weight, bias):
        self.weight, self.bias = weight, bias


class HybridItemTower(nn.Module):
    """item_tower.py:131-286. forward(std_input [B,F], re_input_ids [B,9,R], re_attn_mask [B,9,R],
    text_input_ids [B,S], text_attn_mask [B,S]) -> L2-normalised [B, output_dim]."""

    def __init__(self, std_vocab_size: int, num_std_fields: int, embed_dim: int = 128, output_dim: int = 128,
                 bert_model: Optional[nn.Module] = None):
        super().__init__()
        self.std_embedding = nn.Embedding(std_vocab_size, embed_dim, padding_idx=PAD_ID)
        self.std_field_emb = nn.Parameter(torch.randn(1, num_std_fields, embed_dim))
        self.std_ln = nn.LayerNorm(embed_dim)
        self.re_ln = nn.LayerNorm(embed_dim)
        self.bert_model = bert_model if bert_model is not None else build_local_bert()
        self.bert_config = self.bert_model.config
        bert_dim = self.bert_config.hidden_size
        self.re_proj = nn.Sequential(nn.Linear(bert_dim, embed_dim), nn.LayerNorm(embed_dim), nn.GELU())
        self.re_field_position = nn.Parameter(torch.randn(1, 9, embed_dim))
        self.text_proj = nn.Sequential(nn.Linear(bert_dim, embed_dim), nn.LayerNorm(embed_dim), nn.GELU())
        encoder_layer = nn.TransformerEncoderLayer(d_model=embed_dim, nhead=4, dim_feedforward=embed_dim * 4,
                                                   batch_first=True, dropout=0.1, activation="gelu",
                                                   norm_first=True)
        self.transformer = nn.TransformerEncoder(encoder_layer, num_layers=2, enable_nested_tensor=False)
        self.head = DeepResidualHead(input_dim=embed_dim, output_dim=output_dim)
        self.embed_dim = embed_dim
        self._std_guard = ops.IdRangeGuard("std_embedding (STD ids, utils/vocab.py:436-441)")

    def check_inputs(self):
        """Raise IndexError if any forward so far received an STD id outside the embedding
        (checked on the device; waits for those checks). The serving / training loops call it
        where they synchronise anyway."""
        self._std_guard.check()

    def re_vectors(self, re_input_ids, re_attn_mask):
        """RE fields: BERT word embeddings (no grad) -> re_proj -> masked mean over the field's
        tokens (count clamped at 1e-9) -> + field position -> LayerNorm  (:247-262).

        Only the valid tokens enter the masked mean, so they are packed first: BertEmbeddings on
        the packed ids (rsx_embed3_ln, no [B*9, 32, 768] activation), re_proj + LayerNorm/GELU on
        the packed rows, and the mean as a segmented sum over each field's contiguous tokens.
        Same sums as the reference's (feats * m).sum(1) without the zero terms."""
        B, nf, R = re_input_ids.shape
        emb = self.bert_model.embeddings
        m = re_attn_mask.reshape(-1, R)
        if (emb.word_embeddings.weight.shape[1] % 256 or getattr(emb, "position_embedding_type", "absolute")
                != "absolute"):
            return self._re_vectors_dense(re_input_ids, re_attn_mask)
        flat = (m.reshape(-1) != 0).nonzero().squeeze(1)                     # packed valid tokens
        tok_seg = torch.div(flat, R, rounding_mode="floor")
        counts = m.to(torch.float32).sum(dim=1)                              # [B*9]
        seg = torch.zeros(m.shape[0] + 1, device=m.device, dtype=torch.int64)
        seg[1:] = torch.cumsum((m != 0).sum(dim=1), 0)
        word = ops.bert_embed_packed(emb, re_input_ids.reshape(-1)[flat], flat % R)
        p = self.re_proj
        feats = _ln(_lin(word, p[0]), p[1], gelu=True)                      # [T_valid, d]
        vec = ops.segment_mean(feats, seg, tok_seg, counts)
        vec = vec.reshape(B, nf, -1) + self.re_field_position
        return _ln(vec, self.re_ln)

    def _re_vectors_dense(self, re_input_ids, re_attn_mask):
        B, nf, R = re_input_ids.shape
        with torch.no_grad():
            word = self.bert_model.embeddings(input_ids=re_input_ids.reshape(-1, R))
        p = self.re_proj
        feats = _ln(_lin(word, p[0]), p[1], gelu=True)                      # [B*9, R, d]
        m = re_attn_mask.reshape(-1, R, 1).to(feats.dtype)
        vec = (feats * m).sum(dim=1) / torch.clamp(m.sum(dim=1), min=1e-9)
        vec = vec.reshape(B, nf, -1) + self.re_field_position
        return _ln(vec, self.re_ln)

    def forward(self, std_input, re_input_ids, re_attn_mask, text_input_ids, text_attn_mask):
        # the ids' range is checked on the device (no host sync); an out-of-range id raises
        # IndexError from the next forward or check_inputs() (the callers' sync points)
        std_input = self._std_guard(std_input, self.std_embedding.num_embeddings)
        std_emb = _ln(self.std_embedding(std_input) + self.std_field_emb, self.std_ln)        # :240-243
        re_vec = self.re_vectors(re_input_ids, re_attn_mask)                                   # :247-262
        if (not torch.is_grad_enabled() and not self.bert_model.training
                and bert_packed_ok(self.bert_model, text_input_ids, text_attn_mask)):
            cls = bert_cls_packed(self.bert_model, text_input_ids, text_attn_mask)       # inference
        elif (torch.is_grad_enabled() and _BERT_TRAIN_NATIVE
              and bert_packed_ok(self.bert_model, text_input_ids, text_attn_mask)):
            cls = bert_cls_packed_train(self.bert_model, text_input_ids, text_attn_mask)  # training (SimCSE)
        else:
            cls = self.bert_model(input_ids=text_input_ids, attention_mask=text_attn_mask).last_hidden_state[:, 0, :]
        t = self.text_proj
        text_vec = _ln(_lin(cls, t[0]), t[1], gelu=True).unsqueeze(1)                         # :269-271
        seq = torch.cat([std_emb, re_vec, text_vec], dim=1)                                   # [B, 16, d]
        p = self.transformer.layers[0].dropout.p if self.training else 0.0
        ctx = encoder_stack(self.transformer.layers, seq.contiguous(), None, p, self.training, causal=False)
        out = self.head(ctx.mean(dim=1))
        return ops.l2_normalize(out)


class OptimizedItemTower(nn.Module):
    """item_tower.py:289-305: normalize(Linear -> LayerNorm -> GELU -> Linear)."""

    def __init__(self, input_dim=OUTPUT_DIM_ENCODER, output_dim=OUTPUT_DIM_PROJECTOR):
        super().__init__()
        self.layer = nn.Sequential(nn.Linear(input_dim, input_dim), nn.LayerNorm(input_dim), nn.GELU(),
                                   nn.Linear(input_dim, output_dim))

    def forward(self, x):
        L = self.layer
        y = _lin(_ln(_lin(x, L[0]), L[1], gelu=True), L[3])
        return ops.l2_normalize(y)


class SimCSEModelWrapper(nn.Module):
    """item_tower.py:308-322: encoder -> projector."""

    def __init__(self, encoder: nn.Module, projector: nn.Module):
        super().__init__()
        self.encoder = encoder
        self.projector = projector

    def forward(self, std, re_ids, re_mask, txt_ids, txt_mask):
        return self.projector(self.encoder(std, re_ids, re_mask, txt_ids, txt_mask))


def simcse_loss(emb1, emb2, temperature: float = 0.08):
    """(CE(e1 e2^T / tau, arange) + CE(e2 e1^T / tau, arange)) / 2 (item_tower.py:1072-1079) on
    the fused InfoNCE kernel (no logit matrix): row direction A=e1/B=e2, column direction
    A=e2/B=e1, each the mean over rows of LSE_j S_ij - S_ii."""
    l1 = ops.nce_loss(emb1, emb2, tau=temperature, flags=ops.NCE_PLAIN, tag="simcse")
    l2 = ops.nce_loss(emb2, emb1, tau=temperature, flags=ops.NCE_PLAIN, tag="simcse")
    return (l1 + l2) / 2


@torch.no_grad()
def calculate_metrics(x, y, t=2):
    """item_tower.py:607-629: alignment E||x-y||^2 and uniformity log E exp(-t ||a_i - a_j||^2)
    over the pairs of cat([x, y])."""
    align = (x - y).norm(p=2, dim=1).pow(2).mean().item()
    allv = torch.cat([x, y], dim=0)
    uni = torch.pdist(allv, p=2).pow(2).mul(-t).exp().mean().log().item()
    return align, uni


def simcse_train_step(model, inputs_v1, inputs_v2, optimizer, temperature: float = 0.08, scheduler=None):
    """One batch of train_simcse_from_db's loop (item_tower.py:1060-1085): two dropout views,
    symmetric SimCSE loss, backward, optimizer (+ scheduler) step. fp32 (no GradScaler)."""
    optimizer.zero_grad(set_to_none=True)
    emb1 = model(*inputs_v1)
    emb2 = model(*inputs_v2)
    loss = simcse_loss(emb1, emb2, temperature)
    loss.backward()
    enc = getattr(model, "encoder", model)
    if hasattr(enc, "check_inputs"):
        enc.check_inputs()   # out-of-range STD ids raise before the update, not after it
    optimizer.step()
    if scheduler is not None:
        scheduler.step()
    return loss.detach(), emb1.detach(), emb2.detach()


def train_simcse_from_db(encoder: nn.Module, projector: nn.Module, db_session, batch_size: int, epochs: int,
                         lr: float, checkpoint_path: Optional[str] = None, collator=None, model_dir: str = "models",
                         dropout_prob: float = 0.2, temperature: float = 0.08, seed: Optional[int] = None,
                         check_interval: int = 50):
    """item_tower.py:887-1126: SimCSE training of encoder + projector over every product of the
    source. Products -> TrainingItems with the RAW name (:898-950); the encoder optionally
    resumes from an encoder-only checkpoint (strict, then non-strict, :966-983); AdamW with the
    BERT parameters at lr 1e-5 and the rest at ``lr`` (:995-1018); two corrupted views per
    product (SimCSERecSysDataset, p = 0.2), shuffled, drop_last; linear warm-up schedule over
    10 % of the steps (:1033-1038); per batch ``simcse_train_step`` (both views, symmetric
    loss at tau 0.08 on the fused InfoNCE kernel); alignment / uniformity every
    ``check_interval`` steps; the encoder's state_dict saved per epoch as
    ``encoder_ep{NN}_loss{L:.4f}.pth`` (:1113-1118). fp32 throughout (the reference's CUDA
    path runs fp16 AMP with a GradScaler). Returns the per-epoch average losses."""
    import random

    from transformers import get_linear_schedule_with_warmup

    from .item_data import SimCSECollator, SimCSERecSysDataset, rows_to_items

    rows = db_session.fetch_products()
    if not rows:
        print("[Error] No data found.")
        return []
    products = rows_to_items(rows)
    model = SimCSEModelWrapper(encoder, projector)
    device = next(encoder.parameters()).device
    N.ensure_device(next(encoder.parameters()))
    if checkpoint_path:
        if not os.path.exists(checkpoint_path):
            print(f"Checkpoint file not found: {checkpoint_path}")
            return []
        state = torch.load(checkpoint_path, map_location="cpu", weights_only=True)
        try:
            model.encoder.load_state_dict(state)
        except RuntimeError:
            model.encoder.load_state_dict(state, strict=False)
    model = model.to(device)
    model.train()
    bert_params = [p for n, p in model.named_parameters() if p.requires_grad and "bert_model" in n]
    other_params = [p for n, p in model.named_parameters() if p.requires_grad and "bert_model" not in n]
    optimizer = torch.optim.AdamW([{"params": bert_params, "lr": 1e-5}, {"params": other_params, "lr": lr}])
    rng = random.Random(seed)
    dataset = SimCSERecSysDataset(products, dropout_prob=dropout_prob, rng=rng)
    if collator is None:
        collator = SimCSECollator(std_vocab_size=encoder.std_embedding.num_embeddings)
    gen = torch.Generator().manual_seed(seed) if seed is not None else None
    loader = torch.utils.data.DataLoader(dataset, batch_size=batch_size, shuffle=True, collate_fn=collator,
                                         drop_last=True, num_workers=0, generator=gen)
    total_steps = len(loader) * epochs
    scheduler = get_linear_schedule_with_warmup(optimizer, num_warmup_steps=int(total_steps * 0.1),
                                                num_training_steps=total_steps)
    os.makedirs(model_dir, exist_ok=True)
    history = []
    for epoch in range(epochs):
        total, step = 0.0, 0
        for v1, v2 in loader:
            v1 = [t.to(device, non_blocking=True) for t in v1]
            v2 = [t.to(device, non_blocking=True) for t in v2]
            loss, e1, e2 = simcse_train_step(model, v1, v2, optimizer, temperature, scheduler)
            if step % check_interval == 0:
                align, uni = calculate_metrics(e1, e2)
                print(f"epoch {epoch + 1} step {step} loss {loss.item():.4f} align {align:.4f} uni {uni:.4f}")
            total += float(loss.item())
            step += 1
        avg = total / step if step else float("nan")
        history.append(avg)
        torch.save(encoder.state_dict(), os.path.join(model_dir, f"encoder_ep{epoch + 1:02d}_loss{avg:.4f}.pth"))
    return history
