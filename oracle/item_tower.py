"""CPU restatement of item_tower.py's models and SimCSE loss:
SEResidualBlock :41-75, DeepResidualHead :77-128, HybridItemTower :131-286,
OptimizedItemTower :289-305, SimCSEModelWrapper :308-322, loss :1069-1082,
calculate_metrics :607-629. Plain PyTorch modules in the reference's structure (their own
nn.Sequential / nn.TransformerEncoder forwards), parameter names identical to the package's
so one state_dict drives both.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py; parity unpinned: no reference fixtures;
the BERT is a locally built, randomly initialised transformers.BertModel on both sides).
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

PAD_ID = 0


class OracleSEResidualBlock(nn.Module):
    def __init__(self, dim, dropout=0.2, expansion_factor=4):
        super().__init__()
        self.block = nn.Sequential(
            nn.Linear(dim, dim * expansion_factor), nn.LayerNorm(dim * expansion_factor), nn.GELU(),
            nn.Dropout(dropout), nn.Linear(dim * expansion_factor, dim), nn.LayerNorm(dim))
        self.se_block = nn.Sequential(nn.Linear(dim, dim // 4), nn.ReLU(), nn.Linear(dim // 4, dim), nn.Sigmoid())

    def forward(self, x):  # :66-75
        out = self.block(x)
        return x + out * self.se_block(out)


class OracleDeepResidualHead(nn.Module):
    def __init__(self, input_dim, output_dim=128):
        super().__init__()
        mid_dim, hidden_dim = input_dim * 2, input_dim * 4
        self.expand_layer1 = nn.Sequential(nn.Linear(input_dim, mid_dim), nn.LayerNorm(mid_dim), nn.GELU(),
                                           nn.Dropout(0.1))
        self.expand_layer2 = nn.Sequential(nn.Linear(mid_dim, hidden_dim), nn.LayerNorm(hidden_dim), nn.GELU(),
                                           nn.Dropout(0.1))
        self.res_blocks = nn.Sequential(OracleSEResidualBlock(hidden_dim, 0.2), OracleSEResidualBlock(hidden_dim, 0.2))
        self.final_proj = nn.Linear(hidden_dim, output_dim)
        self.input_skip = nn.Linear(input_dim, output_dim)

    def forward(self, x):  # :114-128
        h = self.res_blocks(self.expand_layer2(self.expand_layer1(x)))
        return self.final_proj(h) + self.input_skip(x)


class OracleHybridItemTower(nn.Module):
    def __init__(self, std_vocab_size, num_std_fields, embed_dim=128, output_dim=128, bert_model=None):
        super().__init__()
        self.std_embedding = nn.Embedding(std_vocab_size, embed_dim, padding_idx=PAD_ID)
        self.std_field_emb = nn.Parameter(torch.randn(1, num_std_fields, embed_dim))
        self.std_ln = nn.LayerNorm(embed_dim)
        self.re_ln = nn.LayerNorm(embed_dim)
        self.bert_model = bert_model
        bert_dim = bert_model.config.hidden_size
        self.re_proj = nn.Sequential(nn.Linear(bert_dim, embed_dim), nn.LayerNorm(embed_dim), nn.GELU())
        self.re_field_position = nn.Parameter(torch.randn(1, 9, embed_dim))
        self.text_proj = nn.Sequential(nn.Linear(bert_dim, embed_dim), nn.LayerNorm(embed_dim), nn.GELU())
        layer = nn.TransformerEncoderLayer(d_model=embed_dim, nhead=4, dim_feedforward=embed_dim * 4,
                                           batch_first=True, dropout=0.1, activation="gelu", norm_first=True)
        self.transformer = nn.TransformerEncoder(layer, num_layers=2, enable_nested_tensor=False)
        self.head = OracleDeepResidualHead(input_dim=embed_dim, output_dim=output_dim)

    def forward(self, std_input, re_input_ids, re_attn_mask, text_input_ids, text_attn_mask):  # :228-286
        B = std_input.shape[0]
        std_emb = self.std_ln(self.std_embedding(std_input) + self.std_field_emb)
        flat_re_ids = re_input_ids.view(-1, re_input_ids.size(-1))
        with torch.no_grad():
            word_embs = self.bert_model.embeddings(input_ids=flat_re_ids)
        re_feats = self.re_proj(word_embs)
        flat_mask = re_attn_mask.view(-1, re_attn_mask.size(-1)).unsqueeze(-1)
        sum_re = torch.sum(re_feats * flat_mask, dim=1)
        count_re = torch.clamp(flat_mask.sum(dim=1), min=1e-9)
        re_vectors = (sum_re / count_re).view(B, 9, -1) + self.re_field_position
        re_vectors = self.re_ln(re_vectors)
        bert_out = self.bert_model(input_ids=text_input_ids, attention_mask=text_attn_mask)
        text_vec = self.text_proj(bert_out.last_hidden_state[:, 0, :]).unsqueeze(1)
        combined = torch.cat([std_emb, re_vectors, text_vec], dim=1)
        out = self.head(self.transformer(combined).mean(dim=1))
        return F.normalize(out, p=2, dim=1)


class OracleOptimizedItemTower(nn.Module):
    def __init__(self, input_dim=128, output_dim=128):
        super().__init__()
        self.layer = nn.Sequential(nn.Linear(input_dim, input_dim), nn.LayerNorm(input_dim), nn.GELU(),
                                   nn.Linear(input_dim, output_dim))

    def forward(self, x):
        return F.normalize(self.layer(x), p=2, dim=1)


def simcse_loss(emb1, emb2, temperature=0.08):  # :1072-1079
    sim = emb1 @ emb2.T / temperature
    labels = torch.arange(emb1.size(0))
    return (F.cross_entropy(sim, labels) + F.cross_entropy(sim.T, labels)) / 2
