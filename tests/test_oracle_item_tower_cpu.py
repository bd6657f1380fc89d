"""CPU checks of the item-tower oracle (test infrastructure): shapes, normalisation, the
SimCSE loss identity on a symmetric case, and the hard-emphasis loss's mining count."""
import torch

from oracle import item_tower as OIT
from oracle import user_tower as O

import recsys_amd  # noqa: F401
from recsys_amd import synth
from recsys_amd.tower_code import v1_refine_usertower as T


def test_oracle_item_tower_shapes_and_norm():
    from transformers import BertConfig, BertModel
    torch.manual_seed(0)
    bert = BertModel(BertConfig(vocab_size=500, hidden_size=32, num_hidden_layers=1, num_attention_heads=2,
                                intermediate_size=64, max_position_embeddings=40))
    m = OIT.OracleHybridItemTower(50, 6, 64, 128, bert_model=bert).eval()
    B = 5
    std = torch.randint(0, 50, (B, 6))
    re = torch.randint(0, 500, (B, 9, 8))
    rm = torch.ones(B, 9, 8, dtype=torch.long)
    rm[:, :, 5:] = 0
    tx = torch.randint(0, 500, (B, 12))
    tm = torch.ones(B, 12, dtype=torch.long)
    y = m(std, re, rm, tx, tm)
    assert y.shape == (B, 128)
    torch.testing.assert_close(y.norm(dim=1), torch.ones(B), atol=1e-5, rtol=0)


def test_oracle_simcse_loss_symmetric():
    e = torch.nn.functional.normalize(torch.randn(16, 8), dim=1)
    l = OIT.simcse_loss(e, e, temperature=0.08)
    s = e @ e.T / 0.08
    ref = torch.nn.functional.cross_entropy(s, torch.arange(16))
    torch.testing.assert_close(l, ref)


def test_oracle_hard_emphasis_num_k():
    torch.manual_seed(1)
    u = torch.randn(301, 16)
    w = torch.randn(50, 16)
    t = torch.randint(0, 50, (301,))
    loss, st = O.full_batch_hard_emphasis_loss(u, w, t, torch.zeros(50), top_k_percent=0.01)
    assert st["num_hard"] == 3 and torch.isfinite(loss)


def test_feature_processor_logq():
    """get_logq_probs (v1_refine_usertower.py:124-137): nan -> 0, + 1e-6, normalise, log,
    padding row -20 — identical to the synthetic-universe helper on the same probs."""
    import numpy as np
    import pandas as pd
    probs = np.array([0.5, np.nan, 0.2, 0.0, 0.3])
    df = pd.DataFrame({"article_id": [11, 12, 13, 14, 15], "raw_probability": probs})
    fp = T.FeatureProcessor(df)
    lq = fp.get_logq_probs("cpu")
    exp = synth.logq_from_probs(probs)
    assert torch.equal(lq, exp)
    assert fp.item2id[13] == 3 and lq[0].item() == -20.0
