"""CPU-only checks of the oracle, the synthetic generator and the module surface."""
import torch
import torch.nn.functional as F

from tests.helpers import small_cfg, small_universe
import recsys_amd  # noqa: F401
from recsys_amd import synth
from oracle import user_tower as O


def _batch(B=6, seed=1):
    items = small_universe(200)
    return items, synth.make_batch(items, B, max_len=50, seed=seed)


def test_explicit_attention_matches_torch_encoder_training_path():
    """The oracle's explicit MHA (safe softmax) == nn.TransformerEncoder in train mode, p=0:
    the exact module call of v1_refine_usertower.py:461-466."""
    cfg = small_cfg(num_items=200)
    torch.manual_seed(0)
    a = O.OracleUserTower(cfg, explicit_attention=True)
    b = O.OracleUserTower(cfg, explicit_attention=False)
    b.load_state_dict(a.state_dict())
    a.train(); b.train()
    items, batch = _batch()
    kw = {k: batch[k] for k in O._FWD_KEYS}
    kw["pretrained_vecs"] = items.pretrained[batch["item_ids"]]
    ya = a(**kw)
    yb = b(**kw)
    assert torch.isfinite(ya).all()
    torch.testing.assert_close(ya, yb, atol=2e-6, rtol=1e-5)


def test_fully_masked_rows_give_out_proj_bias():
    """Trap 1: left-padded query rows have all keys masked -> zero probabilities."""
    cfg = small_cfg(num_items=200)
    torch.manual_seed(0)
    m = O.OracleUserTower(cfg)
    layer = m.transformer_encoder.layers[0]
    h = torch.randn(2, 50, 128)
    pad = torch.zeros(2, 50, dtype=torch.bool)
    pad[0, :10] = True
    out = m._attention(layer, h, pad)
    torch.testing.assert_close(out[0, :10], layer.self_attn.out_proj.bias.expand(10, -1))


def test_padding_rows_nonzero_after_init():
    """Trap 3: _init_weights re-initialises padding rows (v1_refine_usertower.py:408-409)."""
    torch.manual_seed(0)
    m = O.OracleUserTower(small_cfg(num_items=200))
    assert m.item_id_emb.weight[0].abs().sum() > 0
    assert m.time_emb.weight[0].abs().sum() > 0


def test_module_surface_matches_oracle():
    from recsys_amd.tower_code.v1_refine_usertower import SASRecUserTower
    cfg = small_cfg(num_items=300)
    torch.manual_seed(3)
    ref = O.OracleUserTower(cfg)
    torch.manual_seed(3)
    dut = SASRecUserTower(cfg)
    sr, sd = ref.state_dict(), dut.state_dict()
    assert list(sr.keys()) == list(sd.keys())
    for k in sr:
        assert sr[k].shape == sd[k].shape, k
        assert torch.equal(sr[k], sd[k]), f"init differs for {k}"


def test_synthetic_batch_layout():
    items, batch = _batch(B=64, seed=5)
    pad, ids, tgt, tb = batch["padding_mask"], batch["item_ids"], batch["target_ids"], batch["time_bucket_ids"]
    L = ids.shape[1]
    for b in range(ids.shape[0]):
        n = int((~pad[b]).sum())
        assert n >= 1
        assert pad[b, : L - n].all() and not pad[b, L - n:].any()  # left padding
        assert (ids[b, : L - n] == 0).all() and (ids[b, L - n:] > 0).all()
        assert (tb[b, L - n:] >= 1).all() and (tb[b, L - n:] <= 9).all()
        if n > 1:  # SASRec shift: input[t+1] == target[t]  (dataset_peek, v1_refine_usertower.py:14-36)
            assert torch.equal(ids[b, L - n + 1:], tgt[b, L - n:-1])
    side = items.side[ids]
    assert torch.equal(side[..., 0], batch["type_ids"])
    assert items.log_q[0] == -20.0


def test_logq_matches_reference_formula():
    raw = torch.tensor([0.5, float("nan"), 0.25, 0.25]).numpy()
    lq = synth.logq_from_probs(raw)
    p = torch.tensor([0.5, 0.0, 0.25, 0.25]) + 1e-6
    p = p / p.sum()
    torch.testing.assert_close(lq[1:], torch.log(p))
    assert lq[0] == -20.0


def test_oracle_loss_equals_row_lse_form():
    """inbatch_corrected_logq_loss == mean_i(LSE_j S_ij - S_ii) with masks (what the kernel computes)."""
    g = torch.Generator().manual_seed(0)
    n, items = 40, 30
    u = F.normalize(torch.randn(n, 128, generator=g), dim=1)
    w = F.normalize(torch.randn(items, 128, generator=g), dim=1)
    t = torch.randint(1, items, (n,), generator=g)
    users = torch.randint(0, 8, (n,), generator=g)
    lq = torch.log_softmax(torch.randn(items, generator=g), 0)
    ref = O.inbatch_corrected_logq_loss(u, w, t, users, lq)
    s = (u @ w[t].T) / 0.1 - lq[t][None, :]
    excl = ((t[:, None] == t[None, :]) | (users[:, None] == users[None, :])) & ~torch.eye(n, dtype=torch.bool)
    s = s.masked_fill(excl, float("-inf"))
    alt = (torch.logsumexp(s, 1) - s.diagonal()).mean()
    torch.testing.assert_close(ref, alt)


def test_packed_tokens_layout():
    from recsys_amd.tower_code.v1_refine_usertower import PackedTokens
    items, batch = _batch(B=64, seed=9)
    pad = batch["padding_mask"]
    B, L = pad.shape
    pk = PackedTokens(pad)
    valid = ~pad
    # loss rows == output[valid_mask] order (row-major b, t)
    assert torch.equal(pk.flat[pk.valid_tok], valid.reshape(-1).nonzero().squeeze(1))
    last = (valid.sum(1) - 1).clamp(min=0)
    assert torch.equal(pk.flat[pk.last_tok], torch.arange(B) * L + last)
    seg = pk.seg_off.long()
    for b in range(B):
        toks = pk.flat[seg[b]:seg[b + 1]]
        assert ((toks // L) == b).all() and (toks.diff() > 0).all()
        assert (seg[b + 1] - seg[b]) <= L
    # the extra (padded) token of a user is its first packed token and has no valid key before it
    extra = pk.tok_pad.bool()
    assert torch.equal(extra.nonzero().squeeze(1), seg[:-1][pad[torch.arange(B), last]])


def test_get_hash_id_and_side_table():
    """synth.get_hash_id / hashed_side_ids restate v1_usertower_train.py:211-262: md5 of the
    stripped lower-cased text, % hash_size + 1; 0 for empty / unknown / nan / none; unmatched
    items keep zeros; row 0 is the pad row."""
    import hashlib
    from recsys_amd import synth
    h = lambda t: int(hashlib.md5(t.encode("utf-8")).hexdigest(), 16) % 1000 + 1  # noqa: E731
    assert synth.get_hash_id("Vest top") == h("vest top") == synth.get_hash_id("  VEST TOP ")
    for t in ("", None, "Unknown", "NaN", "none"):
        assert synth.get_hash_id(t) == 0
    assert 1 <= synth.get_hash_id("Solid", 7) <= 7
    meta = [{"product_type_name": "Vest top", "colour_group_name": "Black", "graphical_appearance_name": "Solid",
             "section_name": "Womens Everyday Basics"}, None, {"product_type_name": "Sweater"}]
    tab = synth.hashed_side_ids(meta)
    assert tab.shape == (4, 4) and tab.dtype == torch.int64
    assert tab[0].tolist() == [0, 0, 0, 0] and tab[2].tolist() == [0, 0, 0, 0]
    assert tab[1].tolist() == [h("vest top"), h("black"), h("solid"), h("womens everyday basics")]
    assert tab[3].tolist() == [h("sweater"), 0, 0, 0]
