"""CPU contract of the GDCN reranker input (utils/data_preprocessing/feature_processor.py:26-191):
the drop-in FeatureProcessor / RerankerDataset / reranker_collate_fn against the numpy
restatement in oracle/feature_processor.py, the scaler against sklearn, and the tensor contract
(shapes, dtypes, right padding, truncation to the last 50 steps, mask of id 0, target 0 for
non-numeric item ids)."""
import numpy as np
import torch
from sklearn.preprocessing import StandardScaler
from torch.utils.data import DataLoader

import recsys_amd  # noqa: F401
from recsys_amd.utils.data_preprocessing import feature_processor as FP
from oracle import feature_processor as OF
from tests.reranker_data import interactions, make_tables


def test_scaler_matches_sklearn_and_restatement():
    users, items, seqs = make_tables()
    fp = FP.FeatureProcessor(users, items, seqs)
    ref = StandardScaler().fit_transform(items[FP.I_DENSE_COLS].values)
    np.testing.assert_array_equal(fp.items_scaled[FP.I_DENSE_COLS].values, ref)
    np.testing.assert_allclose(OF.standard_scale(items[FP.I_DENSE_COLS].values), ref, rtol=0, atol=1e-12)
    # raw values kept for the cross features; raw_probability untouched
    np.testing.assert_array_equal(fp.items["velocity_1w"].values, items["velocity_1w"].values)
    np.testing.assert_array_equal(fp.items_scaled["raw_probability"].values, items["raw_probability"].values)


def test_collate_matches_restatement():
    users, items, seqs = make_tables()
    fp = FP.FeatureProcessor(users, items, seqs)
    inter = interactions(users, items, n=96)
    # users without a sequence and with > 50 steps are both in the batch
    lens = [len(seqs["sequence_ids"][u]) if u in seqs.index else 0 for u in inter["user_id"]]
    assert min(lens) == 0 and max(lens) > 50
    ds = FP.RerankerDataset(inter, fp)
    got = next(iter(DataLoader(ds, batch_size=len(inter), collate_fn=FP.reranker_collate_fn)))
    exp = OF.reranker_batch(users, items, seqs, inter["user_id"].tolist(), inter["item_id"].tolist(),
                            inter["label"].tolist())
    dense, cat, seq, mask, target, label = got
    assert dense.shape == (96, 12) and dense.dtype == torch.float32
    assert seq.shape[1] == min(50, max(lens)) and seq.dtype == torch.int64
    torch.testing.assert_close(dense, exp[0], rtol=0, atol=2e-7)
    for a, b in zip(got[1:], exp[1:]):
        assert torch.equal(a, b)
    assert (target == 0).sum() >= 0 and int(mask.sum()) == int((seq != 0).sum())


def test_get_cross_features_and_user_tensor():
    users, items, seqs = make_tables()
    fp = FP.FeatureProcessor(users, items, seqs)
    u = list(users.index[:5])
    i = list(items.index[:5])
    cross = fp.get_cross_features(u, i)
    exp = np.stack([items["avg_item_price_log"].values[:5] - users["user_avg_price_log"].values[:5],
                    items["velocity_1w"].values[:5] * users["total_cnt_log"].values[:5],
                    items["velocity_1m"].values[:5] * users["total_cnt_log"].values[:5]], axis=1)
    assert torch.equal(cross, torch.tensor(exp, dtype=torch.float32))
    dense, cat = fp.get_user_tensor(u)
    assert dense.shape == (5, 3) and torch.equal(cat, torch.tensor(users["preferred_channel"].values[:5] - 1))
    assert fp.get_raw_probability(i).shape == (5,)
    ut = FP.UserTowerDataset(u, fp)[0]
    assert ut["seq_ids"].numel() <= 50 and ut["seq_deltas"].numel() == ut["seq_ids"].numel()


def test_device_tables_csr_contract():
    users, items, seqs = make_tables()
    fp = FP.FeatureProcessor(users, items, seqs)
    t = fp.device_tables("cpu")
    off = t["seq_off"]
    assert off.shape == (len(users) + 1,) and int(off[0]) == 0
    for r in (0, 5, len(users) - 1):
        uid = users.index[r]
        s = list(seqs["sequence_ids"][uid]) if uid in seqs.index else []
        assert t["seq_ids"][off[r]:off[r + 1]].tolist() == s
    assert t["u_raw"].dtype == torch.float64 and t["i_scaled"].dtype == torch.float32
    assert int(t["i_num"][3]) == 0  # "A12345"
