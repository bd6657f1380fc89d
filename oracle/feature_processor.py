"""CPU restatement of the GDCN reranker input -- TEST INFRASTRUCTURE ONLY.

Follows reference utils/data_preprocessing/feature_processor.py, vectorised over a batch with
numpy: StandardScaler.fit_transform (:59-65; population std, zero std -> 1), the scaled user /
item dense columns (:70-83), the cross features from the raw log values (:89-111), the
RerankerDataset item (:156-181) and reranker_collate_fn (:184-191: right padding to the batch's
longest sequence, mask = ids != 0). Parity of the scaler is pinned against sklearn (the
reference's own dependency) in tests/test_reranker_input_cpu.py.
"""
import numpy as np
import torch

U_DENSE = ["user_avg_price_log", "total_cnt_log", "recency_log"]
I_DENSE = ["pop_1w_log", "pop_1m_log", "velocity_1w", "velocity_1m", "days_since_release_log", "avg_item_price_log"]


def standard_scale(x):
    """(x - mean) / std over rows, std with ddof 0 and 1 where it is 0 (sklearn StandardScaler)."""
    x = np.asarray(x, dtype=np.float64)
    mean = x.mean(axis=0)
    std = x.std(axis=0)
    std = np.where(std == 0.0, 1.0, std)
    return (x - mean) / std


def reranker_batch(users, items, seqs, user_ids, item_ids, labels, max_len=50):
    """users / items / seqs: DataFrames indexed by customer_id / article_id / customer_id.
    -> (dense [B,12], cat [B], seq [B,L], mask [B,L], target [B], label [B]) torch tensors."""
    u_scaled = standard_scale(users[U_DENSE].values)
    i_scaled = standard_scale(items[I_DENSE].values)
    ur = users.index.get_indexer(list(user_ids))
    ir = items.index.get_indexer(list(item_ids))
    assert (ur >= 0).all() and (ir >= 0).all()
    u_raw, i_raw = users.iloc[ur], items.iloc[ir]
    cross = np.stack([i_raw["avg_item_price_log"].values - u_raw["user_avg_price_log"].values,
                      i_raw["velocity_1w"].values * u_raw["total_cnt_log"].values,
                      i_raw["velocity_1m"].values * u_raw["total_cnt_log"].values], axis=1)
    dense = np.concatenate([u_scaled[ur].astype(np.float32), i_scaled[ir].astype(np.float32),
                            cross.astype(np.float32)], axis=1)
    cat = users["preferred_channel"].values[ur].astype(np.int64) - 1
    rows = []
    for uid in user_ids:
        s = seqs["sequence_ids"].get(uid) if uid in seqs.index else None
        s = [] if s is None else list(s)[-max_len:]
        rows.append(s)
    L = max([len(s) for s in rows] + [0])
    seq = np.zeros((len(rows), L), dtype=np.int64)
    for b, s in enumerate(rows):
        seq[b, :len(s)] = s
    target = np.array([int(s) if str(s).isdigit() else 0 for s in item_ids], dtype=np.int64)
    return (torch.from_numpy(dense), torch.from_numpy(cat), torch.from_numpy(seq),
            torch.from_numpy((seq != 0).astype(np.int64)), torch.from_numpy(target),
            torch.tensor(np.asarray(labels), dtype=torch.float32))
